"""Diagnosis for profiles/r4_swav_weights_on_side_stream_segv.txt.

Hypothesis: the crashing layout made a side stream wait on ITSELF inside the HIP-graph capture
(``sp["stream"].wait_stream(wprep)`` with wprep == sp["stream"] once the weight copies moved onto
pass 0's side stream).  torch implements ``a.wait_stream(b)`` as an event recorded on ``b`` plus
``hipStreamWaitEvent(a, event)``; with a == b inside a capture that is a captured event record
followed by a wait on it on the same stream.

Each case runs in its own child process (a host crash ends only that child) and prints a marker
after capture, after instantiation/first replay and after 20 replays, with faulthandler on.
    python bench/graph_selfwait_probe.py
"""
import os
import subprocess
import sys
import textwrap

CHILD = textwrap.dedent("""
    import faulthandler, sys, torch
    faulthandler.enable(all_threads=True)
    case = sys.argv[1]
    dev = torch.device("cuda", 0)
    x = torch.randn(1 << 20, device=dev)
    side = torch.cuda.Stream(dev)
    side2 = torch.cuda.Stream(dev)

    def body():
        cur = torch.cuda.current_stream(dev)  # inside a capture: the capturing stream
        y = x * 2
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            z = y + 1
        if case in ("self", "self_joined"):
            side.wait_stream(side)          # the crashing layout's self-wait
        if case == "cross":
            side2.wait_stream(side)
            with torch.cuda.stream(side2):
                z = z * 3
            side.wait_stream(side2)
        cur.wait_stream(side)
        return z + y

    # warm-up on a side stream, as the peer does
    ws = torch.cuda.Stream(dev)
    ws.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(ws):
        body()
    torch.cuda.current_stream(dev).wait_stream(ws)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        out = body()
    print("@@ captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("@@ replayed once", flush=True)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    ref = (x * 2 + 1) * (3 if case == "cross" else 1) + x * 2
    print("@@ ok", bool(torch.allclose(out, ref)), flush=True)
""")

# the SwAV peer itself, graphed, with the weight copies on the first side pass's stream (the r4
# layout): "unguarded" restores plain wait_stream calls (self-waits included), "guarded" is the tree
SWAV_CHILD = textwrap.dedent("""
    import faulthandler, sys, torch
    faulthandler.enable(all_threads=True)
    sys.path.insert(0, ".")
    from dedloc_amd.dht import DHT
    from dedloc_amd.models.resnet_swav import SwAVModel
    from dedloc_amd.training.swav_peer import SwavPeer
    from dedloc_amd.utils.config import load_config
    if sys.argv[1] == "unguarded":
        SwAVModel._wait = staticmethod(lambda a, b: a.wait_stream(b))
    cfg = load_config("swav_1node_resnet_submit", [
        "config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=16", "config.DATA.TRAIN.SYNTHETIC_POOL_SIZE=32",
        "config.OPTIMIZER.target_batch_size=64", "config.OPTIMIZER.batch_size_for_tracking=16",
        "config.CHECKPOINT.DIR=/tmp/graph_probe_ckpt", "config.MODEL.CUDA_GRAPH=true",
        "config.MODEL.CUDA_GRAPH_WARMUP=2"])
    dht = DHT(start=True)
    peer = SwavPeer(cfg, torch.device("cuda", 0), dht=dht)
    peer.model.dgrad_weights_stream = "side"
    for it in range(4):
        loss = float(peer.train_step())
        print("@@ iteration", it, "graphed" if peer._graphed is not None else "eager", round(loss, 4), flush=True)
    peer.shutdown(); dht.shutdown()
""")

if __name__ == "__main__":
    for case in ("plain", "cross", "self"):
        r = subprocess.run([sys.executable, "-c", CHILD, case], capture_output=True, text=True, timeout=120)
        print(f"case={case} rc={r.returncode}")
        print(r.stdout.strip())
        if r.returncode != 0:
            print(r.stderr.strip()[-3000:])
    for case in ("guarded", "unguarded"):
        r = subprocess.run([sys.executable, "-c", SWAV_CHILD, case], capture_output=True, text=True, timeout=300)
        print(f"case={case} rc={r.returncode}")
        print(r.stdout.strip())
        if r.returncode != 0:
            print(r.stderr.strip()[-3000:])
