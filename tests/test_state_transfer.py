"""Peer state download (reference ``albert/run_trainer.py:124-128``,
``run_first_peer.py:119-121``) at the reference's size: params + LAMB m, v of ALBERT-large
(3 x 17.8M fp32 = 214 MB).  The donor keeps training while it serves: it copies its state into a
snapshot at the end of every global step, and a request is served from that snapshot — the
server never waits for the donor's step lock (held across averaging rounds and LAMB), and a step
never waits for a transfer."""
import threading
import time

import pytest
import torch

import dedloc_amd.ops  # noqa: F401


@pytest.mark.timeout(300)
def test_albert_large_state_download_does_not_block_donor_steps():
    from dedloc_amd.averaging.averager import download_state
    from dedloc_amd.dht import DHT
    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining
    from dedloc_amd.optim.collaborative import CollaborativeOptimizer
    from dedloc_amd.optim.lamb import FusedLamb

    torch.manual_seed(0)
    model = AlbertForPreTraining(AlbertConfig.from_pretrained("albert-large-v2"))
    flat = model.materialize(torch.device("cpu"))
    n_params = flat.fp32.numel()
    assert 17_000_000 < n_params < 19_000_000, n_params
    opt = FusedLamb(flat, lr=1e-4, weight_decay=0.01, no_decay=model.no_decay_names())
    dht = DHT(listen_on="127.0.0.1:*")
    # target 1 sample: EVERY step() is a global step (accumulate + LAMB under the step lock)
    co = CollaborativeOptimizer(opt, dht=dht, prefix="xfer", target_batch_size=1, batch_size_per_step=1,
                                listen_on="127.0.0.1:*", start=True)
    try:
        flat.grad.normal_(0, 1e-3)
        for _ in range(2):
            co.step()
        durations, stop = [], threading.Event()

        def trainer():
            while not stop.is_set():
                flat.grad.normal_(0, 1e-3)
                t0 = time.perf_counter()
                co.step()
                durations.append((t0, time.perf_counter()))

        snap = []
        serve = co.averager.state_server.get_state

        def timed_snapshot():  # the server's clone of the donor's last snapshot
            a = time.perf_counter()
            out = serve()
            snap.append(time.perf_counter() - a)
            return out

        co.averager.state_server.get_state = timed_snapshot
        th = threading.Thread(target=trainer)
        th.start()
        time.sleep(0.5)
        t0 = time.perf_counter()
        meta, tensors = download_state(co.averager.state_server.endpoint, timeout=120)
        t1 = time.perf_counter()
        time.sleep(0.3)
        stop.set()
        th.join(60)
        nbytes = sum(t.numel() * t.element_size() for t in tensors)
        assert nbytes == 3 * 4 * n_params  # params + exp_avg + exp_avg_sq, fp32
        assert len(tensors) == 3 and meta["_mode"] == "T"
        assert meta["step"] >= 2
        # the snapshot is consistent: the served params are a state the donor actually had
        assert torch.isfinite(tensors[0]).all()
        transfer = t1 - t0
        during = [b - a for a, b in durations if a < t1 and b > t0]
        base = sorted(b - a for a, b in durations if b < t0)
        typical = base[len(base) // 2] if base else min(during)
        print(f"state download: {nbytes / 2**20:.0f} MiB in {transfer:.3f}s ({nbytes / transfer / 2**30:.2f} GiB/s); "
              f"snapshot (incl. waiting for the step lock) {snap[0]:.3f}s; donor steps during it: {len(during)}, "
              f"max {max(during):.3f}s, typical {typical:.3f}s")
        assert len(during) >= 1, "the donor must keep stepping while it serves its state"
        # serving clones the last snapshot without the step lock: it does not wait for the step in
        # progress (one step here is ~1 s of CPU LAMB), and a step is never delayed by the transfer
        assert len(snap) == 1
        assert snap[0] < 0.5 * typical, (snap[0], typical)
        assert max(during) < typical + snap[0] + 0.2, (max(during), typical, snap[0], transfer)
    finally:
        co.shutdown()
        dht.shutdown()


def _joiner(endpoint, q):
    import time as _t

    from dedloc_amd.averaging.averager import download_state

    t0 = _t.perf_counter()
    meta, tensors = download_state(endpoint, timeout=30)
    q.put({"seconds": _t.perf_counter() - t0, "step": meta["step"], "n": len(tensors),
           "p0": float(tensors[0][0])})


@pytest.mark.multiproc
@pytest.mark.timeout(120)
def test_joiner_downloads_from_donor_in_the_middle_of_an_averaging_round():
    """A peer joining while the donor is inside an averaging round (which holds the donor's step
    lock for matchmaking + all-reduce + LAMB, up to averaging_timeout) gets the donor's last global
    step state at once — here a round stalled for 8 s, and the download finishes within 2 s."""
    import multiprocessing as mp

    from dedloc_amd.dht import DHT, get_dht_time
    from dedloc_amd.optim.collaborative import CollaborationState, CollaborativeOptimizer
    from dedloc_amd.optim.lamb import FusedLamb
    from dedloc_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    flat = FlatParams([("w", torch.nn.Parameter(torch.randn(1 << 16))), ("b", torch.nn.Parameter(torch.zeros(64)))],
                      with_bf16=False)
    opt = FusedLamb(flat, lr=1e-3)
    dht = DHT(listen_on="127.0.0.1:*")
    co = CollaborativeOptimizer(opt, dht=dht, prefix="midround", target_batch_size=1, batch_size_per_step=1,
                                listen_on="127.0.0.1:*", start=False)
    try:
        flat.grad.normal_()
        co.step()  # global step 1, alone: the snapshot now holds step 1
        assert co.local_step == 1
        p_step1 = float(flat.fp32[0])
        in_round = threading.Event()

        def stalled_round(**kw):  # a round whose members are slow: holds lock_step for 8 s
            in_round.set()
            time.sleep(8.0)
            return None

        co.averager.step = stalled_round
        co.fetch_collaboration_state = lambda: CollaborationState(1, 2, 1, num_peers=2, num_clients=0,
                                                                  eta_next_step=get_dht_time(),
                                                                  next_fetch_time=get_dht_time() + 60)
        flat.grad.normal_()
        th = threading.Thread(target=co.step)
        th.start()
        assert in_round.wait(10)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        p = ctx.Process(target=_joiner, args=(co.averager.state_server.endpoint, q))
        t0 = time.perf_counter()
        p.start()
        res = q.get(timeout=60)
        p.join(30)
        assert th.is_alive(), "the round must still be in flight when the download completes"
        assert res["seconds"] < 2.0, res
        assert res["step"] == 1 and res["n"] == 3 and res["p0"] == p_step1
        print(f"download mid-round: {res['seconds']:.3f}s (process start included: {time.perf_counter() - t0:.2f}s)")
        th.join(30)
    finally:
        co.shutdown()
        dht.shutdown()
