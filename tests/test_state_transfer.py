"""Peer state download (reference ``albert/run_trainer.py:124-128``,
``run_first_peer.py:119-121``) at the reference's size: params + LAMB m, v of ALBERT-large
(3 x 17.8M fp32 = 214 MB).  The donor keeps training while it serves: ``step()`` may wait only for
the on-device snapshot, never for the transfer itself."""
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

        def timed_snapshot():  # what the server does under the donor's step lock
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
        assert len(during) >= 2, "the donor must keep stepping while it serves its state"
        # the donor's step lock is held for the snapshot only (a clone), then released for the
        # transfer: a step can be delayed by at most one snapshot, never by the transfer
        assert len(snap) == 1
        assert max(during) < typical + snap[0] + 0.2, (max(during), typical, snap[0], transfer)
    finally:
        co.shutdown()
        dht.shutdown()
