"""Single-process unit tests of CollaborativeOptimizer / averaging details.

* a prejoined matchmaking future is bound to the global step it was made for: a peer that goes out
  of sync drops it, and the next global step matches afresh instead of handing a stale group to
  the averager;
* the global step's averaging weight and gradient divisor are device scalars counting finite
  micro-steps only, so the global step never waits for the host;
* a group whose weights sum to 0 is a no-op round (zero deltas), never "adopt member 0";
* CPU members of a mixed (RCCL + gloo) group get a load-balanced part even without --bandwidth.
"""
import time
from concurrent.futures import Future

import pytest
import torch

import dedloc_amd.ops  # noqa: F401  (CPU implementations of the dedloc:: operators)
from dedloc_amd.dht import DHT
from dedloc_amd.optim.collaborative import CollaborationState, CollaborativeOptimizer
from dedloc_amd.optim.lamb import FusedLamb
from dedloc_amd.utils.flat import FlatParams


@pytest.fixture
def collab():
    root = DHT(listen_on="127.0.0.1:*")
    lin = torch.nn.Linear(16, 8)
    flat = FlatParams(lin.named_parameters(), device=torch.device("cpu"), with_bf16=False)
    opt = FusedLamb(flat, lr=1e-3)
    co = CollaborativeOptimizer(opt, dht=root, prefix="unit", target_batch_size=8, batch_size_per_step=4,
                                start=False, listen_on="127.0.0.1:*", peer_id=b"me")
    yield co, flat
    co.shutdown()
    root.shutdown()


def _state(co, step, samples=0, peers=2):
    return CollaborationState(step, samples, co.target_batch_size, num_peers=peers, num_clients=0,
                              eta_next_step=float("inf"), next_fetch_time=time.time() + 60, own_samples=0)


def test_prejoin_dropped_when_out_of_sync_then_fresh_matchmaking(collab, monkeypatch):
    co, flat = collab
    calls = []

    def fake_step(weight=1.0, prejoined=None, **kw):
        calls.append({"weight": weight, "prejoined": prejoined})
        return None

    monkeypatch.setattr(co.averager, "step", fake_step)
    monkeypatch.setattr(co, "load_state_from_peers", lambda **kw: co._drop_prejoin() or False)
    # a prejoin made at step 0 ...
    stale = Future()
    co._prejoin, co._prejoin_key = stale, (0, time.monotonic())
    # ... then the collaboration moves on: this peer is out of sync and must drop it
    co.collaboration_state = _state(co, step=5)
    assert not co.is_synchronized
    co.step(batch_size=4)
    assert co._prejoin is None and co.stats.get("prejoins_dropped") == 1
    # resynchronised at step 5: a full global batch averages with FRESH matchmaking
    co.local_step = 5
    monkeypatch.setattr(co, "fetch_collaboration_state", lambda: _state(co, step=5, samples=8))
    co.collaboration_state = _state(co, step=5, samples=8)
    flat.grad.fill_(1.0)
    co.step(batch_size=4)
    assert len(calls) == 1 and calls[0]["prejoined"] is None
    assert co.local_step == 6


def test_prejoin_for_an_older_step_is_not_used(collab, monkeypatch):
    co, flat = collab
    seen = []
    monkeypatch.setattr(co.averager, "step", lambda weight=1.0, prejoined=None, **kw: seen.append(prejoined))
    monkeypatch.setattr(co, "fetch_collaboration_state", lambda: _state(co, step=co.local_step, samples=8))
    co.collaboration_state = _state(co, step=0, samples=8)
    old = Future()
    co._prejoin, co._prejoin_key = old, (0, time.monotonic() - 3600)  # made an hour ago
    co.step(batch_size=4)
    assert seen == [None] and co.stats["prejoins_dropped"] == 1
    fresh = Future()
    co.collaboration_state = _state(co, step=1, samples=8)
    co._prejoin, co._prejoin_key = fresh, (1, time.monotonic())
    co.step(batch_size=4)
    assert seen[-1] is fresh


def test_weight_and_divisor_count_finite_micro_steps_on_device(collab, monkeypatch):
    co, flat = collab
    got = {}

    def fake_step(weight=1.0, **kw):
        got["weight"] = weight
        got["grad"] = flat.grad.clone()
        return None

    monkeypatch.setattr(co.averager, "step", fake_step)
    monkeypatch.setattr(co, "fetch_collaboration_state", lambda: _state(co, step=0, samples=12))
    co.target_batch_size = 12
    co.collaboration_state = _state(co, step=0, samples=0)
    flat.grad.fill_(2.0)
    co.step(batch_size=4, finite=torch.ones(1))
    flat.grad.zero_()  # a non-finite micro-step: its gradient was zeroed, its flag is 0
    co.step(batch_size=4, finite=torch.zeros(1))
    co.collaboration_state = _state(co, step=0, samples=12)
    flat.grad.fill_(4.0)
    co.step(batch_size=4, finite=torch.ones(1))
    # 2 finite micro-steps of 4 samples out of 3: grad = (2 + 4) / 2, weight = 8 / (12 / 2 peers)
    assert isinstance(got["weight"], torch.Tensor)
    assert float(got["weight"]) == pytest.approx(8 / 6)
    torch.testing.assert_close(got["grad"], torch.full_like(flat.grad, 3.0))
    assert float(co._finite_counts.sum()) == 0.0  # reset for the next global batch


def test_all_zero_weights_leave_tensors_unchanged():
    from dedloc_amd.averaging.allreduce import GroupSpec, butterfly_allreduce

    x = torch.randn(64)
    before = x.clone()
    spec = GroupSpec(ranks=[0], part_sizes=[64], weights=[0.0], contributes=[True], my_index=0)
    butterfly_allreduce([x], spec, "FLOAT16", comm=None)
    torch.testing.assert_close(x, before, rtol=0, atol=0)
    parts = torch.stack([torch.randn(32), torch.randn(32)]).half()
    deltas = torch.full_like(parts, 7.0)
    torch.ops.dedloc.reduce_delta(parts, torch.zeros(2), deltas)
    assert float(deltas.abs().max()) == 0.0


def test_mixed_group_part_sizes():
    """Mixed group (2 GPU members on RCCL + 1 CPU member on gloo): the LP minimises the slowest
    member, so a CPU member with no declared --bandwidth (a 10 Gb/s host link by default) owns no
    part next to xGMI peers — it then neither sends nor receives and cannot slow them down — while
    one that declares an xGMI-class link gets a real share; client mode (0) never owns a part."""
    from dedloc_amd.averaging.averager import DecentralizedAverager as DA
    from dedloc_amd.averaging.load_balancing import load_balance_peers

    pids = [b"a", b"b", b"c"]
    gpu = {b"a", b"b"}
    infos = [{"bandwidth": None}, {"bandwidth": None}, {"bandwidth": None}]
    bws = DA.group_bandwidths(infos, pids, gpu)
    assert bws == [DA.XGMI_MBPS, DA.XGMI_MBPS, DA.DEFAULT_HOST_MBPS]
    parts = load_balance_peers(1_000_000, bws, min_size=0)
    assert sum(parts) == 1_000_000 and parts[2] == 0 and abs(parts[0] - parts[1]) <= 1
    infos[2]["bandwidth"] = 2 * DA.XGMI_MBPS
    parts = load_balance_peers(1_000_000, DA.group_bandwidths(infos, pids, gpu), min_size=0)
    assert parts[2] > 100_000
    infos[2]["bandwidth"] = 0.0  # client mode
    assert load_balance_peers(1000, DA.group_bandwidths(infos, pids, gpu), min_size=0)[2] == 0
    # a homogeneous group of undeclared peers splits evenly
    even = load_balance_peers(1000, DA.group_bandwidths([{"bandwidth": None}] * 2, [b"x", b"y"], None))
    assert even == (500, 500)


def test_imminent_global_step_refreshes_the_view_instead_of_overshooting(collab, monkeypatch):
    """A prejoin made for this step means this micro-step is expected to complete the batch: when
    the (stale) view says "not ready", step() refreshes the collaboration view once (on a GPU after
    waiting for the micro-step on the device) and runs the global step in the same call — instead
    of returning and letting every peer queue one more micro-step past the target."""
    co, flat = collab
    seen = []
    monkeypatch.setattr(co.averager, "step", lambda weight=1.0, prejoined=None, **kw: seen.append(prejoined))
    monkeypatch.setattr(co.averager, "prejoin", lambda **kw: Future())  # no background matchmaking
    fetches = []

    def fetch():
        fetches.append(1)
        return _state(co, step=0, samples=8)  # the other peer's samples are visible now

    monkeypatch.setattr(co, "fetch_collaboration_state", fetch)
    co.collaboration_state = _state(co, step=0, samples=0)  # stale: nobody has reported yet
    fut = Future()
    co._prejoin, co._prejoin_key = fut, (0, time.monotonic())
    flat.grad.fill_(1.0)
    co.step(batch_size=4)
    assert co.local_step == 1 and seen == [fut]
    assert len(fetches) == 1  # the refresh doubles as the global step's fetch
    # without a pending prejoin a stale "not ready" view simply returns (no refresh)
    co._drop_prejoin()
    co.collaboration_state = _state(co, step=1, samples=0)
    co.step(batch_size=4)
    assert co.local_step == 1 and len(fetches) == 1


def test_imminent_wait_happens_once_per_global_step(collab, monkeypatch):
    co, flat = collab
    monkeypatch.setattr(co.averager, "step", lambda **kw: None)
    fetches = []
    monkeypatch.setattr(co, "fetch_collaboration_state",
                        lambda: fetches.append(1) or _state(co, step=0, samples=0))  # never ready
    co.target_batch_size = 100
    co.collaboration_state = _state(co, step=0, samples=0)
    co._prejoin, co._prejoin_key = Future(), (0, time.monotonic())
    for _ in range(4):
        co.step(batch_size=4)
    assert co.local_step == 0 and len(fetches) == 1


def test_successful_round_adopts_the_largest_gathered_step(collab, monkeypatch):
    """hivemind 0.9.x: a peer that averaged with a member one step ahead takes that member's step,
    so step counters inside one group never stay apart (a lagging peer's prejoined groups would
    otherwise miss the others' at the end of a run)."""
    co, flat = collab
    co.local_step = 4
    co.collaboration_state = _state(co, step=5, samples=8)
    monkeypatch.setattr(co, "_refresh_state", lambda: None)
    monkeypatch.setattr(co.averager, "step", lambda **kw: {"group_id": 1, "size": 2, "gathered": [
        {"step": 4}, {"step": 5}], "backend": "gloo"})
    flat.grad.normal_()
    assert co.step(batch_size=4) is not None
    assert co.local_step == 6 and co.stats["steps_adopted"] == 1
    # a failed round adopts nothing
    co.collaboration_state = _state(co, step=6, samples=8)
    monkeypatch.setattr(co.averager, "step", lambda **kw: None)
    co.step(batch_size=4)
    assert co.local_step == 7 and co.stats["steps_adopted"] == 1
