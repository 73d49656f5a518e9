"""FusedLamb semantics on CPU: torch_optimizer's adam mode and torch-format optimizer state dicts."""
import math
import pytest

import torch

import dedloc_amd.ops  # noqa: F401
from dedloc_amd.optim.lamb import FusedLamb
from dedloc_amd.utils.flat import FlatParams

# ALBERT-like naming: no-decay parameters interleave with decayed ones in model order
NAMES = [("emb.weight", (7, 5)), ("emb.LayerNorm.weight", (5,)), ("dense.weight", (3, 5)), ("dense.bias", (3,)),
         ("out.weight", (4, 3))]
NO_DECAY = {"emb.LayerNorm.weight", "dense.bias"}


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(n, torch.nn.Parameter(torch.randn(*s, generator=g))) for n, s in NAMES]


def test_lamb_adam_mode_has_unit_trust_ratio():
    named = _params()
    ref = {n: p.detach().clone() for n, p in named}
    flat = FlatParams(named, with_bf16=False)
    lr, wd, eps, (b1, b2) = 1e-2, 0.01, 1e-6, (0.9, 0.999)
    opt = FusedLamb(flat, lr=lr, weight_decay=wd, eps=eps, betas=(b1, b2), clamp_value=10.0, adam=True,
                    no_decay=NO_DECAY)
    m = {n: torch.zeros_like(p) for n, p in ref.items()}
    v = {n: torch.zeros_like(p) for n, p in ref.items()}
    g = torch.Generator().manual_seed(1)
    for t in range(1, 4):
        grads = {n: torch.randn(p.shape, generator=g) for n, p in ref.items()}
        for n in flat.names:
            flat.g(n).copy_(grads[n])
        opt.step()
        bc = math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        for n, p in ref.items():  # torch_optimizer.Lamb(adam=True, debias=True): trust_ratio = 1
            m[n].mul_(b1).add_(grads[n], alpha=1 - b1)
            v[n].mul_(b2).addcmul_(grads[n], grads[n], value=1 - b2)
            u = m[n] / (v[n].sqrt() + eps) + (0.0 if n in NO_DECAY else wd) * p
            p.add_(u, alpha=-lr * bc)
    for n, p in ref.items():
        torch.testing.assert_close(flat.p(n), p, rtol=1e-5, atol=1e-6)


def test_lamb_loads_torch_format_state_dict():
    # a torch optimizer with the reference's two groups (decayed first, then no-decay) numbers its
    # state group by group: ids 0..2 decayed, 3..4 no-decay — not the model order
    named_t = _params()
    decay = [p for n, p in named_t if n not in NO_DECAY]
    no_decay = [p for n, p in named_t if n in NO_DECAY]
    topt = torch.optim.Adam([{"params": decay, "weight_decay": 0.01}, {"params": no_decay, "weight_decay": 0.0}],
                            lr=3e-3)
    for _, p in named_t:
        p.grad = torch.randn_like(p)
    topt.step()
    sd = topt.state_dict()
    assert sd["param_groups"][1]["params"] == [3, 4]

    flat = FlatParams(_params(), with_bf16=False)
    opt = FusedLamb(flat, lr=1e-3, weight_decay=0.01, no_decay=NO_DECAY)
    opt.load_state_dict(sd)
    by_name = {n: topt.state[p] for n, p in named_t}
    for n in flat.names:
        torch.testing.assert_close(flat.view(opt.exp_avg, n), by_name[n]["exp_avg"])
        torch.testing.assert_close(flat.view(opt.exp_avg_sq, n), by_name[n]["exp_avg_sq"])
    assert opt.step_count == 1 and opt.lr == 3e-3

    # ... and our state dict loads back into a torch optimizer with the same groups
    ours = opt.state_dict()
    named_2 = _params()
    topt2 = torch.optim.Adam([{"params": [p for n, p in named_2 if n not in NO_DECAY], "weight_decay": 0.01},
                              {"params": [p for n, p in named_2 if n in NO_DECAY], "weight_decay": 0.0}], lr=1.0)
    ours["state"] = {k: dict(s, step=torch.tensor(float(s["step"]))) for k, s in ours["state"].items()}
    topt2.load_state_dict(ours)
    for (n, p2) in named_2:
        torch.testing.assert_close(topt2.state[p2]["exp_avg"], by_name[n]["exp_avg"])

    # our own round trip
    flat3 = FlatParams(_params(), with_bf16=False)
    opt3 = FusedLamb(flat3, lr=1e-3, weight_decay=0.01, no_decay=NO_DECAY)
    opt3.load_state_dict(opt.state_dict())
    assert torch.equal(opt3.exp_avg, opt.exp_avg) and torch.equal(opt3.exp_avg_sq, opt.exp_avg_sq)


def test_eta_slack_readiness_rule():
    """CollaborativeOptimizer's ETA slack: begin the global step at the local step boundary nearest
    to the collaboration's ETA instead of the first one after it (0 = hivemind's rule)."""

    from dedloc_amd.dht import DHT, get_dht_time
    from dedloc_amd.optim.collaborative import CollaborationState, CollaborativeOptimizer

    dht = DHT(listen_on="127.0.0.1:*")
    try:
        flat = FlatParams(_params(), with_bf16=False)
        opt = FusedLamb(flat, lr=1e-3)
        co = CollaborativeOptimizer(opt, dht=dht, prefix="slack", target_batch_size=64, batch_size_per_step=4,
                                    start=False, eta_slack=0.5, allow_state_sharing=False)
        co.performance_ema.samples_per_second = 40.0  # one local step of 4 samples = 0.1 s
        now = get_dht_time()
        co.collaboration_state = CollaborationState(0, 40, 64, num_peers=4, num_clients=0, eta_next_step=now + 0.04,
                                                    next_fetch_time=now + 10)
        assert not co.collaboration_state.ready_for_step      # hivemind's rule would run one more step
        assert co._ready_within_slack(4)                       # the ETA is closer than half a step
        co.collaboration_state.eta_next_step = now + 0.2
        assert not co._ready_within_slack(4)                   # two local steps away: keep accumulating
        co.eta_slack = 0.0
        co.collaboration_state.eta_next_step = now + 0.04
        assert not co._ready_within_slack(4)
        co.eta_slack = 0.5
        co.collaboration_state.num_peers = 1                   # alone: nobody to wait for
        assert not co._ready_within_slack(4)
        co.shutdown()
    finally:
        dht.shutdown()


@pytest.mark.parametrize("start", [False, True])
def test_single_peer_steps_exactly_at_target(start):
    """A lone peer knows its own sample count exactly: the global step happens at the local step that
    reaches target_batch_size, not one local step later when a (stale) DHT progress record catches up
    (which made every bench.py N=1 global step 9 micro-steps of 512 instead of 8)."""
    import time

    from dedloc_amd.dht import DHT
    from dedloc_amd.optim.collaborative import CollaborativeOptimizer

    dht = DHT(listen_on="127.0.0.1:*")
    try:
        flat = FlatParams(_params(), with_bf16=False)
        opt = FusedLamb(flat, lr=1e-3)
        co = CollaborativeOptimizer(opt, dht=dht, prefix=f"exact{int(start)}", target_batch_size=8,
                                    batch_size_per_step=2, start=start, allow_state_sharing=False,
                                    min_refresh_period=0.05, default_refresh_period=0.1)
        for call in range(1, 13):
            flat.grad.normal_()
            co.step()
            assert co.local_step == call // 4, (call, co.local_step)
            if start:
                time.sleep(0.03)
        assert co.stats["local_steps"] == 12 and co.stats["global_steps"] == 3
        co.shutdown()
    finally:
        dht.shutdown()


def test_lamb_weight_decay_zero_keeps_two_groups():
    """at weight_decay = 0 the groups must still be [decayed, no_decay] (by name), so a
    reference / HF optimizer.pt (always two groups) loads and our state_dict has the same layout."""
    named_t = _params()
    decay = [p for n, p in named_t if n not in NO_DECAY]
    no_decay = [p for n, p in named_t if n in NO_DECAY]
    topt = torch.optim.Adam([{"params": decay, "weight_decay": 0.0}, {"params": no_decay, "weight_decay": 0.0}],
                            lr=3e-3)
    for _, p in named_t:
        p.grad = torch.randn_like(p)
    topt.step()
    flat = FlatParams(_params(), with_bf16=False)
    opt = FusedLamb(flat, lr=1e-3, weight_decay=0.0, no_decay=NO_DECAY)
    sd = opt.state_dict()
    assert [len(g["params"]) for g in sd["param_groups"]] == [3, 2]
    opt.load_state_dict(topt.state_dict())  # must not raise a group-size mismatch
    by_name = {n: topt.state[p] for n, p in named_t}
    for n in flat.names:
        torch.testing.assert_close(flat.view(opt.exp_avg, n), by_name[n]["exp_avg"])


def test_nonfinite_microstep_does_not_count_samples(tmp_path):
    """A micro-step with non-finite gradients is dropped (its gradient zeroed on the device) and,
    like the reference's GradScaler skipping ``step()``, its samples and micro-step do not count
    toward the global batch: ``local_samples_accumulated`` stays unchanged."""
    from dedloc_amd.cli.arguments import AlbertTrainingArguments, CollaborationArguments, DatasetArguments
    from dedloc_amd.dht import DHT
    from dedloc_amd.models.albert import AlbertConfig
    from dedloc_amd.training.albert_peer import AlbertPeer

    cfg = tmp_path / "cfg"
    AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64).save_pretrained(str(cfg))
    root = DHT(listen_on="127.0.0.1:*")
    peer = None
    try:
        targs = AlbertTrainingArguments(per_device_train_batch_size=2, gradient_accumulation_steps=1, seq_length=64, save_steps=0,
                                        output_dir=str(tmp_path / "out"), seed=0)
        cargs = CollaborationArguments(experiment_prefix="nan", initial_peers=[root.endpoint],
                                       dht_listen_on="127.0.0.1:*", target_batch_size=64, listen_on="127.0.0.1:*")
        peer = AlbertPeer(targs, DatasetArguments(config_path=str(cfg)), cargs, torch.device("cpu"))
        co = peer.collab_opt
        peer.train_step()
        assert co.local_samples_accumulated == 2 and co.local_steps_accumulated == 1
        acc = co.accumulator.clone()
        with torch.no_grad():  # poison the parameters: the next backward yields NaN gradients
            peer.model.flat.fp32.fill_(float("nan"))
            peer.model.flat.refresh_bf16()
        peer.train_step()
        assert co.local_samples_accumulated == 2 and co.local_steps_accumulated == 1
        assert co.stats["nonfinite_steps"] == 1
        torch.testing.assert_close(co.accumulator, acc)  # the zeroed gradient added nothing
    finally:
        if peer is not None:
            peer.shutdown()
        root.shutdown()
