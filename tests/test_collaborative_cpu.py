"""Multi-peer collaborative training on CPU (gloo world, 2-3 processes, tiny ALBERT).

Covers the reference's core loop end to end: DHT progress tracking, ETA-driven global steps,
matchmaking, butterfly all-reduce with LP parts, LAMB, metrics publishing, state download for a
late joiner, and an auxiliary (reducer-only) peer.
"""
import multiprocessing as mp
import os
import socket
import time

import pytest
import torch

pytestmark = pytest.mark.multiproc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _peer(rank, world, port, dht_ep, out_q, cfg, mode=""):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import logging

    logging.basicConfig(level=int(os.environ.get("DEDLOC_TEST_LOGLEVEL", logging.WARNING)))
    from dedloc_amd.cli.arguments import AlbertTrainingArguments, CollaborationArguments, DatasetArguments
    from dedloc_amd.parallel import init_world
    from dedloc_amd.training.albert_peer import AlbertPeer

    rank_, world_, dev = init_world(backend="gloo", device=torch.device("cpu"))
    targs = AlbertTrainingArguments(per_device_train_batch_size=2, gradient_accumulation_steps=1, seq_length=64,
                                    warmup_steps=2, max_steps=1000, learning_rate=3e-3, save_steps=0,
                                    output_dir=f"/tmp/dedloc_test_out_{port}_{rank}", seed=rank)
    dargs = DatasetArguments(config_path=cfg)
    aux = rank in cfg_aux(world) and mode == ""
    cargs = CollaborationArguments(experiment_prefix="test", initial_peers=[dht_ep], dht_listen_on="127.0.0.1:*",
                                   target_batch_size=8, averaging_expiration=3.0, compression="NONE",
                                   min_refresh_period=0.05, default_refresh_period=0.2, metadata_expiration=20,
                                   listen_on="127.0.0.1:*", bandwidth=100.0 + 50 * rank)
    late = rank == world - 1 and world == 3 and not aux and mode == ""
    if mode == "kill":
        aux = False
    if mode == "delay":
        cargs.delay_param_averaging = True
    elif mode == "hetero":
        targs.peer_batch_sizes, targs.peer_slowdowns = "2,1,3", "1,2,1"
        cargs.peer_bandwidths = "200,50,100"
    elif mode == "churn":
        targs.peer_churn = ";;restart@2:2"  # rank 2 is preempted after global step 2 and respawned 2 s later
        targs.throttle = 0.1  # keep the survivors training (and serving state) while rank 2 is away
    elif mode == "kill":
        cargs.metadata_expiration = 6.0  # the dead peer drops out of the collaboration quickly
        cargs.averaging_timeout = 4.0
    if late:
        targs.throttle = 0.0
    elif mode != "churn":
        targs.throttle = 0.05 if world == 3 else 0.0  # keep the early peers busy long enough to overlap
    peer = None
    if late:
        time.sleep(2.0)  # late joiner: must download state
    peer = AlbertPeer(targs, dargs, cargs, dev, pg=None, rank=rank_, auxiliary=aux)
    res = {"rank": rank}
    try:
        if aux:
            t0 = time.time()
            while time.time() - t0 < 20 and peer.collab_opt.local_step < 6:
                peer.collab_opt.step_aux()
                time.sleep(0.05)
        else:
            steps = 3 if world == 2 else (6 if late else 12)
            if mode == "churn":
                steps = 8 if rank == 2 else 20
            if mode == "kill" and rank == 2:
                # a real process death (no clean-up, no tombstone) in the middle of training
                peer.train(max_steps=600, stop_after_global_steps=2, max_seconds=60)
                os.kill(os.getpid(), 9)
            if mode == "kill":
                steps = 8
            peer.train(max_steps=600, stop_after_global_steps=steps, max_seconds=60 if mode != "churn" else 90)
            peer.collab_opt._finish_param_round()
        res["local_step"] = peer.collab_opt.local_step
        res["stats"] = dict(peer.collab_opt.stats)
        res["params"] = peer.model.flat.fp32.clone()
        res["metrics"] = peer.metrics_log
        res["state_loads"] = peer.collab_opt.stats["state_loads"]
        res["batch"] = peer.args.per_device_train_batch_size
        res["bandwidth"] = peer.cargs.bandwidth
        res["churned"] = getattr(peer, "stats_churn", 0)
    finally:
        out_q.put(res)
        time.sleep(2.0)  # keep serving state/averaging for the others a little longer
        peer.shutdown()


def cfg_aux(world):
    return {1} if world == 3 else set()


def _tiny_cfg(tmp_path):
    from dedloc_amd.models.albert import AlbertConfig

    cfg = AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64)
    d = tmp_path / "cfg"
    cfg.save_pretrained(str(d))
    return str(d)


def _run(world, tmp_path, mode="", expect=None):
    from dedloc_amd.dht import DHT

    root = DHT(listen_on="127.0.0.1:*")
    port = _free_port()
    cfg = _tiny_cfg(tmp_path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_peer, args=(r, world, port, root.endpoint, q, cfg, mode)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world if expect is None else expect)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    root.shutdown()
    return sorted(results, key=lambda r: r["rank"])


@pytest.mark.timeout(300)
def test_two_peers_average_and_stay_synchronized(tmp_path):
    res = _run(2, tmp_path)
    for r in res:
        assert r["local_step"] >= 3, r
        assert r["stats"]["averaging_rounds"] >= 1
    # compression NONE + identical starting state (state download) => bitwise-close params
    d = (res[0]["params"] - res[1]["params"]).abs().max().item()
    failed = sum(r["stats"]["averaging_failed"] for r in res)
    # a timed-out matchmaking round legitimately applies local gradients (reference behaviour), which
    # leaves the optimizer states slightly apart; otherwise the peers must be bitwise close
    assert d < (1e-5 if failed == 0 else 5e-2), (d, [r["stats"] for r in res])
    assert all(m["loss"] > 0 for r in res for m in r["metrics"][1:])


@pytest.mark.timeout(300)
def test_aux_peer_and_late_joiner(tmp_path):
    res = _run(3, tmp_path)
    trainer0, aux, late = res
    assert trainer0["local_step"] >= 6 and late["local_step"] >= 6
    assert late["state_loads"] >= 1  # joined late -> downloaded state
    assert late["metrics"][0]["step"] > 0  # ... and resumed at the collaboration's step, not 0
    # once two trainers overlap they average (with the auxiliary peer as an extra reducer)
    assert late["stats"]["averaging_rounds"] >= 1
    assert aux["local_step"] >= 1


@pytest.mark.timeout(300)
def test_delayed_parameter_averaging(tmp_path):
    res = _run(2, tmp_path, mode="delay")
    for r in res:
        assert r["local_step"] >= 3, r
        assert r["stats"].get("param_rounds", 0) >= 1, r["stats"]
    failed = sum(r["stats"]["averaging_failed"] + r["stats"].get("param_rounds_failed", 0) for r in res)
    d = (res[0]["params"] - res[1]["params"]).abs().max().item()
    assert d < (1e-5 if failed == 0 else 5e-2), (d, [r["stats"] for r in res])


@pytest.mark.timeout(300)
def test_heterogeneous_peers(tmp_path):
    res = _run(3, tmp_path, mode="hetero")
    assert [r["batch"] for r in res] == [2, 1, 3]
    assert [r["bandwidth"] for r in res] == [200.0, 50.0, 100.0]
    for r in res:
        assert r["local_step"] >= 6, r
    assert sum(r["stats"]["averaging_rounds"] for r in res) >= 3


@pytest.mark.timeout(300)
def test_churn_restart_rejoins_through_state_download(tmp_path):
    res = _run(3, tmp_path, mode="churn")
    survivor, _, churned = res
    assert churned["churned"] == 1
    assert churned["state_loads"] >= 1  # lost its state -> downloaded it from a live peer
    assert churned["local_step"] >= 8 and survivor["local_step"] >= 8
    assert survivor["stats"]["global_steps"] >= 8  # the others kept training while it was away


@pytest.mark.timeout(300)
def test_peer_process_death_survivors_continue(tmp_path):
    """A peer process is SIGKILLed mid-training (no tombstone, group communicator left dangling):
    the survivors' round with it fails, they abort that communicator, move to a new data-plane
    epoch and keep making global steps — averaging with each other once the dead peer's progress
    record expires."""
    res = _run(3, tmp_path, mode="kill", expect=2)
    assert [r["rank"] for r in res] == [0, 1]
    for r in res:
        assert r["local_step"] >= 8, r
    # after the death the two survivors averaged together again (group of 2 on a fresh epoch)
    assert all(r["stats"]["averaging_rounds"] - r["stats"]["averaging_failed"] >= 3 for r in res), \
        [r["stats"] for r in res]
    d = (res[0]["params"] - res[1]["params"]).abs().max().item()
    assert d < 5e-2, d
