"""The sahajBERT-config micro-step issues no host synchronisation.

sahajBERT trains on Bernoulli-masked streaming data (``mask_mode="hf"``, variable-length rows,
vocabulary 31,995; reference ``sahajbert/run_trainer.py:215-300``).  The HF ``labels`` form would
make the MLM head call ``torch.nonzero`` — a device->host sync per micro-step — so both the
synthetic stream and the host collator (``collate_mlm``, shared by the disk and streaming sources)
also emit fixed-shape ``mlm_positions`` / ``mlm_labels``.  Checked with torch's sync debug mode set
to "error" around forward + backward + clip + accumulate, after a positive control proves the mode
catches a synchronising call on this build."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(B, V, seed=0):
    g = torch.Generator().manual_seed(seed)
    rows = {"input_ids": [], "token_type_ids": [], "special_tokens_mask": [], "sentence_order_label": []}
    for i in range(B):
        n = int(torch.randint(40, 512, (1,), generator=g))
        ids = [2] + torch.randint(5, V, (n - 2,), generator=g).tolist() + [3]
        split = n // 2
        rows["input_ids"].append(ids)
        rows["token_type_ids"].append([0] * split + [1] * (n - split))
        rows["special_tokens_mask"].append([1] + [0] * (n - 2) + [1])
        rows["sentence_order_label"].append(i % 2)
    return rows


@pytest.mark.timeout(300)
def test_sahajbert_micro_step_has_no_host_sync(cuda):
    from dedloc_amd.data.sop_dataset import collate_mlm
    from dedloc_amd.data.synthetic_mlm import SyntheticSOPStream
    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining

    cfg = AlbertConfig.from_pretrained("albert-large-v2")
    cfg.vocab_size = 31995
    model = AlbertForPreTraining(cfg)
    flat = model.materialize(cuda)
    model.train()
    part, out = torch.zeros(256, device=cuda), torch.zeros(2, device=cuda)
    acc = torch.zeros_like(flat.grad)
    meta = {"pad": 0, "mask": 4, "vocab_size": cfg.vocab_size}
    synthetic = SyntheticSOPStream(4, 512, cfg.vocab_size, seed=0, device=cuda, mask_mode="hf",
                                   length_mode="wikitext")
    batches = [synthetic.next_batch(), collate_mlm(_rows(4, cfg.vocab_size), meta, torch.Generator().manual_seed(1),
                                                   device=cuda)]

    def micro_step(b):
        o = model(b["input_ids"], b["attention_mask"], b["token_type_ids"], labels=b.get("labels"),
                  sentence_order_label=b["sentence_order_label"], mlm_positions=b.get("mlm_positions"),
                  mlm_labels=b.get("mlm_labels"))
        o["loss"].backward()
        torch.ops.dedloc.grad_norm_clip(flat.grad, 1.0, part, out)
        torch.ops.dedloc.axpby(acc, flat.grad, 1.0, 1.0)
        flat.zero_grad()
        return o["loss"]

    for b in batches:  # warm-up outside the check (first-call workspace allocations, plans)
        assert "mlm_positions" in b and "labels" in b
        micro_step(b)
    torch.cuda.synchronize()
    prev = torch.cuda.get_sync_debug_mode()
    torch.cuda.set_sync_debug_mode("error")
    try:
        with pytest.raises(RuntimeError):  # positive control: the HF labels path syncs
            torch.nonzero(batches[0]["labels"].reshape(-1) != -100)
        losses = [micro_step(b) for b in batches]
    finally:
        torch.cuda.set_sync_debug_mode(prev)
    assert all(torch.isfinite(l).item() for l in losses)


@pytest.mark.timeout(300)
def test_collaborative_global_step_has_no_host_sync(cuda):
    """A lone peer's micro-steps AND its global step (gradient divide by the device-side finite
    count, LAMB, snapshot, device-timed PerformanceEMA) queue work without waiting for the GPU —
    round 4 drained the queue at every global step to count finite samples on the host."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.optim.collaborative import CollaborativeOptimizer
    from dedloc_amd.optim.lamb import FusedLamb
    from dedloc_amd.utils.flat import FlatParams

    lin = torch.nn.Linear(256, 512).to(cuda)
    flat = FlatParams(lin.named_parameters(), device=cuda)
    opt = FusedLamb(flat, lr=1e-3)
    dht = DHT(listen_on="127.0.0.1:*")
    co = CollaborativeOptimizer(opt, dht=dht, prefix="nosync", target_batch_size=8, batch_size_per_step=4,
                                start=False, listen_on="127.0.0.1:*", peer_id=b"solo")
    try:
        finite = torch.ones(1, device=cuda)
        for _ in range(4):  # warm-up: cached device scalars, first global steps
            flat.grad.normal_()
            co.step(batch_size=4, finite=finite)
        torch.cuda.synchronize()
        step0 = co.local_step
        torch.cuda.set_sync_debug_mode("error")
        try:
            for _ in range(4):
                flat.grad.normal_()
                co.step(batch_size=4, finite=finite)
        finally:
            torch.cuda.set_sync_debug_mode("default")
        assert co.local_step == step0 + 2
        torch.cuda.synchronize()
        co._device_timer.poll()
        assert co._device_timer.updates >= 4 and co.performance_ema.samples_per_second > 0
    finally:
        co.shutdown()
        dht.shutdown()
