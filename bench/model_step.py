"""Single-GPU micro-benchmark of one ALBERT-large training micro-step (fwd + bwd), no collaboration.

--impl dedloc : this framework's kernels (flat buffers, fused ops)
--impl hf     : HF transformers AlbertForPreTraining, bf16 autocast, PyTorch eager/SDPA —
                the "PyTorch-eager on MI355X" baseline BASELINE.md asks to record.
"""
import argparse
import json
import time

import torch


def synthetic(B, S, V, P, dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ids = torch.randint(5, V, (B, S), generator=g)
    tt = torch.zeros(B, S, dtype=torch.long)
    tt[:, S // 2:] = 1
    am = torch.ones(B, S, dtype=torch.long)
    pos = torch.stack([torch.randperm(S - 2, generator=g)[:P] + 1 for _ in range(B)])
    lab = torch.gather(ids, 1, pos)
    sop = torch.randint(0, 2, (B,), generator=g)
    labels = torch.full((B, S), -100, dtype=torch.long)
    labels.scatter_(1, pos, lab)
    return [t.to(dev) for t in (ids, tt, am, pos, lab, sop, labels)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", default="dedloc", choices=["dedloc", "hf"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda")
    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining, flops_per_sample

    cfg = AlbertConfig.albert_large_v2()
    P = round(0.15 * args.seq)
    ids, tt, am, pos, lab, sop, labels = synthetic(args.batch, args.seq, cfg.vocab_size, P, dev)
    if args.impl == "dedloc":
        model = AlbertForPreTraining(cfg)
        model.materialize(dev)
        model.train()

        def step():
            out = model(ids, am, tt, sentence_order_label=sop, mlm_positions=pos, mlm_labels=lab)
            out["loss"].backward()
            return out["loss"]
    else:
        import transformers

        hcfg = transformers.AlbertConfig(**{k: v for k, v in cfg.to_dict().items()
                                            if k not in ("architectures", "model_type")})
        model = transformers.AlbertForPreTraining(hcfg).to(dev).train()

        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(input_ids=ids, attention_mask=am, token_type_ids=tt, labels=labels,
                            sentence_order_label=sop)
            out.loss.backward()
            return out.loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    fl = flops_per_sample(cfg, args.seq, P) * args.batch
    print(json.dumps({"impl": args.impl, "batch": args.batch, "seq": args.seq, "ms_per_microstep": dt * 1e3,
                      "samples_per_s": args.batch / dt, "tflops": fl / dt / 1e12, "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
