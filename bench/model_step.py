"""Single-GPU micro-benchmark of one ALBERT-large training micro-step (fwd + bwd), no collaboration.

--impl dedloc : this framework's kernels (flat buffers, fused ops)
--impl hf     : HF transformers AlbertForPreTraining, bf16 autocast, PyTorch eager/SDPA —
                the "PyTorch-eager on MI355X" baseline BASELINE.md asks to record.
"""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
import argparse
import math
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
    ap.add_argument("--config", default="albert-large-v2",
                    help="albert-large-v2 | albert-base-v2 | albert-xlarge-v2 | albert-xxlarge-v2 | a config.json directory")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--with_optimizer", action="store_true",
                    help="include clip + LAMB every micro-step (upper bound on optimizer cost)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining, flops_per_sample

    cfg = AlbertConfig.from_pretrained(args.config)
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
        params = [p for p in model.parameters() if p.requires_grad]
        state = {id(p): (torch.zeros_like(p), torch.zeros_like(p)) for p in params}
        t_opt = [0]

        @torch.no_grad()
        def eager_lamb(lr=1.76e-3, b1=0.9, b2=0.999, eps=1e-6, wd=0.01, clamp=1e4):
            # torch_optimizer.Lamb(debias=True) written with per-tensor torch ops (reference behaviour)
            t_opt[0] += 1
            t = t_opt[0]
            bc = math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
            for p in params:
                if p.grad is None:
                    continue
                m, v = state[id(p)]
                m.mul_(b1).add_(p.grad, alpha=1 - b1)
                v.mul_(b2).addcmul_(p.grad, p.grad, value=1 - b2)
                wn = p.norm().clamp(0, clamp)
                u = m / (v.sqrt() + eps) + wd * p
                un = u.norm()
                trust = torch.where((wn > 0) & (un > 0), wn / un, torch.ones_like(wn))
                p.add_(u * (-lr * bc * trust))

        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(input_ids=ids, attention_mask=am, token_type_ids=tt, labels=labels,
                            sentence_order_label=sop)
            out.loss.backward()
            if args.with_optimizer:
                torch.nn.utils.clip_grad_norm_(params, 1.0)
                eager_lamb()
                model.zero_grad(set_to_none=False)
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
