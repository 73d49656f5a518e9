"""Same-process A/B of ALBERT-large micro-step variants (cdna_hip_programming.md §5.4 rule 24:
interleaved rounds in ONE process; box-to-box spread on this pool is up to ~10%).

    python bench/ab_step.py --batch 256 --ab residual     # residual add in GEMM epilogue vs in LayerNorm
    python bench/ab_step.py --batch 256 --ab dgradwt      # dgrad GEMMs on transposed weight copies
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dedloc_amd.models.albert as albert  # noqa: E402
from bench.model_step import synthetic  # noqa: E402


def set_variant(ab, v):
    if ab == "residual":
        albert._RESIDUAL_IN_GEMM = v == "B"
    elif ab == "sharedwgrad":  # shared-layer weight-gradient slabs summed once per micro-step (B)
        albert._SHARED_WGRAD = v == "B"
    elif ab == "dgradwt":  # dgrad GEMMs against transposed weight copies (B) vs the plain weights (A)
        albert._DGRAD_WT = v == "B"
    else:
        raise ValueError(ab)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ab", default="residual")
    args = ap.parse_args()
    dev = torch.device("cuda")
    cfg = albert.AlbertConfig.albert_large_v2()
    P = round(0.15 * args.seq)
    ids, tt, am, pos, lab, sop, labels = synthetic(args.batch, args.seq, cfg.vocab_size, P, dev)
    model = albert.AlbertForPreTraining(cfg)
    model.materialize(dev)
    model.train()

    def step():
        out = model(ids, am, tt, sentence_order_label=sop, mlm_positions=pos, mlm_labels=lab)
        out["loss"].backward()
        return out["loss"]

    for v in ("A", "B"):  # warm-up (hipBLASLt autotune of every shape both variants use)
        set_variant(args.ab, v)
        for _ in range(2):
            step()
    torch.cuda.synchronize()
    times = {"A": [], "B": []}
    losses = {}
    for _ in range(args.rounds):
        for v in ("A", "B"):
            set_variant(args.ab, v)
            model.flat.zero_grad()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                loss = step()
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / args.iters)
            losses[v] = float(loss)
    res = {"ab": args.ab, "batch": args.batch}
    for v in ("A", "B"):
        best = min(times[v])
        res[v] = {"ms": round(best * 1e3, 2), "samples_per_s": round(args.batch / best, 1), "loss": round(losses[v], 5)}
    res["B_over_A"] = round(min(times["A"]) / min(times["B"]), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
