"""Downstream fine-tuning of a collaboratively pre-trained ALBERT (sahajBERT recipes).

Reference: ``sahajbert/train_ner.py`` (wikiann-bn token classification, seqeval entity F1) and
``sahajbert/train_ncc.py`` (indic_glue sna.bn news-category classification, accuracy); both run an
HF ``Trainer`` with per-epoch evaluation, ``EarlyStoppingCallback(patience, threshold)``,
``metric_for_best_model="loss"`` and ``load_best_model_at_end=True``, then evaluate on the test split.

Here the same loop runs on the dedloc ALBERT heads (``AlbertForTokenClassification`` /
``AlbertForSequenceClassification``: fused HIP encoder, fp32 flat gradients) with AdamW + linear
decay (the HF Trainer defaults).  There is no network, so the datasets are synthetic stand-ins of the
same label spaces (7 wikiann BIO tags, 6 sna.bn categories) whose labels are a learnable function of
the tokens; ``--model_path`` takes a checkpoint directory written by ``run_first_peer`` /
``save_pretrained`` (the pre-training heads are dropped, the new head is freshly initialised).

    python -m dedloc_amd.cli.finetune --task ner --model_path ckpt/ --output_dir out/
"""
from __future__ import annotations

import argparse
import copy
import json
import logging
import math
import os
from typing import Dict, List, Tuple

import torch

from ..models.albert import AlbertConfig, AlbertForSequenceClassification, AlbertForTokenClassification

logger = logging.getLogger(__name__)

NER_LABELS = ["O", "B-PER", "I-PER", "B-ORG", "I-ORG", "B-LOC", "I-LOC"]  # wikiann
NCC_LABELS = ["kolkata", "state", "national", "sports", "entertainment", "international"]  # sna.bn


# ------------------------------------------------------------------ synthetic task data
def synthetic_ner(n: int, seq_len: int, vocab: int, seed: int) -> List[Dict[str, torch.Tensor]]:
    """Token-classification examples: entity spans are runs of tokens from per-type vocabulary bands,
    tagged B-/I-; [CLS]/[SEP]/padding carry -100 like HF's tokenize_and_align_labels."""
    g = torch.Generator().manual_seed(seed)
    band = max(8, (vocab - 10) // 4)  # vocabulary bands: 0 = plain words, 1..3 = PER/ORG/LOC
    out = []
    for _ in range(n):
        length = int(torch.randint(seq_len // 2, seq_len - 1, (1,), generator=g))
        ids = torch.full((seq_len,), 0, dtype=torch.long)
        labels = torch.full((seq_len,), -100, dtype=torch.long)
        ids[0], labels[0] = 2, -100  # [CLS]
        i = 1
        while i < length - 1:
            if float(torch.rand(1, generator=g)) < 0.25:
                etype = int(torch.randint(1, 4, (1,), generator=g))
                span = int(torch.randint(1, 4, (1,), generator=g))
                for k in range(span):
                    if i >= length - 1:
                        break
                    ids[i] = 10 + etype * band + int(torch.randint(0, band, (1,), generator=g))
                    labels[i] = 2 * etype - 1 if k == 0 else 2 * etype
                    i += 1
            else:
                ids[i] = 10 + int(torch.randint(0, band, (1,), generator=g))
                labels[i] = 0
                i += 1
        ids[i], labels[i] = 3, -100  # [SEP]
        mask = torch.zeros(seq_len, dtype=torch.long)
        mask[: i + 1] = 1
        out.append({"input_ids": ids, "attention_mask": mask, "labels": labels})
    return out


def synthetic_ncc(n: int, seq_len: int, vocab: int, seed: int) -> List[Dict[str, torch.Tensor]]:
    """Sequence-classification examples: the category decides which vocabulary band the keywords of
    the article come from (the rest is shared filler)."""
    g = torch.Generator().manual_seed(seed)
    k = len(NCC_LABELS)
    band = max(8, (vocab - 10) // (k + 1))
    out = []
    for _ in range(n):
        label = int(torch.randint(0, k, (1,), generator=g))
        length = int(torch.randint(seq_len // 2, seq_len, (1,), generator=g))
        ids = 10 + torch.randint(0, band, (seq_len,), generator=g)
        kw = torch.rand(seq_len, generator=g) < 0.3
        ids = torch.where(kw, 10 + (label + 1) * band + torch.randint(0, band, (seq_len,), generator=g), ids)
        ids[0], ids[length - 1] = 2, 3
        ids[length:] = 0
        mask = (torch.arange(seq_len) < length).long()
        out.append({"input_ids": ids, "attention_mask": mask, "labels": torch.tensor(label)})
    return out


def batches(data, bs, shuffle, seed):
    idx = torch.randperm(len(data), generator=torch.Generator().manual_seed(seed)) if shuffle else torch.arange(len(data))
    for s in range(0, len(data), bs):
        rows = [data[int(i)] for i in idx[s:s + bs]]
        yield {k: torch.stack([r[k] for r in rows]) for k in rows[0]}


# ------------------------------------------------------------------ metrics
def _spans(tags: List[str]) -> set:
    """Entity spans of a BIO sequence (seqeval's default IOB2 semantics)."""
    spans, start, etype = set(), None, None
    for i, t in enumerate(tags + ["O"]):
        if t.startswith("B-") or t == "O" or (t.startswith("I-") and t[2:] != etype):
            if start is not None:
                spans.add((start, i, etype))
                start, etype = None, None
            if t.startswith("B-") or t.startswith("I-"):
                start, etype = i, t[2:]
    return spans


def ner_metrics(preds: List[List[str]], refs: List[List[str]]) -> Dict[str, float]:
    tp = fp = fn = 0
    correct = total = 0
    for p, r in zip(preds, refs):
        ps, rs = _spans(p), _spans(r)
        tp += len(ps & rs)
        fp += len(ps - rs)
        fn += len(rs - ps)
        correct += sum(a == b for a, b in zip(p, r))
        total += len(r)
    prec = tp / max(1, tp + fp)
    rec = tp / max(1, tp + fn)
    f1 = 2 * prec * rec / max(1e-12, prec + rec)
    return {"precision": prec, "recall": rec, "f1": f1, "accuracy": correct / max(1, total)}


# ------------------------------------------------------------------ training loop
def build_model(task: str, model_path: str, num_labels: int, device) -> torch.nn.Module:
    cls = AlbertForTokenClassification if task == "ner" else AlbertForSequenceClassification
    if model_path in ("tiny", "albert-large-v2"):
        cfg = AlbertConfig.tiny() if model_path == "tiny" else AlbertConfig.albert_large_v2()
        model = cls(cfg, num_labels=num_labels)
    else:
        model = cls.from_pretrained(model_path, strict=False, num_labels=num_labels)
    model.materialize(device)
    return model


@torch.no_grad()
def evaluate(model, data, task, bs, device) -> Tuple[float, Dict[str, float]]:
    model.eval()
    losses, n = 0.0, 0
    preds, refs = [], []
    for b in batches(data, bs, False, 0):
        b = {k: v.to(device) for k, v in b.items()}
        out = model(b["input_ids"], b["attention_mask"], labels=b["labels"])
        losses += float(out["loss"]) * b["input_ids"].shape[0]
        n += b["input_ids"].shape[0]
        pred = out["logits"].float().argmax(-1).cpu()
        lab = b["labels"].cpu()
        if task == "ner":
            for p, l in zip(pred, lab):
                keep = l != -100
                preds.append([NER_LABELS[i] for i in p[keep].tolist()])
                refs.append([NER_LABELS[i] for i in l[keep].tolist()])
        else:
            preds += pred.tolist()
            refs += lab.tolist()
    model.train()
    if task == "ner":
        metrics = ner_metrics(preds, refs)
    else:
        metrics = {"accuracy": sum(int(p == r) for p, r in zip(preds, refs)) / max(1, len(refs))}
    return losses / max(1, n), metrics


def run(args) -> Dict[str, float]:
    torch.manual_seed(args.seed)
    device = torch.device(args.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    labels = NER_LABELS if args.task == "ner" else NCC_LABELS
    model = build_model(args.task, args.model_path, len(labels), device)
    V = model.config.vocab_size
    make = synthetic_ner if args.task == "ner" else synthetic_ncc
    train = make(args.train_samples, args.max_seq_length, V, args.seed)
    val = make(args.eval_samples, args.max_seq_length, V, args.seed + 1)
    test = make(args.eval_samples, args.max_seq_length, V, args.seed + 2)
    flat = model.flat
    master = flat.fp32
    master.grad = flat.grad
    opt = torch.optim.AdamW([master], lr=args.learning_rate, weight_decay=args.weight_decay)
    steps_per_epoch = math.ceil(len(train) / args.per_device_train_batch_size)
    total = steps_per_epoch * args.num_train_epochs
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: max(0.0, 1.0 - s / max(1, total)))
    best_loss, best_state, bad_epochs, history = float("inf"), None, 0, []
    model.train()
    for epoch in range(args.num_train_epochs):
        for b in batches(train, args.per_device_train_batch_size, True, args.seed + epoch):
            b = {k: v.to(device) for k, v in b.items()}
            flat.zero_grad()
            out = model(b["input_ids"], b["attention_mask"], labels=b["labels"])
            out["loss"].backward()
            torch.nn.utils.clip_grad_norm_([master], args.max_grad_norm)
            opt.step()
            sched.step()
            flat.refresh_bf16()
        val_loss, val_metrics = evaluate(model, val, args.task, args.per_device_eval_batch_size, device)
        history.append({"epoch": epoch + 1, "eval_loss": val_loss, **{f"eval_{k}": v for k, v in val_metrics.items()}})
        logger.info(json.dumps(history[-1]))
        # EarlyStoppingCallback on metric_for_best_model="loss" (lower is better) + load_best_model_at_end
        if val_loss < best_loss - args.early_stopping_threshold:
            best_loss, bad_epochs = val_loss, 0
            best_state = master.detach().clone()
        else:
            bad_epochs += 1
            if bad_epochs >= args.early_stopping_patience:
                logger.info(f"early stopping after epoch {epoch + 1}")
                break
    if best_state is not None:
        master.copy_(best_state)
        flat.refresh_bf16()
    test_loss, test_metrics = evaluate(model, test, args.task, args.per_device_eval_batch_size, device)
    result = {"task": args.task, "epochs_run": len(history), "test_loss": test_loss,
              **{f"test_{k}": v for k, v in test_metrics.items()}, "history": history}
    if args.output_dir:
        os.makedirs(args.output_dir, exist_ok=True)
        model.save_pretrained(args.output_dir)
        with open(os.path.join(args.output_dir, "all_results.json"), "w") as f:
            json.dump(result, f, indent=2)
    return result


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--task", choices=["ner", "ncc"], required=True)
    ap.add_argument("--model_path", default="tiny", help="checkpoint dir, 'albert-large-v2' or 'tiny' (random init)")
    ap.add_argument("--output_dir", default=None)
    ap.add_argument("--num_train_epochs", type=int, default=10)
    ap.add_argument("--learning_rate", type=float, default=5e-5)
    ap.add_argument("--weight_decay", type=float, default=0.0)
    ap.add_argument("--max_grad_norm", type=float, default=1.0)
    ap.add_argument("--per_device_train_batch_size", type=int, default=16)
    ap.add_argument("--per_device_eval_batch_size", type=int, default=32)
    ap.add_argument("--max_seq_length", type=int, default=128)
    ap.add_argument("--early_stopping_patience", type=int, default=1)
    ap.add_argument("--early_stopping_threshold", type=float, default=0.0)
    ap.add_argument("--train_samples", type=int, default=512)
    ap.add_argument("--eval_samples", type=int, default=128)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--device", default=None)
    return ap.parse_args(argv)


def main(argv=None):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    res = run(parse_args(argv))
    print(json.dumps({k: v for k, v in res.items() if k != "history"}))


if __name__ == "__main__":
    main()
