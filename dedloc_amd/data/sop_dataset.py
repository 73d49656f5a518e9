"""Real-text sentence-order-prediction data: build a tokenized dataset on disk, then stream padded,
MLM-masked device batches from it.

Reference behaviour (``albert/tokenize_wikitext103.py:13-104``, ``sahajbert/dataset_streaming.py``):
a document is split into sentences and walked in order; sentences accumulate into a chunk until the
chunk's token count reaches ``max_seq_length`` or the document ends; a chunk of >= 2 sentences is cut
at a uniformly random sentence boundary into segments A and B, which are swapped with probability 0.5
(``sentence_order_label`` = 1 when swapped); the pair is encoded ``[CLS] A [SEP] B [SEP]`` with
longest-first truncation to ``max_seq_length`` and a special-tokens mask.  Batches follow HF's
``DataCollatorForLanguageModeling``: dynamic padding to the longest row, 15 % of the non-special
tokens selected, of those 80 % -> [MASK], 10 % -> a random token, 10 % unchanged, labels -100 elsewhere.

Differences: sentence splitting is a regex on sentence-final punctuation (., !, ?, and the Bengali
danda) instead of NLTK punkt (not installed here); every random draw comes from one seeded
``random.Random`` so a build is reproducible.  ``datasets`` stores the result (``save_to_disk``),
with the tokenizer's special ids in ``sop_meta.json`` so a peer needs no tokenizer at train time.

    python -m dedloc_amd.data.sop_dataset --input corpus.txt --tokenizer tok_dir --output_dir data/sop
"""
from __future__ import annotations

import argparse
import json
import os
import random
import re
from typing import Callable, Dict, Iterable, List, Optional

import torch

_SENT_END = re.compile(r"(?<=[.!?।])\s+")
META = "sop_meta.json"


def split_sentences(text: str) -> List[str]:
    """Sentence split on ., !, ? and the Bengali danda followed by whitespace."""
    return [s.strip() for s in _SENT_END.split(text.strip()) if s.strip()]


def read_documents(path: str) -> Iterable[str]:
    """Documents from a text file (blank-line separated) or a directory of such files."""
    files = [path] if os.path.isfile(path) else sorted(
        os.path.join(path, f) for f in os.listdir(path) if f.endswith(".txt"))
    for fn in files:
        with open(fn, encoding="utf-8") as f:
            doc: List[str] = []
            for line in f:
                if line.strip():
                    doc.append(line.strip())
                elif doc:
                    yield " ".join(doc)
                    doc = []
            if doc:
                yield " ".join(doc)


class SOPInstanceBuilder:
    """Turns documents into SOP instances (dicts of python lists) with one seeded RNG."""

    def __init__(self, tokenizer, max_seq_length: int = 512, seed: int = 0,
                 splitter: Callable[[str], List[str]] = split_sentences):
        self.tok, self.max_len, self.split = tokenizer, max_seq_length, splitter
        self.rng = random.Random(seed)

    def _encode(self, a: List[str], b: List[str]) -> Dict[str, List[int]]:
        return dict(self.tok(" ".join(a), " ".join(b), truncation="longest_first", max_length=self.max_len,
                             return_special_tokens_mask=True, return_token_type_ids=True,
                             return_attention_mask=True))

    def from_document(self, text: str) -> List[Dict[str, List[int]]]:
        sents = self.split(text)
        out, chunk, n_tok = [], [], 0
        for i, s in enumerate(sents):
            chunk.append(s)
            n_tok += len(self.tok.tokenize(s))
            if n_tok < self.max_len and i != len(sents) - 1:
                continue
            if len(chunk) >= 2:  # single-sentence chunks carry no order signal and are dropped
                cut = self.rng.randint(1, len(chunk) - 1)
                first, second = chunk[:cut], chunk[cut:]
                swapped = self.rng.random() < 0.5
                inst = self._encode(second, first) if swapped else self._encode(first, second)
                inst["sentence_order_label"] = int(swapped)
                out.append(inst)
            chunk, n_tok = [], 0
        return out

    def build(self, documents: Iterable[str]) -> Dict[str, List]:
        cols: Dict[str, List] = {}
        for doc in documents:
            if not doc or doc.isspace():
                continue
            for inst in self.from_document(doc):
                for k, v in inst.items():
                    cols.setdefault(k, []).append(v)
        return cols


def special_ids(tokenizer) -> Dict[str, int]:
    return {"cls": tokenizer.cls_token_id, "sep": tokenizer.sep_token_id, "mask": tokenizer.mask_token_id,
            "pad": tokenizer.pad_token_id if tokenizer.pad_token_id is not None else 0,
            "vocab_size": len(tokenizer)}


def build_dataset(documents: Iterable[str], tokenizer, output_dir: str, max_seq_length: int = 512, seed: int = 0):
    """Tokenize ``documents`` into SOP instances and ``save_to_disk`` them (+ ``sop_meta.json``)."""
    import datasets

    cols = SOPInstanceBuilder(tokenizer, max_seq_length, seed).build(documents)
    if not cols:
        raise ValueError("no SOP instance could be built (documents need >= 2 sentences)")
    ds = datasets.Dataset.from_dict(cols)
    ds.save_to_disk(output_dir)
    with open(os.path.join(output_dir, META), "w") as f:
        json.dump(dict(special_ids(tokenizer), max_seq_length=max_seq_length, num_instances=len(ds)), f)
    return ds


def is_sop_dataset(path: Optional[str]) -> bool:
    return bool(path) and os.path.isfile(os.path.join(path, META))


class DiskSOPStream:
    """Infinite, per-peer shuffled device batches from a ``build_dataset`` directory, padded to the
    batch's longest row and MLM-masked like ``DataCollatorForLanguageModeling`` (labels [B, S] form)."""

    def __init__(self, path: str, batch_size: int, seed: int = 0, device="cpu", mlm_probability: float = 0.15):
        import datasets

        self.ds = datasets.load_from_disk(path)
        with open(os.path.join(path, META)) as f:
            self.meta = json.load(f)
        self.B, self.p = batch_size, mlm_probability
        self.device = torch.device(device)
        self.gen = torch.Generator().manual_seed(int(seed) % (2 ** 63))
        self.order: List[int] = []
        self.epoch = 0

    def _next_indices(self) -> List[int]:
        out = []
        while len(out) < self.B:
            if not self.order:  # reshuffle per epoch with the peer's own seed
                self.order = torch.randperm(len(self.ds), generator=self.gen).tolist()
                self.epoch += 1
            out.append(self.order.pop())
        return out

    @torch.no_grad()
    def next_batch(self) -> Dict[str, torch.Tensor]:
        rows = self.ds[self._next_indices()]
        L = max(len(r) for r in rows["input_ids"])
        B = self.B
        pad = self.meta["pad"]
        ids = torch.full((B, L), pad, dtype=torch.long)
        tt = torch.zeros((B, L), dtype=torch.long)
        am = torch.zeros((B, L), dtype=torch.long)
        special = torch.ones((B, L), dtype=torch.bool)
        for i in range(B):
            n = len(rows["input_ids"][i])
            ids[i, :n] = torch.tensor(rows["input_ids"][i])
            tt[i, :n] = torch.tensor(rows["token_type_ids"][i])
            am[i, :n] = 1
            special[i, :n] = torch.tensor(rows["special_tokens_mask"][i], dtype=torch.bool)
        prob = torch.full((B, L), self.p)
        prob.masked_fill_(special, 0.0)
        picked = torch.bernoulli(prob, generator=self.gen).bool()
        labels = torch.where(picked, ids, torch.full_like(ids, -100))
        to_mask = torch.bernoulli(torch.full((B, L), 0.8), generator=self.gen).bool() & picked
        ids = torch.where(to_mask, torch.full_like(ids, self.meta["mask"]), ids)
        to_rand = torch.bernoulli(torch.full((B, L), 0.5), generator=self.gen).bool() & picked & ~to_mask
        rand_tok = torch.randint(self.meta["vocab_size"], (B, L), generator=self.gen)
        ids = torch.where(to_rand, rand_tok, ids)
        batch = {"input_ids": ids, "token_type_ids": tt, "attention_mask": am, "labels": labels,
                 "sentence_order_label": torch.tensor(rows["sentence_order_label"], dtype=torch.long)}
        return {k: v.to(self.device, non_blocking=True) for k, v in batch.items()}


def main(argv=None):
    ap = argparse.ArgumentParser(description="tokenize a text corpus into SOP instances (datasets.save_to_disk)")
    ap.add_argument("--input", required=True, help="text file or directory of .txt files; blank lines separate documents")
    ap.add_argument("--tokenizer", required=True, help="directory loadable by transformers.AutoTokenizer")
    ap.add_argument("--output_dir", required=True)
    ap.add_argument("--max_seq_length", type=int, default=512)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    from transformers import AutoTokenizer

    tok = AutoTokenizer.from_pretrained(a.tokenizer)
    ds = build_dataset(read_documents(a.input), tok, a.output_dir, a.max_seq_length, a.seed)
    tok.save_pretrained(os.path.join(a.output_dir, "tokenizer"))
    print(json.dumps({"instances": len(ds), "output_dir": a.output_dir}))


if __name__ == "__main__":
    main()
