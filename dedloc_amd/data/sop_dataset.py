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
    batch's longest row and MLM-masked like ``DataCollatorForLanguageModeling`` (labels [B, S] form,
    plus the equivalent fixed-shape ``mlm_positions`` / ``mlm_labels`` the model consumes sync-free)."""

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
        return collate_mlm(self.ds[self._next_indices()], self.meta, self.gen, self.p, self.device)


@torch.no_grad()
def collate_mlm(rows: Dict[str, List], meta: Dict[str, int], gen: torch.Generator, p: float = 0.15,
                device=None) -> Dict[str, torch.Tensor]:
    """``DataCollatorForLanguageModeling`` semantics over columnar SOP rows: pad to the longest row,
    select p of the non-special tokens; 80 % -> [MASK], 10 % -> random token, 10 % kept."""
    B = len(rows["input_ids"])
    L = max(len(r) for r in rows["input_ids"])
    ids = torch.full((B, L), meta["pad"], dtype=torch.long)
    tt = torch.zeros((B, L), dtype=torch.long)
    am = torch.zeros((B, L), dtype=torch.long)
    special = torch.ones((B, L), dtype=torch.bool)
    for i in range(B):
        n = len(rows["input_ids"][i])
        ids[i, :n] = torch.tensor(rows["input_ids"][i])
        tt[i, :n] = torch.tensor(rows["token_type_ids"][i])
        am[i, :n] = 1
        special[i, :n] = torch.tensor(rows["special_tokens_mask"][i], dtype=torch.bool)
    prob = torch.full((B, L), p)
    prob.masked_fill_(special, 0.0)
    picked = torch.bernoulli(prob, generator=gen).bool()
    labels = torch.where(picked, ids, torch.full_like(ids, -100))
    to_mask = torch.bernoulli(torch.full((B, L), 0.8), generator=gen).bool() & picked
    ids = torch.where(to_mask, torch.full_like(ids, meta["mask"]), ids)
    to_rand = torch.bernoulli(torch.full((B, L), 0.5), generator=gen).bool() & picked & ~to_mask
    ids = torch.where(to_rand, torch.randint(meta["vocab_size"], (B, L), generator=gen), ids)
    batch = {"input_ids": ids, "token_type_ids": tt, "attention_mask": am, "labels": labels,
             "sentence_order_label": torch.tensor(rows["sentence_order_label"], dtype=torch.long)}
    batch.update(mlm_targets(picked, labels))
    dev = torch.device(device) if device is not None else torch.device("cpu")
    return {k: v.to(dev, non_blocking=True) for k, v in batch.items()}


def mlm_targets(picked: torch.Tensor, labels: torch.Tensor, multiple: int = 8) -> Dict[str, torch.Tensor]:
    """HF ``labels`` [B, L] -> fixed-shape ``mlm_positions`` / ``mlm_labels`` [B, P] (-100 pads), computed
    on the HOST while collating, so the model's MLM head gathers its rows on the device without a
    ``nonzero`` (a host synchronisation per micro-step).  P = the batch's largest masked count rounded
    up to ``multiple`` (few distinct shapes)."""
    counts = picked.sum(1)
    P = max(1, int(counts.max()) if counts.numel() else 1)
    P = (P + multiple - 1) // multiple * multiple
    B, L = picked.shape
    # stable sort puts each row's picked positions first, in order
    order = torch.sort((~picked).to(torch.int8), dim=1, stable=True).indices
    if P > L:
        order = torch.cat([order, torch.zeros(B, P - L, dtype=order.dtype)], 1)
    order = order[:, :P]
    valid = torch.arange(P)[None, :] < counts[:, None]
    pos = torch.where(valid, order, torch.zeros_like(order))
    lab = torch.where(valid, labels.gather(1, pos), torch.full_like(pos, -100))
    return {"mlm_positions": pos, "mlm_labels": lab}


class StreamingSOPStream:
    """sahajBERT's streaming corpus (reference ``sahajbert/dataset_streaming.py``: Wikipedia-bn and
    OSCAR-bn merged with probabilities 0.23 / 0.77, a 10^4-document shuffle buffer seeded per peer,
    SOP instances tokenized on the fly, an endless stream) over local text sources.

    ``sources``: [(path, probability)], each path a text file or directory (``read_documents``);
    every source restarts when exhausted, so the stream never ends."""

    def __init__(self, sources, tokenizer, batch_size: int, seed: int = 0, device="cpu", max_seq_length: int = 512,
                 shuffle_buffer: int = 10_000, mlm_probability: float = 0.15):
        if not sources:
            raise ValueError("no streaming sources")
        total = float(sum(p for _, p in sources))
        self.paths = [s for s, _ in sources]
        self.cum = []
        acc = 0.0
        for _, p in sources:
            acc += p / total
            self.cum.append(acc)
        self.rng = random.Random(seed)
        self.builder = SOPInstanceBuilder(tokenizer, max_seq_length, seed=seed + 1)
        self.meta = special_ids(tokenizer)
        self.B, self.p, self.device = batch_size, mlm_probability, torch.device(device)
        self.gen = torch.Generator().manual_seed(int(seed) % (2 ** 63))
        self.iters = [self._cycle(p) for p in self.paths]
        self.buffer: List[str] = []
        self.shuffle_buffer = max(1, shuffle_buffer)
        self.pending: List[Dict[str, List[int]]] = []
        self.source_counts = [0] * len(self.paths)

    @staticmethod
    def _cycle(path):
        while True:
            n = 0
            for doc in read_documents(path):
                n += 1
                yield doc
            if n == 0:
                raise ValueError(f"source {path} holds no document")

    def _draw_document(self) -> str:
        while len(self.buffer) < self.shuffle_buffer:  # fill / refill the shuffle buffer from the mixture
            u = self.rng.random()
            k = next(i for i, c in enumerate(self.cum) if u <= c or i == len(self.cum) - 1)
            self.source_counts[k] += 1
            self.buffer.append(next(self.iters[k]))
        j = self.rng.randrange(len(self.buffer))
        self.buffer[j], self.buffer[-1] = self.buffer[-1], self.buffer[j]
        return self.buffer.pop()

    def next_batch(self) -> Dict[str, torch.Tensor]:
        while len(self.pending) < self.B:
            self.pending.extend(self.builder.from_document(self._draw_document()))
        rows, self.pending = self.pending[:self.B], self.pending[self.B:]
        cols = {k: [r[k] for r in rows] for k in rows[0]}
        return collate_mlm(cols, self.meta, self.gen, self.p, self.device)


def parse_sources(spec: str):
    """``"path_a:0.23,path_b:0.77"`` -> [(path_a, 0.23), (path_b, 0.77)] (probability defaults to 1)."""
    out = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        path, _, prob = item.rpartition(":")
        if not path or not prob.replace(".", "", 1).isdigit():
            path, prob = item, "1"
        out.append((path, float(prob)))
    return out


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
