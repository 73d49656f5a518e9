"""Synthetic ALBERT pre-training data with the reference's columns and shapes.

The reference tokenizes WikiText-103 into sentence-order-prediction instances
(albert/tokenize_wikitext103.py:13-104): ``[CLS] A [SEP] B [SEP]`` packed up to 512 tokens,
``token_type_ids`` 0/1 for the two segments, ``special_tokens_mask``, ``sentence_order_label``
(segments swapped with p = 0.5), then ``DataCollatorForLanguageModeling`` masks 15 % of the
non-special tokens (80 % [MASK], 10 % random, 10 % unchanged).  There is no network here, so the
same columns are generated on the device from a per-peer seed (the reference seeds shuffling with
``hash(local_public_key)``, run_trainer.py:266-270): random token ids, full 512-token instances
by default (``length_mode="wikitext"`` adds the short document-tail instances).

Two masking forms:
  * ``fixed`` — exactly round(0.15 * n_real) positions per sequence, returned as fixed-shape
    ``mlm_positions``/``mlm_labels`` (BERT's max_predictions_per_seq form; graph-capturable);
  * ``hf`` — Bernoulli(0.15) per token, returned as HF ``labels`` [B, S] with -100 elsewhere AND as
    ``mlm_positions``/``mlm_labels`` [B, P_hf] so the model needs no ``nonzero`` (host sync).  P_hf is
    the mean + 6 sigma of the per-row count (128 at S = 512); a row drawing more (p < 1e-9) keeps
    its first P_hf picks and leaves the rest unmasked, so labels and positions always agree.
"""
from __future__ import annotations

from typing import Dict, Iterator

import torch

CLS_ID, SEP_ID, MASK_ID, PAD_ID = 2, 3, 4, 0
FIRST_REGULAR_ID = 5


class SyntheticSOPStream:
    def __init__(self, batch_size: int, seq_len: int = 512, vocab_size: int = 30000, seed: int = 0,
                 device="cpu", mask_mode: str = "fixed", mlm_probability: float = 0.15,
                 length_mode: str = "full", min_len: int = 64, pattern_period: int = 0):
        self.B, self.S, self.V = batch_size, seq_len, vocab_size
        self.device = torch.device(device)
        self.mask_mode, self.p = mask_mode, mlm_probability
        self.length_mode, self.min_len = length_mode, min_len
        # > 0: LEARNABLE token rows (convergence tests): token i of a row is
        # FIRST_REGULAR_ID + (phase + i) % pattern_period with a random phase per row, so a masked
        # token is predictable from its neighbours; 0: independent uniform tokens (throughput runs)
        self.pattern_period = int(pattern_period)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed) % (2 ** 63))
        self.P = max(1, round(self.p * (seq_len - 3)))
        sd = (seq_len * self.p * (1 - self.p)) ** 0.5
        self.P_hf = min(seq_len, int(-(-(self.p * seq_len + 6 * sd) // 8) * 8))

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        return self

    def __next__(self) -> Dict[str, torch.Tensor]:
        return self.next_batch()

    def _rand(self, *shape, high):
        return torch.randint(0, high, shape, generator=self.gen, device=self.device)

    @torch.no_grad()
    def next_batch(self) -> Dict[str, torch.Tensor]:
        B, S, dev = self.B, self.S, self.device
        if self.length_mode == "full":
            lengths = torch.full((B,), S, device=dev)
        else:  # ~10 % short document tails (the last instance of each document)
            lo = min(self.min_len, max(8, S // 2))  # short sequences: never below 8 tokens
            short = torch.rand(B, generator=self.gen, device=dev) < 0.1
            lengths = torch.where(short, self._rand(B, high=max(1, S - lo)) + lo, torch.full((B,), S, device=dev))
        ar = torch.arange(S, device=dev)[None, :]
        if self.pattern_period > 0:
            phase = self._rand(B, 1, high=self.pattern_period)
            ids = (phase + ar) % min(self.pattern_period, self.V - FIRST_REGULAR_ID) + FIRST_REGULAR_ID
        else:
            ids = self._rand(B, S, high=self.V - FIRST_REGULAR_ID) + FIRST_REGULAR_ID
        # segment A ends at a random split (>= 1 token each side)
        split = (torch.rand(B, generator=self.gen, device=dev) * (lengths - 4).float()).long() + 2
        attn = (ar < lengths[:, None]).long()
        ids = torch.where(ar == 0, CLS_ID, ids)
        ids = torch.where(ar == split[:, None], SEP_ID, ids)
        ids = torch.where(ar == (lengths - 1)[:, None], SEP_ID, ids)
        ids = torch.where(attn.bool(), ids, PAD_ID)
        tt = ((ar > split[:, None]) & attn.bool()).long()
        special = ((ar == 0) | (ar == split[:, None]) | (ar == (lengths - 1)[:, None]) | ~attn.bool()).long()
        sop = self._rand(B, high=2)
        batch = {"input_ids": ids, "token_type_ids": tt, "attention_mask": attn, "special_tokens_mask": special,
                 "sentence_order_label": sop}
        if self.mask_mode == "fixed":
            batch.update(self._mask_fixed(ids, special, lengths))
        else:
            batch.update(self._mask_hf(ids, special))
        return batch

    def _mask_fixed(self, ids, special, lengths):
        B, S, P = self.B, self.S, self.P
        score = torch.rand(B, S, generator=self.gen, device=self.device)
        score = score.masked_fill(special.bool(), 2.0)
        pos = torch.argsort(score, dim=1)[:, :P]
        n_real = (lengths - 3).clamp(min=1)
        n_mask = torch.round(self.p * n_real.float()).long().clamp(min=1, max=P)
        valid = torch.arange(P, device=self.device)[None, :] < n_mask[:, None]
        labels = torch.gather(ids, 1, pos)
        labels = torch.where(valid, labels, torch.full_like(labels, -100))
        pos = torch.where(valid, pos, torch.zeros_like(pos))
        ids = ids.clone()
        r = torch.rand(B, P, generator=self.gen, device=self.device)
        rnd = self._rand(B, P, high=self.V - FIRST_REGULAR_ID) + FIRST_REGULAR_ID
        cur = torch.gather(ids, 1, pos)
        new = torch.where(r < 0.8, torch.full_like(cur, MASK_ID), torch.where(r < 0.9, rnd, cur))
        new = torch.where(valid, new, cur)
        ids.scatter_(1, pos, new)
        return {"input_ids": ids, "mlm_positions": pos, "mlm_labels": labels}

    def _mask_hf(self, ids, special):
        prob = torch.full(ids.shape, self.p, device=self.device).masked_fill(special.bool(), 0.0)
        masked = torch.bernoulli(prob, generator=self.gen).bool()
        P = self.P_hf
        order = torch.sort((~masked).to(torch.int8), dim=1, stable=True).indices[:, :P]  # picks first
        valid = torch.arange(P, device=self.device)[None, :] < masked.sum(1, keepdim=True)
        masked = torch.zeros_like(masked).scatter_(1, order, valid) & masked  # cap at P picks per row
        pos = torch.where(valid, order, torch.zeros_like(order))
        mlm_labels = torch.where(valid, torch.gather(ids, 1, pos), torch.full_like(pos, -100))
        labels = torch.where(masked, ids, torch.full_like(ids, -100))
        r = torch.rand(ids.shape, generator=self.gen, device=self.device)
        rnd = self._rand(*ids.shape, high=self.V - FIRST_REGULAR_ID) + FIRST_REGULAR_ID
        new = torch.where(r < 0.8, torch.full_like(ids, MASK_ID), torch.where(r < 0.9, rnd, ids))
        return {"input_ids": torch.where(masked, new, ids), "labels": labels, "mlm_positions": pos,
                "mlm_labels": mlm_labels}


def peer_seed(local_public_key: bytes, base_seed: int = 0) -> int:
    """Deterministic per-peer seed (the reference uses hash(local_public_key) % 2**31)."""
    import hashlib

    return (int.from_bytes(hashlib.sha256(local_public_key).digest()[:8], "little") + base_seed) % (2 ** 31)
