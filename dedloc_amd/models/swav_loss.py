"""SwAV swapped-prediction loss with Sinkhorn-Knopp assignments and an embedding queue.

Reference: ``swav/vissl/vissl/losses/swav_loss.py:24-380`` (SwAVLoss/SwAVCriterion) with
the DeDLOC modification (``:84-91``, D18): the queue switches on at a *global collaborative* step
(``queue_start_iter`` compared with ``collaboration_state.optimizer_step``), not a local iteration.

Device path: Sinkhorn-Knopp (column-owning workgroups, two scale vectors instead of a rewritten
matrix) and the fused log-softmax x assignment cross-entropy of every crop pair (fwd + bwd in one
launch) are HIP kernels (csrc/kernels/swav.hip); the queue is a ring buffer (no shifting copies).
"""
from __future__ import annotations

import logging
import math
from typing import Sequence

import torch
import torch.nn as nn

from .. import ops as _ops  # noqa: F401  (registers torch.ops.dedloc.*)

logger = logging.getLogger(__name__)


class _SwAVCE(torch.autograd.Function):
    """sum over (assignment crop i, other crop v) of -mean_b <q_i, log_softmax(s_v / T)>, every pair in
    one launch (swav_ce_multi: each crop's score row and its log-sum-exp are read once)."""

    @staticmethod
    def forward(ctx, scores, assignments, crops_for_assign, num_crops, bs, temperature):
        s = scores.contiguous()
        ds = torch.empty(s.shape, dtype=torch.float32, device=s.device)
        loss = torch.zeros(1, dtype=torch.float32, device=s.device)
        n_pairs = (num_crops - 1) * len(crops_for_assign)
        q = torch.stack(assignments) if len(assignments) > 1 else assignments[0].unsqueeze(0)
        torch.ops.dedloc.swav_ce_multi(s, q.contiguous(), list(crops_for_assign), ds, loss, temperature,
                                       1.0 / (bs * n_pairs))
        ctx.save_for_backward(ds)
        ctx.dtype = scores.dtype
        return loss.squeeze(0)

    @staticmethod
    def backward(ctx, dloss):
        (ds,) = ctx.saved_tensors
        return (ds * dloss).to(ctx.dtype), None, None, None, None, None


class SwAVLoss(nn.Module):
    def __init__(self, num_crops: int = 8, crops_for_assign: Sequence[int] = (0, 1), temperature: float = 0.1,
                 epsilon: float = 0.03, num_iters: int = 3, num_prototypes: int = 3000, embedding_dim: int = 128,
                 queue_length: int = 0, queue_start_iter: int = 0, batch_size: int = 64,
                 temp_hard_assignment_iters: int = 0):
        super().__init__()
        self.num_crops, self.crops_for_assign = num_crops, list(crops_for_assign)
        self.temperature, self.epsilon, self.num_iters = temperature, epsilon, num_iters
        self.queue_length, self.queue_start_iter = queue_length, queue_start_iter
        self.temp_hard_assignment_iters = temp_hard_assignment_iters
        self.bs = batch_size
        self.num_iteration = 0  # local iterations (hard-assignment warmup counts these, swav_loss.py:241)
        self.use_queue = self.was_using_queue = False
        if queue_length:
            # uniform(-stdv, stdv) init like swav_loss.py:346-366 (the queue is used as soon as it is enabled)
            stdv = 1.0 / math.sqrt(embedding_dim / 3)
            self.register_buffer("queue", torch.rand(len(self.crops_for_assign), queue_length, embedding_dim)
                                 .mul_(2 * stdv).add_(-stdv))
            self.queue_ptr = 0

    def forward(self, embedding: torch.Tensor, scores: torch.Tensor, prototypes: torch.Tensor,
                training_iterations: int = 0):
        """embedding [num_crops*bs, D], scores [num_crops*bs, K]; ``training_iterations`` is the GLOBAL
        collaborative step (DeDLOC: standard_train_step.py:153 passes collaboration_state.optimizer_step)."""
        bs = self.bs
        self.use_queue = self.queue_length > 0 and training_iterations >= self.queue_start_iter
        if self.use_queue and not self.was_using_queue:
            logger.info(f"Using queue now! global niter = {training_iterations}")
        self.was_using_queue = self.use_queue
        assignments = []
        with torch.no_grad():
            for i, crop_id in enumerate(self.crops_for_assign):
                s = scores[bs * crop_id: bs * (crop_id + 1)].float()
                if self.use_queue:  # queue rows first, current batch last (the kernel emits the last bs rows)
                    s = torch.cat([self._queue_scores(i, prototypes), s])
                q = self._sinkhorn(s.contiguous(), bs)
                if self.num_iteration < self.temp_hard_assignment_iters:
                    q = torch.zeros_like(q).scatter_(1, q.argmax(dim=1, keepdim=True), 1.0)
                assignments.append(q)
        loss = _SwAVCE.apply(scores, assignments, self.crops_for_assign, self.num_crops, bs, self.temperature)
        self.num_iteration += 1
        if self.use_queue:
            self._update_queue(embedding.detach())
        return loss

    def _queue_scores(self, i, prototypes):
        """Scores of queue i against the prototypes, [L, K] fp32, on the GEMM operators (bf16 operands
        like the batch's prototype scores, fp32 accumulation and output)."""
        q = self.queue[i]
        out = torch.zeros(q.shape[0], prototypes.shape[0], dtype=torch.float32, device=q.device)
        torch.ops.dedloc.gemm_acc_f32(q.to(torch.bfloat16), prototypes.detach().to(torch.bfloat16), out, False, True)
        return out

    def _sinkhorn(self, s, bs):
        return torch.ops.dedloc.sinkhorn(s, bs, self.epsilon, self.num_iters)

    @torch.no_grad()
    def _update_queue(self, emb):
        bs, L = self.bs, self.queue_length
        for i, crop_id in enumerate(self.crops_for_assign):
            e = emb[bs * crop_id: bs * (crop_id + 1)].float()
            idx = (torch.arange(bs, device=e.device) + self.queue_ptr) % L
            self.queue[i].index_copy_(0, idx, e)
        self.queue_ptr = (self.queue_ptr + bs) % L
