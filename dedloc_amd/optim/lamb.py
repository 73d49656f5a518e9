"""Fused LAMB / LARC-SGD over flat parameter buffers + the reference's LR schedules.

FusedLamb reproduces ``torch_optimizer.Lamb(..., clamp_value, debias=True)`` exactly as configured
at albert/run_trainer.py:86-94 (formula: SURVEY.md App. F) in two HIP launches for all ~30 tensors
(optim.hip).  Its ``state_dict`` uses torch_optimizer's per-parameter layout so the coordinator's
``optimizer_state.pt`` (albert/run_first_peer.py:133) stays format compatible.

FusedLarcSGD reproduces apex ``LARC(SGD(momentum))`` as configured in
swav/ClassyVision/classy_vision/optim/sgd_collaborative.py:135-144.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional

import torch

from ..utils.flat import FlatParams


class _FlatOptimizer:
    """Minimal torch.optim-like surface (param_groups, state_dict, zero_grad) over FlatParams."""

    def __init__(self, flat: FlatParams, defaults: Dict, weight_decay_of: Dict[str, float], chunk: int = 16384):
        self.flat = flat
        self.defaults = dict(defaults)
        self.param_groups = [dict(defaults, params=list(range(len(flat.names))))]
        self.weight_decay_of = weight_decay_of
        self.tables = flat.chunk_table(chunk, weight_decay_of)
        self.norms = torch.zeros(2 * len(flat.names), dtype=torch.float32, device=flat.device)
        self.step_count = 0
        self.no_decay = set()

    def _is_no_decay(self, name: str) -> bool:
        return name in self.no_decay

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def _per_param(self, buf: torch.Tensor) -> Dict[int, torch.Tensor]:
        return {i: self.flat.view(buf, n).detach().clone().cpu() for i, n in enumerate(self.flat.names)}


class FusedLamb(_FlatOptimizer):
    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-6,
                 weight_decay: float = 0.0, clamp_value: float = 10.0, debias: bool = True,
                 no_decay: Iterable[str] = (), adam: bool = False):
        no_decay = set(no_decay)
        wd = {n: (0.0 if n in no_decay else weight_decay) for n in flat.names}
        super().__init__(flat, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                    clamp_value=clamp_value, debias=debias, adam=adam), wd)
        self.no_decay = no_decay
        self.exp_avg = torch.zeros_like(flat.fp32)
        self.exp_avg_sq = torch.zeros_like(flat.fp32)

    @torch.no_grad()
    def step(self, grad: Optional[torch.Tensor] = None, grad_scale: float = 1.0):
        g = self.flat.grad if grad is None else grad
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        self.step_count += 1
        t = self.step_count
        bc = math.sqrt(1 - b2 ** t) / (1 - b1 ** t) if grp["debias"] else 1.0
        # adam mode (torch_optimizer.Lamb(adam=True)): trust ratio 1.  The kernel's trust is
        # min(||p||, clamp) / ||u|| with "1 when the clamped weight norm is 0", so clamp 0 is exactly that
        clamp = 0.0 if grp["adam"] else grp["clamp_value"]
        ct, cs, cl, twd = self.tables
        torch.ops.dedloc.lamb_step(self.flat.fp32, g, self.exp_avg, self.exp_avg_sq, ct, cs, cl, twd, self.norms,
                                   b1, b2, grp["eps"], grp["lr"] * bc, clamp, grad_scale)
        self.flat.refresh_bf16()

    def state_tensors(self) -> List[torch.Tensor]:
        return [self.exp_avg, self.exp_avg_sq]

    def _groups(self) -> List[List[int]]:
        """Flat indices of the reference's parameter groups, in its order: decayed first, then the
        no-decay group (albert/run_trainer.py:74-84); inside a group, model (flat) order.  Membership
        follows the no-decay NAME rule, not the weight-decay value, so the two groups exist even at
        weight_decay = 0 (a reference optimizer.pt always has two)."""
        nd = [self._is_no_decay(n) for n in self.flat.names]
        groups = [[i for i, f in enumerate(nd) if not f], [i for i, f in enumerate(nd) if f]]
        return [g for g in groups if g]

    def state_dict(self) -> Dict:
        m, v = self._per_param(self.exp_avg), self._per_param(self.exp_avg_sq)
        state = {i: {"step": self.step_count, "exp_avg": m[i], "exp_avg_sq": v[i]} for i in m}
        groups = []
        for idx in self._groups():
            g = {k: v for k, v in self.param_groups[0].items() if k != "params"}
            g["weight_decay"] = self.weight_decay_of[self.flat.names[idx[0]]]
            g["params"] = idx
            groups.append(g)
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, sd: Dict):
        """Accepts this class's own state dicts and torch-format ones (torch.optim / torch_optimizer /
        HF Trainer ``optimizer.pt``), whose ids number the parameters group by group: like
        ``torch.optim.Optimizer.load_state_dict`` the saved ``param_groups[k]['params']`` ids are
        zipped with this optimizer's k-th group."""
        st = sd.get("state", {})
        saved_groups = sd.get("param_groups") or []
        ours = self._groups()
        if saved_groups and [len(g["params"]) for g in saved_groups] == [len(g) for g in ours]:
            id_map = {int(sid): fi for g, idx in zip(saved_groups, ours) for sid, fi in zip(g["params"], idx)}
        elif saved_groups:
            raise ValueError(f"optimizer state has groups of sizes {[len(g['params']) for g in saved_groups]}, "
                             f"this optimizer {[len(g) for g in ours]}")
        else:
            id_map = {i: i for i in range(len(self.flat.names))}
        for sid, s in st.items():
            fi = id_map.get(int(sid))
            if fi is None or not s:
                continue
            n = self.flat.names[fi]
            dst_m, dst_v = self.flat.view(self.exp_avg, n), self.flat.view(self.exp_avg_sq, n)
            if tuple(s["exp_avg"].shape) != tuple(dst_m.shape):
                raise ValueError(f"state {sid} has shape {tuple(s['exp_avg'].shape)}, parameter {n} {tuple(dst_m.shape)}")
            dst_m.copy_(s["exp_avg"])
            dst_v.copy_(s["exp_avg_sq"])
            self.step_count = int(s.get("step", self.step_count))
        if saved_groups:
            self.param_groups[0]["lr"] = saved_groups[0].get("lr", self.param_groups[0]["lr"])


class FusedLarcSGD(_FlatOptimizer):
    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                 nesterov: bool = False, trust_coefficient: float = 0.001, clip: bool = False, eps: float = 1e-8,
                 no_decay: Iterable[str] = ()):
        if nesterov:
            raise NotImplementedError("nesterov LARC-SGD is not used by the reference")
        no_decay = set(no_decay)
        wd = {n: (0.0 if n in no_decay else weight_decay) for n in flat.names}
        super().__init__(flat, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov,
                                    trust_coefficient=trust_coefficient, clip=clip, eps=eps), wd)
        self.no_decay = no_decay
        self.momentum_buffer = torch.zeros_like(flat.fp32)

    @torch.no_grad()
    def step(self, grad: Optional[torch.Tensor] = None, grad_scale: float = 1.0):
        g = self.flat.grad if grad is None else grad
        grp = self.param_groups[0]
        ct, cs, cl, twd = self.tables
        torch.ops.dedloc.larc_sgd_step(self.flat.fp32, g, self.momentum_buffer, ct, cs, cl, twd, self.norms,
                                       grp["lr"], grp["momentum"], grp["trust_coefficient"], grp["eps"],
                                       grp["clip"], self.step_count == 0, grad_scale)
        self.step_count += 1
        self.flat.refresh_bf16()

    def state_tensors(self) -> List[torch.Tensor]:
        return [self.momentum_buffer]

    def state_dict(self) -> Dict:
        buf = self._per_param(self.momentum_buffer)
        return {"state": {i: {"momentum_buffer": b} for i, b in buf.items()},
                "param_groups": [{k: v for k, v in self.param_groups[0].items()}], "step": self.step_count}

    @torch.no_grad()
    def load_state_dict(self, sd: Dict):
        for i, n in enumerate(self.flat.names):
            s = sd.get("state", {}).get(i)
            if s:
                self.flat.view(self.momentum_buffer, n).copy_(s["momentum_buffer"])
        self.step_count = int(sd.get("step", self.step_count))


class LambdaScheduler:
    """torch LambdaLR semantics (``_step_count`` starts at 1, lr = base * f(last_epoch))."""

    def __init__(self, optimizer, lr_lambda):
        self.optimizer = optimizer
        self.lr_lambda = lr_lambda
        self.base_lr = optimizer.param_groups[0]["lr"]
        self.last_epoch = 0
        self._step_count = 1
        self._apply()

    def _apply(self):
        self.optimizer.param_groups[0]["lr"] = self.base_lr * self.lr_lambda(self.last_epoch)

    def step(self):
        self._step_count += 1
        self.last_epoch += 1
        self._apply()

    def get_last_lr(self):
        return [self.optimizer.param_groups[0]["lr"]]

    def state_dict(self):
        return {"last_epoch": self.last_epoch, "_step_count": self._step_count, "base_lr": self.base_lr}

    def load_state_dict(self, sd):
        self.last_epoch, self._step_count = sd["last_epoch"], sd["_step_count"]
        self.base_lr = sd.get("base_lr", self.base_lr)
        self._apply()


def get_linear_schedule_with_warmup(optimizer, num_warmup_steps: int, num_training_steps: int) -> LambdaScheduler:
    """transformers.get_linear_schedule_with_warmup (albert/run_trainer.py:96-98)."""

    def f(step):
        if step < num_warmup_steps:
            return float(step) / float(max(1, num_warmup_steps))
        return max(0.0, float(num_training_steps - step) / float(max(1, num_training_steps - num_warmup_steps)))

    return LambdaScheduler(optimizer, f)


class LinearWarmupCosineAnnealingLR(LambdaScheduler):
    """SwAV's per-collaborative-step schedule (sgd_collaborative.py:25-84, closed form :73-84).

    The reference divides by (warmup_epochs - 1) and breaks for warmup_epochs == 1;
    here warmup_epochs <= 1 means "no warmup".
    """

    def __init__(self, optimizer, warmup_epochs: int, max_epochs: int, warmup_start_lr: float = 0.0,
                 eta_min: float = 0.0):
        base = optimizer.param_groups[0]["lr"]
        self.warmup_epochs, self.max_epochs = warmup_epochs, max_epochs
        self.warmup_start_lr, self.eta_min = warmup_start_lr, eta_min

        def lr_at(s):
            if warmup_epochs > 1 and s < warmup_epochs:
                return warmup_start_lr + s * (base - warmup_start_lr) / (warmup_epochs - 1)
            span = max(1, max_epochs - warmup_epochs)
            return eta_min + 0.5 * (base - eta_min) * (1 + math.cos(math.pi * (s - warmup_epochs) / span))

        super().__init__(optimizer, lambda s: lr_at(s) / base if base else 0.0)
