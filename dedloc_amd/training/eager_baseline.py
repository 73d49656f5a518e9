"""PyTorch-eager baseline for BASELINE.md: the reference's compute stack on MI355X, driven by this
repo's collaborative engine.

The reference trains HF ``transformers.AlbertForPreTraining`` under AMP with
``torch_optimizer.Lamb(debias=True, clamp_value=1e4)`` and ``clip_grad_norm_`` inside the HF Trainer
(``albert/run_trainer.py:73-100,272-285``).  This module reproduces that per-op eager stack (bf16
autocast, SDPA attention, per-tensor LAMB written in torch ops) so that ``bench.py --impl eager``
measures the same metric through the same CollaborativeOptimizer/averaging path as the HIP build —
the "measured baseline" BASELINE.md asks for.  Only the LAMB trust-ratio branch is written with
``torch.where`` instead of host-synchronising Python comparisons (favours the baseline).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional

import torch

from ..utils.flat import FlatParams


class EagerAlbertModel:
    def __init__(self, config, device):
        import transformers

        hcfg = transformers.AlbertConfig(**{k: v for k, v in config.to_dict().items()
                                            if k not in ("architectures", "model_type")})
        self.config = config
        self.device = torch.device(device)
        self.module = transformers.AlbertForPreTraining(hcfg).to(self.device).train()
        self.flat = FlatParams(self.module.named_parameters(), device=self.device, with_bf16=False, autograd=True)

    def train(self):
        self.module.train()
        return self

    def no_decay_names(self):
        return [n for n in self.flat.names if "bias" in n or "LayerNorm.weight" in n]

    def __call__(self, input_ids, attention_mask, token_type_ids, labels=None, sentence_order_label=None,
                 mlm_positions=None, mlm_labels=None):
        if labels is None and mlm_positions is not None:
            labels = torch.full_like(input_ids, -100)
            valid = mlm_labels != -100
            labels.scatter_(1, torch.where(valid, mlm_positions, 0), torch.where(valid, mlm_labels, labels[:, :1]))
        with torch.autocast(device_type=self.device.type, dtype=torch.bfloat16, enabled=self.device.type == "cuda"):
            out = self.module(input_ids=input_ids, attention_mask=attention_mask, token_type_ids=token_type_ids,
                              labels=labels, sentence_order_label=sentence_order_label)
        return {"loss": out.loss}

    def save_pretrained(self, path: str):
        self.module.save_pretrained(path)


class EagerLamb:
    """torch_optimizer.Lamb semantics, one tensor at a time (~10 kernels per parameter tensor)."""

    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-6,
                 weight_decay: float = 0.0, clamp_value: float = 10.0, debias: bool = True,
                 no_decay: Iterable[str] = ()):
        self.flat = flat
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)]
        self.clamp_value, self.debias = clamp_value, debias
        no_decay = set(no_decay)
        self.wd = {n: (0.0 if n in no_decay else weight_decay) for n in flat.names}
        self.exp_avg = torch.zeros_like(flat.fp32)
        self.exp_avg_sq = torch.zeros_like(flat.fp32)
        self.step_count = 0

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, grad: Optional[torch.Tensor] = None, grad_scale: float = 1.0):
        g_all = self.flat.grad if grad is None else grad
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        self.step_count += 1
        t = self.step_count
        bc = math.sqrt(1 - b2 ** t) / (1 - b1 ** t) if self.debias else 1.0
        for n in self.flat.names:
            p = self.flat.params[n].data
            g = self.flat.view(g_all, n)
            m, v = self.flat.view(self.exp_avg, n), self.flat.view(self.exp_avg_sq, n)
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            wn = p.norm().clamp(0, self.clamp_value)
            u = m / v.sqrt().add(grp["eps"])
            if self.wd[n]:
                u.add_(p, alpha=self.wd[n])
            un = u.norm()
            trust = torch.where((wn > 0) & (un > 0), wn / un, torch.ones_like(wn))
            p.add_(u * (-grp["lr"] * bc * trust))

    def state_tensors(self) -> List[torch.Tensor]:
        return [self.exp_avg, self.exp_avg_sq]

    def state_dict(self) -> Dict:
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "param_groups": [dict(self.param_groups[0])]}

    def load_state_dict(self, sd: Dict):
        self.step_count = int(sd.get("step", 0))
        if "exp_avg" in sd:
            self.exp_avg.copy_(sd["exp_avg"])
            self.exp_avg_sq.copy_(sd["exp_avg_sq"])
