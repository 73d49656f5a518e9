"""PyTorch-eager SwAV stack: the reference's compute on stock PyTorch modules (SwAV rows).

The reference trains vissl's ResNet-50 trunk (``swav/vissl/vissl/models/trunks/resnext.py:48-172``:
torchvision Bottlenecks) with the SwAV prototypes head (``swav_prototypes_head.py:61-112``), one
trunk pass per crop (``SINGLE_PASS_EVERY_CROP``, ``base_ssl_model.py:76-105``), the SwAV loss with
Sinkhorn-Knopp (``swav_loss.py:177-326``) and SGD wrapped in apex LARC (``sgd_collaborative.py:
137-144``), under mixed precision.  This module rebuilds that stack from stock ``torch.nn`` modules
and torch ops only — no dedloc kernel anywhere — with state-dict keys identical to
``models/resnet_swav.SwAVModel`` so parameters move between the two:

* ``EagerSwAVModel`` — nn.Conv2d / nn.BatchNorm2d / nn.ReLU / nn.MaxPool2d trunk, nn.Linear /
  nn.BatchNorm1d head, F.normalize; every crop through the trunk on its own (8 passes);
* ``EagerSwAVLoss`` — vissl's formulas op by op (log-sum-exp-stabilised exp, Sinkhorn iterations
  with torch.sum, log_softmax cross-entropy per crop pair, embedding queue);
* ``EagerLarcSGD`` — apex LARC (trust ratio per parameter tensor) + torch SGD momentum, one tensor
  at a time.

Uses: ``bench.py --model swav --impl eager`` (the measured SwAV baseline) and the fp32 twin of the
model-level parity tests (``eager_twin``).  The adaptive-rate branch is ``torch.where`` instead of
apex's host-synchronising Python comparison (favours the baseline).
"""
from __future__ import annotations

import copy
import math
from typing import Dict, Iterable, List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.flat import FlatParams


class EagerBottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        return self.relu(self.bn3(self.conv3(out)) + idt)


class EagerResNet50Trunk(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3)):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)

    def _make_layer(self, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes * 4))
        layers = [EagerBottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        layers += [EagerBottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


class EagerSwAVHead(nn.Module):
    def __init__(self, dims: Sequence[int] = (2048, 2048, 128), num_prototypes: int = 3000):
        super().__init__()
        self.projection_head = nn.Sequential(nn.Linear(dims[0], dims[1]), nn.BatchNorm1d(dims[1]), nn.ReLU(inplace=True),
                                             nn.Linear(dims[1], dims[2]))
        self.prototypes0 = nn.Linear(dims[2], num_prototypes, bias=False)

    def forward(self, x):
        emb = F.normalize(self.projection_head(x), dim=1, p=2)
        return emb, self.prototypes0(emb)


class EagerSwAVModel(nn.Module):
    """vissl's multi-resolution forward: with ``single_pass_every_crop`` every crop runs through the
    trunk on its own (each BatchNorm sees one crop's batch), the features are concatenated, then the
    head."""

    def __init__(self, num_prototypes: int = 3000, single_pass_every_crop: bool = True):
        super().__init__()
        self.trunk = EagerResNet50Trunk()
        self.heads = nn.ModuleList([EagerSwAVHead(num_prototypes=num_prototypes)])
        self.single_pass_every_crop = single_pass_every_crop

    def forward(self, crops: List[torch.Tensor]):
        feats = []
        if self.single_pass_every_crop:
            for c in crops:
                feats.append(self.trunk(c))
        else:
            i = 0
            while i < len(crops):
                j = i
                while j < len(crops) and crops[j].shape[-1] == crops[i].shape[-1]:
                    j += 1
                feats.append(self.trunk(torch.cat(crops[i:j])))
                i = j
        return self.heads[0](torch.cat(feats))

    @torch.no_grad()
    def normalize_prototypes(self):
        w = self.heads[0].prototypes0.weight
        w.copy_(F.normalize(w, dim=1, p=2))

    def prototype_param_names(self):
        return [n for n, _ in self.named_parameters() if "prototypes" in n]


def eager_twin(module: nn.Module, device=None, dtype=torch.float32) -> nn.Module:
    """The stock-PyTorch equivalent of a dedloc SwAV module (SwAVModel, ResNet50Trunk, Bottleneck, or
    an nn.Sequential of Bottlenecks) carrying the same parameters and buffers (state-dict keys are
    identical): the independent reference the parity tests compare the kernels against."""
    from ..models.resnet_swav import Bottleneck, ResNet50Trunk, SwAVModel

    if isinstance(module, SwAVModel):
        twin = EagerSwAVModel(num_prototypes=module.heads[0].prototypes0.out_features,
                              single_pass_every_crop=module.single_pass_every_crop)
    elif isinstance(module, ResNet50Trunk):
        twin = EagerResNet50Trunk()
    elif isinstance(module, Bottleneck):
        twin = _eager_bottleneck_like(module)
    elif isinstance(module, nn.Sequential) and all(isinstance(m, Bottleneck) for m in module):
        twin = nn.Sequential(*[_eager_bottleneck_like(m) for m in module])
    else:
        raise TypeError(f"no eager twin for {type(module).__name__}")
    sd = {k: v.detach().clone() for k, v in module.state_dict().items()}
    twin.load_state_dict(sd)
    twin = twin.to(dtype=dtype)
    return twin.to(device) if device is not None else twin


def _eager_bottleneck_like(m) -> EagerBottleneck:
    inplanes, planes = m.conv1.in_channels, m.conv1.out_channels
    down = None
    if m.downsample is not None:
        c = m.downsample[0]
        down = nn.Sequential(nn.Conv2d(c.in_channels, c.out_channels, 1, stride=c.stride, bias=False),
                             nn.BatchNorm2d(c.out_channels))
    return EagerBottleneck(inplanes, planes, m.conv2.stride[0], down)


# ------------------------------------------------------------------------------------------ loss
@torch.no_grad()
def vissl_sinkhorn(scores: torch.Tensor, epsilon: float, iters: int) -> torch.Tensor:
    """swav_loss.py:177-244 + the log-sum-exp trick of :262-270, world size 1: [n, K] -> [n, K]."""
    a = scores / epsilon
    Q = torch.exp(a - a.max()).t()  # K x n
    Q /= Q.sum()
    K, n = Q.shape
    r = torch.ones(K, device=Q.device, dtype=Q.dtype) / K
    c = torch.ones(n, device=Q.device, dtype=Q.dtype) / n
    curr = Q.sum(dim=1)
    for _ in range(iters):
        Q *= (r / curr).unsqueeze(1)
        Q *= (c / Q.sum(dim=0)).unsqueeze(0)
        curr = Q.sum(dim=1)
    return (Q / Q.sum(dim=0, keepdim=True)).t()


class EagerSwAVLoss(nn.Module):
    """vissl SwAVLoss / SwAVCriterion op by op, with the DeDLOC queue gate on the GLOBAL step
    (``swav_loss.py:84-91``)."""

    def __init__(self, num_crops=8, crops_for_assign=(0, 1), temperature=0.1, epsilon=0.03, num_iters=3,
                 num_prototypes=3000, embedding_dim=128, queue_length=0, queue_start_iter=0, batch_size=64,
                 temp_hard_assignment_iters=0):
        super().__init__()
        self.num_crops, self.crops_for_assign = num_crops, list(crops_for_assign)
        self.temperature, self.epsilon, self.num_iters = temperature, epsilon, num_iters
        self.queue_length, self.queue_start_iter, self.bs = queue_length, queue_start_iter, batch_size
        self.temp_hard_assignment_iters = temp_hard_assignment_iters
        self.num_iteration = 0
        self.use_queue = False
        if queue_length:
            stdv = 1.0 / math.sqrt(embedding_dim / 3)
            self.register_buffer("queue", torch.rand(len(self.crops_for_assign), queue_length, embedding_dim)
                                 .mul_(2 * stdv).add_(-stdv))
            self.queue_ptr = 0

    def forward(self, embedding, scores, prototypes, training_iterations: int = 0):
        bs = self.bs
        self.use_queue = self.queue_length > 0 and training_iterations >= self.queue_start_iter
        total = 0.0
        for i, crop_id in enumerate(self.crops_for_assign):
            with torch.no_grad():
                s = scores[bs * crop_id: bs * (crop_id + 1)].float()
                if self.use_queue:  # vissl: batch rows first, queue after, assignments [:bs]
                    s = torch.cat([s, self.queue[i] @ prototypes.detach().float().t()])
                q = vissl_sinkhorn(s, self.epsilon, self.num_iters)[:bs]
                if self.num_iteration < self.temp_hard_assignment_iters:
                    q = torch.zeros_like(q).scatter_(1, q.argmax(dim=1, keepdim=True), 1.0)
            loss = 0.0
            others = [v for v in range(self.num_crops) if v != crop_id]
            for v in others:
                loss = loss - torch.mean(torch.sum(q * F.log_softmax(scores[bs * v: bs * (v + 1)].float()
                                                                     / self.temperature, dim=1), dim=1))
            total = total + loss / len(others)
        self.num_iteration += 1
        if self.use_queue:
            with torch.no_grad():
                for i, crop_id in enumerate(self.crops_for_assign):
                    e = embedding[bs * crop_id: bs * (crop_id + 1)].detach().float()
                    idx = (torch.arange(bs, device=e.device) + self.queue_ptr) % self.queue_length
                    self.queue[i].index_copy_(0, idx, e)
                self.queue_ptr = (self.queue_ptr + bs) % self.queue_length
        return total / len(self.crops_for_assign)


# ------------------------------------------------------------------------------------- optimizer
class EagerLarcSGD:
    """apex LARC(SGD(momentum)) over the parameter tensors of ``flat``, one tensor at a time (the
    reference's optimizer, sgd_collaborative.py:137-144); the interface of optim.lamb.FusedLarcSGD."""

    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                 trust_coefficient: float = 0.001, clip: bool = False, eps: float = 1e-8,
                 no_decay: Iterable[str] = ()):
        self.flat = flat
        self.param_groups = [dict(lr=lr, momentum=momentum, weight_decay=weight_decay,
                                  trust_coefficient=trust_coefficient, clip=clip, eps=eps)]
        no_decay = set(no_decay)
        self.wd = {n: (0.0 if n in no_decay else weight_decay) for n in flat.names}
        self.momentum_buffer = torch.zeros_like(flat.fp32)
        self.step_count = 0

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, grad: Optional[torch.Tensor] = None, grad_scale: float = 1.0):
        grp = self.param_groups[0]
        g_all = self.flat.grad if grad is None else grad
        lr, mom, tc, eps = grp["lr"], grp["momentum"], grp["trust_coefficient"], grp["eps"]
        for n in self.flat.names:
            p, g, buf = self.flat.view(self.flat.fp32, n), self.flat.view(g_all, n), self.flat.view(self.momentum_buffer, n)
            if grad_scale != 1.0:
                g = g * grad_scale
            wd = self.wd[n]
            pn, gn = torch.norm(p), torch.norm(g)
            rate = tc * pn / (gn + pn * wd + eps)
            if grp["clip"]:
                rate = torch.clamp(rate / lr, max=1.0)
            rate = torch.where((pn != 0) & (gn != 0), rate, torch.ones_like(rate))
            d = (g + wd * p) * rate
            if self.step_count == 0:
                buf.copy_(d)
            else:
                buf.mul_(mom).add_(d)
            p.add_(buf, alpha=-lr)
        self.step_count += 1

    def state_tensors(self) -> List[torch.Tensor]:
        return [self.momentum_buffer]

    def state_dict(self) -> Dict:
        return {"state": {i: {"momentum_buffer": self.flat.view(self.momentum_buffer, n).clone()}
                          for i, n in enumerate(self.flat.names)},
                "param_groups": [dict(self.param_groups[0])], "step": self.step_count}

    @torch.no_grad()
    def load_state_dict(self, sd: Dict):
        for i, n in enumerate(self.flat.names):
            s = sd.get("state", {}).get(i)
            if s:
                self.flat.view(self.momentum_buffer, n).copy_(s["momentum_buffer"])
        self.step_count = int(sd.get("step", self.step_count))


def clone_for_eager(model, device) -> EagerSwAVModel:
    """An EagerSwAVModel with ``model``'s parameters and buffers (same keys), on ``device``."""
    return eager_twin(copy.deepcopy(model).cpu(), device=device)
