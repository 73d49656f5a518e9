"""Flat parameter / gradient storage (MI355X-first memory layout).

All parameters of a model live in ONE contiguous fp32 allocation (each tensor 64-element aligned so
every view is 256-byte aligned), with one bf16 mirror used by the compute kernels and one fp32
gradient buffer that the fused-accumulation ops write into.  Optimizers, gradient clipping,
averaging pack/unpack and state transfer therefore operate on a handful of large buffers with a
single kernel launch each instead of per-tensor loops.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, List, Tuple

import torch

ALIGN = 64


def _round_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class FlatParams:
    """Re-homes ``named_params`` into a flat fp32 buffer; parameters become views into it.

    Two modes:
      * manual-backward models (ALBERT): parameters stop requiring grad; the layer Functions write
        their weight gradients straight into ``grad`` views;
      * ``autograd=True`` (torch-module models such as the SwAV ResNet): parameters keep
        ``requires_grad`` and their ``.grad`` is pre-bound to the ``grad`` view, so autograd's
        AccumulateGrad adds in place into the flat buffer.  With ``channels_last=True`` every 4-D
        parameter (conv weight) is laid out NHWC (KRSC) inside the flat buffer, the layout the
        implicit-GEMM conv kernels read, so weights are never transposed for the forward.
    """

    def __init__(self, named_params: Iterable[Tuple[str, torch.nn.Parameter]], device=None,
                 with_bf16: bool = True, autograd: bool = False, channels_last: bool = False):
        named = list(named_params)
        seen = {}
        self.names: List[str] = []
        self.params: "OrderedDict[str, torch.nn.Parameter]" = OrderedDict()
        for n, p in named:
            if id(p) in seen:  # tied parameters are stored once
                continue
            seen[id(p)] = n
            self.names.append(n)
            self.params[n] = p
        device = device or named[0][1].device
        self.offsets: Dict[str, int] = {}
        off = 0
        for n in self.names:
            self.offsets[n] = off
            off += _round_up(self.params[n].numel())
        self.numel = off
        self.device = torch.device(device)
        self.fp32 = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.bf16 = torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device) if with_bf16 else None
        self.autograd = autograd
        self.nhwc = {n for n in self.names if channels_last and self.params[n].dim() == 4}
        for n in self.names:
            p = self.params[n]
            v = self.view(self.fp32, n)
            v.copy_(p.data)
            p.data = v
            if autograd:
                p.grad = self.view(self.grad, n)
            else:
                p.requires_grad_(False)
        self.refresh_bf16()

    # ------------------------------------------------------------------ views
    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        p = self.params[name]
        o = self.offsets[name]
        if name in self.nhwc:
            k, c, h, w = p.shape
            return buf[o:o + p.numel()].view(k, h, w, c).permute(0, 3, 1, 2)
        return buf[o:o + p.numel()].view(p.shape)

    def rebind_grads(self):
        """Re-attach ``.grad`` views (after something replaced or cleared a parameter's grad)."""
        if self.autograd:
            for n in self.names:
                self.params[n].grad = self.view(self.grad, n)

    def span(self, buf: torch.Tensor, first: str, last: str, shape) -> torch.Tensor:
        """A view over the contiguous range [first, last] (requires the names to be adjacent)."""
        i0, i1 = self.names.index(first), self.names.index(last)
        o0 = self.offsets[first]
        o1 = self.offsets[last] + self.params[last].numel()
        for a, b in zip(self.names[i0:i1], self.names[i0 + 1:i1 + 1]):
            assert self.offsets[a] + self.params[a].numel() == self.offsets[b], f"{a} and {b} are not adjacent"
        return buf[o0:o1].view(*shape)

    def w(self, name):  # bf16 compute view
        return self.view(self.bf16, name)

    def g(self, name):  # fp32 grad view
        return self.view(self.grad, name)

    def p(self, name):  # fp32 master view
        return self.view(self.fp32, name)

    # ------------------------------------------------------------------ maintenance
    @torch.no_grad()
    def refresh_bf16(self):
        if self.bf16 is None:
            return
        if self.fp32.is_cuda:
            torch.ops.dedloc.cast_bf16(self.fp32, self.bf16)
        else:
            self.bf16.copy_(self.fp32)

    def zero_grad(self):
        self.grad.zero_()

    def tensor_table(self):
        """(names, offsets, sizes) of every stored parameter in flat order."""
        return [(n, self.offsets[n], self.params[n].numel()) for n in self.names]

    def chunk_table(self, chunk: int = 16384, weight_decay: Dict[str, float] | None = None):
        """Chunk decomposition for the multi-tensor optimizer kernels.

        Returns device tensors (chunk_tensor int32, chunk_start int64, chunk_len int32, tensor_wd fp32).
        """
        ct, cs, cl, wd = [], [], [], []
        for ti, (n, off, size) in enumerate(self.tensor_table()):
            wd.append(0.0 if weight_decay is None else float(weight_decay.get(n, 0.0)))
            for s in range(0, size, chunk):
                ct.append(ti)
                cs.append(off + s)
                cl.append(min(chunk, size - s))
        dev = self.device
        return (torch.tensor(ct, dtype=torch.int32, device=dev), torch.tensor(cs, dtype=torch.int64, device=dev),
                torch.tensor(cl, dtype=torch.int32, device=dev), torch.tensor(wd, dtype=torch.float32, device=dev))
