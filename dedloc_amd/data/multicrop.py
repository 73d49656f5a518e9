"""Synthetic ImageNet + multi-crop SwAV augmentation, generated on the GPU.

Reference pipeline: ``vissl/data/ssl_transforms/img_pil_to_multicrop.py:11-74``
(RandomResizedCrop 2x224 scale (0.14, 1) + 6x96 scale (0.05, 0.14)), RandomHorizontalFlip(0.5),
``img_pil_color_distortion.py`` (ColorJitter(0.8s, 0.8s, 0.8s, 0.2s) with p=0.8, RandomGrayscale
p=0.2), ``img_pil_gaussian_blur.py`` (p=0.5, radius 0.1-2.0), ToTensor, Normalize, and
``collators/multicrop_collator.py:7-55`` (one stacked tensor per crop position).

There is no ImageNet here (no network), so the source images are a fixed pool of smooth random
RGB images generated on the device (``data="synthetic"``).  Every random draw of a batch is made on
the host into one [n*b, 20] parameter table per crop resolution (``MultiCropAugment.sample_params``);
the augmentation itself is ``torch.ops.dedloc.multicrop`` — four HIP kernels per resolution on the
GPU (csrc/kernels/augment.hip: bilinear RandomResizedCrop+flip, colour jitter + grayscale, separable
Gaussian blur, Normalize + bf16 channels-last store) and ``augment_reference`` (plain tensor ops) on
the CPU and as the numerics reference.  The host never decodes or transforms JPEGs.
Differences from the PIL path: ColorJitter applies its four ops in a fixed order (torchvision
permutes them) and hue is rotated in YIQ space.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import torch
import torch.nn.functional as F

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
NP = 20  # parameter-table row, layout in csrc/kernels/augment.hip
_YIQ = torch.tensor([[0.299, 0.587, 0.114], [0.596, -0.274, -0.322], [0.211, -0.523, 0.312]], dtype=torch.float64)
_LUM = (0.299, 0.587, 0.114)


def _smooth_images(n: int, size: int, gen: torch.Generator, device) -> torch.Tensor:
    """Pool of [n, 3, size, size] images in [0, 1]: multi-octave upsampled noise (natural-ish spectra)."""
    img = torch.zeros(n, 3, size, size, device=device)
    amp = 1.0
    for base in (4, 8, 16, 32, 64):
        noise = torch.rand(n, 3, base, base, generator=gen, device=device)
        img += amp * F.interpolate(noise, size=(size, size), mode="bilinear", align_corners=False)
        amp *= 0.5
    img -= img.amin(dim=(1, 2, 3), keepdim=True)
    img /= img.amax(dim=(1, 2, 3), keepdim=True).clamp_min(1e-6)
    return img


def augment_reference(pool: torch.Tensor, params: torch.Tensor, size: int, rad: int, mean, std) -> torch.Tensor:
    """Tensor-op implementation of ``dedloc::multicrop``: [nb, 3, size, size] bf16, channels-last."""
    prm = params.float()
    nb, dev = prm.shape[0], pool.device
    src = pool.index_select(0, prm[:, 0].long().clamp(0, pool.shape[0] - 1))
    theta = torch.zeros(nb, 2, 3, device=dev)
    theta[:, 0, 0], theta[:, 0, 2], theta[:, 1, 1], theta[:, 1, 2] = prm[:, 1], prm[:, 2], prm[:, 3], prm[:, 4]
    grid = F.affine_grid(theta, [nb, 3, size, size], align_corners=False)
    x = F.grid_sample(src, grid, mode="bilinear", padding_mode="border", align_corners=False)
    lum_w = torch.tensor(_LUM, device=dev).view(1, 3, 1, 1)

    def col(k):
        return prm[:, k].view(nb, 1, 1, 1)

    y = x * col(5)                                                                          # brightness
    gm = (y * lum_w).sum(1, keepdim=True).mean(dim=(2, 3), keepdim=True)
    y = (y - gm) * col(6) + gm                                                              # contrast
    g = (y * lum_w).sum(1, keepdim=True)
    y = (y - g) * col(7) + g                                                                # saturation
    y = torch.einsum("bij,bjhw->bihw", prm[:, 10:19].reshape(nb, 3, 3), y).clamp(0, 1)     # hue
    x = torch.where(col(8) != 0, y, x)
    x = torch.where(col(9) != 0, (x * lum_w).sum(1, keepdim=True).expand_as(x), x)          # grayscale
    k = torch.arange(-rad, rad + 1, device=dev, dtype=torch.float32)
    sigma = prm[:, 19]
    ker = torch.exp(-(k.view(1, -1) ** 2) / (2 * sigma.clamp_min(1e-6).view(-1, 1) ** 2))
    ker = ker / ker.sum(1, keepdim=True)
    ident = (k == 0).float().expand_as(ker)
    ker = torch.where((sigma > 0).view(-1, 1), ker, ident).repeat_interleave(3, dim=0)    # [nb*3, 2rad+1]
    x = x.reshape(1, nb * 3, size, size)
    x = F.conv2d(F.pad(x, (rad, rad, 0, 0), mode="reflect"), ker.view(nb * 3, 1, 1, -1), groups=nb * 3)
    x = F.conv2d(F.pad(x, (0, 0, rad, rad), mode="reflect"), ker.view(nb * 3, 1, -1, 1), groups=nb * 3)
    x = x.view(nb, 3, size, size)
    x = (x - torch.tensor(mean, device=dev).view(1, 3, 1, 1)) / torch.tensor(std, device=dev).view(1, 3, 1, 1)
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


class MultiCropAugment:
    def __init__(self, size_crops: Sequence[int] = (224, 96), num_crops: Sequence[int] = (2, 6),
                 crop_scales: Sequence[Tuple[float, float]] = ((0.14, 1.0), (0.05, 0.14)),
                 flip_p: float = 0.5, color_strength: float = 1.0, color_p: float = 0.8, gray_p: float = 0.2,
                 blur_p: float = 0.5, blur_radius: Tuple[float, float] = (0.1, 2.0),
                 mean=IMAGENET_MEAN, std=IMAGENET_STD):
        self.size_crops, self.num_crops, self.crop_scales = list(size_crops), list(num_crops), list(crop_scales)
        self.flip_p, self.s, self.color_p, self.gray_p = flip_p, color_strength, color_p, gray_p
        self.blur_p, self.blur_radius = blur_p, blur_radius
        self.mean, self.std = tuple(mean), tuple(std)
        self.rad = int(math.ceil(3 * self.blur_radius[1]))

    def sample_params(self, src: torch.Tensor, scale, gen: torch.Generator) -> torch.Tensor:
        """Host-side draws for one crop resolution: [nb, 20] fp32 table (layout: augment.hip)."""
        nb, s = src.shape[0], self.s

        def u(lo, hi):
            return torch.empty(nb, dtype=torch.float64).uniform_(lo, hi, generator=gen)

        def coin(p):
            return torch.rand(nb, dtype=torch.float64, generator=gen) < p

        # RandomResizedCrop(scale, ratio 3/4..4/3) + horizontal flip, normalized coordinates
        area = u(scale[0], scale[1])
        r = torch.exp(u(math.log(3 / 4), math.log(4 / 3)))
        w = torch.sqrt(area * r).clamp(max=1.0)
        h = torch.sqrt(area / r).clamp(max=1.0)
        cx = (torch.rand(nb, dtype=torch.float64, generator=gen) * (1 - w) + w / 2) * 2 - 1
        cy = (torch.rand(nb, dtype=torch.float64, generator=gen) * (1 - h) + h / 2) * 2 - 1
        flip = torch.where(coin(self.flip_p), -1.0, 1.0).double()
        lo, hi = max(0.0, 1 - 0.8 * s), 1 + 0.8 * s
        bright, contrast, sat = u(lo, hi), u(lo, hi), u(lo, hi)
        hue = u(-0.2 * s, 0.2 * s) * (2 * math.pi)
        apply, grey = coin(self.color_p).double(), coin(self.gray_p).double()
        sigma = u(*self.blur_radius)
        sigma = torch.where(coin(self.blur_p), sigma, torch.zeros_like(sigma))
        # hue: rotate the I/Q chroma plane of YIQ, folded into one RGB->RGB matrix per image
        rot = torch.zeros(nb, 3, 3, dtype=torch.float64)
        rot[:, 0, 0] = 1
        rot[:, 1, 1], rot[:, 1, 2], rot[:, 2, 1], rot[:, 2, 2] = hue.cos(), -hue.sin(), hue.sin(), hue.cos()
        M = torch.linalg.inv(_YIQ) @ rot @ _YIQ
        t = torch.stack([src.double(), w * flip, cx, h, cy, bright, contrast, sat, apply, grey], 1)
        return torch.cat([t, M.reshape(nb, 9), sigma.view(-1, 1)], 1).float()

    @torch.no_grad()
    def __call__(self, pool: torch.Tensor, src: torch.Tensor, gen: torch.Generator,
                 out_dtype=torch.bfloat16) -> List[torch.Tensor]:
        """``src``: [b] host indices into ``pool``; one [b, 3, s, s] channels-last tensor per crop."""
        import dedloc_amd.ops  # noqa: F401  (registers dedloc::multicrop)

        b = src.shape[0]
        crops = []
        for size, n, scale in zip(self.size_crops, self.num_crops, self.crop_scales):
            # all n crops of one resolution in one batched pass over n*b images
            params = self.sample_params(src.repeat(n), scale, gen)
            if pool.is_cuda:
                params = params.pin_memory().to(pool.device, non_blocking=True)
            x = torch.ops.dedloc.multicrop(pool, params, size, self.rad, list(self.mean), list(self.std))
            if x.dtype != out_dtype:
                x = x.to(out_dtype)
            crops.extend(x.split(b))
        return crops


class SyntheticMultiCropStream:
    """Per-peer stream of multi-crop batches drawn from a device-resident synthetic image pool."""

    def __init__(self, batch_size: int, device, seed: int = 0, pool_size: int = 1024, image_size: int = 256,
                 augment: MultiCropAugment = None, out_dtype=torch.bfloat16):
        self.batch_size, self.device = batch_size, torch.device(device)
        pool_gen = torch.Generator(device=self.device)
        pool_gen.manual_seed(seed)
        self.pool = _smooth_images(pool_size, image_size, pool_gen, self.device)
        self.gen = torch.Generator().manual_seed(seed)  # host draws: source images, geometry, colour, blur
        self.augment = augment or MultiCropAugment()
        self.out_dtype = out_dtype

    def next_batch(self) -> List[torch.Tensor]:
        idx = torch.randint(0, self.pool.shape[0], (self.batch_size,), generator=self.gen)
        return self.augment(self.pool, idx, self.gen, self.out_dtype)


class StreamPrefetcher:
    """Overlaps batch generation with training: while the caller's stream computes on batch i,
    batch i+1 is produced on a side stream (the reference's DataLoader workers prepare batches
    ahead on the CPU; here the augmentation kernels run ahead on the GPU).  ``next_batch`` makes the
    caller's stream wait for the batch it returns and records that stream on its tensors, so the
    caching allocator never hands their memory to the side stream while the caller still reads it."""

    def __init__(self, source, device):
        self.source = source
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._next = None

    def _launch(self):
        with torch.cuda.stream(self.stream):
            batch = self.source.next_batch()
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._next = (batch, ev)

    def next_batch(self) -> List[torch.Tensor]:
        if self.stream is None:
            return self.source.next_batch()
        if self._next is None:
            self._launch()
        batch, ev = self._next
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for t in batch:
            t.record_stream(cur)
        self._launch()  # the following batch, under this iteration's compute
        return batch

    def __getattr__(self, name):  # pool, batch_size, augment, ... of the wrapped stream
        if name == "source":  # not set yet (copy / unpickle): no recursion through __getattr__
            raise AttributeError(name)
        return getattr(self.source, name)
