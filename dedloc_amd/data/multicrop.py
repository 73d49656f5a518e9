"""Synthetic ImageNet + multi-crop SwAV augmentation, generated on the GPU.

Reference pipeline: ``vissl/data/ssl_transforms/img_pil_to_multicrop.py:11-74``
(RandomResizedCrop 2x224 scale (0.14, 1) + 6x96 scale (0.05, 0.14)), RandomHorizontalFlip(0.5),
``img_pil_color_distortion.py`` (ColorJitter(0.8s, 0.8s, 0.8s, 0.2s) with p=0.8, RandomGrayscale
p=0.2), ``img_pil_gaussian_blur.py`` (p=0.5, radius 0.1-2.0), ToTensor, Normalize, and
``collators/multicrop_collator.py:7-55`` (one stacked tensor per crop position).

There is no ImageNet here (no network), so the source images are a fixed pool of smooth random
RGB images generated on the device (``data="synthetic"``); every augmentation is a batched tensor op
on the GPU (one affine grid_sample per crop position, per-sample colour factors, per-sample
separable Gaussian kernels as one grouped conv), so the host never decodes or transforms JPEGs.
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


class MultiCropAugment:
    def __init__(self, size_crops: Sequence[int] = (224, 96), num_crops: Sequence[int] = (2, 6),
                 crop_scales: Sequence[Tuple[float, float]] = ((0.14, 1.0), (0.05, 0.14)),
                 flip_p: float = 0.5, color_strength: float = 1.0, color_p: float = 0.8, gray_p: float = 0.2,
                 blur_p: float = 0.5, blur_radius: Tuple[float, float] = (0.1, 2.0),
                 mean=IMAGENET_MEAN, std=IMAGENET_STD):
        self.size_crops, self.num_crops, self.crop_scales = list(size_crops), list(num_crops), list(crop_scales)
        self.flip_p, self.s, self.color_p, self.gray_p = flip_p, color_strength, color_p, gray_p
        self.blur_p, self.blur_radius = blur_p, blur_radius
        self.mean, self.std = mean, std

    # ---------------------------------------------------------------- geometry
    @staticmethod
    def _rrc_theta(b: int, scale, ratio, flip_p, gen, device) -> torch.Tensor:
        """Affine grids for RandomResizedCrop (+ horizontal flip) in normalized coordinates."""
        area = torch.empty(b, device=device).uniform_(scale[0], scale[1], generator=gen)
        logr = torch.empty(b, device=device).uniform_(math.log(ratio[0]), math.log(ratio[1]), generator=gen)
        r = torch.exp(logr)
        w = torch.sqrt(area * r).clamp(max=1.0)  # fraction of the source width
        h = torch.sqrt(area / r).clamp(max=1.0)
        cx = (torch.rand(b, device=device, generator=gen) * (1 - w) + w / 2) * 2 - 1
        cy = (torch.rand(b, device=device, generator=gen) * (1 - h) + h / 2) * 2 - 1
        flip = torch.where(torch.rand(b, device=device, generator=gen) < flip_p, -1.0, 1.0)
        theta = torch.zeros(b, 2, 3, device=device)
        theta[:, 0, 0] = w * flip
        theta[:, 0, 2] = cx
        theta[:, 1, 1] = h
        theta[:, 1, 2] = cy
        return theta

    # ---------------------------------------------------------------- photometric
    def _color(self, x: torch.Tensor, gen) -> torch.Tensor:
        b, dev, s = x.shape[0], x.device, self.s

        def u(lo, hi):
            return torch.empty(b, 1, 1, 1, device=dev).uniform_(lo, hi, generator=gen)

        apply = (torch.rand(b, 1, 1, 1, device=dev, generator=gen) < self.color_p).float()
        lum_w = torch.tensor([0.299, 0.587, 0.114], device=dev).view(1, 3, 1, 1)
        y = x
        y = y * u(max(0.0, 1 - 0.8 * s), 1 + 0.8 * s)                                   # brightness
        gray_mean = (y * lum_w).sum(1, keepdim=True).mean(dim=(2, 3), keepdim=True)
        c = u(max(0.0, 1 - 0.8 * s), 1 + 0.8 * s)
        y = (y - gray_mean) * c + gray_mean                                               # contrast
        g = (y * lum_w).sum(1, keepdim=True)
        sat = u(max(0.0, 1 - 0.8 * s), 1 + 0.8 * s)
        y = (y - g) * sat + g                                                             # saturation
        hue = u(-0.2 * s, 0.2 * s) * (2 * math.pi)                                        # hue (YIQ rotation)
        yiq = torch.tensor([[0.299, 0.587, 0.114], [0.596, -0.274, -0.322], [0.211, -0.523, 0.312]], device=dev)
        rgb = torch.linalg.inv(yiq)
        t = torch.einsum("ij,bjhw->bihw", yiq, y)
        ch, sh = torch.cos(hue), torch.sin(hue)
        i2 = t[:, 1:2] * ch - t[:, 2:3] * sh
        q2 = t[:, 1:2] * sh + t[:, 2:3] * ch
        y = torch.einsum("ij,bjhw->bihw", rgb, torch.cat([t[:, :1], i2, q2], 1))
        y = y.clamp(0, 1)
        x = apply * y + (1 - apply) * x
        grey = (torch.rand(b, 1, 1, 1, device=dev, generator=gen) < self.gray_p).float()
        g = (x * lum_w).sum(1, keepdim=True).expand_as(x)
        return grey * g + (1 - grey) * x

    def _blur(self, x: torch.Tensor, gen) -> torch.Tensor:
        b, c, hgt, wid = x.shape
        dev = x.device
        sigma = torch.empty(b, device=dev).uniform_(*self.blur_radius, generator=gen)
        apply = torch.rand(b, device=dev, generator=gen) < self.blur_p
        rad = int(math.ceil(3 * self.blur_radius[1]))
        k = torch.arange(-rad, rad + 1, device=dev, dtype=torch.float32)
        ker = torch.exp(-(k.view(1, -1) ** 2) / (2 * sigma.view(-1, 1) ** 2))
        ker = ker / ker.sum(1, keepdim=True)
        ident = torch.zeros_like(ker)
        ident[:, rad] = 1.0
        ker = torch.where(apply.view(-1, 1), ker, ident)           # p=0.5: identity kernel otherwise
        ker = ker.repeat_interleave(c, dim=0)                        # [b*c, K]
        y = x.reshape(1, b * c, hgt, wid)
        y = F.conv2d(F.pad(y, (rad, rad, 0, 0), mode="reflect"), ker.view(b * c, 1, 1, -1), groups=b * c)
        y = F.conv2d(F.pad(y, (0, 0, rad, rad), mode="reflect"), ker.view(b * c, 1, -1, 1), groups=b * c)
        return y.view(b, c, hgt, wid)

    @torch.no_grad()
    def __call__(self, images: torch.Tensor, gen: torch.Generator, out_dtype=torch.bfloat16) -> List[torch.Tensor]:
        b = images.shape[0]
        mean = torch.tensor(self.mean, device=images.device).view(1, 3, 1, 1)
        std = torch.tensor(self.std, device=images.device).view(1, 3, 1, 1)
        crops = []
        for size, n, scale in zip(self.size_crops, self.num_crops, self.crop_scales):
            # all n crops of one resolution in one batched pass (n*b images): ~70 launches per
            # resolution instead of per crop — the iteration is launch-bound at b=64
            src = images.repeat(n, 1, 1, 1) if n > 1 else images
            theta = self._rrc_theta(n * b, scale, (3 / 4, 4 / 3), self.flip_p, gen, images.device)
            grid = F.affine_grid(theta, [n * b, 3, size, size], align_corners=False)
            x = F.grid_sample(src, grid, mode="bilinear", padding_mode="border", align_corners=False)
            x = self._blur(self._color(x, gen), gen)
            x = ((x - mean) / std).to(out_dtype).contiguous(memory_format=torch.channels_last)
            crops.extend(x.split(b))
        return crops


class SyntheticMultiCropStream:
    """Per-peer stream of multi-crop batches drawn from a device-resident synthetic image pool."""

    def __init__(self, batch_size: int, device, seed: int = 0, pool_size: int = 1024, image_size: int = 256,
                 augment: MultiCropAugment = None, out_dtype=torch.bfloat16):
        self.batch_size, self.device = batch_size, torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.pool = _smooth_images(pool_size, image_size, self.gen, self.device)
        self.augment = augment or MultiCropAugment()
        self.out_dtype = out_dtype

    def next_batch(self) -> List[torch.Tensor]:
        idx = torch.randint(0, self.pool.shape[0], (self.batch_size,), device=self.device, generator=self.gen)
        return self.augment(self.pool.index_select(0, idx), self.gen, self.out_dtype)
