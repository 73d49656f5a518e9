"""ALBERT for pre-training (MLM + sentence-order prediction) on dedloc kernels.

Parity target: HF ``AlbertForPreTraining`` as built by ``albert/run_trainer.py:56-70`` from the
``albert-large-v2`` config.  State-dict keys, shapes, initialisation and
the ``config.json`` / ``pytorch_model.bin`` checkpoint layout are identical to HF, so checkpoints
round-trip with ``transformers`` (tested against it in tests/test_albert_model.py).

MI355X-first execution (not a port of HF's module graph):
  * parameters live in one flat fp32 buffer (``FlatParams``); compute uses its bf16 mirror;
    Q/K/V weights are adjacent so the three projections run as ONE [3H, H] GEMM;
  * attention is the fused flash kernel over the packed QKV buffer (no head transposes);
  * residual add + LayerNorm, embedding gather + LayerNorm and gelu_new are fused HIP kernels;
  * the MLM head runs only on masked positions, and its decoder + softmax-CE is one fused pass;
  * every parameter gradient accumulates in fp32 directly in the flat gradient buffer.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field, fields
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..utils.flat import FlatParams

NEG_BIG = -1.0e30


@dataclass
class AlbertConfig:
    vocab_size: int = 30000
    embedding_size: int = 128
    hidden_size: int = 4096
    num_hidden_layers: int = 12
    num_hidden_groups: int = 1
    num_attention_heads: int = 64
    intermediate_size: int = 16384
    inner_group_num: int = 1
    hidden_act: str = "gelu_new"
    hidden_dropout_prob: float = 0.0
    attention_probs_dropout_prob: float = 0.0
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    classifier_dropout_prob: float = 0.1
    num_labels: Optional[int] = None  # classification heads (HF writes it to config.json as well)
    pad_token_id: int = 0
    bos_token_id: int = 2
    eos_token_id: int = 3
    model_type: str = "albert"
    architectures: List[str] = field(default_factory=lambda: ["AlbertForPreTraining"])

    @classmethod
    def albert_large_v2(cls, **kw) -> "AlbertConfig":
        """The config the reference downloads at albert/arguments.py:97-99."""
        base = dict(vocab_size=30000, embedding_size=128, hidden_size=1024, num_hidden_layers=24,
                    num_hidden_groups=1, num_attention_heads=16, intermediate_size=4096, inner_group_num=1)
        base.update(kw)
        return cls(**base)

    @classmethod
    def albert_base_v2(cls, **kw) -> "AlbertConfig":
        """albert-base-v2 (HF model card sizes): 12 x 768, 12 heads of 64."""
        base = dict(vocab_size=30000, embedding_size=128, hidden_size=768, num_hidden_layers=12,
                    num_hidden_groups=1, num_attention_heads=12, intermediate_size=3072, inner_group_num=1)
        base.update(kw)
        return cls(**base)

    @classmethod
    def albert_xxlarge_v2(cls, **kw) -> "AlbertConfig":
        """albert-xxlarge-v2 (= transformers.AlbertConfig's defaults): 12 x 4096, 64 heads of 64."""
        base = dict(vocab_size=30000, embedding_size=128, hidden_size=4096, num_hidden_layers=12,
                    num_hidden_groups=1, num_attention_heads=64, intermediate_size=16384, inner_group_num=1)
        base.update(kw)
        return cls(**base)

    @classmethod
    def albert_xlarge_v2(cls, **kw) -> "AlbertConfig":
        """albert-xlarge-v2 (HF model card sizes): 24 x 2048, 16 heads of 128 — outside the fused
        attention kernels' head_dim 64, so its attention runs the composed path
        (ops.attn_composed_fwd / _bwd: batched bf16 GEMMs, fp32 scores)."""
        base = dict(vocab_size=30000, embedding_size=128, hidden_size=2048, num_hidden_layers=24,
                    num_hidden_groups=1, num_attention_heads=16, intermediate_size=8192, inner_group_num=1)
        base.update(kw)
        return cls(**base)

    BUILTIN = {"albert-large-v2": "albert_large_v2", "albert-base-v2": "albert_base_v2",
               "albert-xlarge-v2": "albert_xlarge_v2", "albert-xxlarge-v2": "albert_xxlarge_v2"}

    @classmethod
    def tiny(cls, **kw) -> "AlbertConfig":
        base = dict(vocab_size=512, embedding_size=64, hidden_size=128, num_hidden_layers=3, num_hidden_groups=1,
                    num_attention_heads=2, intermediate_size=256, max_position_embeddings=128)
        base.update(kw)
        return cls(**base)

    def to_dict(self) -> Dict:
        d = asdict(self)
        if d.get("num_labels") is None:  # HF's PretrainedConfig rejects num_labels=None
            d.pop("num_labels", None)
        return d

    @classmethod
    def from_dict(cls, d: Dict) -> "AlbertConfig":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    @classmethod
    def from_pretrained(cls, path: str) -> "AlbertConfig":
        """Accepts a directory containing config.json, a json file, or the name 'albert-large-v2' /
        'albert-base-v2' / 'albert-xxlarge-v2' (or the reference-style S3 URL of such a config —
        there is no network, so it maps to the built-in copy)."""
        for name, ctor in cls.BUILTIN.items():
            if path == name or (isinstance(path, str) and path.endswith(f"{name}-config.json")
                                and not os.path.exists(path)):
                return getattr(cls, ctor)()
        if os.path.isdir(path):
            path = os.path.join(path, "config.json")
        with open(path) as f:
            return cls.from_dict(json.load(f))

    def save_pretrained(self, directory: str):
        os.makedirs(directory, exist_ok=True)
        with open(os.path.join(directory, "config.json"), "w") as f:
            json.dump(self.to_dict(), f, indent=2, sort_keys=True)


def _layer_prefix(g: int, i: int) -> str:
    return f"albert.encoder.albert_layer_groups.{g}.albert_layers.{i}."


# The residual sums ride in the output-projection / FFN-down GEMM epilogues (C = h, beta = 1): the
# LayerNorms then read one tensor and write one — 2 of 4 LN HBM passes removed (round 2).
# (Module constants, not environment knobs: tests and bench/ab_step.py flip them in-process.)
_RESIDUAL_IN_GEMM = True
# The backward's data-gradient GEMMs (dX = dY W) run against transposed weight copies made once per
# encoder call (the 24 layers share them): gemm8 with both operands K-inner beats the K-outer-B form
# by 5-10% on these shapes (profiles/gemm8_asm_dma_layouts_T131072.log).
_DGRAD_WT = True
# Weight gradients of the shared layer keep their token-split fp32 slabs across the layer
# applications and add them into the flat gradient once, at the last backward call
# (gemm_acc_f32_shared).
_SHARED_WGRAD = True
# The FFN-up epilogue stores gelu_new'(h) (bf16) for the backward instead of the pre-activation h:
# it shares the forward's exp2 / rcp, and the FFN-down data gradient's epilogue becomes one multiply
# instead of a second sigmoid evaluation per element (gemm_gelu_d / gemm_dmul, gemm8 EPI 6 / 7).
_GELU_GRAD_IN_FWD = True


class _AlbertLayerFn(torch.autograd.Function):
    """One application of the shared ALBERT transformer layer with a hand-scheduled backward.

    fwd: qkv = h Wqkv^T + b (one GEMM) -> flash attention -> dense -> LN(. + h) -> ffn -> gelu_new
         -> ffn_output -> LN(. + h1)
    bwd: every weight gradient accumulates in fp32 into the flat gradient buffer (beta = 1 GEMMs),
         and both residual-branch gradient sums are folded into the dgrad GEMMs (C = ds + dY W),
         so the layer backward launches no standalone elementwise adds.
    """

    @staticmethod
    def forward(ctx, h, mask, lv, H, S, eps):
        O = ops.OPS
        mbias, kvinfo = mask
        qkv = O.gemm(h, lv["wqkv"], lv["bqkv32"], None, False, True, 0)
        att, lse = ops.attn_fwd(qkv, mbias, H, S, 1.0 / math.sqrt(qkv.shape[1] // (3 * H)), kvinfo)
        if _RESIDUAL_IN_GEMM:
            # residual sums ride in the GEMM epilogues (C = h, beta = 1): the LayerNorms then read one
            # tensor and write one (s is the GEMM output itself) — 2 of 4 LN HBM passes removed
            s1 = O.gemm(att, lv["wo"], lv["bo32"], h, False, True, 0)
            h1, _, m1, r1 = O.layernorm_fwd(s1, None, lv["ln1g"], lv["ln1b"], eps)
            # bias + gelu_new fused in the GEMM epilogue; f = gelu_new'(h) (or h itself)
            f, g = (O.gemm_gelu_d if _GELU_GRAD_IN_FWD else O.gemm_gelu)(h1, lv["w1"], lv["b132"])
            s2 = O.gemm(g, lv["w2"], lv["b232"], h1, False, True, 0)
            out, _, m2, r2 = O.layernorm_fwd(s2, None, lv["ln2g"], lv["ln2b"], eps)
        else:
            a = O.gemm(att, lv["wo"], lv["bo32"], None, False, True, 0)
            h1, s1, m1, r1 = O.layernorm_fwd(a, h, lv["ln1g"], lv["ln1b"], eps)
            f, g = (O.gemm_gelu_d if _GELU_GRAD_IN_FWD else O.gemm_gelu)(h1, lv["w1"], lv["b132"])
            f2 = O.gemm(g, lv["w2"], lv["b232"], None, False, True, 0)
            out, s2, m2, r2 = O.layernorm_fwd(f2, h1, lv["ln2g"], lv["ln2b"], eps)
        ctx.save_for_backward(h, qkv, att, lse, s1, m1, r1, h1, f, g, s2, m2, r2)
        ctx.lv, ctx.mask, ctx.H, ctx.S = lv, mask, H, S
        ctx.gelu_d = _GELU_GRAD_IN_FWD
        return out

    @staticmethod
    def backward(ctx, dy):
        O = ops.OPS
        h, qkv, att, lse, s1, m1, r1, h1, f, g, s2, m2, r2 = ctx.saved_tensors
        lv = ctx.lv
        dy = dy.contiguous()
        H = ctx.H
        # LN backward also accumulates colsum(ds) = the bias grad of the Linear that fed it
        ds2 = O.layernorm_bwd(dy, s2, lv["ln2g"], m2, r2, lv["gln2g"], lv["gln2b"], True, lv["gb2"])
        _wgrad(O, ds2, g, lv, "gw2")
        wt = "w2t" in lv  # transposed weight copies present (see _DGRAD_WT)
        # dgrad * gelu'(h) + ffn bias grad, one kernel (f holds gelu'(h) itself, or h)
        dfn = O.gemm_dmul if ctx.gelu_d else O.gemm_dgelu
        df = dfn(ds2, lv["w2t"], f, lv["gb1"], True) if wt else dfn(ds2, lv["w2"], f, lv["gb1"])
        _wgrad(O, df, h1, lv, "gw1")
        dh1 = _dgrad(O, df, lv, "w1", ds2)  # residual branch folded in
        del df
        ds1 = O.layernorm_bwd(dh1, s1, lv["ln1g"], m1, r1, lv["gln1g"], lv["gln1b"], True, lv["gbo"])
        _wgrad(O, ds1, att, lv, "gwo")
        datt = _dgrad(O, ds1, lv, "wo", None)
        # the QKV bias gradient rides in the attention backward (query: colsum dQ, value: colsum
        # datt, key: exactly zero — softmax is shift invariant), no separate column-sum pass
        dqkv = ops.attn_bwd(qkv, ctx.mask[0], att, datt, lse, H, ctx.S, 1.0 / math.sqrt(qkv.shape[1] // (3 * H)),
                          ctx.mask[1], lv["gbqkv"])
        _wgrad(O, dqkv, h, lv, "gwqkv")
        dh = _dgrad(O, dqkv, lv, "wqkv", ds1)
        return dh, None, None, None, None, None


def _wgrad(O, dy, x, lv, name):
    """lv[name] += dY^T X; with the layer's position among the applications of its weights
    (``wg_first`` / ``wg_last``, set by encode) the slab sum is deferred to the last backward call.
    (Forking these GEMMs onto a side stream beside the memory-bound kernels measured 10% slower
    free-running and no gain paired; removed in round 4.)"""
    if "wg_first" in lv:
        O.gemm_acc_f32_shared(dy, x, lv[name], True, False, lv["wg_first"], lv["wg_last"])
    else:
        O.gemm_acc_f32(dy, x, lv[name], True, False)


def _dgrad(O, dy, lv, name, residual):
    """dX = dY W (+ residual), against W^T's forward-layout copy when the layer views carry one."""
    if name + "t" in lv:
        return O.gemm(dy, lv[name + "t"], None, residual, False, True, 0)
    return O.gemm(dy, lv[name], None, residual, False, False, 0)


@torch.no_grad()
def _with_transposed_weights(lv: Dict) -> Dict:
    lv = dict(lv)
    for name in ("wqkv", "wo", "w1", "w2"):
        lv[name + "t"] = lv[name].t().contiguous()
    return lv


class AlbertPreTrainedModel(nn.Module):
    """Shared ALBERT trunk (embeddings, mapping-in, the shared layer group(s), optional pooler) with
    HF-compatible parameter names, flat fp32/bf16 storage and the fused encoder forward.  Heads are
    added by the subclasses (pre-training, sequence / token classification)."""

    add_pooler = True

    def __init__(self, config: AlbertConfig):
        super().__init__()
        self.config = c = config
        self._p: Dict[str, nn.Parameter] = {}
        E, H, I, V = c.embedding_size, c.hidden_size, c.intermediate_size, c.vocab_size
        add = self._add
        add("albert.embeddings.word_embeddings.weight", V, E)
        add("albert.embeddings.position_embeddings.weight", c.max_position_embeddings, E)
        add("albert.embeddings.token_type_embeddings.weight", c.type_vocab_size, E)
        with torch.no_grad():
            self._p["albert.embeddings.word_embeddings.weight"][c.pad_token_id].zero_()
        add("albert.embeddings.LayerNorm.weight", E, init="ones")
        add("albert.embeddings.LayerNorm.bias", E, init="zeros")
        add("albert.encoder.embedding_hidden_mapping_in.weight", H, E)
        add("albert.encoder.embedding_hidden_mapping_in.bias", H, init="zeros")
        for g in range(c.num_hidden_groups):
            for i in range(c.inner_group_num):
                pre = _layer_prefix(g, i)
                add(pre + "full_layer_layer_norm.weight", H, init="ones")
                add(pre + "full_layer_layer_norm.bias", H, init="zeros")
                for n in ("query", "key", "value"):
                    add(pre + f"attention.{n}.weight", H, H)
                for n in ("query", "key", "value"):
                    add(pre + f"attention.{n}.bias", H, init="zeros")
                add(pre + "attention.dense.weight", H, H)
                add(pre + "attention.dense.bias", H, init="zeros")
                add(pre + "attention.LayerNorm.weight", H, init="ones")
                add(pre + "attention.LayerNorm.bias", H, init="zeros")
                add(pre + "ffn.weight", I, H)
                add(pre + "ffn.bias", I, init="zeros")
                add(pre + "ffn_output.weight", H, I)
                add(pre + "ffn_output.bias", H, init="zeros")
        if self.add_pooler:
            add("albert.pooler.weight", H, H)
            add("albert.pooler.bias", H, init="zeros")
        self._add_heads()
        self.flat: Optional[FlatParams] = None

    def _add(self, name, *shape, init="normal"):
        t = torch.empty(*shape)
        if init == "normal":
            t.normal_(0.0, self.config.initializer_range)
        elif init == "ones":
            t.fill_(1.0)
        else:
            t.zero_()
        p = nn.Parameter(t)
        self._p[name] = p
        self.register_parameter(name.replace(".", "__"), p)

    def _add_heads(self):
        pass

    # ------------------------------------------------------------------ parameters / checkpoints
    def hf_named_parameters(self):
        return list(self._p.items())

    def materialize(self, device=None) -> FlatParams:
        """Move parameters into the flat buffers on ``device`` (call once before training)."""
        device = torch.device(device) if device is not None else next(iter(self._p.values())).device
        for p in self._p.values():
            p.data = p.data.to(device)
        self.flat = FlatParams(self.hf_named_parameters(), device=device)
        return self.flat

    def hf_state_dict(self) -> Dict[str, torch.Tensor]:
        """state dict with exactly the HF model class's keys."""
        return {k: v.detach() for k, v in self._p.items()}

    @torch.no_grad()
    def load_hf_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        missing = [k for k in self._p if k not in sd]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:5]}...")
        for k, p in self._p.items():
            if k in sd:
                p.data.copy_(sd[k].to(p.dtype))
        if self.flat is not None:
            self.flat.refresh_bf16()

    def save_pretrained(self, directory: str):
        os.makedirs(directory, exist_ok=True)
        self.config.save_pretrained(directory)
        # tied entries are stored as separate tensors, as HF's torch.save of the state dict does
        sd = {k: v.detach().float().cpu().contiguous().clone() for k, v in self.hf_state_dict().items()}
        torch.save(sd, os.path.join(directory, "pytorch_model.bin"))

    @classmethod
    def from_pretrained(cls, directory: str, strict: Optional[bool] = None, **config_overrides):
        """Load a checkpoint directory.  Head classes loading a pre-training checkpoint keep their
        freshly initialised head (HF behaviour), so ``strict`` defaults to True only for the class
        that wrote it (keys must all be present)."""
        cfg = AlbertConfig.from_pretrained(directory)
        for k, v in config_overrides.items():
            setattr(cfg, k, v)
        model = cls(cfg)
        sd_path = os.path.join(directory, "pytorch_model.bin")
        if os.path.exists(sd_path):
            sd = torch.load(sd_path, map_location="cpu", weights_only=True)
        else:
            from safetensors.torch import load_file

            sd = load_file(os.path.join(directory, "model.safetensors"))
        if strict is None:
            strict = all(k in sd for k in model._p if not k.startswith("albert."))
        model.load_hf_state_dict(sd, strict=strict)
        return model

    def resize_token_embeddings(self, n: int):
        """HF semantics: grow/shrink the (tied) vocabulary; new rows ~ N(0, init_range)."""
        c = self.config
        if n == c.vocab_size:
            return
        assert self.flat is None, "resize before materialize()"
        for key in ("albert.embeddings.word_embeddings.weight", "predictions.bias"):
            if key not in self._p:
                continue
            old = self._p[key].data
            new = torch.empty((n,) + tuple(old.shape[1:]))
            if key.endswith("weight"):
                new.normal_(0.0, c.initializer_range)
            else:
                new.zero_()
            k = min(n, old.shape[0])
            new[:k] = old[:k]
            self._p[key].data = new
        c.vocab_size = n

    def no_decay_names(self) -> List[str]:
        """Reference grouping (albert/run_trainer.py:74-84): names containing 'bias' or
        'LayerNorm.weight' get no weight decay (full_layer_layer_norm.weight *is* decayed — SURVEY App. C.2)."""
        return [n for n in self._p if any(nd in n for nd in ("bias", "LayerNorm.weight"))]

    # ------------------------------------------------------------------ forward
    def _layer_views(self, g: int, i: int):
        f = self.flat
        pre = _layer_prefix(g, i)
        H = self.config.hidden_size
        return dict(
            wqkv=f.span(f.bf16, pre + "attention.query.weight", pre + "attention.value.weight", (3 * H, H)),
            gwqkv=f.span(f.grad, pre + "attention.query.weight", pre + "attention.value.weight", (3 * H, H)),
            bqkv=f.span(f.bf16, pre + "attention.query.bias", pre + "attention.value.bias", (3 * H,)),
            bqkv32=f.span(f.fp32, pre + "attention.query.bias", pre + "attention.value.bias", (3 * H,)),
            bo32=f.p(pre + "attention.dense.bias"), b132=f.p(pre + "ffn.bias"), b232=f.p(pre + "ffn_output.bias"),
            gbqkv=f.span(f.grad, pre + "attention.query.bias", pre + "attention.value.bias", (3 * H,)),
            wo=f.w(pre + "attention.dense.weight"), gwo=f.g(pre + "attention.dense.weight"),
            bo=f.w(pre + "attention.dense.bias"), gbo=f.g(pre + "attention.dense.bias"),
            ln1g=f.p(pre + "attention.LayerNorm.weight"), ln1b=f.p(pre + "attention.LayerNorm.bias"),
            gln1g=f.g(pre + "attention.LayerNorm.weight"), gln1b=f.g(pre + "attention.LayerNorm.bias"),
            w1=f.w(pre + "ffn.weight"), gw1=f.g(pre + "ffn.weight"), b1=f.w(pre + "ffn.bias"), gb1=f.g(pre + "ffn.bias"),
            w2=f.w(pre + "ffn_output.weight"), gw2=f.g(pre + "ffn_output.weight"),
            b2=f.w(pre + "ffn_output.bias"), gb2=f.g(pre + "ffn_output.bias"),
            ln2g=f.p(pre + "full_layer_layer_norm.weight"), ln2b=f.p(pre + "full_layer_layer_norm.bias"),
            gln2g=f.g(pre + "full_layer_layer_norm.weight"), gln2b=f.g(pre + "full_layer_layer_norm.bias"),
        )

    def _albert_layer(self, h, lv, mask, S):
        c = self.config
        return _AlbertLayerFn.apply(h, mask, lv, c.num_attention_heads, S, c.layer_norm_eps)

    def encode(self, input_ids, attention_mask=None, token_type_ids=None):
        """Returns (sequence_output [B*S', H] bf16, S') where S' is S padded to a multiple of 64."""
        assert self.flat is not None, "call model.materialize(device) first"
        c, f = self.config, self.flat
        B, S = input_ids.shape
        Sp = (S + 63) // 64 * 64
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        if Sp != S:
            pad = Sp - S
            input_ids = F.pad(input_ids, (0, pad), value=c.pad_token_id)
            attention_mask = F.pad(attention_mask, (0, pad), value=0)
            if token_type_ids is not None:
                token_type_ids = F.pad(token_type_ids, (0, pad), value=0)
        assert Sp <= c.max_position_embeddings, "sequence longer than max_position_embeddings"
        am = attention_mask.bool()
        mbias = torch.where(am, 0.0, NEG_BIG).to(torch.float32).contiguous()
        # right-padded masks (the usual case) let the attention kernels skip padded key tiles: pass
        # the lengths plus an on-device "every row is a prefix mask" flag (no host sync)
        lens = am.sum(1, dtype=torch.int32)
        prefix = (am == (torch.arange(Sp, device=am.device) < lens[:, None])).all()
        kvinfo = torch.cat([lens, prefix.to(torch.int32).view(1)]).contiguous()
        mask = (mbias, kvinfo)
        emb = "albert.embeddings."
        x = ops.embed_layernorm(
            input_ids, token_type_ids, f.p(emb + "word_embeddings.weight"), f.p(emb + "position_embeddings.weight"),
            f.p(emb + "token_type_embeddings.weight"), f.p(emb + "LayerNorm.weight"), f.p(emb + "LayerNorm.bias"),
            grads=(f.g(emb + "word_embeddings.weight"), f.g(emb + "position_embeddings.weight"),
                   f.g(emb + "token_type_embeddings.weight"), f.g(emb + "LayerNorm.weight"),
                   f.g(emb + "LayerNorm.bias")),
            eps=c.layer_norm_eps)
        m = "albert.encoder.embedding_hidden_mapping_in."
        h = ops.linear(x, f.w(m + "weight"), f.w(m + "bias"), f.g(m + "weight"), f.g(m + "bias"))
        views = [[self._layer_views(g, i) for i in range(c.inner_group_num)] for g in range(c.num_hidden_groups)]
        if _DGRAD_WT and torch.is_grad_enabled():
            views = [[_with_transposed_weights(lv) for lv in row] for row in views]
        per_group = c.num_hidden_layers // c.num_hidden_groups
        group_of = [int(layer / per_group) for layer in range(c.num_hidden_layers)]
        for layer in range(c.num_hidden_layers):
            g = group_of[layer]
            uses = [x for x in range(c.num_hidden_layers) if group_of[x] == g]
            for i in range(c.inner_group_num):
                lv = views[g][i]
                if _SHARED_WGRAD and torch.is_grad_enabled():
                    # backward runs the layers in reverse: the last application is the first to
                    # write the weight's gradient slabs, the first application sums them in
                    lv = dict(lv, wg_first=layer == uses[-1], wg_last=layer == uses[0])
                h = self._albert_layer(h, lv, mask, Sp)
        return h, Sp

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self._p.values())


class AlbertForPreTraining(AlbertPreTrainedModel):
    """HF ``AlbertForPreTraining`` (MLM head with the decoder tied to the word embeddings + SOP head)."""

    def _add_heads(self):
        c = self.config
        E, H, V = c.embedding_size, c.hidden_size, c.vocab_size
        add = self._add
        add("predictions.bias", V, init="zeros")
        add("predictions.dense.weight", E, H)
        add("predictions.dense.bias", E, init="zeros")
        add("predictions.LayerNorm.weight", E, init="ones")
        add("predictions.LayerNorm.bias", E, init="zeros")
        add("sop_classifier.classifier.weight", 2, H)
        add("sop_classifier.classifier.bias", 2, init="zeros")

    def hf_state_dict(self) -> Dict[str, torch.Tensor]:
        """state dict with exactly HF AlbertForPreTraining's keys (tied decoder included)."""
        sd = super().hf_state_dict()
        sd["predictions.decoder.weight"] = sd["albert.embeddings.word_embeddings.weight"]
        sd["predictions.decoder.bias"] = sd["predictions.bias"]
        return sd

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None, sentence_order_label=None,
                mlm_positions=None, mlm_labels=None, return_logits=False):
        """HF-compatible pre-training forward.

        MLM targets either as HF ``labels`` [B, S] (-100 = ignore) or as fixed-shape
        ``mlm_positions``/``mlm_labels`` [B, P] (BERT's max_predictions_per_seq form; -100 pads) —
        the fixed form needs no host synchronisation and is graph-capturable.
        """
        c, f = self.config, self.flat
        B, S = input_ids.shape
        h, Sp = self.encode(input_ids, attention_mask, token_type_ids)
        out = {}
        # ---- MLM head on masked positions only
        if mlm_positions is None and labels is not None:
            flat_lab = labels.reshape(-1)
            pos = torch.nonzero(flat_lab != -100).squeeze(1)
            b_idx, s_idx = pos // S, pos % S
            rows = b_idx * Sp + s_idx
            tgt = flat_lab[pos]
        elif mlm_positions is not None:
            P = mlm_positions.shape[1]
            rows = (torch.arange(B, device=h.device)[:, None] * Sp + mlm_positions).reshape(-1)
            tgt = mlm_labels.reshape(-1)
        else:
            rows, tgt = None, None
        loss = None
        if rows is not None:
            hm = h.index_select(0, rows)
            p = "predictions."
            t = ops.linear(hm, f.w(p + "dense.weight"), f.w(p + "dense.bias"), f.g(p + "dense.weight"),
                           f.g(p + "dense.bias"))
            t = ops.gelu_new(t)
            t = ops.add_layernorm(t, None, f.p(p + "LayerNorm.weight"), f.p(p + "LayerNorm.bias"),
                                  f.g(p + "LayerNorm.weight"), f.g(p + "LayerNorm.bias"), c.layer_norm_eps)
            wname = "albert.embeddings.word_embeddings.weight"
            logits = ops.linear(t, f.w(wname), f.w(p + "bias"), f.g(wname), f.g(p + "bias"))
            mlm_loss = ops.cross_entropy(logits, tgt)
            out["mlm_loss"] = mlm_loss
            loss = mlm_loss
            if return_logits:
                out["prediction_logits_masked"] = logits
        # ---- SOP head on [CLS]
        cls = h.view(B, Sp, -1)[:, 0].contiguous()
        pooled = ops.tanh(ops.linear(cls, f.w("albert.pooler.weight"), f.w("albert.pooler.bias"),
                                     f.g("albert.pooler.weight"), f.g("albert.pooler.bias")))
        if self.training and c.classifier_dropout_prob > 0:
            pooled = F.dropout(pooled, c.classifier_dropout_prob, True)
        s = "sop_classifier.classifier."
        sop_logits = ops.linear(pooled, f.w(s + "weight"), f.w(s + "bias"), f.g(s + "weight"), f.g(s + "bias"))
        out["sop_logits"] = sop_logits
        if sentence_order_label is not None:
            sop_loss = ops.cross_entropy(sop_logits, sentence_order_label)
            out["sop_loss"] = sop_loss
            loss = sop_loss if loss is None else loss + sop_loss
        out["loss"] = loss
        return out


class AlbertForSequenceClassification(AlbertPreTrainedModel):
    """HF ``AlbertForSequenceClassification``: pooler(tanh) on [CLS] -> dropout -> classifier.
    Cross-entropy for ``num_labels > 1``, MSE for regression (``num_labels == 1``).  Used by the
    sahajBERT NCC fine-tuning recipe (reference sahajbert/train_ncc.py)."""

    def __init__(self, config: AlbertConfig, num_labels: Optional[int] = None):
        self.num_labels = int(num_labels or config.num_labels or 2)
        config.num_labels = self.num_labels
        super().__init__(config)

    def _add_heads(self):
        self._add("classifier.weight", self.num_labels, self.config.hidden_size)
        self._add("classifier.bias", self.num_labels, init="zeros")

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None):
        c, f = self.config, self.flat
        B = input_ids.shape[0]
        h, Sp = self.encode(input_ids, attention_mask, token_type_ids)
        cls = h.view(B, Sp, -1)[:, 0].contiguous()
        pooled = ops.tanh(ops.linear(cls, f.w("albert.pooler.weight"), f.w("albert.pooler.bias"),
                                     f.g("albert.pooler.weight"), f.g("albert.pooler.bias")))
        if self.training and c.classifier_dropout_prob > 0:
            pooled = F.dropout(pooled, c.classifier_dropout_prob, True)
        logits = ops.linear(pooled, f.w("classifier.weight"), f.w("classifier.bias"), f.g("classifier.weight"),
                            f.g("classifier.bias"))
        out = {"logits": logits}
        if labels is not None:
            if self.num_labels == 1:
                out["loss"] = F.mse_loss(logits.float().view(-1), labels.float().view(-1))
            else:
                out["loss"] = ops.cross_entropy(logits, labels)
        return out


class AlbertForTokenClassification(AlbertPreTrainedModel):
    """HF ``AlbertForTokenClassification`` (no pooler): dropout -> per-token classifier, CE over the
    positions whose label != -100.  Used by the sahajBERT NER recipe (reference sahajbert/train_ner.py)."""

    add_pooler = False

    def __init__(self, config: AlbertConfig, num_labels: Optional[int] = None):
        self.num_labels = int(num_labels or config.num_labels or 2)
        config.num_labels = self.num_labels
        super().__init__(config)

    def _add_heads(self):
        self._add("classifier.weight", self.num_labels, self.config.hidden_size)
        self._add("classifier.bias", self.num_labels, init="zeros")

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None):
        c, f = self.config, self.flat
        B, S = input_ids.shape
        h, Sp = self.encode(input_ids, attention_mask, token_type_ids)
        if self.training and c.classifier_dropout_prob > 0:
            h = F.dropout(h, c.classifier_dropout_prob, True)
        logits = ops.linear(h, f.w("classifier.weight"), f.w("classifier.bias"), f.g("classifier.weight"),
                            f.g("classifier.bias"))
        out = {"logits": logits.view(B, Sp, -1)[:, :S]}
        if labels is not None:
            lab = labels
            if Sp != S:
                lab = F.pad(labels, (0, Sp - S), value=-100)
            out["loss"] = ops.cross_entropy(logits, lab.reshape(-1))
        return out


def flops_per_sample(config: AlbertConfig, seq_len: int, masked_per_seq: int) -> float:
    """Model FLOPs (fwd+bwd = 3x fwd) per training sample, used for MFU reporting."""
    c = config
    H, I, E = c.hidden_size, c.intermediate_size, c.embedding_size
    per_tok_layer = 2 * (4 * H * H + 2 * H * I)
    attn = 2 * 2 * seq_len * H
    fwd = seq_len * (c.num_hidden_layers * (per_tok_layer + attn) + 2 * E * H)
    fwd += masked_per_seq * (2 * H * E + 2 * E * c.vocab_size)
    return 3.0 * fwd
