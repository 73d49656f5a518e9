"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (GPU tier)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

OPS = None


@pytest.fixture(autouse=True)
def _ops(cuda):
    global OPS
    import dedloc_amd.ops  # noqa: F401

    OPS = torch.ops.dedloc


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("D", [64, 128, 768, 1024, 2048, 4096])
@pytest.mark.parametrize("with_res", [False, True])
def test_layernorm(cuda, D, with_res):
    torch.manual_seed(0)
    rows = 1000
    x = torch.randn(rows, D, device=cuda).bfloat16()
    r = torch.randn(rows, D, device=cuda).bfloat16() if with_res else None
    g = torch.rand(D, device=cuda) + 0.5
    b = torch.randn(D, device=cuda)
    y, s, mean, rstd = OPS.layernorm_fwd(x, r, g, b, 1e-12)
    s_ref = x.float() + (r.float() if with_res else 0)
    s_ref.requires_grad_(True)
    y_ref = F.layer_norm(s_ref, (D,), g, b, 1e-12)
    assert rel(y, y_ref) < 1e-2
    dy = torch.randn(rows, D, device=cuda).bfloat16()
    dg = torch.zeros(D, device=cuda)
    db = torch.zeros(D, device=cuda)
    ds = OPS.layernorm_bwd(dy, s, g, mean, rstd, dg, db, False)
    gref = torch.autograd.grad(y_ref, [s_ref], dy.float())[0]
    assert rel(ds, gref) < 2e-2
    xh = (s.float() - mean[:, None]) * rstd[:, None]
    assert rel(dg, (dy.float() * xh).sum(0)) < 1e-3
    assert rel(db, dy.float().sum(0)) < 1e-3


def test_gelu(cuda):
    x = torch.randn(4096, 512, device=cuda).bfloat16()
    y = OPS.gelu_fwd(x)
    xr = x.float().requires_grad_(True)
    yr = F.gelu(xr, approximate="tanh")
    assert rel(y, yr) < 1e-2
    dy = torch.randn_like(x)
    dx = OPS.gelu_bwd(dy, x)
    assert rel(dx, torch.autograd.grad(yr, xr, dy.float())[0]) < 1e-2


def _attn_ref(qkv, mask, H, S):
    T, ld = qkv.shape
    D = ld // (3 * H)
    B = T // S
    x = qkv.float().reshape(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    bias = torch.where(mask.bool(), 0.0, float("-inf"))[:, None, None, :]
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias)
    return o.permute(0, 2, 1, 3).reshape(B * S, H * D)


@pytest.mark.parametrize("B,H,S", [(2, 2, 64), (2, 4, 128), (4, 16, 512), (1, 3, 192)])
def test_attention(cuda, B, H, S):
    torch.manual_seed(1)
    D = 64
    qkv = (torch.randn(B * S, 3 * H * D, device=cuda) * 1.5).bfloat16()
    mask = torch.ones(B, S, device=cuda, dtype=torch.long)
    mask[-1, S - S // 4:] = 0
    mbias = torch.where(mask.bool(), 0.0, -1e30).float()
    out, lse = OPS.attn_fwd(qkv, mbias, H, S, 1 / math.sqrt(D))
    qkv_r = qkv.float().requires_grad_(True)
    ref = _attn_ref(qkv_r, mask, H, S)
    assert rel(out, ref) < 1.5e-2, rel(out, ref)
    dout = torch.randn_like(out)
    dbias = torch.full((3 * H * D,), 0.25, device=cuda)
    dqkv = OPS.attn_bwd(qkv, mbias, out, dout, lse, H, S, 1 / math.sqrt(D), None, dbias)
    g_ref = torch.autograd.grad(ref, qkv_r, dout.float())[0]
    for part in range(3):
        sl = slice(part * H * D, (part + 1) * H * D)
        assert rel(dqkv[:, sl], g_ref[:, sl]) < 3e-2, (part, rel(dqkv[:, sl], g_ref[:, sl]))
    # fused QKV bias gradient (accumulated): query = colsum(dQ), key = 0 exactly (softmax shift
    # invariance: the reference's colsum(dK) is rounding noise around 0), value = colsum(dout)
    HD = H * D
    bref = g_ref.sum(0)
    assert rel(dbias[:HD] - 0.25, dqkv[:, :HD].float().sum(0)) < 1e-4
    assert rel(dbias[:HD] - 0.25, bref[:HD]) < 3e-2
    assert torch.equal(dbias[HD:2 * HD], torch.full_like(dbias[HD:2 * HD], 0.25))
    assert bref[HD:2 * HD].abs().max().item() < 1e-3 * bref[:HD].abs().max().item() + 1e-3
    assert rel(dbias[2 * HD:] - 0.25, bref[2 * HD:]) < 1e-2


def test_attention_large_logits(cuda):
    # forces the online-softmax rescale path: one key spikes late in the sequence
    B, H, S, D = 1, 2, 256, 64
    qkv = torch.randn(B * S, 3 * H * D, device=cuda).bfloat16()
    qkv[200, H * D:2 * H * D] *= 12
    out, lse = OPS.attn_fwd(qkv, None, H, S, 1 / math.sqrt(D))
    ref = _attn_ref(qkv.float(), torch.ones(B, S, device=cuda), H, S)
    assert rel(out, ref) < 1.5e-2


def _kvinfo(mask):
    lens = mask.sum(1).int()
    prefix = (mask.bool() == (torch.arange(mask.shape[1], device=mask.device) < lens[:, None])).all()
    return torch.cat([lens, prefix.int().view(1)]).contiguous()


@pytest.mark.parametrize("lens", [(256, 200, 64, 37), (256, 256, 256, 256), (1, 65, 128, 255)])
def test_attention_kv_lengths(cuda, lens):
    """Right-padded masks via kvinfo: padded key tiles are skipped, the boundary tile is masked."""
    torch.manual_seed(3)
    B, H, S, D = len(lens), 2, 256, 64
    qkv = (torch.randn(B * S, 3 * H * D, device=cuda) * 1.5).bfloat16()
    mask = (torch.arange(S, device=cuda)[None, :] < torch.tensor(lens, device=cuda)[:, None]).long()
    mbias = torch.where(mask.bool(), 0.0, -1e30).float()
    kvinfo = _kvinfo(mask)
    assert kvinfo[-1].item() == 1
    out, lse = OPS.attn_fwd(qkv, mbias, H, S, 1 / math.sqrt(D), kvinfo)
    out_b, _ = OPS.attn_fwd(qkv, mbias, H, S, 1 / math.sqrt(D))  # generic bias path
    qkv_r = qkv.float().requires_grad_(True)
    ref = _attn_ref(qkv_r, mask, H, S)
    assert rel(out, ref) < 1.5e-2, rel(out, ref)
    assert rel(out, out_b) < 1e-2
    dout = torch.randn_like(out)
    dqkv = OPS.attn_bwd(qkv, mbias, out, dout, lse, H, S, 1 / math.sqrt(D), kvinfo)
    g_ref = torch.autograd.grad(ref, qkv_r, dout.float())[0]
    for part in range(3):
        sl = slice(part * H * D, (part + 1) * H * D)
        assert rel(dqkv[:, sl], g_ref[:, sl]) < 3e-2, (part, rel(dqkv[:, sl], g_ref[:, sl]))
    # keys past a row's length get exactly zero dK / dV
    for b, n in enumerate(lens):
        if n < S:
            assert dqkv[b * S + n:(b + 1) * S, H * D:].abs().max().item() == 0.0


def test_attention_non_prefix_mask_falls_back_to_bias(cuda):
    torch.manual_seed(4)
    B, H, S, D = 2, 2, 128, 64
    qkv = torch.randn(B * S, 3 * H * D, device=cuda).bfloat16()
    mask = torch.ones(B, S, device=cuda, dtype=torch.long)
    mask[0, 10:20] = 0  # a hole: not a prefix mask
    mbias = torch.where(mask.bool(), 0.0, -1e30).float()
    kvinfo = _kvinfo(mask)
    assert kvinfo[-1].item() == 0
    out, lse = OPS.attn_fwd(qkv, mbias, H, S, 1 / math.sqrt(D), kvinfo)
    ref = _attn_ref(qkv.float(), mask, H, S)
    assert rel(out, ref) < 1.5e-2


def test_attention_deferred_rescale_ramp(cuda):
    """Data-dependent deferred-max rescale: key magnitudes ramp up tile by tile, at different rates per
    head, so some rows cross the rescale threshold at different tiles and others never do."""
    torch.manual_seed(5)
    B, H, S, D = 2, 4, 512, 64
    qkv = torch.randn(B * S, 3 * H * D, device=cuda)
    ramp = 1.0 + torch.arange(S, device=cuda).float() / 64.0  # grows per 64-key tile
    for h in range(H):
        cols = slice(H * D + h * D, H * D + (h + 1) * D)
        qkv[:, cols] *= (ramp.repeat(B) ** (0.5 * h))[:, None]
    qkv = qkv.bfloat16()
    out, lse = OPS.attn_fwd(qkv, None, H, S, 1 / math.sqrt(D))
    qkv_r = qkv.float().requires_grad_(True)
    ref = _attn_ref(qkv_r, torch.ones(B, S, device=cuda), H, S)
    assert rel(out, ref) < 1.5e-2, rel(out, ref)
    dout = torch.randn_like(out)
    dqkv = OPS.attn_bwd(qkv, None, out, dout, lse, H, S, 1 / math.sqrt(D))
    g_ref = torch.autograd.grad(ref, qkv_r, dout.float())[0]
    assert rel(dqkv, g_ref) < 3e-2


@pytest.mark.parametrize("S,lens,generic", [(192, (192, 100, 64), False), (512, (512, 300, 17), False),
                                             (256, (256, 130, 200), True), (64, (64, 33, 1), False),
                                             (1024, (1024, 700, 513), False)])
def test_attention_kernels_masks_and_tails(cuda, S, lens, generic):
    """The flash-attention kernels forward and backward (incl. the fused QKV bias gradient), on
    length masks and on the generic additive bias; S = 192 leaves the last 256-query block of the
    two-sub-block kernels partly empty."""
    torch.manual_seed(11)
    B, H, D = len(lens), 2, 64
    qkv = (torch.randn(B * S, 3 * H * D, device=cuda) * 1.5).bfloat16()
    mask = (torch.arange(S, device=cuda)[None, :] < torch.tensor(lens, device=cuda)[:, None]).long()
    if generic:
        mask[0, 5:9] = 0  # a hole: not a prefix mask -> the additive-bias path
    mbias = torch.where(mask.bool(), 0.0, -1e30).float()
    kvinfo = _kvinfo(mask)
    out, lse = OPS.attn_fwd(qkv, mbias, H, S, 1 / math.sqrt(D), kvinfo)
    qkv_r = qkv.float().requires_grad_(True)
    ref = _attn_ref(qkv_r, mask, H, S)
    assert rel(out, ref) < 1.5e-2, rel(out, ref)
    dout = torch.randn_like(out)
    dbias = torch.zeros(3 * H * D, device=cuda)
    dqkv = OPS.attn_bwd(qkv, mbias, out, dout, lse, H, S, 1 / math.sqrt(D), kvinfo, dbias)
    g_ref = torch.autograd.grad(ref, qkv_r, dout.float())[0]
    for part in range(3):
        sl = slice(part * H * D, (part + 1) * H * D)
        assert rel(dqkv[:, sl], g_ref[:, sl]) < 3e-2, (part, rel(dqkv[:, sl], g_ref[:, sl]))
    HD = H * D
    assert rel(dbias[:HD], dqkv[:, :HD].float().sum(0)) < 1e-4
    assert rel(dbias[2 * HD:], dout.float().sum(0)) < 1e-4


def test_embedding(cuda):
    torch.manual_seed(2)
    B, S, E, V = 4, 128, 128, 1000
    ids = torch.randint(0, V, (B * S,), device=cuda)
    tt = torch.randint(0, 2, (B * S,), device=cuda)
    w = torch.randn(V, E, device=cuda)
    p = torch.randn(512, E, device=cuda)
    t = torch.randn(2, E, device=cuda)
    g = torch.rand(E, device=cuda) + 0.5
    b = torch.randn(E, device=cuda)
    y, s, mean, rstd = OPS.embed_ln_fwd(ids, tt, w, p, t, g, b, S, 1e-12)
    pos = torch.arange(B * S, device=cuda) % S
    ref = F.layer_norm(w[ids] + p[pos] + t[tt], (E,), g, b, 1e-12)
    assert rel(y, ref) < 1e-2
    ds = torch.randn(B * S, E, device=cuda).bfloat16()
    dw, dp, dt = torch.zeros_like(w), torch.zeros_like(p), torch.zeros_like(t)
    OPS.embed_bwd(ds, ids, tt, dw, dp, dt, S)
    dw_r = torch.zeros_like(w).index_add_(0, ids, ds.float())
    dp_r = torch.zeros_like(p).index_add_(0, pos, ds.float())
    dt_r = torch.zeros_like(t).index_add_(0, tt, ds.float())
    assert rel(dw, dw_r) < 1e-4 and rel(dp, dp_r) < 1e-4 and rel(dt, dt_r) < 1e-4


@pytest.mark.parametrize("V", [30000, 2, 31995])
def test_xent(cuda, V):
    M = 300
    x = (torch.randn(M, V, device=cuda) * 3).bfloat16()
    lab = torch.randint(0, V, (M,), device=cuda)
    lab[::7] = -100
    loss, dl = OPS.xent_fwd_bwd(x, lab, False, -100)
    xr = x.float().requires_grad_(True)
    lr = F.cross_entropy(xr, lab, ignore_index=-100)
    assert abs(loss.item() - lr.item()) < 1e-3 * max(1, abs(lr.item()))
    assert rel(dl, torch.autograd.grad(lr, xr)[0]) < 1e-2


def _chunks(sizes, wd, dev, chunk=1000):
    ct, cs, cl = [], [], []
    off = 0
    offs = []
    for i, n in enumerate(sizes):
        offs.append(off)
        for s in range(0, n, chunk):
            ct.append(i)
            cs.append(off + s)
            cl.append(min(chunk, n - s))
        off += n
    return (torch.tensor(ct, dtype=torch.int32, device=dev), torch.tensor(cs, dtype=torch.int64, device=dev),
            torch.tensor(cl, dtype=torch.int32, device=dev), torch.tensor(wd, dtype=torch.float32, device=dev), offs)


def test_lamb_matches_reference(cuda):
    torch.manual_seed(3)
    sizes = [4096, 1000, 37, 2500]
    wd = [0.01, 0.0, 0.01, 0.0]
    n = sum(sizes)
    p = torch.randn(n, device=cuda)
    ct, cs, cl, twd, offs = _chunks(sizes, wd, cuda)
    m = torch.zeros(n, device=cuda)
    v = torch.zeros(n, device=cuda)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    norms = torch.zeros(2 * len(sizes), device=cuda)
    lr, b1, b2, eps = 1.76e-3, 0.9, 0.999, 1e-6
    for step in range(1, 4):
        g = torch.randn(n, device=cuda)
        bc = math.sqrt(1 - b2 ** step) / (1 - b1 ** step)
        OPS.lamb_step(p, g, m, v, ct, cs, cl, twd, norms, b1, b2, eps, lr * bc, 10.0, 1.0)
        for i, (o, sz) in enumerate(zip(offs, sizes)):  # torch_optimizer.Lamb formula
            sl = slice(o, o + sz)
            mr[sl] = b1 * mr[sl] + (1 - b1) * g[sl]
            vr[sl] = b2 * vr[sl] + (1 - b2) * g[sl] ** 2
            wn = pr[sl].norm().clamp(0, 10.0)
            u = mr[sl] / (vr[sl].sqrt() + eps) + wd[i] * pr[sl]
            un = u.norm()
            trust = 1.0 if (wn == 0 or un == 0) else (wn / un).item()
            pr[sl] -= lr * bc * trust * u
    assert rel(p, pr) < 1e-5 and rel(m, mr) < 1e-5 and rel(v, vr) < 1e-4


def test_larc_sgd(cuda):
    torch.manual_seed(4)
    sizes = [3000, 64]
    wd = [1e-6, 1e-6]
    n = sum(sizes)
    p = torch.randn(n, device=cuda)
    buf = torch.zeros(n, device=cuda)
    ct, cs, cl, twd, offs = _chunks(sizes, wd, cuda)
    norms = torch.zeros(4, device=cuda)
    pr, br = p.clone(), buf.clone()
    lr, mom, trust = 0.3, 0.9, 1e-3
    for step in range(3):
        g = torch.randn(n, device=cuda)
        OPS.larc_sgd_step(p, g, buf, ct, cs, cl, twd, norms, lr, mom, trust, 1e-8, False, step == 0, 1.0)
        for i, (o, sz) in enumerate(zip(offs, sizes)):
            sl = slice(o, o + sz)
            pn, gn = pr[sl].norm(), g[sl].norm()
            a = trust * pn / (gn + pn * wd[i] + 1e-8)
            d = (g[sl] + wd[i] * pr[sl]) * a
            br[sl] = d if step == 0 else mom * br[sl] + d
            pr[sl] -= lr * br[sl]
    assert rel(p, pr) < 1e-5


def test_clip_and_axpby(cuda):
    g = torch.randn(100003, device=cuda) * 3
    ref = g.clone()
    part = torch.zeros(256, device=cuda)
    out = torch.zeros(2, device=cuda)
    OPS.grad_norm_clip(g, 1.0, part, out)
    n = ref.norm()
    assert abs(out[0].item() - n.item()) < 1e-3 * n.item() and out[1].item() == 1.0
    assert rel(g, ref * (1.0 / (n + 1e-6))) < 1e-5
    y = torch.randn(100003, device=cuda)
    y0 = y.clone()
    OPS.axpby(y, g, 0.5, 2.0)
    assert rel(y, 0.5 * y0 + 2.0 * g) < 1e-6
    g[5] = float("nan")
    OPS.grad_norm_clip(g, 1.0, part, out)
    assert out[1].item() == 0.0


@pytest.mark.parametrize("wire", [torch.float16, torch.bfloat16, torch.float32])
def test_pack_reduce_unpack(cuda, wire):
    n, k = 10007, 3
    xs = [torch.randn(n, device=cuda) for _ in range(k)]
    ws = [1.0, 2.0, 0.5]
    parts = torch.empty(k, n, dtype=wire, device=cuda)
    for i in range(k):
        OPS.pack(xs[i], parts[i], ws[i])
    avg = torch.empty(n, dtype=wire, device=cuda)
    OPS.reduce_parts(parts, k, avg, 1.0 / sum(ws))
    ref = sum(w * x for w, x in zip(ws, xs)) / sum(ws)
    tol = 1e-6 if wire == torch.float32 else (2e-3 if wire == torch.float16 else 1e-2)
    assert rel(avg, ref) < tol
    dst = torch.zeros(n, device=cuda)
    OPS.unpack(avg, dst, None)
    assert rel(dst, ref) < tol
    snap = torch.randn(n, device=cuda)
    loc = snap + 1.0
    OPS.unpack(avg, loc, snap)  # delta rule
    assert rel(loc, ref + 1.0) < tol * 3


@pytest.mark.parametrize("wire", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("k", [3, 20])  # 20 > the kernel's 16 register slots
def test_reduce_delta_and_unpack_add(cuda, wire, k):
    """The averaging path: per-sender deltas of the fp32 weighted mean, added to the fp32 master."""
    n = 10007
    torch.manual_seed(0)
    masters = [torch.randn(n, device=cuda) + 4.0 for _ in range(k)]
    ws = torch.rand(k, device=cuda) + 0.25
    parts = torch.empty(k, n, dtype=wire, device=cuda)
    for i in range(k):
        OPS.pack(masters[i], parts[i], 1.0)
    deltas = torch.empty_like(parts)
    OPS.reduce_delta(parts, ws, deltas)
    pf = parts.float()
    avg = (pf * ws[:, None]).sum(0) / ws.sum()
    ref = avg[None, :] - pf  # fp32 reference of the same op
    tol = 1e-6 if wire == torch.float32 else (2e-3 if wire == torch.float16 else 1e-2)
    assert (deltas.float() - ref).abs().max().item() <= tol * ref.abs().max().item() + 1e-6
    for i in range(k):
        m = masters[i].clone()
        OPS.unpack(deltas[i], m, None, True)
        torch.testing.assert_close(m, masters[i] + deltas[i].float())
    # identical contributions: deltas are exactly zero, the fp32 master is untouched
    same = parts[0:1].expand(k, n).contiguous()
    OPS.reduce_delta(same, ws, deltas)
    assert deltas.float().abs().max().item() == 0.0


def test_gemm_paths(cuda):
    a = torch.randn(300, 128, device=cuda).bfloat16()
    w = torch.randn(200, 128, device=cuda).bfloat16()
    b = torch.randn(200, device=cuda).bfloat16()
    y = OPS.gemm(a, w, b, None, False, True, 0)
    assert rel(y, a.float() @ w.float().t() + b.float()) < 1e-2
    c = torch.ones(200, 128, device=cuda)
    dy = torch.randn(300, 200, device=cuda).bfloat16()
    OPS.gemm_acc_f32(dy, a, c, True, False)
    assert rel(c, 1 + dy.float().t() @ a.float()) < 1e-2


@pytest.mark.parametrize("T,N,K", [(8192, 1024, 1024), (4096, 768, 256), (8192, 4096, 1024)])
def test_gemm_acc_f32_token_split(cuda, T, N, K):
    """Weight-gradient path: the token dimension is split into a strided batched GEMM + slab sum."""
    torch.manual_seed(7)
    x = torch.randn(T, K, device=cuda).bfloat16()
    dy = torch.randn(T, N, device=cuda).bfloat16()
    c = torch.randn(N, K, device=cuda)
    ref = c + dy.float().t() @ x.float()
    OPS.gemm_acc_f32(dy, x, c, True, False)
    assert rel(c, ref) < 1e-5, rel(c, ref)


def test_gemm_residual_and_bias_epilogue(cuda):
    torch.manual_seed(8)
    x = torch.randn(1024, 512, device=cuda).bfloat16()
    w = torch.randn(768, 512, device=cuda).bfloat16()
    b = torch.randn(768, device=cuda)
    r = torch.randn(1024, 768, device=cuda).bfloat16()
    assert rel(OPS.gemm(x, w, b, None, False, True, 0), x.float() @ w.float().t() + b) < 1e-2
    w2 = torch.randn(512, 768, device=cuda).bfloat16()
    assert rel(OPS.gemm(x, w2, None, r, False, False, 0), r.float() + x.float() @ w2.float()) < 1e-2


def test_albert_gpu_matches_cpu(cuda):
    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining

    torch.manual_seed(0)
    cfg = AlbertConfig.tiny(hidden_size=256, num_attention_heads=4, intermediate_size=1024, embedding_size=128)
    m_cpu = AlbertForPreTraining(cfg)
    m_gpu = AlbertForPreTraining(cfg)
    m_gpu.load_hf_state_dict(m_cpu.hf_state_dict())
    m_cpu.materialize("cpu")
    m_gpu.materialize(cuda)
    m_cpu.eval()
    m_gpu.eval()
    B, S = 2, 128
    ids = torch.randint(5, cfg.vocab_size, (B, S))
    am = torch.ones(B, S, dtype=torch.long)
    am[1, 100:] = 0
    labels = torch.full((B, S), -100)
    labels[:, 3:20] = ids[:, 3:20]
    sop = torch.tensor([0, 1])
    oc = m_cpu(ids, am, None, labels=labels, sentence_order_label=sop)
    og = m_gpu(ids.to(cuda), am.to(cuda), None, labels=labels.to(cuda), sentence_order_label=sop.to(cuda))
    assert abs(oc["loss"].item() - og["loss"].item()) < 2e-2
    oc["loss"].backward()
    og["loss"].backward()
    assert rel(m_gpu.flat.grad.cpu(), m_cpu.flat.grad) < 5e-2


@pytest.fixture
def force_mfma():
    """(The default dispatch: gemm8 -> gemm.hip -> gemm_small; kept as a marker of the MFMA tests.)"""
    yield


@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (1000, 512, 256), (4096, 3072, 1024)])
def test_mfma_gemm_nt_nn(cuda, force_mfma, M, N, K):
    torch.manual_seed(5)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16()
    bias = torch.randn(N, device=cuda)
    res = torch.randn(M, N, device=cuda).bfloat16()
    ref = a.float() @ w.float().t() + bias
    y = OPS.gemm(a, w, bias, None, False, True, 0)
    assert rel(y, ref) < 1e-2
    y = OPS.gemm(a, w, bias, res, False, True, 0)
    assert rel(y, ref + res.float()) < 1e-2
    # dgrad form: dy [M, N] @ w [N, K]  (B operand K-outer)
    dy = torch.randn(M, N, device=cuda).bfloat16()
    dx = OPS.gemm(dy, w, None, None, False, False, 0)
    assert rel(dx, dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("T,N,K", [(2048, 256, 256), (8192, 1024, 512)])
def test_mfma_gemm_wgrad_splitk(cuda, force_mfma, T, N, K):
    torch.manual_seed(6)
    dy = torch.randn(T, N, device=cuda).bfloat16()
    x = torch.randn(T, K, device=cuda).bfloat16()
    g = torch.ones(N, K, device=cuda)
    OPS.gemm_acc_f32(dy, x, g, True, False)
    assert rel(g, 1 + dy.float().t() @ x.float()) < 1e-3


def test_mfma_gemm_gelu_epilogues(cuda, force_mfma):
    torch.manual_seed(7)
    M, H, I = 1024, 256, 1024
    x = torch.randn(M, H, device=cuda).bfloat16()
    w1 = (torch.randn(I, H, device=cuda) * 0.1).bfloat16()
    b1 = torch.randn(I, device=cuda)
    f, g = OPS.gemm_gelu(x, w1, b1)
    fr = x.float() @ w1.float().t() + b1
    assert rel(f, fr) < 1e-2
    assert rel(g, F.gelu(fr, approximate="tanh")) < 2e-2
    w2 = (torch.randn(H, I, device=cuda) * 0.1).bfloat16()
    ds = torch.randn(M, H, device=cuda).bfloat16()
    db = torch.zeros(I, device=cuda)
    df = OPS.gemm_dgelu(ds, w2, f, db)
    fr2 = f.float().requires_grad_(True)
    gr = F.gelu(fr2, approximate="tanh")
    dref = torch.autograd.grad(gr, fr2, ds.float() @ w2.float())[0]
    assert rel(df, dref) < 2e-2
    assert rel(db, df.float().sum(0)) < 1e-3


@pytest.mark.parametrize("M,H,I", [(1024, 256, 1024), (4096, 1024, 4096), (1000, 256, 512)])
def test_gemm_gelu_derivative_forms(cuda, M, H, I):
    """gemm_gelu_d stores gelu_new'(h) next to gelu_new(h); gemm_dmul multiplies the data gradient
    by it: the pair equals the pre-activation pair gemm_gelu / gemm_dgelu to bf16 accuracy and the
    fp32 reference (gemm8 EPI 6 / 7 at the 256-multiple shapes, the unfused kernels otherwise)."""
    torch.manual_seed(11)
    x = torch.randn(M, H, device=cuda).bfloat16()
    w1 = (torch.randn(I, H, device=cuda) * 0.1).bfloat16()
    b1 = torch.randn(I, device=cuda)
    d, g = OPS.gemm_gelu_d(x, w1, b1)
    f, g0 = OPS.gemm_gelu(x, w1, b1)
    assert torch.equal(g, g0)
    hr = f.float().requires_grad_(True)
    gr = F.gelu(hr, approximate="tanh")
    dref = torch.autograd.grad(gr.sum(), hr)[0]
    assert rel(d, dref) < 5e-3
    w2 = (torch.randn(H, I, device=cuda) * 0.1).bfloat16()
    ds = torch.randn(M, H, device=cuda).bfloat16()
    db, db0 = torch.zeros(I, device=cuda), torch.zeros(I, device=cuda)
    df = OPS.gemm_dmul(ds, w2, d, db)
    df0 = OPS.gemm_dgelu(ds, w2, f, db0)
    ref = (ds.float() @ w2.float()) * dref
    assert rel(df, ref) < 1e-2 and rel(df, df0) < 1e-2
    assert rel(db, df.float().sum(0)) < 1e-3 and rel(db, db0) < 1e-2
    dbt = torch.zeros(I, device=cuda)
    dft = OPS.gemm_dmul(ds, w2.t().contiguous(), d, dbt, True)
    assert rel(dft, df) < 1e-2 and rel(dbt, db) < 1e-2


def test_gemm_dgelu_transposed_weight(cuda):
    """gemm_dgelu(trans_w=True) against W^T's forward-layout copy equals the plain-weight form."""
    torch.manual_seed(17)
    M, H, I = 2048, 256, 1024
    w2 = (torch.randn(H, I, device=cuda) * 0.1).bfloat16()
    ds = torch.randn(M, H, device=cuda).bfloat16()
    f = torch.randn(M, I, device=cuda).bfloat16()
    db, dbt = torch.zeros(I, device=cuda), torch.zeros(I, device=cuda)
    df = OPS.gemm_dgelu(ds, w2, f, db)
    dft = OPS.gemm_dgelu(ds, w2.t().contiguous(), f, dbt, True)
    fr = f.float().requires_grad_(True)
    dref = torch.autograd.grad(F.gelu(fr, approximate="tanh"), fr, ds.float() @ w2.float())[0]
    assert dft.shape == (M, I)
    assert rel(dft, dref) < 2e-2 and rel(dft, df) < 1e-2
    assert rel(dbt, dft.float().sum(0)) < 1e-3 and rel(dbt, db) < 1e-2


def test_albert_layer_dgrad_transposed_weights(cuda):
    """The ALBERT layer backward on transposed weight copies matches the plain-weight backward."""
    from dedloc_amd.models import albert as A

    cfg = A.AlbertConfig.tiny(hidden_size=256, intermediate_size=1024, num_attention_heads=4, num_hidden_layers=2)
    torch.manual_seed(18)
    model = A.AlbertForPreTraining(cfg)
    model.materialize(cuda)
    ids = torch.randint(5, cfg.vocab_size, (4, 128), device=cuda)
    grads = {}
    for wt in (False, True):
        A._DGRAD_WT = wt
        model.flat.grad.zero_()
        h, _ = model.encode(ids)
        h.float().pow(2).mean().backward()
        grads[wt] = model.flat.grad.clone()
    A._DGRAD_WT = True
    assert torch.isfinite(grads[True]).all()
    assert rel(grads[True], grads[False]) < 2e-2


@pytest.mark.parametrize("groups", [1, 2])
def test_albert_shared_weight_gradient_slabs(cuda, groups):
    """Deferred slab sums of the shared layer's weight gradients (gemm_acc_f32_shared) match one
    slab sum per layer call, over two backward passes (the first call of each pass resets the
    slabs) and with two layer groups (each group's weights have their own first / last call)."""
    from dedloc_amd.models import albert as A

    cfg = A.AlbertConfig.tiny(hidden_size=256, intermediate_size=1024, num_attention_heads=4, num_hidden_layers=4,
                              num_hidden_groups=groups, max_position_embeddings=512)
    torch.manual_seed(19)
    model = A.AlbertForPreTraining(cfg)
    model.materialize(cuda)
    ids = torch.randint(5, cfg.vocab_size, (8, 512), device=cuda)
    grads = {}
    try:
        for shared in (False, True):
            A._SHARED_WGRAD = shared
            model.flat.grad.zero_()
            for _ in range(2):
                h, _ = model.encode(ids)
                h.float().pow(2).mean().backward()
            grads[shared] = model.flat.grad.clone()
    finally:
        A._SHARED_WGRAD = True
    assert torch.isfinite(grads[True]).all()
    assert rel(grads[True], grads[False]) < 1e-3


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 512, 192), (777, 1024, 320), (2048, 256, 4096)])
def test_gemm8_pipeline_depths(cuda, force_mfma, M, N, K):
    """gemm8.hip: K-tile counts 1, 3, 5 and 64 exercise the prologue, the odd-tile buffer parity and
    the counted-vmcnt tail; an M tail exercises the clamped loads / masked stores."""
    torch.manual_seed(8)
    a = (torch.rand(M, K, device=cuda) * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device=cuda) * 2 - 1).bfloat16()
    bias = torch.randn(N, device=cuda)
    y = OPS.gemm(a, w, bias, None, False, True, 0)
    assert rel(y, a.float() @ w.float().t() + bias) < 8e-3
    dy = (torch.rand(M, N, device=cuda) * 2 - 1).bfloat16()
    assert rel(OPS.gemm(dy, w, None, None, False, False, 0), dy.float() @ w.float()) < 8e-3
    if M % 256 == 0:  # wgrad: reduction over the M rows, output [N, K]
        g = torch.full((N, K), 0.5, device=cuda)
        OPS.gemm_acc_f32(dy, a, g, True, False)
        assert rel(g, 0.5 + dy.float().t() @ a.float()) < 1e-5


def test_gemm_register_staged_backend(cuda):
    """The register-staged gemm.hip takes the wide outputs outside gemm8's contract (N % 256 != 0,
    more than 192 columns): N = 384 and 640, with bias and residual, against fp32."""
    torch.manual_seed(9)
    for N in (384, 640):
        a = torch.randn(512, 256, device=cuda).bfloat16()
        w = torch.randn(N, 256, device=cuda).bfloat16()
        b = torch.randn(N, device=cuda)
        r = torch.randn(512, N, device=cuda).bfloat16()
        assert rel(OPS.gemm(a, w, b, r, False, True, 0), a.float() @ w.float().t() + b + r.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(512, 3000, 128), (1000, 128, 3000), (37, 70, 96), (3000, 128, 512),
                                   (65576, 128, 1024), (2048, 30000, 128)])
def test_gemm_small_odd_shapes(cuda, M, N, K):
    """Shapes outside the tiled kernels' contracts (the SwAV prototypes: N = 3000; their gradient
    GEMMs: K = 3000; ALBERT's N = 128 embedding mapping over many tokens and the tied decoder's
    30000-wide gradients, whose long reductions split into fp32 slabs) run on gemm_small.hip:
    forward with bias, dgrad (K-outer B) and the fp32 accumulating weight gradient, against fp32
    references."""
    torch.manual_seed(19)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16()
    b = torch.randn(N, device=cuda)
    assert rel(OPS.gemm(a, w, b, None, False, True, 0), a.float() @ w.float().t() + b) < 1e-2
    dy = torch.randn(M, N, device=cuda).bfloat16()
    assert rel(OPS.gemm(dy, w, None, None, False, False, 0), dy.float() @ w.float()) < 1e-2
    g = torch.full((N, K), 0.25, device=cuda)
    OPS.gemm_acc_f32(dy, a, g, True, False)
    assert rel(g, 0.25 + dy.float().t() @ a.float()) < 1e-3


def test_gemm_small_strided_views(cuda):
    """Operands that are column slices of wider tensors (row stride != width), aligned and not."""
    torch.manual_seed(23)
    for off in (0, 3):
        big_a = torch.randn(300, 200, device=cuda).bfloat16()
        big_w = torch.randn(90, 200, device=cuda).bfloat16()
        a, w = big_a[:, off:off + 136], big_w[:, off:off + 136]
        assert rel(OPS.gemm(a, w, None, None, False, True, 0), a.float() @ w.float().t()) < 1e-2
        g = torch.zeros(90, 136, device=cuda)
        dy = torch.randn(300, 90, device=cuda).bfloat16()
        OPS.gemm_acc_f32(dy, a, g, True, False)
        assert rel(g, dy.float().t() @ a.float()) < 1e-3


@pytest.mark.parametrize("Bn,M,N,K", [(48, 512, 512, 64), (6, 192, 64, 192), (5, 37, 70, 96)])
def test_gemm_small_batched_bmm(cuda, Bn, M, N, K):
    """OPS.bmm (gemm_small's batched launch, gridDim.z = batch) against fp32 torch.bmm: plain,
    transposed-view operands read in place (the composed attention's K^T, P^T, dS^T), bf16 and fp32
    outputs."""
    torch.manual_seed(29)
    a = torch.randn(Bn, M, K, device=cuda).bfloat16()
    b = torch.randn(Bn, K, N, device=cuda).bfloat16()
    ref = torch.bmm(a.float(), b.float())
    out32 = OPS.bmm(a, b, True)
    assert out32.dtype == torch.float32 and rel(out32, ref) < 1e-5
    assert rel(OPS.bmm(a, b, False), ref) < 1e-2
    at = torch.randn(Bn, K, M, device=cuda).bfloat16().transpose(1, 2)
    bt = torch.randn(Bn, N, K, device=cuda).bfloat16().transpose(1, 2)
    assert rel(OPS.bmm(at, bt, True), torch.bmm(at.float(), bt.float())) < 1e-5
    assert rel(OPS.bmm(at, b, False), torch.bmm(at.float(), b.float())) < 1e-2


@pytest.mark.timeout(240)
def test_albert_pretraining_converges_on_gpu(cuda):
    """End to end through the HIP kernels: a small shared-layer ALBERT memorises one fixed MLM+SOP batch
    under fused LAMB + global-norm clipping (the collaborative step's optimizer path); the loss must
    fall well below its start, with finite gradients throughout."""
    from dedloc_amd.data.synthetic_mlm import SyntheticSOPStream
    from dedloc_amd.models import albert as A
    from dedloc_amd.optim.lamb import FusedLamb

    torch.manual_seed(0)
    cfg = A.AlbertConfig.tiny(hidden_size=256, intermediate_size=1024, num_attention_heads=4, num_hidden_layers=4,
                              max_position_embeddings=128, vocab_size=1000)
    model = A.AlbertForPreTraining(cfg)
    model.materialize(cuda)
    model.train()
    opt = FusedLamb(model.flat, lr=2e-2, weight_decay=0.01, clamp_value=1e4, no_decay=model.no_decay_names())
    batch = SyntheticSOPStream(16, 128, cfg.vocab_size, seed=3, device=cuda).next_batch()
    losses = []
    for _ in range(150):  # CPU reference ops, same seeds: 7.65 -> 1.98
        model.flat.grad.zero_()
        out = model(batch["input_ids"], batch["attention_mask"], batch["token_type_ids"],
                    sentence_order_label=batch["sentence_order_label"], mlm_positions=batch["mlm_positions"],
                    mlm_labels=batch["mlm_labels"])
        out["loss"].backward()
        gn = model.flat.grad.norm()
        model.flat.grad.mul_(torch.clamp(1.0 / (gn + 1e-6), max=1.0))  # max_grad_norm = 1.0
        opt.step()
        losses.append(float(out["loss"].detach()))
    assert all(math.isfinite(v) for v in losses)
    assert losses[-1] < 0.5 * losses[0], (losses[0], losses[-1])


def test_scale_by_device_scalar(cuda):
    """scale_by_: in-place bf16 scale by a device scalar (the cross-entropy backward's upstream
    gradient), a no-op when the scalar is exactly 1; odd length exercises the tail."""
    torch.manual_seed(31)
    x = torch.randn(1001, device=cuda).bfloat16()
    ref = x.clone()
    OPS.scale_by_(x, torch.ones(1, device=cuda))
    assert torch.equal(x, ref)
    OPS.scale_by_(x, torch.full((1,), 0.5, device=cuda))
    assert torch.equal(x, (ref.float() * 0.5).bfloat16())


@pytest.mark.parametrize("n", [4096, 1000004])
def test_add_slabs_zero(cuda, n):
    """add_slabs_zero_: out += sum of the [S, n] slab rows (fp32, float4 lanes + tail), then the slabs
    read zero — the concurrent SwAV passes' side gradients folded into the flat gradient."""
    torch.manual_seed(32)
    out = torch.randn(n, device=cuda)
    slabs = torch.randn(3, n, device=cuda)
    ref = out.double() + slabs.double().sum(0)
    OPS.add_slabs_zero_(out, slabs)
    torch.testing.assert_close(out.double(), ref, rtol=1e-6, atol=1e-5)
    assert not slabs.any()
