"""Shape fuzzing of the HIP kernels with hypothesis ("every HIP kernel against a
PyTorch-eager oracle ... use hypothesis shape fuzzing").  Each property draws shapes inside the
contract the op advertises (the binding rejects anything else) and compares against an fp32 PyTorch
reference of the same op.  Derandomized, so a failure reproduces; few examples per property to keep
the GPU tier short."""
import math

import pytest
import torch
import torch.nn.functional as F

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, assume, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu
FUZZ = settings(max_examples=12, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture])


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.fixture(scope="module")
def O():
    import dedloc_amd.ops  # noqa: F401

    return torch.ops.dedloc


@FUZZ
@given(rows=st.integers(1, 3000), D=st.sampled_from([64, 128, 256, 512, 768, 1024, 2048, 4096]), res=st.booleans(),
       seed=st.integers(0, 2**16))
def test_layernorm_fuzz(cuda, O, rows, D, res, seed):
    torch.manual_seed(seed)
    x = (torch.randn(rows, D, device=cuda) * 2).bfloat16()
    r = torch.randn(rows, D, device=cuda).bfloat16() if res else None
    g, b = torch.rand(D, device=cuda) + 0.5, torch.randn(D, device=cuda)
    y, s, mean, rstd = O.layernorm_fwd(x, r, g, b, 1e-12)
    s_ref = (x.float() + (r.float() if res else 0)).requires_grad_(True)
    y_ref = F.layer_norm(s_ref, (D,), g, b, 1e-12)
    assert rel(y, y_ref) < 1e-2
    dy = torch.randn(rows, D, device=cuda).bfloat16()
    dg, db, dsum = torch.zeros(D, device=cuda), torch.zeros(D, device=cuda), torch.zeros(D, device=cuda)
    ds = O.layernorm_bwd(dy, s, g, mean, rstd, dg, db, True, dsum)
    gref = torch.autograd.grad(y_ref, s_ref, dy.float())[0]
    assert rel(ds, gref) < 2e-2
    assert rel(db, dy.float().sum(0)) < 1e-3
    assert rel(dsum, ds.float().sum(0)) < 1e-3


def _attn_ref(qkv, mask, H, S):
    T, ld = qkv.shape
    D = ld // (3 * H)
    B = T // S
    x = qkv.float().reshape(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    bias = torch.where(mask.bool(), 0.0, float("-inf"))[:, None, None, :]
    o = F.scaled_dot_product_attention(x[0], x[1], x[2], attn_mask=bias)
    return o.permute(0, 2, 1, 3).reshape(B * S, H * D)


@FUZZ
@given(B=st.integers(1, 3), H=st.integers(1, 4), S=st.sampled_from([64, 128, 192, 256, 384, 512]),
       data=st.data())
def test_attention_fuzz(cuda, O, B, H, S, data):
    torch.manual_seed(data.draw(st.integers(0, 2**16)))
    D = 64
    lens = data.draw(st.lists(st.integers(1, S), min_size=B, max_size=B))
    qkv = (torch.randn(B * S, 3 * H * D, device=cuda) * 1.5).bfloat16()
    mask = (torch.arange(S, device=cuda)[None, :] < torch.tensor(lens, device=cuda)[:, None]).long()
    mbias = torch.where(mask.bool(), 0.0, -1e30).float()
    kvinfo = torch.cat([mask.sum(1).int(), torch.ones(1, dtype=torch.int32, device=cuda)]).contiguous()
    use_len = data.draw(st.booleans())
    out, lse = O.attn_fwd(qkv, mbias, H, S, 1 / math.sqrt(D), kvinfo if use_len else None)
    qkv_r = qkv.float().requires_grad_(True)
    ref = _attn_ref(qkv_r, mask, H, S)
    assert rel(out, ref) < 1.5e-2
    dout = torch.randn_like(out)
    dqkv = O.attn_bwd(qkv, mbias, out, dout, lse, H, S, 1 / math.sqrt(D), kvinfo if use_len else None)
    g_ref = torch.autograd.grad(ref, qkv_r, dout.float())[0]
    # absolute floor: with a single live key softmax is exactly 1, so dQ and dK are 0 up to
    # rounding noise (~1e-7) on both sides and only dV carries signal
    floor = 1e-4 * g_ref.norm().item()
    for part in range(3):
        sl = slice(part * H * D, (part + 1) * H * D)
        err = (dqkv[:, sl].float() - g_ref[:, sl]).norm().item()
        assert err <= 3e-2 * g_ref[:, sl].norm().item() + floor, (part, err)


@FUZZ
@given(rows=st.integers(1, 600), V=st.integers(2, 40000), seed=st.integers(0, 2**16))
def test_xent_fuzz(cuda, O, rows, V, seed):
    torch.manual_seed(seed)
    x = (torch.randn(rows, V, device=cuda) * 3).bfloat16()
    lab = torch.randint(0, V, (rows,), device=cuda)
    lab[::5] = -100
    if (lab != -100).sum() == 0:
        lab[0] = 0
    loss, dl = O.xent_fwd_bwd(x, lab, False, -100)
    xr = x.float().requires_grad_(True)
    lr = F.cross_entropy(xr, lab, ignore_index=-100)
    assert abs(loss.item() - lr.item()) < 1e-3 * max(1, abs(lr.item()))
    assert rel(dl, torch.autograd.grad(lr, xr)[0]) < 1e-2


@FUZZ
@given(n=st.integers(1, 50000), k=st.integers(1, 20), offset=st.integers(0, 7),
       wire=st.sampled_from([torch.float16, torch.bfloat16, torch.float32]), seed=st.integers(0, 2**16))
def test_averaging_kernels_fuzz(cuda, O, n, k, offset, wire, seed):
    """Butterfly parts have arbitrary LP-chosen sizes and start at arbitrary element offsets of the
    wire buffer: pack / reduce_delta / unpack must be exact for any length and alignment."""
    torch.manual_seed(seed)
    masters = [torch.randn(n, device=cuda) + 2.0 for _ in range(k)]
    ws = torch.rand(k, device=cuda) + 0.25
    parts = torch.empty(k * n + offset, dtype=wire, device=cuda)[offset:].view(k, n)    # misaligned start
    deltas = torch.empty(k * n + offset, dtype=wire, device=cuda)[offset:].view(k, n)
    for i in range(k):
        O.pack(masters[i], parts[i], 1.0)
    if wire != torch.float16:  # bf16 / fp32: round-to-nearest-even, exactly torch's cast
        assert torch.equal(parts.float(), torch.stack(masters).to(wire).float())
    O.reduce_delta(parts, ws, deltas)
    pf = parts.float()
    ref = ((pf * ws[:, None]).sum(0) / ws.sum())[None, :] - pf
    tol = 1e-6 if wire == torch.float32 else (2e-3 if wire == torch.float16 else 1e-2)
    assert (deltas.float() - ref).abs().max().item() <= tol * (ref.abs().max().item() + 1.0)
    dst = torch.zeros(n + offset, device=cuda)[offset:]
    m0 = masters[0].clone()
    dst.copy_(m0)
    O.unpack(deltas[0], dst, None, True)
    torch.testing.assert_close(dst, m0 + deltas[0].float())


@FUZZ
@given(M=st.integers(1, 700), N=st.integers(1, 96).map(lambda v: 8 * v), K=st.integers(1, 96).map(lambda v: 8 * v),
       bias=st.booleans(), res=st.booleans(), seed=st.integers(0, 2**16))
def test_gemm_library_path_fuzz(cuda, O, M, N, K, bias, res, seed):
    """Forward (NT, bias / residual epilogues), data-gradient (NN) and fp32 weight-gradient (TN,
    token-split) GEMMs on the library path for arbitrary M and multiple-of-8 N, K."""
    torch.manual_seed(seed)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16()
    b = torch.randn(N, device=cuda) if bias else None
    r = torch.randn(M, N, device=cuda).bfloat16() if res else None
    ref = x.float() @ w.float().t() + (b if bias else 0) + (r.float() if res else 0)
    assert rel(O.gemm(x, w, b, r, False, True, 0), ref) < 1e-2
    dy = torch.randn(M, N, device=cuda).bfloat16()
    assert rel(O.gemm(dy, w, None, None, False, False, 0), dy.float() @ w.float()) < 1e-2
    c = torch.randn(N, K, device=cuda)
    ref_c = c + dy.float().t() @ x.float()
    O.gemm_acc_f32(dy, x, c, True, False)
    assert rel(c, ref_c) < 1e-4


@FUZZ
@given(n=st.integers(1, 8), C=st.sampled_from([64, 128, 256, 512, 1024, 2048]), H=st.integers(1, 20),
       relu=st.booleans(), res=st.booleans(), groups=st.sampled_from([1, 2]), seed=st.integers(0, 2**16))
def test_batchnorm_fuzz(cuda, O, n, C, H, relu, res, groups, seed):
    assume(n * H * H > 1)  # training-mode BN needs more than one value per channel and group
    torch.manual_seed(seed)
    N = n * groups
    cl = torch.channels_last
    x = (torch.randn(N, C, H, H, device=cuda) * 2 + 0.3).bfloat16().contiguous(memory_format=cl)
    r = torch.randn(N, C, H, H, device=cuda).bfloat16().contiguous(memory_format=cl) if res else None
    g, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, mean, rstd = O.bn_fwd(x, r, g, b, rm, rv, 1e-5, 0.1, relu, groups)
    xr = x.float().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    ys = [F.batch_norm(c, None, None, g, b, training=True, eps=1e-5) for c in xr.chunk(groups)]
    yr = torch.cat(ys) + (rr if res else 0)
    if relu:
        yr = yr.clamp_min(0)
    assert rel(y, yr) < 1e-2
    dy = torch.randn_like(y)
    dx, dres, dgamma, dbeta = O.bn_bwd(dy, y, x, mean, rstd, g, relu, res, beta=b)
    gx = torch.autograd.grad(yr, [xr] + ([rr] if res else []), dy.float())
    # absolute floor: with very few values per channel dx is mostly cancellation
    assert (dx.float() - gx[0]).norm().item() <= 2e-2 * gx[0].norm().item() + 1e-3 * dy.float().norm().item()
    if res:
        assert rel(dres, gx[1]) < 1e-2


@FUZZ
@given(bs=st.integers(1, 128), extra=st.integers(0, 300), K=st.integers(2, 4000), seed=st.integers(0, 2**16))
def test_sinkhorn_and_swav_ce_fuzz(cuda, O, bs, extra, K, seed):
    torch.manual_seed(seed)
    n = bs + extra
    e = F.normalize(torch.randn(n, 128, device=cuda), dim=1)
    p = F.normalize(torch.randn(K, 128, device=cuda), dim=1)
    s = (e @ p.t()).contiguous()
    q = O.sinkhorn(s, bs, 0.03, 3)
    ref = O.sinkhorn(s.cpu(), bs, 0.03, 3)  # the op's fp32 PyTorch CPU implementation
    assert q.shape == (bs, K)
    assert torch.allclose(q.cpu(), ref, atol=1e-6, rtol=2e-3)
    scores = (torch.randn(bs, K, device=cuda) * 0.5)
    ds = torch.zeros(bs, K, device=cuda)
    loss = torch.zeros(1, device=cuda)
    O.swav_ce(scores, q, ds, loss, 0.1, 1.0 / bs)
    sr = scores.cpu().requires_grad_(True)
    lref = -(q.cpu() * torch.log_softmax(sr / 0.1, -1)).sum(1).mean()
    (gref,) = torch.autograd.grad(lref, sr)
    assert abs(loss.item() - lref.item()) < 1e-4 * max(1.0, abs(lref.item()))
    assert torch.allclose(ds.cpu(), gref, atol=1e-6, rtol=1e-3)


@FUZZ
@given(N=st.integers(1, 3), Cin=st.sampled_from([64, 128, 192, 256]), Cout=st.sampled_from([64, 128, 192, 256]),
       H=st.integers(3, 20), geo=st.sampled_from([(1, 1, 0), (1, 2, 0), (3, 1, 1), (3, 2, 1)]),
       seed=st.integers(0, 2**16))
def test_conv_fuzz(cuda, O, N, Cin, Cout, H, geo, seed):
    """NHWC convolution forward / data gradient / fp32 weight gradient (the per-shape routing:
    conv.hip implicit GEMM, the tiled GEMM kernels for wide pointwise convs) at arbitrary spatial
    sizes."""
    k, stride, pad = geo
    cl = torch.channels_last
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, Cin, H, H, generator=g).bfloat16().to(cuda).contiguous(memory_format=cl)
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).bfloat16().to(cuda)
    w = w.contiguous(memory_format=cl)
    P = (H + 2 * pad - k) // stride + 1
    dy = torch.randn(N, Cout, P, P, generator=g).bfloat16().to(cuda).contiguous(memory_format=cl)
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=stride, padding=pad)
    dxr, dwr = torch.autograd.grad(yr, [xr, wr], dy.float())
    y = O.conv2d_fwd(x, w, stride, pad)
    assert y.shape == yr.shape and rel(y, yr) < 1e-2
    dx = O.conv2d_dgrad(dy, w, stride, pad, H, H)
    assert dx.shape == dxr.shape and rel(dx, dxr) < 1e-2
    dw = torch.zeros(Cout, Cin, k, k, device=cuda).contiguous(memory_format=cl)
    O.conv2d_wgrad(dy, x, dw, stride, pad)
    assert rel(dw, dwr) < 1e-3


@FUZZ
@given(rows=st.integers(1, 2000), N=st.integers(1, 512).map(lambda v: 8 * v), seed=st.integers(0, 2**16))
def test_gelu_fuzz(cuda, O, rows, N, seed):
    """GELU forward and GELU backward fused with the bias-gradient column sums."""
    torch.manual_seed(seed)
    h = (torch.randn(rows, N, device=cuda) * 2).bfloat16()
    hr = h.float().requires_grad_(True)
    yr = F.gelu(hr, approximate="tanh")
    assert rel(O.gelu_fwd(h), yr) < 1e-2
    dy = torch.randn(rows, N, device=cuda).bfloat16()
    db = torch.zeros(N, device=cuda)
    dh = O.gelu_bwd(dy, h, db)
    (gref,) = torch.autograd.grad(yr, hr, dy.float())
    assert rel(dh, gref) < 1e-2
    assert rel(db, dh.float().sum(0)) < 1e-3


@FUZZ
@given(sizes=st.lists(st.integers(1, 5000), min_size=1, max_size=8), seed=st.integers(0, 2**16))
def test_lamb_fuzz(cuda, O, sizes, seed):
    """Fused 2-phase multi-tensor LAMB over an arbitrary tensor list (chunked per 1000 elements) vs the
    torch_optimizer.Lamb formula (debias, per-tensor trust ratio, clamp, no-decay tensors)."""
    torch.manual_seed(seed)
    wd = [0.01 if i % 2 == 0 else 0.0 for i in range(len(sizes))]
    n = sum(sizes)
    ct, cs, cl, offs = [], [], [], []
    off = 0
    for i, sz in enumerate(sizes):
        offs.append(off)
        for s0 in range(0, sz, 1000):
            ct.append(i)
            cs.append(off + s0)
            cl.append(min(1000, sz - s0))
        off += sz
    ct = torch.tensor(ct, dtype=torch.int32, device=cuda)
    cs = torch.tensor(cs, dtype=torch.int64, device=cuda)
    cl = torch.tensor(cl, dtype=torch.int32, device=cuda)
    twd = torch.tensor(wd, dtype=torch.float32, device=cuda)
    p = torch.randn(n, device=cuda)
    m, v = torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    norms = torch.zeros(2 * len(sizes), device=cuda)
    lr, b1, b2, eps = 1.76e-3, 0.9, 0.999, 1e-6
    for step in range(1, 3):
        g = torch.randn(n, device=cuda)
        bc = math.sqrt(1 - b2 ** step) / (1 - b1 ** step)
        O.lamb_step(p, g, m, v, ct, cs, cl, twd, norms, b1, b2, eps, lr * bc, 10.0, 1.0)
        for i, (o, sz) in enumerate(zip(offs, sizes)):
            sl = slice(o, o + sz)
            mr[sl] = b1 * mr[sl] + (1 - b1) * g[sl]
            vr[sl] = b2 * vr[sl] + (1 - b2) * g[sl] ** 2
            wn = pr[sl].norm().clamp(0, 10.0)
            u = mr[sl] / (vr[sl].sqrt() + eps) + wd[i] * pr[sl]
            un = u.norm()
            trust = 1.0 if (wn == 0 or un == 0) else (wn / un).item()
            pr[sl] -= lr * bc * trust * u
    assert rel(p, pr) < 1e-5 and rel(m, mr) < 1e-5 and rel(v, vr) < 1e-4


@FUZZ
@given(n=st.integers(1, 300000), max_norm=st.floats(0.1, 10.0), seed=st.integers(0, 2**16))
def test_clip_axpby_fuzz(cuda, O, n, max_norm, seed):
    torch.manual_seed(seed)
    g = torch.randn(n, device=cuda) * 3
    ref = g.clone()
    part = torch.zeros(256, device=cuda)
    out = torch.zeros(2, device=cuda)
    O.grad_norm_clip(g, max_norm, part, out)
    nrm = ref.norm().item()
    assert abs(out[0].item() - nrm) <= 1e-4 * nrm + 1e-6 and out[1].item() == 1.0
    assert rel(g, ref * min(1.0, max_norm / (nrm + 1e-6))) < 1e-5
    y = torch.randn(n, device=cuda)
    y0 = y.clone()
    O.axpby(y, g, 0.25, -1.5)
    assert rel(y, 0.25 * y0 - 1.5 * g) < 1e-6


@settings(max_examples=6, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(hidden=st.sampled_from([128, 256, 768]), layers=st.integers(1, 3), shared=st.booleans(),
       B=st.integers(1, 3), S=st.integers(8, 160), seed=st.integers(0, 2**16), data=st.data())
def test_albert_config_fuzz_gpu_matches_cpu(cuda, O, hidden, layers, shared, B, S, seed, data):
    """Whole ALBERT pre-training step through the HIP kernels vs the same model on the CPU reference ops,
    over hidden sizes (768 = albert-base), layer / group counts, batch, unpadded lengths and padding."""
    from dedloc_amd.models import albert as A

    torch.manual_seed(seed)
    cfg = A.AlbertConfig.tiny(hidden_size=hidden, intermediate_size=4 * hidden, num_attention_heads=hidden // 64,
                              num_hidden_layers=layers, num_hidden_groups=1 if shared else layers,
                              max_position_embeddings=256)
    m_cpu = A.AlbertForPreTraining(cfg)
    m_gpu = A.AlbertForPreTraining(cfg)
    m_gpu.load_hf_state_dict(m_cpu.hf_state_dict())
    m_cpu.materialize("cpu")
    m_gpu.materialize(cuda)
    m_cpu.eval()
    m_gpu.eval()
    lens = data.draw(st.lists(st.integers(2, S), min_size=B, max_size=B))
    ids = torch.randint(5, cfg.vocab_size, (B, S))
    am = (torch.arange(S)[None, :] < torch.tensor(lens)[:, None]).long()
    labels = torch.full((B, S), -100)
    for b, n in enumerate(lens):
        labels[b, 1:n:3] = ids[b, 1:n:3]
    sop = torch.randint(0, 2, (B,))
    oc = m_cpu(ids, am, None, labels=labels, sentence_order_label=sop)
    og = m_gpu(ids.to(cuda), am.to(cuda), None, labels=labels.to(cuda), sentence_order_label=sop.to(cuda))
    assert abs(og["loss"].item() - oc["loss"].item()) < 3e-2 * max(1.0, abs(oc["loss"].item()))
    oc["loss"].backward()
    og["loss"].backward()
    assert rel(m_gpu.flat.grad.cpu(), m_cpu.flat.grad) < 6e-2
