"""SwAV path: loss/Sinkhorn semantics vs the vissl formulas, config overrides, multi-crop, LR schedule,
flat autograd params, and one collaborative SwAV peer step (CPU); HIP kernels vs fp32 references (GPU).

The reference formulas below are transcriptions of the math in
``swav/vissl/vissl/losses/swav_loss.py:177-326`` written directly in torch (vissl is not importable here).
"""
import math

import pytest
import torch

import dedloc_amd.ops  # noqa: F401
from dedloc_amd.models.swav_loss import SwAVLoss
from dedloc_amd.optim.lamb import FusedLarcSGD, LinearWarmupCosineAnnealingLR
from dedloc_amd.utils.config import load_config, parse_cli
from dedloc_amd.utils.flat import FlatParams


def vissl_sinkhorn(scores, eps, iters):
    """Q = exp((s - max)/eps)^T, r = 1/K, c = 1/n, iters x (row scale, col scale), final col normalise."""
    Q = torch.exp((scores - scores.max()) / eps).t().double()
    Q /= Q.sum()
    K, n = Q.shape
    r, c = torch.ones(K, dtype=Q.dtype) / K, torch.ones(n, dtype=Q.dtype) / n
    for _ in range(iters):
        u = Q.sum(1)
        Q *= (r / u).unsqueeze(1)
        Q *= (c / Q.sum(0)).unsqueeze(0)
    return (Q / Q.sum(0, keepdim=True)).t().float()


def vissl_loss(scores, bs, num_crops, crops_for_assign, eps, iters, T, queue_scores=None):
    total = 0
    for i, cid in enumerate(crops_for_assign):
        with torch.no_grad():
            s = scores[bs * cid: bs * (cid + 1)].detach()
            if queue_scores is not None:
                s = torch.cat([s, queue_scores[i]])  # vissl: batch first, queue after, take [:bs]
            q = vissl_sinkhorn(s, eps, iters)[:bs]
        loss = 0
        for v in [v for v in range(num_crops) if v != cid]:
            loss -= torch.mean(torch.sum(q * torch.log_softmax(scores[bs * v: bs * (v + 1)] / T, dim=1), dim=1))
        total += loss / (num_crops - 1)
    return total / len(crops_for_assign)


def test_sinkhorn_cpu_matches_vissl():
    torch.manual_seed(0)
    s = torch.randn(40, 30) * 0.3
    q = torch.ops.dedloc.sinkhorn(s, 8, 0.05, 3)
    ref = vissl_sinkhorn(s, 0.05, 3)[-8:]
    assert torch.allclose(q, ref, atol=1e-5, rtol=1e-4)
    assert torch.allclose(q.sum(1), torch.ones(8), atol=1e-5)


@pytest.mark.parametrize("use_queue", [False, True])
def test_swav_loss_and_grad_vs_vissl(use_queue):
    torch.manual_seed(1)
    bs, nc, K, D, L = 6, 4, 20, 16, 12
    protos = torch.nn.functional.normalize(torch.randn(K, D), dim=1)
    emb = torch.nn.functional.normalize(torch.randn(nc * bs, D), dim=1)
    scores = (emb @ protos.t()).requires_grad_(True)
    crit = SwAVLoss(num_crops=nc, crops_for_assign=(0, 1), temperature=0.1, epsilon=0.05, num_iters=3,
                    num_prototypes=K, embedding_dim=D, queue_length=L if use_queue else 0, queue_start_iter=5,
                    batch_size=bs)
    queue_before = crit.queue.clone() if use_queue else None
    loss = crit(emb, scores, protos, training_iterations=7)
    (g,) = torch.autograd.grad(loss, scores)
    s2 = scores.detach().clone().requires_grad_(True)
    # queue scores: bf16 operands, fp32 accumulation (the precision of every prototype-score GEMM)
    qs = [queue_before[i].bfloat16().float() @ protos.bfloat16().float().t() for i in range(2)] if use_queue else None
    ref = vissl_loss(s2, bs, nc, (0, 1), 0.05, 3, 0.1, qs)
    (gref,) = torch.autograd.grad(ref, s2)
    assert abs(loss.item() - ref.item()) < 1e-4 * max(1.0, abs(ref.item()))
    assert torch.allclose(g, gref, atol=1e-5, rtol=1e-3)
    if use_queue:  # the newest batch embeddings entered the queue
        assert torch.allclose(crit.queue[0, :bs], emb[:bs]) and torch.allclose(crit.queue[1, :bs], emb[bs:2 * bs])


def test_swav_queue_gated_by_global_step():
    crit = SwAVLoss(num_crops=2, crops_for_assign=(0,), num_prototypes=8, embedding_dim=4, queue_length=4,
                    queue_start_iter=10, batch_size=2)
    emb = torch.nn.functional.normalize(torch.randn(4, 4), dim=1)
    protos = torch.nn.functional.normalize(torch.randn(8, 4), dim=1)
    crit(emb, emb @ protos.t(), protos, training_iterations=9)
    assert not crit.use_queue
    crit(emb, emb @ protos.t(), protos, training_iterations=10)
    assert crit.use_queue


def test_hard_assignment_warmup():
    crit = SwAVLoss(num_crops=2, crops_for_assign=(0,), num_prototypes=8, embedding_dim=4, batch_size=3,
                    temp_hard_assignment_iters=1)
    captured = []
    orig = crit._sinkhorn
    crit._sinkhorn = lambda s, bs: captured.append(orig(s, bs)) or captured[-1]
    emb = torch.nn.functional.normalize(torch.randn(6, 4), dim=1)
    protos = torch.nn.functional.normalize(torch.randn(8, 4), dim=1)
    l1 = crit(emb, emb @ protos.t(), protos)
    l2 = crit(emb, emb @ protos.t(), protos)
    assert l1.item() != pytest.approx(l2.item())  # first call used one-hot targets, second soft ones


def test_config_overrides():
    name, ov, rest = parse_cli(["config=pretrain/swav/swav_1node_resnet_submit",
                                "config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=32", "+config.OPTIMIZER.lr=1.2",
                                "+config.OPTIMIZER.dht_initial_peers=['1.2.3.4:5']", "--max_iterations", "3"])
    assert rest == ["--max_iterations", "3"]
    cfg = load_config(name, ov)
    assert cfg.DATA.TRAIN.BATCHSIZE_PER_REPLICA == 32
    assert cfg.OPTIMIZER.lr == 1.2
    assert cfg.OPTIMIZER.dht_initial_peers == ["1.2.3.4:5"]
    assert cfg.LOSS.swav_loss.queue.queue_length == 3840 and cfg.LOSS.swav_loss.epsilon == 0.03
    assert cfg.get_path("OPTIMIZER.larc_config.trust_coefficient") == 0.001


def test_linear_warmup_cosine_matches_reference_closed_form():
    """sgd_collaborative.py:73-84 closed form (warmup_epochs > 1)."""
    w = torch.nn.Parameter(torch.zeros(4))
    flat = FlatParams([("w", w)], with_bf16=False)
    opt = FusedLarcSGD(flat, lr=2.4)
    sch = LinearWarmupCosineAnnealingLR(opt, warmup_epochs=5, max_epochs=20, warmup_start_lr=0.3, eta_min=0.0048)
    for e in range(25):
        if e < 5:
            ref = 0.3 + e * (2.4 - 0.3) / 4
        else:
            ref = 0.0048 + 0.5 * (2.4 - 0.0048) * (1 + math.cos(math.pi * (e - 5) / 15))
        assert opt.param_groups[0]["lr"] == pytest.approx(ref, rel=1e-9)
        sch.step()


def test_flat_autograd_channels_last_grads_accumulate_in_place():
    conv = torch.nn.Conv2d(3, 8, 3, bias=True)
    ref = torch.nn.Conv2d(3, 8, 3, bias=True)
    ref.load_state_dict(conv.state_dict())
    flat = FlatParams(conv.named_parameters(), with_bf16=False, autograd=True, channels_last=True)
    assert conv.weight.is_contiguous(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 9, 9)
    for _ in range(2):
        conv(x).square().sum().backward()
        ref(x).square().sum().backward()
    assert conv.weight.grad.data_ptr() == flat.view(flat.grad, "weight").data_ptr()
    assert torch.allclose(flat.view(flat.grad, "weight"), ref.weight.grad, atol=1e-5)
    assert torch.allclose(flat.view(flat.grad, "bias"), ref.bias.grad, atol=1e-5)
    flat.zero_grad()
    assert conv.weight.grad.abs().sum() == 0


def test_multicrop_shapes_cpu():
    from dedloc_amd.data.multicrop import MultiCropAugment, SyntheticMultiCropStream

    aug = MultiCropAugment(size_crops=(32, 16), num_crops=(2, 3))
    s = SyntheticMultiCropStream(3, "cpu", seed=1, pool_size=4, image_size=48, augment=aug, out_dtype=torch.float32)
    crops = s.next_batch()
    assert [tuple(c.shape) for c in crops] == [(3, 3, 32, 32)] * 2 + [(3, 3, 16, 16)] * 3
    assert all(torch.isfinite(c).all() for c in crops)
    assert crops[0].is_contiguous(memory_format=torch.channels_last)
    again = SyntheticMultiCropStream(3, "cpu", seed=1, pool_size=4, image_size=48, augment=aug,
                                     out_dtype=torch.float32).next_batch()
    assert all(torch.equal(a, b) for a, b in zip(crops, again))  # per-peer seed fixes every draw


def test_multicrop_params_cover_the_reference_transforms():
    """Parameter table statistics match the vissl transform probabilities (flip 0.5, colour 0.8,
    grayscale 0.2, blur 0.5) and RandomResizedCrop's area range."""
    from dedloc_amd.data.multicrop import MultiCropAugment

    aug = MultiCropAugment()
    gen = torch.Generator().manual_seed(0)
    p = aug.sample_params(torch.zeros(20000, dtype=torch.long), (0.05, 0.14), gen)
    assert abs((p[:, 1] < 0).float().mean() - 0.5) < 0.02
    assert abs(p[:, 8].mean() - 0.8) < 0.02 and abs(p[:, 9].mean() - 0.2) < 0.02
    assert abs((p[:, 19] > 0).float().mean() - 0.5) < 0.02
    area = p[:, 1].abs() * p[:, 3]
    assert area.min() >= 0.05 - 1e-4 and area.max() <= 0.14 + 1e-4
    M = p[0, 10:19].view(3, 3)
    assert torch.allclose(M.sum(1), torch.ones(3), atol=1e-4)  # a hue rotation keeps greys grey


@pytest.mark.gpu
def test_multicrop_kernels_match_reference(cuda):
    """augment.hip (sample / colour / blur / normalize) vs the tensor-op reference on the same table."""
    from dedloc_amd.data.multicrop import MultiCropAugment, _smooth_images, augment_reference

    pool = _smooth_images(6, 64, torch.Generator(device=cuda).manual_seed(0), cuda)
    aug = MultiCropAugment()
    gen = torch.Generator().manual_seed(3)
    # 224 / 96: the bench's crop sizes (several row bands per image in the fused colour-blur kernel)
    for size, scale in ((40, (0.14, 1.0)), (16, (0.05, 0.14)), (224, (0.14, 1.0)), (96, (0.05, 0.14))):
        params = aug.sample_params(torch.randint(0, 6, (24,), generator=gen), scale, gen)
        out = torch.ops.dedloc.multicrop(pool, params.to(cuda), size, aug.rad, list(aug.mean), list(aug.std))
        ref = augment_reference(pool.cpu(), params, size, aug.rad, aug.mean, aug.std)
        assert out.dtype == torch.bfloat16 and out.is_contiguous(memory_format=torch.channels_last)
        err = (out.cpu().float() - ref.float()).abs()
        assert err.max() < 0.05 and err.mean() < 2e-3, (err.max(), err.mean())


def _tiny_cfg(extra=()):
    return load_config("swav_1node_resnet_submit", [
        "config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=2", "config.DATA.TRAIN.MULTICROP.size_crops=[32,16]",
        "config.DATA.TRAIN.MULTICROP.num_crops=[2,2]",
        "config.DATA.TRAIN.SYNTHETIC_POOL_SIZE=4", "config.DATA.TRAIN.SYNTHETIC_IMAGE_SIZE=48",
        "config.MODEL.HEAD.num_clusters=16", "config.LOSS.swav_loss.queue.queue_length=4",
        "config.LOSS.swav_loss.queue.start_iter=0", "config.OPTIMIZER.target_batch_size=4",
        "config.OPTIMIZER.batch_size_for_tracking=2",
        "config.MODEL.TEMP_FROZEN_PARAMS_ITER_MAP=[['heads.0.prototypes0.weight', 1]]",
        "config.OPTIMIZER.warmup_epochs=2", "config.OPTIMIZER.max_epochs=10", *extra])


def test_swav_peer_cpu_steps_and_checkpoint(tmp_path):
    from dedloc_amd.dht import DHT
    from dedloc_amd.training.swav_peer import SwavPeer

    cfg = _tiny_cfg([f"config.CHECKPOINT.DIR={tmp_path}"])
    dht = DHT(start=True)
    peer = SwavPeer(cfg, "cpu", dht=dht)
    try:
        w = peer.model.heads[0].prototypes0.weight
        w0 = w.detach().clone()
        peer.train_step()  # iteration 0: prototypes frozen (their grad is zeroed)
        assert torch.allclose(w.norm(dim=1), torch.ones(w.shape[0]), atol=1e-5)
        losses = [float(peer.train_step()) for _ in range(3)]
        assert all(math.isfinite(x) for x in losses)
        trunk_w = peer.model.trunk.conv1.weight
        assert trunk_w.grad.abs().sum() == 0  # zeroed after each collaborative step() call
        path = peer.save_checkpoint()
        sd = torch.load(path, map_location="cpu", weights_only=True)
        assert sd["iteration"] == 4 and "heads.0.prototypes0.weight" in sd["model"]
        snapshot = w.detach().clone()
        with torch.no_grad():
            w.add_(1.0)
        peer.load_checkpoint(str(tmp_path / "checkpoint.torch"))
        assert torch.allclose(w, snapshot)
        assert not torch.allclose(w0, snapshot) or peer.collab_opt.local_step == 0
    finally:
        peer.shutdown()
        dht.shutdown()


def test_swav_peer_eager_stack_cpu_steps(tmp_path):
    """SwavPeer(impl="eager") — stock nn modules, vissl-formula loss, apex LARC in torch ops (the
    measured SwAV baseline of bench.py --impl eager) — runs collaborative iterations, and loads the
    dedloc model's parameters by state-dict key."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.models.resnet_swav import SwAVModel
    from dedloc_amd.training.swav_peer import SwavPeer

    cfg = _tiny_cfg([f"config.CHECKPOINT.DIR={tmp_path}"])
    dht = DHT(start=True)
    peer = SwavPeer(cfg, "cpu", dht=dht, impl="eager")
    try:
        assert not any(type(m).__module__.startswith("dedloc_amd.models") for m in peer.model.modules())
        peer.model.load_state_dict(SwAVModel(num_prototypes=int(cfg.MODEL.HEAD.num_clusters)).state_dict())
        losses = [float(peer.train_step()) for _ in range(2)]
        assert all(math.isfinite(x) for x in losses)
        w = peer.model.heads[0].prototypes0.weight
        assert torch.allclose(w.norm(dim=1), torch.ones(w.shape[0]), atol=1e-5)
    finally:
        peer.shutdown()
        dht.shutdown()


# ----------------------------------------------------------------------------- GPU tier
@pytest.mark.gpu
@pytest.mark.parametrize("n,bs,K", [(64, 64, 3000), (64 + 3840, 64, 3000), (100, 37, 777)])
def test_sinkhorn_gpu_vs_fp32_reference(cuda, n, bs, K):
    torch.manual_seed(0)
    e = torch.nn.functional.normalize(torch.randn(n, 128, device=cuda), dim=1)
    p = torch.nn.functional.normalize(torch.randn(K, 128, device=cuda), dim=1)
    s = (e @ p.t()).contiguous()
    q = torch.ops.dedloc.sinkhorn(s, bs, 0.03, 3)
    ref = vissl_sinkhorn(s.cpu(), 0.03, 3)[-bs:]  # vissl's formula (fp64 Sinkhorn), the op emits the last bs rows
    assert q.shape == (bs, K)
    assert torch.allclose(q.cpu(), ref, atol=1e-6, rtol=2e-3), (q.cpu() - ref).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_swav_ce_gpu_vs_fp32_reference(cuda, dtype):
    torch.manual_seed(0)
    rows, K = 64, 3000
    s = (torch.randn(rows, K, device=cuda) * 0.5).to(dtype)
    q = torch.softmax(torch.randn(rows, K, device=cuda) * 3, -1)
    ds = torch.zeros(rows, K, device=cuda)
    loss = torch.zeros(1, device=cuda)
    torch.ops.dedloc.swav_ce(s, q, ds, loss, 0.1, 1.0 / rows)
    sr = s.float().cpu().requires_grad_(True)
    lref = -(q.cpu() * torch.log_softmax(sr / 0.1, -1)).sum(1).mean()
    (g,) = torch.autograd.grad(lref, sr)
    assert abs(loss.item() - lref.item()) < 1e-4 * abs(lref.item())
    assert torch.allclose(ds.cpu(), g, atol=1e-6, rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_swav_ce_multi_gpu_vs_fp32_reference(cuda, dtype):
    """Every (assignment crop, other crop) pair in one launch, against plain fp32 PyTorch: the loss
    sum_i sum_{v != crop_i} -mean_b <q_i, log_softmax(s_v / T)> / n_pairs and its score gradient."""
    torch.manual_seed(0)
    bs, nc, K, T = 32, 8, 3000, 0.1
    s = (torch.randn(nc * bs, K, device=cuda) * 0.5).to(dtype)
    q = torch.softmax(torch.randn(2, bs, K, device=cuda) * 3, -1)
    ds = torch.full((nc * bs, K), 7.0, device=cuda)  # written, not accumulated
    loss = torch.zeros(1, device=cuda)
    n_pairs = 2 * (nc - 1)
    torch.ops.dedloc.swav_ce_multi(s, q, [0, 1], ds, loss, T, 1.0 / (bs * n_pairs))
    sr = s.float().cpu().requires_grad_(True)
    lref = 0
    for i, cid in enumerate((0, 1)):
        for v in range(nc):
            if v != cid:
                lref = lref - (q[i].cpu() * torch.log_softmax(sr[v * bs:(v + 1) * bs] / T, -1)).sum(1).mean()
    lref = lref / n_pairs
    (g,) = torch.autograd.grad(lref, sr)
    assert abs(loss.item() - lref.item()) < 1e-4 * abs(lref.item())
    assert torch.allclose(ds.cpu(), g, atol=1e-7, rtol=1e-3)


@pytest.mark.gpu
def test_row_normalize_gpu(cuda):
    w = torch.randn(3000, 128, device=cuda)
    ref = torch.nn.functional.normalize(w, dim=1)
    torch.ops.dedloc.row_normalize_(w)
    assert torch.allclose(w, ref, atol=1e-6)


@pytest.mark.gpu
def test_swav_loss_gpu_matches_vissl_formula(cuda):
    """The GPU SwAV loss (Sinkhorn and cross-entropy kernels, queue scores on the GEMM kernels)
    against vissl's formulas in plain fp32 PyTorch (vissl_loss above), loss and score gradient."""
    torch.manual_seed(2)
    bs, nc, K, D, L = 16, 8, 3000, 128, 64
    protos = torch.nn.functional.normalize(torch.randn(K, D), dim=1)
    emb = torch.nn.functional.normalize(torch.randn(nc * bs, D), dim=1)
    scores = emb @ protos.t()
    crit = SwAVLoss(num_crops=nc, crops_for_assign=(0, 1), num_prototypes=K, embedding_dim=D, queue_length=L,
                    queue_start_iter=0, batch_size=bs).to(cuda)
    queue_before = crit.queue.cpu().clone()
    s_gpu = scores.to(cuda).requires_grad_(True)
    loss = crit(emb.to(cuda), s_gpu, protos.to(cuda), 5)
    loss.backward()
    s_ref = scores.clone().requires_grad_(True)
    qs = [queue_before[i].bfloat16().float() @ protos.bfloat16().float().t() for i in range(2)]
    ref = vissl_loss(s_ref, bs, nc, (0, 1), 0.03, 3, 0.1, qs)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * abs(ref.item())
    g, gr = s_gpu.grad.cpu(), s_ref.grad
    assert ((g - gr).norm() / gr.norm()).item() < 1e-3
    assert (g - gr).abs().max().item() < 1e-2 * gr.abs().max().item()


@pytest.mark.gpu
def test_swav_loss_gpu_matches_cpu(cuda):
    torch.manual_seed(2)
    bs, nc, K, D = 16, 8, 3000, 128
    protos = torch.nn.functional.normalize(torch.randn(K, D), dim=1)
    emb = torch.nn.functional.normalize(torch.randn(nc * bs, D), dim=1)
    scores = emb @ protos.t()
    kw = dict(num_crops=nc, crops_for_assign=(0, 1), num_prototypes=K, embedding_dim=D, queue_length=64,
              queue_start_iter=0, batch_size=bs)
    torch.manual_seed(3)
    c_cpu = SwAVLoss(**kw)
    torch.manual_seed(3)
    c_gpu = SwAVLoss(**kw).to(cuda)
    s1 = scores.clone().requires_grad_(True)
    s2 = scores.to(cuda).requires_grad_(True)
    l1 = c_cpu(emb, s1, protos, 5)
    l2 = c_gpu(emb.to(cuda), s2, protos.to(cuda), 5)
    l1.backward()
    l2.backward()
    assert abs(l1.item() - l2.item()) < 1e-3 * abs(l1.item())
    # the GPU queue scores run on the bf16 GEMM kernels (the reference's queue product runs under
    # fp16 autocast), so the Sinkhorn targets carry operand rounding: compare the whole gradient
    g2, g1 = s2.grad.cpu(), s1.grad
    assert ((g2 - g1).norm() / g1.norm()).item() < 1e-2
    assert (g2 - g1).abs().max().item() < 3e-2 * g1.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_swav_peer_gpu_step(cuda, tmp_path, graph):
    """Eager and HIP-graph (MODEL.CUDA_GRAPH: forward and backward graphs replayed after 3 eager
    iterations, weight gradients still written in place into the flat buffer) peer iterations."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.training.swav_peer import SwavPeer

    cfg = load_config("swav_1node_resnet_submit", [
        "config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=8", "config.DATA.TRAIN.SYNTHETIC_POOL_SIZE=16",
        "config.LOSS.swav_loss.queue.start_iter=0", "config.LOSS.swav_loss.queue.queue_length=64",
        "config.OPTIMIZER.target_batch_size=16", "config.OPTIMIZER.batch_size_for_tracking=8",
        f"config.CHECKPOINT.DIR={tmp_path}", f"config.MODEL.CUDA_GRAPH={graph}"])
    dht = DHT(start=True)
    peer = SwavPeer(cfg, cuda, dht=dht)
    try:
        losses = [float(peer.train_step()) for _ in range(5 if graph else 3)]
        if graph:
            assert peer._graphed is not None
        assert all(math.isfinite(x) for x in losses), losses
        w = peer.model.heads[0].prototypes0.weight
        assert torch.allclose(w.norm(dim=1), torch.ones(w.shape[0], device=cuda), atol=1e-4)
    finally:
        peer.shutdown()
        dht.shutdown()


@pytest.mark.gpu
def test_swav_peer_gpu_nan_check_is_async_and_stops(cuda, tmp_path):
    """The GPU peer's NaN-loss check copies the device flag to pinned memory and reads it at the
    next check (no host sync per check): finite iterations never stop, and a non-finite loss dumps
    the state and raises within a few LOG_FREQUENCY periods."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.training.swav_peer import SwavPeer

    cfg = load_config("swav_1node_resnet_submit", [
        "config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=8", "config.DATA.TRAIN.SYNTHETIC_POOL_SIZE=16",
        "config.OPTIMIZER.target_batch_size=100000", "config.OPTIMIZER.batch_size_for_tracking=8",
        f"config.CHECKPOINT.DIR={tmp_path}", "config.MODEL.CUDA_GRAPH=false", "config.LOG_FREQUENCY=2"])
    dht = DHT(start=True)
    peer = SwavPeer(cfg, cuda, dht=dht)
    try:
        for _ in range(6):
            peer.train_step()
        torch.cuda.synchronize()
        assert not list(tmp_path.glob("nan_dump_iteration*.torch"))
        with torch.no_grad():  # a trunk weight: the NaN must survive the fused BN+ReLU and the max pool
            peer.model.trunk.conv1.weight.fill_(float("nan"))
            peer.flat.refresh_bf16()
        with pytest.raises(FloatingPointError):
            for _ in range(12):
                peer.train_step()
                torch.cuda.synchronize()  # the copies land; the next check reads them
        assert len(list(tmp_path.glob("nan_dump_iteration*.torch"))) == 1
    finally:
        peer.shutdown()
        dht.shutdown()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [False, True, "side"])
def test_swav_graph_capture_stream_layouts(cuda, tmp_path, layout):
    """HIP-graph capture of the concurrent trunk passes with the data-gradient weights prepared on the
    main stream (False, the default), on a stream of their own (True) or on the first side pass's
    stream ("side": the round-4 layout whose first
    graphed iteration crashed on the host — it made that stream wait on itself inside the capture,
    which SwAVModel._wait now skips): the graphed iterations replay and match the eager peer."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.training.swav_peer import SwavPeer

    peers, dhts = [], []
    for graph in (False, True):
        cfg = load_config("swav_1node_resnet_submit", [
            "config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=16", "config.DATA.TRAIN.SYNTHETIC_POOL_SIZE=32",
            "config.OPTIMIZER.target_batch_size=64", "config.OPTIMIZER.batch_size_for_tracking=16",
            f"config.CHECKPOINT.DIR={tmp_path}/{graph}", f"config.MODEL.CUDA_GRAPH={graph}",
            "config.MODEL.CUDA_GRAPH_WARMUP=2"])
        dhts.append(DHT(start=True))
        peers.append(SwavPeer(cfg, cuda, dht=dhts[-1]))
        peers[-1].model.dgrad_weights_stream = layout
    try:
        for it in range(4):  # iterations 2 and 3 replay the graphs (no LARC step in between)
            crops = peers[0].data.next_batch()
            la = float(peers[0].train_step([c.clone() for c in crops]))
            lb = float(peers[1].train_step([c.clone() for c in crops]))
            assert math.isfinite(la) and abs(la - lb) <= 2e-2 * abs(la), (it, la, lb)
        assert peers[1]._graphed is not None
    finally:
        for p in peers:
            p.shutdown()
        for d in dhts:
            d.shutdown()


@pytest.mark.gpu
def test_swav_peer_graph_matches_eager(cuda, tmp_path):
    """The graph-replayed iteration computes what the eager one does: two peers from the same
    initialisation, fed the same crops, with the queue active, through collaborative LARC steps
    (every second iteration).  Compared are the iterations up to the first LARC step after the
    capture: later on the two runs drift apart like any two runs do (fp32 statistics atomics sum in
    a different order each run, and random-init ResNets at 8-16 images per BN group amplify that —
    scripts/diag_trunk_paths.py)."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.training.swav_peer import SwavPeer

    peers, dhts = [], []
    for graph in (False, True):
        cfg = load_config("swav_1node_resnet_submit", [
            "config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=16", "config.DATA.TRAIN.SYNTHETIC_POOL_SIZE=32",
            "config.LOSS.swav_loss.queue.start_iter=0", "config.LOSS.swav_loss.queue.queue_length=64",
            "config.OPTIMIZER.target_batch_size=32", "config.OPTIMIZER.batch_size_for_tracking=16",
            f"config.CHECKPOINT.DIR={tmp_path}/{graph}", f"config.MODEL.CUDA_GRAPH={graph}",
            "config.MODEL.CUDA_GRAPH_WARMUP=2"])
        dhts.append(DHT(start=True))
        peers.append(SwavPeer(cfg, cuda, dht=dhts[-1]))
    try:
        for it in range(4):  # iterations 2 and 3 replay the graphs; the LARC step follows iteration 3
            crops = peers[0].data.next_batch()
            la = float(peers[0].train_step([c.clone() for c in crops]))
            lb = float(peers[1].train_step([c.clone() for c in crops]))
            assert math.isfinite(la) and abs(la - lb) <= 2e-2 * abs(la), (it, la, lb)
        assert peers[1]._graphed is not None
        pa, pb = peers[0].flat.fp32, peers[1].flat.fp32
        assert ((pa - pb).norm() / pa.norm()).item() < 2e-2
    finally:
        for p in peers:
            p.shutdown()
        for d in dhts:
            d.shutdown()


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,relu,res", [(8, 64, 28, True, False), (16, 256, 7, True, True), (4, 2048, 3, False, False),
                                            (32, 512, 6, True, True), (2, 128, 56, False, True)])
def test_fused_bn_act_vs_torch(cuda, N, C, H, relu, res):
    torch.manual_seed(9)
    cl = torch.channels_last
    x = (torch.randn(N, C, H, H, device=cuda) * 2 + 0.5).bfloat16().contiguous(memory_format=cl)
    r = torch.randn(N, C, H, H, device=cuda).bfloat16().contiguous(memory_format=cl) if res else None
    g = torch.rand(C, device=cuda) + 0.5
    b = torch.randn(C, device=cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    y, mean, rstd = torch.ops.dedloc.bn_fwd(x, r, g, b, rm, rv, 1e-5, 0.1, relu)
    xr = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    yr = torch.nn.functional.batch_norm(xr, rm_ref, rv_ref, gr, br, training=True, momentum=0.1, eps=1e-5)
    if res:
        yr = yr + rr
    if relu:
        yr = yr.clamp_min(0)
    assert y.is_contiguous(memory_format=cl)
    assert ((y.float() - yr).norm() / yr.norm()).item() < 1e-2
    assert torch.allclose(rm, rm_ref, atol=1e-3, rtol=1e-3) and torch.allclose(rv, rv_ref, atol=1e-3, rtol=1e-3)
    dy = torch.randn_like(y)
    dx, dres, dgamma, dbeta = torch.ops.dedloc.bn_bwd(dy, y, x, mean, rstd, g, relu, res)
    grads = torch.autograd.grad(yr, [xr, gr, br] + ([rr] if res else []), dy.float())

    def rel(a, b_):
        return ((a.float() - b_).norm() / (b_.norm() + 1e-12)).item()

    assert rel(dx, grads[0]) < 2e-2, rel(dx, grads[0])
    assert rel(dgamma, grads[1]) < 1e-2 and rel(dbeta, grads[2]) < 1e-2
    if res:
        assert rel(dres, grads[3]) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,G", [(8, 64, 28, 1), (16, 256, 7, 1), (12, 128, 12, 3), (4, 2048, 3, 2)])
def test_bn_bwd_relu_mask_from_x_equals_mask_from_y(cuda, N, C, H, G):
    """BatchNorm+ReLU without a residual: the backward's ReLU mask recomputed from x (beta given, y
    never read) gives the same gradients as the mask read from y, statistics groups included."""
    torch.manual_seed(13)
    cl = torch.channels_last
    x = (torch.randn(N, C, H, H, device=cuda) * 2 + 0.3).bfloat16().contiguous(memory_format=cl)
    g, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, mean, rstd = torch.ops.dedloc.bn_fwd(x, None, g, b, rm, rv, 1e-5, 0.1, True, G)
    dy = torch.randn_like(y)
    ref = torch.ops.dedloc.bn_bwd(dy, y, x, mean, rstd, g, True, False)
    garbage = torch.full_like(y, float("nan"))  # proves y is not read on the x-mask path
    out = torch.ops.dedloc.bn_bwd(dy, garbage, x, mean, rstd, g, True, False, beta=b)
    # not bitwise: both calls sum the statistics with fp32 atomics in run-dependent order, which can
    # flip the bf16 rounding of a few dx elements (measured up to 4e-5 relative)
    for a, r in ((out[0], ref[0]), (out[2], ref[2]), (out[3], ref[3])):
        assert torch.isfinite(a.float()).all()
        assert ((a.float() - r.float()).norm() / (r.float().norm() + 1e-12)).item() < 5e-4


@pytest.mark.gpu
def test_bnact_module_fused_matches_stock(cuda):
    from dedloc_amd.models.resnet_swav import BNAct

    torch.manual_seed(10)
    m1 = BNAct(256, relu=True).to(cuda)
    m2 = torch.nn.BatchNorm2d(256).to(cuda)  # stock module, fp32, + residual + ReLU in torch ops
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(16, 256, 14, 14, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    y1 = m1(x, r)
    y2 = (m2(x.float()) + r.float()).clamp_min(0)
    assert ((y1.float() - y2.float()).norm() / y2.float().norm()).item() < 2e-2
    assert torch.allclose(m1.running_mean, m2.running_mean, atol=1e-3)
    assert int(m1.num_batches_tracked) == int(m2.num_batches_tracked) == 1


@pytest.mark.gpu
def test_fused_bn_stat_groups_match_per_chunk(cuda):
    torch.manual_seed(11)
    cl = torch.channels_last
    G, n, C, H = 3, 4, 128, 12
    x = (torch.randn(G * n, C, H, H, device=cuda) + torch.arange(G * n, device=cuda).view(-1, 1, 1, 1) * 0.1)
    x = x.bfloat16().contiguous(memory_format=cl)
    g, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, mean, rstd = torch.ops.dedloc.bn_fwd(x, None, g, b, rm, rv, 1e-5, 0.1, True, G)
    rm_ref, rv_ref = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    xr = x.float().requires_grad_(True)
    ys = [torch.nn.functional.batch_norm(c, rm_ref, rv_ref, g, b, training=True, momentum=0.1).clamp_min(0)
          for c in xr.chunk(G)]
    yr = torch.cat(ys)
    assert ((y.float() - yr).norm() / yr.norm()).item() < 1e-2
    assert torch.allclose(rm, rm_ref, atol=1e-3) and torch.allclose(rv, rv_ref, atol=1e-3, rtol=1e-3)
    dy = torch.randn_like(y)
    dx, _, dgamma, dbeta = torch.ops.dedloc.bn_bwd(dy, y, x, mean, rstd, g, True, False)
    (gx,) = torch.autograd.grad(yr, xr, dy.float())
    assert ((dx.float() - gx).norm() / gx.norm()).item() < 2e-2


def test_swav_single_pass_semantics_batched_equals_per_crop_cpu():
    """Batched equal-resolution trunk passes with per-crop BN statistics == one trunk pass per crop
    (fp32 on CPU: bit-identical)."""
    import copy

    from dedloc_amd.models.resnet_swav import SwAVModel

    torch.manual_seed(12)
    m1 = SwAVModel(num_prototypes=16, single_pass_every_crop=True).train()
    m2 = copy.deepcopy(m1)
    cl = torch.channels_last
    crops = [torch.randn(2, 3, 32, 32).contiguous(memory_format=cl) for _ in range(2)]
    crops += [torch.randn(2, 3, 16, 16).contiguous(memory_format=cl) for _ in range(2)]
    e1, s1 = m1(crops)
    e2, s2 = m2.heads[0](torch.cat([m2.trunk(c) for c in crops]))
    assert torch.allclose(s1, s2, atol=1e-5)
    assert torch.allclose(m1.trunk.layer3[0].bn2.running_var, m2.trunk.layer3[0].bn2.running_var, atol=1e-6)
    assert int(m1.trunk.bn1.num_batches_tracked) == int(m2.trunk.bn1.num_batches_tracked) == 4


@pytest.mark.gpu
def test_swav_single_pass_semantics_fused_gpu(cuda):
    """Same on the GPU fused-BN path, compared after the stem + layer1 (deeper, the bf16 rounding of
    different conv batch sizes is amplified by the random-init network; bn_debug.py shows the
    per-layer drift growing smoothly, no layer jumps)."""
    import copy

    from dedloc_amd.models.resnet_swav import SwAVModel

    torch.manual_seed(12)
    # hand-written convs: per-pixel results do not depend on the batch size, so the comparison isolates
    # the BN statistics groups (MIOpen may pick a different algorithm for the 3x larger batch)
    m1 = SwAVModel(num_prototypes=64, single_pass_every_crop=True, conv_impl="hip").to(cuda).train()
    m2 = copy.deepcopy(m1)
    cl = torch.channels_last
    crops = [torch.randn(4, 3, 64, 64, device=cuda).bfloat16().contiguous(memory_format=cl) for _ in range(3)]

    def stem_layer1(m, x):
        t = m.trunk
        return t.layer1(t.maxpool(t.bn1(t.conv1(x))))

    with torch.autocast("cuda", dtype=torch.bfloat16):
        m1.set_bn_stat_groups(3)
        o1 = stem_layer1(m1, torch.cat(crops))
        m1.set_bn_stat_groups(1)
        o2 = torch.cat([stem_layer1(m2, c) for c in crops])
    assert ((o1.float() - o2.float()).norm() / o2.float().norm()).item() < 1e-2
    bn1, bn2 = m1.trunk.layer1[0].bn1, m2.trunk.layer1[0].bn1
    assert torch.allclose(bn1.running_mean, bn2.running_mean, atol=2e-3)
    assert int(bn1.num_batches_tracked) == int(bn2.num_batches_tracked) == 3


def test_swav_nan_loss_dumps_state_and_stops(tmp_path):
    """CheckNanLossHook semantics: a non-finite loss is caught at the next global-step report, the
    peer state is dumped to the checkpoint dir and the peer stops; phase timers land in the metrics."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.training.swav_peer import SwavPeer

    cfg = _tiny_cfg([f"config.CHECKPOINT.DIR={tmp_path}", "config.LOG_FREQUENCY=2"])
    dht = DHT(start=True)
    peer = SwavPeer(cfg, "cpu", dht=dht)
    try:
        for _ in range(4):
            peer.train_step()
        rec = peer.metrics_log[-1]
        assert rec["fwd_ms"] > 0 and rec["loss_bwd_ms"] > 0 and rec["data_n"] >= 1
        with torch.no_grad():
            peer.model.trunk.conv1.weight.fill_(float("nan"))
        with pytest.raises(FloatingPointError):
            for _ in range(4):
                peer.train_step()
        dumps = list(tmp_path.glob("nan_dump_iteration*.torch"))
        assert len(dumps) == 1
        sd = torch.load(dumps[0], map_location="cpu", weights_only=True)
        assert not math.isfinite(sd["loss_sum"]) and "model" in sd
    finally:
        peer.shutdown()
        dht.shutdown()


@pytest.mark.gpu
def test_trunk_bn_pass_workspace_and_inplace_grads(cuda, monkeypatch):
    """Per-pass zeroed BN statistics workspace, batched num_batches_tracked, in-place dgamma/dbeta
    accumulation and the forward-scoped bf16 conv weight cache give the same gradients, running
    statistics and counters as the per-call path (two trunk passes with 2 and 6 stat groups).
    The conv-epilogue statistics (which need the workspace) are off here: they sum in another fp32
    order, and through 16 random-init blocks with 8-row BN groups that alone decorrelates the
    gradients (test_swav_kernels_gpu.py covers them per block)."""
    from dedloc_amd.models import resnet_swav as rs
    from dedloc_amd.models.resnet_swav import BNAct, ResNet50Trunk
    from dedloc_amd.utils.flat import FlatParams

    monkeypatch.setattr(rs.ConvNHWC, "epilogue_stats", False)

    torch.manual_seed(0)
    out = {}
    for fast in (False, "again", True):
        torch.manual_seed(0)
        trunk = ResNet50Trunk().to(cuda).to(memory_format=torch.channels_last)
        flat = FlatParams(trunk.named_parameters(), device=cuda, with_bf16=False, autograd=True)
        ResNet50Trunk.pass_workspace = fast is True
        BNAct.inplace_grad = fast is True
        try:
            g = torch.Generator(device="cpu").manual_seed(1)
            for G, res in ((2, 64), (6, 32)):
                for m in trunk.modules():
                    if isinstance(m, BNAct):
                        m.stat_groups = G
                x = torch.randn(2 * G, 3, res, res, generator=g).to(cuda).bfloat16().contiguous(
                    memory_format=torch.channels_last)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    y = trunk(x)
                y.float().pow(2).mean().backward()
        finally:
            ResNet50Trunk.pass_workspace = True
            BNAct.inplace_grad = True
        out[fast] = (flat.grad.clone(), torch.cat([b.float().flatten() for n, b in trunk.named_buffers()]))
    g0, b0 = out[False]
    ga, ba = out["again"]  # the per-call path re-run: run-to-run spread (fp32 atomics in the BN
    g1, b1 = out[True]     # statistics, amplified through 50 bf16 layers into the deep running stats)

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()

    assert torch.isfinite(g1).all()
    assert rel(g1, g0) < 1e-3
    assert rel(b1, b0) < max(3 * rel(ba, b0), 1e-4), (rel(b1, b0), rel(ba, b0))
    n_tracked = [b for n, b in ResNet50Trunk().named_buffers() if n.endswith("num_batches_tracked")]
    assert len(n_tracked) == 53 and b1[-1].item() == 8.0  # 2 + 6 statistics groups counted


@pytest.mark.gpu
@pytest.mark.parametrize("splits", [(1, 1), (2, 1), (2, 2)])
def test_concurrent_trunk_passes_match_sequential(cuda, splits):
    """SwAVModel.concurrent_passes (the crop groups' trunk passes on several streams — one per
    resolution, or with pass_splits a resolution cut into passes of whole crops — each side pass's
    parameter gradients in a buffer of its own added by after_backward, its running-statistics
    updates merged after the join in crop order) gives the sequential path's gradients, running
    statistics and counters.  The sequential path run twice gives the run-to-run spread (fp32
    atomics in the BN statistics) the comparison allows for."""
    from dedloc_amd.models.resnet_swav import SwAVModel
    from dedloc_amd.utils.flat import FlatParams

    CLF = torch.channels_last

    def run(concurrent):
        torch.manual_seed(0)
        model = SwAVModel(num_prototypes=100).to(cuda).to(memory_format=CLF).train()
        flat = FlatParams(model.named_parameters(), device=cuda, with_bf16=True, autograd=True, channels_last=True)
        model.bind_flat(flat)
        model.concurrent_passes = concurrent
        model.pass_splits = splits
        g = torch.Generator(device="cpu").manual_seed(1)
        for _ in range(2):  # two iterations: the stand-ins / second-pass gradients are re-zeroed
            crops = [torch.randn(8, 3, 64, 64, generator=g).to(cuda).bfloat16().contiguous(memory_format=CLF)
                     for _ in range(2)]
            crops += [torch.randn(8, 3, 32, 32, generator=g).to(cuda).bfloat16().contiguous(memory_format=CLF)
                      for _ in range(4)]
            with torch.autocast("cuda", dtype=torch.bfloat16):
                emb, scores = model(crops)
            (scores.float().pow(2).mean() + emb.float().pow(2).mean()).backward()
            model.after_backward()
        torch.cuda.synchronize()
        conc = getattr(model, "_conc", None)
        ran = 0 if conc is None else len(conc["passes"]) + 1
        bufs = torch.cat([b.float().flatten() for _, b in model.named_buffers()])
        return flat.grad.clone(), bufs, ran

    g0, b0, r0 = run(False)
    ga, ba, _ = run(False)
    g1, b1, r1 = run(True)
    assert r0 == 0 and r1 == 2 + (splits[0] - 1) + (splits[1] - 1)

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()

    assert torch.isfinite(g1).all()
    assert rel(g1, g0) < max(3 * rel(ga, g0), 2e-3), (rel(g1, g0), rel(ga, g0))
    assert rel(b1, b0) < max(3 * rel(ba, b0), 1e-4), (rel(b1, b0), rel(ba, b0))


def test_join_batch_views_adjacent_crops_and_copies_otherwise():
    """join_batch: the multi-crop pipeline's split outputs (back to back in one channels-last buffer)
    join without a copy; anything else falls back to torch.cat with the same values."""
    from dedloc_amd.models.resnet_swav import join_batch

    base = torch.randn(12, 3, 8, 8).contiguous(memory_format=torch.channels_last)
    parts = base.split(4)
    j = join_batch(parts)
    assert j.data_ptr() == base.data_ptr() and torch.equal(j, base)
    assert j.is_contiguous(memory_format=torch.channels_last)
    assert join_batch(parts[1:]).data_ptr() == parts[1].data_ptr()
    shuffled = [parts[2], parts[0]]
    k = join_batch(shuffled)
    assert k.data_ptr() != parts[2].data_ptr() and torch.equal(k, torch.cat(shuffled))
    sep = [torch.randn(4, 3, 8, 8), torch.randn(4, 3, 8, 8)]
    assert torch.equal(join_batch(sep), torch.cat(sep))
    assert join_batch(parts[:1]) is parts[0]


def test_add_slabs_zero_cpu():
    """add_slabs_zero_ (the side-pass gradient fold): CPU implementation."""
    out = torch.randn(64)
    slabs = torch.randn(3, 64)
    ref = out + slabs.sum(0)
    torch.ops.dedloc.add_slabs_zero_(out, slabs)
    assert torch.allclose(out, ref) and not slabs.any()


def test_pass_plan_cuts_groups_into_whole_crops():
    """SwAVModel._pass_plan: a resolution group with one statistics group per crop is cut into
    pass_splits[i] passes of whole crops (views, crop order kept); a group whose statistics span
    the whole group, or whose crop count the split does not divide, stays one pass."""
    from dedloc_amd.models.resnet_swav import SwAVModel

    m = SwAVModel.__new__(SwAVModel)
    m.pass_splits = (2, 1)
    a, b = torch.randn(4, 3, 8, 8), torch.randn(12, 3, 4, 4)
    plan = m._pass_plan([(a, 2), (b, 6)])
    assert [(x.shape[0], g) for x, g in plan] == [(2, 1), (2, 1), (12, 6)]
    assert plan[0][0].data_ptr() == a.data_ptr() and plan[1][0].data_ptr() == a[2:].data_ptr()
    m.pass_splits = (2, 2)
    assert [(x.shape[0], g) for x, g in m._pass_plan([(a, 2), (b, 6)])] == [(2, 1), (2, 1), (6, 3), (6, 3)]
    m.pass_splits = (4, 4)  # 4 does not divide 2 crops / 6 crops
    assert [(x.shape[0], g) for x, g in m._pass_plan([(a, 2), (b, 6)])] == [(4, 2), (12, 6)]
    m.pass_splits = (2, 2)  # statistics over the whole group (g = 1): never cut
    assert [(x.shape[0], g) for x, g in m._pass_plan([(a, 1), (b, 1)])] == [(4, 1), (12, 1)]
