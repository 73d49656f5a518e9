"""SwAV model-level parity and training dynamics against stock PyTorch.

* The full SwAVModel (ResNet-50 trunk + projection MLP + prototypes) with the SwAV loss at b = 8,
  crops 2 x 224 + 6 x 96, one backward: loss and every parameter gradient against the same
  parameters in stock fp32 PyTorch modules (``training/swav_eager.eager_twin``: nn.Conv2d,
  nn.BatchNorm2d, ...) with vissl's loss formulas (``EagerSwAVLoss``).  Random-init ResNets with
  8-sample BatchNorm groups amplify any rounding through their 16 blocks, so gradients are bounded
  relative to what stock bf16 autocast of the same modules gets (the same idea as the Bottleneck
  tests in test_conv.py).
* 100 collaborative LARC-SGD steps of the dedloc SwavPeer and of the eager stack (``impl="eager"``:
  stock modules, vissl loss, apex LARC in torch ops) from the same weights on the same crops: the
  loss curves agree within a stated band.

Reference: ``swav/vissl/vissl/losses/swav_loss.py:177-326``,
``vissl/trainer/train_steps/standard_train_step.py:87-229``, ``vissl/models/trunks/resnext.py:48-172``.
"""
import pytest
import torch

from conftest import record_margin

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _crops(device, bs, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    out = []
    for size, n in ((224, 2), (96, 6)):
        for _ in range(n):
            out.append(torch.randn(bs, 3, size, size, generator=g).to(device).bfloat16()
                       .contiguous(memory_format=CL))
    return out


@pytest.mark.timeout(300)
def test_full_swav_model_and_loss_match_fp32_twin(cuda):
    from dedloc_amd.models.resnet_swav import SwAVModel
    from dedloc_amd.models.swav_loss import SwAVLoss
    from dedloc_amd.training.swav_eager import EagerSwAVLoss, eager_twin
    from dedloc_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    bs, nc = 8, 8
    model = SwAVModel(num_prototypes=3000)
    model.normalize_prototypes()
    ref = eager_twin(model, device=cuda).train()
    stock = eager_twin(model, device=cuda).train()
    model.to(cuda).train()
    flat = FlatParams(model.named_parameters(), device=cuda, with_bf16=True, autograd=True, channels_last=True)
    model.bind_flat(flat)
    model.concurrent_passes = True
    crops = _crops(cuda, bs, seed=1)
    loss_kw = dict(num_crops=nc, crops_for_assign=(0, 1), temperature=0.1, epsilon=0.03, num_iters=3,
                   num_prototypes=3000, embedding_dim=128, queue_length=0, batch_size=bs)

    with torch.autocast("cuda", dtype=torch.bfloat16):
        emb, scores = model(crops)
    loss = SwAVLoss(**loss_kw).to(cuda)(emb.float(), scores, model.heads[0].prototypes0.weight, 0)
    loss.backward()
    model.after_backward()

    emb_r, scores_r = ref([c.float() for c in crops])
    loss_r = EagerSwAVLoss(**loss_kw).to(cuda)(emb_r, scores_r, ref.heads[0].prototypes0.weight, 0)
    loss_r.backward()

    with torch.autocast("cuda", dtype=torch.bfloat16):
        emb_s, scores_s = stock(crops)
    loss_s = EagerSwAVLoss(**loss_kw).to(cuda)(emb_s.float(), scores_s, stock.heads[0].prototypes0.weight, 0)
    loss_s.backward()

    assert torch.isfinite(loss) and abs(loss.item() - loss_r.item()) < 1e-2 * abs(loss_r.item()), \
        (loss.item(), loss_r.item(), loss_s.item())
    rp, sp = dict(ref.named_parameters()), dict(stock.named_parameters())
    ours_all, ref_all, stock_all = [], [], []
    worst = []
    for n in flat.names:
        g = flat.view(flat.grad, n).float()
        gr, gs = rp[n].grad.float(), sp[n].grad.float()
        ours_all.append(g.reshape(-1))
        ref_all.append(gr.reshape(-1))
        stock_all.append(gs.reshape(-1))
        worst.append((n, _rel(g, gr), _rel(gs, gr)))
    ours_err = _rel(torch.cat(ours_all), torch.cat(ref_all))
    stock_err = _rel(torch.cat(stock_all), torch.cat(ref_all))
    print(f"loss ours {loss.item():.5f} fp32 {loss_r.item():.5f} bf16-stock {loss_s.item():.5f}; flat gradient "
          f"rel err ours {ours_err:.4f} stock bf16 {stock_err:.4f}")
    head = [(n, o, s) for n, o, s in worst if n.startswith("heads.")]
    record_margin("swav_model_and_loss_vs_fp32_twin", loss_ours=loss.item(), loss_fp32=loss_r.item(),
                  loss_stock_bf16=loss_s.item(), loss_rel_delta=abs(loss.item() - loss_r.item()) / abs(loss_r.item()),
                  loss_bound=1e-2, grad_rel_err_ours=ours_err, grad_rel_err_stock_bf16=stock_err,
                  grad_bound=1.3 * stock_err + 5e-3,
                  head_worst=max(((o, n) for n, o, _ in head), default=(0.0, None)),
                  head_worst_ratio_to_stock=max((o / max(s, 1e-12) for _, o, s in head), default=0.0))
    assert ours_err < 1.3 * stock_err + 5e-3, (ours_err, stock_err)
    # the head (after the trunk's drift has been summed into 2048 features) tightly
    for n, o, s in worst:
        if n.startswith("heads."):
            assert o < 1.3 * s + 1e-2, (n, o, s)


@pytest.mark.timeout(600)
def test_swav_training_curve_matches_eager_stack(cuda, tmp_path):
    """100 collaborative steps (lone peer, target = one local batch: every iteration is a global LARC
    step) of the dedloc peer and the eager stack from the same weights on the same crops."""
    from dedloc_amd.data.multicrop import MultiCropAugment, SyntheticMultiCropStream
    from dedloc_amd.dht import DHT
    from dedloc_amd.training.swav_peer import SwavPeer
    from dedloc_amd.utils.config import load_config

    bs, steps = 16, 100
    ov = [f"config.DATA.TRAIN.BATCHSIZE_PER_REPLICA={bs}", f"config.OPTIMIZER.batch_size_for_tracking={bs}",
          f"config.OPTIMIZER.target_batch_size={bs}", "config.DATA.TRAIN.PREFETCH=false",
          "config.OPTIMIZER.warmup_epochs=10", "config.OPTIMIZER.max_epochs=200", "config.OPTIMIZER.lr=4.8",
          "config.OPTIMIZER.warmup_start_lr=0.3", f"config.CHECKPOINT.DIR={tmp_path}",
          "config.CHECKPOINT.AUTO_RESUME=false", "config.CHECKPOINT.CHECKPOINT_ITER_FREQUENCY=0",
          "config.MODEL.TEMP_FROZEN_PARAMS_ITER_MAP=[]"]
    cfg = load_config("swav_1node_resnet_submit", ov)
    peers, dhts = [], []
    try:
        for impl in ("dedloc", "eager"):
            d = DHT(start=True)
            dhts.append(d)
            peers.append(SwavPeer(cfg, cuda, dht=d, impl=impl))
        ours, eager = peers
        with torch.no_grad():  # same initial weights (identical state-dict keys)
            eager.model.load_state_dict(ours.model.state_dict())
        mc = cfg.DATA.TRAIN.MULTICROP
        aug = MultiCropAugment(size_crops=mc.size_crops, num_crops=mc.num_crops,
                               crop_scales=[tuple(s) for s in mc.crop_scales])
        data = SyntheticMultiCropStream(bs, cuda, seed=7, pool_size=64, image_size=256, augment=aug,
                                        out_dtype=torch.bfloat16)
        curves = ([], [])
        for _ in range(steps):
            crops = data.next_batch()
            for k, p in enumerate(peers):
                curves[k].append(float(p.train_step([c.clone() for c in crops])))
        assert ours.collab_opt.local_step == steps and eager.collab_opt.local_step == steps
        a, b = torch.tensor(curves[0]), torch.tensor(curves[1])
        first, last = a[:10].mean().item(), a[-20:].mean().item()
        print(f"SwAV loss, first 10 / last 20 steps: dedloc {first:.4f} / {last:.4f}, eager "
              f"{b[:10].mean().item():.4f} / {b[-20:].mean().item():.4f}; max |diff| {((a - b).abs().max()):.4f}")
        assert torch.isfinite(a).all() and torch.isfinite(b).all()
        # the band: 20-step running means within 2% of each other over the whole run
        ra = a.unfold(0, 20, 1).mean(1)
        rb = b.unfold(0, 20, 1).mean(1)
        record_margin("swav_training_curve_vs_eager_stack", steps=steps, first10_ours=first, last20_ours=last,
                      first10_eager=b[:10].mean().item(), last20_eager=b[-20:].mean().item(),
                      max_abs_step_diff=(a - b).abs().max().item(),
                      running_mean_max_rel_diff=((ra - rb).abs() / rb.abs()).max().item(), band=0.02)
        assert last < first - 0.05, (first, last)  # it trains
        assert ((ra - rb).abs() / rb.abs()).max().item() < 0.02, ((ra - rb).abs() / rb.abs()).max().item()
    finally:
        for p in peers:
            p.collab_opt.shutdown()
        for d in dhts:
            d.shutdown()
