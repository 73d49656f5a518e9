"""Collaborative SwAV peer: vissl's SelfSupervisionTrainer + standard_train_step + swav hooks, with the
``sgd_collaborative`` optimizer, flattened into one explicit loop.

Per local iteration (reference ``vissl/trainer/train_steps/standard_train_step.py:87-229``):

    crops (8 x [b, 3, S, S], generated on the GPU)         V11  data/multicrop.py
    -> embeddings, scores = model(crops)  (bf16 autocast)    V7/V8  models/resnet_swav.py
    -> SwAV loss with the GLOBAL collaborative step          V9/D18 models/swav_loss.py
    -> backward (grads land in the flat fp32 buffer)
    -> freeze prototypes for the first N local iterations    V10 FreezeParametersHook
    -> CollaborativeOptimizer.step(batch)                    D17 (LARC-SGD, target 32768, FLOAT16 wire)
    -> L2-normalise prototypes                              V10 NormalizePrototypesHook

Deliberate differences: bf16 autocast instead of apex O1 fp16 + loss scaling (V15); activation
checkpointing off by default (P11); optimizer state is shared through the DHT state server and saved
in local checkpoints (the reference's ``get_classy_state`` returns None, D17).

``impl="eager"`` swaps the model, loss and optimizer for the stock-PyTorch stack of
``training/swav_eager.py`` (the measured SwAV baseline); data, hooks and the collaborative engine
stay the same.
"""
from __future__ import annotations

import json
import logging
import math
import time
from pathlib import Path
from typing import Optional

import torch

from ..data.multicrop import MultiCropAugment, StreamPrefetcher, SyntheticMultiCropStream
from ..dht import DHT, get_dht_time
from ..metrics import LocalMetrics, make_validators
from ..models.resnet_swav import SwAVModel, join_batch
from ..models.swav_loss import SwAVLoss
from ..optim.collaborative import CollaborativeOptimizer
from ..optim.lamb import FusedLarcSGD, LinearWarmupCosineAnnealingLR
from ..utils.flat import FlatParams
from ..utils.perf import PerfStats

logger = logging.getLogger(__name__)


def _no_decay_names(model, regularize_bn: bool, regularize_bias: bool):
    """vissl optimizer_helper.py:25-43: split BN / bias params out of weight decay when not regularized."""
    out = set()
    bn_types = (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)
    for mname, m in model.named_modules():
        for pname, _ in m.named_parameters(recurse=False):
            full = f"{mname}.{pname}" if mname else pname
            if isinstance(m, bn_types) and not regularize_bn:
                out.add(full)
            elif pname == "bias" and not regularize_bias:
                out.add(full)
    return out


def _port_endpoint(port) -> str:
    return "0.0.0.0:*" if str(port) in ("any", "*", "0", "None") else f"0.0.0.0:{port}"


class SwavPeer:
    def __init__(self, cfg, device, dht: Optional[DHT] = None, rank: int = 0, impl: str = "dedloc"):
        if impl not in ("dedloc", "eager"):
            raise ValueError(f"impl must be 'dedloc' or 'eager', got {impl!r}")
        self.cfg, self.impl = cfg, impl
        self.device = torch.device(device)
        torch.manual_seed(int(cfg.get("SEED_VALUE", 0)))
        mcfg, lcfg, ocfg = cfg.MODEL, cfg.LOSS.swav_loss, cfg.OPTIMIZER
        dcfg = cfg.DATA.TRAIN
        self.batch_size = int(dcfg.BATCHSIZE_PER_REPLICA)
        if impl == "eager":
            from .swav_eager import EagerSwAVModel

            self.model = EagerSwAVModel(num_prototypes=int(mcfg.HEAD.num_clusters),
                                        single_pass_every_crop=bool(mcfg.SINGLE_PASS_EVERY_CROP))
            self.model.to(self.device, memory_format=torch.channels_last)
        else:
            self.model = SwAVModel(num_prototypes=int(mcfg.HEAD.num_clusters),
                                   single_pass_every_crop=bool(mcfg.SINGLE_PASS_EVERY_CROP),
                                   checkpoint_stages=bool(mcfg.ACTIVATION_CHECKPOINTING.USE_ACTIVATION_CHECKPOINTING),
                                   conv_impl=mcfg.get("CONV_IMPL") or None)
            self.model.to(self.device)
        self.model.train()
        hooks = cfg.get("HOOKS") or {}
        self.check_nan = bool(hooks.get("CHECK_NAN", True))
        self.log_frequency = max(1, int(cfg.get("LOG_FREQUENCY", 10)))
        # vissl PerfTimer/LogPerfTimeMetricsHook (V20): HIP-event phase timers, reported per global step
        self.perf = PerfStats(self.device, enabled=bool(hooks.get("PERF_STATS", True)),
                              sample_every=int(cfg.get("LOG_FREQUENCY", 10)) if self.device.type == "cuda" else 1)
        self.flat = FlatParams(self.model.named_parameters(), device=self.device,
                               with_bf16=self.device.type == "cuda" and impl == "dedloc", autograd=True,
                               channels_last=bool(mcfg.get("CHANNELS_LAST", True)))
        if impl == "dedloc":
            self.model.bind_flat(self.flat)  # GEMM / conv weights read from the flat buffer's bf16 mirror
            # the crop groups' trunk passes on several streams (SwAVModel.concurrent_passes: one per
            # resolution, CONCURRENT_SPLITS cuts a resolution into passes of whole crops; this
            # trainer calls after_backward after every backward).  Fallback (2, 1), the shipped
            # config's value: the two 224 crops as two passes beside the 96-crop pass — three passes
            # of similar work instead of a 224 group ~1.8x the 96 group (b=64: +6.4% over (1, 1),
            # profiles/r5_swav_pass_splits.txt)
            self.model.concurrent_passes = bool(cfg.MODEL.get("CONCURRENT_PASSES", True))
            self.model.pass_splits = tuple(int(v) for v in cfg.MODEL.get("CONCURRENT_SPLITS", (2, 1)))
        self.model.normalize_prototypes()
        larc = ocfg.larc_config
        assert ocfg.use_larc, "we can't use collab sgd without larc (sgd_collaborative.py:138)"
        no_decay = _no_decay_names(self.model, bool(ocfg.regularize_bn), bool(ocfg.regularize_bias))
        if impl == "eager":
            from .swav_eager import EagerLarcSGD

            assert not bool(ocfg.nesterov), "nesterov LARC-SGD is not used by the reference"
            self.opt = EagerLarcSGD(self.flat, lr=float(ocfg.lr), momentum=float(ocfg.momentum),
                                    weight_decay=float(ocfg.weight_decay),
                                    trust_coefficient=float(larc.trust_coefficient), clip=bool(larc.clip),
                                    eps=float(larc.eps), no_decay=no_decay)
        else:
            self.opt = FusedLarcSGD(self.flat, lr=float(ocfg.lr), momentum=float(ocfg.momentum),
                                    weight_decay=float(ocfg.weight_decay), nesterov=bool(ocfg.nesterov),
                                    trust_coefficient=float(larc.trust_coefficient), clip=bool(larc.clip),
                                    eps=float(larc.eps), no_decay=no_decay)
        self.scheduler = LinearWarmupCosineAnnealingLR(self.opt, warmup_epochs=int(ocfg.warmup_epochs),
                                                       max_epochs=int(ocfg.max_epochs),
                                                       warmup_start_lr=float(ocfg.warmup_start_lr),
                                                       eta_min=float(ocfg.eta_min))
        validators, self.local_public_key = make_validators(ocfg.exp_prefix)
        self.dht = dht or DHT(initial_peers=list(ocfg.dht_initial_peers or []),
                              listen_on=_port_endpoint(ocfg.dht_listen_on_port), start=True,
                              record_validators=validators)
        self.collab_opt = CollaborativeOptimizer(
            self.opt, dht=self.dht, scheduler=self.scheduler, prefix=ocfg.exp_prefix,
            compression_type=str(ocfg.get("compression", "FLOAT16")),
            target_batch_size=int(ocfg.get("target_batch_size", 32768)),
            batch_size_per_step=int(ocfg.batch_size_for_tracking), verbose=True, start=True,
            peer_id=self.local_public_key, target_group_size=int(ocfg.target_group_size),
            listen_on=_port_endpoint(ocfg.averager_listen_on_port),
            averaging_expiration=float(ocfg.get("averaging_expiration", 5.0)),
            metadata_expiration=float(ocfg.get("metadata_expiration", 30)),
            averaging_timeout=float(ocfg.get("averaging_timeout", 30)), device=self.device)
        q = lcfg.queue
        loss_cls = SwAVLoss
        if impl == "eager":
            from .swav_eager import EagerSwAVLoss as loss_cls
        self.loss_fn = loss_cls(num_crops=sum(dcfg.MULTICROP.num_crops), crops_for_assign=lcfg.crops_for_assign,
                                temperature=float(lcfg.temperature), epsilon=float(lcfg.epsilon),
                                num_iters=int(lcfg.num_iters), num_prototypes=int(mcfg.HEAD.num_clusters),
                                embedding_dim=int(mcfg.HEAD.dims[-1]), queue_length=int(q.queue_length),
                                queue_start_iter=int(q.start_iter), batch_size=self.batch_size,
                                temp_hard_assignment_iters=int(lcfg.get("temp_hard_assignment_iters", 0)))
        self.loss_fn.to(self.device)
        mc = dcfg.MULTICROP
        aug = MultiCropAugment(size_crops=mc.size_crops, num_crops=mc.num_crops,
                               crop_scales=[tuple(s) for s in mc.crop_scales], flip_p=float(mc.flip_p),
                               color_strength=float(mc.color_strength), blur_p=float(mc.blur_p),
                               blur_radius=tuple(mc.blur_radius))
        seed = int.from_bytes(self.local_public_key[-8:], "little") ^ int(cfg.get("SEED_VALUE", 0))
        self.data = SyntheticMultiCropStream(self.batch_size, self.device, seed=seed,
                                             pool_size=int(dcfg.get("SYNTHETIC_POOL_SIZE", 1024)),
                                             image_size=int(dcfg.get("SYNTHETIC_IMAGE_SIZE", 256)), augment=aug,
                                             out_dtype=torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        if self.device.type == "cuda" and bool(dcfg.get("PREFETCH", True)):
            self.data = StreamPrefetcher(self.data, self.device)  # next batch's crops under this step's compute
        self.frozen = [(name, int(iters)) for name, iters in (mcfg.get("TEMP_FROZEN_PARAMS_ITER_MAP") or [])]
        self.use_graph = bool(mcfg.get("CUDA_GRAPH", False)) and self.device.type == "cuda" and \
            not bool(mcfg.ACTIVATION_CHECKPOINTING.USE_ACTIVATION_CHECKPOINTING) and impl == "dedloc"
        self.graph_warmup = int(mcfg.get("CUDA_GRAPH_WARMUP", 3))  # eager iterations before the capture
        self._graphed = None
        self.iteration = 0
        self._loss_sum = torch.zeros((), device=self.device)
        self._finite_part = torch.zeros(256, device=self.device)
        self._finite_out = torch.zeros(3, device=self.device)  # [grad norm, finite, 1 - finite]
        self.mini_steps = 0
        self.last_reported_step = -1
        self.metrics_log = []

    # ------------------------------------------------------------------ one local iteration
    # ------------------------------------------------------------------ HIP-graph capture
    def _build_graph(self, crops):
        """Capture the trunk+head forward and its backward as two HIP graphs sharing one memory pool
        (MODEL.CUDA_GRAPH).  The iteration launches ~1100 kernels, many of them a few microseconds
        long, so eager launching leaves the GPU idle between them; a replay issues each graph with
        one call.  Unlike ``make_graphed_callables`` nothing changes in the gradient flow: every
        conv / BN / linear weight gradient is still written in place into the flat gradient buffer
        (the captured kernels hold its fixed address), so no per-parameter grads are materialised
        or accumulated.  The SwAV loss (Sinkhorn over a queue that switches on at a global step,
        host-side ring pointer) stays eager between the two replays: the forward graph's
        embeddings / scores are its inputs and the gradient w.r.t. the scores is copied into the
        backward graph's static seed.  Warm-up iterations run on a side stream first (first-call
        allocations, kernel attributes), after which gradients and BN statistics are restored."""
        model = self.model
        # static inputs laid out like the pipeline's crops: one buffer per resolution, the crops its
        # batch slices (the model then joins them without a copy, and each replay refills them with
        # one copy per resolution)
        static = []
        for grp in self._resolution_groups(crops):
            static.extend(join_batch(grp).detach().clone().split(grp[0].shape[0]))
        grads = self.flat.grad.clone()
        bufs = {k: v.clone() for k, v in model.named_buffers()}

        def fwd():
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16, cache_enabled=False):
                return model(static)

        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):
                emb, scores = fwd()
                torch.autograd.backward([scores], [torch.ones_like(scores)])
                model.after_backward()
        torch.cuda.current_stream(self.device).wait_stream(side)
        g_fwd, g_bwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        # thread_local: the averager / DHT threads may touch the device while the trainer captures
        with torch.cuda.graph(g_fwd, capture_error_mode="thread_local"):
            emb, scores = fwd()
        seed = torch.zeros_like(scores)
        with torch.cuda.graph(g_bwd, pool=g_fwd.pool(), capture_error_mode="thread_local"):
            torch.autograd.backward([scores], [seed])
            model.after_backward()
        with torch.no_grad():
            self.flat.grad.copy_(grads)
            for k, v in model.named_buffers():
                v.copy_(bufs[k])
        self.flat.rebind_grads()
        return {"fwd": g_fwd, "bwd": g_bwd, "in": static, "emb": emb, "scores": scores, "seed": seed}

    @staticmethod
    def _resolution_groups(crops):
        out = []
        for c in crops:
            if out and out[-1][0].shape == c.shape:
                out[-1].append(c)
            else:
                out.append([c])
        return out

    def _graph_iteration(self, crops):
        """One forward + loss + backward through the captured graphs (see _build_graph)."""
        gr = self._graphed
        i = 0
        for grp in self._resolution_groups(crops):
            join_batch(gr["in"][i:i + len(grp)]).copy_(join_batch(grp))
            i += len(grp)
        with self.perf.phase("fwd"):
            gr["fwd"].replay()
        with self.perf.phase("loss_bwd"):
            scores = gr["scores"].detach().requires_grad_(True)
            proto = self.model.heads[0].prototypes0.weight
            loss = self.loss_fn(gr["emb"].detach().float(), scores, proto,
                                training_iterations=int(self.collab_opt.local_step))
            loss.backward()
            gr["seed"].copy_(scores.grad)
            gr["bwd"].replay()
        return loss

    def _forward(self, crops):
        with torch.autocast(device_type=self.device.type, dtype=torch.bfloat16,
                            enabled=self.device.type == "cuda"):
            return self.model(crops)

    def train_step(self, crops=None):
        with self.perf.phase("data"):
            crops = crops if crops is not None else self.data.next_batch()
        if self.use_graph and self.iteration >= self.graph_warmup:
            if self._graphed is None:
                self._graphed = self._build_graph(crops)
            loss = self._graph_iteration(crops)
        else:
            with self.perf.phase("fwd"):
                emb, scores = self._forward(crops)
            with self.perf.phase("loss_bwd"):
                proto = self.model.heads[0].prototypes0.weight
                loss = self.loss_fn(emb.float(), scores, proto, training_iterations=int(self.collab_opt.local_step))
                loss.backward()
                if self.impl == "dedloc":
                    self.model.after_backward()
        for name, iters in self.frozen:  # FreezeParametersHook (state_update_hooks.py:235-280)
            if self.iteration < iters:
                name = name[len("module."):] if name.startswith("module.") else name
                self.flat.view(self.flat.grad, name).zero_()
        self._loss_sum += loss.detach()
        finite = None
        if self.impl == "dedloc":
            # every micro-step: the gradient's finite flag on the device; a non-finite step's gradient
            # is zeroed there and its samples do not count (collab_opt.step(finite=...)), so it can
            # never be averaged into the other peers — with no host sync
            torch.ops.dedloc.grad_norm_clip(self.flat.grad, 0.0, self._finite_part, self._finite_out)
            torch.ops.dedloc.axpby(self.flat.grad, self.flat.grad, 0.0, 0.0, self._finite_out[2:3])
            finite = self._finite_out[1:2]
        if self.check_nan and (self.iteration + 1) % self.log_frequency == 0:
            self._check_nan_async()
        with self.perf.phase("collab_step"):
            self.collab_opt.step(batch_size=self.batch_size, finite=finite)
        self.opt.zero_grad()
        self.model.normalize_prototypes()  # NormalizePrototypesHook.on_update (swav_hooks.py:63-92)
        self.iteration += 1
        self.perf.next_iteration()
        self.mini_steps += 1
        self._on_step_end()
        return loss.detach()

    def _on_step_end(self):
        co = self.collab_opt
        if co.local_step == self.last_reported_step:
            return
        self.last_reported_step = co.local_step
        loss = float(self._loss_sum.item())
        if self.check_nan and not math.isfinite(loss):
            self._nan_dump(loss)
        stats = LocalMetrics(step=int(co.local_step), samples_per_second=float(co.performance_ema.samples_per_second),
                             samples_accumulated=int(co.local_samples_accumulated), loss=loss,
                             mini_steps=int(self.mini_steps))
        self.dht.store(co.prefix + "_metrics", stats.model_dump(), expiration_time=get_dht_time() + 600,
                       subkey=self.local_public_key, return_future=True)
        rec = dict(stats.model_dump(), time=time.time(), iteration=self.iteration, lr=self.opt.param_groups[0]["lr"],
                   queue=bool(self.loss_fn.use_queue), **self.perf.report())
        self.metrics_log.append(rec)
        if self.cfg.get("METRICS_FILE"):
            with open(self.cfg.METRICS_FILE, "a") as f:
                f.write(json.dumps(rec) + "\n")
        logger.info(f"collaborative step {co.local_step}: loss {loss / max(1, self.mini_steps):.4f} "
                    f"lr {self.opt.param_groups[0]['lr']:.4g}")
        self._loss_sum.zero_()
        self.mini_steps = 0

    def _check_nan_async(self):
        """Every LOG_FREQUENCY iterations: queue a device-to-pinned-host copy of the running loss's
        finite flag behind this iteration, and act on the flags that have landed (the previous
        check's, typically).  A blocking read here drained the GPU queue every LOG_FREQUENCY
        iterations and left the device idle while the host refilled it; this way a non-finite loss
        is still caught within ~2 LOG_FREQUENCY iterations and at every global-step report."""
        pend = self.__dict__.setdefault("_nan_pending", [])
        flag = torch.isfinite(self._loss_sum)
        if flag.is_cuda:
            host = torch.empty((), dtype=torch.bool, pin_memory=True)
            host.copy_(flag, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            pend.append((host, ev))
        else:
            pend.append((flag, None))
        while pend:
            host, ev = pend[0]
            if ev is not None and not ev.query():
                break
            pend.pop(0)
            if not bool(host):
                self._nan_dump(float(self._loss_sum))

    def _nan_dump(self, loss: float):
        """vissl CheckNanLossHook (``state_update_hooks.py:207-233``) / the SwAV loss's NaN dump: save
        the model, optimizer and loss state next to the checkpoints, then stop this peer.  Checked every
        LOG_FREQUENCY iterations without a host sync (``_check_nan_async``) and at every global-step
        report, where the loss is read anyway."""
        d = Path(self.cfg.CHECKPOINT.DIR)
        d.mkdir(parents=True, exist_ok=True)
        path = d / f"nan_dump_iteration{self.iteration}.torch"
        state = self.state_dict()
        state["loss_sum"] = loss
        torch.save(state, path)
        logger.error(f"non-finite SwAV loss ({loss}) at iteration {self.iteration}; state dumped to {path}")
        raise FloatingPointError(f"non-finite SwAV loss at iteration {self.iteration} (dump: {path})")

    # ------------------------------------------------------------------ checkpoints (V19)
    def state_dict(self):
        return {"model": {k: v.detach().cpu().contiguous() for k, v in self.model.state_dict().items()},
                "optimizer": self.opt.state_dict(), "iteration": self.iteration,
                "collab_step": int(self.collab_opt.local_step),
                "loss": {k: v.cpu() for k, v in self.loss_fn.state_dict().items()}}

    def save_checkpoint(self, directory: Optional[str] = None):
        d = Path(directory or self.cfg.CHECKPOINT.DIR)
        d.mkdir(parents=True, exist_ok=True)
        path = d / f"model_iteration{self.iteration}.torch"
        torch.save(self.state_dict(), path)
        link = d / "checkpoint.torch"
        if link.is_symlink() or link.exists():
            link.unlink()
        link.symlink_to(path.name)
        return path

    @torch.no_grad()
    def load_checkpoint(self, path: str):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        own = self.model.state_dict()
        for k, v in sd["model"].items():
            own[k].copy_(v)
        self.opt.load_state_dict(sd["optimizer"])
        self.iteration = int(sd["iteration"])
        self.collab_opt.local_step = max(self.collab_opt.local_step, int(sd["collab_step"]))
        self.collab_opt.update_scheduler()
        self.loss_fn.load_state_dict({k: v.to(self.device) for k, v in sd["loss"].items()})

    def maybe_resume(self):
        if not self.cfg.CHECKPOINT.get("AUTO_RESUME", False):
            return False
        link = Path(self.cfg.CHECKPOINT.DIR) / "checkpoint.torch"
        if link.exists():
            logger.info(f"resuming from {link.resolve()}")
            self.load_checkpoint(str(link))
            return True
        return False

    def train(self, max_iterations: Optional[int] = None, stop_after_global_steps: Optional[int] = None,
              max_seconds: Optional[float] = None):
        self.collab_opt.load_state_from_peers()
        t0, start = time.time(), self.collab_opt.local_step
        freq = int(self.cfg.CHECKPOINT.get("CHECKPOINT_ITER_FREQUENCY", 0) or 0)
        while max_iterations is None or self.iteration < max_iterations:
            self.train_step()
            if freq and self.iteration % freq == 0:
                self.save_checkpoint()
            if stop_after_global_steps is not None and self.collab_opt.local_step - start >= stop_after_global_steps:
                break
            if max_seconds is not None and time.time() - t0 > max_seconds:
                break

    def shutdown(self):
        self.collab_opt.shutdown()
        self.dht.shutdown()
