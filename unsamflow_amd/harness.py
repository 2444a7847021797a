"""Training-step harness around the hot path (the benchmark's "step").

Reproduces the shape of the reference's training step
(trainer/kitti_trainer_ar.py:108-317 with trainer/base_trainer.py:141-169):

    res = model(img1, img2, with_bk=True)
    flows = [cat(f12, f21)]                       # :113-117
    loss = unFlowLoss(flows, img1, img2).mean()   # :127-133
    optimizer.zero_grad(set_to_none=True); loss.backward()          # :309-310
    clip_grad_norm_(params, max_grad_norm); optimizer.step(); scheduler.step()  # :313-317

with Adam(betas=(momentum, beta), eps=1e-7) over the bias / weight parameter
groups (base_trainer.py:141-169) and OneCycleLR. Data is synthetic (U[0,1)
frames, as ``/255`` images of datasets/flow_datasets.py:59-63). With
``ddp=True`` the model is wrapped in DistributedDataParallel (train.py:116-120):
one process per GPU, gradient all-reduce over RCCL ("nccl" backend) / gloo.

The per-step host syncs of the reference's logging (``loss.item()``,
kitti_trainer_ar.py:284-293) are not part of the step.
"""
from __future__ import annotations

from typing import Callable

import torch

from .flow_loss import unFlowLoss
from .pwclite import PWCLite


def param_groups(model: torch.nn.Module, train_cfg) -> list[dict]:
    """Bias / weight / other groups as utils/torch_utils.py:27-40 (empty groups dropped)."""
    named = list(model.named_parameters())
    groups = [
        {"params": [p for n, p in named if ".bias" in n], "weight_decay": train_cfg.bias_decay},
        {"params": [p for n, p in named if ".weight" in n], "weight_decay": train_cfg.weight_decay},
        {"params": [p for n, p in named if ".bias" not in n and ".weight" not in n], "weight_decay": 0},
    ]
    return [g for g in groups if g["params"]]


def synthetic_pair(B: int, H: int, W: int, device, seed: int = 42, with_seg: bool = False, n_seg: int = 32):
    """U[0,1) frame pair [B,3,H,W] (+ piecewise-constant segment maps [B,1,H,W] as float)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    img1 = torch.rand(B, 3, H, W, generator=g).to(device)
    img2 = torch.rand(B, 3, H, W, generator=g).to(device)
    if not with_seg:
        return img1, img2, None, None
    blk = 32
    segs = []
    for _ in range(2):
        ids = torch.randint(0, n_seg, (B, 1, (H + blk - 1) // blk, (W + blk - 1) // blk), generator=g).float()
        seg = ids.repeat_interleave(blk, 2).repeat_interleave(blk, 3)[:, :, :H, :W]
        segs.append(seg.contiguous().to(device))
    return img1, img2, segs[0], segs[1]


class TrainStep:
    """One PWCLite fwd(with_bk) + unFlowLoss + bwd + clip + Adam + OneCycleLR step."""

    def __init__(self, cfg, device, ddp: bool = False, corr_module=None, warp_fn: Callable | None = None,
                 loss_kwargs: dict | None = None, fused_adam: bool | None = None, seed: int = 42,
                 channels_last: bool = False, occ_backward_fn: Callable | None = None,
                 capturable: bool = False):
        torch.manual_seed(seed)
        self.cfg = cfg
        self.device = torch.device(device)
        model = PWCLite(cfg.model, corr_module=corr_module, warp_fn=warp_fn).to(self.device)
        if channels_last:  # NHWC weights/activations for MIOpen's NHWC convolutions
            model = model.to(memory_format=torch.channels_last)
        self.module = model
        if ddp:
            ids = [self.device.index] if self.device.type == "cuda" else None
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=ids)
        self.model = model
        self.loss_fn = unFlowLoss(cfg.loss, warp_fn=warp_fn, occ_backward_fn=occ_backward_fn,
                                  **(loss_kwargs or {}))
        t = cfg.train
        if fused_adam is None:
            fused_adam = self.device.type == "cuda"
        # capturable: the step counters and the learning rate live on the device
        # (the scheduler fills the lr tensor in place), so the step can be
        # captured into a HIP graph (GraphedTrainStep)
        lr = torch.tensor(float(t.lr), device=self.device) if capturable else t.lr
        self.optimizer = torch.optim.Adam(param_groups(self.module, t), lr, betas=(t.momentum, t.beta), eps=1e-7,
                                          fused=fused_adam or None, capturable=capturable)
        sched = t.get("lr_scheduler")
        if sched and sched.module == "OneCycleLR":
            p = dict(sched.params)
            p.update(epochs=t.epoch_num, steps_per_epoch=t.epoch_size)
            self.scheduler = torch.optim.lr_scheduler.OneCycleLR(self.optimizer, **p)
        else:
            self.scheduler = torch.optim.lr_scheduler.ExponentialLR(self.optimizer, gamma=1)
        self.max_grad_norm = t.max_grad_norm
        # None, or a list that every call appends one (start, after backward, end)
        # triple of device events to: the optimizer step (clip + Adam + scheduler)
        # timed apart from fwd + loss + bwd (bench.py)
        self.phase_events: list | None = None

    def forward_loss(self, img1, img2, full_seg1=None, full_seg2=None):
        res = self.model(img1, img2, full_seg1, full_seg2, with_bk=True)
        flows = [torch.cat([a, b], 1) for a, b in zip(res["flows_12"], res["flows_21"])]
        kw = {}
        if full_seg1 is not None:
            kw = dict(full_seg1=full_seg1, full_seg2=full_seg2)
        loss, l_ph, l_sm, fmean, _, _ = self.loss_fn(flows, img1, img2, **kw)
        return loss.mean(), flows

    def __call__(self, img1, img2, full_seg1=None, full_seg2=None):
        ev = None
        if self.phase_events is not None:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
        loss, _ = self.forward_loss(img1, img2, full_seg1, full_seg2)
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        if ev is not None:
            ev[1].record()
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.max_grad_norm)
        self.optimizer.step()
        self.scheduler.step()
        if ev is not None:
            ev[2].record()
            self.phase_events.append(ev)
        return loss.detach()


class FlatGrads:
    """Every parameter's .grad as a view of one flat fp32 buffer: static
    addresses for graph capture, and ONE all-reduce bucket per step for data
    parallelism (10 MB for PWCLite: one RCCL ring all-reduce over xGMI instead
    of DDP's per-bucket hooks). Backward accumulates into the views, so the
    buffer is zeroed at the start of every step."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        for p in self.params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero_(self):
        self.flat.zero_()

    def all_reduce_mean(self, group=None):
        import torch.distributed as dist

        world = dist.get_world_size(group)
        if world > 1:
            dist.all_reduce(self.flat, group=group)
            self.flat.div_(world)


def broadcast_params(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Replicas start from rank ``src``'s weights (what DDP's constructor does)."""
    import torch.distributed as dist

    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t, src, group=group)


class GraphedTrainStep:
    """The TrainStep replayed from HIP graphs (torch.cuda.CUDAGraph): the ~4k
    kernel launches of a PWCLite step (MIOpen convolutions, torch elementwise
    work and this library's kernels) are captured once and re-issued by one
    graph launch, so the step no longer pays per-launch host cost.

    Single process: one graph = zero grads + fwd(with_bk) + unFlowLoss + bwd +
    clip_grad_norm_ + Adam(capturable). Data parallel (world > 1): graph A =
    zero + fwd + loss + bwd into the flat gradient buffer, then one eager
    all-reduce of that buffer over RCCL, then graph B = clip + Adam. OneCycleLR
    runs eagerly between replays (it fills the device lr tensor in place).
    Inputs are static buffers: ``load()`` copies new frames in before a replay.
    """

    def __init__(self, step: TrainStep, img1, img2, full_seg1=None, full_seg2=None, warmup: int = 3,
                 group=None):
        import torch.distributed as dist

        self.step = step
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.inputs = [None if t is None else t.clone() for t in (img1, img2, full_seg1, full_seg2)]
        self.grads = FlatGrads(step.module.parameters())
        dev = step.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # allocator pools, solver selection, optimizer state
            for _ in range(warmup):  # real training steps, as TrainStep.__call__
                self._fwd_bwd()
                self._reduce()
                self._update()
                self.step.scheduler.step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        if self.world == 1:
            self.graph_a = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_a):
                self.loss = self._fwd_bwd()
                self._update()
            self.graph_b = None
        else:
            self.graph_a = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_a):
                self.loss = self._fwd_bwd()
            self.graph_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_b, pool=self.graph_a.pool()):
                self._update()

    def _fwd_bwd(self):
        self.grads.zero_()
        loss, _ = self.step.forward_loss(*self.inputs)
        loss.backward()
        return loss.detach()

    def _reduce(self):
        if self.world > 1:
            self.grads.all_reduce_mean(self.group)

    def _update(self):
        torch.nn.utils.clip_grad_norm_(self.grads.params, self.step.max_grad_norm)
        self.step.optimizer.step()

    def load(self, img1, img2, full_seg1=None, full_seg2=None):
        for dst, src in zip(self.inputs, (img1, img2, full_seg1, full_seg2)):
            if dst is not None:
                dst.copy_(src)

    def __call__(self):
        self.graph_a.replay()
        if self.graph_b is not None:
            self._reduce()
            self.graph_b.replay()
        self.step.scheduler.step()
        return self.loss

