"""Capture the warp-backward inputs of the training step (GPU box): runs a few
KITTI steps of the bench workload, saves the largest level's (x, flow,
grad_output) of the last step to gpurun_out/warp_bwd_l4.pt and prints, per
level, how many source pixels share a north-west cell beyond the 4 bin slots
(the overflow the binned gather adds separately)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import ops  # noqa: E402
from unsamflow_amd.config import kitti_base  # noqa: E402
from unsamflow_amd.harness import TrainStep, synthetic_pair  # noqa: E402

seen = {}
_orig = ops.warp_backward


def spy(x, flow, grad_out, pad="border", need_x=True, need_flow=True):
    seen[tuple(x.shape)] = (x.detach().clone(), flow.detach().clone(), grad_out.detach().clone(), pad)
    return _orig(x, flow, grad_out, pad, need_x, need_flow)


def overflow(flow, pad):
    B, _, H, W = flow.shape
    f = flow[:, :2].float()
    ys, xs = torch.meshgrid(torch.arange(H, device=f.device), torch.arange(W, device=f.device), indexing="ij")
    ix, iy = xs + f[:, 0], ys + f[:, 1]
    if pad == "border":
        ix, iy = ix.clamp(0, W - 1), iy.clamp(0, H - 1)
    xw, yn = ix.floor().long(), iy.floor().long()
    ok = (xw >= -1) & (xw < W) & (yn >= -1) & (yn < H)
    cell = (torch.arange(B, device=f.device).view(B, 1, 1) * (H + 1) + yn + 1) * (W + 1) + xw + 1
    cnt = torch.bincount(cell[ok].flatten(), minlength=B * (H + 1) * (W + 1))
    return int((cnt - 4).clamp(min=0).sum()), int((cnt > 4).sum()), float(f.abs().max())


def main():
    dev = torch.device("cuda:0")
    ops.warp_backward = spy
    step = TrainStep(kitti_base(), dev, seed=42)
    img1, img2, _, _ = synthetic_pair(8, 256, 832, dev)
    for _ in range(8):
        step(img1, img2)
    torch.cuda.synchronize()
    for shp, (x, flow, g, pad) in sorted(seen.items(), key=lambda kv: kv[0][2] * kv[0][3]):
        n_px, n_cells, fmax = overflow(flow, pad)
        print(f"{shp} pad={pad} |flow|max={fmax:.2f} overflow pixels={n_px} cells={n_cells}", flush=True)
    big = max(seen, key=lambda s: s[2] * s[3] if s[1] > 3 else 0)
    x, flow, g, pad = seen[big]
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save({"x": x.cpu(), "flow": flow.cpu(), "g": g.cpu(), "pad": pad}, "gpurun_out/warp_bwd_l4.pt")


if __name__ == "__main__":
    main()
