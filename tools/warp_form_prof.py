"""Per-kernel durations of the two warp-backward forms at one level, for
rocprofv3 --kernel-trace --stats (GPU box):
  rocprofv3 --kernel-trace --stats -d gpurun_out/wf -- python tools/warp_form_prof.py [B C H W]
Both forms run alternately on the same inputs (smooth synthetic flow), so the
stats file holds the persistent form's kernels (warp_bwd_kernel<..., 2>,
warp_gx_bins_kernel<true>) beside the four-launch form's (<..., 1>, <false>,
zero_fill_kernel, warp_gx_ovf_kernel)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import ops  # noqa: E402


def main():
    B, C, H, W = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (16, 32, 64, 208)))
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(B, C, H, W, generator=g).to(dev)
    gout = torch.randn(B, C, H, W, generator=g).to(dev)
    # smooth flow of a few pixels (as the decoder's upsampled flows)
    base = torch.randn(B, 2, H // 8 + 1, W // 8 + 1, generator=g) * float(os.environ.get("FLOW_SCALE", "0.5"))
    flow = torch.nn.functional.interpolate(base, size=(H, W), mode="bilinear", align_corners=True).to(dev)
    if os.path.exists("gpurun_out/warp_bwd_l4.pt"):  # the training step's own inputs (warp_flow_capture.py)
        d = torch.load("gpurun_out/warp_bwd_l4.pt", weights_only=True)
        x, flow, gout = d["x"].to(dev), d["flow"].to(dev), d["g"].to(dev)
        print("captured inputs", tuple(x.shape))
    for _ in range(3):
        for form in (None, 0):
            ops.WARP_PERSIST_MAX_PIXELS = form
            ops.warp_backward(x, flow, gout, "border")
    torch.cuda.synchronize()
    for _ in range(20):
        for form in (None, 0):
            ops.WARP_PERSIST_MAX_PIXELS = form
            ops.warp_backward(x, flow, gout, "border")
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
