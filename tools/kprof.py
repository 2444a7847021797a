"""Launch each hot-path kernel N times at PWCLite's KITTI call-site shapes (B=8
pairs: the decoder's sites at batch 16 = both with_bk directions stacked,
PWCLite.batch_directions; the loss's at 8),
plain (no graphs) so rocprofv3 --pmc attributes counters per dispatch.
Usage: rocprofv3 --pmc <counters> --kernel-trace --output-format csv -d DIR -o run -- python3 tools/kprof.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib  # noqa: E402
from unsamflow_amd.kernel_timer import site_launcher  # noqa: E402

KITTI = [(192, 4, 13), (128, 8, 26), (96, 16, 52), (64, 32, 104), (32, 64, 208)]
DB = int(os.environ.get("KPROF_DECODER_B", "16"))  # decoder batch: 2 x 8 pairs
SITES = [("corr_fwd", (DB, C, H, W)) for C, H, W in KITTI]
SITES += [("corr_fwd_leaky", (DB, C, H, W)) for C, H, W in KITTI]
SITES += [("corr_bwd", (DB, C, H, W, True, True)) for C, H, W in KITTI]
# one direction at a time (where the backward's traffic comes from)
SITES += [("corr_bwd", (DB, C, H, W, n1, not n1)) for C, H, W in KITTI[3:] for n1 in (True, False)]
SITES += [("corr_bwd_leaky", (DB, C, H, W, True, True)) for C, H, W in KITTI]
SITES += [("warp_fwd", (DB, C, H, W, "border")) for C, H, W in KITTI[1:]]
SITES += [("warp_fwd_up", (DB, C, H, W, "border")) for C, H, W in KITTI[1:]]
SITES += [("warp_bwd", (DB, C, H, W, "border", True, True)) for C, H, W in KITTI[1:]]
SITES += [("warp_fwd", (8, 3, 256, 832, "border")), ("warp_bwd", (8, 3, 256, 832, "border", False, True))]
SITES += [("convex_up", (DB, H, W, 4)) for _, H, W in KITTI]
SITES += [("convex_up_bwd", (DB, H, W, 4)) for _, H, W in KITTI]
SITES += [("occ_bwd", (8, 1, 256, 832)), ("occ_vis_pair", (8, 1, 256, 832)), ("area_pyramid", (8, 3, 256, 832))]
SITES += [("photo_fwd", (8, 3, 256 >> i, 832 >> i, "border")) for i in range(4)]
SITES += [("photo_fwd_grad", (8, 3, 256 >> i, 832 >> i, "border")) for i in range(4)]
SITES += [("photo_pair_grad", (8, 3, 256 >> i, 832 >> i, "border")) for i in range(4)]
SITES += [("photo_bwd", (8, 2, 256 >> i, 832 >> i)) for i in range(4)]
# every decoder level's convex upsampling in one launch (the training step's form; finest first)
CPYR = tuple(v for _, H, W in KITTI[::-1] for v in (H, W))
SITES += [("convex_pyr", (DB,) + CPYR + (4,)), ("convex_pyr_bwd", (DB,) + CPYR + (4,))]
# the four loss scales in one launch (the training step's form)
PYR = tuple(v for i in range(4) for v in (256 >> i, 832 >> i))
SITES += [("photo_pyr_grad", (8, 3) + PYR + ("border",)), ("photo_pyr_bwd", (8, 2) + PYR)]
# BASELINE config 2 (single-level correlation, B=8 C=128 32x104)
SITES += [("corr_fwd", (8, 128, 32, 104)), ("corr_bwd", (8, 128, 32, 104, True, True))]


def selected_sites():
    """SITES, or the subset whose op is listed in KPROF_OPS (comma-separated)."""
    only = os.environ.get("KPROF_OPS")
    return [s for s in SITES if not only or s[0] in only.split(",")]


SEPARATOR = "stream_copy_kernel"  # the marker kernel between launches (usf_stream_copy_f32 of 4 floats)


def main():
    """Per site: its launcher (setup kernels), then n x (separator, launch),
    then a closing separator. tools/pmc_traffic.py cuts the dispatch list at
    the separators, so every launch's kernels -- however many one call runs
    (persistent two-launch forms, split forwards, fills) -- are summed as that
    launch, and the setup kernels fall outside every launch."""
    lib = _lib.load()
    if os.environ.get("USF_PHOTO_VARIANT"):  # usf_set_variant op 3: one pair kernel, only -1 / 0 accepted
        v = int(os.environ["USF_PHOTO_VARIANT"])
        if lib.usf_set_variant(3, v) < 0:
            sys.exit(f"usf_set_variant(3, {v}) refused: no such photometric variant")
    dev = torch.device("cuda:0")
    n = int(os.environ.get("KPROF_N", "3"))
    # calibration: a plain 256 MiB device copy (16-B loads/stores) for FETCH/WRITE_SIZE scaling
    a = torch.empty(64 * 1024 * 1024, device=dev)
    b = torch.empty_like(a)
    for _ in range(n):
        b.copy_(a)
    sa, sb = torch.zeros(4, device=dev), torch.empty(4, device=dev)
    stream = _lib.stream_handle(dev)

    def sep():
        _lib.check(lib.usf_stream_copy_f32(sa.data_ptr(), sb.data_ptr(), 4, stream), "usf_stream_copy_f32")

    for op, key in selected_sites():
        fn = site_launcher(op, key, dev)
        for _ in range(n):
            sep()
            fn()
        sep()
        torch.cuda.synchronize()
    print("kprof done")


if __name__ == "__main__":
    main()
