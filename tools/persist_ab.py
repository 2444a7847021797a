"""Warm (graph replay) and cold device time of the warp backward and the
occlusion mask in their persistent two-launch forms (ops.warp_backward /
ops.occ_backward: usf_warp_bwd_persist_f32, usf_occ_backward_persist_f32)
against the per-call forms (usf_warp_bwd_ex_f32: fill + filing + gather +
overflow pass; usf_occ_backward_f32: fill + splat + threshold), same process,
same inputs (kernel_timer.site_launcher's smooth +-2 px flow).
Usage (GPU box): python tools/persist_ab.py --out gpurun_out/persist_ab.json"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd import _lib, ops  # noqa: E402
from unsamflow_amd.kernel_timer import device_time_cold_us, device_time_us  # noqa: E402

KITTI = [(128, 8, 26), (96, 16, 52), (64, 32, 104), (32, 64, 208)]


def flow_field(B, H, W, dev):
    yy = torch.linspace(0, 6.2832, H, device=dev).view(1, 1, H, 1)
    xx = torch.linspace(0, 6.2832, W, device=dev).view(1, 1, 1, W)
    return (2.0 * torch.sin(2 * xx) * torch.cos(yy)).expand(B, 2, H, W).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/persist_ab.json")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    rows = []
    for C, H, W in KITTI:
        B = 16
        g = torch.Generator(device=dev).manual_seed(C)
        x = torch.randn(B, C, H, W, device=dev, generator=g)
        go = torch.randn(B, C, H, W, device=dev, generator=g)
        flow = flow_field(B, H, W, dev)
        gx, gf = torch.empty_like(x), torch.empty(B, 2, H, W, device=dev)
        n = int(lib.usf_warp_bwd_workspace(B, H, W))
        ws = torch.empty(n, device=dev, dtype=torch.uint8)

        def ex():
            rc = lib.usf_warp_bwd_ex_f32(x.data_ptr(), flow.data_ptr(), 2 * H * W, go.data_ptr(), gx.data_ptr(),
                                         gf.data_ptr(), ws.data_ptr(), n, B, C, H, W, _lib.PAD_BORDER,
                                         _lib.stream_handle(dev))
            _lib.check(rc, "usf_warp_bwd_ex_f32")

        def persist():
            ops.warp_backward(x, flow, go, "border", True, True)

        for name, fn in (("ex4", ex), ("persist2", persist), ("ex4", ex), ("persist2", persist)):
            rows.append(dict(op="warp_bwd", shape=[B, C, H, W], form=name, warm_us=round(device_time_us(fn), 2),
                             cold_us=round(device_time_cold_us(fn), 2)))
            print(json.dumps(rows[-1]), flush=True)
    B, H, W = 8, 256, 832
    flow = flow_field(B, H, W, dev)
    occ = torch.empty(B, 1, H, W, device=dev)

    def occ_ex():
        rc = lib.usf_occ_backward_f32(flow.data_ptr(), 2 * H * W, occ.data_ptr(), B, H, W, 0.2,
                                      _lib.stream_handle(dev))
        _lib.check(rc, "usf_occ_backward_f32")

    for name, fn in (("ex3", occ_ex), ("persist2", lambda: ops.occ_backward(flow, 0.2)), ("ex3", occ_ex),
                     ("persist2", lambda: ops.occ_backward(flow, 0.2))):
        rows.append(dict(op="occ_bwd", shape=[B, 1, H, W], form=name, warm_us=round(device_time_us(fn), 2),
                         cold_us=round(device_time_cold_us(fn), 2)))
        print(json.dumps(rows[-1]), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
