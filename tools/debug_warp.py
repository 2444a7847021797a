"""Debug: locate GPU-vs-oracle warp mismatches at the 832x256 zeros case."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import hashrng
from oracle.warp import warp_forward_np, _taps
from unsamflow_amd import ops
B, C, H, W = 2, 3, 256, 832
seed = C * 7 + H
x = hashrng.uniform((B, C, H, W), seed)
flow = hashrng.symmetric((B, 2, H, W), seed + 1, 40.0)
dev = torch.device("cuda:0")
for pad in ("zeros", "border"):
    out = ops.warp_forward(torch.from_numpy(x).to(dev), torch.from_numpy(flow).to(dev), pad).cpu().numpy()
    ref = warp_forward_np(x, flow, pad)
    d = np.abs(out - ref)
    print(pad, "max", d.max(), "n>1e-5", int((d > 1e-5).sum()))
    idx = np.argwhere(d > 1e-5)[:8]
    t = _taps(flow, H, W, pad)
    for b, c, yy, xx in idx:
        u, v = flow[b, 0, yy, xx], flow[b, 1, yy, xx]
        print(f"  b{b} c{c} y{yy} x{xx} u={u!r} v={v!r} gpu={out[b,c,yy,xx]!r} ref={ref[b,c,yy,xx]!r} "
              f"xw={t['xw'][b,yy,xx]} yn={t['yn'][b,yy,xx]} w={t['w'][b,yy,xx]!r} n={t['n'][b,yy,xx]!r}")
