"""Launch the warp backward (default path) N times at one decoder site on one
of tools/warpab.py's flow fields (zero / pm2 / pm8 / shift), plain launches, for
rocprofv3 --kernel-trace --stats.
Usage: rocprofv3 ... -- python3 tools/warp_kprof2.py FLOW [B C H W]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.warpab import flows  # noqa: E402
from unsamflow_amd import ops  # noqa: E402

name = sys.argv[1]
B, C, H, W = (int(v) for v in sys.argv[2:6]) if len(sys.argv) >= 6 else (16, 32, 64, 208)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, C, H, W, device=dev, generator=g)
go = torch.randn(B, C, H, W, device=dev, generator=g)
fl = flows(B, H, W, dev, g)[name]
for _ in range(int(os.environ.get("KPROF_N", "10"))):
    ops.warp_backward(x, fl, go, "border", True, True)
torch.cuda.synchronize()
