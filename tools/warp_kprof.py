"""Launch the warp backward (default path) N times at one decoder site on the
smooth +-2 px field, plain launches, for rocprofv3 --kernel-trace --stats.
Usage: rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/warp_kprof.py [B C H W]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd.kernel_timer import site_launcher  # noqa: E402

shape = tuple(int(v) for v in sys.argv[1:5]) if len(sys.argv) >= 5 else (16, 32, 64, 208)
fn = site_launcher("warp_bwd", shape + ("border", True, True), torch.device("cuda:0"))
for _ in range(int(os.environ.get("KPROF_N", "10"))):
    fn()
torch.cuda.synchronize()
