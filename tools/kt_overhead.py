"""Cost of the per-launch HIP events (KernelTimer) on the training step (GPU
box): 4 alternating rounds of 10 KITTI steps with the timer off / on, wall
time per step in ms. Round 6: 39.89 ms off vs 40.17 ms on (median), which is
why bench.py brackets only the roofline site inside its timed region."""
import sys, time, torch
sys.path.insert(0, '.')
from unsamflow_amd.config import kitti_base
from unsamflow_amd.harness import TrainStep, synthetic_pair
from unsamflow_amd.kernel_timer import KernelTimer
dev = torch.device('cuda:0')
step = TrainStep(kitti_base(), dev, seed=42)
i1, i2, _, _ = synthetic_pair(8, 256, 832, dev)
for _ in range(8): step(i1, i2)
torch.cuda.synchronize()
res = {True: [], False: []}
for r in range(4):
    for en in (False, True):
        torch.cuda.synchronize()
        with KernelTimer(enabled=en):
            t0 = time.perf_counter()
            for _ in range(10): step(i1, i2)
            torch.cuda.synchronize()
        res[en].append((time.perf_counter() - t0) / 10 * 1e3)
print({k: [round(x, 3) for x in v] for k, v in res.items()})
