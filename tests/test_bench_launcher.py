"""bench.py --gpus N starts its own N ranks when no torch.distributed
environment is set (the driver's plain `python bench.py --gpus N`), as the
reference trainer spawns its world itself (train.py:228-234, per-rank batch
train.py:82). Runs the launcher on CPU/gloo (`--device cpu`: the cpu_baseline
step, a plumbing test, never a measurement) with N=2 and checks the one JSON
line rank 0 prints."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=600):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("config", ["kitti", "sintel_mf"])
def test_bench_spawns_two_ranks_on_gloo(config):
    hw = ["64", "128"] if config == "kitti" else ["128", "256"]  # sintel_mf: its capture size (test_ddp_cpu)
    p = _run(["--device", "cpu", "--gpus", "2", "--steps", "1", "--warmup", "0", "--batch", "1",
              "--hw", *hw, "--config", config])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 2 and out["config"]["per_gpu_batch"] == 1
    assert out["scaling"] == "weak"
    assert out["value"] > 0 and out["device"].startswith("cpu")
    assert ("Sintel" in out["metric"]) == (config == "sintel_mf")
    assert out["final_loss"] == out["final_loss"]  # finite (not NaN)


@pytest.mark.timeout(300)
def test_bench_rejects_mismatched_world():
    """Under an external launcher, --gpus must equal WORLD_SIZE (no silent one-rank run)."""
    p = _run(["--device", "cpu", "--gpus", "2", "--steps", "1", "--warmup", "0", "--batch", "1",
              "--hw", "64", "128"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE" in p.stderr
