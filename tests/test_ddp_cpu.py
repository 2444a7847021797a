"""Multi-process data parallelism of the training step (train.py:42-147 pattern:
one process per device, DDP, per-rank batch = global // world) on CPU with the
gloo backend, world_size 2. Checks: the DDP all-reduce leaves identical
gradients on both ranks, equal to the mean of the two ranks' local (non-DDP)
gradients, and the optimizer step keeps the replicas identical."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, cfg_name="kitti"):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.hashrng import hash_init_
    from oracle.torch_ref import OracleCorrelation, oracle_flow_warp, oracle_occu_mask_backward
    from unsamflow_amd.config import kitti_base, sintel_mf
    from unsamflow_amd.harness import TrainStep, synthetic_pair

    # sintel_mf: SURVEY config 5, the mask-feature branch (SAM segments one-hot
    # encoded, pwclite.py:355-357) under DDP, as the reference's Sintel run
    # (train.py:116-120, 228-234)
    cfg = kitti_base() if cfg_name == "kitti" else sintel_mf()
    step = TrainStep(cfg, "cpu", ddp=True, corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp,
                     occ_backward_fn=oracle_occu_mask_backward)
    hash_init_(step.module, seed=3)
    # DDP broadcast happened at construction; re-sync after the deterministic init
    for p in step.module.parameters():
        dist.broadcast(p.data, 0)
    # sintel_mf at its golden-capture size (tests/golden/pwclite_sintel_mf.npz): at 64x128
    # this config's backward has non-finite feature-pyramid gradients even on one
    # process (its coarsest levels shrink to a few pixels), so replicas cannot be compared
    hw = (64, 128) if cfg_name == "kitti" else (128, 256)
    img1, img2, s1, s2 = synthetic_pair(1, *hw, "cpu", seed=100 + rank, with_seg=cfg_name != "kitti")

    # local gradient without communication
    with step.model.no_sync():  # forward AND backward inside: no all-reduce
        loss_local, _ = step.forward_loss(img1, img2, s1, s2)
        loss_local.backward()
    local = [p.grad.detach().clone() for p in step.module.parameters()]
    step.optimizer.zero_grad(set_to_none=True)

    # DDP gradient (all-reduce average)
    loss, _ = step.forward_loss(img1, img2, s1, s2)
    loss.backward()
    ddp = [p.grad.detach().clone() for p in step.module.parameters()]
    torch.save({"local": local, "ddp": ddp}, os.path.join(out_dir, f"rank{rank}.pt"))

    # a full optimizer step keeps the replicas in sync
    step(img1, img2, s1, s2)
    flat = torch.cat([p.detach().reshape(-1) for p in step.module.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1])
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cfg_name", ["kitti", "sintel_mf"])
def test_ddp_two_ranks_gloo(tmp_path, cfg_name):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), cfg_name), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for a, b, l0, l1 in zip(r0["ddp"], r1["ddp"], r0["local"], r1["local"]):
        assert torch.equal(a, b)
        torch.testing.assert_close(a, (l0 + l1) / 2, atol=1e-7, rtol=1e-5)
    assert any(not torch.equal(l0, l1) for l0, l1 in zip(r0["local"], r1["local"]))


def _flat_worker(rank, world, port, out_dir):
    """The graphed multi-GPU step's exchange (harness.FlatGrads): parameters
    broadcast from rank 0, local backward into the flat gradient buffer, ONE
    all-reduce of that buffer, mean -> equals DDP's averaged gradient; then
    clip + Adam keep the replicas identical."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.hashrng import hash_init_
    from oracle.torch_ref import OracleCorrelation, oracle_flow_warp, oracle_occu_mask_backward
    from unsamflow_amd.config import kitti_base
    from unsamflow_amd.harness import FlatGrads, TrainStep, broadcast_params, synthetic_pair

    cfg = kitti_base()
    step = TrainStep(cfg, "cpu", corr_module=OracleCorrelation(4), warp_fn=oracle_flow_warp,
                     occ_backward_fn=oracle_occu_mask_backward, seed=7 + rank)
    hash_init_(step.module, seed=3 + rank)  # replicas differ until the broadcast
    broadcast_params(step.module)
    img1, img2, _, _ = synthetic_pair(1, 64, 128, "cpu", seed=100 + rank)
    grads = FlatGrads(step.module.parameters())
    for _ in range(2):  # the buffer is re-zeroed each step (no stale accumulation)
        grads.zero_()
        loss, _ = step.forward_loss(img1, img2)
        loss.backward()
    local = grads.flat.clone()
    grads.all_reduce_mean()
    torch.save({"local": local, "mean": grads.flat.clone()}, os.path.join(out_dir, f"flat{rank}.pt"))
    torch.nn.utils.clip_grad_norm_(grads.params, step.max_grad_norm)
    step.optimizer.step()
    flat = torch.cat([p.detach().reshape(-1) for p in step.module.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1])
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_flat_gradient_allreduce_two_ranks_gloo(tmp_path):
    world = 2
    mp.spawn(_flat_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "flat0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "flat1.pt", weights_only=True)
    assert torch.equal(r0["mean"], r1["mean"])
    torch.testing.assert_close(r0["mean"], (r0["local"] + r1["local"]) / 2, atol=1e-7, rtol=1e-5)
    assert not torch.equal(r0["local"], r1["local"])
