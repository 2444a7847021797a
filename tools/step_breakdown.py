"""Where a PWCLite training step spends GPU time, by phase (CUDA events, B=8,
KITTI 832x256): model fwd, model bwd (given the flow grads), loss fwd+bwd on
detached flows, clip+Adam. Each phase is timed over N repetitions after warmup.

Usage (GPU box): python tools/step_breakdown.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from unsamflow_amd.config import kitti_base  # noqa: E402
from unsamflow_amd.harness import TrainStep, synthetic_pair  # noqa: E402


def timeit(fn, n=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n


def main():
    dev = torch.device("cuda:0")
    st = TrainStep(kitti_base(), dev)
    img1, img2, _, _ = synthetic_pair(8, 256, 832, dev)
    res = {}
    res["full step"] = timeit(lambda: st(img1, img2))
    if os.environ.get("CL") == "1":  # experiment: channels_last model + inputs
        st2 = TrainStep(kitti_base(), dev, channels_last=True)
        c1 = img1.contiguous(memory_format=torch.channels_last)
        c2 = img2.contiguous(memory_format=torch.channels_last)
        res["full step channels_last"] = timeit(lambda: st2(c1, c2))
        del st2

    def model_fwd():
        with torch.no_grad():
            st.model(img1, img2, with_bk=True)
    res["model fwd (no grad)"] = timeit(model_fwd)

    def model_fwd_bwd():
        out = st.model(img1, img2, with_bk=True)
        flows = [torch.cat([a, b], 1) for a, b in zip(out["flows_12"], out["flows_21"])]
        torch.autograd.backward(flows, [torch.ones_like(f) * 1e-3 for f in flows])
    res["model fwd+bwd"] = timeit(model_fwd_bwd)

    out = st.model(img1, img2, with_bk=True)
    flows = [torch.cat([a, b], 1).detach() for a, b in zip(out["flows_12"], out["flows_21"])]

    def loss_fwd():
        with torch.no_grad():
            st.loss_fn(flows, img1, img2)
    res["loss fwd (no grad)"] = timeit(loss_fwd)

    def loss_fwd_bwd():
        fl = [f.clone().requires_grad_() for f in flows]
        loss = st.loss_fn(fl, img1, img2)[0].mean()
        loss.backward()
    res["loss fwd+bwd"] = timeit(loss_fwd_bwd)

    def opt():
        torch.nn.utils.clip_grad_norm_(st.model.parameters(), 10.0)
        st.optimizer.step()
    res["clip + Adam"] = timeit(opt)
    for k, v in res.items():
        print(f"{k:22s} {v:8.2f} ms")


if __name__ == "__main__":
    main()
