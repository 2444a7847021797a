"""HBM traffic per launch of each hot-path call site from rocprofv3 PMC passes.

Input: the FETCH_SIZE and WRITE_SIZE passes of tools/gpu_pmc.sh over
tools/kprof.py (each its own rocprofv3 --pmc run with --kernel-trace only).
kprof.py launches, in order: a 256 MiB device copy (n times, calibration),
then every site of kprof.SITES n times, each launch behind a separator kernel
(kprof.SEPARATOR); the usf:: dispatches between two separators are one launch,
however many kernels it runs. The summary carries the library's build id
(usf_build_id): bench.py only takes a traffic figure measured on the build it
has loaded.

Correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE under-reports
wide streaming reads by 2x on gfx950 and other access widths are uncalibrated,
so both counters are scaled by the factor that makes the calibration copy
read / write exactly its 268,435,456 bytes. Output: JSON with, per site,
fetch/write KiB (median over launches), corrected traffic bytes per launch and
the algorithmic bytes for comparison.

Usage: python tools/pmc_traffic.py gpurun_out/pmc > profiles/rNN_pmc_traffic.json
"""
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

COPY_BYTES = 64 * 1024 * 1024 * 4


def per_dispatch(path, counter):
    rows = list(csv.DictReader(open(path)))
    d = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        did = int(r["Dispatch_Id"])
        d.setdefault(did, [r["Kernel_Name"], 0.0])
        d[did][1] += float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def launches(rows, nsites, n):
    """Cut the dispatch list at the separator kernels (tools/kprof.py): per
    site n launches, each the list of (kernel, value) of its usf:: kernels."""
    from kprof import SEPARATOR

    seps = [i for i, (name, _) in enumerate(rows) if SEPARATOR in name]
    if len(seps) != nsites * (n + 1):
        raise SystemExit(f"expected {nsites * (n + 1)} separator dispatches, found {len(seps)}")
    out = []
    for s in range(nsites):
        base = s * (n + 1)
        out.append([[(name, v) for name, v in rows[seps[base + j] + 1:seps[base + j + 1]] if "usf::" in name]
                    for j in range(n)])
    return out


def short(name):
    """Kernel name without return type, namespaces and argument list."""
    n = name.replace("void ", "", 1).replace("usf::(anonymous namespace)::", "").replace("usf::", "")
    return n.split("(")[0]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    from kprof import selected_sites
    from unsamflow_amd import _lib
    from unsamflow_amd.kernel_timer import corr_bytes, warp_bytes

    n = int(os.environ.get("KPROF_N", "3"))
    fetch = per_dispatch(f"{root}/p3/run_counter_collection.csv", "FETCH_SIZE")
    write = per_dispatch(f"{root}/p4/run_counter_collection.csv", "WRITE_SIZE")

    def calib(rows):
        from kprof import SEPARATOR

        copies = [v for name, v in rows if "copy" in name.lower() and SEPARATOR not in name][:n]
        return COPY_BYTES / (statistics.median(copies) * 1024)

    f_read, f_write = calib(fetch), calib(write)
    sites_list = selected_sites()
    lf, lw = launches(fetch, len(sites_list), n), launches(write, len(sites_list), n)
    lib = _lib.load()  # host-only queries (no GPU work)
    sites = []
    for (op, key), fl, wl in zip(sites_list, lf, lw):
        fk = statistics.median(sum(v for _, v in launch) for launch in fl)
        wk = statistics.median(sum(v for _, v in launch) for launch in wl)
        # per kernel of the launch (median over the launches), in launch order
        names = [short(k) for k, _ in fl[0]]
        per_kernel = [{"kernel": nm,
                       "fetch_kib": round(statistics.median(launch[i][1] for launch in fl if len(launch) > i), 1),
                       "write_kib": round(statistics.median(launch[i][1] for launch in wl if len(launch) > i), 1)}
                      for i, nm in enumerate(names)]
        if op in ("convex_pyr", "convex_pyr_bwd"):
            B, f = key[0], key[-1]
            hw = [(key[i], key[i + 1]) for i in range(1, len(key) - 1, 2)]
            H, W = hw[0]
        elif op in ("photo_pyr_grad", "photo_pyr_bwd"):
            B, C = key[:2]
            hw = [(key[i], key[i + 1]) for i in range(2, len(key) - (op == "photo_pyr_grad"), 2)]
            H, W = hw[0]
        elif op == "photo_bwd":
            B, ndir, H, W = key
        elif op.startswith("convex_up"):
            B, H, W, f = key
        else:
            B, C, H, W = key[:4]
        if op.startswith("corr"):
            alg = corr_bytes(*key[:4], backward=op.startswith("corr_bwd"))
            if op in ("corr_bwd_leaky", "corr_fwd_leaky"):
                # the sign mask: written by the decoder's forward, read by its backward
                alg += 8 * lib.usf_corr_act_mask_words(B, H, W, 4)
        elif op == "convex_up":
            alg = 4 * B * H * W * (2 + 11 * f * f)
        elif op == "convex_up_bwd":
            alg = 4 * B * H * W * (4 + 20 * f * f)
        elif op == "warp_fwd":
            alg = warp_bytes(*key[:4])
        elif op == "warp_fwd_up":  # + the [B,2,H/2,W/2] coarse flow read (the upsampled flow written instead of read)
            alg = warp_bytes(*key[:4]) + 4 * B * 2 * (H // 2) * (W // 2)
        elif op == "warp_bwd":
            alg = warp_bytes(*key[:4], True, key[5], key[6])
        elif op == "area_pyramid":
            alg = int(4 * B * C * H * W * (1 + 1 / 4 + 1 / 16 + 1 / 64))
        elif op == "occ_bwd":
            alg = 4 * B * H * W * 3  # flow in, mask out (ops.occ_backward)
        elif op == "occ_vis_pair":
            alg = 4 * B * H * W * 6  # 4-channel flow in, two masks out (ops.occ_vis_pair)
        elif op == "photo_fwd":
            alg = 4 * B * H * W * (2 * C + 3)
        elif op == "photo_fwd_grad":
            alg = 4 * B * H * W * (2 * C + 7)  # + the [B,4,H,W] gradient basis written
        elif op == "photo_pair_grad":
            # both directions, every input read once: im1, im2, flow4,
            # both masks; the 8 basis planes written once (ops.photo_loss_pair_forward)
            alg = 4 * B * H * W * (2 * C + 4 + 2 + 8)
        elif op == "convex_pyr":
            alg = sum(4 * B * h * w * (2 + 11 * f * f) for h, w in hw)
        elif op == "convex_pyr_bwd":
            alg = sum(4 * B * h * w * (4 + 20 * f * f) for h, w in hw)
        elif op == "photo_pyr_grad":  # every scale's photo_pair_grad bytes
            alg = sum(4 * B * h * w * (2 * C + 4 + 2 + 8) for h, w in hw)
        elif op == "photo_pyr_bwd":  # basis in, grad_flow out, both directions per scale
            alg = sum(4 * B * h * w * 12 for h, w in hw)
        else:
            alg = 4 * B * H * W * 6 * ndir  # photo_bwd: basis in, grad_flow out
        traffic = fk * 1024 * f_read + wk * 1024 * f_write
        row = {"op": op, "shape": list(key), "fetch_kib": round(fk, 1), "write_kib": round(wk, 1),
               "read_bytes": int(fk * 1024 * f_read), "write_bytes": int(wk * 1024 * f_write),
               "traffic_bytes": int(traffic), "algorithmic_bytes": int(alg),
               "traffic_over_algorithmic": round(traffic / alg, 3), "kernels": per_kernel}
        if op == "photo_pair_grad":  # reads against the read-once minimum (48 B/px at C = 3)
            row["read_once_bytes"] = 4 * B * H * W * (2 * C + 4 + 2)
            row["read_over_read_once"] = round(row["read_bytes"] / row["read_once_bytes"], 3)
        sites.append(row)
    print(json.dumps({"build_id": lib.usf_build_id().decode(),
                      "calibration": {"copy_bytes": COPY_BYTES, "fetch_scale": round(f_read, 4),
                                      "write_scale": round(f_write, 4), "launches_per_site": n},
                      "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-trace only) "
                                "over tools/kprof.py, scaled by a 256 MiB copy calibration",
                      "sites": sites}, indent=1))


if __name__ == "__main__":
    main()
