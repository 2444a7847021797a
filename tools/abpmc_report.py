"""Summarise tools/gpu_corrab_pmc.sh output: FETCH (x2 calibrated) and WRITE MB per kernel launch shape."""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abpmc"
match = sys.argv[2] if len(sys.argv) > 2 else "corr_bwd"
for lib in sorted(glob.glob(f"{root}/lib_*/")):
    n = os.path.basename(lib.rstrip("/"))
    res = collections.OrderedDict()
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{lib}/{c}/**/run_counter_collection.csv", recursive=True)
        if not f:
            continue
        per = collections.defaultdict(list)
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(f[0])):
            if match not in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"].split("(")[0].split("::")[-1][:50], r["Grid_Size"])
            per[key].append(float(r["Counter_Value"]))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in per.items():
            res.setdefault(k, {})[c] = statistics.median(v)
            res[k]["us"] = statistics.median(dur[k])
    for (kn, g), d in res.items():
        fetch = 2 * d.get("FETCH_SIZE", 0) / 1024
        wr = d.get("WRITE_SIZE", 0) / 1024
        print(f"{n:12s} {kn:50s} grid={g:>8} fetch={fetch:8.1f}MB write={wr:7.1f}MB us={d['us']:.1f}")
