"""Cross-check bench.py's roofline timing against rocprofv3.

Reads the JSON line of a bench.py run made under
``USF_ROCTX=1 rocprofv3 --kernel-trace --stats --kernel-rename --marker-trace``
and that run's kernel_stats.csv, where every hot-path launch is listed under
its call-site name (unsamflow_amd.kernel_timer.site_name). Prints, for the
roofline site and every other hot-path site, the bench's in-step event mean
next to rocprof's summed kernel duration per launch of that site (rocprof
also counts the warm-up steps and the untimed per-site pass; a site whose launch runs two kernels -- the
split forward's reduce, the leaky backward's derivative pass, the photometric
final reduction -- is the sum of both).

The profiler inflates the in-step time of two-kernel sites (the gap between
their kernels), so the profiled run's own largest site can differ from the
unprofiled bench's. With a third argument (the unprofiled bench.py line) the
check is made for THAT run's roofline site and also reports its unprofiled
in-step mean.

Usage: python tools/roofline_check.py bench_prof.json run_kernel_stats.csv [bench.json]
"""
import csv
import json
import sys


def main():
    bench = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    stats = {r["Name"]: r for r in csv.DictReader(open(sys.argv[2]))}
    roof = bench["roofline"]
    # every launch rocprof saw: warm-up, bench.py's untimed per-site pass, timed steps
    site_pass = bench.get("site_pass_steps")
    if site_pass is None:  # lines written before the field existed
        site_pass = max(3, min(bench["steps"], 10)) if "site_pass_mean_us" in bench["roofline"] else 0
    steps = bench["steps"] + bench["warmup"] + site_pass
    sites = []
    levels = bench["levels"]
    if levels and isinstance(levels[0], list):  # compact rows (bench.py LEVEL_FIELDS)
        levels = [dict(zip(bench["levels_fields"], r)) for r in levels]
    for row in levels:
        st = stats.get(row["site"])
        entry = {"site": row["site"], "bench_in_step_us": row["in_step_us"], "rocprof_avg_us": None,
                 "rocprof_calls": int(st["Calls"]) if st else None}
        if st:
            launches = row["calls_per_step"] * steps
            entry["kernels_per_launch"] = max(1, round(int(st["Calls"]) / launches))
            entry["rocprof_avg_us"] = round(float(st["TotalDurationNs"]) / 1e3 / launches, 2)
        if st:
            entry["rel_diff"] = round(entry["rocprof_avg_us"] / row["in_step_us"] - 1, 4)
        sites.append(entry)
    out = {}
    if len(sys.argv) > 3:  # the unprofiled run's roofline site and mean
        main_roof = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])["roofline"]
        out["profiled_run_roofline_site"] = roof["site"]
        roof = main_roof
    top = next(e for e in sites if e["site"] == roof["site"])
    out = {"roofline_site": roof["site"], "roofline_mean_us": roof["mean_us"],
           "rocprof_avg_us": top["rocprof_avg_us"],
           "rel_diff": round(top["rocprof_avg_us"] / roof["mean_us"] - 1, 4) if top["rocprof_avg_us"] else None,
           **out, "sites": sites}
    print(json.dumps(out, indent=1))
    return 0 if top["rocprof_avg_us"] is not None else 1


if __name__ == "__main__":
    sys.exit(main())
