"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc.sh (one row per kernel+grid, median of repeats)."""
import collections
import csv
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
data = collections.OrderedDict()
for i in range(1, 5):
    try:
        rows = list(csv.DictReader(open(f"{root}/p{i}/run_counter_collection.csv")))
    except FileNotFoundError:
        continue
    per = collections.OrderedDict()
    for r in rows:
        k = (r["Kernel_Name"], r["Grid_Size"], r["Workgroup_Size"])
        did = r["Dispatch_Id"]
        per.setdefault(k, {}).setdefault(did, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        per[k][did]["_dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k, ds in per.items():
        agg = data.setdefault(k, {})
        names = set().union(*[d.keys() for d in ds.values()])
        for n in names:
            agg[n] = statistics.median(d[n] for d in ds.values() if n in d)


def short(name):
    name = name.replace("void usf::(anonymous namespace)::", "")
    return name.split("(")[0][:60]


for (name, grid, wg), c in data.items():
    if "usf" not in name and "copyBuffer" not in name:
        continue
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    line = f"{short(name):60s} grid={grid:>8} wg={wg:>4} dur={c.get('_dur_us', 0):7.1f}us"
    if "SQ_WAVES" in c:
        line += (f" waves={c['SQ_WAVES']:.0f} active={c['SQ_ACTIVE_INST_ANY'] / wc:.2f} wait={c['SQ_WAIT_ANY'] / wc:.2f}"
                 f" waitinst={c['SQ_WAIT_INST_ANY'] / wc:.2f} valu={c['SQ_ACTIVE_INST_VALU'] / wc:.2f}"
                 f" lds={c['SQ_ACTIVE_INST_LDS'] / wc:.2f}")
    if "SQ_INSTS_VALU" in c:
        line += (f" | valuI={c['SQ_INSTS_VALU']:.3g} ldsI={c['SQ_INSTS_LDS']:.3g} saluI={c['SQ_INSTS_SALU']:.3g}"
                 f" bankconf={c['SQ_LDS_BANK_CONFLICT']:.3g} waitLDS={c['SQ_WAIT_INST_LDS']:.3g}")
        # effective clock = GRBM_GUI_ACTIVE / 8 XCDs / wall time; the quotient reads
        # high for dispatches under ~0.3 ms (MI355X_MICROARCH.md, DVFS give-back), so
        # it is only printed for longer ones (the r03 report showed 2.4-5.9 "GHz")
        if "GRBM_GUI_ACTIVE" in c and c.get("_dur_us", 0) >= 300:
            line += f" clk={c['GRBM_GUI_ACTIVE'] / 8 / c['_dur_us'] / 1e3:.2f}GHz"
    if "FETCH_SIZE" in c:
        line += f" | FETCH={c['FETCH_SIZE'] / 1024:.1f}MB"
    if "WRITE_SIZE" in c:
        line += f" WRITE={c['WRITE_SIZE'] / 1024:.1f}MB"
    print(line)
