"""Print rocprofv3 kernel_stats.csv rows compactly: name (shortened), calls, avg/min us.
Usage: python tools/kstats.py <run_kernel_stats.csv> [...]"""
import csv
import re
import sys

for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(anonymous namespace\)::|usf::|void ", "", r["Name"])
        name = re.sub(r"\((float const\*|float\*|int|usf|long).*", "", name)[:80]
        print(f"{name:80s} {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.2f} min {float(r['MinNs'])/1e3:8.2f}")
