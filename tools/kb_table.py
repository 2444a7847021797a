"""Print a kbench JSON as one row per (op, shape): default time and per-variant times (us)."""
import json
import sys
from collections import defaultdict

rows = defaultdict(dict)
for r in json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kbench.json")):
    rows[(r["op"], tuple(r["shape"]))][r.get("variant", "-")] = r["us"]
for (op, shape), v in rows.items():
    d = v.pop(-1, v.pop("-", None))
    alts = " ".join(f"v{k}={t:.1f}" for k, t in sorted(v.items()))
    print(f"{op:9s} {str(shape):42s} default={d:7.2f}  {alts}")
