"""Per-kernel (name, grid) duration stats from a rocprofv3 sqlite results db
(rocprofv3 without --output-format csv). Usage: python tools/r04/dbstats.py <run_results.db> [filter]"""
import collections
import sqlite3
import statistics
import sys

con = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = con.execute(
    "select s.kernel_name, d.grid_size_x, d.grid_size_y, d.grid_size_z, d.end - d.start "
    "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
agg = collections.OrderedDict()
for name, gx, gy, gz, dur in rows:
    n = name.replace("void usf::(anonymous namespace)::", "").split("(")[0]
    if flt and flt not in n:
        continue
    agg.setdefault((n[:70], gx, gy, gz), []).append(dur / 1e3)
for (n, gx, gy, gz), v in agg.items():
    print(f"{n:70s} grid=({gx},{gy},{gz}) n={len(v):4d} med={statistics.median(v):8.2f} min={min(v):8.2f} us")
