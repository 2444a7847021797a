"""Markdown per-site table for DESIGN.md §5 from a bench.py line and its PMC
traffic summary: python tools/design_table.py profiles/<tag>_bench.json [profiles/<tag>_pmc_traffic.json]"""
import json
import sys


def main():
    b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    traffic = {}
    if len(sys.argv) > 2:
        for v in json.load(open(sys.argv[2]))["sites"]:
            traffic[(v["op"], tuple(v["shape"]))] = v["traffic_over_algorithmic"]
    rows = [dict(zip(b["levels_fields"], r)) for r in b["levels"]]
    print("| call site (B×C×H×W …) | per step | in-step µs | warm µs | cold µs | HBM frac (cold) | PMC traffic / algorithmic |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        parts = r["site"].split(":")
        op = parts[1]
        shape = [int(x) for x in parts[2].split("x")]
        rest = parts[3:]
        key = None
        for (o, sh), t in traffic.items():
            if o == op and list(sh[:4]) == shape[:4] and [str(x) for x in sh[4:]] == rest[:len(sh) - 4]:
                key = t
        name = f"{op} {parts[2]}" + ("" if not rest else " " + ":".join(rest))
        print(f"| {name} | {r['calls_per_step']:g} | {r['in_step_us']} | {r['device_us']} | {r['cold_us']} | "
              f"{r['hbm_frac']} | {'' if key is None else str(key) + '×'} |")


if __name__ == "__main__":
    main()
