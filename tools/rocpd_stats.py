#!/usr/bin/env python3
"""Per-kernel statistics (calls, total / average / min / max ms) from a rocprofv3
SQLite output (rocpd *_results.db), the same columns as --stats' kernel_stats.csv.

  python tools/rocpd_stats.py gpurun_out/prof/x_results.db [> profiles/r03/x_kernel_stats.csv]
"""
import sqlite3
import sys
from collections import defaultdict


def main(db):
    c = sqlite3.connect(db)
    names = {kid: (disp or name) for kid, name, disp in
             c.execute("select id, kernel_name, display_name from rocpd_info_kernel_symbol")}
    agg = defaultdict(list)
    for kid, st, en in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        agg[names.get(kid, str(kid))].append((en - st) * 1e-6)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    tot = sum(sum(v) for _, v in rows)
    print('"Name","Calls","TotalDurationMs","AverageMs","MinMs","MaxMs","Percentage"')
    for n, v in rows:
        print(f'"{n}",{len(v)},{sum(v):.4f},{sum(v) / len(v):.4f},{min(v):.4f},{max(v):.4f},{100 * sum(v) / tot:.2f}')


if __name__ == "__main__":
    main(sys.argv[1])
