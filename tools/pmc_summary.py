#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs of bench.py into profiles/pmc_<workload>.json.

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE reads exactly half of the bytes of
a wide coalesced streaming read on gfx950, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  FETCH_SIZE and WRITE_SIZE
are collected in separate passes (tools/pmc_run.sh).

usage: tools/pmc_summary.py <pmc_dir> <workload> <m> <cells> [out.json] [dominant-kernel-prefix] [u_share]
The dominant kernel is the one bench.py's roofline names (its "kernel" field):
k_tail<..., m, ...> or, with the two-vector passes, k_p2d<J, ...>; pass its
prefix (e.g. "k_p2d<12") to pick a pass, else the fused tail is taken.  u_share:
the fraction of the NLSE tail launches that also wrote u (only the last step of an
nls_step call does; tools/profile_round.sh's PMC runs: 2 of 7), default 1.
"""
import collections
import csv
import json
import os
import re
import sys


def load(pmc_dir):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in sorted(os.listdir(pmc_dir)):
        f = os.path.join(pmc_dir, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void nls::", "").replace("nls::", "")
            agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    pmc_dir, workload, m, cells = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join("profiles", f"pmc_{workload}.json")
    d = load(pmc_dir)
    J = m - 2
    esz = 8 if workload.startswith("sg") else 16
    kernels = {}
    for name, c in sorted(d.items()):
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        rd = 2.0 * c["FETCH_SIZE"] * 1024
        wr = c["WRITE_SIZE"] * 1024
        e = {"read_bytes": rd, "write_bytes": wr, "bytes_per_cell": (rd + wr) / cells}
        if "TCC_HIT_sum" in c:
            h, mi = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
            e["l2_hit_rate"] = h / max(h + mi, 1)
        kernels[name] = e
    # dominant kernel: the fused final pass when the step has one, else k_update<m-2>;
    # a k_p2d<J> pass when asked for
    want = sys.argv[6] if len(sys.argv) > 6 and sys.argv[6] not in ("", "-") else None
    dom, alg = None, None
    if want and want.startswith("k_p2d<"):
        J = int(re.search(r"k_p2d<(\d+)", want).group(1))
        dom = next((k for k in kernels if k.startswith(f"k_p2d<{J}, ")), None)
        hz = dom is not None and dom.endswith("true>")
        alg = (J + 1 + (2 if hz else 1)) * esz * cells
    if dom is None:
        dom = next((k for k in kernels if re.fullmatch(rf"k_tail<(nls::)?cplx, [23], {m}, (true|false), 0>", k)), None)
        alg = (m + (float(sys.argv[7]) if len(sys.argv) > 7 else 1.0)) * esz * cells
    if dom is None:
        dom = next((k for k in kernels if re.fullmatch(rf"k_update<[^,]*, [23], {J}(, (true|false))?>", k)), None)
        alg = (J + 2) * esz * cells
    res = {
        "workload": workload, "m": m, "cells": cells,
        "dominant_kernel": dom,
        "bytes_per_launch": (kernels[dom]["read_bytes"] + kernels[dom]["write_bytes"]) if dom else None,
        "algorithmic_bytes_per_launch": alg,
        "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-counting of wide streaming reads); "
                      "write = WRITE_SIZE x 1024; separate --pmc passes",
        "kernels": kernels,
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("dominant_kernel", "bytes_per_launch", "algorithmic_bytes_per_launch")}))


if __name__ == "__main__":
    main()
