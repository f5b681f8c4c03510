#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc runs (any counter set),
with the derived fractions this repo uses:
  bytes   read = 2 x FETCH_SIZE x 1 KiB (gfx950 half-counting), write = WRITE_SIZE x 1 KiB
  SQ      ACTIVE_INST_ANY / WAIT_ANY / WAIT_INST_ANY as fractions of SQ_WAVE_CYCLES,
          instructions per wave (SQ_INSTS_* / SQ_WAVES)
usage: tools/pmc_table.py <pmc_dir> [cells] [kernel-regex]"""
import collections
import csv
import glob
import os
import re
import sys


def load(pmc_dir):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    files = glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void nls::", "").replace("nls::", "")
            agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    d = load(sys.argv[1])
    cells = float(sys.argv[2]) if len(sys.argv) > 2 else 512.0 ** 3
    pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    for k in sorted(d):
        if pat and not pat.search(k):
            continue
        c = d[k]
        parts = []
        if "FETCH_SIZE" in c:
            parts.append(f"rd {2 * c['FETCH_SIZE'] * 1024 / cells:7.1f} B/cell")
        if "WRITE_SIZE" in c:
            parts.append(f"wr {c['WRITE_SIZE'] * 1024 / cells:6.1f} B/cell")
        if "TCC_HIT_sum" in c:
            parts.append(f"L2hit {c['TCC_HIT_sum'] / max(c['TCC_HIT_sum'] + c.get('TCC_MISS_sum', 0), 1):.2f}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
                if n in c:
                    parts.append(f"{n[3:].lower()} {c[n] / wc:.2f}")
        if "SQ_LDS_IDX_ACTIVE" in c:
            parts.append(f"lds_bank_conflict/idx_active {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
        wv = c.get("SQ_WAVES")
        if wv:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM"):
                if n in c:
                    parts.append(f"{n[9:].lower()}/wave {c[n] / wv:.0f}")
        if not parts:
            parts = [f"{n} {v:.4g}" for n, v in sorted(c.items())]
        print(f"{k[:60]:60s} " + "  ".join(parts))


if __name__ == "__main__":
    main()
