"""Placement diagnosis table (tools/place_diag.sh): the rocprofv3 counter records of
one process split into the placement probe's candidates (each candidate's probe starts
with k_nl_init: the cold step after the reset) and the bench's own steps, then per
segment and kernel family: mean duration and the counters per dispatch, with the
derived average L2->fabric read latency (TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ, cycles) and
fabric bytes per cell.
  python tools/place_diag.py DIR [DIR ...]    (DIR = one pass's output directory)"""
import collections
import csv
import glob
import os
import sys

FAMILIES = [("k_tail", "k_tail<"), ("k_p2d<12>", "k_p2d<12,"), ("k_p2d<0>", "k_p2d<0,"),
            ("k_p2d<6>", "k_p2d<6,"), ("k_alpha_l2", "k_alpha_l2<")]
CELLS = 512 ** 3


def load(d):
    """{dispatch: (name, start, end, {counter: value summed over dimension rows})}"""
    rows = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                i = int(r["Dispatch_Id"])
                e = rows.setdefault(i, [r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), {}])
                e[3][r["Counter_Name"]] = e[3].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return dict(sorted(rows.items()))


def segments(rows):
    segs, cur = [], None
    for i, (name, a, b, c) in rows.items():
        if "k_nl_init" in name:
            cur = []
            segs.append(cur)
        if cur is not None:
            cur.append((name, a, b, c))
    return segs


def main():
    for d in sys.argv[1:]:
        rows = load(d)
        segs = segments(rows)
        print(f"== {d}: {len(segs)} segments (probe candidates, then the bench)")
        ctrs = sorted({k for r in rows.values() for k in r[3]})
        for si, seg in enumerate(segs):
            tag = f"cand{si}" if si < len(segs) - 1 else "bench"
            out = [f"{tag:6s} step-kernels {sum(b - a for _, a, b, _ in seg) / 1e6:8.2f} ms"]
            for fam, pre in FAMILIES:
                ds = [(a, b, c) for n, a, b, c in seg if pre in n.replace(" ", "").replace("nls::", "")]
                if not ds:
                    continue
                ms = sum(b - a for a, b, _ in ds) / len(ds) / 1e6
                cs = {k: sum(c.get(k, 0.0) for _, _, c in ds) / len(ds) for k in ctrs}
                s = f" | {fam} {ms:.3f} ms"
                if cs.get("TCC_EA0_RDREQ") and "TCC_EA0_RDREQ_LEVEL" in cs:
                    s += f" rdlat {cs['TCC_EA0_RDREQ_LEVEL'] / cs['TCC_EA0_RDREQ']:.0f}"
                if cs.get("TCC_EA0_WRREQ") and "TCC_EA0_WRREQ_LEVEL" in cs:
                    s += f" wrlat {cs['TCC_EA0_WRREQ_LEVEL'] / cs['TCC_EA0_WRREQ']:.0f}"
                for k in ctrs:
                    if k.endswith("LEVEL"):
                        continue
                    v = cs[k]
                    s += f" {k} {v / CELLS:.3f}/cell" if k in ("FETCH_SIZE", "WRITE_SIZE") else f" {k} {v:.3g}"
                out.append(s)
            print("".join(out))


if __name__ == "__main__":
    main()
