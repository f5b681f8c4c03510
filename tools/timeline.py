"""Busy / idle accounting of the bench's own dispatches from a rocprofv3 kernel trace.

Takes the dispatches after the last k_nl_init (the bench's warm-up, timed and timing-pass
steps; tools/trace_stats.py), and reports for the window between the first and the last of
them: the union of busy intervals (any kernel running), the idle time (no kernel running),
the time two or more kernels overlap, and the largest idle gaps with the kernels either
side.  The bench line's ms_per_step against busy / steps says how much of a step is kernel
boundaries rather than kernels.
  python tools/timeline.py RUN_kernel_trace.csv [STEPS]"""
import csv
import sys


def main():
    with open(sys.argv[1]) as f:
        rows = [r for r in csv.DictReader(f) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_nl_init" in r["Kernel_Name"]]
    rows = rows[starts[-1]:] if starts else rows
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows]
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    # sweep: busy union and >= 2 concurrency
    ev = sorted([(s, 1) for s, _, _ in iv] + [(e, -1) for _, e, _ in iv])
    busy = over = 0
    depth, last = 0, t0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            over += t - last
        depth += d
        last = t
    span = t1 - t0
    print(f"dispatches {len(iv)}  window {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  "
          f"idle {(span - busy) / 1e6:.3f} ms  overlapped {over / 1e6:.3f} ms")
    if len(sys.argv) > 2:
        k = int(sys.argv[2])
        print(f"per step ({k} steps in the window): window {span / 1e6 / k:.3f}  busy {busy / 1e6 / k:.3f}  "
              f"idle {(span - busy) / 1e6 / k:.3f}  overlapped {over / 1e6 / k:.3f} ms")
    # idle gaps
    gaps, end, prev = [], iv[0][1], iv[0][2]
    for s, e, n in iv[1:]:
        if s > end:
            gaps.append((s - end, prev, n))
        if e > end:
            end, prev = e, n
    gaps.sort(reverse=True)
    tot = sum(g for g, _, _ in gaps)
    print(f"idle gaps {len(gaps)}, total {tot / 1e6:.3f} ms; largest:")
    for g, a, b in gaps[:15]:
        print(f"  {g / 1e3:8.1f} us  after {a}  before {b}")
    # idle by the kernel that starts after the gap
    by = {}
    for g, _, b in gaps:
        c = by.setdefault(b, [0, 0])
        c[0] += g
        c[1] += 1
    print("idle before each kernel (total us, gaps):")
    for b, (g, c) in sorted(by.items(), key=lambda x: -x[1][0])[:15]:
        print(f"  {g / 1e3:9.1f} {c:5d}  {b}")


if __name__ == "__main__":
    main()
