"""Per-kernel statistics of the bench's own steps from a rocprofv3 kernel trace.

rocprofv3 --stats summarises every dispatch of the process, which on a large single-rank
handle includes the basis placement probe at nls_create (NLS_PLACE candidates x 4 steps,
DESIGN.md section 4 "Placement").  The probe's candidates and the bench each start with
k_nl_init (the cold step after a new state), so the dispatches after the LAST k_nl_init
are exactly the bench's warm-up, timed and timing-pass steps.  Prints a CSV in the
--stats layout (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs) over
those dispatches, plus the whole-trace and probe counts on stderr.
  python tools/trace_stats.py RUN_kernel_trace.csv > stats.csv"""
import collections
import csv
import sys


def main():
    with open(sys.argv[1]) as f:
        rows = [r for r in csv.DictReader(f) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_nl_init" in r["Kernel_Name"]]
    first = starts[-1] if starts else 0
    bench = rows[first:]
    print(f"# {len(rows)} dispatches in the trace; {len(starts) - 1 if starts else 0} probe candidates before "
          f"the bench; {len(bench)} bench dispatches from the last k_nl_init", file=sys.stderr)
    acc = collections.defaultdict(list)
    for r in bench:
        acc[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in acc.values())
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), f"{sum(v) / len(v):.1f}", f"{100.0 * sum(v) / total:.3f}", min(v), max(v)])


if __name__ == "__main__":
    main()
