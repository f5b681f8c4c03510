#!/usr/bin/env python3
"""Format the parity records the GPU tests append to $NLS_PARITY_LOG
(conftest.record_parity) as a table: per case and checkpoint the GPU error
against the oracle, the oracle's self-floor (one-ulp perturbed u0), the numpy
twin's distance to the oracle, the test's bound and the GPU / self-floor ratio.

  python tools/parity_floor.py gpurun_out/parity.jsonl > profiles/r03/parity_floor.txt
"""
import json
import sys


def fmt(v):
    return "-" if v is None else f"{v:.2e}"


def main(path):
    cases = []
    with open(path) as f:
        for ln in f:
            if ln.strip():
                cases.append(json.loads(ln))
    print("# GPU error vs the oracle, the oracle's self-floor and the numpy twin, per checkpoint")
    print("# self-floor: max over two seeds of rel-L2(oracle(u0 + 1 ulp noise), oracle(u0))")
    print("# propagated: rel-L2(oracle continued from the GPU's step-1 field, oracle) -- the GPU's first-step")
    print("#   deviation as the reference algorithm amplifies it (2D stiff NLSE cases)")
    print("# bound: max(1e-10, 32 x self-floor) where the test allows the floor (and <= 4 x propagated), else 1e-10")
    worst = 0.0
    for c in cases:
        print(f"\n## {c['case']}")
        print(f"{'checkpoint':>10} {'gpu_err':>10} {'self_floor':>10} {'twin':>10} {'propagated':>10} {'bound':>9} "
              f"{'gpu/self':>9} {'gpu/prop':>9}")
        for r in c["rows"]:
            rat = r.get("ratio_gpu_self")
            if rat is not None and r["self_floor"] > 1e-12:
                worst = max(worst, rat)
            pr = r.get("propagated")
            rp = (r["gpu_err"] / pr) if pr else None
            print(f"{r['checkpoint']:>10} {fmt(r['gpu_err']):>10} {fmt(r['self_floor']):>10} "
                  f"{fmt(r['twin_floor']):>10} {fmt(pr):>10} {fmt(r['bound']):>9} "
                  f"{('-' if rat is None else f'{rat:.2f}'):>9} {('-' if rp is None else f'{rp:.2f}'):>9}")
    print(f"\n# largest gpu/self-floor ratio where the self-floor exceeds 1e-12: {worst:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
