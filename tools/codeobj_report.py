#!/usr/bin/env python3
"""Per k_p2d instantiation: VGPR / AGPR / SGPR (spills), LDS and private segment
from the gfx950 code object's metadata, the march loop's VMEM operations and
s_waitcnt vmcnt values, and the contract check of tests/codeobj.py.

  python tools/codeobj_report.py > profiles/r03/k_p2d_codeobj.txt
"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import codeobj as C  # noqa: E402


def main():
    lib = os.path.join(ROOT, "nonlinear-solvers_amd", "lib", "libnls_amd.so")
    sched = C.P2dSchedule(os.path.join(ROOT, "nonlinear-solvers_amd", "csrc", "nls_pass2d.hpp"))
    rows = []
    with tempfile.TemporaryDirectory() as wd:
        for co in C.gfx950_objects(lib, wd):
            funcs = C.disassemble(co)
            if any(C.p2d_params(n) for n in funcs):
                rows += C.check_p2d(funcs, C.metadata(co), sched)
    print("# k_p2d<J, HZ, D2, PR> in libnls_amd.so (gfx950): resources and the vmcnt contract")
    print("# loop VMEM: static count in the march loop (DMA rows x4 / halo pieces / stores; stores may")
    print("# appear once per full/ragged-tile branch); vmcnt: waits in the loop == p2d_after")
    print(f"{'J':>2} {'HZ':>2} {'D2':>2} {'PR':>2} {'vgpr':>4} {'agpr':>4} {'sgpr':>4} {'spill_s':>7} {'spill_v':>7} "
          f"{'lds':>6} {'priv':>4} {'dwordx4':>7} {'dword':>5} {'store':>5} {'vmcnt':>10} {'insns':>5}  check")
    for _n, probs, r in sorted(rows, key=lambda t: (t[2]["J"], t[2]["HZ"], t[2]["D2"], t[2]["PR"])):
        v = r["loop_vmem"]
        print(f"{r['J']:>2} {r['HZ']:>2} {r['D2']:>2} {r['PR']:>2} {r['vgpr']:>4} {r['agpr']:>4} {r['sgpr']:>4} "
              f"{r['sgpr_spill']:>7} {r['vgpr_spill']:>7} {r['lds']:>6} {r['private']:>4} "
              f"{v.get('global_load_lds_dwordx4', 0):>7} {v.get('global_load_lds_dword', 0):>5} "
              f"{v.get('global_store_dwordx4', 0):>5} {','.join(map(str, r['loop_vmcnt_waits'])):>10} "
              f"{r['loop_instructions']:>5}  {'ok' if not probs else '; '.join(probs)}")


if __name__ == "__main__":
    main()
