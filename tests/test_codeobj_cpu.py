"""CPU: the hand-counted vmcnt schedule of k_p2d holds in the compiled gfx950 code
object (tests/codeobj.py; nls_pass2d.hpp:30-38, p2d_after / wait_step).  For every
k_p2d<J, HZ, D2, PR, A> instantiation: no scratch / buffer / flat access (so no accessed
private segment), no VGPR spill; the march loop issues exactly the source's DMA loads and
stores; and its s_waitcnt vmcnt values are exactly the source's p2d_after values."""
import os

import pytest

import codeobj as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "nonlinear-solvers_amd", "lib", "libnls_amd.so")
HDR = os.path.join(ROOT, "nonlinear-solvers_amd", "csrc", "nls_pass2d.hpp")

pytestmark = pytest.mark.skipif(not (C.available() and os.path.exists(LIB)),
                                reason="ROCm llvm tools or the built library missing")


@pytest.fixture(scope="module")
def p2d_results(tmp_path_factory):
    sched = C.P2dSchedule(HDR)
    out = []
    for co in C.gfx950_objects(LIB, str(tmp_path_factory.mktemp("co"))):
        funcs = C.disassemble(co)
        if any(C.p2d_params(n) for n in funcs):
            out += C.check_p2d(funcs, C.metadata(co), sched)
    return out


def test_every_p2d_instantiation_found(p2d_results):
    got = {(r["J"], r["HZ"], r["D2"], r["PR"], r["A"]) for _n, _p, r in p2d_results}
    want = {(J, hz, d2, pr, 0) for J in range(0, 16, 2) for hz in (0, 1) for d2, pr in ((0, 0), (1, 0), (1, 1))}
    want |= {(J, hz, 0, 0, 1) for J in range(0, 24, 2) for hz in (0, 1)}  # the G2 operator (nls_pass2a.hip)
    want |= {(J, hz, 0, 1, 2) for J in range(0, 16, 2) for hz in (0, 1)}  # G2 on real cell pairs (Klein-Gordon)
    assert got == want


def test_p2d_vmcnt_contract_holds(p2d_results):
    bad = [(r["J"], r["HZ"], r["D2"], r["PR"], r["A"], p) for _n, p, r in p2d_results if p]
    assert not bad, bad


def test_checker_flags_an_extra_vmem_op():
    """The loop check is not vacuous: one more load in a synthetic loop body fails it
    (a J-ring pass: J = 12, 2 S rows + 12 J rows per step, 2 halo pieces, 2 stores)."""
    sched = C.P2dSchedule(HDR)
    J = 12
    assert not sched.jreg(J)
    name = f"_ZN3nls5k_p2dILi{J}ELb1ELb0ELb0ELb0EEEv"
    waits = [(0x0f0 + 4 * i, "s_waitcnt", f"vmcnt({w})") for i, w in enumerate(sched.waits(J, 2))]
    body = waits + \
        [(0x104 + 4 * i, "global_load_lds_dwordx4", "v[2:3], off") for i in range(2 + J)] + \
        [(0x180, "global_load_lds_dword", ""), (0x184, "global_load_lds_dword", ""),
         (0x188, "global_store_dwordx4", ""), (0x18c, "global_store_dwordx4", ""),
         (0x190, "s_cbranch_scc1", f"<{name}+0x0f0>")]
    ins = [(0x0, "s_load_dwordx2", "")] + body
    md = {name: {"private_segment_fixed_size": "0", "vgpr_spill_count": "0"}}
    assert C.check_p2d({name: ins}, md, sched)[0][1] == []
    extra = ins[:-1] + [(0x18e, "scratch_load_dword", "v1, off"), ins[-1]]
    probs = C.check_p2d({name: extra}, md, sched)[0][1]
    assert probs and any("scratch" in p for p in probs)


def test_register_row_kinds():
    """Kind 3 (the isotropic 2D passes) follows kind 0's ring rules except where its
    register rows start: 3D from J = 2, 2D from J = 8 (nls_pass2d.hpp p2d_kind / p2d_jreg);
    the code-object check above reads the instantiations through the same rules."""
    s = C.P2dSchedule(HDR)
    assert [J for J in range(0, 15, 2) if s.jreg(J, 0)] == [J for J in range(s.JREG_MINJ, s.JREG_MAXJ + 1, 2)]
    assert [J for J in range(0, 15, 2) if s.jreg(J, 3)] == [J for J in range(s.JREG2D_MINJ, s.JREG_MAXJ + 1, 2)]
    assert s.JREG2D_MINJ > s.JREG_MINJ
    for J in range(0, 15, 2):
        if s.jreg(J, 0) == s.jreg(J, 3):  # same storage form: identical schedule
            assert (s.occ(J, 0), s.ds(J, 0), s.np(J, 0), s.early(J, 0)) == (s.occ(J, 3), s.ds(J, 3), s.np(J, 3),
                                                                         s.early(J, 3))
            assert s.waits(J, 2, 0) == s.waits(J, 2, 3)
        else:  # 3D register rows, 2D J ring
            assert s.np(J, 0) == 0 and s.np(J, 3) >= 1


def test_new_round6_kernels_have_no_scratch(tmp_path):
    """The round-6 kernels (the fused column-sum + coefficient launch, the fused basis end,
    the four-vector first passes k_p4d0 and k_p4r) keep everything in registers and LDS: no VGPR spill, no
    scratch instruction, and no private segment beyond the call frame of the eigensolve
    (k_tail_chain calls eigen_phase_jacobi, __noinline__, exactly as k_reduce_final does)."""
    want = ("k_colsum_p2coef", "k_tail_chain", "k_p4d0", "k_p4r")
    seen = set()
    for co in C.gfx950_objects(LIB, str(tmp_path)):
        md = C.metadata(co)
        funcs = C.disassemble(co)
        frame = [int(v.get("private_segment_fixed_size", "0")) for n, v in md.items() if "k_reduce_final" in n]
        for name, ins in funcs.items():
            hit = [w for w in want if w in name]
            if not hit:
                continue
            seen.add(hit[0])
            meta = md.get(name, {})
            allowed = max(frame) if hit[0] == "k_tail_chain" and frame else 0
            assert int(meta.get("private_segment_fixed_size", "0")) <= allowed, name
            assert str(meta.get("vgpr_spill_count", "0")) == "0", name
            assert not [m for _a, m, _o in ins if m.startswith("scratch_")], name
    assert seen == set(want)
