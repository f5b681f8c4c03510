"""Static checks on the gfx950 code object of libnls_amd.so (test infrastructure;
tests/test_codeobj_cpu.py, tools/codeobj_report.py).

k_p2d (nonlinear-solvers_amd/csrc/nls_pass2d.hpp:30-38, p2d_after / wait_step) counts
the completion of its LDS-DMA loads by hand: `s_waitcnt vmcnt(N)` with N a
compile-time count of the VMEM operations the wave issued after the one a step
needs.  That holds only if every VMEM operation in the march loop is one the
source issues.  A scratch access (register spill, a lambda capture kept on the
stack) or any other global load/store the compiler adds would shift the counts
and turn into stale LDS reads -- wrong numbers, not a fault.  These helpers
disassemble the code object with ROCm's llvm-objdump and read the kernel
metadata with llvm-readelf.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
OBJDUMP = os.path.join(LLVM, "llvm-objdump")
READELF = os.path.join(LLVM, "llvm-readelf")

_INS = re.compile(r"^\s+([a-z_0-9]+)\b(.*?)//\s*([0-9A-Fa-f]+):(.*)$")
_TGT = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
_SYM = re.compile(r"^([0-9a-f]+) <([^>]+)>:")
VMEM_PREFIX = ("global_", "buffer_", "scratch_", "flat_")


def available() -> bool:
    return os.path.exists(OBJDUMP) and os.path.exists(READELF)


def gfx950_objects(lib_path: str, workdir: str | None = None) -> list[str]:
    """Extract the gfx950 code objects of a HIP shared library (llvm-objdump
    --offloading writes them next to its input, so it runs on a copy)."""
    wd = workdir or tempfile.mkdtemp(prefix="nls_co_")
    dst = os.path.join(wd, os.path.basename(lib_path))
    shutil.copyfile(lib_path, dst)
    subprocess.run([OBJDUMP, "--offloading", dst], check=True, capture_output=True, cwd=wd)
    return sorted(os.path.join(wd, f) for f in os.listdir(wd) if f.endswith("gfx950"))


def disassemble(co: str) -> dict[str, list[tuple[int, str, str]]]:
    """{symbol: [(address, mnemonic, operands)]} of every function in a code object."""
    out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                         text=True).stdout
    funcs, cur = {}, None
    for ln in out.splitlines():
        m = _SYM.match(ln)
        if m:
            cur = m.group(2)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _INS.match(ln)
        if m:
            # operands, then the branch target objdump adds in the comment (<sym+0xOFF>)
            tgt = _TGT.search(m.group(4))
            funcs[cur].append((int(m.group(3), 16), m.group(1),
                               m.group(2).strip() + (f" <{tgt.group(1)}+0x{tgt.group(2)}>" if tgt else "")))
    return funcs


def metadata(co: str) -> dict[str, dict[str, str]]:
    """{kernel name: {key: value}} of the scalar amdhsa kernel metadata fields."""
    out = subprocess.run([READELF, "--notes", co], check=True, capture_output=True, text=True).stdout
    kernels, cur, indent = {}, None, None
    for ln in out.splitlines():
        m = re.match(r"^(\s*)- \.agpr_count:\s*(\S+)", ln)
        if m and (indent is None or len(m.group(1)) == indent):
            indent = len(m.group(1))
            cur = {"agpr_count": m.group(2)}
            continue
        if cur is None:
            continue
        m = re.match(r"^(\s*)\.([a-z_]+):\s*(\S+)\s*$", ln)
        if m and len(m.group(1)) == indent + 2:
            cur[m.group(2)] = m.group(3)
            if m.group(2) == "name":
                kernels[m.group(3)] = cur
    return kernels


def main_loop(ins: list[tuple[int, str, str]], fname: str) -> list[tuple[int, str, str]]:
    """The instructions of the widest backward-branch span (the march loop; the
    compiler rotates/peels it, so the span runs from the earliest target of a
    backward branch inside the last such region to the last backward branch)."""
    if not ins:
        return []
    base = ins[0][0]  # objdump prints branch targets as <symbol+0xOFF>
    spans = []
    for addr, mn, ops in ins:
        if not mn.startswith("s_branch") and not mn.startswith("s_cbranch"):
            continue
        m = _TGT.search(ops)
        if not m or m.group(1) != fname:
            continue
        tgt = base + int(m.group(2), 16)
        if tgt <= addr:
            spans.append((tgt, addr))
    if not spans:
        return []
    lo, hi = max(spans, key=lambda s: s[1] - s[0])
    # merge the backward branches that overlap the widest span (rotated loops)
    for a, b in spans:
        if a <= hi and b >= lo:
            lo, hi = min(lo, a), max(hi, b)
    return [i for i in ins if lo <= i[0] <= hi]


_P2D = re.compile(r"k_p2dILi(\d+)ELb([01])ELb([01])ELb([01])ELb([01])E")


def p2d_params(name: str):
    """(J, HZ, D2, PR, A) of a mangled k_p2d<J, HZ, D2, PR, A> symbol, else None."""
    m = _P2D.search(name)
    return tuple(int(g) for g in m.groups()) if m else None


def vmem_counts(ins) -> dict[str, int]:
    c = {}
    for _a, mn, _o in ins:
        if mn.startswith(VMEM_PREFIX):
            c[mn] = c.get(mn, 0) + 1
    return c


def p2d_loop_loads(J: int, A: int = 0, jreg: bool = False) -> dict[str, int]:
    """VMEM loads of one march step as the source issues them: 2 S rows (1 KiB each
    + a 4-byte halo piece on 16 lanes), with A = 1 the two c rows (one 16-B DMA + one
    4-byte halo piece), with A = 2 (cell pairs) two c rows staged as S rows are, and
    the J rows (J-ring DMAs, or with jreg register loads)."""
    ca = {0: (0, 0), 1: (1, 1), 2: (2, 2)}[A]
    d = {"global_load_lds_dwordx4": 2 + (0 if jreg else J) + ca[0], "global_load_lds_dword": 2 + ca[1]}
    if jreg:
        d["global_load_dwordx4"] = J
    return d


class P2dSchedule:
    """Python restatement of nls_pass2d.hpp's ring/wait constexprs (p2d_occ, p2d_ds,
    p2d_early, p2d_np, p2d_after's issue replay, p2d_i0), with the tuning macros'
    defaults read from the header itself so that the two cannot drift apart."""

    def __init__(self, header: str):
        src = open(header).read()

        def define(name):
            return int(re.search(rf"#define {name} (\d+)", src).group(1))

        def const(name):
            return int(eval(re.search(rf"constexpr int {name} = ([^;]+);", src).group(1),
                            {"P2D_TR": self.TR, "P2D_SR": 8, "P2D_CRB": 512, "__builtins__": {}}))
        self.OCC0, self.OCC2 = define("NLS_P2D_OCC0"), define("NLS_P2D_OCC2_MAXJ")
        self.OCC2A, self.EARLYA, self.DS1A = define("NLS_P2A_OCC2_MAXJ"), define("NLS_P2A_EARLY"), define("NLS_P2A_DS1")
        self.DS2, self.DS3 = define("NLS_P2D_DS2_MAXJ"), define("NLS_P2D_DS3_MAXJ")
        self.DS2O = define("NLS_P2D_DS2O_MAXJ")
        self.EARLY, self.NPMAX = define("NLS_P2D_EARLY"), define("NLS_P2D_NP_MAX")
        self.PRE_LA = define("NLS_P2D_PRE_LA")
        self.RF = define("NLS_P2D_RF")
        self.JPF = define("NLS_P2D_JPF_MAXJ")
        self.JREG = define("NLS_P2D_JREG")
        self.JREG_MINJ, self.JREG_MAXJ = define("NLS_P2D_JREG_MINJ"), define("NLS_P2D_JREG_MAXJ")
        self.JREG2D_MINJ = define("NLS_P2D_JREG2D_MINJ")
        self.JREGA_MINJ, self.JREGA_MAXJ = define("NLS_P2A_JREG_MINJ"), define("NLS_P2A_JREG_MAXJ")
        self.OCC2A2 = define("NLS_P2A2_OCC2_MAXJ")
        self.EXT1 = define("NLS_P2D_EXT1")
        self.SR, self.SRB, self.LR = const("P2D_SR"), const("P2D_SRB"), const("P2D_LR")
        self.CSB = const("P2D_CSB")
        self.LDS = 160 * 1024

    TR = 4

    @staticmethod
    def kind(A):
        """p2d_kind: kind 3 (the isotropic 2D passes) is kind 0 except for p2d_jreg."""
        return 0 if A == 3 else A

    def jreg(self, J, A=0):
        """J rows loaded into registers (no J ring)."""
        if not self.JREG:
            return False
        if A == 0:
            return self.JREG_MINJ <= J <= self.JREG_MAXJ
        if A == 3:
            return self.JREG2D_MINJ <= J <= self.JREG_MAXJ
        if A == 1:
            return self.JREGA_MINJ <= J <= self.JREGA_MAXJ
        return 0 < J <= self.OCC2A2

    def occ(self, J, A=0):
        if A == 1:
            return 2 if (J <= self.OCC2A or self.jreg(J, A)) else 1
        if A == 2:
            return 2 if J <= self.OCC2A2 else 1
        return self.OCC0 if J == 0 else (2 if J <= self.OCC2 or self.jreg(J, A) else 1)

    def ds(self, J, A=0):
        o = self.occ(J, A)
        if self.kind(A):
            return (2 if J == 0 and A == 1 else 1) if o == 2 else (3 if J <= self.DS3 else (1 if J >= 22 else self.DS1A))
        if o >= 3:
            return 1
        if o == 2:
            return 3 if J == 0 else (2 if J <= self.DS2 else 1)
        if J == 0:
            return 6
        if J <= self.DS3:
            return 3
        if J <= self.DS2O:
            return 2
        return 1 if (J <= 12 or not self.EARLY) else 0

    def early(self, J, A=0):
        if self.kind(A):
            return bool(self.EARLYA) and self.occ(J, A) == 1 and J < 22
        return bool(self.EARLY) and self.occ(J, A) == 1

    def np(self, J, A=0):
        if J == 0 or self.jreg(J, A):
            return 0
        nsl = self.ds(J, A) + 3 + (1 if self.early(J, A) else 0)
        csb = self.SR * self.SRB if A == 2 else (self.CSB if self.kind(A) else 0)
        ocp2 = A == 2 and self.occ(J, A) == 2  # no EXT1 x-halo area, coefficients in registers
        lxb = 0 if (ocp2 or not self.EXT1) else 2 * self.TR * 2 * 16  # P2D_LXB
        off_j = nsl * self.SR * self.SRB + nsl * csb + 2 * self.LR * 1024 + lxb
        avail = self.LDS // self.occ(J, A) - off_j - (0 if ocp2 else 2 * (J + 1) * 16)
        return min(avail // (self.TR * 1024 * J), self.NPMAX)

    def late(self, J, A=0):
        return J > 0 and self.np(J, A) == 1

    def jpf(self, J, A=0):
        """Register-row pass with plane k+1's rows loaded one step ahead (p2d_jpf)."""
        return self.jreg(J, A) and self.kind(A) == 0 and J <= self.JPF

    def rf(self, J, A=0):
        """J slot refilled with plane k + NP right after its rows are read (p2d_rf)."""
        return bool(self.RF) and self.kind(A) == 0 and J > 0 and not self.jreg(J, A) and self.np(J, A) >= 2

    def nsl(self, J, A=0):
        return self.ds(J, A) + 3 + (1 if self.early(J, A) else 0)

    def dspre(self, J, A=0):
        """Look-ahead S groups issued ahead of the J groups and the prologue's wait."""
        pre = min(self.ds(J, A), self.nsl(J, A) - 4) if self.PRE_LA else 0
        return pre if pre > 0 else self.ds(J, A)

    def after(self, J, stw, i, A=0):
        DS, NP, NSD = self.ds(J, A), self.np(J, A), {0: 4, 1: 6, 2: 8}[self.kind(A)]
        early, late, jreg, rf = self.early(J, A), self.late(J, A), self.jreg(J, A), self.rf(J, A)
        n = lastS = lastJ = 0
        pre = self.dspre(J, A)
        for d in range(pre):
            n += NSD
            if d == i:
                lastS = n
        if J > 0 and not jreg:
            for d in range(1 if late else (NP if rf else NP - 1)):
                n += J
                if d == i:
                    lastJ = n
        for d in range(pre, DS):
            n += NSD
            if d == i:
                lastS = n
        if self.jpf(J, A):
            n += J  # plane k0's J rows, the last prologue loads
        s = 0
        while True:
            if jreg:
                n += J  # the step's J row loads at its top
            if early:
                n += NSD
                if s + DS == i:
                    lastS = n
                if J > 0 and not late and not jreg and not rf:
                    n += J
                    if s + NP - 1 == i:
                        lastJ = n
            if s == i:
                break
            if not early:
                n += NSD
                if s + DS == i:
                    lastS = n
                if J > 0 and not late and not jreg and not rf:
                    n += J
                    if s + NP - 1 == i:
                        lastJ = n
            if late or rf:  # the slot just read takes plane s + 1 / s + NP
                n += J
                if s + (1 if late else NP) == i:
                    lastJ = n
            n += stw
            s += 1
        return min(n - lastS, n - lastJ if J > 0 and not jreg else 1 << 20)

    def waits(self, J, stw, A=0):
        """The vmcnt values wait_step<J, STW, A> can emit (steps 0 .. p2d_i0)."""
        i0 = self.ds(J, A) + self.np(J, A) + 1
        return sorted({min(63, max(0, self.after(J, stw, i, A))) for i in range(i0 + 1)})


def check_p2d(funcs, meta, sched: P2dSchedule):
    """Per k_p2d instantiation: (name, problems list, record dict).  Checks: no
    scratch / buffer / flat access (nor an accessed private segment) and no VGPR spill; the march
    loop issues exactly the source's loads per step (2 + J DMA rows + 2 halo
    pieces) and its STW stores (once, or once per full / ragged-tile branch), no
    other VMEM operation; and its s_waitcnt vmcnt values are exactly the
    hand-counted p2d_after values of the source (so no compiler-added VMEM op
    shifted the count)."""
    res = []
    for name, ins in sorted(funcs.items()):
        prm = p2d_params(name)
        if prm is None or name.endswith(".kd"):
            continue
        J, hz, d2, pr, A = prm
        A = (2 if pr else 1) if A else 0  # the ring functions' anisotropic kind
        K = 3 if (A == 0 and d2) else A   # ... and the kind the ring / wait rules take (KA)
        probs = []
        allv = vmem_counts(ins)
        bad = {k: v for k, v in allv.items() if k.startswith(("scratch_", "buffer_", "flat_"))}
        if bad:
            probs.append(f"scratch/buffer/flat ops in the kernel: {bad}")
        md = meta.get(name, {})
        # a private segment the code never touches (the register scavenger's reserved
        # emergency slot next to many SGPR spills) issues no VMEM op: only one that is
        # accessed -- by the scratch / buffer / flat ops flagged above -- breaks the count
        if md.get("private_segment_fixed_size", "0") != "0" and bad:
            probs.append(f"private segment {md.get('private_segment_fixed_size')} B")
        if md.get("vgpr_spill_count", "0") != "0":
            probs.append(f"vgpr spills {md.get('vgpr_spill_count')}")
        loop = main_loop(ins, name)
        got = vmem_counts(loop)
        stw = 1 + hz
        loads = {k: v for k, v in got.items() if k != "global_store_dwordx4"}
        jreg = sched.jreg(J, K)
        if loads != p2d_loop_loads(J, A, jreg):
            probs.append(f"march loop loads {loads} != the source's {p2d_loop_loads(J, A, jreg)}")
        if got.get("global_store_dwordx4", 0) not in (stw, 2 * stw):
            probs.append(f"march loop stores {got.get('global_store_dwordx4', 0)} (STW = {stw})")
        waits = sorted({int(re.search(r"vmcnt\((\d+)\)", o).group(1)) for _a, mn, o in loop
                        if mn == "s_waitcnt" and "vmcnt" in o})
        # jreg: the compiler adds its own counted waits for the J register loads
        if (not set(sched.waits(J, stw, K)) <= set(waits)) if jreg else waits != sched.waits(J, stw, K):
            probs.append(f"march loop vmcnt waits {waits} != p2d_after {sched.waits(J, stw, K)}")
        rec = {"J": J, "HZ": hz, "D2": d2, "PR": pr, "A": A, "vgpr": md.get("vgpr_count"), "agpr": md.get("agpr_count"),
               "sgpr": md.get("sgpr_count"), "sgpr_spill": md.get("sgpr_spill_count"),
               "vgpr_spill": md.get("vgpr_spill_count"), "lds": md.get("group_segment_fixed_size"),
               "private": md.get("private_segment_fixed_size"), "loop_vmem": got, "loop_vmcnt_waits": waits,
               "loop_instructions": len(loop)}
        res.append((name, probs, rec))
    return res
