"""Resource record of kernels in libnls_amd.so: VGPR/AGPR/SGPR, spills, LDS, private
segment, instructions of the widest loop and their class mix.
  python tools/kinfo.py REGEX [lib]      (REGEX against the mangled kernel name)"""
import collections
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import codeobj  # noqa: E402


def classify(mn):
    if mn.startswith(("global_load_lds", "buffer_load_dword_lds")):
        return "dma"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith("s_waitcnt") or mn.startswith("s_barrier") or mn.startswith("s_nop"):
        return "wait"
    if mn.startswith("s_"):
        return "salu"
    if mn.startswith(("v_accvgpr",)):
        return "agpr"
    if mn.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane"
    if "f64" in mn:
        return "f64"
    return "valu"


def main():
    pat = re.compile(sys.argv[1])
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(HERE), "nonlinear-solvers_amd", "lib",
                                                           "libnls_amd.so")
    for co in codeobj.gfx950_objects(lib):
        md = codeobj.metadata(co)
        funcs = codeobj.disassemble(co)
        for name in sorted(md):
            if not pat.search(name):
                continue
            m = md[name]
            fn = name
            ins = funcs.get(fn, [])
            loop = codeobj.main_loop(ins, fn)
            mix = collections.Counter(classify(mn) for _, mn, _ in loop)
            print(f"{name[:90]:90s} v{m.get('vgpr_count')} a{m.get('agpr_count')} s{m.get('sgpr_count')} "
                  f"sspill{m.get('sgpr_spill_count')} vspill{m.get('vgpr_spill_count')} "
                  f"lds{m.get('group_segment_fixed_size')} priv{m.get('private_segment_fixed_size')} "
                  f"loop{len(loop)} " + " ".join(f"{k}:{v}" for k, v in sorted(mix.items())))


if __name__ == "__main__":
    main()
