"""CPU: the timing-only diagnostic switches are off in the product build.  NLS_DIAG_HALO
(nls_stencil.hpp) and NLS_DIAG_P2HALO (nls_pass2d.hpp) drop halo loads and give WRONG
results; they exist only for variant libraries built by tools/build_lib_variant.sh.  The
XCD-banded tail queue stays off by default too; the four-vector first
pass (NLS_P4, k_p4r) is on by default since round 6 and k_p4r is its kernel."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nonlinear-solvers_amd", "csrc")


def _default(path, macro):
    src = open(os.path.join(CSRC, path)).read()
    m = re.search(r"#ifndef %s\s*\n#define %s (\d+)" % (macro, macro), src)
    assert m, f"{macro} default not found in {path}"
    return int(m.group(1))


def test_diagnostic_switches_default_off():
    assert _default("nls_stencil.hpp", "NLS_DIAG_HALO") == 0
    assert _default("nls_pass2d.hpp", "NLS_DIAG_P2HALO") == 0
    assert _default("nls_api.cpp", "NLS_P4") == 1
    assert _default("nls_pass4.hip", "NLS_P4_KIND") == 2
    assert _default("nls_common.hpp", "NLS_TQ_XCD") == 0


def test_product_build_defines_no_diagnostic():
    mk = open(os.path.join(ROOT, "Makefile")).read()
    assert "NLS_DIAG" not in mk and "-DNLS_P4" not in mk
    ge = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    assert "NLS_DIAG" not in ge
