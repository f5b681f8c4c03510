"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
entry point include/nls.h declares, validates configs before touching a device,
and the CLI drivers keep the reference's argv/exit-code contract
(device/nlse_call.cpp:13-24, 51-56)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "nonlinear-solvers_amd", "bin")
HEADER = os.path.join(ROOT, "include", "nls.h")

nls_amd = pytest.importorskip("nls_amd")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*\*?\s*(nls_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    L = nls_amd.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(nls_amd.EXPORTED_SYMBOLS) == syms
    assert L.nls_abi_version() == 6
    out = subprocess.run(["nm", "-D", "--defined-only", nls_amd.lib_path()], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (nls_\w+)", out))
    assert set(syms) <= exported


def test_config_default_matches_reference_defaults():
    L = nls_amd.lib()
    c = nls_amd.Config()
    L.nls_config_default(C.byref(c))
    assert c.krylov_m == 10                       # device/nlse_solver_dev.hpp:48
    assert tuple(c.sigma1) == (0.0, 0.5)          # device/nlse_cq_solver.hpp:19
    assert tuple(c.sigma2) == (-0.5, 0.0)
    assert c.nranks == 1 and c.rank == 0 and c.device == -1


@pytest.mark.parametrize("kw,msg", [
    (dict(m=0), "krylov_m"), (dict(m=33), "krylov_m"), (dict(dim=4), "dim"),
    (dict(nx=1), "grid too small"), (dict(dx=0.0), "dx"), (dict(nranks=2), "rccl_id"),
    (dict(equation=10), "unknown equation"), (dict(equation=3, nx=2), "need >= 3 cells"), (dict(equation=4, ny=2), "need >= 3 cells"),
    (dict(equation=3, dim=3, nz=3, nranks=2, group=True), "2 planes per rank"),
    # 32-bit cell indices of the stencil march: (planes + 2) * plane + pad < 2^31
    (dict(dim=2, nx=50000, ny=50000, equation=2), "32-bit cell indices"),
    (dict(dim=3, nx=1300, ny=1300, nz=1300), "32-bit cell indices"),
    (dict(dim=3, nx=2048, ny=2048, nz=2048, nranks=4, group=True), "32-bit cell indices"),
])
def test_invalid_config_rejected_before_device(kw, msg):
    base = dict(dim=2, nx=16, ny=16, nz=1, dx=0.5)
    base.update(kw)
    m = base.pop("m", 10)
    nranks = base.pop("nranks", 1)
    eq = base.pop("equation", 0)
    grp = nls_amd.Group(nranks) if base.pop("group", False) else None
    with pytest.raises(nls_amd.NlsError) as e:
        nls_amd.Solver(base["dim"], base["nx"], base["ny"], base["nz"], base["dx"], m=m, nranks=nranks,
                       equation=eq, group=grp)
    assert e.value.code == -1 and msg in str(e.value)


def run(args, **kw):
    return subprocess.run(args, capture_output=True, text=True, timeout=60, **kw)


def test_index_limit_boundary_not_rejected_early():
    """Just below the limit ((nzl + 4) * P + pad < 2^31: two ghost planes per side)
    the config passes validation (it then needs a device: on this CPU-only host
    creation fails with a HIP error, not NLS_ERR_ARG); one plane more is rejected."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("would allocate ~ 2^31 cells on a GPU")
    with pytest.raises(nls_amd.NlsError) as e:
        nls_amd.Solver(3, 1024, 1024, 2043, 0.1, m=3)
    assert "32-bit" not in str(e.value)
    with pytest.raises(nls_amd.NlsError) as e:
        nls_amd.Solver(3, 1024, 1024, 2044, 0.1, m=3)
    assert e.value.code == -1 and "32-bit" in str(e.value)


@pytest.mark.parametrize("prog", ["nlse_call", "nlse_cq_call", "to_nlse_call", "to_nlse_cq_call"])
def test_driver_usage_exit_code(prog):
    r = run([os.path.join(BIN, prog)])
    assert r.returncode == 1 and "Usage:" in r.stderr
    r = run([os.path.join(BIN, prog)] + ["8"] * 8)
    assert r.returncode == 1 and "Usage:" in r.stderr


@pytest.mark.parametrize("prog", ["sg_single_dev", "sg_double_dev", "sg_hyperbolic_dev", "phi4_dev"])
def test_gautschi_g2_driver_usage(prog, tmp_path):
    """phi4_driver_dev.cpp:17-28: 11 or 12 argv, else usage + exit 1; u0 of the wrong
    shape -> "Error: Input array dimensions mismatch" + exit 1 (before any device call)."""
    for n in (0, 9, 12):
        r = run([os.path.join(BIN, prog)] + ["8"] * n)
        assert r.returncode == 1 and "Usage:" in r.stderr
    np.save(tmp_path / "u0.npy", np.zeros((8, 9)))
    np.save(tmp_path / "v0.npy", np.zeros((8, 9)))
    r = run([os.path.join(BIN, prog), "8", "8", "1", "1", str(tmp_path / "u0.npy"), str(tmp_path / "v0.npy"),
             str(tmp_path / "o.npy"), "1", "10", "2"])
    assert r.returncode == 1 and "Input array dimensions mismatch" in r.stderr


def test_driver_shape_mismatch(tmp_path):
    u = np.zeros((16, 12), complex)
    f = tmp_path / "u0.npy"
    np.save(f, u)
    r = run([os.path.join(BIN, "nlse_call"), "12", "12", "10", "10", str(f), str(tmp_path / "o.npy"),
             "1.5", "10", "5"])
    assert r.returncode == 1
    assert "Input array dimensions mismatch" in r.stderr and "Expected: 12x12" in r.stderr


def test_driver_guards_zero_snapshot_frequency(tmp_path):
    f = tmp_path / "u0.npy"
    np.save(f, np.ones((8, 8), complex))
    r = run([os.path.join(BIN, "nlse_call"), "8", "8", "10", "10", str(f), str(tmp_path / "o.npy"),
             "1.5", "5", "10"])
    assert r.returncode == 1 and "num_snapshots" in r.stderr


def test_sg_driver_rejects_positional():
    r = run([os.path.join(BIN, "sg_driver_dev"), "256"])
    assert r.returncode == 1 and "Usage" in r.stderr


@pytest.mark.parametrize("shape,dtype", [((7,), complex), ((5, 3), complex), ((2, 3, 4), complex),
                                         ((4, 2, 3, 2), complex), ((6,), float), ((3, 5), float)])
def test_npy_codec_roundtrip(tmp_path, shape, dtype):
    rng = np.random.default_rng(0)
    a = rng.standard_normal(shape)
    if dtype is complex:
        a = a + 1j * rng.standard_normal(shape)
    f, g = tmp_path / "a.npy", tmp_path / "b.npy"
    np.save(f, a)
    mode = "copy-c16" if dtype is complex else "copy-f8"
    r = run([os.path.join(BIN, "npy_tool"), mode, str(f), str(g)])
    assert r.returncode == 0, r.stderr
    b = np.load(g)
    assert b.dtype == a.dtype and b.shape == a.shape and np.array_equal(a, b)
    r = run([os.path.join(BIN, "npy_tool"), "shape", str(g)])
    assert r.stdout.split() == [str(s) for s in shape]


def test_npy_codec_rejects_wrong_dtype(tmp_path):
    f = tmp_path / "a.npy"
    np.save(f, np.zeros((3, 3), np.float32))
    r = run([os.path.join(BIN, "npy_tool"), "copy-c16", str(f), str(tmp_path / "b.npy")])
    assert r.returncode == 1 and "dtype" in r.stderr


# ---- G2 drivers (nlse_3d_dev / nlse_2d_dev): argv and input contract, no GPU needed


@pytest.mark.parametrize("prog,npos", [("nlse_3d_dev", 13), ("nlse_2d_dev", 11), ("nlse_sewi_3d_dev", 13),
                                      ("nlse_sewi_2d_dev", 11), ("kg_gautschi_3d_dev", 15),
                                      ("kg_gautschi_2d_dev", 13)])
def test_g2_driver_usage(prog, npos):
    for k in (0, npos - 2, npos - 1, npos + 1):   # nlse_cubic_driver_3d.cpp:20-31 (argc != 14)
        r = run([os.path.join(BIN, prog)] + ["8"] * k)
        assert r.returncode == 1 and "Usage:" in r.stderr and "input_m.npy input_c.npy" in r.stderr


def _g2_files(tmp_path, ushape, mshape, cshape):
    paths = []
    for name, shp, dt in (("u0", ushape, complex), ("m", mshape, float), ("c", cshape, float)):
        f = tmp_path / f"{name}.npy"
        np.save(f, np.ones(shp, dt))
        paths.append(str(f))
    return paths


def test_g2_driver_shape_checks(tmp_path):
    exe = os.path.join(BIN, "nlse_3d_dev")
    out = str(tmp_path / "o.npy")
    u, mf, cf = _g2_files(tmp_path, (6, 5, 4), (6, 5, 4), (6, 5, 4))
    r = run([exe, "4", "5", "7", "2", "2", "2", u, out, "1", "10", "5", mf, cf])
    assert r.returncode == 1 and "Input array dimensions mismatch" in r.stderr
    u, mf, cf = _g2_files(tmp_path, (6, 5, 4), (6, 5, 3), (6, 5, 4))
    r = run([exe, "4", "5", "6", "2", "2", "2", u, out, "1", "10", "5", mf, cf])
    assert r.returncode == 1 and "Coupling array dimensions mismatch" in r.stderr and "Faulty m" in r.stderr
    u, mf, cf = _g2_files(tmp_path, (6, 5, 4), (6, 5, 4), (5, 4))
    r = run([exe, "4", "5", "6", "2", "2", "2", u, out, "1", "10", "5", mf, cf])
    assert r.returncode == 1 and "Faulty c" in r.stderr
    u, mf, cf = _g2_files(tmp_path, (6, 5, 4), (6, 5, 4), (6, 5, 4))
    r = run([exe, "4", "5", "6", "2", "2", "2", u, out, "1", "3", "5", mf, cf])
    assert r.returncode == 1 and "num_snapshots" in r.stderr
    # 2D: the reference checks [nx, ny] (nlse_cubic_driver_2d.cpp:49-56)
    u, mf, cf = _g2_files(tmp_path, (6, 6), (6, 6), (6, 5))
    r = run([os.path.join(BIN, "nlse_2d_dev"), "6", "6", "2", "2", u, out, "1", "10", "5", mf, cf])
    assert r.returncode == 1 and "Faulty c" in r.stderr


# ---- G2 cubic-quintic driver (nlse_cubic_quintic_dev): argv and input contract


def test_cq_g2_driver_usage_and_shape(tmp_path):
    """nlse_cubic_quintic_driver_dev.cpp:16-27: 11 or 12 positional args, else usage +
    exit 1; :58-63 u0 must be [ny, nx] ("Expected: nyxnx")."""
    exe = os.path.join(BIN, "nlse_cubic_quintic_dev")
    for k in (0, 10, 13):
        r = run([exe] + ["8"] * k)
        assert r.returncode == 1 and "Usage:" in r.stderr and "[input_m.npy]" in r.stderr
    f = tmp_path / "u0.npy"
    np.save(f, np.ones((6, 5), complex))
    out = str(tmp_path / "o.npy")
    r = run([exe, "6", "5", "2", "2", "1", "0.5", str(f), out, "1", "10", "5"])
    assert r.returncode == 1 and "Input array dimensions mismatch" in r.stderr and "Expected: 5x6" in r.stderr
    np.save(f, np.ones((5, 6), complex))
    r = run([exe, "6", "5", "2", "2", "1", "0.5", str(f), out, "1", "3", "5"])
    assert r.returncode == 1 and "num_snapshots" in r.stderr


def test_abi_exports_cq_g2_equation():
    assert nls_amd.NLSE_CQ_G2 == 9
    with open(os.path.join(ROOT, "include", "nls.h")) as fh:
        assert "NLS_NLSE_CQ_G2 = 9" in fh.read()


def test_comm_size_rejects_null_handle():
    """nls_comm_size (the ranks bench.py reports) fails cleanly without a handle or
    an output pointer -- no device needed."""
    import ctypes as C
    L = nls_amd.lib()
    n, tr = C.c_int32(-7), C.c_int32(-7)
    assert L.nls_comm_size(None, C.byref(n), C.byref(tr)) == -1
    assert n.value == -7 and tr.value == -7


def test_placement_and_peer_state_reject_null_handle():
    """nls_placement / nls_peer_state (ABI 6) fail cleanly without a handle or an output
    pointer, leaving the outputs untouched -- no device needed."""
    import ctypes as C
    L = nls_amd.lib()
    n, k = C.c_int32(-7), C.c_int32(-7)
    ms = (C.c_float * 8)()
    assert L.nls_placement(None, C.byref(n), C.byref(k), ms, 8) == -1
    assert n.value == -7 and k.value == -7
    st = C.c_int32(-7)
    assert L.nls_peer_state(None, C.byref(st)) == -1 and st.value == -7


def test_library_build_matches_sources():
    """Build provenance: the loaded libnls_amd.so was compiled from exactly the library
    sources of this tree (nls_build_info's compiled-in sha256 of csrc/*.{hip,hpp,cpp} +
    include/nls.h).  On the GPU box, where the prebuilt library travels with the tree,
    the same test says whether the two still match."""
    info = nls_amd.build_info()
    assert info["arch"] == "gfx950"
    assert info["src_sha256"] == nls_amd.sources_sha256()
