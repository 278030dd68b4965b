"""CPU-only checks of the boundary and host logic (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from rf_ray_tracing_warp_amd import _lib
from rf_ray_tracing_warp_amd.mesh import load_stl, sphere
from rf_ray_tracing_warp_amd.tracer import cir_flags

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(REPO, "include", "rfrt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    names = _declared()
    assert len(names) >= 10
    for n in names:
        assert hasattr(L, n), n
    assert L.rt_version() == 1


def test_error_channel_without_gpu_work():
    L = _lib.lib()
    # invalid arguments are rejected before any device call
    rc = L.rt_trace(None, None, None, 3, 0, 10, None, None, None, None, None, None)
    assert rc == -1
    assert b"invalid" in L.rt_last_error()
    with pytest.raises(_lib.RfrtError):
        _lib.check(rc, "rt_trace")
    assert L.rt_compact_workspace_bytes(1_000_000) >= 8 * (1_000_000 // 2048)


def test_stl_loader_room():
    m = load_stl(os.path.join(REPO, "models", "room.stl"))
    assert m.faces.shape == (44, 3) and m.vertices.shape == (24, 3)
    e = load_stl(os.path.join(REPO, "models", "almost_empty.stl"))
    assert e.faces.shape == (12, 3) and e.vertices.shape == (8, 3)
    np.testing.assert_allclose(e.bounds, [[-0.05] * 3, [0.05] * 3], atol=1e-7)


def test_stl_ascii_roundtrip(tmp_path):
    m = load_stl(os.path.join(REPO, "models", "room.stl"))
    lines = ["solid t"]
    for f in m.faces:
        lines += ["facet normal 0 0 0", "outer loop"]
        lines += ["vertex %r %r %r" % tuple(float(x) for x in m.vertices[i].astype(np.float32)) for i in f]
        lines += ["endloop", "endfacet"]
    lines.append("endsolid t")
    p = tmp_path / "a.stl"
    p.write_text("\n".join(lines))
    a = load_stl(str(p))
    np.testing.assert_array_equal(a.triangles.astype(np.float32), m.triangles.astype(np.float32))


def test_rx_icosphere_shape():
    s = sphere((-10, 0, 5), 0.1, 1)  # tracer.py:27
    assert s.vertices.shape == (42, 3) and s.faces.shape == (80, 3)
    r = np.linalg.norm(s.vertices - [-10, 0, 5], axis=1)
    np.testing.assert_allclose(r, 0.1, rtol=1e-12)


def test_nep50_cir_flags():
    assert cir_flags(2.998e8, 100e9) == 0
    assert cir_flags(np.float64(2.998e8), 100e9) == _lib.RT_CIR_C_F64
    assert cir_flags(2.998e8, np.float64(100e9)) == _lib.RT_CIR_FS_F64
    assert cir_flags(np.float32(2.998e8), 100e9) == 0


@pytest.mark.parametrize("c", [2.998e8, 299800000, np.float64(2.998e8), np.float32(2.998e8), np.int64(299800000),
                               np.int32(299800000), np.int16(30000), np.uint64(299800000), np.float16(3e4),
                               np.array(2.998e8), np.array(2.998e8, np.float32)])
@pytest.mark.parametrize("fs", [100e9, 100_000_000_000, np.float64(100e9), np.float32(100e9), np.int64(10 ** 11),
                                np.uint32(4_000_000_000)])
def test_nep50_cir_flags_follow_numpy_promotion(c, fs):
    """tracer.py:115 with distance a np.float32: the flags select float64 exactly where NumPy 2 does
    (strong NumPy integer types such as np.int64 promote float32 to float64, Python scalars do not)."""
    d = np.float32(37.5)
    q = d / c
    val = q * fs
    f = cir_flags(c, fs)
    assert bool(f & _lib.RT_CIR_C_F64) == (np.asarray(q).dtype == np.float64)
    if not f & _lib.RT_CIR_C_F64:
        assert bool(f & _lib.RT_CIR_FS_F64) == (np.asarray(val).dtype == np.float64)
    else:
        assert np.asarray(val).dtype == np.float64


def _fx_to_double(words):
    L = _lib.lib()
    w = np.ascontiguousarray(np.asarray(words, dtype=np.uint64).reshape(-1, 3))
    out = np.zeros(len(w))
    _lib.check(L.rt_selftest_fx(w.ctypes.data, out.ctypes.data, len(w), 0), "rt_selftest_fx")
    return out


def _fx_exact(words):
    from fractions import Fraction
    w0, w1, w2 = (int(x) for x in words)
    return Fraction(w0 + (w1 << 64) + (w2 << 128), 1 << 136)


def test_fixed_point_to_double_is_correctly_rounded_everywhere():
    """coverage.hip fx_to_double (the coverage bin sums, rounded once): every window position,
    including a saturated value whose top bit is bit 191 (the shift by 64 there)."""
    rng = np.random.default_rng(7)
    cases = [(0, 0, 0), (1, 0, 0), (~0 & (2**64 - 1), 0, 0), (0, 1, 0), (0, 0, 1), (2**63, 2**63, 2**63),
             (2**64 - 1, 2**64 - 1, 2**64 - 1), (1, 0, 2**63), (0, 1, 2**63), (0, 0, 2**63), (2**64 - 1, 2**64 - 1, 0)]
    for top in range(0, 192, 3):
        for _ in range(4):
            v = int(rng.integers(0, 2**63)) | (1 << 63)
            lo = int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))
            x = (lo | (v << 128)) >> (191 - top) if top < 191 else (lo | (v << 128))
            cases.append((x & (2**64 - 1), (x >> 64) & (2**64 - 1), x >> 128))
    got = _fx_to_double(cases)
    for c, g in zip(cases, got):
        assert g == float(_fx_exact(c)), (c, g)  # float(Fraction) rounds to nearest even


def test_fixed_point_from_double_truncates_exactly():
    L = _lib.lib()
    a = np.array([0.0, 1e-6, 3.5e-41, 2.0**-136, 2.0**-137, 1.0, 123.456, 2.0**55, 2.0**56 * 0.75, 5e-324], np.float64)
    w = np.zeros((len(a), 3), np.uint64)
    _lib.check(L.rt_selftest_fx(w.ctypes.data, a.ctypes.data, len(a), 1), "rt_selftest_fx")
    from fractions import Fraction
    for x, ww in zip(a, w):
        want = int(Fraction(float(x)) * (1 << 136))  # truncation below the unit 2^-136
        assert _fx_exact(ww) * (1 << 136) == want, x
