"""rt_trace_cir (trace + one fused launch for the ordered compaction and the impulse response) gives
exactly what rt_trace + rt_compact + rt_cir give (tracer.py:67-117): every output bit, on the
brute-force path (the trace kernel counts received rows per chunk) and the BVH path (a separate
count kernel), with no, few and many received rows, call after call on one workspace."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr  # noqa: E402
from rf_ray_tracing_warp_amd.mesh import load_stl, sphere, synthetic_terrain  # noqa: E402
from rf_ray_tracing_warp_amd.tracer import cir_flags  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DEV = "cuda:0"
C, FS, NB = 2.998e8, 100e9, 10000


@pytest.fixture(scope="module", autouse=True)
def _gpu(require_gpu):
    lib()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _separate(env, rx, tx, B, off, n, amp0):
    P = B + 1
    tr = torch.empty((n, P, 3), dtype=torch.float32, device=DEV)
    rc = torch.empty_like(tr)
    mk = torch.empty(n, dtype=torch.int32, device=DEV)
    L = lib()
    check(L.rt_trace(env.handle, tx.ctypes.data, rx.handle if rx else None, B, off, n, ptr(tr), ptr(rc), ptr(mk),
                     None, None, _s()), "rt_trace")
    ws = torch.empty(int(L.rt_compact_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    idx = torch.empty(n, dtype=torch.int64, device=DEV)
    cnt = torch.empty(1, dtype=torch.int64, device=DEV)
    check(L.rt_compact(ptr(mk), n, ptr(ws), ws.numel(), ptr(idx), ptr(cnt), _s()), "rt_compact")
    ir = torch.zeros(NB, dtype=torch.float64, device=DEV)
    check(L.rt_cir(ptr(rc), ptr(idx), ptr(cnt), n, B, amp0, C, FS, cir_flags(C, FS), NB, ptr(ir), None, None, _s()),
          "rt_cir")
    k = int(cnt.item())
    return tr.cpu().numpy(), rc.cpu().numpy(), mk.cpu().numpy(), idx[:k].cpu().numpy(), ir.cpu().numpy()


def _fused(env, rx, tx, B, off, n, amp0, ws, calls=1):
    P = B + 1
    tr = torch.empty((n, P, 3), dtype=torch.float32, device=DEV)
    rc = torch.empty_like(tr)
    mk = torch.empty(n, dtype=torch.int32, device=DEV)
    idx = torch.empty(n, dtype=torch.int64, device=DEV)
    cnt = torch.empty(1, dtype=torch.int64, device=DEV)
    ir = torch.full((NB,), 7.0, dtype=torch.float64, device=DEV)  # overwritten, not accumulated
    L = lib()
    for _ in range(calls):
        check(L.rt_trace_cir(env.handle, tx.ctypes.data, rx.handle if rx else None, B, off, n, ptr(tr), ptr(rc),
                             ptr(mk), amp0, C, FS, cir_flags(C, FS), NB, ptr(ir), ptr(idx), ptr(cnt), ptr(ws),
                             ws.numel(), _s()), "rt_trace_cir")
    k = int(cnt.item())
    return tr.cpu().numpy(), rc.cpu().numpy(), mk.cpu().numpy(), idx[:k].cpu().numpy(), ir.cpu().numpy()


def _check(a, b):
    for x, y in zip(a, b):
        assert x.shape == y.shape
        assert np.ascontiguousarray(x).tobytes() == np.ascontiguousarray(y).tobytes()


@pytest.mark.parametrize("rxc,r,n,off", [
    ((-10.0, 0.0, 5.0), 0.1, 1_000_000, 0),      # K2: ~1 received row
    ((8.5, 0.5, 5.0), 1.5, 300_000, 12_345),      # a large receiver near the TX: tens of thousands
    (None, 0.0, 50_001, 0),                        # no receiver: nothing received, a partial chunk
])
def test_trace_cir_equals_separate_calls_room(rxc, r, n, off):
    room = load_stl(os.path.join(REPO, "models", "room.stl"))
    env = DeviceMesh(room.vertices, room.faces, 0)
    rx = DeviceMesh(*(lambda m: (m.vertices, m.faces))(sphere(rxc, r, 1)), 0) if rxc else None
    tx = np.asarray((10.0, 0.0, 5.0), np.float32)
    ws = torch.zeros(int(lib().rt_trace_cir_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    ref = _separate(env, rx, tx, 3, off, n, 1.0 / n)
    got = _fused(env, rx, tx, 3, off, n, 1.0 / n, ws, calls=2)  # the second call reuses the workspace
    _check(got, ref)
    if rxc is None:
        assert len(got[3]) == 0 and not got[4].any()
    elif r > 1:
        assert len(got[3]) > 10_000


def test_trace_cir_equals_separate_calls_bvh():
    t = synthetic_terrain(256, 50.0)
    env = DeviceMesh(t.vertices, t.faces, 0)
    m = sphere((2.0, 1.0, 3.0), 1.0, 1)
    rx = DeviceMesh(m.vertices, m.faces, 0)
    tx = np.asarray((10.0, 0.0, 4.5), np.float32)
    n = 200_000
    ws = torch.zeros(int(lib().rt_trace_cir_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    ref = _separate(env, rx, tx, 5, 0, n, 1.0 / n)
    got = _fused(env, rx, tx, 5, 0, n, 1.0 / n, ws)
    _check(got, ref)
    assert len(got[3]) > 0


def test_trace_profile_stats_counts_kernels():
    room = load_stl(os.path.join(REPO, "models", "room.stl"))
    env = DeviceMesh(room.vertices, room.faces, 0)
    tx = np.asarray((10.0, 0.0, 5.0), np.float32)
    n = 100_000
    ws = torch.zeros(int(lib().rt_trace_cir_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    L = lib()
    L.rt_profile(1)
    _fused(env, None, tx, 3, 0, n, 1.0 / n, ws, calls=3)
    L.rt_profile(0)
    st = np.zeros(4)
    check(L.rt_trace_profile_stats(st.ctypes.data, 4), "rt_trace_profile_stats")
    assert st[0] == 3 and 0 < st[2] <= st[1] <= st[3] < 100


def test_compute_cir_above_the_fused_cap_takes_the_uncapped_path(monkeypatch):
    """rt_trace_cir takes at most 2^25 rays per call; Tracer.compute_cir falls back to
    rt_trace + rt_compact + rt_cir above that (no cap, like the reference's tracer.py).  The cap is
    lowered here so a small burst crosses it: both paths give the same paths and impulse response."""
    from rf_ray_tracing_warp_amd import Tracer
    room = load_stl(os.path.join(REPO, "models", "room.stl"))
    t = Tracer(room, C, FS, 100e-9, 3, 300_000, device=0)
    ref_paths, ref_ir = t.compute_cir(np.array((10.0, 0.0, 5.0)), 1, np.array((8.5, 0.5, 5.0)), 1.5)
    monkeypatch.setattr(Tracer, "TRACE_CIR_MAX_RAYS", 1000)
    paths, ir = t.compute_cir(np.array((10.0, 0.0, 5.0)), 1, np.array((8.5, 0.5, 5.0)), 1.5)
    assert len(paths) == len(ref_paths) > 10_000
    assert all(np.array_equal(a, b) for a, b in zip(paths, ref_paths))
    assert ir.tobytes() == ref_ir.tobytes()
