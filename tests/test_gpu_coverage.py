"""Coverage map on the GPU (shared-trajectory algorithm) vs the oracle's literal per-cell loop
(coverage.py:38-57: per cell a full trace + host CIR + np.convolve power).  Needs an MI355X.

Bar: the per-cell sparse impulse responses have identical bins; each cell's impulse response agrees
within 1e-5 relative norm-wise (max |diff| <= 1e-5 * max |ir|) and its power within 1e-5 relative
(north_star); cells that receive nothing are NaN in both.  Single entries are compared norm-wise
because the reference's float32 np.arccos (NumPy SIMD, a few ulp) moves an amplitude whose Fresnel
factor sits near its zero by more than 1e-5 of itself ("Tolerances")."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import oracle as orc  # noqa: E402
from rf_ray_tracing_warp_amd._lib import check, lib, ptr  # noqa: E402
from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid, phase_step  # noqa: E402
from rf_ray_tracing_warp_amd.mesh import load_stl  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module", autouse=True)
def _gpu(require_gpu):
    lib()


@pytest.fixture(scope="module")
def room():
    return load_stl(os.path.join(REPO, "models", "room.stl"))


def _compare(cov, grid, env_np, tx, B, N, win=100e-9):
    power = cov.run(tx, 1).reshape(-1)
    cells, bins, amps = cov.impulse_responses()
    E = orc.Mesh(env_np.vertices, env_np.faces)
    ref_p, ref_irs, ref_cr = orc.coverage_loop(E, tx, grid.centers().reshape(-1, 3), B, N, win=win, with_cr=True)
    for c in range(grid.num_cells):
        sel = cells == c
        rb = np.nonzero(ref_irs[c])[0]
        np.testing.assert_array_equal(bins[sel], rb, err_msg=f"cell {c}")
        if len(rb):
            scale = np.abs(ref_irs[c]).max()
            assert np.abs(amps[sel] - ref_irs[c][rb]).max() <= 1e-5 * scale, f"cell {c}"
    np.testing.assert_array_equal(np.isnan(power), np.isnan(ref_p))
    ok = ~np.isnan(ref_p)
    # (1) same computation as the reference with the arccos rounded once: agreement to 1e-9
    np.testing.assert_allclose(power[ok], ref_cr[ok], rtol=1e-9)
    # (2) vs the reference itself: 1e-5, plus exactly the spread its own float32 arccos rounding causes
    allowed = 1e-5 * np.abs(ref_p[ok]) + 1.01 * np.abs(ref_cr[ok] - ref_p[ok])
    assert np.all(np.abs(power[ok] - ref_p[ok]) <= allowed)
    assert np.mean(np.abs(power[ok] - ref_p[ok]) <= 1e-5 * np.abs(ref_p[ok])) >= 0.9
    return power, ref_p


@pytest.mark.parametrize("grid,tx,B,N", [
    (CoverageGrid.square(12, 15, 5), (10, 0, 5), 3, 30_000),                  # K3 shape, coarse
    (CoverageGrid(8.0, -0.5, 4.6, 0.13, 0.11, 0.2, 10, 10, 5), (10, 0, 5), 3, 20_000),  # around/at the TX
    (CoverageGrid.from_ranges(range(-15, 16, 6), range(-15, 16, 6), range(0, 16, 5)), (10, 0, 5), 2, 20_000),
    # longer paths: the replay continues through its receiver on the first win's line for several
    # bounces (the receiver-group mask of k_win, the clear-receiver shortcut), then reflects
    (CoverageGrid(7.0, -1.6, 4.6, 0.5, 0.45, 0.4, 8, 8, 2), (10, 0, 5), 5, 15_000),
    (CoverageGrid(7.0, -1.6, 4.6, 0.5, 0.45, 0.4, 8, 8, 2), (10, 0, 5), 1, 15_000),
])
def test_coverage_matches_per_cell_loop(room, grid, tx, B, N):
    cov = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid)
    power, ref = _compare(cov, grid, room, tx, B, N)
    assert np.isfinite(ref).sum() >= 3  # the test exercises cells that receive paths
    cov.close()


def test_coverage_cell_at_transmitter(room):
    """The cell centred on the TX: every ray starts inside its receiver sphere (Q3: and leaves it
    at t = radius), and its neighbours at 0.3 m receive dense direct bursts."""
    grid = CoverageGrid(9.7, -0.3, 5.0, 0.3, 0.3, 1.0, 3, 3, 1)
    cov = Coverage(room, 2.998e8, 100e9, 100e-9, 3, 20_000, grid)
    power, ref = _compare(cov, grid, room, (10.0, 0.0, 5.0), 3, 20_000)
    cov.close()


def test_coverage_sharded_ownership(room):
    """Each rank fills exactly the cells of its x columns (dist.owns_cell); the rest stay 0."""
    from rf_ray_tracing_warp_amd.dist import owns_cell
    grid, tx, B, N = CoverageGrid(-7.0, -6.0, 2.0, 1.3, 1.1, 2.5, 11, 7, 2), (10, 0, 5), 3, 20_000
    whole = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid).run_device(tx).cpu().numpy()
    for S in (2, 4, 8, 13):
        for r in range(S):
            part = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid, shard_index=r, shard_count=S).run_device(tx)
            part = part.cpu().numpy()
            mine = np.array([owns_cell(c, r, S, grid.nx) for c in range(grid.num_cells)])
            assert (part[~mine] == 0).all()
            np.testing.assert_array_equal(np.isnan(part[mine]), np.isnan(whole[mine]))
            ok = mine & ~np.isnan(whole)
            np.testing.assert_array_equal(part[ok], whole[ok])


def test_coverage_sharded_sum_equals_whole(room):
    grid, tx, B, N = CoverageGrid.square(16, 15, 5), (10, 0, 5), 3, 20_000
    whole = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid).run(tx)
    parts = [Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid, shard_index=s, shard_count=3).run_device(tx).clone()
             for s in range(3)]
    total = (parts[0] + parts[1] + parts[2]).cpu().numpy().reshape(whole.shape)
    np.testing.assert_array_equal(np.isnan(total), np.isnan(whole))
    ok = ~np.isnan(whole)
    np.testing.assert_array_equal(total[ok], whole[ok])


def test_power_dense_matches_numpy():
    rng = np.random.default_rng(3)
    n, win, rows = 10000, 100e-9, 24
    irs = np.zeros((rows, n))
    for r in range(rows):
        K = int(rng.integers(0, 30))
        irs[r, rng.choice(n, K, replace=False)] = rng.uniform(1e-8, 1e-5, K)
    irs[1, :] = 0
    irs[1, 4999] = 1e-6  # isolated sin(0) sample
    irs[2, :] = 0
    irs[2, [0, 9999]] = [2e-6, 3e-6]
    t = torch.from_numpy(irs).cuda()
    out = torch.empty(rows, dtype=torch.float64, device="cuda")
    scratch = torch.empty(rows * n * 16, dtype=torch.uint8, device="cuda")
    check(lib().rt_power_dense(ptr(t), rows, n, phase_step(win, n), ptr(scratch), scratch.numel(), ptr(out),
                               torch.cuda.current_stream().cuda_stream))
    got = out.cpu().numpy()
    ref = np.array([orc.signal_power(irs[r], win) for r in range(rows)])
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    np.testing.assert_allclose(got[ok], ref[ok], rtol=1e-9)


def test_coverage_on_bvh_terrain():
    """K5 shape (coverage on the large-mesh BVH path), small: terrain 256^2 vertices, 10x10 cells."""
    from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
    t = synthetic_terrain(256, 50.0)
    grid = CoverageGrid(7.0, -1.0, 2.0, 0.7, 0.25, 1.0, 10, 10, 1)
    tx, B, N = (10.0, 0.0, 4.5), 3, 20_000
    cov = Coverage(t, 2.998e8, 100e9, 200e-9, B, N, grid)
    power, ref = _compare(cov, grid, t, tx, B, N, win=200e-9)
    assert np.isfinite(ref).sum() >= 3
    cov.close()


def _ray_sharded(env, grid, tx, B, N, S, win=100e-9, env_mesh=None, segments=True, mode="rays"):
    """S ray-sharded plans in one process, through the path run() takes: trace_rows -> each
    owner's (key, sum) rows in source-rank order (what the all-to-all delivers) -> power_from_rows,
    and the owners' maps summed (what the power-map gather does across S GPUs).  segments: the
    owners merge the per-source segments (rt_coverage_power_packed), else they sort the rows
    (rt_coverage_power_rows).  mode "sectors": the ranks' rays are wedges of initial azimuth
    (rt_coverage_create_sectors) instead of ray-id ranges."""
    plans = [Coverage(env, 2.998e8, 100e9, win, B, N, grid, shard_index=r, shard_count=S, shard_mode=mode,
                      env_mesh=env_mesh) for r in range(S)]
    sent = []
    for p in plans:
        rows, counts = p.trace_rows(tx, 1)
        sent.append((rows.clone(), counts))
    total = torch.zeros(grid.num_cells, dtype=torch.float64, device="cuda")
    irs = []
    for d, p in enumerate(plans):
        parts, segs = [], []
        for rows, counts in sent:
            off = sum(counts[:d])
            parts.append(rows[off:off + counts[d]])
            segs.append(counts[d])
        total += p.power_from_rows(torch.cat(parts), segs if segments else None)
        p.check()
        irs.append(p.impulse_responses())
    for p in plans:
        p.close()
    return total.cpu().numpy(), irs


_ray_sharded_rows = _ray_sharded


@pytest.mark.parametrize("S", [1, 2, 3, 8])
def test_coverage_ray_sharded_equals_whole(room, S):
    """Ray shards + record exchange give the single-GPU map bit for bit: each (cell, bin) is summed
    exactly (fixed point) per shard and over shards, so the f64 sums and powers are the same."""
    grid, tx, B, N = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2), (10, 0, 5), 3, 60_000
    cov = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid)
    whole = cov.run_device(tx).cpu().numpy()
    wc, wb, wa = cov.impulse_responses()
    cov.close()
    total, irs = _ray_sharded(room, grid, tx, B, N, S)
    np.testing.assert_array_equal(np.isnan(total), np.isnan(whole))
    ok = ~np.isnan(whole)
    assert ok.sum() >= 20
    np.testing.assert_allclose(total[ok], whole[ok], rtol=1e-12)
    # owners' sparse impulse responses partition the whole run's, with the same bins
    c = np.concatenate([x[0] for x in irs])
    b = np.concatenate([x[1] for x in irs])
    a = np.concatenate([x[2] for x in irs])
    o = np.lexsort((b, c))
    np.testing.assert_array_equal(c[o], wc)
    np.testing.assert_array_equal(b[o], wb)
    np.testing.assert_allclose(a[o], wa, rtol=1e-12)


@pytest.mark.parametrize("S", [2, 3, 8])
def test_coverage_sector_sharded_equals_whole(room, S):
    """Sector shards (each rank traces the rays of one wedge of initial azimuth, rays chosen by
    direction rather than by id) give the single-GPU map and sparse impulse responses bit for bit:
    any partition of a cell's rays sums to the same fixed-point integers."""
    grid, tx, B, N = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2), (10, 0, 5), 3, 60_000
    cov = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid)
    whole = cov.run_device(tx).cpu().numpy()
    wc, wb, wa = cov.impulse_responses()
    cov.close()
    total, irs = _ray_sharded_rows(room, grid, tx, B, N, S, mode="sectors")
    assert (~np.isnan(whole)).sum() >= 20
    np.testing.assert_array_equal(total, whole)
    c = np.concatenate([x[0] for x in irs])
    b = np.concatenate([x[1] for x in irs])
    a = np.concatenate([x[2] for x in irs])
    o = np.lexsort((b, c))
    np.testing.assert_array_equal(c[o], wc)
    np.testing.assert_array_equal(b[o], wb)
    assert a[o].tobytes() == wa.tobytes()


def test_coverage_sector_sharded_bvh_terrain():
    from rf_ray_tracing_warp_amd._lib import DeviceMesh
    from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
    t = synthetic_terrain(256, 50.0)
    env = DeviceMesh(t.vertices, t.faces, 0)
    grid, tx, B, N = CoverageGrid(4.0, -6.0, 2.0, 0.9, 0.8, 1.0, 16, 16, 1), (10.0, 0.0, 4.5), 3, 40_000
    cov = Coverage(t, 2.998e8, 100e9, 200e-9, B, N, grid, env_mesh=env)
    whole = cov.run_device(tx).cpu().numpy()
    cov.close()
    total, _ = _ray_sharded_rows(t, grid, tx, B, N, 8, win=200e-9, env_mesh=env, mode="sectors")
    assert (~np.isnan(whole)).sum() >= 10
    np.testing.assert_array_equal(total, whole)


@pytest.mark.parametrize("S", [1, 3, 8])
def test_power_segments_equal_sorted_records(room, S):
    """The owner stage's segment merge (each source rank's records arrive sorted, merged by rank:
    rt_coverage_power_packed) gives exactly the sorted path's (rt_coverage_power_rows) maps and
    impulse responses."""
    grid, tx, B, N = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2), (10, 0, 5), 3, 60_000
    t_sort, irs_sort = _ray_sharded(room, grid, tx, B, N, S, segments=False)
    t_merge, irs_merge = _ray_sharded(room, grid, tx, B, N, S, segments=True)
    assert t_sort.tobytes() == t_merge.tobytes()
    assert np.isfinite(t_sort).sum() >= 20
    for a, b in zip(irs_sort, irs_merge):
        for x, y in zip(a, b):
            assert x.tobytes() == y.tobytes()


def test_trace_rows_grow(room):
    """A row buffer too small for a trace stage's rows is grown and the rows fetched from the plan
    (rt_coverage_records_packed, no second trace): the same rows, in the same order."""
    grid, tx, B, N = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2), (10, 0, 5), 3, 60_000
    p = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid, shard_index=2, shard_count=3, shard_mode="rays")
    rows, c = p.trace_rows(tx, 1)
    r = rows.cpu().numpy()
    assert sum(c) > 100
    p._rows = torch.empty((1, 4), dtype=torch.int64, device="cuda")
    rows3, c3 = p.trace_rows(tx, 1)
    assert c3 == c and p._rows.shape[0] > 1
    assert rows3.cpu().numpy().tobytes() == r.tobytes()
    p.close()


def test_coverage_ray_sharded_vs_oracle(room):
    """Ray-sharded (4 shards) against the per-cell reference loop, through the same bar as above."""
    grid, tx, B, N = CoverageGrid.square(10, 15, 5), (10, 0, 5), 3, 24_000
    total, irs = _ray_sharded(room, grid, tx, B, N, 4)
    E = orc.Mesh(room.vertices, room.faces)
    ref_p, ref_irs, ref_cr = orc.coverage_loop(E, tx, grid.centers().reshape(-1, 3), B, N, win=100e-9, with_cr=True)
    np.testing.assert_array_equal(np.isnan(total), np.isnan(ref_p))
    ok = ~np.isnan(ref_p)
    assert ok.sum() >= 3
    np.testing.assert_allclose(total[ok], ref_cr[ok], rtol=1e-9)


def test_coverage_ray_sharded_bvh_terrain():
    from rf_ray_tracing_warp_amd._lib import DeviceMesh
    from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
    t = synthetic_terrain(256, 50.0)
    env = DeviceMesh(t.vertices, t.faces, 0)
    grid, tx, B, N = CoverageGrid(4.0, -6.0, 2.0, 0.9, 0.8, 1.0, 16, 16, 1), (10.0, 0.0, 4.5), 3, 40_000
    cov = Coverage(t, 2.998e8, 100e9, 200e-9, B, N, grid, env_mesh=env)
    whole = cov.run_device(tx).cpu().numpy()
    cov.close()
    total, _ = _ray_sharded(t, grid, tx, B, N, 8, win=200e-9, env_mesh=env)
    assert (~np.isnan(whole)).sum() >= 10
    np.testing.assert_array_equal(total, whole)


def test_power_from_rows_every_sweep_path(room):
    """The closed-form power of k_power_small (<= 16 bins), k_power's LDS event sweep (17..192) and
    its range-split sweep (> 192; no full-size map cell has that many) against np.convolve, fed
    through rt_coverage_power_rows (rows of fixed-point sums from rt_coverage_amps_to_sums) with
    synthetic per-cell impulse responses."""
    rng = np.random.default_rng(8)
    sizes = [0, 1, 2, 5, 16, 17, 64, 191, 192, 193, 400, 2500, 9999]
    grid = CoverageGrid(0.0, 0.0, 5.0, 1.0, 1.0, 1.0, len(sizes), 1, 1)
    n, win = 10000, 100e-9
    irs = np.zeros((len(sizes), n))
    for c, K in enumerate(sizes):
        if K:
            irs[c, np.sort(rng.choice(n, K, replace=False))] = rng.uniform(1e-9, 1e-5, K)
    irs[2, :] = 0
    irs[2, [4999, 5000]] = [1e-6, 2e-6]  # the isolated sin(0) sample next to an active one
    cells, bins = np.nonzero(irs)
    keys = torch.from_numpy(((cells.astype(np.uint64) << np.uint64(32)) | bins.astype(np.uint64)).view(np.int64)).cuda()
    amps = torch.from_numpy(irs[cells, bins]).cuda()
    cov = Coverage(room, 2.998e8, 100e9, win, 3, 1000, grid, shard_mode="rays")
    got = cov.power_from_amplitudes(keys, amps).cpu().numpy()
    cov.close()
    ref = np.array([orc.signal_power(irs[c], win) for c in range(len(sizes))])
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    np.testing.assert_allclose(got[ok], ref[ok], rtol=1e-9)


def test_fixed_point_bin_sums_are_exact(room):
    """Per-bin sums (rt_coverage_amps_to_sums + the owner's reduce): every bin's f64 amplitude is the
    correctly rounded exact sum of its records truncated to the 2^-136 unit, whatever their order,
    over amplitudes spanning 1e-25 .. 1e-2 and bins of 1 .. 5000 records."""
    from fractions import Fraction
    import math
    rng = np.random.default_rng(11)
    grid = CoverageGrid(0.0, 0.0, 5.0, 1.0, 1.0, 1.0, 4, 1, 1)
    recs = []
    for cell, (nb, per) in enumerate([(5, 1), (40, 7), (3, 5000), (200, 3)]):
        for b in rng.choice(9000, nb, replace=False):
            for _ in range(per):
                recs.append((cell, int(b), float(10.0 ** rng.uniform(-25, -2))))
    rng.shuffle(recs)
    cells = np.array([r[0] for r in recs], np.uint64)
    bins = np.array([r[1] for r in recs], np.uint64)
    amps = np.array([r[2] for r in recs], np.float64)
    keys = torch.from_numpy(((cells << np.uint64(32)) | bins).view(np.int64)).cuda()
    cov = Coverage(room, 2.998e8, 100e9, 100e-9, 3, 1000, grid, shard_mode="rays")
    cov.power_from_amplitudes(keys, torch.from_numpy(amps).cuda())
    c, b, a = cov.impulse_responses()
    cov.close()
    unit = Fraction(1, 2 ** 136)
    exact = {}
    for (cc, bb, x) in recs:
        exact[(cc, bb)] = exact.get((cc, bb), 0) + math.floor(Fraction(x) / unit)
    assert len(a) == len(exact)
    for cc, bb, x in zip(c, b, a):
        assert x == float(exact[(int(cc), int(bb))] * unit), (cc, bb)


def test_trace_rows_into_small_buffer_fetches_packed(room):
    """Coverage.trace_rows with a too-small row buffer: rt_coverage_trace_rows_finish reports it,
    and the rows come from rt_coverage_records_packed (no second trace) -- the same rows, in the
    same order, as with a buffer that was large enough."""
    grid, tx, B, N = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2), (10, 0, 5), 3, 60_000
    p = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid, shard_index=0, shard_count=2, shard_mode="rays")
    r1, c1 = p.trace_rows(tx, 1)
    r1 = r1.clone()
    assert sum(c1) > 100
    p._rows = torch.empty((1, 4), dtype=torch.int64, device="cuda")
    r2, c2 = p.trace_rows(tx, 1)
    assert c1 == c2 and p._rows.shape[0] >= sum(c1)
    assert r1.cpu().numpy().tobytes() == r2.cpu().numpy().tobytes()
    p.close()


def _owner_segments_case(room, nseg, sizes, seed):
    """rt_coverage_power_packed on `sizes[c]` random bins per cell c of an nx x 1 x 1 grid, each
    (cell, bin)'s fixed-point amplitude split over up to 3 of nseg source segments (each segment in
    key order), against the sorted path (rt_coverage_power_rows) on the same rows: maps and
    impulse responses bit for bit."""
    rng = np.random.default_rng(seed)
    grid = CoverageGrid(0.0, 0.0, 5.0, 1.0, 1.0, 1.0, len(sizes), 1, 1)
    n, win = 10000, 100e-9
    keys = []
    for c, K in enumerate(sizes):
        for b in np.sort(rng.choice(n, K, replace=False)) if K else []:
            keys.append((c << 32) | int(b))
    keys = np.array(keys, np.uint64)
    cov = Coverage(room, 2.998e8, 100e9, win, 3, 1000, grid, shard_mode="rays")
    amps = torch.from_numpy(rng.uniform(1e-9, 1e-5, len(keys))).cuda()
    from rf_ray_tracing_warp_amd.coverage import amps_to_sums
    full = amps_to_sums(amps).cpu().numpy().view(np.uint64)  # (n, 3) fixed point, w0 least significant
    # split each record's fixed point into parts on distinct random segments (exact: integer limbs)
    seg_rows = [[] for _ in range(nseg)]
    for i, k in enumerate(keys):
        parts = int(rng.integers(1, min(nseg, 3) + 1))
        segs = rng.choice(nseg, parts, replace=False)
        rest = full[i].copy()
        for j, sg in enumerate(segs):
            if j == parts - 1:
                piece = rest.copy()
            else:  # take the low word's low half: no borrow across words
                piece = np.array([rest[0] & np.uint64(0xFFFFFFFF), 0, 0], np.uint64)
                rest = rest - piece
            seg_rows[sg].append((k, piece))
    k_all, s_all, counts = [], [], []
    for rows in seg_rows:
        rows.sort(key=lambda r: int(r[0]))
        counts.append(len(rows))
        k_all += [r[0] for r in rows]
        s_all += [r[1] for r in rows]
    kt = torch.from_numpy(np.array(k_all, np.uint64).view(np.int64)).cuda()
    st = torch.from_numpy(np.array(s_all, np.uint64).reshape(-1, 3).view(np.int64)).cuda()
    rows = torch.cat([kt.reshape(-1, 1), st], dim=1).contiguous()
    got = cov.power_from_rows(rows, counts).cpu().numpy().copy()
    gi = cov.impulse_responses()
    ref = cov.power_from_rows(rows).cpu().numpy().copy()
    ri = cov.impulse_responses()
    cov.close()
    assert got.tobytes() == ref.tobytes()
    assert np.isfinite(ref).sum() == sum(1 for K in sizes if K)
    for x, y in zip(gi, ri):
        assert x.tobytes() == y.tobytes()


@pytest.mark.parametrize("nseg", [1, 3, 8, 9])
def test_owner_segments_every_sweep_path(room, nseg):
    """The owner stage on segments (lockstep merge for <= 8 sources, the general merge above that)
    on cells of 0 .. 9999 bins (every sweep: thread, wave, range-split)."""
    _owner_segments_case(room, nseg, [0, 1, 2, 5, 16, 17, 64, 191, 192, 193, 400, 2500, 9999], 21 + nseg)


@pytest.mark.parametrize("nseg", [2, 8])
def test_owner_segments_many_cells(room, nseg):
    """The segment merge on a 1500-cell map of mostly small cells (0-16 bins: thread sweeps), some
    of 17-200 bins (wave sweeps) and two of 2500 / 3000."""
    rng = np.random.default_rng(5 + nseg)
    sizes = [int(x) for x in rng.choice([0, 0, 1, 2, 3, 5, 8, 16], 1500)]
    for c, K in zip(rng.choice(1500, 40, replace=False), rng.integers(17, 200, 40)):
        sizes[int(c)] = int(K)
    sizes[700], sizes[1201] = 2500, 3000
    _owner_segments_case(room, nseg, sizes, 77 + nseg)


@pytest.mark.parametrize("nseg", [1, 3, 12])
def test_owner_stage_rejects_unordered_segments(room, nseg):
    """Received rows that break the owner stage's precondition (each segment strictly ascending) are
    counted by the merge and reported by Coverage.check (RfrtError) instead of a silently wrong map
    (ADVICE r4); the report clears, and the same rows in key order pass.  nseg 12 takes the
    k_merge_segments path, 1 and 3 k_merge_lockstep."""
    n = 240
    grid = CoverageGrid(0.0, 0.0, 5.0, 1.0, 1.0, 1.0, n, 1, 1)
    cov = Coverage(room, 2.998e8, 100e9, 100e-9, 3, 1000, grid, shard_mode="rays")
    keys = np.array([(c << 32) | 7 for c in range(n)], np.uint64)
    rows = np.zeros((n, 4), np.uint64)
    rows[:, 0] = keys
    rows[:, 1] = 1 << 40
    counts = [n // nseg] * nseg
    counts[-1] += n - sum(counts)
    bad = rows.copy()
    o = counts[0]
    bad[o - 2], bad[o - 1] = rows[o - 1], rows[o - 2]  # two rows of the first segment swapped
    from rf_ray_tracing_warp_amd._lib import RfrtError
    cov.power_from_rows(torch.from_numpy(bad.view(np.int64)).cuda(), counts)
    with pytest.raises(RfrtError, match="out of key order"):
        cov.check()
    cov.check()  # reported once, then cleared
    good = cov.power_from_rows(torch.from_numpy(rows.view(np.int64)).cuda(), counts).cpu().numpy()
    cov.check()
    assert np.isfinite(good).sum() == n
    cov.close()


def _map_and_irs(env, grid, tx, B, N, clear):
    old = os.environ.get("RFRT_COV_CLEAR")
    os.environ["RFRT_COV_CLEAR"] = "1" if clear else "0"  # read at plan creation
    try:
        cov = Coverage(env, 2.998e8, 100e9, 100e-9, B, N, grid)
    finally:
        if old is None:
            os.environ.pop("RFRT_COV_CLEAR")
        else:
            os.environ["RFRT_COV_CLEAR"] = old
    p = cov.run_device(tx).cpu().numpy().copy()
    irs = cov.impulse_responses()
    cov.close()
    return p, irs


@pytest.mark.parametrize("grid,N,least", [
    (CoverageGrid(-0.75, 1.55, 5.0, 0.125, 0.1, 1.0, 12, 10, 1), 20_000, 5),   # across the partition (x in +-0.4, y < 2)
    (CoverageGrid(14.62, -14.95, 0.05, 0.09, 0.1, 0.11, 5, 4, 3), 50_000, 1),  # a corner: wall, wall and floor
])
def test_clear_receivers_equal_full_replay(room, grid, N, least):
    """Cells whose receiver ball holds no environment face skip the replay's environment query while
    the path is inside their receiver (k_clear_cells); cells at or inside walls keep it.  Maps and
    impulse responses equal the replay that always queries (RFRT_COV_CLEAR=0) bit for bit, on grids
    with both kinds of cell, and the oracle's per-cell loop within the coverage bar."""
    tx, B = (10.0, 0.0, 5.0), 3
    p0, i0 = _map_and_irs(room, grid, tx, B, N, clear=False)
    p1, i1 = _map_and_irs(room, grid, tx, B, N, clear=True)
    assert p0.tobytes() == p1.tobytes()
    for x, y in zip(i0, i1):
        assert x.tobytes() == y.tobytes()
    cov = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid)
    power, ref = _compare(cov, grid, room, tx, B, N)
    assert np.isfinite(ref).sum() >= least
    cov.close()


@pytest.mark.parametrize("S", [1, 3])
def test_trace_rows_async_equals_trace_rows(room, S):
    """The two-halves trace stage (trace_rows_async: no host wait, send counts left on the device;
    trace_rows_finish: one wait) gives trace_rows' rows and counts bit for bit, and the device send
    counts equal the host ones; a small first row buffer takes the fetch path in both."""
    grid, tx, B, N = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2), (10, 0, 5), 3, 60_000
    for r in range(S):
        a = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid, shard_index=r, shard_count=S, shard_mode="rays")
        b = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid, shard_index=r, shard_count=S, shard_mode="rays")
        b._rows = torch.empty((16, 4), dtype=torch.int64, device="cuda:0")  # forces the fetch
        for _ in range(2):
            r0, c0 = a.trace_rows(tx, 1)
            r0 = r0.clone()
            sc = b.trace_rows_async(tx, 1)
            r1, c1 = b.trace_rows_finish()
            assert c0 == c1 and sum(c0) > 0
            assert sc.cpu().tolist() == c1
            assert r0.cpu().numpy().tobytes() == r1.cpu().numpy().tobytes()
        a.close()
        b.close()


def test_exchange_counts_async_over_rccl(room):
    """dist.exchange_counts_async on a one-rank "nccl" (RCCL) group: the counts' all-to-all queued
    on the stream and copied to pinned memory, read after one stream wait."""
    import socket
    import torch.distributed as dist
    from rf_ray_tracing_warp_amd import dist as rdist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        assert rdist.device_collectives()
        sc = torch.tensor([12345], dtype=torch.int64, device="cuda:0")
        host = rdist.exchange_counts_async(sc)
        torch.cuda.current_stream().synchronize()
        assert host.is_pinned() and host.tolist() == [12345]
    finally:
        dist.destroy_process_group()


def test_whole_map_sort_after_regrowth_short_list(room):
    """The fault class of round 5 (r5y): k_sel_scatter writes the whole-map replay-order keys at the
    plan's capacity-based workspace layout (rord_key_bytes(cap)), and the replay-order sort must take
    its key / value pointers from the same layout -- a list far shorter than the capacity, after a
    regrowth, read keys from the wrong place (an illegal address).  Here every whole-map list takes
    the device-wide sort over k_sel_scatter's keys (rt_debug_replay_window_max(0); by default only
    one GPU's K3 / K5 maps do).  Run 1: a dense 3-layer grid around the TX overflows the plan's
    initial 2^20 candidates and regrows it.  Run 2, same plan: the TX far away, a few thousand first
    wins against a capacity of millions.  Both maps against the oracle's per-cell loop on sampled
    cells (coverage bar: identical bins, 1e-5 norm-wise impulse responses, 1e-9 power vs the
    rounded-once arccos)."""
    L = lib()
    grid = CoverageGrid(9.2, -0.8, 4.95, 0.05, 0.05, 0.05, 32, 32, 3)
    B, N = 3, 100_000
    E = orc.Mesh(room.vertices, room.faces)
    cen = grid.centers().reshape(-1, 3)
    check(L.rt_debug_replay_window_max(0))
    try:
        cov = Coverage(room, 2.998e8, 100e9, 100e-9, B, N, grid)
        for run, tx in enumerate([(10.0, 0.0, 5.0), (-12.0, 9.0, 11.0)]):
            power = cov.run(tx, 1).reshape(-1)
            cells, bins, amps = cov.impulse_responses()
            if run == 0:
                assert cov.last_candidates > (1 << 20), cov.last_candidates  # the first run regrew the plan
                cap = cov.last_candidates
            else:
                assert 0 < cov.last_first_wins < cap // 20, (cov.last_first_wins, cap)  # nl << cap
            rng = np.random.default_rng(run)
            recv = np.unique(cells)
            picks = np.union1d(rng.choice(recv, min(24, len(recv)), replace=False),
                               rng.choice(grid.num_cells, 6, replace=False))
            for c in picks:
                ref = orc.coverage_cell(E, tx, cen[c], B, N)
                sel = cells == c
                rb = np.nonzero(ref["ir"])[0]
                np.testing.assert_array_equal(bins[sel], rb, err_msg=f"run {run} cell {c}")
                assert np.isnan(power[c]) == np.isnan(ref["power"]), f"run {run} cell {c}"
                if len(rb):
                    assert np.abs(amps[sel] - ref["ir"][rb]).max() <= 1e-5 * np.abs(ref["ir"]).max()
                    np.testing.assert_allclose(power[c], ref["power_cr"], rtol=1e-9, err_msg=f"run {run} cell {c}")
        cov.close()
    finally:
        check(L.rt_debug_replay_window_max(-1))


def test_bench_exits_nonzero_on_an_unordered_segment():
    """bench.py validates its own coverage maps: after the timed maps it asks the plan for the
    device-side error report (Coverage.check), so a received segment out of key order (the owner
    stage's precondition, broken on purpose by --debug-unordered-rows: two rows of a segment
    swapped) ends the run with a non-zero status instead of a rate for a wrong map."""
    import subprocess
    import sys
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--legs", "k2,k3", "--steps", "2", "--warmup", "1",
           "--settle-steps", "0", "--no-cpu-baseline", "--coverage-grid", "32", "--coverage-rays", "50000",
           "--coverage-runs", "1", "--rays", "100000", "--debug-unordered-rows"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "out of key order" in r.stderr, r.stderr[-2000:]
