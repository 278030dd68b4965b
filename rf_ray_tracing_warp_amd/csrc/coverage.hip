// coverage.hip -- coverage.py (coverage.py:38-57) on the device, exact, by shared trajectories.
//
// The reference runs a full Tracer.compute_cir per receiver cell (cells x N x B queries) and then
// main.py/coverage.py's signal power (np.convolve with a sampled 2.4 GHz sine).  Every cell sees
// the same rays (rand_init(tid) depends on tid only, kernel.py:51) and a receiver miss never moves
// the ray (kernel.py:85-98), so for every cell a ray follows its environment-only trajectory
// bit for bit until the first bounce k where that cell's receiver wins (hit, and nearer than the
// environment or the environment missed).  This file:
//
//   k_traj    trace every ray once against the environment only: p_k, d_k, t_env_k (SoA in HBM)
//   k_cols    for every segment (p_k, d_k, [0, min(t_env_k, max_t)]) and z layer: the lattice
//             columns its padded capsule crosses -> column items                      [capsule raster]
//   k_cells   one column item per lane (balanced: a grazing ray's hundreds of cells spread over
//             many lanes): ball test of the few cells of the column -> keys (cell, ray, k)
//   k_win     exact receiver test of each candidate (the cell's icosphere, 80 faces, unrolled) and
//             the first-win check (earlier bounces of the same (cell, ray) re-tested where their
//             segment reaches the cell's ball) -> flags, compacted in order (k_sel_count + k_sel_scatter)
//   k_replay  replay from (p_k, d_k) with the full per-cell semantics of kernel.py:57-98, then the
//             CIR body of tracer.py:101-117 -> record (owner | cell | bin | ray key, amp), in a
//             coherent order (direction x coarse position keys)
// Appends use one atomic per wave (prefix sum of the lanes' counts).
//   sort + reduce-by-key: per-cell sparse impulse response, bins ascending, each bin summed in
//             ray order (the ray is the key's lowest field)
//   k_power   closed-form mean square of the nonzero samples of ir (*) sin(2 pi 2.4e9 t)
//             ('same' mode, np.nonzero) over the piecewise-constant active-bin intervals
//
// Cost: N*B environment queries + (#candidates) receiver tests + (#received) replays, instead of
// cells*N*B*(env + receiver) queries.  Results equal the per-cell reference loop (tests compare
// against the oracle's per-cell trace + NumPy power); cells are sharded by x column (ix % ranks).
#include <hipcub/hipcub.hpp>
#include <math.h>

#include <algorithm>
#include <atomic>
#include <numeric>
#include <vector>

#include "../../include/rfrt.h"
#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_icosphere1.h"
#include "rt_internal.h"

namespace {


struct CovParams {
  const float4* env_perm;
  const float4* env_nrm;
  int env_nf;
  rt::BvhView env_bvh;  // large environments (USE_BVH instantiations)
  float tx[3];
  int B;
  int64_t n;           // rays
  int64_t ray_offset;  // global id of ray 0
  rt_grid g;
  double r_rx;       // receiver radius (tracer.py:26 rx_radius)
  double r_pad;      // conservative ball radius for candidate search
  int shard, nshard;  // cells in x columns ix % nshard == shard are ours
  const int32_t* order;  // k_traj row order (direction-sorted for BVH environments) or null
  unsigned long long* zero_ctr;  // k_traj zeroes these 4 counters for the candidate passes (no fill launch)
  // trajectory SoA [k][n]
  // trajectories, [ray][bounce] x 2 float4: (p.xyz, t_env), (d.xyz, 0) -- 32 B per ray-bounce,
  // so a random (ray, bounce) read or a direction-sorted write touches one or two lines
  float4* traj;
  uint8_t* nseg;
  // column items and candidates (wave-aggregated appends; counts on the device)
  uint64_t* items;
  int64_t item_cap;
  unsigned long long* item_count;
  uint64_t* keys;
  int64_t cap;
  unsigned long long* count;
  // CIR
  double amp0;
  float c32, fs32;
  double c64, fs64;
  int flags;
  int64_t n_bins;
  // record keys (record_key): ray-sharded runs put the owning rank of the record's cell
  // ((cell % nx) % own_world) above the cell, so one sort groups the records by destination
  int own_world, own_shift;
  int bin_bits, cell_bits;
  // per-cell bits (k_clear_cells): no environment face within r_clear of the cell's centre, or null
  const uint32_t* clear;
};
__device__ __forceinline__ float4 traj_p(const CovParams& p, int64_t r, int k) { return p.traj[2 * (r * p.B + k)]; }
__device__ __forceinline__ float4 traj_d(const CovParams& p, int64_t r, int k) { return p.traj[2 * (r * p.B + k) + 1]; }

__device__ __forceinline__ int64_t ncells(const rt_grid& g) { return g.nx * g.ny * g.nz; }

// cell -> (i, j, k) in 32-bit unsigned arithmetic (cells < 2^32, rt_coverage_create): a 64-bit
// division by a run-time divisor is a ~100-instruction sequence on the GPU, and the receiver tests
// of k_win and k_replay take the cell's centre on every query
__device__ __forceinline__ void cell_ijk(const rt_grid& g, int64_t cell, uint32_t& i, uint32_t& j, uint32_t& k) {
  const uint32_t c = (uint32_t)cell, nx = (uint32_t)g.nx, ny = (uint32_t)g.ny;
  const uint32_t q = c / nx;
  i = c - q * nx;
  k = q / ny;
  j = q - k * ny;
}
__device__ __forceinline__ void cell_center(const rt_grid& g, int64_t cell, double c[3]) {
  uint32_t i, j, k;
  cell_ijk(g, cell, i, j, k);
  c[0] = g.x0 + (double)i * g.dx;
  c[1] = g.y0 + (double)j * g.dy;
  c[2] = g.z0 + (double)k * g.dz;
}

// environment closest hit from the LDS table (same code path as the trace kernel)
__device__ __forceinline__ rt::Hit env_query_lds(const float4* tab, int nf, const rt::Shear& s) {
  rt::LazyHit h;  // faces in ascending order: the division waits for the winner (rt_device.h)
  rt::lazy_init(h);
  const int off = s.kcase * 3;
  for (int f = 0; f < nf; ++f) {
    const float4 q0 = tab[f * 18 + off + 0];
    const float4 q1 = tab[f * 18 + off + 1];
    const float c2 = tab[f * 18 + off + 2].x;
    float T, det;
    if (rt::tri_test(s, q0, q1, c2, T, det)) rt::lazy_consider(h, T, det, f);
  }
  return rt::lazy_finish(h);
}

template <bool USE_BVH>
__device__ __forceinline__ rt::Hit env_query(const CovParams& p, const float4* tab, const rt::Shear& s, float3 o,
                                            float3 d, float tcull = RT_MAX_T) {
  if constexpr (USE_BVH) {
    return rt::bvh_query(p.env_bvh, s, o, d, tcull);
  } else {
    return env_query_lds(tab, p.env_nf, s);
  }
}
template <bool USE_BVH>
__device__ __forceinline__ void stage_env(const CovParams& p, float4* lds_tab) {
  if constexpr (!USE_BVH) {
    for (int i = threadIdx.x; i < p.env_nf * 18; i += blockDim.x) lds_tab[i] = p.env_perm[i];
    __syncthreads();
  }
}

// The cell's receiver: vertex i = (float)(unit_i * r + centre) in double, exactly mesh.sphere() +
// astype(float32) (tracer.py:27-28), permuted to the ray's shear axes where a face is tested.
// Three earlier forms of the query gave the same bits -- all 42 vertices in registers (126 live
// floats), three vertices per face recomputed (twice the vertex VALU), and the 12 icosahedron
// corners in registers with each group's midpoints generated (72 vertex evaluations); the culled
// group form below replaced them (K3 map 8.84 / 10.41 / 7.18 -> 5.96 ms); removed in
// round 5, last in commit 43de9a4.
// Faces 4g..4g+3 of icosphere(1) subdivide icosahedron face g (trimesh's subdivide order): with
// the corners c0 c1 c2 (vertex ids < 12) and edge midpoints m01 m12 m20 of face g they are
// (c0 m01 m20), (m01 c1 m12), (m20 m12 c2), (m01 m12 m20).  kIcoGroup[g] = {c0, c1, c2, m01, m12, m20}.
struct IcoGroups {
  int v[RT_ICO1_NF / 4][6];
};
constexpr IcoGroups ico_groups() {
  IcoGroups G{};
  for (int g = 0; g < RT_ICO1_NF / 4; ++g) {
    G.v[g][0] = rt_ico1_f[4 * g][0];
    G.v[g][1] = rt_ico1_f[4 * g + 1][1];
    G.v[g][2] = rt_ico1_f[4 * g + 2][2];
    G.v[g][3] = rt_ico1_f[4 * g][1];
    G.v[g][4] = rt_ico1_f[4 * g + 1][2];
    G.v[g][5] = rt_ico1_f[4 * g][2];
  }
  return G;
}
constexpr IcoGroups kIcoGroup = ico_groups();
constexpr int kGroupFace[4][3] = {{0, 3, 5}, {3, 1, 4}, {5, 4, 2}, {3, 4, 5}};
constexpr bool ico_groups_ok() {
  for (int g = 0; g < RT_ICO1_NF / 4; ++g) {
    for (int j = 0; j < 6; ++j)
      if ((j < 3) != (kIcoGroup.v[g][j] < 12)) return false;
    for (int f = 0; f < 4; ++f)
      for (int k = 0; k < 3; ++k)
        if (rt_ico1_f[4 * g + f][k] != kIcoGroup.v[g][kGroupFace[f][k]]) return false;
  }
  return true;
}
static_assert(ico_groups_ok(), "rt_icosphere1.h is not in trimesh's subdivide order");

// ---- culled receiver query.  The 80 faces come in 20 groups of 4 (one subdivided icosahedron face
// each, kIcoGroup), every group inside a ball (rt_ico1_gball, unit coordinates).  A face the
// watertight test can accept has its triangle within rounding of the ray's line, so a group whose
// ball (radius padded for the f32 vertex and test rounding) the line misses, or which lies wholly
// behind the origin, holds no face that can be hit.  The passing groups are split at the line's
// closest approach to the centre: the near side first; then a far group is needed only if its
// ball's entry t is not beyond the best hit so far (a convex receiver is crossed at most twice, so
// after a near-side hit the far side is usually skipped).  Each lane walks its own groups (~3 on
// average, ~5 for the slowest lane of a wave, against 20 for the full test), with the group's
// vertices computed as make_rx_perm computes them -- (float)(unit * r + centre) in double, the
// products unit * r staged in LDS -- so every hit is bit-identical to rx_query's.
// The shear cases' axis orders (kx, ky, kz) by rt::Shear::kcase = kz * 2 + swap (make_shear).
constexpr int kCaseAxes[6][3] = {{1, 2, 0}, {2, 1, 0}, {2, 0, 1}, {0, 2, 1}, {0, 1, 2}, {1, 0, 2}};
struct RxLds {
  double ur[6][RT_ICO1_NV][4];   // rt_ico1_v * r (make_rx_perm's double product), per shear case in
                                 // that case's (kx, ky, kz) order (w unused): a vertex needs no selects
  uint64_t vid[RT_ICO1_NF / 4];  // the group's vertex ids c0 c1 c2 m01 m12 m20, 6 bits each
  float4 gb[RT_ICO1_NF / 4];     // group ball: centre * r (f32) and radius * r
  float gmw[RT_ICO1_NF / 4];     // |centre * r|^2 - (radius * r)^2
};
__device__ __forceinline__ void stage_rx(RxLds& L, double r) {
  for (int i = threadIdx.x; i < 6 * RT_ICO1_NV * 3; i += blockDim.x) {
    const int kc = i / (RT_ICO1_NV * 3), rem = i % (RT_ICO1_NV * 3), v = rem / 3, k = rem % 3;
    L.ur[kc][v][k] = rt_ico1_v[v][kCaseAxes[kc][k]] * r;
  }
  const float rf = (float)r;
  for (int g = threadIdx.x; g < RT_ICO1_NF / 4; g += blockDim.x) {
    uint64_t w = 0;
    for (int j = 0; j < 6; ++j) w |= (uint64_t)kIcoGroup.v[g][j] << (6 * j);
    L.vid[g] = w;
    const float mx = rt_ico1_gball[g][0] * rf, my = rt_ico1_gball[g][1] * rf, mz = rt_ico1_gball[g][2] * rf;
    const float mw = rt_ico1_gball[g][3] * rf;
    L.gb[g] = make_float4(mx, my, mz, mw);
    L.gmw[g] = (mx * mx + my * my + mz * mz) - mw * mw;
  }
  __syncthreads();
}

// cp: the cell centre in the query's (kx, ky, kz) order.  The vertices come from the LDS table of
// the query's shear case, already in that order: three adds per vertex instead of three adds and
// six selects (K3 map 3.80 -> 3.67 ms, K5 3.61 -> 3.50 ms, bit-identical; r5p / r5q)
__device__ __forceinline__ void rx_group(const RxLds& L, const double cp[3], const rt::Shear& s, int gi, rt::Hit& h) {
  const uint64_t w = L.vid[gi];
  float3 v[6];
  const double(*ur)[4] = L.ur[s.kcase];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int vi = (int)((w >> (6 * j)) & 63);
    const double2 xy = *reinterpret_cast<const double2*>(&ur[vi][0]);
    v[j] = make_float3((float)(xy.x + cp[0]), (float)(xy.y + cp[1]), (float)(ur[vi][2] + cp[2]));
  }
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const float3 a = v[kGroupFace[f][0]], b = v[kGroupFace[f][1]], q = v[kGroupFace[f][2]];
    float T, det;
    if (rt::tri_test(s, make_float4(a.x, a.y, a.z, b.x), make_float4(b.y, b.z, q.x, q.y), q.z, T, det))
      rt::hit_consider(h, T, det, 4 * gi + f);
  }
}

// ROLLED: the 20-group ball test as a loop over the table (constants by scalar loads) instead of
// unrolled -- fewer VGPRs (K3 k_replay 167 -> 125, so 4 waves per SIMD without spills), slower where
// the occupancy does not change (k_win 0.95 -> 1.01 ms, K5 replay 1.23 -> 1.30 ms; r3zc)
// lmask: the groups to consider, when a query on the same line from an earlier origin found them
// already (its line_out: the groups whose padded ball the line passes and that are not wholly
// behind that origin).  A query from a later origin on the line -- a replay that continues through
// its receiver with the direction unchanged -- needs only those groups' origin-dependent tests
// (behind the new origin, near / far): any other group's ball misses the line or lies behind the
// earlier origin, so it holds no face the ray can meet.  The two origins' rounding moves the line by
// ~1e-6 of the coordinates, far inside the pad.
constexpr uint32_t kAllGroups = (1u << (RT_ICO1_NF / 4)) - 1;
template <bool ROLLED = false>
__device__ __forceinline__ rt::Hit rx_query_culled(const RxLds& L, const rt_grid& g, int64_t cell, double r, float3 o,
                                                   float3 d, uint32_t lmask = kAllGroups,
                                                   uint32_t* line_out = nullptr) {
  const rt::Shear s = rt::make_shear(o, d);
  double c[3];
  cell_center(g, cell, c);
  // line geometry in double: t0 = closest approach to the centre, u = centre -> that point
  const double qx = c[0] - o.x, qy = c[1] - o.y, qz = c[2] - o.z;
  const double dd = (double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z;
  const double t0 = (qx * d.x + qy * d.y + qz * d.z) / dd;
  const float ux = (float)(t0 * d.x - qx), uy = (float)(t0 * d.y - qy), uz = (float)(t0 * d.z - qz);
  const float ddf = (float)dd, inv_dd = (float)(1.0 / dd), inv_len = (float)(1.0 / sqrt(dd)), t0f = (float)t0;
  // pad: f32 vertices (half an ulp of the coordinates) and the watertight test's rounding
  const double amax = fmax(fmax(fabs(c[0]), fabs(c[1])), fmax(fabs(c[2]), fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z))));
  const float pad = (float)(1e-3 * r + 2e-5 * (1.0 + amax) + 4e-6 * fabs(t0) * sqrt(dd));
  // Per group, with the unit direction e = d / |d| and u perpendicular to it: the squared distance
  // from the ball centre m to the line is |m - u|^2 - (m.e)^2 = |m|^2 + |u|^2 - 2 m.u - (m.e)^2, and
  // the centre's line parameter is t0 + (m.e) / |d|.  ~20 VALU per group against ~45 for the cross
  // product form (removed in round 5); its f32 rounding (~1e-7 r^2 in the squared distance) is far inside the
  // pad (1e-3 r), so the test stays conservative and every hit is the same.
  (void)ddf;
  (void)inv_dd;
  const float ex = d.x * inv_len, ey = d.y * inv_len, ez = d.z * inv_len;
  // per query: dist^2 <= R^2 with R = m.w + pad is (|m|^2 - m.w^2) + (|u|^2 - pad^2) - 2 m.u - (m.e)^2
  // - 2 pad m.w <= 0; the ball's far end is not behind the origin when m.e + m.w >= -t0 |d| - pad
  const float uq = fmaf(-pad, pad, ux * ux + uy * uy + uz * uz), pad2 = 2.0f * pad;
  const float tback = fmaf(-t0f, (float)sqrt(dd), -pad);
  // an opaque offset per query: otherwise the 100 loop-invariant LDS words are hoisted out of the
  // callers' loops into registers (k_win 129 VGPRs spilled)
  int z = 0;
  asm volatile("" : "+v"(z));
  const float4* gb = L.gb + z;
  const float* gmw = L.gmw + z;
  uint32_t ok_bits = 0, pos_bits = 0;  // groups that pass; groups beyond the closest approach (m.e > 0)
  float far_tmin = INFINITY;           // the nearest ball entry of the passing far groups
  if (lmask == kAllGroups) {
#pragma unroll(ROLLED ? 1 : 4)
    for (int gi = 0; gi < RT_ICO1_NF / 4; ++gi) {
      const float4 m = gb[gi];
      const float me = fmaf(m.x, ex, fmaf(m.y, ey, m.z * ez));
      const float mu = fmaf(m.x, ux, fmaf(m.y, uy, m.z * uz));
      const float v = fmaf(-me, me, fmaf(-2.0f, mu, fmaf(-m.w, pad2, gmw[gi] + uq)));
      const bool ok = (v <= 0.0f) & (me + m.w >= tback);
      ok_bits |= (ok ? 1u : 0u) << gi;
      pos_bits |= (me > 0.0f ? 1u : 0u) << gi;
      if (ok & (me > 0.0f)) far_tmin = fminf(far_tmin, fmaf(me - (m.w + pad), inv_len, t0f));
    }
    if (line_out) *line_out = ok_bits;
  } else {
    for (uint32_t q = lmask; q; q &= q - 1) {
      const int gi = __builtin_ctz(q);
      const float4 m = gb[gi];
      const float me = fmaf(m.x, ex, fmaf(m.y, ey, m.z * ez));
      const bool ok = me + m.w >= tback;
      ok_bits |= (ok ? 1u : 0u) << gi;
      pos_bits |= (me > 0.0f ? 1u : 0u) << gi;
      if (ok & (me > 0.0f)) far_tmin = fminf(far_tmin, fmaf(me - (m.w + pad), inv_len, t0f));
    }
  }
  uint32_t near = ok_bits & ~pos_bits, far = ok_bits & pos_bits;
  // the centre in the query's axis order (rx_group's vertices come permuted from LDS)
  auto pickd = [&](int k) { return k == 0 ? c[0] : (k == 1 ? c[1] : c[2]); };
  const double cp[3] = {pickd(s.kx), pickd(s.ky), pickd(s.kz)};
  rt::Hit h;
  rt::hit_init(h);
  while (near) {
    const int gi = __builtin_ctz(near);
    near &= near - 1;
    rx_group(L, cp, s, gi, h);
  }
  if (far_tmin > h.t) far = 0;  // every far face's t is beyond the near hit (ties kept)
  while (far) {
    const int gi = __builtin_ctz(far);
    far &= far - 1;
    rx_group(L, cp, s, gi, h);
  }
  return h;
}

// Minimum waves per SIMD the coverage kernels are built for (launch bounds).  Unbounded, k_traj<true>
// took 98 VGPRs (4 waves) and k_replay 201 (2 waves); 5 and 3 (96 and 168 VGPRs) measured K5 6.06 ->
// 5.59 ms and K3 6.01 -> 5.60 ms per map; re-measured at the round-2 end (r2zk).  LDS scenes (K3)
// replay at 4 waves with the rolled receiver ball test (125 VGPRs, no spills): K3 replay 2.067 ->
// 1.917 ms (r3zc); BVH scenes keep 3 (the walk stack's 32 KB of LDS and 155 VGPRs).
constexpr int kTrajWaves = 5, kReplayWaves = 4, kReplayWavesBvh = 3;

// ------------------------------------------------------------------ 1. environment trajectories
template <bool USE_BVH>
__global__ __launch_bounds__(256, kTrajWaves) void k_traj(CovParams p) {
  extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
  if (p.zero_ctr && blockIdx.x == 0 && threadIdx.x < 4) p.zero_ctr[threadIdx.x] = 0ull;
  stage_env<USE_BVH>(p, lds_tab);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t ir = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ir < p.n; ir += stride) {
    const int64_t r = p.order ? (int64_t)p.order[ir] : ir;
    float3 dir = rt::ray_dir(p.ray_offset + r);
    float3 pos = make_float3(p.tx[0], p.tx[1], p.tx[2]);
    int nseg = 0;
    for (int k = 0; k < p.B; ++k) {
      const rt::Shear s = rt::make_shear(pos, dir);
      const rt::Hit he = env_query<USE_BVH>(p, lds_tab, s, pos, dir);
      // stored at slot ir, the processing position: the ray's identity downstream is its slot (only
      // the initial direction needs the global id), so a direction-sorted burst writes its
      // trajectories contiguously instead of scattering 32-B pieces over the array
      float4* tp = p.traj + 2 * (ir * p.B + k);
      tp[0] = make_float4(pos.x, pos.y, pos.z, he.face < 0 ? INFINITY : he.t);
      tp[1] = make_float4(dir.x, dir.y, dir.z, 0.0f);
      nseg = k + 1;
      if (he.face < 0) break;  // escapes: this segment is infinite, later iterations repeat the miss
      pos.x = fmaf(dir.x, he.t, pos.x);
      pos.y = fmaf(dir.y, he.t, pos.y);
      pos.z = fmaf(dir.z, he.t, pos.z);
      const float4 n4 = p.env_nrm[he.face];
      const float3 n = make_float3(n4.x, n4.y, n4.z);
      const float sc = 2.0f * rt::dot3(dir, n);
      dir.x = fmaf(-sc, n.x, dir.x);
      dir.y = fmaf(-sc, n.y, dir.y);
      dir.z = fmaf(-sc, n.z, dir.z);
    }
    p.nseg[ir] = (uint8_t)nseg;
  }
}

// k_traj for BVH scenes with few rays (a ray-sharded rank's share): G lanes per ray (4, or 16 for
// the most nearly horizontal quarter), each walking its share of the tree below the root's
// grandchildren (rt::split_init); the group's closest hit is the ray's.  Same trajectories bit for
// bit; the slowest ray's chain of dependent node fetches is split over the lanes.
constexpr int kTrajSplitG = 4;
// 4 waves per SIMD: 120 VGPRs, no spills (5: 96 + 23 spilled); K5 rank of 8 1.204 -> 1.154 ms (r3z)
// Slots [s0, s1) over blocks [0, nblk) of the launch's share (block index b within it).
template <int G>
__device__ __forceinline__ void traj_split_body(const CovParams& p, int64_t s0, int64_t s1, int64_t b, int64_t nblk) {
  constexpr int LG = G == 16 ? 4 : 2;
  const int j = threadIdx.x & (G - 1);
  const int64_t stride = (nblk * blockDim.x) >> LG;
  // every lane of a wave runs the same number of iterations (the shuffles need them all)
  const int64_t nit = (s1 - s0 + stride - 1) / stride;
  for (int64_t it = 0; it < nit; ++it) {
    const int64_t ir = s0 + it * stride + ((b * blockDim.x + threadIdx.x) >> LG);
    const bool valid = ir < s1;
    const int64_t r = valid ? (p.order ? (int64_t)p.order[ir] : ir) : 0;
    float3 dir = rt::ray_dir(p.ray_offset + r);
    float3 pos = make_float3(p.tx[0], p.tx[1], p.tx[2]);
    int nseg = 0;
    bool alive = valid;
    for (int k = 0; k < p.B; ++k) {
      const rt::Shear s = rt::make_shear(pos, dir);
      rt::Walk4 w;
      rt::WalkStack st = rt::make_stack();
      bool active = false;
      if (alive) {
        rt::split_init<G>(w, st, p.env_bvh, s, pos, dir, j);
        active = true;
      } else {
        rt::hit_init(w.h);
        w.tc = RT_MAX_T;
      }
      while (__any(active)) {
        if (active) active = w.step(p.env_bvh, s, st);
        w.tc = fminf(w.tc, rt::group_min_t<G>(w.h.t));  // cull with the group's best hit so far
      }
      const rt::Hit he = rt::group_hit<G>(w.h);
      if (!alive) continue;
      if (j == 0) {
        float4* tp = p.traj + 2 * (ir * p.B + k);  // slot ir, as k_traj
        tp[0] = make_float4(pos.x, pos.y, pos.z, he.face < 0 ? INFINITY : he.t);
        tp[1] = make_float4(dir.x, dir.y, dir.z, 0.0f);
      }
      nseg = k + 1;
      if (he.face < 0) {
        alive = false;  // escapes: this segment is infinite, later iterations repeat the miss
        continue;
      }
      pos.x = fmaf(dir.x, he.t, pos.x);
      pos.y = fmaf(dir.y, he.t, pos.y);
      pos.z = fmaf(dir.z, he.t, pos.z);
      const float4 n4 = p.env_nrm[he.face];
      const float3 n = make_float3(n4.x, n4.y, n4.z);
      const float sc = 2.0f * rt::dot3(dir, n);
      dir.x = fmaf(-sc, n.x, dir.x);
      dir.y = fmaf(-sc, n.y, dir.y);
      dir.z = fmaf(-sc, n.z, dir.z);
    }
    if (valid && j == 0) p.nseg[ir] = (uint8_t)nseg;
  }
}
// The first n1 slots -- the most nearly horizontal rays of the banded order, whose long grazing
// walks set the time -- G1 lanes per ray on blocks [0, nb1) (dispatched first), the rest G2 lanes
// per ray on the other blocks.  A K5 rank of 8 (kernel trace, means over the rank plans): 4 lanes
// for every ray 218-220 us; 16 lanes for the first 3/16, 1/4, 5/16, 3/8, 1/2 of the slots 206,
// 189-192, 203-205, 202, 212 us (r6w, r6x).  (16 lanes for every ray: no faster than 4, round 4.)
constexpr int kTrajSplitWide = 16;   // lanes per ray of the first quarter
constexpr int kTrajWideShare = 4;    // that quarter: slots [0, n / kTrajWideShare)
template <int G1, int G2>
__global__ __launch_bounds__(256, 4) void k_traj_split(CovParams p, int64_t n1, unsigned nb1) {
  if (p.zero_ctr && blockIdx.x == 0 && threadIdx.x < 4) p.zero_ctr[threadIdx.x] = 0ull;
  if (blockIdx.x < nb1) traj_split_body<G1>(p, 0, n1, blockIdx.x, nb1);
  else traj_split_body<G2>(p, n1, p.n, blockIdx.x - nb1, gridDim.x - nb1);
}

// k_traj for brute-force scenes with few rays (a ray-sharded rank's share, kTrajLdsSplit): G
// lanes per ray, lane j testing the faces f = j, j + G, ... of the LDS table (ascending, so the
// deferred division's order rule holds within the lane); the lexicographic (t, face) minimum of the
// G lanes (group_hit) is the ray's closest hit, bit for bit the one-lane loop's.  A K3 rank of 8
// has 125k rays: one lane per ray is ~490 waves for 1024 SIMDs, and the kernel took as long as one
// wave's 3 x 44 face tests (41 us against 20 for an eighth of the one-GPU pass).
constexpr int kTrajLdsSplit = 4;
template <int G>
__global__ __launch_bounds__(256) void k_traj_lds_split(CovParams p) {
  extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
  constexpr int LG = G == 8 ? 3 : (G == 4 ? 2 : 1);
  static_assert(G == 2 || G == 4 || G == 8, "2, 4 or 8 lanes per ray");
  if (p.zero_ctr && blockIdx.x == 0 && threadIdx.x < 4) p.zero_ctr[threadIdx.x] = 0ull;
  stage_env<false>(p, lds_tab);
  const int j = threadIdx.x & (G - 1);
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> LG;
  const int64_t nit = (p.n + stride - 1) / stride;  // every lane of a wave runs the same iterations
  for (int64_t it = 0; it < nit; ++it) {
    const int64_t ir = it * stride + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> LG);
    const bool valid = ir < p.n;
    const int64_t r = valid ? (p.order ? (int64_t)p.order[ir] : ir) : 0;
    float3 dir = rt::ray_dir(p.ray_offset + r);
    float3 pos = make_float3(p.tx[0], p.tx[1], p.tx[2]);
    int nseg = 0;
    bool alive = valid;
    for (int k = 0; k < p.B; ++k) {
      const rt::Shear s = rt::make_shear(pos, dir);
      rt::LazyHit lh;
      rt::lazy_init(lh);
      if (alive) {
        const int off = s.kcase * 3;
        for (int f = j; f < p.env_nf; f += G) {
          const float4 q0 = lds_tab[f * 18 + off + 0];
          const float4 q1 = lds_tab[f * 18 + off + 1];
          const float c2 = lds_tab[f * 18 + off + 2].x;
          float T, det;
          if (rt::tri_test(s, q0, q1, c2, T, det)) rt::lazy_consider(lh, T, det, f);
        }
      }
      const rt::Hit he = rt::group_hit<G>(rt::lazy_finish(lh));
      if (!alive) continue;
      if (j == 0) {
        float4* tp = p.traj + 2 * (ir * p.B + k);  // slot ir, as k_traj
        tp[0] = make_float4(pos.x, pos.y, pos.z, he.face < 0 ? INFINITY : he.t);
        tp[1] = make_float4(dir.x, dir.y, dir.z, 0.0f);
      }
      nseg = k + 1;
      if (he.face < 0) {
        alive = false;  // escapes: this segment is infinite, later iterations repeat the miss
        continue;
      }
      pos.x = fmaf(dir.x, he.t, pos.x);
      pos.y = fmaf(dir.y, he.t, pos.y);
      pos.z = fmaf(dir.z, he.t, pos.z);
      const float4 n4 = p.env_nrm[he.face];
      const float3 n = make_float3(n4.x, n4.y, n4.z);
      const float sc = 2.0f * rt::dot3(dir, n);
      dir.x = fmaf(-sc, n.x, dir.x);
      dir.y = fmaf(-sc, n.y, dir.y);
      dir.z = fmaf(-sc, n.z, dir.z);
    }
    if (valid && j == 0) p.nseg[ir] = (uint8_t)nseg;
  }
}

// ------------------------------------------------------------------ 2. candidate cells per segment
// One atomic per 256-thread block: exclusive prefix of the threads' counts (wave scan + LDS),
// thread 0 reserves the block's total.  Every thread of the block must call it (inactive: c = 0);
// one same-address atomic per wave measured 1.6 ms for 8.5M keys, per block it is 4x fewer.
__device__ __forceinline__ unsigned long long block_append(unsigned long long* ctr, unsigned c, unsigned& prefix) {
  __shared__ unsigned wsum[4];
  __shared__ unsigned long long bbase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  unsigned before = 0;
  for (int j = 0; j < w; ++j) before += wsum[j];
  if (threadIdx.x == 0) {
    const unsigned total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    bbase = total ? atomicAdd(ctr, (unsigned long long)total) : 0ull;
  }
  __syncthreads();
  prefix = before + x - c;
  const unsigned long long b = bbase;
  __syncthreads();  // wsum / bbase are reused by the next call
  return b;
}

// does the segment x(t) = o + t d, t in [0, tmax] pass within rp of centre c?  (double, conservative)
__device__ __forceinline__ bool seg_ball(const double o[3], const double d[3], double tmax, const double c[3],
                                         double rp2) {
  const double w0 = c[0] - o[0], w1 = c[1] - o[1], w2 = c[2] - o[2];
  const double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
  double t = (w0 * d[0] + w1 * d[1] + w2 * d[2]) / dd;
  t = t < 0.0 ? 0.0 : (t > tmax ? tmax : t);
  const double e0 = o[0] + t * d[0] - c[0], e1 = o[1] + t * d[1] - c[1], e2 = o[2] + t * d[2] - c[2];
  return e0 * e0 + e1 * e1 + e2 * e2 <= rp2;
}

__device__ __forceinline__ int64_t clampi(int64_t v, int64_t lo, int64_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

// t-interval of the segment inside |x_axis(t) - c| <= rp  intersected with [t0, t1]
__device__ __forceinline__ bool slab(double o, double d, double c, double rp, double& t0, double& t1) {
  if (fabs(d) < 1e-300) return fabs(o - c) <= rp;
  double a = (c - rp - o) / d, b = (c + rp - o) / d;
  if (a > b) {
    const double t = a;
    a = b;
    b = t;
  }
  t0 = fmax(t0, a);
  t1 = fmin(t1, b);
  return t0 <= t1;
}

// geometry of one segment (shared by k_cols and k_cells so both see identical doubles)
struct Seg {
  double o[3], d[3], tmax;
  int A, Bx;  // walk axis (major of |d.x|, |d.y|) and cross axis
};
__device__ __forceinline__ Seg load_seg(const CovParams& p, int64_t r, int k) {
  Seg s;
  const float4 tp = traj_p(p, r, k), td = traj_d(p, r, k);
  s.o[0] = tp.x;
  s.o[1] = tp.y;
  s.o[2] = tp.z;
  s.d[0] = td.x;
  s.d[1] = td.y;
  s.d[2] = td.z;
  const double te = tp.w;
  s.tmax = te < (double)RT_MAX_T ? te : (double)RT_MAX_T;
  s.A = fabs(s.d[0]) >= fabs(s.d[1]) ? 0 : 1;
  s.Bx = 1 - s.A;
  return s;
}
// column range of layer kz: [ia0, ia1] (empty if ia0 > ia1), t-range of the layer slab in ta, tb
__device__ __forceinline__ void seg_columns(const CovParams& p, const Seg& s, int64_t kz, double& ta, double& tb,
                                            int64_t& ia0, int64_t& ia1) {
  const rt_grid& g = p.g;
  const double rp = p.r_pad;
  ia0 = 1;
  ia1 = 0;
  ta = 0.0;
  tb = s.tmax;
  if (!slab(s.o[2], s.d[2], g.z0 + (double)kz * g.dz, rp, ta, tb)) return;
  const double a0 = s.A == 0 ? g.x0 : g.y0, da = s.A == 0 ? g.dx : g.dy;
  const int64_t na = s.A == 0 ? g.nx : g.ny;
  const double qa0 = s.o[s.A] + ta * s.d[s.A], qa1 = s.o[s.A] + tb * s.d[s.A];
  const double amin = fmin(qa0, qa1) - rp, amax = fmax(qa0, qa1) + rp;
  if ((amax - a0) / da < -1.0 || (amin - a0) / da > (double)na) return;
  ia0 = clampi((int64_t)floor((amin - a0) / da), 0, na - 1);
  ia1 = clampi((int64_t)ceil((amax - a0) / da), 0, na - 1);
}

// Cells are owned by x column: ix % nshard == shard.  A strip of fixed ix (s.A == 0) is either
// wholly ours or not: advance ia0 to the first owned strip and step by nshard.  Strips of fixed
// iy (s.A == 1) are all kept; column_cells steps through their owned ix instead.
__device__ __forceinline__ void owned_strips(const CovParams& p, const Seg& s, int64_t& ia0, int64_t& step) {
  step = 1;
  if (p.nshard > 1 && s.A == 0) {
    ia0 += ((p.shard - ia0 % p.nshard) % p.nshard + p.nshard) % p.nshard;
    step = p.nshard;
  }
}

// pass A: per ray, the (segment, layer, column) items.  item = r<<40 | k<<36 | kz<<24 | ia
// Each lane finds its ray's column spans (<= B segments x nz layers) and keeps them in LDS, the block
// reserves its range with one atomic, and then all 256 threads write the block's items together:
// item q of the block belongs to the lane whose exclusive prefix is the last one <= q (a binary
// search over the lanes' prefixes in LDS) and to that lane's span whose start is the last one <= q.
// (Each lane writing its own items serially made a wave last as long as its longest ray: up to ~770
// stores for a segment across the whole room; K3 rank of 8 49 us for 125k rays.)  Plans with more
// than kColSpans spans per ray (B x nz) keep the serial writes.
constexpr int kColSpans = 4;
struct ColSpan {
  int32_t ia0;   // first column
  uint32_t n;    // columns
  uint32_t tag;  // step << 16 | k << 12 | kz
};
// Rows are visited in groups of kColGroup consecutive trajectory slots, group g at slot group
// (g * gstep) % ngroups (gstep coprime to ngroups, ~ngroups / 16): a block's 16 groups sample the
// whole burst.  The items' order is the append order either way (one atomic per block), so only the
// load balance changes: in the direction-banded order of a sector shard the long, nearly horizontal
// segments -- hundreds of columns each -- are the first slots, and consecutive slots put them all
// into the same few blocks (K3 rank of 8: 82 us, against 22 us with slots in ray-id order).
constexpr int kColGroup = 16;
__global__ __launch_bounds__(256) void k_cols(CovParams p, int64_t ngroups, int64_t gstep) {
  __shared__ uint32_t s_pre[256];  // the lanes' exclusive item prefixes in the block
  __shared__ uint32_t s_tot;
  __shared__ int64_t s_row[256];
  __shared__ ColSpan s_span[kColSpans][256];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool spans_ok = (int64_t)p.B * p.g.nz <= kColSpans && p.g.nz <= 4096 && p.nshard < 65536;
  const int64_t nslots = ngroups * kColGroup;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < nslots; base += stride) {
    const int64_t i = base + threadIdx.x;
    const int64_t r = (i / kColGroup * gstep) % ngroups * kColGroup + i % kColGroup;
    const bool active = i < nslots && r < p.n;
    unsigned c = 0;
    int nsp = 0;
    const int ns = active ? p.nseg[r] : 0;
    for (int k = 0; k < ns; ++k) {
      const Seg s = load_seg(p, r, k);
      for (int64_t kz = 0; kz < p.g.nz; ++kz) {
        double ta, tb;
        int64_t ia0, ia1;
        seg_columns(p, s, kz, ta, tb, ia0, ia1);
        int64_t step;
        owned_strips(p, s, ia0, step);
        if (ia1 >= ia0) {
          const unsigned n = (unsigned)((ia1 - ia0) / step + 1);
          if (spans_ok) s_span[nsp++][threadIdx.x] = ColSpan{(int32_t)ia0, n, (uint32_t)(step << 16 | k << 12 | kz)};
          c += n;
        }
      }
    }
    if (spans_ok)
      for (int j = nsp; j < kColSpans; ++j) s_span[j][threadIdx.x].n = 0u;
    unsigned pre;
    const unsigned long long at = block_append(p.item_count, c, pre);
    if (!spans_ok) {
      int64_t w = (int64_t)(at + pre);
      for (int k = 0; k < ns; ++k) {
        const Seg s = load_seg(p, r, k);
        for (int64_t kz = 0; kz < p.g.nz; ++kz) {
          double ta, tb;
          int64_t ia0, ia1;
          seg_columns(p, s, kz, ta, tb, ia0, ia1);
          int64_t step;
          owned_strips(p, s, ia0, step);
          for (int64_t ia = ia0; ia <= ia1; ia += step, ++w)
            if (w < p.item_cap)
              p.items[w] = ((uint64_t)r << 40) | ((uint64_t)k << 36) | ((uint64_t)kz << 24) | (uint64_t)ia;
        }
      }
      continue;
    }
    s_pre[threadIdx.x] = pre;
    s_row[threadIdx.x] = r;
    if (threadIdx.x == 255) s_tot = pre + c;
    __syncthreads();
    const uint32_t tot = s_tot;
    for (uint32_t q = threadIdx.x; q < tot; q += blockDim.x) {
      int lo = 0, hi = 255;  // last lane with s_pre <= q
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= q) lo = mid;
        else hi = mid - 1;
      }
      uint32_t off = q - s_pre[lo];  // the item's index in lane lo's list
      int j = 0;
      while (j + 1 < kColSpans && off >= s_span[j][lo].n) off -= s_span[j++][lo].n;
      const ColSpan sp = s_span[j][lo];
      const int64_t w = (int64_t)at + q;
      if (w < p.item_cap) {
        const uint64_t k = (sp.tag >> 12) & 15u, kz = sp.tag & 0xFFFu, step = sp.tag >> 16;
        p.items[w] = ((uint64_t)s_row[lo] << 40) | (k << 36) | (kz << 24) | (uint64_t)(sp.ia0 + (int64_t)off * step);
      }
    }
    __syncthreads();  // s_pre, s_tot and the spans are rewritten by the next block-row
  }
}

// pass B: one column item per lane -> candidate keys (cell, ray, k) for the cells of our shard
// sink(j, key) receives the item's j-th candidate key
template <typename Sink>
__device__ __forceinline__ unsigned column_cells(const CovParams& p, uint64_t item, Sink sink) {
  const rt_grid& g = p.g;
  const double rp = p.r_pad, rp2 = rp * rp;
  const int64_t r = (int64_t)(item >> 40), ia = (int64_t)(item & 0xFFFFFF), kz = (int64_t)((item >> 24) & 0xFFF);
  const int k = (int)((item >> 36) & 15);
  const Seg s = load_seg(p, r, k);
  double ta, tb;
  int64_t ia0, ia1;
  seg_columns(p, s, kz, ta, tb, ia0, ia1);
  const double a0 = s.A == 0 ? g.x0 : g.y0, da = s.A == 0 ? g.dx : g.dy;
  const double b0 = s.Bx == 0 ? g.x0 : g.y0, db = s.Bx == 0 ? g.dx : g.dy;
  const int64_t nb = s.Bx == 0 ? g.nx : g.ny;
  double t0 = ta, t1 = tb;
  unsigned c = 0;
  if (!slab(s.o[s.A], s.d[s.A], a0 + (double)ia * da, rp, t0, t1)) return 0;
  const double qb0 = s.o[s.Bx] + t0 * s.d[s.Bx], qb1 = s.o[s.Bx] + t1 * s.d[s.Bx];
  const double bmin = fmin(qb0, qb1) - rp, bmax = fmax(qb0, qb1) + rp;
  if ((bmax - b0) / db < -1.0 || (bmin - b0) / db > (double)nb) return 0;
  const int64_t ib0 = clampi((int64_t)floor((bmin - b0) / db), 0, nb - 1);
  const int64_t ib1 = clampi((int64_t)ceil((bmax - b0) / db), 0, nb - 1);
  int64_t ibs = ib0, step = 1;
  if (p.nshard > 1 && s.A == 1) {  // ib = ix: visit our columns only
    ibs += ((p.shard - ib0 % p.nshard) % p.nshard + p.nshard) % p.nshard;
    step = p.nshard;
  }
  for (int64_t ib = ibs; ib <= ib1; ib += step) {
    const int64_t ix = s.A == 0 ? ia : ib, iy = s.A == 0 ? ib : ia;
    const int64_t cell = (kz * g.ny + iy) * g.nx + ix;
    // cell_center's values from the indices at hand (its divisions recover exactly these)
    const double cc[3] = {g.x0 + (double)ix * g.dx, g.y0 + (double)iy * g.dy, g.z0 + (double)kz * g.dz};
    if (seg_ball(s.o, s.d, s.tmax, cc, rp2)) {
      sink(c, ((uint64_t)cell << 28) | ((uint64_t)r << 4) | (uint64_t)k);
      ++c;
    }
  }
  return c;
}

// One pass: an item's keys are kept in the thread's LDS slots while the block reserves its
// output range; only items with more than kCellBuf candidates run the geometry a second time.
constexpr int kCellBuf = 8;  // 16 KB of LDS per block instead of 32 (r2zj: candidates stage 0.640 -> 0.636 ms on K3, 0.49 -> 0.48 on K5)

// Items per thread between two appends: every append is one atomic on the device-wide candidate
// counter, and same-address atomics serialize (~10 ns each): one item per thread made k_cells a
// chain of ~35k appends on a whole map (K3 map 426 us, K5 314 us; ranks 59 / 45 us).  Four items
// per thread on whole maps (K3 185, K5 188 us), two on a rank's ~1M items (K3 35, K5 30 us: four
// left too few blocks for a rank's items; r6ze).  Eight were slower (K3 map 305 us: the thread's
// LDS slots overflow, and the overflowing items run their geometry twice).
constexpr int kCellsQMax = 4;
constexpr int64_t kCellsQ4Items = 4 << 20;  // column items from which four per thread
__global__ __launch_bounds__(256) void k_cells(CovParams p) {
  __shared__ uint64_t sbuf[kCellBuf][256];
  const int64_t nitems = (int64_t)min(*p.item_count, (unsigned long long)p.item_cap);
  const int qn = nitems >= kCellsQ4Items ? 4 : 2;  // grid-uniform
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * qn;
  const int tid = threadIdx.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * qn; base < nitems; base += stride) {
    uint64_t item[kCellsQMax];
    unsigned cq[kCellsQMax];
    unsigned c = 0;
#pragma unroll
    for (int q = 0; q < kCellsQMax; ++q) {
      const int64_t i = base + q * 256 + tid;
      const bool active = q < qn && i < nitems;
      item[q] = active ? p.items[i] : 0;
      const unsigned c0 = c;
      cq[q] = active ? column_cells(p, item[q], [&](unsigned j, uint64_t key) {
        if (c0 + j < (unsigned)kCellBuf) sbuf[c0 + j][tid] = key;
      }) : 0;
      c += cq[q];
    }
    unsigned pre;
    const unsigned long long at = block_append(p.count, c, pre);
    if (c && (int64_t)(at + pre + c) <= p.cap) {
      uint64_t* dst = p.keys + at + pre;
      if (c <= (unsigned)kCellBuf) {
        for (unsigned j = 0; j < c; ++j) dst[j] = sbuf[j][tid];
      } else {
        unsigned off = 0;
#pragma unroll
        for (int q = 0; q < kCellsQMax; ++q) {
          if (cq[q]) column_cells(p, item[q], [&](unsigned j, uint64_t key) { dst[off + j] = key; });
          off += cq[q];
        }
      }
    }
  }
}

// np.dot / norm on float32 3-vectors and _bounce_amplitude (tracer.py:106-113), as cir.hip
__device__ __forceinline__ float npdot(const float* a, const float* b) {
  const float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2];
  return (float)(((double)p0 + (double)p1) + (double)p2);
}
// cos(asin(x)) is evaluated as sqrt(1 - x^2) (|x| <= 1/5, so the root is >= 0.979 and the
// identity costs ~1 ulp) and theta's sine and cosine come from one sincos -- the replay's per-vertex
// f64 work without the arcsine and one cosine (K3 replay 2.50 -> 2.35 ms, r2zh).  Amplitudes move by
// ~1e-16 relative, far inside the 1e-9 the coverage tests hold the device to.
// sincos_q1: sin and cos of x in [0, pi/2 + 1e-6] (bounce_amp's theta): one Cody-Waite step against
// pi/2 above pi/4 (x - pio2_1 is exact there), then the classic fdlibm kernels on [-pi/4, pi/4]
// (< 1 ulp).  ocml's general sincos carries the large-argument (Payne-Hanek) reduction, whose
// registers k_replay cannot afford beside its other f64 work (18 VGPRs spilled, 76 B scratch per lane).
__device__ __forceinline__ void sincos_q1(double x, double& s, double& c) {
  const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
  const bool hi = x > 0.78539816339744828;
  const double a = hi ? x - pio2_1 : x;  // exact
  const double r = hi ? a - pio2_1t : a;
  const double rl = hi ? (a - r) - pio2_1t : 0.0;
  const double z = r * r, w = z * z;
  // __kernel_sin(r, rl, 1)
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
               S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double sr = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  const double v = z * r;
  const double sk = r - ((z * (0.5 * rl - v * sr) - rl) - v * S1);
  // __kernel_cos(r, rl)
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
               C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double cr = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z, cw = 1.0 - hz;
  const double ck = cw + (((1.0 - cw) - hz) + (z * cr - r * rl));
  s = hi ? ck : sk;   // x = pi/2 + r: sin x = cos r, cos x = -sin r
  c = hi ? -sk : ck;
}
__device__ __forceinline__ double bounce_amp(float angle) {
  if (isnan(angle)) return 0.0;
  const double theta = (double)(1.57079637050628662109375f - angle / 2.0f);
  double st, ct;
  sincos_q1(theta, st, ct);
  const double x = st / 5.0;
  const double cti = sqrt(1.0 - x * x);
  const double q = (cti - 5.0 * ct) / (cti + 5.0 * ct);
  double amp = -(q * q);
  if (amp < -1.0) amp = -1.0;
  if (isnan(amp)) return 0.0;
  return -amp;
}

// Incremental form of tracer.py:104-113 for a path that grows one point at a time: distance is
// the ordered float32 sum of segment norms, amplitude the ordered product of _bounce_amplitude over
// interior vertices -- identical operations to the loop over (p1, p2, p3) triples.  The amplitude
// is deferred: during the bounce loop each interior vertex's cosine (the f32 value acos is taken of)
// goes to the thread's LDS column, and the f64 product of _bounce_amplitude factors is formed after
// the loop, in the same vertex order -- the same multiplications of the same values, so the same
// bits.  The f64 acos and sincos then no longer add their registers to the queries' live state:
// k_replay<false> spilled 21 VGPRs (88 B of scratch per lane) with them inside the loop.
// A path has at most B + 1 points (the TX, then one per bounce), so at most B - 1 interior vertices.
struct PathAccD {
  float prev[3], seg[3];
  float* cosv;  // this thread's LDS column: interior vertex i's cosine at cosv[256 * i]
  int npts, nint, ncap;
  float dist;
  __device__ __forceinline__ void start(float x, float y, float z) {
    prev[0] = x;
    prev[1] = y;
    prev[2] = z;
    npts = 1;
    nint = 0;
    dist = 0.0f;
  }
  __device__ __forceinline__ void add(float x, float y, float z) {
    const float s2[3] = {x - prev[0], y - prev[1], z - prev[2]};
    if (npts >= 2) {  // vertex prev is interior: angle between seg (p1->p2) and s2 (p2->p3)
      const float l1 = sqrtf(npdot(seg, seg));
      if (nint < ncap) cosv[256 * nint] = npdot(seg, s2) / (l1 * sqrtf(npdot(s2, s2)));
      ++nint;
    }
    dist += sqrtf(npdot(s2, s2));
    seg[0] = s2[0];
    seg[1] = s2[1];
    seg[2] = s2[2];
    prev[0] = x;
    prev[1] = y;
    prev[2] = z;
    ++npts;
  }
};
// The factor of a vertex whose cosine is one of the kAmpTab floats at and just below 1 -- a path
// through a receiver (its entry point is collinear with the points either side: the cosine
// rounds to 1 or a few ulp below it) -- comes from a table that each block fills with the same
// function of the same values, so the bits are the same; other cosines evaluate it.
constexpr int kAmpTab = 128;
__device__ __forceinline__ void stage_amp_tab(double* tab) {
  for (int i = threadIdx.x; i < kAmpTab; i += blockDim.x)
    tab[i] = bounce_amp((float)acos((double)__uint_as_float(0x3F800000u - (uint32_t)i)));
}
// amp0 times the factors of the first n interior vertices, in path order (tracer.py:104-113)
__device__ __forceinline__ double amp_product(const float* cosv, int n, double amp0, const double* tab) {
  double amp = amp0;
#pragma unroll 1
  for (int i = 0; i < n; ++i) {
    const float c = cosv[256 * i];
    const uint32_t u = 0x3F800000u - __float_as_uint(c);  // ulps below 1 (wraps for c > 1, c < 0, NaN)
    amp *= u < (uint32_t)kAmpTab ? tab[u] : bounce_amp((float)acos((double)c));
  }
  return amp;
}

// ------------------------------------------------------------------ 3-4. receiver test, first win, replay
// Record key (compact): [owner | cell | bin] with the field widths of CovParams.  Sorting it groups
// the records by destination rank, then (cell, bin); the bins are summed exactly (Fx192), so the
// order of the records within a bin -- tracer.py:116 adds them in ray order -- cannot matter.
// With several owners the cell field is the cell's index among its owner's cells,
// (rest * nxo + ix / own_world) with nxo = ceil(nx / own_world): bits_for(ncell / world) instead of
// bits_for(ncell), so a K3 rank's key is 30 bits (3 radix passes) instead of 33 (4).
__device__ __forceinline__ uint64_t record_key(const CovParams& p, int64_t cell, int64_t bin) {
  uint64_t own = 0, lc = (uint64_t)cell;
  if (p.own_world > 1) {
    const uint32_t nx = (uint32_t)p.g.nx, w = (uint32_t)p.own_world, c = (uint32_t)cell;
    const uint32_t rest = c / nx, ix = c - rest * nx, nxo = (nx + w - 1) / w, iq = ix / w;
    own = (uint64_t)(ix - iq * w);
    lc = (uint64_t)rest * nxo + iq;
  }
  return (own << p.cell_bits | lc) << p.bin_bits | (uint64_t)bin;
}

// Does the receiver of `cell` win bounce k of ray r (kernel.py:85: hit, and the environment missed
// or is strictly farther)?  tr: the receiver's t.
__device__ __forceinline__ bool rx_wins(const CovParams& p, const RxLds& L, int64_t cell, int64_t r, int k,
                                        float& tr, uint32_t* line_out) {
  const float4 tp = traj_p(p, r, k), td = traj_d(p, r, k);
  const rt::Hit hr = rx_query_culled(L, p.g, cell, p.r_rx, make_float3(tp.x, tp.y, tp.z), make_float3(td.x, td.y, td.z),
                                     kAllGroups, line_out);
  tr = hr.t;
  return hr.face >= 0 && (isinf(tp.w) || tp.w > hr.t);
}

// The first bounce at which the receiver of `cell` wins is the one replayed.  A candidate
// (cell, r, k) exists for exactly the segments whose padded capsule reaches the cell's ball
// (column_cells' final seg_ball test on the same doubles), so an earlier winning bounce k' < k can
// only be a segment passing seg_ball: k_win re-tests those (rare; k < B).

// Replay of (cell, r) from its first winning bounce k0 (receiver t = tr) with the full per-cell
// semantics of kernel.py:57-98, then the CIR body of tracer.py:101-117: the record's key (~0 when
// the path adds nothing: delay past the window, or amplitude 0) and amplitude.
template <bool USE_BVH, bool RX_FIRST>
__device__ __forceinline__ void replay(const CovParams& p, const float4* lds_tab, const RxLds& L, const double* amp_tab,
                                       int64_t cell, int64_t r, int k0, float tr, uint32_t line, uint64_t& okey,
                                       double& oamp) {
  // the B - 1 columns after the environment table in dynamic LDS (k_replay's launch sizes it)
  PathAccD acc;
  acc.cosv = reinterpret_cast<float*>(const_cast<float4*>(lds_tab) + (USE_BVH ? 0 : (size_t)p.env_nf * 18)) + threadIdx.x;
  acc.ncap = p.B - 1;
  const float4 t0 = traj_p(p, r, 0);
  acc.start(t0.x, t0.y, t0.z);  // p_0 = tx
  for (int q = 1; q <= k0; ++q) {       // environment prefix p_1 .. p_k0
    const float4 tq = traj_p(p, r, q);
    acc.add(tq.x, tq.y, tq.z);
  }
  const float4 tk = traj_p(p, r, k0), tdk = traj_d(p, r, k0);
  float3 pos = make_float3(tk.x, tk.y, tk.z);
  const float3 dir = make_float3(tdk.x, tdk.y, tdk.z);
  // bounce k0: the receiver wins at t = tr
  pos.x = fmaf(dir.x, tr, pos.x);
  pos.y = fmaf(dir.y, tr, pos.y);
  pos.z = fmaf(dir.z, tr, pos.z);
  acc.add(pos.x, pos.y, pos.z);
  float rec_dist = acc.dist;
  int rec_nint = acc.nint;
  float3 d = dir;
  // Clear receiver (k_clear_cells: no environment face within r_clear of the centre).  While pos is
  // a hit on this cell's receiver, a receiver hit at t means the segment pos -> hit lies inside the
  // ball (both ends on the icosphere, which is convex and inside the ball), so no environment face
  // can be hit at t' <= t: the receiver wins (kernel.py:85) whatever the environment query returns,
  // and it is skipped.  The typical record -- first win on entering the ball, the exit at the next
  // bounce -- then needs no environment query at all.
  const bool clear = p.clear && ((p.clear[(uint64_t)cell >> 5] >> (cell & 31)) & 1u);
  bool inside = true;  // pos is a hit on this cell's receiver (the first win)
  // while no environment hit has turned the ray, it is still on the first win's line: the receiver
  // query needs only the groups that line passes (k_win found them)
  uint32_t lmask = line ? line : kAllGroups;
  for (int b = k0 + 1; b < p.B; ++b) {  // kernel.py:57-98 with this cell's receiver
    const rt::Shear s = rt::make_shear(pos, d);
    rt::Hit he, hr;
    // receiver first: at the last bounce only a receiver hit can still change the record, so a
    // miss there ends the path without the environment query (K3: most first wins at bounce 0
    // leave their receiver at bounce 1 and miss it at bounce 2)
    hr = USE_BVH ? rx_query_culled(L, p.g, cell, p.r_rx, pos, d, lmask)
                 : rx_query_culled<true>(L, p.g, cell, p.r_rx, pos, d, lmask);
    if (hr.face < 0 && b + 1 >= p.B) break;
    if (clear && inside && hr.face >= 0) {
      pos.x = fmaf(d.x, hr.t, pos.x);
      pos.y = fmaf(d.y, hr.t, pos.y);
      pos.z = fmaf(d.z, hr.t, pos.z);
      acc.add(pos.x, pos.y, pos.z);
      rec_dist = acc.dist;
      rec_nint = acc.nint;
      continue;
    }
    if constexpr (RX_FIRST) {
      // the environment culled at the receiver's t: every environment hit with t <= hr.t is
      // still found exactly (rt_bvh.h), and one beyond it loses to the receiver whatever it is
      // (kernel.py:85), so the decision and the chosen hit are unchanged
      he = env_query<USE_BVH>(p, lds_tab, s, pos, d, hr.face >= 0 ? hr.t : RT_MAX_T);
    } else {
      he = env_query<USE_BVH>(p, lds_tab, s, pos, d);
    }
    const bool env_hit = he.face >= 0, rx_hit = hr.face >= 0;
    if (rx_hit && (!env_hit || he.t > hr.t)) {
      pos.x = fmaf(d.x, hr.t, pos.x);
      pos.y = fmaf(d.y, hr.t, pos.y);
      pos.z = fmaf(d.z, hr.t, pos.z);
      acc.add(pos.x, pos.y, pos.z);
      rec_dist = acc.dist;  // received_paths = traced prefix through this point (kernel.py:89-90)
      rec_nint = acc.nint;
      inside = true;
    } else if (env_hit) {
      inside = false;
      lmask = kAllGroups;  // reflected: a new line
      // after the last bounce only a receiver hit could still change the record: an environment
      // hit there ends the path, its vertex (and its angle's f64 amplitude) unused
      if (b + 1 >= p.B) break;
      pos.x = fmaf(d.x, he.t, pos.x);
      pos.y = fmaf(d.y, he.t, pos.y);
      pos.z = fmaf(d.z, he.t, pos.z);
      acc.add(pos.x, pos.y, pos.z);
      const float4 n4 = p.env_nrm[he.face];
      const float3 n = make_float3(n4.x, n4.y, n4.z);
      const float sc = 2.0f * rt::dot3(d, n);
      d.x = fmaf(-sc, n.x, d.x);
      d.y = fmaf(-sc, n.y, d.y);
      d.z = fmaf(-sc, n.z, d.z);
    } else {
      break;
    }
  }
  const double rec_amp = amp_product(acc.cosv, rec_nint, p.amp0, amp_tab);
  double dl;
  if (p.flags & RT_CIR_C_F64) {
    dl = ((double)rec_dist / p.c64) * p.fs64;
  } else {
    const float q = rec_dist / p.c32;
    dl = (p.flags & RT_CIR_FS_F64) ? (double)q * p.fs64 : (double)(q * p.fs32);
  }
  const int64_t bin = (int64_t)dl;
  // amplitudes are >= 0; a zero one (NaN angle -> _bounce_amplitude 0, tracer.py:35-37) leaves
  // impulse_response[bin] untouched, so it must not become an active bin of the power sweep
  const bool keep = bin < p.n_bins && rec_amp != 0.0;
  okey = keep ? record_key(p, cell, bin) : ~0ull;
  oamp = keep ? rec_amp : 0.0;
}

// ---- clear receivers: cells whose ball of radius r_clear (the receiver radius plus a pad far above
// the f32 rounding of the icosphere's vertices, of a receiver hit point and of an environment t) holds
// no point of any environment face.  Squared point-triangle distance in double (closest point by
// Voronoi region); a degenerate face or a NaN compares as "not clear".  One thread per cell, once per
// plan: brute force over the faces for table scenes, a ball-box walk of the 4-wide BVH otherwise (a
// stack overflow also answers "not clear").
__device__ __forceinline__ double pt_tri_d2(const double p[3], const double a[3], const double b[3], const double c[3]) {
  double ab[3], ac[3], ap[3], bp[3], cp[3];
  for (int i = 0; i < 3; ++i) {
    ab[i] = b[i] - a[i];
    ac[i] = c[i] - a[i];
    ap[i] = p[i] - a[i];
    bp[i] = p[i] - b[i];
    cp[i] = p[i] - c[i];
  }
  auto dot = [](const double* x, const double* y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
  auto d2of = [&](double x, double y, double z) { return x * x + y * y + z * z; };
  const double d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.0 && d2 <= 0.0) return dot(ap, ap);  // vertex a
  const double d3 = dot(ab, bp), d4 = dot(ac, bp);
  if (d3 >= 0.0 && d4 <= d3) return dot(bp, bp);  // vertex b
  const double vc = d1 * d4 - d3 * d2;
  if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) {  // edge ab
    const double v = d1 / (d1 - d3);
    return d2of(ap[0] - v * ab[0], ap[1] - v * ab[1], ap[2] - v * ab[2]);
  }
  const double d5 = dot(ab, cp), d6 = dot(ac, cp);
  if (d6 >= 0.0 && d5 <= d6) return dot(cp, cp);  // vertex c
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {  // edge ac
    const double w = d2 / (d2 - d6);
    return d2of(ap[0] - w * ac[0], ap[1] - w * ac[1], ap[2] - w * ac[2]);
  }
  const double va = d3 * d6 - d5 * d4;
  if (va <= 0.0 && d4 - d3 >= 0.0 && d5 - d6 >= 0.0) {  // edge bc
    const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    return d2of(bp[0] - w * (c[0] - b[0]), bp[1] - w * (c[1] - b[1]), bp[2] - w * (c[2] - b[2]));
  }
  const double den = 1.0 / (va + vb + vc), v = vb * den, w = vc * den;  // inside the face
  return d2of(ap[0] - ab[0] * v - ac[0] * w, ap[1] - ab[1] * v - ac[1] * w, ap[2] - ab[2] * v - ac[2] * w);
}
__device__ __forceinline__ bool face_far(const double p[3], const float4 q0, const float4 q1, float c2z, double R2) {
  const double a[3] = {q0.x, q0.y, q0.z}, b[3] = {q0.w, q1.x, q1.y}, c[3] = {q1.z, q1.w, c2z};
  return pt_tri_d2(p, a, b, c) > R2;  // NaN: not far
}
template <bool USE_BVH>
__global__ __launch_bounds__(256) void k_clear_cells(CovParams p, double r_clear, uint32_t* clear) {
  const int64_t nc = ncells(p.g);
  const double R2 = r_clear * r_clear;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < nc; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cell = base + threadIdx.x;
    bool ok = cell < nc;
    if (ok) {
      double c[3];
      cell_center(p.g, cell, c);
      if constexpr (!USE_BVH) {
        for (int f = 0; f < p.env_nf && ok; ++f)  // case 4 of the table: kx, ky, kz = x, y, z (raw corners)
          ok = face_far(c, p.env_perm[f * 18 + 12], p.env_perm[f * 18 + 13], p.env_perm[f * 18 + 14].x, R2);
      } else {
        int st[RT_BVH_STACK];
        int sp = 0;
        st[sp++] = 0;
        while (ok && sp > 0) {
          const float4* w = p.env_bvh.wide + 8 * (int64_t)st[--sp];
          const float4 lx = w[0], hx = w[1], ly = w[2], hy = w[3], lz = w[4], hz = w[5], rf = w[6];
          const float L[3][4] = {{lx.x, lx.y, lx.z, lx.w}, {ly.x, ly.y, ly.z, ly.w}, {lz.x, lz.y, lz.z, lz.w}};
          const float H[3][4] = {{hx.x, hx.y, hx.z, hx.w}, {hy.x, hy.y, hy.z, hy.w}, {hz.x, hz.y, hz.z, hz.w}};
          const int ref[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
          for (int q = 0; q < 4 && ok; ++q) {
            if (ref[q] == -1) continue;
            double d2 = 0.0;
            for (int k = 0; k < 3; ++k) {
              const double e = fmax(fmax((double)L[k][q] - c[k], c[k] - (double)H[k][q]), 0.0);
              d2 += e * e;
            }
            if (!(d2 <= R2)) continue;  // the child's box misses the ball
            if (ref[q] >= 0) {
              if (sp < RT_BVH_STACK) st[sp++] = ref[q];
              else ok = false;
            } else {
              const int pk = ~ref[q], first = pk >> 3, count = pk & 7;
              for (int j = 0; j < count && ok; ++j) {
                const float4* fr = p.env_bvh.lcomp + (int64_t)(first + j) * 3;
                ok = face_far(c, fr[0], fr[1], fr[2].x, R2);
              }
            }
          }
        }
      }
    }
    const uint64_t m = __ballot(ok);  // one 32-bit word per half wave (cells base + 32 h ..)
    const int lane = threadIdx.x & 63;
    if ((lane & 31) == 0 && cell < nc) clear[(uint64_t)cell >> 5] = (uint32_t)(m >> lane);
  }
}

// Per candidate (cell, ray, k), in whatever order k_cells appended them: the exact receiver test
// and the first-win check; first wins are flagged with their receiver t, to be compacted and
// replayed in a coherent order by k_replay.  (Replaying inside this kernel on brute-force scenes
// measured 37% slower on K3, 10.1 vs 7.4 ms per map: the replay's divergent tail and registers
// held every candidate's wave.)
// 6 waves per SIMD: 80 VGPRs, spill-free with the dot-form ball test: K3 k_win 0.935 -> 0.895 ms, K5
// 0.79 -> 0.76 (r3ze); before it, 5 waves (96 VGPRs, 60 B scratch) beat 4 and 6: 1.03 -> 0.98 ms (r2zj).
// With the per-case receiver vertices (RxLds::ur) it spills 9 VGPRs (40 B) at 6 waves and still
// beats the spill-free form: K3 k_win 0.90-0.91 -> 0.85 ms; at 5 waves (94 VGPRs, no spills) 0.86 ms
// (profiles/r5q_cov_rx_perm_ab.jsonl)
// candidates of this attempt, 0 if they overflowed the buffers (k_win, the first-win list and the
// early replay then do nothing: a lane's keys that would cross the capacity are not written, and
// reading the hole took the replay to illegal addresses in the N = 4 one-GPU rehearsal)
__device__ __forceinline__ int64_t cand_count(const unsigned long long* n_dev, int64_t cap) {
  const int64_t n = (int64_t)*n_dev;
  return n > cap ? 0 : n;
}
__global__ __launch_bounds__(256, 6) void k_win(CovParams p, const uint64_t* keys, const unsigned long long* nkeys_dev,
                                             int64_t cap, uint8_t* first_flag, float* trx, uint32_t* gmask) {
  __shared__ RxLds L;
  __shared__ uint32_t s_line[256];  // this lane's line groups, parked during the group tests
  stage_rx(L, p.r_rx);
  // the candidate count; past the capacity the keys have holes (k_cells skips a lane's keys that
  // would cross it) and the host reruns the attempt, so this one tests nothing
  const int64_t nkeys = cand_count(nkeys_dev, cap);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nkeys; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    const int64_t cell = (int64_t)(key >> 28), r = (int64_t)((key >> 4) & 0xFFFFFF);
    const int k = (int)(key & 15);
    // bounce k, and before it (rarely) the earlier bounces whose segment reaches the cell's ball
    // (first_win): one receiver query site, so the unrolled query is inlined once
    double cc[3];
    cell_center(p.g, cell, cc);
    const double rp2 = p.r_pad * p.r_pad;
    bool first = true;
    float tr = 0.0f;
#pragma unroll 1
    for (int q = 0; q <= k; ++q) {
      if (q < k) {
        const Seg sq = load_seg(p, r, q);
        if (!seg_ball(sq.o, sq.d, sq.tmax, cc, rp2)) continue;
      }
      float t;
      // the line's groups parked in LDS (no register held across the group tests); a winning
      // earlier bounce leaves its own mask, unused: that candidate is no first win
      const bool w = rx_wins(p, L, cell, r, q, t, s_line + threadIdx.x);
      if (q == k) {
        first = w;
        tr = t;
      } else if (w) {
        first = false;
        break;
      }
    }
    first_flag[i] = first ? 1 : 0;
    trx[i] = tr;
    gmask[i] = s_line[threadIdx.x];
  }
}

// The first wins' candidate indices in candidate order (as hipCUB's DeviceSelect::Flagged, which
// needs the candidate count on the host), with the count read on the device: G blocks, each over
// one contiguous tile.  k_sel_count counts a tile's flags; k_sel_scatter adds the counts of the
// tiles before it (<= G values from L2) and writes its indices in order.  (One atomic per wave on
// a single counter instead measured 1.4 ms on K3: 123k contended atomics.)
// A first win as the replay reads it: its candidate key (cell, ray slot, bounce) and receiver t,
// gathered once in candidate order by k_sel_scatter (coherent reads: the candidates are in ray
// order) instead of through list -> keys / trx at every replayed record (three scattered 8-B / 4-B
// reads, each a line: K3 k_replay fetched 1.24 GB per launch at L2 hit 0.19).  The window order
// writes the items themselves in processing order, so a rank's replay reads them sequentially.
struct ReplayItem {
  uint64_t key;
  float trx;
  uint32_t line;  // the receiver groups the first win's line passes (rx_query_culled's lmask)
};
// Replay order key of list entry li.  A wave runs as long as its lane with the most bounces left
// after the first win, so the remaining bounce count (2 bits) leads; then the receiver groups the
// first win's line passes (k_win's mask, 20 bits folded to 14): the replay's receiver queries on
// that line test those groups, so lanes with the same mask run the same group loops and read the
// same LDS entries.  Only the processing order changes: records are written at li.  Against the
// round-4 key (initial direction on an 8x8 octahedral grid, then a 16x16 Morton cell of the
// receiver): K3 replay 1.355 -> 1.21 ms, K5 1.03 -> 0.87 ms on one GPU (device-wide sort); a rank's
// 4096-entry windows gain nothing either way (r5s, r5t, r5u; lowest / highest group as the key:
// no better).  (The ray slot instead of direction and cell on brute-force scenes, 32x32 direction
// cells and longest replays first were measured no better in round 4 and removed in round 5.)
__device__ __forceinline__ uint16_t replay_key(int B, uint64_t key, uint32_t line) {
  const int k0 = (int)(key & 15);
  const uint32_t rem = (uint32_t)min(max(B - 1 - k0, 0), 3);  // bounces left, in 2 bits
  return (uint16_t)(rem << 14 | ((line & 0x3FFFu) ^ (line >> 14)));
}
__device__ __forceinline__ int64_t sel_tile(int64_t n, int G) { return ((n + G - 1) / G + 255) / 256 * 256; }
__device__ __forceinline__ int block_sum(int v, int* s4) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s4[threadIdx.x >> 6] = v;
  __syncthreads();
  return s4[0] + s4[1] + s4[2] + s4[3];
}
__global__ __launch_bounds__(256) void k_sel_count(const uint8_t* flag, const unsigned long long* n_dev, int64_t cap,
                                                   int32_t* counts) {
  __shared__ int s4[4];
  const int64_t n = cand_count(n_dev, cap), tile = sel_tile(n, gridDim.x);
  const int64_t lo = (int64_t)blockIdx.x * tile, hi = min(lo + tile, n);
  int c = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) c += flag[i] != 0;
  c = block_sum(c, s4);
  if (threadIdx.x == 0) counts[blockIdx.x] = c;
}
__global__ __launch_bounds__(256) void k_sel_scatter(const uint8_t* flag, const unsigned long long* n_dev, int64_t cap,
                                                     const int32_t* counts, const uint64_t* keys, const float* trx,
                                                     const uint32_t* gmask, ReplayItem* items,
                                                     unsigned long long* nlist, int B, uint16_t* okey,
                                                     int32_t* oval, unsigned long long* host_cnt) {
  __shared__ int s4[4];
  __shared__ int w4[4];
  const int64_t n = cand_count(n_dev, cap), tile = sel_tile(n, gridDim.x);
  const int64_t lo = (int64_t)blockIdx.x * tile, hi = min(lo + tile, n);
  int before = 0;
  for (int j = threadIdx.x; j < (int)blockIdx.x; j += blockDim.x) before += counts[j];
  int64_t base = block_sum(before, s4);
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    const unsigned long long nl = (unsigned long long)(base + counts[blockIdx.x]);
    *nlist = nl;
    // the host's copy of the candidate, item and list counts, in pinned (coherent) memory: one
    // store each instead of a copy launch after this kernel
    host_cnt[0] = n_dev[0];
    host_cnt[1] = n_dev[1];
    host_cnt[2] = nl;
    __threadfence_system();
  }
  const int wave = threadIdx.x >> 6;
  for (int64_t i0 = lo; i0 < hi; i0 += blockDim.x) {  // block-uniform
    const int64_t i = i0 + threadIdx.x;
    const bool f = i < hi && flag[i] != 0;
    const uint64_t m = __ballot(f);
    if ((threadIdx.x & 63) == 0) w4[wave] = __popcll(m);
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wave; ++w) off += w4[w];
    const int step = w4[0] + w4[1] + w4[2] + w4[3];
    if (f) {
      const int64_t k = base + off + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const ReplayItem it{keys[i], trx[i], gmask[i]};
      items[k] = it;
      if (okey) {  // the device-wide replay order's (key, entry) pairs, as k_replay_keys writes them
        okey[k] = replay_key(B, it.key, it.line);
        oval[k] = (int32_t)k;
      }
    }
    base += step;
    __syncthreads();  // w4 is rewritten by the next step
  }
}

__global__ __launch_bounds__(256) void k_replay_keys(CovParams p, const ReplayItem* items, int64_t nl,
                                                     uint16_t* okey, int32_t* oval) {
  for (int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; li < nl; li += (int64_t)gridDim.x * blockDim.x) {
    okey[li] = replay_key(p.B, items[li].key, items[li].line);
    oval[li] = (int32_t)li;
  }
}

// The replay order by windows: list entries [w W, (w + 1) W), W = 1024 * kReplayWinItems, sorted by
// replay_key inside the window by one 1024-thread block in LDS -- one launch instead of
// k_replay_keys and a device-wide radix sort (hipCUB: ~8 launches and fills, ~100 us per K3 rank of
// 8, profiles/r3b_k3.timeline.txt).  A wave still gets lanes with the same bounces left and nearby
// directions and cells, from its window instead of from the whole list.  The order kernel writes
// the processing order (4-B item indices) and the replay gathers its items through it, inside the
// window just read (L2-resident; copying the 16-B items instead: K3 rank order 19 -> 37 us).
// 4096-entry windows: twice the blocks for a rank's list (K5 rank of 8 1.088 -> 1.003 ms, K3 0.99 ->
// 0.92, r4c).  Larger lists (one GPU's whole map: K3 7.9M, K5 6.4M first wins) keep the
// device-wide sort: there the windows cost more replay coherence than the sort's launches (K5 map
// 4.73 -> 5.21 ms with windows, K3 4.94 -> 5.13 ms; profiles/r3d_*).
constexpr int kReplayWinItems = 4;
constexpr int kReplayWin = 1024 * kReplayWinItems;
constexpr int64_t kReplayWindowMax = 1 << 21;
// rt_debug_replay_window_max: the parity tests lower the threshold to 0 so that small whole-map
// lists take the device-wide sort over k_sel_scatter's pre-written order keys (the path of one
// GPU's K3 / K5 map), e.g. after a regrowth that leaves the list far shorter than the capacity
std::atomic<int64_t> g_replay_window_max{kReplayWindowMax};
template <bool USE_BVH>
__global__ __launch_bounds__(1024) void k_replay_order(CovParams p, const ReplayItem* items, int64_t nl,
                                                       const unsigned long long* nl_dev, int32_t* order) {
  using Sort = rocprim::block_radix_sort<uint16_t, 1024, kReplayWinItems, int32_t>;
  __shared__ typename Sort::storage_type st;
  if (nl_dev) nl = min(nl, (int64_t)*nl_dev);  // launched before the host knows the list length
  if ((int64_t)blockIdx.x * kReplayWin >= nl) return;
  const int64_t base = (int64_t)blockIdx.x * kReplayWin + (int64_t)threadIdx.x * kReplayWinItems;
  uint16_t k[kReplayWinItems];
  int32_t v[kReplayWinItems];
#pragma unroll
  for (int i = 0; i < kReplayWinItems; ++i) {
    const int64_t li = base + i;
    k[i] = li < nl ? replay_key(p.B, items[li].key, items[li].line) : (uint16_t)0xFFFF;
    v[i] = (int32_t)li;
  }
  Sort().sort(k, v, st);
#pragma unroll
  for (int i = 0; i < kReplayWinItems; ++i)
    if (base + i < nl) order[base + i] = v[i];
}

template <bool USE_BVH, bool RX_FIRST>
__global__ __launch_bounds__(256, USE_BVH ? kReplayWavesBvh : kReplayWaves) void k_replay(CovParams p, const ReplayItem* items,
                                                int64_t nl, const unsigned long long* nl_dev,
                                                const int32_t* order, uint64_t* out_key, double* out_amp) {
  extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
  __shared__ RxLds L;
  __shared__ double s_amp[kAmpTab];
  if (nl_dev) nl = min(nl, (int64_t)*nl_dev);  // see k_replay_order
  if ((int64_t)blockIdx.x * blockDim.x >= nl) return;
  stage_amp_tab(s_amp);  // made visible by stage_rx's barrier
  stage_rx(L, p.r_rx);
  stage_env<USE_BVH>(p, lds_tab);
  for (int64_t jl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; jl < nl; jl += (int64_t)gridDim.x * blockDim.x) {
    const ReplayItem it = items[order ? (int64_t)order[jl] : jl];
    const uint64_t key = it.key;
    const int64_t cell = (int64_t)(key >> 28), r = (int64_t)((key >> 4) & 0xFFFFFF);
    // records at the processing position jl: their order is irrelevant (they are sorted by key
    // and summed exactly), and consecutive lanes then write consecutive 8-B words instead of
    // scattering them (K3 k_replay wrote 445 MB for 126 MB of records, r2zm)
    replay<USE_BVH, RX_FIRST>(p, lds_tab, L, s_amp, cell, r, (int)(key & 15), it.trx, it.line, out_key[jl],
                              out_amp[jl]);
  }
}

// compact record key -> the (owner << own_shift | cell << 32 | bin) key of the reduced records
struct WideKey {
  int ray_bits, bin_bits, cell_bits, own_shift;
  int64_t nx, world;  // world > 1: the cell field is owner-local (record_key)
  bool identity = false;  // the keys are wide already (merged received segments)
  __host__ __device__ __forceinline__ uint64_t operator()(uint64_t k) const {
    if (k == ~0ull || identity) return k;
    const uint64_t bin = (k >> ray_bits) & ((1ull << bin_bits) - 1);
    uint64_t cell = (k >> (ray_bits + bin_bits)) & ((1ull << cell_bits) - 1);
    const uint64_t own = k >> (ray_bits + bin_bits + cell_bits);
    if (world > 1) {  // 32-bit division (cells < 2^32): a 64-bit one is ~100 instructions
      const uint32_t nxo = (uint32_t)((nx + world - 1) / world), c32 = (uint32_t)cell, q = c32 / nxo;
      cell = (uint64_t)q * (uint64_t)nx + (uint64_t)(c32 - q * nxo) * (uint64_t)world + own;
    }
    return own << own_shift | cell << 32 | bin;
  }
};

// wide (cell << 32 | bin) keys received from other ranks -> compact [cell | bin] for the sort
// ... and the record indices the sort carries as its payload (one launch for both)
__global__ __launch_bounds__(256) void k_compact_keys(const uint64_t* in, int64_t stride, int64_t n, int bin_bits,
                                                      uint64_t* out, int64_t* idx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = in[i * stride];
    out[i] = k == ~0ull ? ~0ull : ((k >> 32) << bin_bits | (k & 0xFFFFFFFFull));
    idx[i] = i;
  }
}

// The owner stage's records arrive as nseg segments (one per source rank), each sorted by its wide
// key (the order rt_coverage_trace_rows_async writes).  Their stable merge by (key, segment) needs no sort: the merged
// position of element i of segment s is its index in s plus, over every other segment, the number
// of elements with a smaller key (a larger-or-equal one for the segments before s) -- nseg - 1
// binary searches over L2-resident keys.  One launch instead of a record sort (rocPRIM's merge sort,
// 9 launches, ~77 us for a K3 rank's 200k records).
constexpr int kMaxSegs = 64;
struct SegOffsets {
  int64_t off[kMaxSegs + 1];
  int nseg;
};
__global__ __launch_bounds__(256) void k_merge_segments(const uint64_t* keys, int64_t kstride, SegOffsets so,
                                                        uint64_t* keys_out, int64_t* idx_out, unsigned* bad) {
  const int64_t n = so.off[so.nseg];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int sg = 0;
    while (sg + 1 < so.nseg && so.off[sg + 1] <= i) ++sg;
    const uint64_t k = keys[i * kstride];
    if (i > so.off[sg] && keys[(i - 1) * kstride] >= k) atomicAdd(bad, 1u);  // precondition: strictly ascending
    int64_t pos = i - so.off[sg];
    for (int t = 0; t < so.nseg; ++t) {
      if (t == sg) continue;
      int64_t a = so.off[t], b = so.off[t + 1];  // first element > k (t < sg) or >= k (t > sg)
      while (a < b) {
        const int64_t m = (a + b) >> 1;
        const uint64_t km = keys[m * kstride];
        if (km < k || (t < sg && km == k)) a = m + 1;
        else b = m;
      }
      pos += a - so.off[t];
    }
    keys_out[pos] = k;
    idx_out[pos] = i;
  }
}
// The same merge with the nseg - 1 binary searches of an element run in lockstep (NS >= nseg
// segments, `steps` = the longest search): each step issues its loads for every segment at once,
// so a thread waits `steps` memory latencies instead of (nseg - 1) x steps -- the searches over
// L2-resident keys are a chain of dependent loads, and k_merge_segments' time was that chain
// (52 us for a K5 owner's 465k records, profiles/r3zg_k5_rank_timeline.txt).
template <int NS>
__global__ __launch_bounds__(256) void k_merge_lockstep(const uint64_t* keys, int64_t kstride, SegOffsets so,
                                                        int steps, uint64_t* keys_out, int64_t* idx_out,
                                                        unsigned* bad) {
  const int64_t n = so.off[so.nseg];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int sg = 0;
    while (sg + 1 < so.nseg && so.off[sg + 1] <= i) ++sg;
    const uint64_t k = keys[i * kstride];
    if (i > so.off[sg] && keys[(i - 1) * kstride] >= k) atomicAdd(bad, 1u);  // precondition: strictly ascending
    int64_t a[NS], len[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      a[t] = t < so.nseg ? so.off[t] : 0;
      len[t] = (t < so.nseg && t != sg) ? so.off[t + 1] - so.off[t] : 0;
    }
    for (int st = 0; st < steps; ++st) {
      uint64_t km[NS];
#pragma unroll
      for (int t = 0; t < NS; ++t) {  // every segment's probe first: independent loads
        const int64_t m = a[t] + (len[t] >> 1);
        km[t] = keys[(len[t] > 0 ? m : i) * kstride];
      }
#pragma unroll
      for (int t = 0; t < NS; ++t) {  // first element > k (t < sg) or >= k (t > sg)
        if (len[t] > 0) {
          const int64_t half = len[t] >> 1;
          const bool right = km[t] < k || (t < sg && km[t] == k);
          a[t] = right ? a[t] + half + 1 : a[t];
          len[t] = right ? len[t] - half - 1 : half;
        }
      }
    }
    int64_t pos = i - so.off[sg];
#pragma unroll
    for (int t = 0; t < NS; ++t)
      if (t < so.nseg && t != sg) pos += a[t] - so.off[t];
    keys_out[pos] = k;
    idx_out[pos] = i;
  }
}

// ------------------------------------------------------------------ 5. closed-form signal power
// sin and cos of 2*pi*turns, reduced in turns (|2*pi*frac| <= pi keeps ocml on its short path;
// the arguments here reach thousands of radians, where the general reduction is slow)
__device__ __forceinline__ void sincos_turns(double turns, double& s, double& c) {
  const double f = turns - rint(turns);
  sincos(6.283185307179586 * f, &s, &c);
}

struct PowerParams {
  int64_t n_bins;
  int64_t half;   // (n-1)//2 : np.convolve 'same' offset
  double alpha;   // phase per sample: (2*pi*2.4e9) * (window/(n-1))
  double turns;   // alpha / (2*pi)
  double sin_a, cos_a;
  double sin_n, cos_n;  // of alpha * n_bins (the sweep end; host, like sin_a / cos_a)
};

__device__ __forceinline__ void two_sum(double& s, double& c, double x) {  // Neumaier running sum
  const double t = s + x;
  c += fabs(s) >= fabs(x) ? (s - t) + x : (x - t) + s;
  s = t;
}

// Terms accessor T of a sparse impulse response with ascending bins m_k:
//   T.m(k)            m_k
//   T.cs(k, c, s)     a_k cos(alpha (half - m_k)), a_k sin(alpha (half - m_k))
//   T.start(k, s, c)  sin, cos of alpha * s_k      (s_k = first sample where term k is active)
//   T.stop(k, s, c)   sin, cos of alpha * (e_k + 1) (e_k = last one)
// Sweep of the sample range [xb, xe): the active terms at xb (those with s_k <= xb <= e_k, a
// contiguous run [ie, is) because s_k and e_k both ascend with k) are summed directly, then each
// interval of constant active set is closed in form, clipped at xe.  Every interval boundary is
// xb, xe or some s_k / e_k + 1, so the interval's sin(L alpha) and sin/cos((u+v) alpha) follow
// from the boundaries' precomputed sines by angle addition (no per-interval sincos).
// Adds sum(y^2) into (total, tc) and the number of nonzero samples into count.
template <typename Terms>
__device__ void power_range(int64_t lo, int64_t hi, const PowerParams& P, const Terms& T, int64_t xb, int64_t xe,
                            double& total, double& tc, int64_t& count) {
  const int64_t n = P.n_bins, half = P.half;
  double Ps = 0, Pc = 0, Qs = 0, Qc = 0;  // running sums of a_k cos(alpha c_k), a_k sin(alpha c_k)
  auto mk = [&](int64_t k) { return T.m(k); };
  auto sk = [&](int64_t k) { const int64_t m = mk(k); return m - half > 0 ? m - half : 0; };
  auto ek = [&](int64_t k) { const int64_t m = mk(k); const int64_t e = m + (n - 1 - half); return e < n - 1 ? e : n - 1; };
  auto term = [&](int64_t k, double sgn) {  // sgn = +-1: sgn*(a*c) == (sgn*a)*c bit for bit
    double c, s;
    T.cs(k, c, s);
    two_sum(Ps, Pc, sgn * c);
    two_sum(Qs, Qc, sgn * s);
  };
  int64_t is = lo, ie = lo;  // active terms = [ie, is)
  int64_t x = xb;
  double sx = 0.0, cx = 1.0;  // sin, cos of alpha * x (sincos of 0 is exactly that: no call for xb = 0)
  if (xb != 0) sincos_turns(P.turns * (double)xb, sx, cx);
  if (xb > 0) {  // first term starting after xb, first term ending at or after xb
    int64_t a = lo, b = hi;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (sk(m) <= xb) a = m + 1; else b = m;
    }
    is = a;
    a = lo;
    b = is;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (ek(m) < xb) a = m + 1; else b = m;
    }
    ie = a;
  }
  const double sa = P.sin_a, ca = P.cos_a;
  bool first = true;
  while (true) {
    bool started_alone = false;
    int64_t nstart = 0;
    if (first && xb > 0) {
      for (int64_t k = ie; k < is; ++k) {
        term(k, 1.0);
        nstart += sk(k) == x ? 1 : 0;
      }
    } else {
      while (is < hi && sk(is) <= x) {
        term(is, 1.0);
        ++is;
        ++nstart;
      }
      while (ie < is && ek(ie) < x) {
        term(ie, -1.0);
        ++ie;
      }
    }
    first = false;
    if (is - ie == 1 && nstart == 1) started_alone = (mk(is - 1) - half == x);  // sin(0) = 0 exactly
    int64_t nx = xe;
    double snx, cnx;
    int src = 0;  // 0: xe, 1: start of term is, 2: end of term ie
    if (is < hi && sk(is) < nx) {
      nx = sk(is);
      src = 1;
    }
    if (ie < is && ek(ie) + 1 < nx) {
      nx = ek(ie) + 1;
      src = 2;
    }
    if (src == 1) T.start(is, snx, cnx);
    else if (src == 2) T.stop(ie, snx, cnx);
    else if (nx == n) {  // the sweep end: one value for every cell, from the host
      snx = P.sin_n;
      cnx = P.cos_n;
    } else {
      sincos_turns(P.turns * (double)nx, snx, cnx);
    }
    if (ie < is) {
      const double Pv = Ps + Pc, Qv = Qs + Qc;
      const int64_t L = nx - x;
      // sin(L a) = sin(a nx - a x); (u + v) a = a x + a nx - a
      const double sl = snx * cx - cnx * sx;
      const double s2 = sx * cnx + cx * snx, c2 = cx * cnx - sx * snx;  // of a x + a nx
      const double ssu = s2 * ca - c2 * sa, csu = c2 * ca + s2 * sa;
      const double D = sl * csu / sa, E = sl * ssu / sa;
      const double sss = 0.5 * ((double)L - D), scc = 0.5 * ((double)L + D), ssc = 0.5 * E;
      two_sum(total, tc, Pv * Pv * sss + Qv * Qv * scc + 2.0 * Pv * Qv * ssc);
      count += L - (started_alone ? 1 : 0);
    }
    if (nx >= xe) break;
    x = nx;
    sx = snx;
    cx = cnx;
  }
}

// terms from precomputed arrays (k_terms), indexed like the unique keys
struct TermArrays {
  const uint64_t* keys;
  const double *tcos, *tsin, *ev;  // ev: [sin s, cos s, sin e1, cos e1] per key
  __device__ __forceinline__ int64_t m(int64_t k) const { return (int64_t)(keys[k] & 0xFFFFFFFFull); }
  __device__ __forceinline__ void cs(int64_t k, double& c, double& s) const {
    c = tcos[k];
    s = tsin[k];
  }
  __device__ __forceinline__ void start(int64_t k, double& s, double& c) const {
    s = ev[4 * k];
    c = ev[4 * k + 1];
  }
  __device__ __forceinline__ void stop(int64_t k, double& s, double& c) const {
    s = ev[4 * k + 2];
    c = ev[4 * k + 3];
  }
};

// mean square of the nonzero samples of y = ir (*) sin, for a sparse ir with ascending bins m[k]
template <typename Terms>
__device__ double power_sparse(int64_t lo, int64_t hi, const PowerParams& P, const Terms& T) {
  if (hi <= lo) return __builtin_nan("");
  double total = 0.0, tc = 0.0;
  int64_t count = 0;
  power_range(lo, hi, P, T, 0, P.n_bins, total, tc, count);
  return count > 0 ? (total + tc) / (double)count : __builtin_nan("");
}

// per unique (cell, bin): the phase terms of the sweep, computed once in parallel
__global__ __launch_bounds__(256) void k_terms(const uint64_t* ukeys, const double* uamps, const int64_t* nuniq,
                                               PowerParams P, double* tcos, double* tsin, double* ev) {
  const int64_t nu = *nuniq;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = (int64_t)(ukeys[u] & 0xFFFFFFFFull);
    double sp, cp;
    sincos_turns(P.turns * (double)(P.half - m), sp, cp);
    tcos[u] = uamps[u] * cp;
    tsin[u] = uamps[u] * sp;
    const int64_t st = m - P.half > 0 ? m - P.half : 0;
    const int64_t e = m + (P.n_bins - 1 - P.half), e1 = (e < P.n_bins - 1 ? e : P.n_bins - 1) + 1;
    sincos_turns(P.turns * (double)st, ev[4 * u], ev[4 * u + 1]);
    sincos_turns(P.turns * (double)e1, ev[4 * u + 2], ev[4 * u + 3]);
  }
}

// one thread per cell of ours (x columns ix % nshard == shard); other cells are left to the
// caller's zero fill, the power map being sum-reduced across ranks
// [start, end) of every cell's run in the sorted unique keys (cells without keys keep 0, 0)
// [start, end) of every cell's run in the sorted unique keys, stamped with the run's epoch: a
// cell whose stamp is not this run's has no keys (so the arrays never need a fill).  Also resets
// *nbig for k_power_small (stream order: it runs before).
__global__ __launch_bounds__(256) void k_cell_ranges(const uint64_t* ukeys, const int64_t* nuniq, int64_t ncell,
                                                     int32_t* cstart, int32_t* cend, int32_t* cepoch, int32_t epoch,
                                                     unsigned* nbig) {
  const int64_t nu = *nuniq;
  if (blockIdx.x == 0 && threadIdx.x == 0) *nbig = 0u;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t c = ukeys[u] >> 32;
    if (c >= (uint64_t)ncell) continue;  // dropped records (~0) sort last
    if (u == 0 || (ukeys[u - 1] >> 32) != c) {
      cstart[c] = (int32_t)u;
      cepoch[c] = epoch;
    }
    if (u == nu - 1 || (ukeys[u + 1] >> 32) != c) cend[c] = (int32_t)(u + 1);
  }
}

constexpr int kPowLds = 192;  // terms per wave staged in LDS (3 per lane); larger cells read global memory
constexpr int kPowSmall = 16;  // cells with at most this many terms: k_power_small (one thread each, large maps)
// Small maps: kPowGroup lanes per cell for cells of at most kPowGroupMax terms.  K3 map / rank of 8,
// k_power_small + k_power (us): 8 lanes up to 16 terms 60 + 103 / 19 + 22; 16 lanes up to 32 terms
// 62 + 54 / 19 + 14; 16 up to 64 89 + 17 / 27 + 15; 8 up to 32 75 + 54 / 25 + 14 (r6zo)
constexpr int kPowGroup = 16, kPowGroupMax = 32;
constexpr int64_t kPowGroupMaxCells = 131072;  // maps of at most this many cells (the map's, not a shard's)
// (Copying each thread's terms into its LDS column first measured K3 rank 37 -> 33 us but K5 rank
// 42 -> 65 us -- 53 KB of LDS, 3 waves per CU; r3f.  Removed in round 5.)

// double-double helpers for the compensated prefix sums
__device__ __forceinline__ void dd_add(double& h, double& l, double bh, double bl) {
  const double s = h + bh, bb = s - h, e = (h - (s - bb)) + (bh - bb);
  const double t = l + bl + e;
  h = s + t;
  l = t - (h - s);
}

// sum(y^2) over one interval [x, nx) with active sums P, Q, given sin/cos at x and nx
__device__ __forceinline__ double interval_sq(double Pv, double Qv, int64_t L, double sx, double cx, double snx,
                                              double cnx, const PowerParams& P) {
  const double sa = P.sin_a, ca = P.cos_a;
  const double sl = snx * cx - cnx * sx;                            // sin(L a)
  const double s2 = sx * cnx + cx * snx, c2 = cx * cnx - sx * snx;  // of a x + a nx
  const double ssu = s2 * ca - c2 * sa, csu = c2 * ca + s2 * sa;    // of a (x + nx - 1)
  const double D = sl * csu / sa, E = sl * ssu / sa;
  return Pv * Pv * (0.5 * ((double)L - D)) + Qv * Qv * (0.5 * ((double)L + D)) + 2.0 * Pv * Qv * (0.5 * E);
}

// Cells of ours with 0..KMAX terms, G lanes per cell (kPowGroup lanes up to kPowGroupMax terms for
// maps of at most kPowGroupMaxCells cells; G = 1 is the serial sweep of power_sparse up to kPowSmall).  G > 1: the cell's terms are staged in the wave's LDS with compensated
// (double-double) prefix sums of a cos / a sin, and each lane closes the intervals that start at its
// events, as k_power does for larger cells -- equal to the serial sweep up to the order of summation.
// (One thread per cell made the kernel as long as one thread's chain of up to 2 x 16 intervals, each
// a few dependent loads and two f64 divisions: K3 rank of 8 ~40 us for 8k cells.)
// Larger cells are listed (big[], count in *nbig; one atomic per wave) for k_power, which then
// visits only them (it used to stride over every cell of the map to skip the small ones: 1M cell
// ranges read per K5 map for a few thousand large cells).
template <int G, int KMAX = kPowSmall>
__global__ __launch_bounds__(64) void k_power_small(TermArrays T, const int32_t* cstart, const int32_t* cend,
                                                     const int32_t* cepoch, int32_t epoch, rt_grid g, int shard,
                                                     int nshard, PowerParams P, double* power, int32_t* big,
                                                     unsigned* nbig) {
  static_assert(G == 1 || G == 4 || G == 8 || G == 16, "1, 4, 8 or 16 lanes per cell");
  constexpr int NG = 64 / G, TP = (KMAX + G - 1) / G;  // cells per wave, terms per lane
  constexpr int KL = G > 1 ? KMAX : 1;                // LDS slots per cell (the serial form has none)
  __shared__ int32_t s_st[NG][KL], s_e1[NG][KL], s_m[NG][KL];
  __shared__ double s_pch[NG][KL + 1], s_pcl[NG][KL + 1], s_psh[NG][KL + 1], s_psl[NG][KL + 1];
  __shared__ double s_ev[NG][4 * KL];
  const int64_t nxo = g.nx > shard ? (g.nx - shard + nshard - 1) / nshard : 0;
  const int64_t nown = nxo * g.ny * g.nz;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63, j = lane & (G - 1), gi = lane / G;
  if (nshard > 1) {  // other ranks' cells: 0 (the map is sum-reduced), instead of a fill
    // 32-bit index arithmetic (cells < 2^32, rt_coverage_create): a 64-bit division by a run-time
    // divisor is a ~100-instruction sequence, and this loop visits every cell of the map
    const uint32_t ncell = (uint32_t)(g.nx * g.ny * g.nz), nx = (uint32_t)g.nx, ns = (uint32_t)nshard;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < ncell; c += (uint32_t)stride)
      if ((c % nx) % ns != (uint32_t)shard) power[c] = 0.0;
  }
  const int64_t n = P.n_bins, half = P.half;
  const double sn = P.sin_n, cn = P.cos_n;  // sin/cos at the sweep end
  const int64_t gstride = stride / G;
  const int64_t nit = (nown + gstride - 1) / gstride;  // the same count for every lane (LDS reuse)
  for (int64_t it = 0; it < nit; ++it) {
    const int64_t t = it * gstride + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G);
    bool is_big = false, small = false;
    int64_t c = 0, lo = 0, hi = 0;
    if (t < nown) {
      // the owned cell of index t (32-bit: cells < 2^32; a 64-bit division is ~100 instructions)
      if (nshard == 1) {
        c = t;
      } else {
        const uint32_t tt = (uint32_t)t, nx32 = (uint32_t)nxo, rest = tt / nx32, jx = tt - rest * nx32;
        c = (int64_t)rest * g.nx + shard + (int64_t)jx * nshard;
      }
      const bool has = cepoch[c] == epoch;
      lo = has ? cstart[c] : 0;
      hi = has ? cend[c] : 0;
      small = hi - lo <= KMAX;
      is_big = !small;
    }
    const uint64_t m = __ballot(is_big && j == 0);
    if (m) {
      unsigned b0 = 0;
      if (lane == 0) b0 = atomicAdd(nbig, (unsigned)__popcll(m));
      b0 = __shfl(b0, 0, 64);
      if (is_big && j == 0) {
        const unsigned r = (unsigned)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        big[b0 + r] = (int32_t)c;
      }
    }
    if constexpr (G == 1) {
      if (small) power[c] = power_sparse(lo, hi, P, T);  // NaN when empty
    } else {
      const int K = small ? (int)(hi - lo) : 0;
      // stage: TP consecutive terms per lane, local compensated sums, then a scan over the group
      double lch = 0, lcl = 0, lsh = 0, lsl = 0;
#pragma unroll
      for (int q = 0; q < TP; ++q) {
        const int k = j * TP + q;
        if (k < K) {
          const int64_t mk = T.m(lo + k);
          s_m[gi][k] = (int32_t)mk;
          s_st[gi][k] = (int32_t)(mk - half > 0 ? mk - half : 0);
          const int64_t e = mk + (n - 1 - half);
          s_e1[gi][k] = (int32_t)((e < n - 1 ? e : n - 1) + 1);
          for (int r = 0; r < 4; ++r) s_ev[gi][4 * k + r] = T.ev[4 * (lo + k) + r];
          dd_add(lch, lcl, T.tcos[lo + k], 0.0);
          dd_add(lsh, lsl, T.tsin[lo + k], 0.0);
        }
      }
      double ech = lch, ecl = lcl, esh = lsh, esl = lsl;  // inclusive scan of the lanes' sums
#pragma unroll
      for (int o = 1; o < G; o <<= 1) {
        const double a = __shfl_up(ech, o, G), b = __shfl_up(ecl, o, G);
        const double a2 = __shfl_up(esh, o, G), b2 = __shfl_up(esl, o, G);
        if (j >= o) {
          dd_add(ech, ecl, a, b);
          dd_add(esh, esl, a2, b2);
        }
      }
      dd_add(ech, ecl, -lch, -lcl);  // exclusive
      dd_add(esh, esl, -lsh, -lsl);
#pragma unroll
      for (int q = 0; q < TP; ++q) {
        const int k = j * TP + q;
        if (k < K) {
          s_pch[gi][k] = ech;
          s_pcl[gi][k] = ecl;
          s_psh[gi][k] = esh;
          s_psl[gi][k] = esl;
          dd_add(ech, ecl, T.tcos[lo + k], 0.0);
          dd_add(esh, esl, T.tsin[lo + k], 0.0);
          if (k == K - 1) {
            s_pch[gi][K] = ech;
            s_pcl[gi][K] = ecl;
            s_psh[gi][K] = esh;
            s_psl[gi][K] = esl;
          }
        }
      }
      __syncthreads();  // one wave per block
      const int32_t* st = s_st[gi];
      const int32_t* e1 = s_e1[gi];
      auto upper = [&](const int32_t* a, int32_t x) {  // first index with a[i] > x
        int l = 0, r = K;
        while (l < r) {
          const int mm = (l + r) >> 1;
          if (a[mm] <= x) l = mm + 1; else r = mm;
        }
        return l;
      };
      auto lower = [&](const int32_t* a, int32_t x) {  // first index with a[i] >= x
        int l = 0, r = K;
        while (l < r) {
          const int mm = (l + r) >> 1;
          if (a[mm] < x) l = mm + 1; else r = mm;
        }
        return l;
      };
      double total = 0.0, tcomp = 0.0;
      int64_t count = 0;
      for (int ev = j; ev < 2 * K; ev += G) {
        const bool is_start = ev < K;
        const int k = is_start ? ev : ev - K;
        const int32_t x = is_start ? st[k] : e1[k];
        if (x >= n) continue;  // the sweep ends at n
        // one lane per distinct event position: starts first, an end only where no start is
        if (k > 0 && (is_start ? st[k - 1] : e1[k - 1]) == x) continue;
        if (!is_start && upper(st, x) != lower(st, x)) continue;
        const int is = upper(st, x), ie = upper(e1, x);
        if (ie >= is) continue;  // nothing active
        const int nstart = is - lower(st, x);
        const bool alone = (is - ie == 1) && nstart == 1 && ((int64_t)s_m[gi][is - 1] - half == (int64_t)x);
        int64_t nx = n;
        double snx = sn, cnx = cn;
        if (is < K && st[is] < nx) {
          nx = st[is];
          snx = s_ev[gi][4 * is];
          cnx = s_ev[gi][4 * is + 1];
        }
        if (e1[ie] < nx) {
          nx = e1[ie];
          snx = s_ev[gi][4 * ie + 2];
          cnx = s_ev[gi][4 * ie + 3];
        }
        const double sx = is_start ? s_ev[gi][4 * k] : s_ev[gi][4 * k + 2];
        const double cx = is_start ? s_ev[gi][4 * k + 1] : s_ev[gi][4 * k + 3];
        double Ph = s_pch[gi][is], Pl = s_pcl[gi][is], Qh = s_psh[gi][is], Ql = s_psl[gi][is];
        dd_add(Ph, Pl, -s_pch[gi][ie], -s_pcl[gi][ie]);
        dd_add(Qh, Ql, -s_psh[gi][ie], -s_psl[gi][ie]);
        two_sum(total, tcomp, interval_sq(Ph + Pl, Qh + Ql, nx - x, sx, cx, snx, cnx, P));
        count += nx - x - (alone ? 1 : 0);
      }
#pragma unroll
      for (int o = G / 2; o >= 1; o >>= 1) {
        const double t2 = __shfl_down(total, o, G), c2 = __shfl_down(tcomp, o, G);
        const int64_t n2 = __shfl_down(count, o, G);
        if (j < o) {
          two_sum(total, tcomp, t2);
          tcomp += c2;
          count += n2;
        }
      }
      if (small && j == 0) power[c] = count > 0 ? (total + tcomp) / (double)count : __builtin_nan("");
      __syncthreads();  // the LDS slots are reused by the next cells
    }
  }
}

// One wave per cell of ours (x columns ix % nshard == shard; the caller zero-fills the rest, the
// map being sum-reduced across ranks).  Up to kPowLds terms: the terms are staged in LDS with
// compensated (double-double) prefix sums of a cos / a sin, and every lane closes the intervals
// that start at its events (a term's first sample, or the sample after its last): the active
// run [ie, is) comes from two binary searches and P, Q from prefix differences, so no lane
// walks the active set.  Larger cells: the sample axis is split into 64 ranges swept by
// power_range.  Either way equal to the serial sweep up to the order of summation.  (One
// thread per cell was a chain of dependent global loads per interval: the kernel lasted as long
// as its slowest cell whatever the cell count.)
__global__ __launch_bounds__(256) void k_power(TermArrays G, const int32_t* cstart, const int32_t* cend,
                                               const int32_t* big, const unsigned* nbig, PowerParams P, double* power) {
  __shared__ int32_t s_st[4][kPowLds], s_e1[4][kPowLds], s_m[4][kPowLds];
  __shared__ double s_pch[4][kPowLds + 1], s_pcl[4][kPowLds + 1], s_psh[4][kPowLds + 1], s_psl[4][kPowLds + 1];
  __shared__ double s_ev[4][4 * kPowLds];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t n = P.n_bins, half = P.half;
  const int64_t nown = *nbig;
  const double sn = P.sin_n, cn = P.cos_n;  // sin/cos at the sweep end
  for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < nown; t += (int64_t)gridDim.x * 4) {
    const int64_t c = big[t];
    const int64_t lo = cstart[c], hi = cend[c], K = hi - lo;
    double total = 0.0, tcomp = 0.0;
    int64_t count = 0;
    if (K <= kPowLds) {
      const int K32 = (int)K;
      // stage: 3 consecutive terms per lane, local compensated sums, then a wave scan
      double lch = 0, lcl = 0, lsh = 0, lsl = 0;
      for (int q = 0; q < 3; ++q) {
        const int k = lane * 3 + q;
        if (k < K32) {
          const int64_t m = G.m(lo + k);
          s_m[w][k] = (int32_t)m;
          s_st[w][k] = (int32_t)(m - half > 0 ? m - half : 0);
          const int64_t e = m + (n - 1 - half);
          s_e1[w][k] = (int32_t)((e < n - 1 ? e : n - 1) + 1);
          for (int r = 0; r < 4; ++r) s_ev[w][4 * k + r] = G.ev[4 * (lo + k) + r];
          dd_add(lch, lcl, G.tcos[lo + k], 0.0);
          dd_add(lsh, lsl, G.tsin[lo + k], 0.0);
        }
      }
      // exclusive scan of the lanes' (double-double) sums
      double ech = lch, ecl = lcl, esh = lsh, esl = lsl;  // inclusive first
      for (int o = 1; o < 64; o <<= 1) {
        const double a = __shfl_up(ech, o, 64), b = __shfl_up(ecl, o, 64);
        const double a2 = __shfl_up(esh, o, 64), b2 = __shfl_up(esl, o, 64);
        if (lane >= o) {
          dd_add(ech, ecl, a, b);
          dd_add(esh, esl, a2, b2);
        }
      }
      // to exclusive: subtract own sum
      dd_add(ech, ecl, -lch, -lcl);
      dd_add(esh, esl, -lsh, -lsl);
      for (int q = 0; q < 3; ++q) {
        const int k = lane * 3 + q;
        if (k < K32) {
          s_pch[w][k] = ech;
          s_pcl[w][k] = ecl;
          s_psh[w][k] = esh;
          s_psl[w][k] = esl;
          dd_add(ech, ecl, G.tcos[lo + k], 0.0);
          dd_add(esh, esl, G.tsin[lo + k], 0.0);
          if (k == K32 - 1) {
            s_pch[w][K32] = ech;
            s_pcl[w][K32] = ecl;
            s_psh[w][K32] = esh;
            s_psl[w][K32] = esl;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int32_t* st = s_st[w];
      const int32_t* e1 = s_e1[w];
      auto upper = [&](const int32_t* a, int32_t x) {  // first index with a[i] > x
        int l = 0, r = K32;
        while (l < r) {
          const int mm = (l + r) >> 1;
          if (a[mm] <= x) l = mm + 1; else r = mm;
        }
        return l;
      };
      auto lower = [&](const int32_t* a, int32_t x) {  // first index with a[i] >= x
        int l = 0, r = K32;
        while (l < r) {
          const int mm = (l + r) >> 1;
          if (a[mm] < x) l = mm + 1; else r = mm;
        }
        return l;
      };
      for (int ev = lane; ev < 2 * K32; ev += 64) {
        const bool is_start = ev < K32;
        const int k = is_start ? ev : ev - K32;
        const int32_t x = is_start ? st[k] : e1[k];
        if (x >= n) continue;  // the sweep ends at n
        // one lane per distinct event position: starts first, an end only where no start is
        if (k > 0 && (is_start ? st[k - 1] : e1[k - 1]) == x) continue;
        if (!is_start && upper(st, x) != lower(st, x)) continue;
        const int is = upper(st, x), ie = upper(e1, x);
        if (ie >= is) continue;  // nothing active
        const int nstart = is - lower(st, x);
        const bool alone = (is - ie == 1) && nstart == 1 && ((int64_t)s_m[w][is - 1] - half == (int64_t)x);
        int64_t nx = n;
        double snx = sn, cnx = cn;
        if (is < K32 && st[is] < nx) {
          nx = st[is];
          snx = s_ev[w][4 * is];
          cnx = s_ev[w][4 * is + 1];
        }
        if (e1[ie] < nx) {
          nx = e1[ie];
          snx = s_ev[w][4 * ie + 2];
          cnx = s_ev[w][4 * ie + 3];
        }
        const double sx = is_start ? s_ev[w][4 * k] : s_ev[w][4 * k + 2];
        const double cx = is_start ? s_ev[w][4 * k + 1] : s_ev[w][4 * k + 3];
        double Ph = s_pch[w][is], Pl = s_pcl[w][is], Qh = s_psh[w][is], Ql = s_psl[w][is];
        dd_add(Ph, Pl, -s_pch[w][ie], -s_pcl[w][ie]);
        dd_add(Qh, Ql, -s_psh[w][ie], -s_psl[w][ie]);
        two_sum(total, tcomp, interval_sq(Ph + Pl, Qh + Ql, nx - x, sx, cx, snx, cnx, P));
        count += nx - x - (alone ? 1 : 0);
      }
    } else if (K > kPowLds) {
      const int64_t xb = n * lane / 64, xe = n * (lane + 1) / 64;
      if (xe > xb) power_range(lo, hi, P, G, xb, xe, total, tcomp, count);
    }
    for (int o = 32; o >= 1; o >>= 1) {
      const double t2 = __shfl_down(total, o, 64), c2 = __shfl_down(tcomp, o, 64);
      const int64_t n2 = __shfl_down(count, o, 64);
      if (lane < o) {
        two_sum(total, tcomp, t2);
        tcomp += c2;
        count += n2;
      }
    }
    if (lane == 0) power[c] = count > 0 ? (total + tcomp) / (double)count : __builtin_nan("");
    __builtin_amdgcn_wave_barrier();  // LDS slots are reused by the wave's next cell
  }
}

// power of dense impulse responses (one per row), e.g. from the per-cell reference loop
__global__ __launch_bounds__(64) void k_power_dense(const double* ir, int64_t rows, PowerParams P, uint64_t* scratch_keys,
                                                    double* scratch_amps, double* power) {
  const int64_t row = blockIdx.x;
  if (row >= rows || threadIdx.x != 0) return;
  const double* x = ir + row * P.n_bins;
  uint64_t* kk = scratch_keys + row * P.n_bins;
  double* aa = scratch_amps + row * P.n_bins;
  int64_t K = 0;
  for (int64_t m = 0; m < P.n_bins; ++m)
    if (x[m] != 0.0) {
      kk[K] = (uint64_t)m;
      aa[K] = x[m];
      ++K;
    }
  struct {
    const uint64_t* kk;
    const double* aa;
    PowerParams P;
    __device__ int64_t m(int64_t k) const { return (int64_t)kk[k]; }
    __device__ void cs(int64_t k, double& c, double& s) const {
      double sp, cp;
      sincos_turns(P.turns * (double)(P.half - (int64_t)kk[k]), sp, cp);
      c = aa[k] * cp;
      s = aa[k] * sp;
    }
    __device__ void start(int64_t k, double& s, double& c) const {
      const int64_t m = (int64_t)kk[k], st = m - P.half > 0 ? m - P.half : 0;
      sincos_turns(P.turns * (double)st, s, c);
    }
    __device__ void stop(int64_t k, double& s, double& c) const {
      const int64_t m = (int64_t)kk[k], e = m + (P.n_bins - 1 - P.half);
      sincos_turns(P.turns * (double)((e < P.n_bins - 1 ? e : P.n_bins - 1) + 1), s, c);
    }
  } T{kk, aa, P};
  power[row] = power_sparse(0, K, P, T);
}

}  // namespace

// ------------------------------------------------------------------ host side
struct rt_coverage {
  int device = 0;
  const rt_mesh* env = nullptr;
  int B = 0;
  int64_t n = 0, ray_offset = 0;
  int64_t n_total = 0;     // rays per cell of the whole burst (amplitude tx_power / n_total)
  bool ray_mode = false;   // ray-sharded: candidates for every cell, records grouped by owner
  bool sectors = false;    // ray-sharded by initial azimuth (rt_coverage_create_sectors): ray_order holds
                           // the plan's global ray ids (ray_offset 0) in banded order, set at creation
  rt_grid grid{};
  double r_rx = 0.1;
  int shard = 0, nshard = 1;
  // buffers
  float4* traj = nullptr;  // n * B * 2 float4
  int32_t* ray_order = nullptr;  // BVH scenes: the plan's rays sorted by initial direction (first run)
  uint8_t* nseg = nullptr;
  uint64_t *keys = nullptr, *keys_sorted = nullptr, *okeys = nullptr, *okeys_sorted = nullptr, *ukeys = nullptr;
  double *oamps = nullptr, *oamps_sorted = nullptr, *uamps = nullptr;
  double *tcos = nullptr, *tsin = nullptr;  // per unique (cell, bin): phase terms of the power sweep
  double* ev = nullptr;                      // per unique (cell, bin): sin/cos at its start and end sample
  int32_t *cstart = nullptr, *cend = nullptr;  // per cell: its run in the unique keys
  int32_t* cepoch = nullptr;                   // per cell: the run (range_epoch) that wrote cstart/cend
  int32_t range_epoch = 0;
  int32_t* bigcells = nullptr;  // per cell slot: the cells k_power sweeps (more terms than k_power_small takes)
  int32_t* runs = nullptr;  // exact run sums: [cap] head flags, [cap] their scan, [cap] run starts, [64] counters
  // k_owner_runs' look-back: [cap / kOwnTile + 1] state words, [ticket counter, error count]; host:
  // tickets issued so far, the call's tag
  uint64_t* own_states = nullptr;
  unsigned long long* own_aux = nullptr;
  uint64_t own_tag = 0;
  uint64_t* send_tails = nullptr;  // k_send_runs' look-back payloads: [2][cap / kOwnTile + 2][5] tagged words
  uint8_t* win = nullptr;
  uint8_t* first_flag = nullptr;
  float* trx = nullptr;
  uint32_t* gmask = nullptr;  // per candidate: the receiver groups its line passes (k_win)
  ReplayItem* ritems = nullptr;  // first wins, in candidate order
  uint32_t* clear = nullptr;      // clear receivers, one bit per cell (k_clear_cells), on the first run
  bool clear_on = true;           // RFRT_COV_CLEAR=0 at creation: the replay always queries the environment
  uint64_t* items = nullptr;
  int64_t item_cap = 0;
  unsigned long long* counters = nullptr;  // [0] candidates, [1] column items, [2] replay list (int64)
  int64_t* nuniq = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  int64_t cap = 0;
  int64_t last_candidates = 0;
  int64_t last_list = 0;  // first wins of the last run (sizes the early replay's grid)
  int64_t last_received = 0;  // first-win (cell, ray) records of the last run
  void* rord = nullptr;        // replay-order sort workspace (16-bit keys + int32 rows, x2, + hipCUB)
  size_t rord_bytes = 0;
  int64_t* bounds = nullptr;   // ray mode: [world + 1] starts of each owner's run in the reduced records
  int64_t n_out = 0;           // ray mode: valid reduced records of the last trace stage
  int64_t pend_ncand = 0, pend_nlist = 0, pend_max_out = -1;  // trace stage awaiting its host half
  // rt_coverage_profile: stage events of the last run and its work counts (device, [0] traced
  // ray-bounces = sum of the trajectories' segments, [1] replayed ray-bounces)
  bool profile = false;
  hipEvent_t pev[8] = {};
  unsigned long long* hcnt = nullptr;  // pinned copy of counters[0..2] (the candidate stage's read-back)
  unsigned long long* hcnt_dev = nullptr;  // the same words as the kernels address them
  int64_t* hbounds = nullptr;          // pinned (ray mode): the trace stage's owner bounds [world + 1], then the look-back error count
  int64_t* hbounds_dev = nullptr;
  hipEvent_t ev_cnt = nullptr;         // recorded after that copy
  bool ev_rec[8] = {};
  unsigned long long* work = nullptr;
};

namespace {

// Exact per-bin sums.  tracer.py:116-117 adds a bin's amplitudes one by one in f64, in ray order.
// Here every amplitude is converted exactly (truncated below 2^-136) to a 192-bit unsigned fixed
// point number with unit 2^-136 and integer part below 2^56, the bin's values are added as
// integers, and the sum is rounded once to f64 (correctly rounded).  Integer addition is
// associative, so the result does not depend on the order of the records, on how the rays are
// sharded over ranks, or on the thread timing of the reduction: ray-sharded maps equal the
// one-GPU map bit for bit, and the sort needs no ray field in its key.  It differs from the
// reference's sequential f64 sum by that sum's own rounding (~1e-16 relative); amplitudes below
// ~1e-26 lose relative precision (they are 2^-136-quantised).
//
// (Round 1 summed doubles with hipcub::DeviceReduce::ReduceByKey, whose decoupled look-back
// combines tile partials in a timing-dependent order: the transmitter cells' long runs changed in
// the last bit from run to run.  Round 2 first moved to rocPRIM's deterministic_reduce_by_key over
// a (cell, bin, ray) sort; the fixed point makes the ray field and the deterministic variant
// unnecessary.  DESIGN.md §6.)
struct Fx192 {
  uint64_t w0, w1, w2;  // w0 least significant
};
struct FxPlus {
  __host__ __device__ __forceinline__ Fx192 operator()(const Fx192& a, const Fx192& b) const {
    Fx192 r;
    r.w0 = a.w0 + b.w0;
    const uint64_t c0 = r.w0 < a.w0;
    const uint64_t t = a.w1 + b.w1;
    const uint64_t c1 = t < a.w1;
    r.w1 = t + c0;
    r.w2 = a.w2 + b.w2 + (c1 | (r.w1 < t));
    return r;
  }
};
// amplitude (finite, >= 0) -> fixed point, truncated below the unit 2^-136; saturates at 2^56
__host__ __device__ __forceinline__ Fx192 fx_from_double(double a) {
  Fx192 r{0, 0, 0};
  uint64_t bits;
  memcpy(&bits, &a, 8);
  bits &= ~(1ull << 63);
  int e = (int)(bits >> 52);
  uint64_t m = bits & ((1ull << 52) - 1);
  if (e == 0x7ff) return r;  // not finite: no contribution (never produced by the replay)
  if (e == 0) e = 1;         // subnormal
  else m |= 1ull << 52;
  const int sh = e - 939;  // a = m 2^(e-1075) = m 2^sh units of 2^-136
  if (sh < 0) {
    r.w0 = sh <= -64 ? 0 : m >> (-sh);
  } else if (sh > 139) {
    r.w0 = r.w1 = r.w2 = ~0ull;
  } else {
    const int w = sh >> 6, b = sh & 63;
    const uint64_t lo = m << b, hi = b ? m >> (64 - b) : 0;
    if (w == 0) {
      r.w0 = lo;
      r.w1 = hi;
    } else if (w == 1) {
      r.w1 = lo;
      r.w2 = hi;
    } else {
      r.w2 = lo;
    }
  }
  return r;
}
// fixed point -> the nearest double (round to nearest even, a sticky bit for the cut-off bits)
__host__ __device__ __forceinline__ double fx_to_double(const Fx192& x) {
  int top;
  if (x.w2) top = 128 + 63 - __builtin_clzll(x.w2);
  else if (x.w1) top = 64 + 63 - __builtin_clzll(x.w1);
  else if (x.w0) top = 63 - __builtin_clzll(x.w0);
  else return 0.0;
  if (top < 64) return ldexp((double)x.w0, -136);
  const int sh = top - 63;  // 1 .. 128: window = bits [sh, sh + 63]
  uint64_t win, sticky;
  if (sh < 64) {
    win = (x.w0 >> sh) | (x.w1 << (64 - sh));
    sticky = x.w0 & ((1ull << sh) - 1);
  } else if (sh == 64) {
    win = x.w1;
    sticky = x.w0;
  } else if (sh < 128) {
    const int b = sh - 64;
    win = (x.w1 >> b) | (x.w2 << (64 - b));
    sticky = x.w0 | (x.w1 & ((1ull << b) - 1));
  } else {  // top bit of w2 set (a saturated value): the window is w2 itself
    win = x.w2;
    sticky = x.w0 | x.w1;
  }
  return ldexp((double)(win | (sticky ? 1ull : 0ull)), sh - 136);
}

// The exact sums of the runs of equal keys in sorted records, in place of a generic reduce-by-key
// (rocPRIM's took 357 us per 7.9M records with the 24-B fixed-point value, 127 us with f64).
// Integer sums throughout, so the tiling cannot change a bit.
struct AmpVal {  // sorted replay records: f64 amplitudes
  const double* a;
  __device__ __forceinline__ Fx192 operator()(int64_t i) const { return fx_from_double(a[i]); }
};
struct SumVal {  // received records: fixed-point sums, in sorted-index order
  const uint64_t* words;  // sum of record j at words[j * stride .. + 2]
  const int64_t* idx;
  int64_t stride = 3;     // 3: an Fx192 array; 4: packed (key, sum) rows, words = rows + 1
  __device__ __forceinline__ Fx192 operator()(int64_t i) const {
    const uint64_t* q = words + idx[i] * stride;
    return Fx192{q[0], q[1], q[2]};
  }
};

// ---- Run sums in three launches.  The sorted records are cut into
// ntiles <= kMaxTiles tiles of T records (T a multiple of 64); a record is a run head when its key
// differs from the previous record's.
//   k_tile_heads  per tile: its number of heads
//   k_tile_sums   one wave per tile: its first unique index (sum of the earlier tiles' heads), then
//                 64-record chunks in order -- a segmented inclusive scan of the Fx192 values by head
//                 flags, the open run's running sum carried from chunk to chunk.  Runs that end in
//                 the tile are written (key, exact sum, f64); the part of the tile before its first
//                 head (headpart) and the open run at its end (tailpart) are left for k_cross_tiles
//   k_cross_tiles one wave per tile whose last run goes on into the next tile: tailpart + the
//                 headparts of the following tiles up to the first one with a head
// Integer sums throughout (Fx192), so the tiling cannot change a bit.  The round-2 form took 7
// launches and three passes over the records (flags, scan, starts, ...; ~90 us on a K3 rank of 8,
// profiles/r3b_k3_rank_timeline.txt; removed in round 5).
constexpr int64_t kMaxTiles = 4096;  // each wave of k_tile_sums sums the earlier tiles' heads: <= 64 per lane
constexpr int64_t kMinTile = 256;    // 4 chunks per wave: enough waves to fill the GPU on a rank's ~1M records
struct TileMeta {
  int32_t* heads;   // [ntiles]
  int64_t* tail_u;  // [ntiles] unique index of the run open at the tile's end, -1 if it ends there
  Fx192* headpart;  // [ntiles] sum of the records before the tile's first head (whole tile if none)
  Fx192* tailpart;  // [ntiles] sum of the open run's records in the tile
};
// wave sum of a Fx192 (xor butterfly; every lane ends with the total)
__device__ __forceinline__ Fx192 wave_fx_sum(Fx192 x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    Fx192 y;
    y.w0 = __shfl_xor(x.w0, o, 64);
    y.w1 = __shfl_xor(x.w1, o, 64);
    y.w2 = __shfl_xor(x.w2, o, 64);
    x = FxPlus()(x, y);
  }
  return x;
}
__device__ __forceinline__ Fx192 shfl_fx(const Fx192& x, int src) {
  return Fx192{__shfl(x.w0, src, 64), __shfl(x.w1, src, 64), __shfl(x.w2, src, 64)};
}
__device__ __forceinline__ Fx192 shfl_up_fx(const Fx192& x, int o) {
  return Fx192{__shfl_up(x.w0, o, 64), __shfl_up(x.w1, o, 64), __shfl_up(x.w2, o, 64)};
}
__global__ __launch_bounds__(256) void k_tile_heads(const uint64_t* keys, int64_t n, int64_t T, int32_t* heads) {
  __shared__ int s4[4];
  const int64_t lo = (int64_t)blockIdx.x * T, hi = lo + T < n ? lo + T : n;
  int c = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) c += (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
  c = block_sum(c, s4);
  if (threadIdx.x == 0) heads[blockIdx.x] = c;
}
template <typename Val>
__global__ __launch_bounds__(64) void k_tile_sums(const uint64_t* keys, Val val, int64_t n, int64_t T, int64_t ntiles,
                                                  TileMeta tm, WideKey wk, uint64_t* ukeys, Fx192* usums,
                                                  double* uamps, int64_t* nuniq) {
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  const int64_t lo = t * T, hi = lo + T < n ? lo + T : n;
  int64_t base = 0;  // unique index of the tile's first head
  for (int64_t j = lane; j < t; j += 64) base += tm.heads[j];
  for (int o = 32; o >= 1; o >>= 1) base += __shfl_xor(base, o, 64);
  if (t == ntiles - 1 && lane == 0) *nuniq = base + tm.heads[t];
  const Fx192 zero{0, 0, 0};
  const bool first_is_head = lo == 0 || keys[lo] != keys[lo - 1];
  Fx192 carry = zero;     // running sum of the run open at the end of the previous chunk
  bool carry_pre = !first_is_head;  // that run began before the tile
  int64_t u = base - 1;   // unique index of the open run
  for (int64_t c0 = lo; c0 < hi; c0 += 64) {
    const int64_t i = c0 + lane;
    const bool valid = i < hi;
    const uint64_t k = valid ? keys[i] : 0;
    const bool head = valid && (i == 0 || k != keys[i - 1]);
    // the record after this one starts a new run (the tile's last record: left to the tile end)
    const bool ends = valid && i + 1 < hi && keys[i + 1] != k;
    Fx192 v = valid ? val(i) : zero;
    // segmented inclusive scan: v = sum of this lane's run from its start in this chunk to here
    bool f = head;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const Fx192 y = shfl_up_fx(v, o);
      const bool fy = __shfl_up(f ? 1 : 0, o, 64) != 0;
      if (lane >= o && !f) v = FxPlus()(v, y);
      if (lane >= o) f = f || fy;
    }
    const uint64_t hb = __ballot(head);
    const int fh = hb ? __builtin_ctzll(hb) : 64;  // first head lane of the chunk
    if (lane < fh) v = FxPlus()(v, carry);         // lanes of the run carried into the chunk
    const uint64_t below = lane ? (hb & (~0ull >> (64 - lane))) : 0ull;
    const int64_t ul = u + __popcll(below) + (head ? 1 : 0);  // this lane's run
    if (head) ukeys[ul] = wk(k);
    if (ends) {
      if (lane < fh && carry_pre) {
        tm.headpart[t] = v;  // the run that began before the tile: its part in this tile
      } else {
        usums[ul] = v;
        uamps[ul] = fx_to_double(v);
      }
    }
    const int nvalid = (int)(hi - c0 < 64 ? hi - c0 : 64);
    carry = shfl_fx(v, nvalid - 1);
    if (hb) carry_pre = false;
    u += __popcll(hb);
  }
  if (lane == 0) {  // the run open at the end of the tile
    const bool goes_on = hi < n && keys[hi] == keys[hi - 1];
    if (first_is_head) tm.headpart[t] = zero;  // nothing before the tile's first head
    if (carry_pre) {  // no head in the tile: all of it belongs to a run that began earlier
      tm.headpart[t] = carry;
      tm.tail_u[t] = -1;
    } else if (goes_on) {
      tm.tailpart[t] = carry;
      tm.tail_u[t] = u;
    } else {
      usums[u] = carry;
      uamps[u] = fx_to_double(carry);
      tm.tail_u[t] = -1;
    }
  }
}
__global__ __launch_bounds__(256) void k_cross_tiles(int64_t ntiles, TileMeta tm, Fx192* usums, double* uamps) {
  const int lane = threadIdx.x & 63;
  const int64_t ta = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ta >= ntiles) return;
  const int64_t u = tm.tail_u[ta];
  if (u < 0) return;  // wave-uniform
  const Fx192 zero{0, 0, 0};
  Fx192 acc = lane == 0 ? tm.tailpart[ta] : zero;
  for (int64_t t0 = ta + 1; t0 < ntiles; t0 += 64) {
    const int64_t t = t0 + lane;
    const bool in = t < ntiles;
    const bool has_head = in && tm.heads[t] > 0;
    const uint64_t hb = __ballot(has_head);
    const int stop = hb ? __builtin_ctzll(hb) : 64;  // the run ends in tile t0 + stop
    if (in && lane <= stop) acc = FxPlus()(acc, tm.headpart[t]);
    if (hb || t0 + 64 >= ntiles) break;
  }
  acc = wave_fx_sum(acc);
  if (lane == 0) {
    usums[u] = acc;
    uamps[u] = fx_to_double(acc);
  }
}

// ---- Owner stage, runs + terms + cell ranges in one launch.  After the segment
// merge, a run of equal keys holds at most one record per source rank (each rank's segment has
// unique keys), so it is at most nseg long: the record that heads a run sums it on its own, reading
// on past its tile's end when the run crosses it (a run that began in an earlier tile is its head's).
// The unique index of a head is the number of heads before it: per tile of kOwnTile records a
// count, combined across tiles by decoupled look-back (tiles taken in order from a ticket counter;
// every state word carries the call's tag, so nothing is reset between calls).  Each head then
// writes its key and f64 sum, its power-sweep terms (k_terms) and, at cell boundaries, the cell's
// range (k_cell_ranges).  Replaces k_tile_heads, k_tile_sums, k_cross_tiles, k_terms and
// k_cell_ranges (five launches) on merged segments.
constexpr int kOwnItems = 4, kOwnTile = 256 * kOwnItems;
// Tiles are taken in order from a ticket counter (one same-address atomic per block), so a block
// only ever waits on tiles that running blocks hold.  Taking the tile from the block index was ~13 us
// faster per rank of 8 on an idle GPU, but unsafe: each XCD dispatches its share of the workgroups
// on its own, so a block can wait on a predecessor its XCD cannot place while other work fills it.
// With four processes on one GPU (the N = 4 rehearsal) the waits ran out, the prefixes were wrong
// and the power sweeps read out of bounds (profiles/r4zd_rehearse_4.log; with tickets:
// r4zf_ticket_*.log).  Removed in round 5 (last in commit 43de9a4).
constexpr uint64_t kOwnAgg = 1ull << 38, kOwnInc = 2ull << 38, kOwnCount = (1ull << 38) - 1;
constexpr uint64_t kOwnTagMask = ~(kOwnInc | kOwnAgg | kOwnCount);
// Look-back tiles are numbered by a ticket counter, not by the block index (blocks of different XCDs
// start in no fixed order; waiting on a tile that is not running deadlocked in the round-4 N = 4
// rehearsal).  The counter is zero before every launch: the block that draws the last ticket (one
// per block) sets it back, so no fill precedes the launch and a launch that never ran leaves it 0.
__device__ __forceinline__ uint32_t take_ticket(unsigned long long* ticket) {
  const uint32_t t = (uint32_t)atomicAdd(ticket, 1ull);
  if (t == gridDim.x - 1) atomicExch(ticket, 0ull);  // every other block holds its ticket already
  return t;
}
struct OwnerRuns {
  const uint64_t* keys;  // merged wide keys [n]
  SumVal val;            // the record sums in merged order
  int64_t n;
  uint64_t* states;      // [tiles] look-back words
  unsigned long long* ticket;
  uint64_t tag;
  unsigned* errors;
  uint64_t* ukeys;
  double *uamps, *tcos, *tsin, *ev;
  int64_t* nuniq;
  int64_t ncell;
  int32_t *cstart, *cend, *cepoch;
  int32_t epoch;
  unsigned* nbig;
  PowerParams P;
};
__global__ __launch_bounds__(256) void k_owner_runs(OwnerRuns a) {
  __shared__ uint32_t s_tile;
  __shared__ int s_w[4];
  __shared__ int64_t s_prefix;
  if (threadIdx.x == 0) s_tile = take_ticket(a.ticket);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.nbig = 0u;  // k_power_small lists the big cells afresh
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t i0 = tile * kOwnTile + (int64_t)threadIdx.x * kOwnItems;
  uint64_t k[kOwnItems];
  bool head[kOwnItems];
  int c = 0;
  uint64_t prev = i0 > 0 && i0 - 1 < a.n ? a.keys[i0 - 1] : ~0ull;
#pragma unroll
  for (int j = 0; j < kOwnItems; ++j) {
    const int64_t i = i0 + j;
    k[j] = i < a.n ? a.keys[i] : ~0ull;
    head[j] = i < a.n && (i == 0 || k[j] != prev);
    prev = k[j];
    c += head[j] ? 1 : 0;
  }
  // block exclusive scan of the heads
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  int before = 0;
  for (int q = 0; q < w; ++q) before += s_w[q];
  const int total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  if (w == 0) {  // the look-back, by wave 0: lane L reads the state of tile jbase - L
    uint64_t* st = a.states + tile;
    if (lane == 0)
      __hip_atomic_store(st, a.tag | (tile == 0 ? kOwnInc : kOwnAgg) | (uint64_t)total, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    if (tile > 0) {
      int spins = 0;
      for (int64_t jbase = tile - 1;;) {  // windows of 64 predecessors: the nearest inclusive one
        const int64_t j = jbase - lane;
        const uint64_t sv = j >= 0 ? __hip_atomic_load(a.states + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const bool ready = j < 0 || (sv & kOwnTagMask) == a.tag;
        const uint64_t incm = __ballot(j >= 0 && ready && (sv & kOwnInc) != 0);
        const int stop = incm ? __builtin_ctzll(incm) : 63;
        const uint64_t used = stop == 63 ? ~0ull : ((2ull << stop) - 1);
        if (__ballot(!ready) & used) {  // a tile up to the inclusive one has not published yet
          if (++spins > (1 << 22)) {
            if (lane == 0) atomicAdd(a.errors, 1u);
            break;
          }
          continue;
        }
        uint64_t cnt = (j >= 0 && lane <= stop) ? (sv & kOwnCount) : 0ull;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        excl += cnt;
        if (incm || jbase < 64) break;  // tile 0 always publishes an inclusive state
        jbase -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(st, a.tag | kOwnInc | (excl + (uint64_t)total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_prefix = (int64_t)excl;
      if (i0 + kOwnTile >= a.n) *a.nuniq = (int64_t)excl + total;  // the last tile
    }
  }
  __syncthreads();
  int64_t u = s_prefix + before + x - c;  // unique index of this thread's first head
  const PowerParams& P = a.P;
#pragma unroll
  for (int j = 0; j < kOwnItems; ++j) {
    if (!head[j]) continue;
    const int64_t i = i0 + j;
    const uint64_t key = k[j];
    Fx192 acc = a.val(i);
    int64_t e = i + 1;
    for (; e < a.n; ++e) {  // <= nseg records
      const uint64_t ke = a.keys[e];
      if (ke != key) break;
      acc = FxPlus()(acc, a.val(e));
    }
    const double amp = fx_to_double(acc);
    a.ukeys[u] = key;
    a.uamps[u] = amp;
    const int64_t m = (int64_t)(key & 0xFFFFFFFFull);
    double sp, cp;
    sincos_turns(P.turns * (double)(P.half - m), sp, cp);
    a.tcos[u] = amp * cp;
    a.tsin[u] = amp * sp;
    const int64_t st = m - P.half > 0 ? m - P.half : 0;
    const int64_t en = m + (P.n_bins - 1 - P.half), e1 = (en < P.n_bins - 1 ? en : P.n_bins - 1) + 1;
    sincos_turns(P.turns * (double)st, a.ev[4 * u], a.ev[4 * u + 1]);
    sincos_turns(P.turns * (double)e1, a.ev[4 * u + 2], a.ev[4 * u + 3]);
    const uint64_t cell = key >> 32;
    if (cell < (uint64_t)a.ncell) {  // (a ~0 key never arrives from another rank)
      const uint64_t pk = i > 0 ? a.keys[i - 1] : ~0ull;
      if (i == 0 || (pk >> 32) != cell) {
        a.cstart[cell] = (int32_t)u;
        a.cepoch[cell] = a.epoch;
      }
      if (e >= a.n || (a.keys[e] >> 32) != cell) a.cend[cell] = (int32_t)(u + 1);
    }
    ++u;
  }
}

// ---- Trace-stage reduce in one launch: the sorted replay records of a ray-sharded
// rank -> its unique (owner, cell, bin) keys with their exact sums, the send rows and the owner
// bounds.  Tiles of kSendTile records in ticket order; each thread holds kSendItems consecutive records.  A
// run of equal keys may be any length (a K3 rank's transmitter cell: ~125k records in one bin), so
// the sums are a segmented scan: per tile its head count and its segmented tail (the sum after its
// last head, or of the whole tile if it has none), combined across tiles by decoupled look-back --
// the state word carries the call's tag, the head bit and the count; the Fx192 tails sit beside it
// as five words of 40 bits, each carrying the tag too, so every word validates itself and no fence
// orders them (an agent-scope release / acquire pair per tile -- L2 write-back and invalidate across
// the XCDs -- made the kernel 0.28-0.32 ms, profiles/r4i_sendruns_fenced_k3_rank_timeline.txt).
// Every run is written by its last
// record: key, exact sum, f64, its row (packed 32 B or key + sum) and, at owner changes, the bounds.
// Replaces k_tile_heads, k_tile_sums, k_cross_tiles and k_bounds_strip (four launches, ~50 us per
// rank of 8, profiles/r4h_k5.timeline.txt).  Integer sums: the same bits in any grouping.
// 8 records per thread (k_owner_runs keeps 4): K3 rank of 8 48 -> 38 us, K5 46 -> 42 us; 8 for the
// owner stage too was slower there (K3 21 -> 35 us), 2 here 70 us (r6zh)
constexpr int kSendItems = 8, kSendTile = 256 * kSendItems;
static_assert(kSendTile >= kOwnTile, "k_send_runs uses k_owner_runs' tile states (sized per kOwnTile)");
constexpr uint64_t kSendHead = 1ull << 37, kSendCount = (1ull << 37) - 1;
struct SegFx {  // segmented sum of a stretch of records: h = it holds a head, t = the sum after its last head
  bool h;
  Fx192 t;
};
__device__ __forceinline__ SegFx seg_op(const SegFx& a, const SegFx& b) {  // a, then b
  return SegFx{a.h || b.h, b.h ? b.t : FxPlus()(a.t, b.t)};
}
__device__ __forceinline__ SegFx shfl_up_seg(const SegFx& x, int o) {
  return SegFx{__shfl_up(x.h ? 1 : 0, o, 64) != 0, shfl_up_fx(x.t, o)};
}
// an Fx192 as five tagged words (tag24 << 40 | 40 payload bits), stored and loaded one by one
__device__ __forceinline__ void put_tail(uint64_t* q, const Fx192& t, uint64_t tag24) {
  const uint64_t M = (1ull << 40) - 1, tg = tag24 << 40;
  const uint64_t c[5] = {t.w0 & M, (t.w0 >> 40 | t.w1 << 24) & M, (t.w1 >> 16) & M, (t.w1 >> 56 | t.w2 << 8) & M,
                         t.w2 >> 32};
#pragma unroll
  for (int i = 0; i < 5; ++i) __hip_atomic_store(q + i, tg | c[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct SendRuns {
  const uint64_t* keys;  // sorted compact record keys [n], dropped records (~0) last
  const double* amps;
  int64_t n;
  uint64_t* states;
  uint64_t *agg_tail, *inc_tail;  // [tiles][5] tagged words
  unsigned long long* ticket;
  uint64_t tag;
  unsigned* errors;
  WideKey wk;
  int world, own_shift;
  uint64_t* ukeys;
  Fx192* usums;
  double* uamps;
  int64_t* nuniq;
  int64_t* bounds;
  uint64_t* out;     // 32-B (key without the owner field, sum words 0..2) rows
  int64_t cap;       // rows the caller's buffer holds
};
__global__ __launch_bounds__(256) void k_send_runs(SendRuns a) {
  __shared__ uint32_t s_tile;
  __shared__ int s_wc[4];
  __shared__ SegFx s_ws[4];
  __shared__ int64_t s_prefix;
  __shared__ Fx192 s_carry;
  if (threadIdx.x == 0) s_tile = take_ticket(a.ticket);
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t i0 = tile * kSendTile + (int64_t)threadIdx.x * kSendItems;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const Fx192 zero{0, 0, 0};
  uint64_t k[kSendItems];
  Fx192 v[kSendItems];
  bool head[kSendItems];
  const uint64_t key_before = i0 > 0 && i0 - 1 < a.n ? a.keys[i0 - 1] : ~0ull;
  const uint64_t key_after = i0 + kSendItems < a.n ? a.keys[i0 + kSendItems] : ~0ull;
  uint64_t prev = key_before;
  int c = 0;
  SegFx th{false, zero};
#pragma unroll
  for (int j = 0; j < kSendItems; ++j) {
    const int64_t i = i0 + j;
    k[j] = i < a.n ? a.keys[i] : ~0ull;
    head[j] = i < a.n && (i == 0 || k[j] != prev);
    prev = k[j];
    v[j] = i < a.n ? fx_from_double(a.amps[i]) : zero;
    c += head[j] ? 1 : 0;
    th = seg_op(th, SegFx{head[j], v[j]});
  }
  // inclusive wave scans of the head counts and of the segmented sums
  int x = c;
  SegFx sx = th;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    const SegFx sy = shfl_up_seg(sx, o);
    if (lane >= o) {
      x += y;
      sx = seg_op(sy, sx);
    }
  }
  if (lane == 63) {
    s_wc[w] = x;
    s_ws[w] = sx;
  }
  SegFx lx = shfl_up_seg(sx, 1);  // the lanes before this one
  if (lane == 0) lx = SegFx{false, zero};
  __syncthreads();
  int before = x - c;
  SegFx pre{false, zero};
  for (int q = 0; q < w; ++q) {
    before += s_wc[q];
    pre = seg_op(pre, s_ws[q]);
  }
  pre = seg_op(pre, lx);  // this tile's records before this thread
  if (w == 0) {  // the look-back, by wave 0: one round trip per predecessor tile
    const int total = s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3];
    SegFx T = s_ws[0];
    for (int q = 1; q < 4; ++q) T = seg_op(T, s_ws[q]);
    uint64_t* st = a.states + tile;
    const uint64_t hb = T.h ? kSendHead : 0ull, tag24 = a.tag >> 40;
    if (lane == 0) {
      if (tile == 0) {
        put_tail(a.inc_tail, T.t, tag24);
        __hip_atomic_store(st, a.tag | kOwnInc | hb | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        put_tail(a.agg_tail + 5 * tile, T.t, tag24);
        __hip_atomic_store(st, a.tag | kOwnAgg | hb | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    uint64_t excl = 0;
    SegFx carry{false, zero};  // the tiles before this one, segmented
    if (tile > 0) {
      // windows of 64 predecessors, lane L reading tile jbase - L (state word and both tails): the
      // nearest inclusive tile and the aggregates after it in one round trip
      const uint64_t M40 = (1ull << 40) - 1;
      int spins = 0;
      for (int64_t jbase = tile - 1;;) {
        const int64_t j = jbase - lane;
        bool ready = true, inc = false;
        SegFx x{false, zero};
        uint64_t cnt = 0;
        if (j >= 0) {
          const uint64_t sv = __hip_atomic_load(a.states + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          uint64_t wa[5], wi[5];
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            wa[i] = __hip_atomic_load(a.agg_tail + 5 * j + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wi[i] = __hip_atomic_load(a.inc_tail + 5 * j + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          inc = (sv & kOwnInc) != 0;
          ready = (sv & kOwnTagMask) == a.tag;
          const uint64_t* wq = inc ? wi : wa;
#pragma unroll
          for (int i = 0; i < 5; ++i) ready = ready && (wq[i] >> 40) == tag24;
          inc = inc && ready;
          uint64_t c5[5];
#pragma unroll
          for (int i = 0; i < 5; ++i) c5[i] = wq[i] & M40;
          x = SegFx{inc || (sv & kSendHead) != 0,
                    Fx192{c5[0] | c5[1] << 40, c5[1] >> 24 | c5[2] << 16 | c5[3] << 56, c5[3] >> 8 | c5[4] << 32}};
          cnt = sv & kSendCount;
        }
        const uint64_t incm = __ballot(j >= 0 && inc);
        const int stop = incm ? __builtin_ctzll(incm) : 63;  // the lanes 0 .. stop are combined
        const uint64_t used = stop == 63 ? ~0ull : ((2ull << stop) - 1);
        if (__ballot(j >= 0 && !ready) & used) {  // a tile in the window has not published yet
          if (++spins > (1 << 22)) {
            if (lane == 0) atomicAdd(a.errors, 1u);
            break;
          }
          continue;
        }
        if (lane > stop || j < 0) {
          x = SegFx{false, zero};
          cnt = 0;
        }
        // older tiles (higher lanes) first: lane i takes lane i + o's stretch as the one before its own
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const SegFx y{__shfl_down(x.h ? 1 : 0, o, 64) != 0,
                        Fx192{__shfl_down(x.t.w0, o, 64), __shfl_down(x.t.w1, o, 64), __shfl_down(x.t.w2, o, 64)}};
          const uint64_t cy = __shfl_down(cnt, o, 64);
          if (lane + o < 64) {
            x = seg_op(y, x);
            cnt += cy;
          }
        }
        const SegFx W{__shfl(x.h ? 1 : 0, 0, 64) != 0, shfl_fx(x.t, 0)};
        excl += __shfl(cnt, 0, 64);
        carry = seg_op(W, carry);
        if (incm || jbase < 64) break;  // an inclusive tile reached (tile 0 always publishes one)
        jbase -= 64;
      }
      if (lane == 0) {
        put_tail(a.inc_tail + 5 * tile, seg_op(carry, T).t, tag24);
        __hip_atomic_store(st, a.tag | kOwnInc | hb | (excl + (uint64_t)total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (lane == 0) {
      s_prefix = (int64_t)excl;
      s_carry = carry.t;
      if (tile * kSendTile + kSendTile >= a.n) *a.nuniq = (int64_t)excl + total;  // the last tile
    }
  }
  __syncthreads();
  int64_t u = s_prefix + before - 1;               // the run open before this thread's first record
  Fx192 acc = seg_op(SegFx{true, s_carry}, pre).t;  // its sum so far
  const uint64_t mask = (1ull << a.own_shift) - 1;
#pragma unroll
  for (int j = 0; j < kSendItems; ++j) {
    const int64_t i = i0 + j;
    if (i >= a.n) break;
    if (head[j]) {
      ++u;
      acc = v[j];
      const uint64_t kp = j ? k[j - 1] : key_before;
      const int lo = i == 0 ? -1 : (kp == ~0ull ? a.world : (int)(a.wk(kp) >> a.own_shift));
      const int hi = k[j] == ~0ull ? a.world : (int)(a.wk(k[j]) >> a.own_shift);
      for (int o = lo + 1; o <= hi; ++o) a.bounds[o] = u;  // owners lo+1 .. hi start at u
    } else {
      acc = FxPlus()(acc, v[j]);
    }
    const uint64_t next = j + 1 < kSendItems ? k[j + 1] : key_after;
    if (i + 1 < a.n && next == k[j]) continue;  // the run goes on
    const uint64_t wkey = a.wk(k[j]);
    a.ukeys[u] = wkey;
    a.usums[u] = acc;
    a.uamps[u] = fx_to_double(acc);
    if (a.out && k[j] != ~0ull && u < a.cap) {
      typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
      u64x2* row = reinterpret_cast<u64x2*>(a.out + 4 * u);  // 32-B rows: two 16-B stores
      row[0] = u64x2{wkey & mask, acc.w0};
      row[1] = u64x2{acc.w1, acc.w2};
    }
    if (i + 1 == a.n) {  // the owners after the last record's start at the end
      const int hi = k[j] == ~0ull ? a.world : (int)(wkey >> a.own_shift);
      for (int o = hi + 1; o <= a.world; ++o) a.bounds[o] = u + 1;
    }
  }
}

// send counts from the owner bounds (rt_coverage_trace_rows_async: they stay on the device)
// the send counts on the device, and the owner bounds plus the look-back error word into the
// plan's pinned (coherent) host words -- stores instead of two copy launches
__global__ __launch_bounds__(64) void k_bounds_to_counts(const int64_t* bounds, int world, int64_t* counts,
                                                         int64_t* host_bounds, const uint64_t* err) {
  for (int o = threadIdx.x; o < world; o += blockDim.x) counts[o] = bounds[o + 1] - bounds[o];
  for (int o = threadIdx.x; o <= world; o += blockDim.x) host_bounds[o] = bounds[o];
  if (threadIdx.x == 0) host_bounds[world + 1] = (int64_t)*err;
  __threadfence_system();
}

__global__ __launch_bounds__(256) void k_amps_to_fx(const double* amps, int64_t n, Fx192* sums) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    sums[i] = fx_from_double(amps[i]);
}

int free_cands(rt_coverage* c, hipStream_t s) {
  // Work still in flight may read these buffers: the early window replay is launched before the
  // host sees the candidate counts, and an overflow regrows the buffers right after (a K3 rank of
  // 4 with 250k rays overflows the initial 8-per-ray capacity on its first run: the replay then
  // read freed memory, an illegal address in the N = 4 rehearsal, profiles/r4zb_rehearse_4.log).
  // Growth is rare (first runs), so wait for the plan's stream here (s: the stream of the call that
  // grows; the plan's work is ordered on it).  A fault of earlier work surfaces as this call's error.
  // Work the plan queued on ANOTHER stream (Python passes torch's current stream, which may differ
  // between calls on one plan; rt_coverage_create passes the null stream) is not covered by that
  // wait: what makes the frees below safe for it is hipFree itself, which synchronises the whole
  // device before it releases memory (HIP's documented hipFree semantics; the stream-ordered
  // hipFreeAsync is deliberately not used here).  The same holds for alloc_items.
  RT_HIP(hipStreamSynchronize(s));
  for (void* q : {(void*)c->keys, (void*)c->keys_sorted, (void*)c->okeys, (void*)c->okeys_sorted, (void*)c->ukeys,
                  (void*)c->oamps, (void*)c->oamps_sorted, (void*)c->uamps, (void*)c->tcos, (void*)c->tsin, (void*)c->ev,
                  (void*)c->win, (void*)c->trx,
                  (void*)c->gmask, (void*)c->first_flag, c->tmp, c->rord, (void*)c->runs, (void*)c->ritems})
    if (q) (void)hipFree(q);
  c->keys = c->keys_sorted = c->okeys = c->okeys_sorted = c->ukeys = nullptr;
  c->oamps = c->oamps_sorted = c->uamps = c->tcos = c->tsin = c->ev = nullptr;
  c->win = nullptr;
  c->first_flag = nullptr;
  c->trx = nullptr;
  c->gmask = nullptr;
  c->ritems = nullptr;
  c->runs = nullptr;
  if (c->own_states) (void)hipFree(c->own_states);
  c->own_states = nullptr;
  if (c->send_tails) (void)hipFree(c->send_tails);
  c->send_tails = nullptr;
  c->tmp = nullptr;
  c->tmp_bytes = 0;
  c->rord = nullptr;
  c->rord_bytes = 0;
  c->cap = 0;
  return RT_OK;
}


size_t rord_key_bytes(int64_t n) { return ((size_t)n * 2 + 255) / 256 * 256; }
size_t rord_row_bytes(int64_t n) { return ((size_t)n * 4 + 255) / 256 * 256; }

// Record sorts (stable, on the low end_bit key bits).  rocprim sends 8-byte-key radix sorts of up
// to 1M items to a block merge sort (~15 launches), otherwise to Onesweep (ceil(bits / 8) passes,
// each a fill + a sort launch).  rocprofv3, one K3 rank of 8 (tools/cov_profile.py): the trace
// stage's ~0.7M records on 51 bits take 238 us merged vs ~205 us by Onesweep; the owner stage's
// ~0.2M (31 bits) are faster merged (owner stage 0.23 vs 0.29 ms) and K5's ~0.47M (36 bits) by
// Onesweep (0.46 vs 0.50 ms).  So: Onesweep from 300k items, rocprim's default below.
// 10-bit digits and 1024-thread blocks (rocprim's gfx950 default is 8 bits per pass;
// tools/gpu_sortvar.sh: K5 rank of 8 1.58 -> 1.53 ms).  Smaller sort tiles for a rank's < 2M
// records (512 x 8, 256 x 8, 512 x 4 with 10-bit digits, 256 x 8 with 8-bit) fill more CUs and were
// slower: K3 rank of 8 with collectives 0.856-0.926 vs 0.856-0.867 ms (profiles/r6o_sort_tile_ab.jsonl).
using OnesweepCfg =
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 10,
                                        rocprim::block_radix_rank_algorithm::match>;
using OnesweepOnly = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, OnesweepCfg, 0>;
constexpr int64_t kOnesweepMinItems = 300000;

// rocPRIM's Onesweep with its host loop rewritten (the kernels are rocPRIM's own, rocprim::detail, so
// the sort is the same): rocPRIM's driver fills the digit histogram, then before every pass the
// pass's look-back states and its ordered block id -- 1 + 2 x passes fills of ~5 us each (a K5 rank
// of 8: 9 of its 17 sort launches).  Here one fill zeroes the histogram and every pass's states and
// block id together, then the histogram, the scan and one launch per pass.  The sorted keys and
// values always end in kout / vout (the passes alternate through the scratch so that the last one
// writes them).  The look-back states of all passes are allocated together (radix x blocks x
// places, i.e. places x rocPRIM's one-pass size), which is what lets one fill serve every pass.
// rocprim::detail is not a stable interface: this driver is compiled only against the rocPRIM it
// was written and checked for (ROCm 7.2's 4.2.0, kRocprimDetailVersion); any other version takes
// rocprim::radix_sort_pairs with the same Onesweep configuration (same results, more fills).
constexpr int kRocprimDetailVersion = 400200;
template <class Cfg, typename K, typename V>
hipError_t onesweep_pairs(void* temp, size_t& storage, const K* kin, K* kout, const V* vin, V* vout, unsigned n,
                          unsigned end_bit, hipStream_t s) {
#if ROCPRIM_VERSION == 400200
  static_assert(ROCPRIM_VERSION == kRocprimDetailVersion, "onesweep_pairs: checked against rocPRIM 4.2.0 only");
  namespace rd = rocprim::detail;
  using config = rd::wrapped_radix_sort_onesweep_config<Cfg, K, V>;
  using bid_t = rd::block_id_wrapper<unsigned int, true>;
  using state_t = rd::onesweep_lookback_state;
  rd::target_arch arch;
  hipError_t e = rd::host_target_arch(s, arch);
  if (e != hipSuccess) return e;
  const rd::radix_sort_onesweep_config_params params = rd::dispatch_target_arch<config, false>(arch);
  const unsigned rb = params.radix_bits_per_place, radix = 1u << rb;
  const unsigned hist_ipb = params.histogram.block_size * params.histogram.items_per_thread;
  const unsigned sort_ipb = params.sort.block_size * params.sort.items_per_thread;
  const unsigned places = (end_bit + rb - 1) / rb;
  const unsigned sblocks = (n + sort_ipb - 1) / sort_ipb;
  const size_t al = 256;
  auto up = [&](size_t b) { return (b + al - 1) / al * al; };
  const size_t b_off = up(sizeof(unsigned) * radix * places), b_tmp = up(sizeof(unsigned) * radix);
  const size_t b_states = up(sizeof(state_t) * (size_t)radix * sblocks * places), b_bid = up(sizeof(unsigned) * places);
  const size_t b_keys = up(sizeof(K) * n), b_vals = up(sizeof(V) * n);
  const size_t zero_bytes = b_off + b_tmp + b_states + b_bid;
  if (!temp) {
    storage = zero_bytes + b_keys + b_vals;
    return hipSuccess;
  }
  if (storage < zero_bytes + b_keys + b_vals || n == 0 || places == 0) return hipErrorInvalidValue;
  char* base = static_cast<char*>(temp);
  unsigned* offsets = reinterpret_cast<unsigned*>(base);
  unsigned* offsets_tmp = reinterpret_cast<unsigned*>(base + b_off);
  state_t* states = reinterpret_cast<state_t*>(base + b_off + b_tmp);
  unsigned* bids = reinterpret_cast<unsigned*>(base + b_off + b_tmp + b_states);
  K* ktmp = reinterpret_cast<K*>(base + zero_bytes);
  V* vtmp = reinterpret_cast<V*>(base + zero_bytes + b_keys);
  if ((e = hipMemsetAsync(base, 0, zero_bytes, s)) != hipSuccess) return e;
  const rocprim::identity_decomposer dec{};
  {
    const unsigned hblocks = (n + hist_ipb - 1) / hist_ipb, hfull = n % hist_ipb == 0 ? hblocks : hblocks - 1;
    auto hist = [=](auto arch_config) {
      static constexpr rd::radix_sort_onesweep_config_params P = decltype(arch_config)::params;
      rd::onesweep_histograms<P.histogram.block_size, P.histogram.items_per_thread, P.radix_bits_per_place, false>(
          kin, offsets, n, hfull, dec, 0u, end_bit);
    };
    e = rd::execute_launch_plan<config, decltype(hist), rd::radix_sort_onesweep_histogram_config_selector>(
        arch, hist, dim3(hblocks), dim3(params.histogram.block_size), 0, s);
    if (e != hipSuccess) return e;
    auto scan = [=](auto arch_config) {
      static constexpr rd::radix_sort_onesweep_config_params P = decltype(arch_config)::params;
      rd::onesweep_scan_histograms<P.histogram.block_size, P.radix_bits_per_place>(offsets);
    };
    e = rd::execute_launch_plan<config, decltype(scan), rd::radix_sort_onesweep_histogram_config_selector>(
        arch, scan, dim3(places), dim3(params.histogram.block_size), 0, s);
    if (e != hipSuccess) return e;
  }
  const unsigned sfull = n % sort_ipb == 0 ? sblocks : sblocks - 1;
  // pass p reads the previous pass's output; the last pass writes kout / vout
  for (unsigned p = 0; p < places; ++p) {
    const unsigned bit = p * rb, cur_bits = std::min(rb, end_bit - bit);
    const bool into_out = ((places - 1 - p) % 2) == 0;  // the pass that ends in kout alternates back from the last
    const K* ki = p == 0 ? kin : (into_out ? ktmp : kout);
    const V* vi = p == 0 ? vin : (into_out ? vtmp : vout);
    K* ko = into_out ? kout : ktmp;
    V* vo = into_out ? vout : vtmp;
    bid_t bid = bid_t::create(bids + p);
    state_t* st = states + (size_t)radix * sblocks * p;
    unsigned* off_in = offsets + p * radix;
    auto iter = [=](auto arch_config) {
      static constexpr rd::radix_sort_onesweep_config_params P = decltype(arch_config)::params;
      rd::onesweep_iteration<P.sort.block_size, P.sort.items_per_thread, P.radix_bits_per_place, false,
                             P.radix_rank_algorithm>(ki, ko, vi, vo, n, off_in, offsets_tmp, st, dec, bit, cur_bits,
                                                     sfull, bid);
    };
    e = rd::execute_launch_plan<config, decltype(iter), rd::radix_sort_onesweep_sort_config_selector>(
        arch, iter, dim3(sblocks), dim3(params.sort.block_size), 0, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
#else
  using Only = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, Cfg, 0>;
  return rocprim::radix_sort_pairs<Only>(temp, storage, kin, kout, vin, vout, n, 0u, end_bit, s);
#endif
}

template <typename V>
hipError_t sort_records(void* tmp, size_t& bytes, const uint64_t* kin, uint64_t* kout, const V* vin, V* vout,
                        int64_t n, int end_bit, hipStream_t s) {
  if (n >= kOnesweepMinItems) {
    // rocPRIM's Onesweep kernels with one fill (onesweep_pairs); one batch: rocPRIM splits at 2^30
    if (n < ((int64_t)1 << 30)) {
      if (!tmp) {  // the workspace of either driver (the plan sizes it once for both)
        size_t b1 = 0, b2 = 0;
        hipError_t e =
            onesweep_pairs<OnesweepCfg, uint64_t, V>(nullptr, b1, kin, kout, vin, vout, (unsigned)n, (unsigned)end_bit, s);
        if (e == hipSuccess)
          e = rocprim::radix_sort_pairs<OnesweepOnly>(nullptr, b2, kin, kout, vin, vout, (unsigned)n, 0u,
                                                      (unsigned)end_bit, s);
        bytes = std::max(b1, b2);
        return e;
      }
      return onesweep_pairs<OnesweepCfg, uint64_t, V>(tmp, bytes, kin, kout, vin, vout, (unsigned)n, (unsigned)end_bit,
                                                      s);
    }
    return rocprim::radix_sort_pairs<OnesweepOnly>(tmp, bytes, kin, kout, vin, vout, (unsigned)n, 0u,
                                                   (unsigned)end_bit, s);
  }
  return rocprim::radix_sort_pairs(tmp, bytes, kin, kout, vin, vout, (unsigned)n, 0u, (unsigned)end_bit, s);
}

int alloc_cands(rt_coverage* c, int64_t cap, hipStream_t s) {
  if (int rc = free_cands(c, s)) return rc;
  RT_HIP(hipMalloc(&c->keys, cap * 8));
  RT_HIP(hipMalloc(&c->keys_sorted, cap * 8));
  RT_HIP(hipMalloc(&c->okeys, cap * 8));
  RT_HIP(hipMalloc(&c->okeys_sorted, cap * 8));
  RT_HIP(hipMalloc(&c->ukeys, cap * 8));
  RT_HIP(hipMalloc(&c->oamps, cap * 8));
  RT_HIP(hipMalloc(&c->oamps_sorted, cap * 8));
  RT_HIP(hipMalloc(&c->uamps, cap * 8));
  RT_HIP(hipMalloc(&c->tcos, cap * 8));
  RT_HIP(hipMalloc(&c->tsin, cap * 8));
  RT_HIP(hipMalloc(&c->ev, cap * 32));
  RT_HIP(hipMalloc(&c->first_flag, cap));
  RT_HIP(hipMalloc(&c->trx, cap * 4));
  RT_HIP(hipMalloc(&c->gmask, cap * 4));
  RT_HIP(hipMalloc(&c->ritems, cap * sizeof(ReplayItem)));
  RT_HIP(hipMalloc(&c->runs, (cap * 3 + 64) * 4));  // tile heads / open-run indices (run_sums), counters
  // k_owner_runs' states: zero = no tag (tags start at 1 << 40)
  RT_HIP(hipMalloc(&c->own_states, ((size_t)cap / kOwnTile + 2) * 8));
  RT_HIP(hipMemset(c->own_states, 0, ((size_t)cap / kOwnTile + 2) * 8));
  RT_HIP(hipMalloc(&c->send_tails, ((size_t)cap / kOwnTile + 2) * 2 * 5 * 8));
  RT_HIP(hipMemset(c->send_tails, 0, ((size_t)cap / kOwnTile + 2) * 2 * 5 * 8));  // tag 0: never a call's
  size_t b1 = 0, b2 = 0, b3 = 0;
  RT_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, c->keys, c->keys_sorted, (int)cap, 0, 64));
  size_t b2m = 0;  // both sort_records paths: Onesweep at cap, the merge sort below its threshold
  RT_HIP(sort_records(nullptr, b2, c->okeys, c->okeys_sorted, c->oamps, c->oamps_sorted, cap, 64, 0));
  RT_HIP(sort_records(nullptr, b2m, c->okeys, c->okeys_sorted, c->oamps, c->oamps_sorted,
                      std::min<int64_t>(cap, kOnesweepMinItems - 1), 64, 0));
  b2 = std::max(b2, b2m);
  size_t b2i = 0;  // the owner stage sorts (key, record index) pairs
  RT_HIP(sort_records(nullptr, b2i, c->okeys, c->okeys_sorted, (const int64_t*)c->oamps, (int64_t*)c->oamps_sorted, cap,
                      64, 0));
  b3 = b2i;
  c->tmp_bytes = std::max(std::max(b1, b2), b3);
  RT_HIP(hipMalloc(&c->tmp, c->tmp_bytes));
  // replay-order sort workspace for up to cap records (one allocation per growth, not per run)
  size_t b5 = 0;
  RT_HIP((onesweep_pairs<rocprim::default_config, uint16_t, int32_t>(nullptr, b5, (uint16_t*)nullptr, (uint16_t*)nullptr,
                                                                     (int32_t*)nullptr, (int32_t*)nullptr, (unsigned)cap, 16u,
                                                                     nullptr)));
  c->rord_bytes = 2 * rord_key_bytes(cap) + 2 * rord_row_bytes(cap) + b5;
  RT_HIP(hipMalloc(&c->rord, c->rord_bytes));
  c->cap = cap;
  return RT_OK;
}

int alloc_items(rt_coverage* c, int64_t cap, hipStream_t s) {
  RT_HIP(hipStreamSynchronize(s));  // as free_cands: nothing in flight may still read the old list
  if (c->items) (void)hipFree(c->items);
  c->items = nullptr;
  RT_HIP(hipMalloc(&c->items, cap * 8));
  c->item_cap = cap;
  return RT_OK;
}

// rt_debug_poison: every buffer of the plan (and a block of the default pool, for the
// stream-ordered workspaces) is filled with the poison byte before a run
int poison_plan(rt_coverage* c, hipStream_t s) {
  const int b = rt::g_poison & 0xFF;
  const int64_t nc = c->grid.nx * c->grid.ny * c->grid.nz;
  struct {
    void* p;
    size_t n;
  } bufs[] = {{c->traj, sizeof(float4) * 2 * (size_t)c->B * c->n}, {c->nseg, (size_t)c->n},
              {c->keys, (size_t)c->cap * 8}, {c->keys_sorted, (size_t)c->cap * 8}, {c->okeys, (size_t)c->cap * 8},
              {c->okeys_sorted, (size_t)c->cap * 8}, {c->ukeys, (size_t)c->cap * 8}, {c->oamps, (size_t)c->cap * 8},
              {c->oamps_sorted, (size_t)c->cap * 8}, {c->uamps, (size_t)c->cap * 8}, {c->tcos, (size_t)c->cap * 8},
              {c->tsin, (size_t)c->cap * 8}, {c->ev, (size_t)c->cap * 32}, {c->first_flag, (size_t)c->cap},
              {c->trx, (size_t)c->cap * 4}, {c->gmask, (size_t)c->cap * 4},
              {c->ritems, (size_t)c->cap * sizeof(ReplayItem)}, {c->items, (size_t)c->item_cap * 8},
              {c->tmp, c->tmp_bytes}, {c->rord, c->rord_bytes}, {c->counters, 32}, {c->nuniq, 8},
              {c->cstart, sizeof(int32_t) * (size_t)nc}, {c->cend, sizeof(int32_t) * (size_t)nc},
              {c->bigcells, sizeof(int32_t) * (size_t)nc}, {c->cepoch, sizeof(int32_t) * (size_t)nc},
              {c->bounds, c->bounds ? sizeof(int64_t) * (size_t)(c->nshard + 1) : 0},
              {c->runs, ((size_t)c->cap * 3 + 64) * 4}};
  for (auto& q : bufs)
    if (q.p && q.n) RT_HIP(hipMemsetAsync(q.p, b, q.n, s));
  return rt::poison_pool((size_t)256 << 20, s);
}

void prof_mark(rt_coverage* c, int i, hipStream_t s) {
  if (!c->profile) return;
  if (!c->pev[i] && hipEventCreate(&c->pev[i]) != hipSuccess) return;
  c->ev_rec[i] = hipEventRecord(c->pev[i], s) == hipSuccess;
}

// work counts for the rooflines (profiling only): sum of nseg, and sum over replayed records of
// the bounces the replay runs (its first-win bounce plus the B - 1 - k0 full queries after it)
__global__ __launch_bounds__(256) void k_count_segments(const uint8_t* nseg, int64_t n, unsigned long long* out) {
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc += nseg[i];
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}
__global__ __launch_bounds__(256) void k_count_replay(const ReplayItem* items, int64_t nl, int B,
                                                      unsigned long long* out) {
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += (int64_t)gridDim.x * blockDim.x)
    acc += (unsigned long long)(B - (int)(items[i].key & 15));
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

// BVH trajectories of at most this many rays run 16 / 4 lanes per ray (RFRT_TRAJ_SPLIT_MAX, 0 = never)
int64_t traj_split_max_rays() {
  static const int64_t v = [] {
    const char* e = getenv("RFRT_TRAJ_SPLIT_MAX");
    return e ? (int64_t)atoll(e) : (int64_t)262144;
  }();
  return v;
}

// replay on BVH scenes: the environment traversal culled at the receiver's t (default), or not
// culled (RFRT_COV_RXFIRST=0, for A/B checks); either way the receiver is queried first
bool replay_rx_first() {
  static const bool v = [] {
    const char* e = getenv("RFRT_COV_RXFIRST");
    return !(e && e[0] == '0');
  }();
  return v;
}

int bits_for(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

int64_t cov_ncell(const rt_coverage* c) { return c->grid.nx * c->grid.ny * c->grid.nz; }
int own_shift(const rt_coverage* c) { return 32 + bits_for((uint64_t)cov_ncell(c)); }

// reduced ray-mode records are sorted by (owner, cell, bin): bounds[o] = first record of owner o,
// bounds[world] = the valid records (the dropped ~0 keys sort last)
// Owner bounds and send buffers in one launch: every thread finds the owner boundaries at its
// record and writes the record's row, if it is valid (dropped records, ~0, sort last) and inside the
// caller's capacity (the host sees the count and grows the buffer when it was too small)
__global__ __launch_bounds__(256) void k_bounds_strip(const uint64_t* ukeys, const Fx192* usums, const int64_t* nuniq,
                                                      int world, int64_t cap, int shift, int64_t* bounds,
                                                      uint64_t* out) {
  const int64_t nu = *nuniq;
  const uint64_t mask = (1ull << shift) - 1;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= nu; u += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = u < nu ? ukeys[u] : ~0ull;
    const int64_t hi = k == ~0ull ? (int64_t)world : (int64_t)(k >> shift);
    const int64_t lo = u == 0 ? -1 : (ukeys[u - 1] == ~0ull ? (int64_t)world : (int64_t)(ukeys[u - 1] >> shift));
    for (int64_t o = lo + 1; o <= hi; ++o) bounds[o] = u;  // owners lo+1 .. hi start at u
    if (out && k != ~0ull && u < cap) {
      const Fx192 v = usums[u];
      typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
      u64x2* row = reinterpret_cast<u64x2*>(out + 4 * u);  // 32-B rows: two 16-B stores
      row[0] = u64x2{k & mask, v.w0};
      row[1] = u64x2{v.w1, v.w2};
    }
  }
}

// field widths of the compact record key [owner | cell | bin | ray]
struct KeyBits {
  int ray, bin, cell, own;
  int total() const { return own + cell + bin + ray; }
};
KeyBits key_bits(const rt_coverage* c, int64_t n_bins) {
  KeyBits k;
  k.ray = 0;  // bins are summed exactly (Fx192), so the order within a bin needs no ray field
  k.bin = std::max(1, bits_for((uint64_t)(n_bins - 1)));
  k.own = c->ray_mode ? bits_for((uint64_t)(c->nshard - 1)) : 0;
  const int64_t world = c->ray_mode ? c->nshard : 1;
  const int64_t nown = (c->grid.nx + world - 1) / world * c->grid.ny * c->grid.nz;  // cells per owner (record_key)
  k.cell = std::max(1, bits_for((uint64_t)(nown - 1)));
  return k;
}
// Sort end bit of the replay's records.  Dropped records carry ~0 and must sort after every valid
// key: with end_bit = total they do whenever no valid key has all `total` bits set (an all-ones
// bin, owner-local cell or owner field is out of range), which saves the extra bit -- and, at
// 30 bits, a whole radix pass (K3).
int record_sort_bits(const rt_coverage* c, const KeyBits& k, int64_t n_bins) {
  const int64_t world = c->ray_mode ? c->nshard : 1;
  const int64_t nown = (c->grid.nx + world - 1) / world * c->grid.ny * c->grid.nz;
  const bool safe = ((1ll << k.bin) - 1 >= n_bins) || ((1ll << k.cell) - 1 >= nown) ||
                    (k.own > 0 && (1ll << k.own) - 1 >= world);
  return k.total() + (safe ? 0 : 1);
}
// the compact keys of the sort -> wide keys; `owner_local`: the cell field is record_key's
// owner-local index (the trace stage of a ray-sharded plan), else a global cell id
WideKey wide_key(const rt_coverage* c, const KeyBits& k, bool owner_local = true) {
  return WideKey{k.ray, k.bin, k.cell, own_shift(c), c->grid.nx, owner_local && c->ray_mode ? (int64_t)c->nshard : 1};
}

// Stages 1-4 (trajectories, candidates, exact receiver tests, replay): the first-win records of
// this plan's rays as (compact record key, amplitude) in c->okeys / c->oamps, in candidate order.
int cov_records(rt_coverage* c, const float* tx_pos, double tx_power, double light_speed, double sample_rate,
                int flags, int64_t n_bins, hipStream_t s, int64_t* ncand_out, int64_t* nlist_out) {
  CovParams p{};
  p.env_perm = c->env->perm;
  p.env_nrm = c->env->nrm;
  p.env_nf = (int)c->env->nf;
  p.env_bvh = rt::bvh_view(c->env);
  const bool bvh = c->env->nodes != nullptr;
  for (int k = 0; k < 3; ++k) p.tx[k] = tx_pos[k];
  p.B = c->B;
  p.n = c->n;
  p.ray_offset = c->ray_offset;
  p.g = c->grid;
  p.r_rx = c->r_rx;
  {
    // every receiver vertex lies within r of the centre (|unit| = 1 up to rounding); pad for f32/f64 rounding
    const double amax = fmax(fabs(c->grid.x0) + fabs(c->grid.dx) * (double)c->grid.nx,
                             fmax(fabs(c->grid.y0) + fabs(c->grid.dy) * (double)c->grid.ny,
                                  fabs(c->grid.z0) + fabs(c->grid.dz) * (double)c->grid.nz));
    p.r_pad = c->r_rx * (1.0 + 1e-3) + 1e-5 * (1.0 + amax);
  }
  // cell-sharded plans skip other ranks' columns from the candidate passes on; ray-sharded plans
  // find candidates in every cell and tag each record with its cell's owner instead
  p.shard = c->ray_mode ? 0 : c->shard;
  p.nshard = c->ray_mode ? 1 : c->nshard;
  p.own_world = c->ray_mode ? c->nshard : 1;
  p.own_shift = own_shift(c);
  p.traj = c->traj;
  p.nseg = c->nseg;
  p.count = c->counters;
  p.item_count = c->counters + 1;
  p.amp0 = tx_power / (double)(c->n_total > 0 ? c->n_total : c->n);
  p.c32 = (float)light_speed;
  p.fs32 = (float)sample_rate;
  p.c64 = light_speed;
  p.fs64 = sample_rate;
  p.flags = flags;
  p.n_bins = n_bins;
  if (c->clear_on && !c->clear) {  // once per plan: the clear receivers (k_clear_cells)
    const int64_t nc = c->grid.nx * c->grid.ny * c->grid.nz;
    RT_HIP(hipMalloc(&c->clear, sizeof(uint32_t) * (size_t)((nc + 31) / 32)));
    const double amax = fmax(fabs(c->grid.x0) + fabs(c->grid.dx) * (double)c->grid.nx,
                             fmax(fabs(c->grid.y0) + fabs(c->grid.dy) * (double)c->grid.ny,
                                  fabs(c->grid.z0) + fabs(c->grid.dz) * (double)c->grid.nz));
    // the pad: 2e-3 r + 1e-4 (1 + |coordinates|), against ~1e-5 of f32 rounding in a hit point
    const double r_clear = c->r_rx * (1.0 + 2e-3) + 1e-4 * (1.0 + amax);
    const dim3 gcl((unsigned)std::min<int64_t>((nc + 255) / 256, 8192));
    if (bvh) hipLaunchKernelGGL(k_clear_cells<true>, gcl, dim3(256), 0, s, p, r_clear, c->clear);
    else hipLaunchKernelGGL(k_clear_cells<false>, gcl, dim3(256), 0, s, p, r_clear, c->clear);
    RT_HIP(hipGetLastError());
    RT_HIP(hipStreamSynchronize(s));  // once: later runs may come on other streams
  }
  p.clear = c->clear_on ? c->clear : nullptr;
  const size_t lds = bvh ? 0 : (size_t)p.env_nf * 18 * sizeof(float4);
  // k_replay: the deferred amplitude's B - 1 cosine columns follow the environment table
  const size_t lds_replay = lds + (size_t)std::max(p.B - 1, 1) * 256 * sizeof(float);
  const unsigned grid_rays = (unsigned)std::min<int64_t>((c->n + 255) / 256, 4096);
  p.order = nullptr;
  p.zero_ctr = c->counters;  // zeroed by the trajectory kernel (first attempt; retries use a fill)
  for (bool& r : c->ev_rec) r = false;
  if (bvh) {  // direction-sorted rows: coherent BVH traversal (as rt_trace)
    // The order depends only on the plan's ray ids (their initial directions, kernel.py:51-52), so
    // the plan sorts once, on its first run, and keeps the permutation (rt_trace, which has no
    // plan, sorts per call).  K5: ~0.1 ms per one-GPU map, a fixed ~30 us per rank of 8.
    // The plan's ray order puts the most nearly horizontal rays first (dir_order_banded: K5 rank of 8
    // 1.031 -> 0.982 ms, K5 map 3.77 -> 3.68 ms, r4z3); it depends only on the plan's ray ids, so the
    // library computes it once (dir_order_cached) and the plan keeps its own copy (the library's
    // entries may be evicted).
    if (!c->ray_order) {
      const int32_t* o = rt::dir_order_cached(c->ray_offset, c->n, s);
      if (!o) return RT_EHIP;
      RT_HIP(hipMalloc(&c->ray_order, sizeof(int32_t) * (size_t)c->n));
      RT_HIP(hipMemcpyAsync(c->ray_order, o, sizeof(int32_t) * (size_t)c->n, hipMemcpyDeviceToDevice, s));
    }
    p.order = c->ray_order;
    prof_mark(c, 0, s);
    if (c->n <= traj_split_max_rays()) {  // too few rays to fill the GPU: 16 / 4 lanes per ray
      const int64_t n1 = c->n / kTrajWideShare;
      const unsigned nb1 = (unsigned)std::max<int64_t>(1, (kTrajSplitWide * n1 + 255) / 256);
      const unsigned nb2 = (unsigned)std::max<int64_t>(1, (kTrajSplitG * (c->n - n1) + 255) / 256);
      hipLaunchKernelGGL((k_traj_split<kTrajSplitWide, kTrajSplitG>), dim3(nb1 + nb2), dim3(256), 0, s, p, n1, nb1);
    } else
      hipLaunchKernelGGL(k_traj<true>, dim3(grid_rays), dim3(256), lds, s, p);
    prof_mark(c, 1, s);
    p.order = nullptr;
  } else {
    p.order = c->sectors ? c->ray_order : nullptr;  // sector plans: the listed global ids
    prof_mark(c, 0, s);
    if (c->n <= traj_split_max_rays())  // few rays: G lanes per ray
      hipLaunchKernelGGL(k_traj_lds_split<kTrajLdsSplit>,
                         dim3((unsigned)std::min<int64_t>((kTrajLdsSplit * c->n + 255) / 256, 8192)), dim3(256),
                         lds, s, p);
    else
      hipLaunchKernelGGL(k_traj<false>, dim3(grid_rays), dim3(256), lds, s, p);
    prof_mark(c, 1, s);
    p.order = nullptr;
  }
  RT_HIP(hipGetLastError());
  if (c->profile) {
    RT_HIP(hipMemsetAsync(c->work, 0, 16, s));
    hipLaunchKernelGGL(k_count_segments, dim3(1024), dim3(256), 0, s, c->nseg, c->n, c->work);
  }
  // candidates: column items (pass A) then cells (pass B), the exact receiver tests and the
  // first-win list, with one host synchronize for all three counts (k_win and k_sel_* read the
  // candidate count on the device); grow and retry on overflow
  const KeyBits kb = key_bits(c, n_bins);
  if (kb.total() > 62) {
    rt::set_error("rt_coverage_run: rays x cells x bins x ranks exceed the 63-bit record key");
    return RT_EINVAL;
  }
  p.bin_bits = kb.bin;
  p.cell_bits = kb.cell;
  int64_t ncand = 0, nrec = 0, nlist = 0;
  const unsigned grid_items = 4096;
  // k_cols' slot-group stride: coprime to the group count, so that a block's 16 groups spread over
  // a rank-sized burst (one round of blocks, where the heavy blocks would set the time); a whole map
  // keeps its slots in order (stride 1: many rounds of blocks balance it, and the scattered
  // trajectory reads cost more -- one-GPU maps 62 -> 70 us with the stride, r6z)
  const int64_t col_groups = std::max<int64_t>(1, (c->n + kColGroup - 1) / kColGroup);
  int64_t col_step = 1;
  if (c->n <= traj_split_max_rays()) {
    col_step = std::max<int64_t>(1, col_groups / 16);
    while (std::gcd(col_step, col_groups) != 1) ++col_step;
  }
  // Replay launched before the list length reaches the host (early replay): the kernels read it
  // from the device counter, so the host's counter read-back and its wake-up (~36 us per K3 rank
  // of 8, profiles/r3j_k3.timeline.txt) overlap the replay instead of idling the GPU.  Only for
  // lists the window order takes (a rank's share); the whole-map lists keep the device-wide sort,
  // which needs the length on the host.  The previous run's length sizes the grid.
  // The replay-order workspace, laid out for the plan's capacity (k_sel_scatter fills its first half
  // before the list length is known): keys in / out, entries in / out, then the sort's scratch.
  // Taken afresh at every use: an overflowing attempt regrows the buffers (alloc_cands).
  struct Rord {
    uint16_t *k_in, *k_out;
    int32_t *v_in, *v_out;
    void* tmp;
    size_t tmp_bytes;
  };
  auto rord = [c]() {
    const size_t rkb = rord_key_bytes(c->cap), rrb = rord_row_bytes(c->cap);
    char* w = (char*)c->rord;
    return Rord{(uint16_t*)w, (uint16_t*)(w + rkb), (int32_t*)(w + 2 * rkb), (int32_t*)(w + 2 * rkb + rrb),
                w + 2 * rkb + 2 * rrb, c->rord_bytes - 2 * rkb - 2 * rrb};
  };
  // whole-map lists (plans not replayed early) get their order keys from k_sel_scatter
  const bool pre_keys = !(c->ray_mode && c->nshard > 1);
  auto launch_replay = [&](int64_t nl, const unsigned long long* nl_dev, bool windows, int64_t grid_hint) {
    const unsigned grid_l = (unsigned)std::max<int64_t>(1, std::min<int64_t>((grid_hint + 255) / 256, 8192));
    const Rord ro = rord();
    uint16_t* k_in = ro.k_in;
    uint16_t* k_out = ro.k_out;
    int32_t* v_in = ro.v_in;
    int32_t* v_out = ro.v_out;
    if (windows) {
      const unsigned grid_w = (unsigned)((nl + kReplayWin - 1) / kReplayWin);
      if (bvh)
        hipLaunchKernelGGL(k_replay_order<true>, dim3(grid_w), dim3(1024), 0, s, p, c->ritems, nl, nl_dev, v_out);
      else
        hipLaunchKernelGGL(k_replay_order<false>, dim3(grid_w), dim3(1024), 0, s, p, c->ritems, nl, nl_dev, v_out);
    } else {
      if (!pre_keys)  // (k_sel_scatter wrote them for plans whose lists are not replayed early)
        hipLaunchKernelGGL(k_replay_keys, dim3(grid_l), dim3(256), 0, s, p, c->ritems, nl, k_in, v_in);
      size_t sb = ro.tmp_bytes;
      RT_HIP((onesweep_pairs<rocprim::default_config, uint16_t, int32_t>(ro.tmp, sb, k_in, k_out, v_in, v_out,
                                                                         (unsigned)nl, 16u, s)));
    }
    prof_mark(c, 4, s);
    // the processing order (window order or the device-wide sort) of the items
    const ReplayItem* rit = c->ritems;
    const int32_t* rord = v_out;
    // BVH scenes: receiver first, the traversal culled at its t (K5 replay 3.47 -> 2.7 ms); the
    // LDS brute force tests every face anyway (a plane-culled variant measured 5% slower on K3,
    // a receiver-first one skipping faces beyond the receiver's t 5% slower too: 2.50 vs 2.63 ms,
    // profiles/r2x_cov_rxfirst_lds_ab.jsonl)
    if (bvh && replay_rx_first())
      hipLaunchKernelGGL((k_replay<true, true>), dim3(grid_l), dim3(256), lds_replay, s, p, rit, nl, nl_dev, rord,
                         c->okeys, c->oamps);
    else if (bvh)
      hipLaunchKernelGGL((k_replay<true, false>), dim3(grid_l), dim3(256), lds_replay, s, p, rit, nl, nl_dev, rord,
                         c->okeys, c->oamps);
    else
      hipLaunchKernelGGL((k_replay<false, false>), dim3(grid_l), dim3(256), lds_replay, s, p, rit, nl, nl_dev, rord,
                         c->okeys, c->oamps);
    prof_mark(c, 5, s);
    RT_HIP(hipGetLastError());
    return 0;
  };
  bool replayed = false;
  for (int attempt = 0;; ++attempt) {
    p.items = c->items;
    p.item_cap = c->item_cap;
    p.keys = c->keys;
    p.cap = c->cap;
    if (attempt > 0) RT_HIP(hipMemsetAsync(c->counters, 0, 32, s));
    hipLaunchKernelGGL(k_cols, dim3(grid_rays), dim3(256), 0, s, p, col_groups, col_step);
    hipLaunchKernelGGL(k_cells, dim3(grid_items), dim3(256), 0, s, p);
    const unsigned grid_c = (unsigned)std::min<int64_t>((c->cap + 255) / 256, 8192);
    prof_mark(c, 2, s);
    hipLaunchKernelGGL(k_win, dim3(grid_c), dim3(256), 0, s, p, c->keys, (const unsigned long long*)c->counters,
                       c->cap, c->first_flag, c->trx, c->gmask);
    prof_mark(c, 3, s);
    {  // ordered first-win list; tile counts in c->tcos (free until the run sums)
      const unsigned G = (unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, c->cap / 2048));
      int32_t* tiles = reinterpret_cast<int32_t*>(c->tcos);
      hipLaunchKernelGGL(k_sel_count, dim3(G), dim3(256), 0, s, c->first_flag, (const unsigned long long*)c->counters,
                         c->cap, tiles);
      hipLaunchKernelGGL(k_sel_scatter, dim3(G), dim3(256), 0, s, c->first_flag,
                         (const unsigned long long*)c->counters, c->cap, tiles, c->keys, c->trx, c->gmask, c->ritems,
                         c->counters + 2, p.B, pre_keys ? rord().k_in : nullptr, pre_keys ? rord().v_in : nullptr,
                         c->hcnt_dev);
    }
    RT_HIP(hipGetLastError());
    // k_sel_scatter wrote the counters to pinned memory ahead of the replay, and the host waits for
    // that kernel only; the list holds at most cap entries (one per candidate)
    RT_HIP(hipEventRecord(c->ev_cnt, s));
    // early (windowed) replay only for rank plans of a ray-sharded map, whose lists are a rank's
    // share: a one-GPU or cell-sharded plan's whole-map list takes the device-wide sort,
    // which needs the length on the host.  The previous run's length (or the cap) sizes the grid and
    // vetoes the window order once a rank's list outgrows kReplayWindowMax; the kernels stride over
    // the device count either way, so a stale length costs time, never correctness.
    replayed = c->ray_mode && c->nshard > 1 &&
               (c->last_list > 0 ? c->last_list : c->cap) <= g_replay_window_max.load();
    if (replayed) {
      int rc = launch_replay(c->cap, (const unsigned long long*)c->counters + 2, true,
                             c->last_list > 0 ? c->last_list + c->last_list / 8 : c->cap);
      if (rc) return rc;
    }
    RT_HIP(hipEventSynchronize(c->ev_cnt));
    const unsigned long long h[3] = {c->hcnt[0], c->hcnt[1], c->hcnt[2]};
    ncand = (int64_t)h[0];
    const int64_t nitems = (int64_t)h[1];
    nlist = (int64_t)h[2];
    if (ncand <= c->cap && nitems <= c->item_cap) break;
    if (attempt >= 3) {
      rt::set_error("rt_coverage_run: candidate buffers keep overflowing");
      return RT_EHIP;
    }
    if (nitems > c->item_cap) {
      int rc = alloc_items(c, nitems + nitems / 4 + 1024, s);
      if (rc) return rc;
      continue;  // keys were produced from a truncated item list: redo
    }
    int rc = alloc_cands(c, ncand + ncand / 4 + 1024, s);
    if (rc) return rc;
  }
  if (ncand > ((int64_t)1 << 31) - 1) {
    rt::set_error("rt_coverage_run: more than 2^31 candidates; shard the rays");
    return RT_EINVAL;
  }
  c->last_candidates = ncand;
  c->last_list = nlist;
  *ncand_out = ncand;
  if (ncand > 0) {
    if (nlist > 0) {
      if (!replayed) {
        int rc = launch_replay(nlist, nullptr, nlist <= g_replay_window_max.load(), nlist);
        if (rc) return rc;
      }
      if (c->profile)
        hipLaunchKernelGGL(k_count_replay, dim3(1024), dim3(256), 0, s, c->ritems, nlist, p.B, c->work + 1);
    }
    nrec = nlist;
  }
  c->last_received = nrec;
  *nlist_out = nrec;
  return RT_OK;
}

Fx192* plan_sums(rt_coverage* c) { return reinterpret_cast<Fx192*>(c->ev); }  // 32 B per slot, free until k_terms

int grow_for(rt_coverage* c, int64_t n, hipStream_t s) {
  // records gathered from several ranks can outgrow this rank's candidate buffers
  return n > c->cap ? alloc_cands(c, n + n / 4 + 1024, s) : RT_OK;
}

// exact sums of the runs of sorted records (keys in c->okeys_sorted) into c->ukeys / plan_sums /
// c->nuniq, then their f64 values into c->uamps
template <typename Val>
int run_sums(rt_coverage* c, Val val, int64_t n, WideKey wk, hipStream_t s) {
  const int64_t T = std::max<int64_t>(kMinTile, (n + 64 * kMaxTiles - 1) / (64 * kMaxTiles) * 64);
  const int64_t ntiles = (n + T - 1) / T;
  TileMeta tm;
  tm.heads = c->runs;
  tm.tail_u = reinterpret_cast<int64_t*>(c->runs + 2 * kMaxTiles);
  tm.headpart = reinterpret_cast<Fx192*>(c->tcos);  // free until k_terms
  tm.tailpart = tm.headpart + kMaxTiles;
  hipLaunchKernelGGL(k_tile_heads, dim3((unsigned)ntiles), dim3(256), 0, s, c->okeys_sorted, n, T, tm.heads);
  hipLaunchKernelGGL(k_tile_sums<Val>, dim3((unsigned)ntiles), dim3(64), 0, s, c->okeys_sorted, val, n, T, ntiles, tm,
                     wk, c->ukeys, plan_sums(c), c->uamps, c->nuniq);
  hipLaunchKernelGGL(k_cross_tiles, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, ntiles, tm, plan_sums(c),
                     c->uamps);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

// sort + exact reduce of this plan's records (c->okeys / c->oamps or caller buffers)
int cov_reduce(rt_coverage* c, const uint64_t* keys, const double* amps, int64_t n, int sort_bits, WideKey wk,
               hipStream_t s) {
  int rc = grow_for(c, n, s);
  if (rc) return rc;
  size_t tb = c->tmp_bytes;
  RT_HIP(sort_records(c->tmp, tb, keys, c->okeys_sorted, amps, c->oamps_sorted, n, sort_bits < 64 ? sort_bits : 64, s));
  return run_sums(c, AmpVal{c->oamps_sorted}, n, wk, s);
}

// owner stage: received (compact key, Fx192 sum) records -> sorted by key (index payload), summed
// keys: compact keys of the records; words: record j's exact sum at words[j * stride .. + 2]
int cov_reduce_sums(rt_coverage* c, const uint64_t* keys, const uint64_t* words, int64_t stride, int64_t n,
                    int sort_bits, WideKey wk, hipStream_t s) {
  int rc = grow_for(c, n, s);
  if (rc) return rc;
  int64_t* idx = reinterpret_cast<int64_t*>(c->oamps);  // filled by k_compact_keys
  int64_t* idx_sorted = reinterpret_cast<int64_t*>(c->oamps_sorted);
  size_t tb = c->tmp_bytes;
  RT_HIP(sort_records(c->tmp, tb, keys, c->okeys_sorted, (const int64_t*)idx, idx_sorted, n,
                      sort_bits < 64 ? sort_bits : 64, s));
  return run_sums(c, SumVal{words, idx_sorted, stride}, n, wk, s);
}

// Closed-form signal power of this plan's cells from the reduced records in c->ukeys / c->uamps
// (nrec: host upper bound of their count); other ranks' cells are zero-filled.
PowerParams power_params(int64_t n_bins, double alpha) {
  PowerParams P;
  P.n_bins = n_bins;
  P.half = (n_bins - 1) / 2;
  P.alpha = alpha;
  P.turns = alpha / 6.283185307179586;
  P.sin_a = sin(alpha);
  P.cos_a = cos(alpha);
  {  // as sincos_turns: the phase reduced to [-1/2, 1/2] turn first
    const double t = P.turns * (double)n_bins, f = t - std::rint(t);
    P.sin_n = sin(6.283185307179586 * f);
    P.cos_n = cos(6.283185307179586 * f);
  }
  return P;
}
// ranges_done: the terms, cell ranges (epoch c->range_epoch) and nbig reset were already written
// (k_owner_runs)
int cov_power(rt_coverage* c, int64_t nrec, int64_t n_bins, double alpha, double* power, hipStream_t s,
              bool ranges_done = false) {
  const int64_t ncell = cov_ncell(c);
  const PowerParams P = power_params(n_bins, alpha);
  // one wave per owned cell, 4 per block
  const unsigned grid_cells = (unsigned)std::min<int64_t>((ncell / c->nshard + 4) / 4, 4096);
  // one thread (kPowGroup lanes on small maps) per small cell, 64 per block: each sweep is a chain,
  // so a sharded map's few thousand cells must still spread over every CU
  const unsigned grid_small = (unsigned)std::min<int64_t>((ncell / c->nshard + 64) / 64, 16384);
  const TermArrays terms{c->ukeys, c->tcos, c->tsin, c->ev};
  // cells with more terms than k_power_small takes, listed by it for k_power (count reset by k_cell_ranges)
  int32_t* big = c->bigcells;
  unsigned* nbig = reinterpret_cast<unsigned*>(c->runs + 3 * c->cap + 1);
  if (!ranges_done) {
    const int32_t epoch = ++c->range_epoch;  // cells not stamped with it have no keys (k_cell_ranges)
    const unsigned grid_u = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nrec + 255) / 256, 8192));
    if (nrec > 0)
      hipLaunchKernelGGL(k_terms, dim3(grid_u), dim3(256), 0, s, c->ukeys, c->uamps, c->nuniq, P, c->tcos, c->tsin,
                         c->ev);
    hipLaunchKernelGGL(k_cell_ranges, dim3(grid_u), dim3(256), 0, s, c->ukeys, c->nuniq, ncell, c->cstart, c->cend,
                       c->cepoch, epoch, nbig);
  }
  const int32_t epoch = c->range_epoch;
  // Small maps: kPowGroup lanes per cell -- a rank of a sharded map owns few cells, and the chain of
  // one thread's serial sweep set its time (K3 rank of 8, 8k cells: 40 -> 19 us; the whole K3 map,
  // 65k cells, 55 -> 61 us).  Large maps: one thread per cell, the grouped form's staging and
  // searches cost more than they overlap (K5 map, 1M cells: 146 vs 231 us; K5 rank 48 vs 44 us,
  // r6r).  The choice depends on the map, never on the shard, so that every cell's power is summed
  // in the same order whoever owns it (a sharded map equals the whole map bit for bit).
  if (ncell <= kPowGroupMaxCells)
    hipLaunchKernelGGL((k_power_small<kPowGroup, kPowGroupMax>), dim3(std::min<int64_t>((int64_t)grid_small * kPowGroup, 65536)),
                       dim3(64), 0, s, terms, c->cstart, c->cend, c->cepoch, epoch, c->grid, c->shard, c->nshard, P,
                       power, big, nbig);
  else
    hipLaunchKernelGGL(k_power_small<1>, dim3(grid_small), dim3(64), 0, s, terms, c->cstart, c->cend, c->cepoch,
                       epoch, c->grid, c->shard, c->nshard, P, power, big, nbig);
  if (nrec > 0)
    hipLaunchKernelGGL(k_power, dim3(grid_cells), dim3(256), 0, s, terms, c->cstart, c->cend, big, nbig, P, power);
  RT_HIP(hipGetLastError());
  return RT_OK;
}
}  // namespace

extern "C" {

int rt_coverage_create(int device, const rt_mesh* env, int max_bounces, int64_t n_rays, int64_t ray_offset,
                       const rt_grid* grid, double rx_radius, int shard_index, int shard_count, rt_coverage** out) {
  if (!out || !env || !grid || max_bounces < 1 || max_bounces > 15 || n_rays <= 0 || n_rays > (1 << 24) ||
      shard_count < 1 || shard_index < 0 || shard_index >= shard_count || grid->nx < 1 || grid->ny < 1 || grid->nz < 1 ||
      rx_radius <= 0) {
    rt::set_error("rt_coverage_create: invalid arguments (max_bounces 1..15, n_rays 1..2^24 per call)");
    return RT_EINVAL;
  }
  const int64_t nc = grid->nx * grid->ny * grid->nz;
  if (bits_for((uint64_t)nc) > 32) {
    rt::set_error("rt_coverage_create: too many cells");
    return RT_EINVAL;
  }
  rt::DeviceGuard dg(device);
  RT_HIP(dg.err);
  int rc = RT_OK;
  rt_coverage* c = new rt_coverage();
  c->device = device;
  c->env = env;
  c->B = max_bounces;
  c->n = n_rays;
  c->ray_offset = ray_offset;
  c->grid = *grid;
  c->r_rx = rx_radius;
  c->shard = shard_index;
  c->nshard = shard_count;
  {
    const char* e = getenv("RFRT_COV_CLEAR");  // A/B and equivalence tests
    c->clear_on = !(e && e[0] == '0');
  }
  hipError_t e = hipMalloc(&c->traj, sizeof(float4) * 2 * max_bounces * n_rays);
  if (e == hipSuccess) e = hipMalloc(&c->nseg, n_rays);
  if (e == hipSuccess) e = hipMalloc(&c->counters, 32);
  if (e == hipSuccess) e = hipMalloc(&c->nuniq, 8);
  if (e == hipSuccess) e = hipMemset(c->nuniq, 0, 8);  // rt_coverage_received before any run: nothing
  if (e == hipSuccess) e = hipMalloc(&c->cstart, sizeof(int32_t) * nc);
  if (e == hipSuccess) e = hipMalloc(&c->cend, sizeof(int32_t) * nc);
  if (e == hipSuccess) e = hipMalloc(&c->bigcells, sizeof(int32_t) * nc);
  if (e == hipSuccess) e = hipMalloc(&c->cepoch, sizeof(int32_t) * nc);
  if (e == hipSuccess) e = hipMemset(c->cepoch, 0, sizeof(int32_t) * nc);  // epochs start at 1
  if (e == hipSuccess) e = hipMalloc(&c->own_aux, 16);
  if (e == hipSuccess) e = hipMemset(c->own_aux, 0, 16);
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->hcnt, 32, hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->hcnt_dev, c->hcnt, 0);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_cnt, hipEventDisableTiming);
  if (e != hipSuccess) {
    rt_coverage_destroy(c);
    return rt::hip_fail(e, "rt_coverage_create");
  }
  rc = alloc_cands(c, std::max<int64_t>(1 << 20, 8 * n_rays), nullptr);  // nothing in flight yet
  if (!rc) rc = alloc_items(c, std::max<int64_t>(1 << 20, 8 * n_rays), nullptr);
  if (rc) {
    rt_coverage_destroy(c);
    return rc;
  }
  *out = c;
  return RT_OK;
}

int rt_coverage_destroy(rt_coverage* c) {
  if (!c) return RT_OK;
  rt::DeviceGuard dg(c->device);
  (void)hipDeviceSynchronize();  // the plan does not know its callers' streams; errors are not reported here
  (void)free_cands(c, nullptr);
  if (c->traj) (void)hipFree(c->traj);
  if (c->ray_order) (void)hipFree(c->ray_order);
  if (c->clear) (void)hipFree(c->clear);
  if (c->nseg) (void)hipFree(c->nseg);
  if (c->counters) (void)hipFree(c->counters);
  if (c->nuniq) (void)hipFree(c->nuniq);
  if (c->cstart) (void)hipFree(c->cstart);
  if (c->cend) (void)hipFree(c->cend);
  if (c->bigcells) (void)hipFree(c->bigcells);
  if (c->cepoch) (void)hipFree(c->cepoch);
  if (c->own_aux) (void)hipFree(c->own_aux);
  if (c->items) (void)hipFree(c->items);
  if (c->bounds) (void)hipFree(c->bounds);
  if (c->work) (void)hipFree(c->work);
  for (hipEvent_t e : c->pev)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_cnt) (void)hipEventDestroy(c->ev_cnt);
  if (c->hcnt) (void)hipHostFree(c->hcnt);
  if (c->hbounds) (void)hipHostFree(c->hbounds);
  delete c;
  return RT_OK;
}

int rt_coverage_run(rt_coverage* c, const float* tx_pos, double tx_power, double light_speed, double sample_rate,
                    int flags, int64_t n_bins, double alpha, double* power, int64_t* stats, void* stream) {
  if (!c || !tx_pos || !power || n_bins < 1 || n_bins >= ((int64_t)1 << 32) || c->ray_mode) {
    rt::set_error(c && c->ray_mode ? "rt_coverage_run: a ray-sharded plan runs through rt_coverage_trace_rows_async"
                                   : "rt_coverage_run: invalid arguments");
    return RT_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  int64_t ncand = 0, nlist = 0;
  int rc = rt::g_poison >= 0 ? poison_plan(c, s) : RT_OK;
  if (rc) return rc;
  rc = cov_records(c, tx_pos, tx_power, light_speed, sample_rate, flags, n_bins, s, &ncand, &nlist);
  if (rc) return rc;
  // records grouped by (cell, bin) and summed exactly (Fx192); dropped records (~0) sort last
  prof_mark(c, 6, s);
  if (nlist > 0) {
    const KeyBits kb = key_bits(c, n_bins);
    rc = cov_reduce(c, c->okeys, c->oamps, nlist, record_sort_bits(c, kb, n_bins), wide_key(c, kb), s);
    if (rc) return rc;
  } else {
    RT_HIP(hipMemsetAsync(c->nuniq, 0, 8, s));
  }
  rc = cov_power(c, nlist, n_bins, alpha, power, s);
  if (rc) return rc;
  prof_mark(c, 7, s);
  if (stats) {
    stats[0] = ncand;
    stats[1] = nlist;
  }
  return RT_OK;
}

int rt_coverage_create_rays(int device, const rt_mesh* env, int max_bounces, int64_t n_rays_total, int64_t ray_offset,
                            int64_t n_rays, const rt_grid* grid, double rx_radius, int rank, int world,
                            rt_coverage** out) {
  if (!out || world < 1 || rank < 0 || rank >= world || n_rays_total < 1 || ray_offset < 0 ||
      ray_offset + n_rays > n_rays_total || !grid || grid->nx < 1 || grid->ny < 1 || grid->nz < 1) {
    rt::set_error("rt_coverage_create_rays: invalid arguments (0 <= rank < world, ray range inside the burst)");
    return RT_EINVAL;
  }
  const uint64_t nc = (uint64_t)(grid->nx * grid->ny * grid->nz);
  if (32 + bits_for(nc) + bits_for((uint64_t)(world - 1)) > 63) {
    rt::set_error("rt_coverage_create_rays: cells x ranks exceed the 63-bit record key");
    return RT_EINVAL;
  }
  rt_coverage* c = nullptr;
  int rc = rt_coverage_create(device, env, max_bounces, n_rays, ray_offset, grid, rx_radius, rank, world, &c);
  if (rc) return rc;
  c->n_total = n_rays_total;
  c->ray_mode = true;
  if (hipMalloc(&c->bounds, sizeof(int64_t) * (world + 1)) != hipSuccess ||
      hipHostMalloc((void**)&c->hbounds, sizeof(int64_t) * (world + 2), hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&c->hbounds_dev, c->hbounds, 0) != hipSuccess) {
    rt_coverage_destroy(c);
    return rt::hip_fail(hipErrorOutOfMemory, "rt_coverage_create_rays");
  }
  *out = c;
  return RT_OK;
}

constexpr int kSectorSlices = 4;
int rt_coverage_create_sectors(int device, const rt_mesh* env, int max_bounces, int64_t n_rays_total,
                               const rt_grid* grid, double rx_radius, int rank, int world, rt_coverage** out) {
  if (!out || world < 1 || rank < 0 || rank >= world || n_rays_total < world || n_rays_total > (1 << 24)) {
    rt::set_error("rt_coverage_create_sectors: invalid arguments (0 <= rank < world <= n_rays_total <= 2^24)");
    return RT_EINVAL;
  }
  // Four interleaved wedges per rank (pieces r, r + W, r + 2W, r + 3W of the azimuth order): one
  // wedge per rank left the ranks unbalanced (the transmitter sits off-centre: K3 rank trace stages
  // 0.575-0.693 ms, K5 0.667-0.820), four balance them and keep the locality (K3 slowest rank with
  // the modelled collectives 0.875 ms against 0.933 for ray-id ranges and 0.891 for 16 wedges; K5
  // 1.124 / 1.149 / 1.142 ms; profiles/r6b_*, r6f_*)
  const int slices = (int64_t)world * kSectorSlices <= n_rays_total ? kSectorSlices : 1;
  const int64_t m = rt::sector_ray_count(n_rays_total, rank, world, slices);
  rt_coverage* c = nullptr;
  int rc = rt_coverage_create_rays(device, env, max_bounces, n_rays_total, 0, m, grid, rx_radius, rank, world, &c);
  if (rc) return rc;
  rt::DeviceGuard dg(device);
  c->sectors = true;
  c->ray_offset = 0;
  if (hipMalloc(&c->ray_order, sizeof(int32_t) * (size_t)m) != hipSuccess) {
    rt_coverage_destroy(c);
    return rt::hip_fail(hipErrorOutOfMemory, "rt_coverage_create_sectors");
  }
  rc = rt::sector_ray_ids(n_rays_total, rank, world, slices, c->ray_order, nullptr);
  if (rc) {
    rt_coverage_destroy(c);
    return rc;
  }
  *out = c;
  return RT_OK;
}

namespace {
// The trace stage of a ray-sharded plan: this rank's first-win records, summed exactly per
// (owner, cell, bin) and written as 32-B rows (key without the owner field, three sum words) into
// rows_out, grouped by owner (rank 0 first), when they fit (max_out rows); the send counts go to
// counts_dev on the device.  No host wait: trace_rows_finish does it.
int trace_rows_impl(rt_coverage* c, const float* tx_pos, double tx_power, double light_speed, double sample_rate,
                    int flags, int64_t n_bins, uint64_t* rows_out, int64_t max_out, int64_t* counts_dev,
                    hipStream_t s) {
  if (!c || !c->ray_mode || !tx_pos || !counts_dev || n_bins < 1 || n_bins >= ((int64_t)1 << 32)) {
    rt::set_error("rt_coverage_trace_rows_async: invalid arguments (needs a ray-sharded plan)");
    return RT_EINVAL;
  }
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  const int world = c->nshard;
  int64_t ncand = 0, nlist = 0;
  int rc = rt::g_poison >= 0 ? poison_plan(c, s) : RT_OK;
  if (rc) return rc;
  rc = cov_records(c, tx_pos, tx_power, light_speed, sample_rate, flags, n_bins, s, &ncand, &nlist);
  if (rc) return rc;
  // local exact sum per (owner, cell, bin); runs of each owner are then contiguous
  prof_mark(c, 6, s);
  if (nlist > 0) {
    const KeyBits kb = key_bits(c, n_bins);
    // the send rows are written before the host synchronizes (no launch after it)
    if ((rc = grow_for(c, nlist, s))) return rc;
    size_t tb = c->tmp_bytes;
    const int sb = record_sort_bits(c, kb, n_bins);
    RT_HIP(sort_records(c->tmp, tb, c->okeys, c->okeys_sorted, c->oamps, c->oamps_sorted, nlist, sb < 64 ? sb : 64, s));
    SendRuns a{};
    a.keys = c->okeys_sorted;
    a.amps = c->oamps_sorted;
    a.n = nlist;
    a.states = c->own_states;
    const int64_t ntiles = (nlist + kSendTile - 1) / kSendTile;
    a.agg_tail = c->send_tails;
    a.inc_tail = a.agg_tail + 5 * (c->cap / kOwnTile + 2);
    a.ticket = c->own_aux;
    a.errors = reinterpret_cast<unsigned*>(c->own_aux + 1);
    a.tag = (c->own_tag++ % 0xFFFFFEull + 1ull) << 40;
    a.wk = wide_key(c, kb);
    a.world = world;
    a.own_shift = own_shift(c);
    a.ukeys = c->ukeys;
    a.usums = plan_sums(c);
    a.uamps = c->uamps;
    a.nuniq = c->nuniq;
    a.bounds = c->bounds;
    a.out = rows_out;
    a.cap = max_out;
    hipLaunchKernelGGL(k_send_runs, dim3((unsigned)ntiles), dim3(256), 0, s, a);
    RT_HIP(hipGetLastError());
    prof_mark(c, 7, s);
    // into pinned memory by k_bounds_to_counts (a pageable copy stages through the host: ~20 us of
    // gap per rank; two copy launches ~10 us): the bounds and the count of look-back waits that gave
    // up (k_send_runs here, k_owner_runs of an earlier owner stage), whose sums would be wrong, so
    // the run fails instead
    hipLaunchKernelGGL(k_bounds_to_counts, dim3(1), dim3(64), 0, s, c->bounds, world, counts_dev, c->hbounds_dev,
                       (const uint64_t*)(c->own_aux + 1));
  } else {
    for (int o = 0; o <= world + 1; ++o) c->hbounds[o] = 0;  // nothing sent (no copy in flight)
    RT_HIP(hipMemsetAsync(counts_dev, 0, sizeof(int64_t) * world, s));
  }
  RT_HIP(hipGetLastError());
  c->pend_ncand = ncand;
  c->pend_nlist = nlist;
  c->pend_max_out = max_out;
  return RT_OK;
}

// The host half of a trace stage: waits for the stream, then the bounds and the look-back error
// word copied to pinned memory by trace_rows_impl give the send counts.
int trace_rows_finish(rt_coverage* c, int64_t* counts, int64_t* stats, hipStream_t s) {
  const int world = c->nshard;
  RT_HIP(hipStreamSynchronize(s));
  if (const int64_t w = c->hbounds[world + 1]) {
    c->hbounds[world + 1] = 0;
    RT_HIP(hipMemset(c->own_aux + 1, 0, 8));
    rt::set_error((w & 0xFFFFFFFFll) ? "rt_coverage_trace_rows_finish: a look-back wait timed out (results discarded)"
                                     : "rt_coverage_trace_rows_finish: the previous owner stage received a segment "
                                       "out of key order (its power map was wrong)");
    return RT_EHIP;
  }
  for (int o = 0; o < world; ++o) counts[o] = c->hbounds[o + 1] - c->hbounds[o];
  c->n_out = c->hbounds[world];
  if (stats) {
    stats[0] = c->pend_ncand;
    stats[1] = c->pend_nlist;
    stats[2] = c->n_out <= c->pend_max_out ? 1 : 0;  // the rows are in the caller's buffer
  }
  return RT_OK;
}
}  // namespace

int rt_coverage_trace_rows_async(rt_coverage* c, const float* tx_pos, double tx_power, double light_speed,
                                 double sample_rate, int flags, int64_t n_bins, uint64_t* rows_out, int64_t max_out,
                                 int64_t* counts_dev, void* stream) {
  if (!rows_out || max_out < 0 || (reinterpret_cast<uintptr_t>(rows_out) & 15) || !counts_dev) {
    rt::set_error("rt_coverage_trace_rows_async: invalid arguments (16-B aligned rows_out, max_out >= 0, counts_dev)");
    return RT_EINVAL;
  }
  return trace_rows_impl(c, tx_pos, tx_power, light_speed, sample_rate, flags, n_bins, rows_out, max_out, counts_dev,
                         (hipStream_t)stream);
}

int rt_coverage_trace_rows_finish(rt_coverage* c, int64_t* counts, int64_t* stats, void* stream) {
  if (!c || !c->ray_mode || !counts || c->pend_max_out < 0) {
    rt::set_error("rt_coverage_trace_rows_finish: invalid arguments (after rt_coverage_trace_rows_async)");
    return RT_EINVAL;
  }
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  const int rc = trace_rows_finish(c, counts, stats, (hipStream_t)stream);
  c->pend_max_out = -1;
  return rc;
}

int rt_coverage_records_packed(rt_coverage* c, uint64_t* rows_out, int64_t max_out, void* stream) {
  if (!c || !c->ray_mode || (c->n_out > 0 && !rows_out) || max_out < c->n_out ||
      (reinterpret_cast<uintptr_t>(rows_out) & 15)) {
    rt::set_error("rt_coverage_records_packed: invalid arguments (16-B aligned rows, max_out >= the sum of the counts)");
    return RT_EINVAL;
  }
  if (c->n_out == 0) return RT_OK;
  hipStream_t s = (hipStream_t)stream;
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  // the reduced records are still in the plan (ukeys / sums, valid ones first): the same rows
  // k_send_runs writes (its bounds are rewritten with the same values)
  hipLaunchKernelGGL(k_bounds_strip, dim3((unsigned)std::min<int64_t>((c->n_out + 256) / 256, 4096)), dim3(256), 0, s,
                     c->ukeys, plan_sums(c), c->nuniq, c->nshard, max_out, own_shift(c), c->bounds, rows_out);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

int rt_coverage_amps_to_sums(const double* amps, int64_t n, uint64_t* sums, void* stream) {
  if (n < 0 || (n > 0 && (!amps || !sums))) {
    rt::set_error("rt_coverage_amps_to_sums: invalid arguments");
    return RT_EINVAL;
  }
  if (n == 0) return RT_OK;
  hipLaunchKernelGGL(k_amps_to_fx, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, amps, n, (Fx192*)sums);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

int rt_coverage_power_rows(rt_coverage* c, const uint64_t* rows, int64_t n, int64_t n_bins, double alpha, double* power,
                           void* stream) {
  if (!c || !c->ray_mode || n < 0 || (n > 0 && !rows) || !power || n_bins < 1 || n_bins >= ((int64_t)1 << 32) ||
      n > ((int64_t)1 << 31) - 1) {
    rt::set_error("rt_coverage_power_rows: invalid arguments");
    return RT_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  int rc = rt::g_poison >= 0 ? poison_plan(c, s) : RT_OK;
  if (rc) return rc;
  c->ev_rec[6] = c->ev_rec[7] = false;
  prof_mark(c, 6, s);
  if (n > 0) {
    // received (cell << 32 | bin) keys -> compact [cell | bin]; the partial sums are exact
    // fixed point, so their order is irrelevant
    if ((rc = grow_for(c, n, s))) return rc;
    KeyBits kb = key_bits(c, n_bins);
    kb.ray = 0;
    kb.own = 0;
    kb.cell = std::max(1, bits_for((uint64_t)(cov_ncell(c) - 1)));  // received keys carry global cells
    hipLaunchKernelGGL(k_compact_keys, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0, s, rows,
                       (int64_t)4, n, kb.bin, c->keys_sorted, reinterpret_cast<int64_t*>(c->oamps));
    RT_HIP(hipGetLastError());
    // received keys are valid ones (a ~0 key, never sent, would need the extra bit to sort last)
    const bool safe = ((1ll << kb.bin) - 1 >= n_bins) || ((1ll << kb.cell) - 1 >= cov_ncell(c));
    rc = cov_reduce_sums(c, c->keys_sorted, rows + 1, 4, n, kb.total() + (safe ? 0 : 1), wide_key(c, kb, false), s);
  } else {
    RT_HIP(hipMemsetAsync(c->nuniq, 0, 8, s));
  }
  if (!rc) rc = cov_power(c, n, n_bins, alpha, power, s);
  if (!rc) prof_mark(c, 7, s);
  return rc;
}

// The owner stage on received rows (key, sum words 0..2) arriving as nseg segments, segment t =
// seg_counts[t] rows from rank t, each strictly ascending by key: merged by rank, not sorted.
int rt_coverage_power_packed(rt_coverage* c, const uint64_t* rows, const int64_t* seg_counts, int nseg, int64_t n_bins,
                             double alpha, double* power, void* stream) {
  if (!c || !c->ray_mode || nseg < 1 || nseg > kMaxSegs || !seg_counts || !power || n_bins < 1 ||
      n_bins >= ((int64_t)1 << 32)) {
    rt::set_error("rt_coverage_power_packed: invalid arguments (1 <= nseg <= 64)");
    return RT_EINVAL;
  }
  constexpr int64_t stride = 4;  // (key, sum) rows: keys = rows, sums = rows + 1
  const uint64_t* keys = rows;
  const uint64_t* sums = rows ? rows + 1 : nullptr;
  SegOffsets so{};
  so.nseg = nseg;
  for (int t = 0; t < nseg; ++t) {
    if (seg_counts[t] < 0) {
      rt::set_error("rt_coverage_power_packed: negative segment count");
      return RT_EINVAL;
    }
    so.off[t + 1] = so.off[t] + seg_counts[t];
  }
  const int64_t n = so.off[nseg];
  if ((n > 0 && !rows) || n > ((int64_t)1 << 31) - 1) {
    rt::set_error("rt_coverage_power_packed: invalid arguments");
    return RT_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  int rc = rt::g_poison >= 0 ? poison_plan(c, s) : RT_OK;
  if (rc) return rc;
  c->ev_rec[6] = c->ev_rec[7] = false;
  prof_mark(c, 6, s);
  bool fused = false;
  if (n > 0) {
    if ((rc = grow_for(c, n, s))) return rc;
    int64_t* idx_sorted = reinterpret_cast<int64_t*>(c->oamps_sorted);
    // (G lanes per element, one binary search each, then a group sum: no faster on K3's 200k
    // records, 46 -> 76 us on K5's 465k -- the searches' loads, not their latency, set the time)
    int64_t longest = 0;
    for (int t = 0; t < nseg; ++t) longest = std::max<int64_t>(longest, seg_counts[t]);
    const int steps = bits_for((uint64_t)longest);  // a search over len keys takes <= bits(len) halvings
    const dim3 gm((unsigned)std::min<int64_t>((n + 255) / 256, 8192));
    // segments out of key order: counted in the high word of own_aux[1] (rt_coverage_check)
    unsigned* bad = reinterpret_cast<unsigned*>(c->own_aux + 1) + 1;
    if (nseg <= 2)
      hipLaunchKernelGGL(k_merge_lockstep<2>, gm, dim3(256), 0, s, keys, stride, so, steps, c->okeys_sorted, idx_sorted, bad);
    else if (nseg <= 4)
      hipLaunchKernelGGL(k_merge_lockstep<4>, gm, dim3(256), 0, s, keys, stride, so, steps, c->okeys_sorted, idx_sorted, bad);
    else if (nseg <= 8)
      hipLaunchKernelGGL(k_merge_lockstep<8>, gm, dim3(256), 0, s, keys, stride, so, steps, c->okeys_sorted, idx_sorted, bad);
    else
      hipLaunchKernelGGL(k_merge_segments, gm, dim3(256), 0, s, keys, stride, so, c->okeys_sorted, idx_sorted, bad);
    RT_HIP(hipGetLastError());
    if (nseg <= 8) {
      OwnerRuns a{};
      a.keys = c->okeys_sorted;
      a.val = SumVal{sums, idx_sorted, stride};
      a.n = n;
      a.states = c->own_states;
      a.ticket = c->own_aux;
      a.errors = reinterpret_cast<unsigned*>(c->own_aux + 1);
      const int64_t ntiles = (n + kOwnTile - 1) / kOwnTile;
      a.tag = (c->own_tag++ % 0xFFFFFEull + 1ull) << 40;
      a.ukeys = c->ukeys;
      a.uamps = c->uamps;
      a.tcos = c->tcos;
      a.tsin = c->tsin;
      a.ev = c->ev;
      a.nuniq = c->nuniq;
      a.ncell = cov_ncell(c);
      a.cstart = c->cstart;
      a.cend = c->cend;
      a.cepoch = c->cepoch;
      a.epoch = ++c->range_epoch;
      a.nbig = reinterpret_cast<unsigned*>(c->runs + 3 * c->cap + 1);
      a.P = power_params(n_bins, alpha);
      hipLaunchKernelGGL(k_owner_runs, dim3((unsigned)ntiles), dim3(256), 0, s, a);
      RT_HIP(hipGetLastError());
      fused = true;
    } else {
      WideKey wk{};
      wk.identity = true;
      rc = run_sums(c, SumVal{sums, idx_sorted, stride}, n, wk, s);
    }
  } else {
    RT_HIP(hipMemsetAsync(c->nuniq, 0, 8, s));
  }
  if (!rc) rc = cov_power(c, n, n_bins, alpha, power, s, fused);
  if (!rc) prof_mark(c, 7, s);
  return rc;
}

int rt_coverage_check(rt_coverage* c, int64_t* out, void* stream) {
  if (!c) {
    rt::set_error("rt_coverage_check: null plan");
    return RT_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  unsigned long long w = 0;
  RT_HIP(hipMemcpyAsync(&w, c->own_aux + 1, 8, hipMemcpyDeviceToHost, s));
  RT_HIP(hipStreamSynchronize(s));
  const int64_t timeouts = (int64_t)(w & 0xFFFFFFFFull), rejected = (int64_t)(w >> 32);
  if (out) {
    out[0] = timeouts;
    out[1] = rejected;
  }
  if (w) {
    RT_HIP(hipMemsetAsync(c->own_aux + 1, 0, 8, s));
    RT_HIP(hipStreamSynchronize(s));
    rt::set_error(timeouts ? "rt_coverage_check: a look-back wait timed out (the last results are wrong)"
                           : "rt_coverage_check: an owner-stage segment was out of key order (the last power "
                             "map is wrong)");
    return RT_EHIP;
  }
  return RT_OK;
}

int rt_debug_replay_window_max(int64_t n) {
  g_replay_window_max.store(n < 0 ? kReplayWindowMax : n);
  return RT_OK;
}

int rt_coverage_profile(rt_coverage* c, int enable) {
  if (!c) {
    rt::set_error("rt_coverage_profile: null plan");
    return RT_EINVAL;
  }
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  if (enable && !c->work) RT_HIP(hipMalloc(&c->work, 16));
  c->profile = enable != 0;
  return RT_OK;
}

int rt_coverage_last_profile(rt_coverage* c, double* out, int n) {
  if (!c || !out || n < 10) {
    rt::set_error("rt_coverage_last_profile: invalid arguments (out needs 10 doubles)");
    return RT_EINVAL;
  }
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  for (int i = 0; i < n; ++i) out[i] = NAN;
  auto span = [&](int a, int b) -> double {
    if (!c->profile || !c->ev_rec[a] || !c->ev_rec[b]) return NAN;
    float ms = 0.0f;
    if (hipEventSynchronize(c->pev[b]) != hipSuccess || hipEventElapsedTime(&ms, c->pev[a], c->pev[b]) != hipSuccess)
      return NAN;
    return (double)ms;
  };
  out[0] = span(0, 1);  // k_traj
  out[1] = span(1, 2);  // candidates: k_cols + k_cells (+ the host read of their counts)
  out[2] = span(2, 3);  // k_win
  out[3] = span(4, 5);  // k_replay
  out[4] = span(6, 7);  // record sort + reduce-by-key + power (or + owner bounds in ray mode)
  out[5] = span(0, 7);  // whole run
  if (c->profile && c->work) {
    unsigned long long w[2] = {0, 0};
    RT_HIP(hipMemcpy(w, c->work, 16, hipMemcpyDeviceToHost));
    out[6] = (double)w[0];
    out[7] = (double)w[1];
  }
  out[8] = (double)c->last_candidates;
  out[9] = (double)c->last_received;
  return RT_OK;
}

int rt_coverage_received(rt_coverage* c, uint64_t* keys_out, double* amps_out, int64_t max_out, int64_t* n_out,
                         void* stream) {
  // the per-cell sparse impulse responses of the last run (rt_coverage_run, or this rank's cells
  // after its owner stage): (cell << 32 | bin, amplitude), ascending
  if (!c || !n_out) {
    rt::set_error("rt_coverage_received: invalid arguments");
    return RT_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  rt::DeviceGuard dg(c->device);
  RT_HIP(dg.err);
  int64_t nu = 0;
  RT_HIP(hipMemcpyAsync(&nu, c->nuniq, 8, hipMemcpyDeviceToHost, s));
  RT_HIP(hipStreamSynchronize(s));
  if (nu > 0) {  // records dropped by the replay (bin past the window, zero amplitude) sort last as ~0
    uint64_t last = 0;
    RT_HIP(hipMemcpyAsync(&last, c->ukeys + nu - 1, 8, hipMemcpyDeviceToHost, s));
    RT_HIP(hipStreamSynchronize(s));
    if (last == ~0ull) --nu;
  }
  *n_out = nu;
  const int64_t m = std::min(nu, max_out);
  if (m > 0 && keys_out) RT_HIP(hipMemcpyAsync(keys_out, c->ukeys, m * 8, hipMemcpyDeviceToDevice, s));
  if (m > 0 && amps_out) RT_HIP(hipMemcpyAsync(amps_out, c->uamps, m * 8, hipMemcpyDeviceToDevice, s));
  return RT_OK;
}

// host self-test of the exact fixed point (tests/test_abi_host.py): op 0 = fx_to_double of n
// (w0, w1, w2) triples in w, op 1 = fx_from_double of the n doubles in a into w
int rt_selftest_fx(uint64_t* w, double* a, int64_t n, int op) {
  if (n < 0 || (n > 0 && (!w || !a)) || (op != 0 && op != 1)) {
    rt::set_error("rt_selftest_fx: invalid arguments");
    return RT_EINVAL;
  }
  for (int64_t i = 0; i < n; ++i) {
    if (op == 0) {
      a[i] = fx_to_double(Fx192{w[3 * i], w[3 * i + 1], w[3 * i + 2]});
    } else {
      const Fx192 f = fx_from_double(a[i]);
      w[3 * i] = f.w0;
      w[3 * i + 1] = f.w1;
      w[3 * i + 2] = f.w2;
    }
  }
  return RT_OK;
}

int rt_power_dense(const double* impulse_responses, int64_t rows, int64_t n_bins, double alpha, void* scratch,
                   int64_t scratch_bytes, double* power, void* stream) {
  if (!impulse_responses || rows < 0 || n_bins < 1 || !power || scratch_bytes < rows * n_bins * 16) {
    rt::set_error("rt_power_dense: invalid arguments (scratch >= rows*n_bins*16 bytes)");
    return RT_EINVAL;
  }
  if (rows == 0) return RT_OK;
  const PowerParams P = power_params(n_bins, alpha);
  uint64_t* kk = (uint64_t*)scratch;
  double* aa = (double*)(kk + rows * n_bins);
  hipLaunchKernelGGL(k_power_dense, dim3((unsigned)rows), dim3(64), 0, (hipStream_t)stream, impulse_responses, rows, P,
                     kk, aa, power);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

}  // extern "C"
