// trace.hip -- trace_paths_kernel (kernel.py:38-98) as CDNA4 HIP.
//
// One lane = one ray (global ray id = ray_offset + row).  The whole bounce loop runs in
// registers: position, direction and the P = B+1 path points never leave VGPRs until the
// final row stores.  The environment mesh is staged once per workgroup into LDS as the
// host-built permuted-corner table (288 B/face), so every lane reads its shear case with a
// conflict-free ds_read_b128 (6 cases = 6 distinct 16-B slots per face).  The receiver mesh
// (80 faces for the reference's icosphere) stays in HBM/L2: a conservative bounding-sphere
// test keeps nearly every wave from touching it.
//
// Semantics kept from the reference: no early exit (Q1: a miss repeats
// forever, so it is skipped, which changes nothing), an RX hit does not stop the ray (Q2),
// no t_min (Q3), no renormalisation after reflect (Q4), traced_paths is scratch (Q6).
#include <math.h>

#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>

#include "rt_bvh.h"
#include "rt_cir.h"
#include "rt_device.h"
#include "rt_internal.h"

#ifndef RT_DIAG_CAND  // diagnostics builds only (tools/k2_cand_stats.py)
#define RT_DIAG_CAND 0
#endif

namespace {

struct TraceArgs {
  const float4* env_perm;
  const float4* env_nrm;
  int env_nf;
  rt::BvhView env_bvh;  // used when the kernel is instantiated with USE_BVH
  const float4* rx_perm;
  int rx_nf;
  float rx_c[3];
  float rx_r2;  // conservative squared radius of the receiver's bounding sphere
  float tx[3];
  int64_t ray_offset;
  int64_t n;
  float* traced;    // (n, P, 3) or null
  float* received;  // (n, P, 3) or null
  uint32_t* mask;   // (n) or null
  int32_t* hit_kind;  // (n, B) or null
  int32_t* hit_face;  // (n, B) or null
  const int32_t* order;  // processing order of the rows (null = identity), see launch_trace
  const int32_t* sched;  // processing order of the 256-row chunks (null = identity), see chunk_schedule
  uint32_t* cost;        // per-chunk cost to record (null = off): wave time, 10 ns ticks, summed
  bool fused;             // brute-force kernels under rt_trace_cir: list received rows, per-path CIR
  rt::TraceCirFused fz;
  bool sparse_rx;  // received rows / mask words filled beforehand (k_fill_received): store only received rays'
  bool box_cull;   // bounces >= 1 of sorted brute-force bursts: the wave's candidate faces (wave_boxes)
  float env_pad;   // face boxes padded by 1e-5 * (1 + scene's largest |coordinate|), as the BVH's boxes
  // bounce 0: the receiver ball seen from the TX, unit axis rx_u and half-angle (sin, cos); rx_all0 when the
  // TX is inside (or nearly inside) the ball
  float rx_u[3], rx_sin, rx_cos;
  bool rx_all0;
  float cone_rho_max;  // bounce 0: wave cones when every |d_l - d_0| is below this
};

// Closest hit over a brute-force face list whose permuted table lives at `tab`
// (LDS for the environment, global for the receiver).
template <typename Ptr>
__device__ __forceinline__ rt::Hit query_faces(Ptr tab, int nf, const rt::Shear& s) {
  rt::LazyHit h;  // faces in ascending order: the division waits for the winner (rt_device.h)
  rt::lazy_init(h);
  const int off = s.kcase * 3;
  // unrolled by four: fewer loop branches / SALU per face (K2 115.1 -> 114.0 us against two, r2zc)
#pragma unroll 4
  for (int f = 0; f < nf; ++f) {
    const float4 q0 = tab[f * 18 + off + 0];
    const float4 q1 = tab[f * 18 + off + 1];
    const float c2 = tab[f * 18 + off + 2].x;
    float T, det;
    if (rt::tri_test(s, q0, q1, c2, T, det)) rt::lazy_consider(h, T, det, f);
  }
  return rt::lazy_finish(h);
}

// Can a receiver hit possibly be nearer than t_limit?  Conservative: the receiver's faces all
// lie inside the ball (centre c, squared radius r2 padded on the host).
__device__ __forceinline__ bool rx_maybe(const TraceArgs& a, float3 o, float3 d, float t_limit) {
  const float ox = o.x - a.rx_c[0], oy = o.y - a.rx_c[1], oz = o.z - a.rx_c[2];
  const float cc = ox * ox + oy * oy + oz * oz - a.rx_r2;
  if (cc <= 0.0f) return true;  // origin inside the ball
  const float b = ox * d.x + oy * d.y + oz * d.z;
  if (b >= 0.0f) return false;  // ball behind the origin
  const float dd = d.x * d.x + d.y * d.y + d.z * d.z;
  const float disc = b * b - dd * cc;
  if (disc < 0.0f) return false;
  const float t_enter = (-b - sqrtf(disc)) / dd;
  return t_enter <= t_limit * 1.0001f + 1e-4f;
}

// Row stores of the register-resident kernels.  Brute-force kernels use non-temporal (streaming)
// stores -- the rows are written once and not read back by this step, and a wave's rows are
// consecutive, so its stores fill whole lines.  The BVH kernels write direction-sorted rows at
// scattered row indices, every 72-B row a few partial lines; streaming stores sent each piece to
// memory on its own (1.0 GB written per K4 launch for 0.31 GB of rows), while ordinary stores let
// L2 merge a row's pieces first: 0.47 GB, and the K4 kernel 1230 -> 880 us (profiles/r3s_*).
// (8-byte row stores, rows transposed across the wave with ds_bpermute, XCD-affine row windows and
// the path points in LDS were measured no better and removed in round 5; last in commit 43de9a4.)
// received rows = NaN, row_mask = 0, in row order with 16-B streaming stores (BVH bursts, see trace_body)
__global__ __launch_bounds__(256) void k_fill_received(float* received, int64_t nwords, uint32_t* mask, int64_t n) {
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, str = (int64_t)gridDim.x * blockDim.x;
  const uint32_t qn = 0x7FC00000u;
  if (received) {
    uint32_t* w = reinterpret_cast<uint32_t*>(received);
    const int64_t head = (int64_t)((16 - (reinterpret_cast<uintptr_t>(w) & 15)) & 15) / 4;  // words to 16-B alignment
    const int64_t h = head < nwords ? head : nwords;
    const int64_t nv = (nwords - h) / 4;
    u4v* v = reinterpret_cast<u4v*>(w + h);
    for (int64_t i = tid; i < nv; i += str) __builtin_nontemporal_store(u4v{qn, qn, qn, qn}, v + i);
    if (tid < h) w[tid] = qn;
    for (int64_t i = h + 4 * nv + tid; i < nwords; i += str) w[i] = qn;
  }
  if (mask) {
    const int64_t h = (int64_t)((16 - (reinterpret_cast<uintptr_t>(mask) & 15)) & 15) / 4;
    const int64_t hh = h < n ? h : n;
    const int64_t nv = (n - hh) / 4;
    u4v* v = reinterpret_cast<u4v*>(mask + hh);
    for (int64_t i = tid; i < nv; i += str) __builtin_nontemporal_store(u4v{0u, 0u, 0u, 0u}, v + i);
    if (tid < hh) mask[tid] = 0u;
    for (int64_t i = hh + 4 * nv + tid; i < n; i += str) mask[i] = 0u;
  }
}

template <int P, bool NT>
__device__ __forceinline__ void store_row_fixed(float* dst, const float (*pts)[3]) {
  if constexpr ((P * 3) % 4 == 0) {  // 16-B aligned rows (P = 4, 8): 16-byte stores
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v* d4 = reinterpret_cast<f4v*>(dst);
#pragma unroll
    for (int j = 0; j < P * 3 / 4; ++j) {
      const int i = 4 * j;
      const f4v v = {pts[i / 3][i % 3], pts[(i + 1) / 3][(i + 1) % 3], pts[(i + 2) / 3][(i + 2) % 3],
                     pts[(i + 3) / 3][(i + 3) % 3]};
      if constexpr (NT) __builtin_nontemporal_store(v, d4 + j);
      else d4[j] = v;
    }
  } else {
#pragma unroll
    for (int i = 0; i < P * 3; ++i) {
      if constexpr (NT) __builtin_nontemporal_store(pts[i / 3][i % 3], dst + i);
      else dst[i] = pts[i / 3][i % 3];
    }
  }
}

// environment closest hit: LDS brute force (small meshes) or BVH (large meshes)
template <bool USE_BVH>
__device__ __forceinline__ rt::Hit env_hit_query(const TraceArgs& a, const float4* lds_tab, const rt::Shear& s,
                                                 float3 o, float3 d) {
  if constexpr (USE_BVH) {
    return rt::bvh_query(a.env_bvh, s, o, d);
  } else {
    return query_faces(lds_tab, a.env_nf, s);
  }
}

// ------------------------------------------------------------------ bounce-0 candidate faces
// Every ray of a burst starts at the TX, so the directions that can hit face f at bounce 0 form
// the cone spanned by the TX and the face's corners: d must lie on the inner side of the three
// planes through the TX and each edge -- the signs the watertight test's U, V, W compute, up to
// rounding.  Each block stages, per face, the three unit inner edge normals e_i (from the
// identity-permuted corners) and a margin m; a lane keeps face f as a bounce-0 candidate when
// e_i . d >= -m for all three.  m = 1e-3 rad plus 64 ulp of the scene's coordinate scale over the
// face's nearest corner distance -- far wider than the watertight test's rounding of U, V, W, so
// no face the test could accept is dropped; faces that are degenerate or within 1e-3 * scale of
// the TX get zero normals (always candidates).  The lane then runs the exact test over its
// candidates only, in ascending face order (room.stl: 1.8 candidates per ray, 4.1 per wave, of
// 44 faces), so every output bit is unchanged.
constexpr int kConeMaxFaces = 64;  // candidate set = one 64-bit mask per lane

__device__ __forceinline__ void stage_cones(const TraceArgs& a, float4* cone) {
  for (int f = threadIdx.x; f < a.env_nf; f += blockDim.x) {
    const float4 q0 = a.env_perm[f * 18 + 12], q1 = a.env_perm[f * 18 + 13];  // case 4: kx,ky,kz = x,y,z
    const float c2 = a.env_perm[f * 18 + 14].x;
    const float o[3] = {a.tx[0], a.tx[1], a.tx[2]};
    const float v[3][3] = {{q0.x - o[0], q0.y - o[1], q0.z - o[2]},
                           {q0.w - o[0], q1.x - o[1], q1.y - o[2]},
                           {q1.z - o[0], q1.w - o[1], c2 - o[2]}};
    float scale = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fabsf(o[2]));
    scale = fmaxf(scale, fmaxf(fmaxf(fabsf(q0.x), fabsf(q0.y)), fabsf(q0.z)));
    scale = fmaxf(scale, fmaxf(fmaxf(fabsf(q0.w), fabsf(q1.x)), fabsf(q1.y)));
    scale = fmaxf(scale, fmaxf(fmaxf(fabsf(q1.z), fabsf(q1.w)), fabsf(c2)));
    float len[3], n[3][3];
    for (int i = 0; i < 3; ++i) {
      const float* p = v[i];
      const float* q = v[(i + 1) % 3];
      n[i][0] = p[1] * q[2] - p[2] * q[1];
      n[i][1] = p[2] * q[0] - p[0] * q[2];
      n[i][2] = p[0] * q[1] - p[1] * q[0];
      len[i] = sqrtf(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    }
    const float det = n[0][0] * v[2][0] + n[0][1] * v[2][1] + n[0][2] * v[2][2];
    const float dmin = fminf(fminf(len[0], len[1]), len[2]);
    bool cull = dmin > 1e-3f * scale && det != 0.0f && isfinite(det);
    float4 e[3];
    const float m = 1e-3f + 64.0f * 0x1p-23f * scale / dmin;  // f32 rounding here is ~1e-6 rad
    for (int i = 0; i < 3; ++i) {
      const float nl = sqrtf(n[i][0] * n[i][0] + n[i][1] * n[i][1] + n[i][2] * n[i][2]);
      cull = cull && nl > 0.0f && isfinite(nl);
      const float k = det > 0.0f ? 1.0f / nl : -1.0f / nl;  // inner side: the opposite corner's
      e[i] = make_float4(n[i][0] * k, n[i][1] * k, n[i][2] * k, m);
    }
    for (int i = 0; i < 3; ++i) cone[3 * f + i] = cull ? e[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

// bounce-0 closest hit: this lane's candidate faces only, ascending (LazyHit's order rule)
// The wave's candidates at once (wave_cones: every lane of the wave active, directions within
// rho of lane 0's): lane j tests face j's cone against lane 0's direction with the margin widened by
// the wave's largest |d_l - d_0|.  For a unit edge normal e, e.d_l >= e.d_0 - |d_l - d_0|, so a face
// some lane's own test keeps passes the widened test: the wave's mask holds every lane's
// candidates, and testing a few more faces exactly cannot change a lane's closest hit.  One round
// of ~15 instructions instead of nf rounds per lane; on direction-sorted bursts the widened set is
// about as small as a lane's own.
__device__ __forceinline__ uint64_t wave_cones(const float4* cone, int nf, float3 d, float3 d0, float rho) {
  const int lane = threadIdx.x & 63;
  bool in = false;
  if (lane < nf) {
    const float4 e0 = cone[3 * lane], e1 = cone[3 * lane + 1], e2 = cone[3 * lane + 2];
    const float a0 = fmaf(e0.z, d0.z, fmaf(e0.y, d0.y, e0.x * d0.x));
    const float a1 = fmaf(e1.z, d0.z, fmaf(e1.y, d0.y, e1.x * d0.x));
    const float a2 = fmaf(e2.z, d0.z, fmaf(e2.y, d0.y, e2.x * d0.x));
    in = fminf(fminf(a0, a1), a2) >= -(e0.w + rho);
  }
  (void)d;
  return __ballot(in);
}

// closest hit over the candidate faces `cand` (bit f = face f), ascending (LazyHit's order rule)
__device__ __forceinline__ rt::Hit query_list(const float4* tab, const rt::Shear& s, uint64_t cand) {
  rt::LazyHit h;
  rt::lazy_init(h);
  const int off = s.kcase * 3;
  while (cand) {
    const int f = __builtin_ctzll(cand);
    cand &= cand - 1;
    const float4 q0 = tab[f * 18 + off + 0];
    const float4 q1 = tab[f * 18 + off + 1];
    const float c2 = tab[f * 18 + off + 2].x;
    float T, det;
    if (rt::tri_test(s, q0, q1, c2, T, det)) rt::lazy_consider(h, T, det, f);
  }
  return rt::lazy_finish(h);
}

// ------------------------------------------------------------------ bounce >= 1 candidate faces
// After a reflection the rays of a direction-sorted wave still start close together (on the patch
// their bounce-0 rays hit) and point in similar directions.  wave_boxes bounds the wave's live rays by
// an origin box [ol, oh] and per-axis direction intervals [dl, dh], and lane j tests face j's box
// against that bundle: per axis with dl > 0, every ray of the bundle is inside the face's slab only
// for t in [(fl - oh) / dh, (fh - ol) / dl] (mirrored for dh < 0; no bound when the interval holds
// 0).  A ray's own per-axis intervals lie inside the bundle's, so a face some lane could hit passes;
// the lanes then run the exact test over the wave's candidates only, in ascending face order, and
// every output bit is unchanged.  The face boxes are padded by 1e-5 * (1 + scene scale) and rounded
// outward, the same invariant the BVH's boxes rest on (rt_bvh.h: an accepted hit lies inside its
// face's padded box), and the compare keeps the BVH slab's slack.
// Slot nf holds the receiver ball's box (when nf < 64): its bit tells whether any lane of the wave
// can reach the receiver, so most waves skip rx_maybe.  Groups of 32 or 16 lanes per bundle measured
// slower (113.6 / 116.1 against 110.3 us, r5ai): tighter bundles, but more face rounds.
__device__ __forceinline__ float4 pad_lo(float x, float y, float z, float p) {
  return make_float4(nextafterf(x - p, -INFINITY), nextafterf(y - p, -INFINITY), nextafterf(z - p, -INFINITY), 0.0f);
}
__device__ __forceinline__ float4 pad_hi(float x, float y, float z, float p) {
  return make_float4(nextafterf(x + p, INFINITY), nextafterf(y + p, INFINITY), nextafterf(z + p, INFINITY), 0.0f);
}
__device__ __forceinline__ void stage_boxes(const TraceArgs& a, float4* box) {
  const float p = a.env_pad;
  for (int f = threadIdx.x; f < a.env_nf; f += blockDim.x) {
    const float4 q0 = a.env_perm[f * 18 + 12], q1 = a.env_perm[f * 18 + 13];  // case 4: x, y, z
    const float c2 = a.env_perm[f * 18 + 14].x;
    box[2 * f] = pad_lo(fminf(fminf(q0.x, q0.w), q1.z), fminf(fminf(q0.y, q1.x), q1.w), fminf(fminf(q0.z, q1.y), c2), p);
    box[2 * f + 1] =
        pad_hi(fmaxf(fmaxf(q0.x, q0.w), q1.z), fmaxf(fmaxf(q0.y, q1.x), q1.w), fmaxf(fmaxf(q0.z, q1.y), c2), p);
  }
  if (threadIdx.x == 0 && a.env_nf < 64) {  // the receiver ball (no receiver: an empty box, never reached)
    const float r = a.rx_nf > 0 ? sqrtf(a.rx_r2) : 0.0f;
    box[2 * a.env_nf] = a.rx_nf > 0 ? pad_lo(a.rx_c[0] - r, a.rx_c[1] - r, a.rx_c[2] - r, p)
                                    : make_float4(INFINITY, INFINITY, INFINITY, 0.0f);
    box[2 * a.env_nf + 1] = a.rx_nf > 0 ? pad_hi(a.rx_c[0] + r, a.rx_c[1] + r, a.rx_c[2] + r, p)
                                        : make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
  }
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
// minimum over the 64 lanes (every lane active): DPP within rows of 16, then two lane swaps
__device__ __forceinline__ float wave_min(float x) {
  x = fminf(x, dpp_f<0xB1>(x));   // quad_perm [1,0,3,2]
  x = fminf(x, dpp_f<0x4E>(x));   // quad_perm [2,3,0,1]
  x = fminf(x, dpp_f<0x141>(x));  // row_half_mirror
  x = fminf(x, dpp_f<0x140>(x));  // row_mirror
  x = fminf(x, __shfl_xor(x, 16, 64));
  return fminf(x, __shfl_xor(x, 32, 64));
}

__device__ __forceinline__ void bundle_axis(float fl, float fh, float ol, float oh, float dl, float dh, float& tlo,
                                            float& thi) {
  if (dl > 0.0f) {
    thi = fminf(thi, (fh - ol) / dl);
    const float e = fl - oh;
    if (e > 0.0f) tlo = fmaxf(tlo, e / dh);
  } else if (dh < 0.0f) {
    thi = fminf(thi, (oh - fl) / -dh);
    const float e = ol - fh;
    if (e > 0.0f) tlo = fmaxf(tlo, e / -dl);
  }
}

// every lane of the wave must call it; lanes with alive == false do not constrain the bundle.
// Bit f < nf: face f is a candidate; bit nf (nf < 64): the receiver ball can be reached.
__device__ __forceinline__ uint64_t wave_boxes(const float4* box, int nf, bool alive, float3 o, float3 d) {
  const int lane = threadIdx.x & 63;
  const bool mine = lane <= nf && lane < 64;
  const int f = mine ? lane : 0;
  const float4 bl = box[2 * f], bh = box[2 * f + 1];
  float tlo = 0.0f, thi = INFINITY;
  const float inf = INFINITY;
  // axis by axis, so only one axis' four bounds are live at a time
  bundle_axis(bl.x, bh.x, wave_min(alive ? o.x : inf), -wave_min(alive ? -o.x : inf), wave_min(alive ? d.x : inf),
              -wave_min(alive ? -d.x : inf), tlo, thi);
  bundle_axis(bl.y, bh.y, wave_min(alive ? o.y : inf), -wave_min(alive ? -o.y : inf), wave_min(alive ? d.y : inf),
              -wave_min(alive ? -d.y : inf), tlo, thi);
  bundle_axis(bl.z, bh.z, wave_min(alive ? o.z : inf), -wave_min(alive ? -o.z : inf), wave_min(alive ? d.z : inf),
              -wave_min(alive ? -d.z : inf), tlo, thi);
  return __ballot(mine && tlo <= fmaf(thi, 1.00002f, 1e-6f));
}

__device__ __forceinline__ rt::Hit query_cone(const float4* tab, const float4* cone, int nf, const rt::Shear& s,
                                              float3 d, uint64_t wave_cand = 0, bool use_wave = false) {
  uint64_t cand = 0;
  if (use_wave) {
    cand = wave_cand;
  } else {
#pragma unroll 4
    for (int f = 0; f < nf; ++f) {
      const float4 e0 = cone[3 * f], e1 = cone[3 * f + 1], e2 = cone[3 * f + 2];
      const float d0 = fmaf(e0.z, d.z, fmaf(e0.y, d.y, e0.x * d.x));
      const float d1 = fmaf(e1.z, d.z, fmaf(e1.y, d.y, e1.x * d.x));
      const float d2 = fmaf(e2.z, d.z, fmaf(e2.y, d.y, e2.x * d.x));
      const bool in = fminf(fminf(d0, d1), d2) >= -e0.w;
      cand |= (uint64_t)in << f;
    }
  }
  return query_list(tab, s, cand);
}

template <bool USE_BVH>
__device__ __forceinline__ void stage_env(const TraceArgs& a, float4* lds_tab) {
  if constexpr (!USE_BVH) {  // stage the environment table (coalesced float4 copy)
    const int nvec = a.env_nf * 18;
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) lds_tab[i] = a.env_perm[i];
    __syncthreads();
  }
}

// rt_trace_cir on brute-force meshes (tracer.py:87-117): the trace kernel lists each wave's
// received rows as it goes -- bits of the chunk's 256-bit row mask, the chunk's count and its
// group-of-64-chunks count (lane 0, three atomics, rare).  No block barriers on this path (a
// barrier per chunk held every early wave's registers until its block's slowest wave was done).
// Then ONE small kernel, k_trace_cir_tail, compacts the rows in ray order (chunk order, then bit
// order), computes each path's (bin, amplitude) and accumulates the impulse response in path
// order.  Measured alternatives (tools/k2_fused_variants.py, K2 room, 1M rays):
//   * finishing in the trace kernel's last block (an atomic ticket per block, the last one does
//     the tail) cost the step 11 us in tickets alone -- every block waits on its ticket's round
//     trip before it frees its slot -- plus 12 us of tail; a ticket per wave doubled the step;
//   * the per-path double arithmetic in the trace kernel (by the lane that found the row) runs
//     inside a 72-VGPR budget, spilled, and kept that wave -- often one of the last -- busy for
//     ~10 us after its rays were done.
// One block of 512.  Wave 0 scans the group counts (two levels: only groups with rows are
// expanded into their chunks' counts and row masks), writes the ordered index list, zeroes the
// counts and masks it used and -- while a row of 64 groups (1M rays) holds at most 256 received
// paths -- computes each path's (bin, amplitude) on the lane that found it; the other waves zero
// the impulse response meanwhile.  Denser bursts leave the per-path arithmetic to all 512
// threads after the barrier.  Then wave 0 accumulates in path order.  K2 (one received path per
// burst), rocprofv3: an empty kernel in this place takes 5.1 us, the scan and compaction add 0.2 us,
// the path's double arithmetic 2.8 us, the accumulation (before its shuffle loops were cut to the
// batch's paths) 4.5 us.
__global__ __launch_bounds__(512) void k_trace_cir_tail(rt::TraceCirFused fz, int64_t n, const float* received,
                                                         int P) {
  __shared__ int64_t s_total;
  __shared__ int s_parallel;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave > 0) {
    if (fz.ir)
      for (int64_t b = threadIdx.x - 64; b < fz.k.n_bins; b += blockDim.x - 64) fz.ir[b] = 0.0;
  } else {
    const int64_t nch = (n + 255) / 256;
    const int64_t ngrp = (nch + 63) / 64;
    int64_t base = 0;  // rows before the current row of groups (wave-uniform)
    bool parallel = false;
    for (int64_t g0 = 0; g0 < ngrp; g0 += 64) {
      const int64_t g = g0 + lane;
      const int32_t gc = g < ngrp ? fz.gcounts[g] : 0;
      int64_t gincl = gc;
      for (int o = 1; o < 64; o <<= 1) {
        const int64_t v = __shfl_up(gincl, o, 64);
        if (lane >= o) gincl += v;
      }
      const bool inline_cir = __shfl(gincl, 63, 64) <= 256;
      parallel |= !inline_cir;
      for (uint64_t gm = __ballot(gc > 0); gm; gm &= gm - 1) {  // groups with rows, in order
        const int gl = __builtin_ctzll(gm);
        const int64_t gg = g0 + gl;
        const int64_t gbase = base + __shfl(gincl, gl, 64) - __shfl((int64_t)gc, gl, 64);
        const int64_t c = gg * 64 + lane;
        const int32_t cc = c < nch ? fz.counts[c] : 0;
        int64_t cincl = cc;
        for (int o = 1; o < 64; o <<= 1) {
          const int64_t v = __shfl_up(cincl, o, 64);
          if (lane >= o) cincl += v;
        }
        if (cc > 0) {
          int64_t k = gbase + cincl - cc;
          uint64_t mw[4];
#pragma unroll
          for (int w = 0; w < 4; ++w) mw[w] = fz.masks[c * 4 + w];  // four independent loads
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            for (uint64_t bits = mw[w]; bits; bits &= bits - 1) {
              const int64_t row = c * 256 + w * 64 + __builtin_ctzll(bits);
              fz.index[k] = row;
              if (inline_cir) rt::cir_row(received + row * P * 3, P, fz.k, fz.cbin + k, fz.camp + k);
              ++k;
            }
            if (mw[w]) fz.masks[c * 4 + w] = 0;  // ready for the next call on this workspace
          }
          fz.counts[c] = 0;
        }
        if (lane == 0) fz.gcounts[gg] = 0;
      }
      base += __shfl(gincl, 63, 64);
    }
    if (lane == 0) {
      *fz.count = base;
      s_total = base;
      s_parallel = parallel;
    }
  }
  __syncthreads();
  const int64_t total = s_total;
  if (s_parallel) {  // dense bursts: every path's arithmetic over the whole block (same values)
    for (int64_t k = threadIdx.x; k < total; k += blockDim.x)
      rt::cir_row(received + fz.index[k] * P * 3, P, fz.k, fz.cbin + k, fz.camp + k);
    __syncthreads();
  }
  if (wave == 0 && fz.ir) rt::ir_accumulate_wave(fz.cbin, fz.camp, total, fz.k.n_bins, fz.ir, false);
}

template <int B, bool USE_BVH>
__device__ __forceinline__ void trace_body(const TraceArgs& a) {
  constexpr int P = B + 1;
  // row stores: ordinary (L2 merges a row's pieces; see store_row_fixed) -- the bursts that matter
  // run in direction-sorted order (launch_trace), brute force included
  extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
  float4* cone = lds_tab + (size_t)a.env_nf * 18;  // bounce-0 edge normals after the face table
  const bool use_cone = !USE_BVH && a.env_nf <= kConeMaxFaces;
  float4* box = cone + (size_t)a.env_nf * 3;  // bounce >= 1 face boxes after the cone normals
  const bool use_box = use_cone && a.order && a.box_cull;  // block-uniform
  if (use_cone) stage_cones(a, cone);  // made visible by stage_env's barrier
  if (use_box) stage_boxes(a, box);
  stage_env<USE_BVH>(a, lds_tab);

  const float qnan = __builtin_nanf("");
  // block-uniform loop over 256-row chunks (the same rows per thread as a grid-stride loop), so a
  // wave can list its part of a chunk's received rows for rt_trace_cir
  for (int64_t c0 = blockIdx.x; c0 * 256 < a.n; c0 += gridDim.x) {
    const int64_t chunk = a.sched ? (int64_t)a.sched[c0] : c0;
    const uint64_t t_begin = a.cost ? wall_clock64() : 0;
    const int64_t irow = chunk * 256 + threadIdx.x;
    const bool valid = irow < a.n;
    const int64_t row = valid ? (a.order ? (int64_t)a.order[irow] : irow) : 0;
    const float3 dir0 = rt::ray_dir(a.ray_offset + row);
    // bounce 0 on a direction-sorted burst: the wave's cone candidates at once (wave_cones), when
    // every lane has a ray and the directions lie within 0.05 of lane 0's
    uint64_t wave_cand = 0;
    bool use_wave = false, rx_wave0 = true;
    if (use_cone && a.order) {  // block-uniform
      const float3 d0 = make_float3(__shfl(dir0.x, 0, 64), __shfl(dir0.y, 0, 64), __shfl(dir0.z, 0, 64));
      const float ex = dir0.x - d0.x, ey = dir0.y - d0.y, ez = dir0.z - d0.z;
      float rho = valid ? sqrtf(fmaf(ex, ex, fmaf(ey, ey, ez * ez))) : INFINITY;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) rho = fmaxf(rho, __shfl_xor(rho, o, 64));
      use_wave = rho < a.cone_rho_max;  // wave-uniform (an invalid lane makes it +inf)
      if (use_wave) wave_cand = wave_cones(cone, a.env_nf, dir0, d0, fmaf(rho, 1.001f, 1e-6f));
      // the receiver ball at bounce 0: a lane can reach it only if angle(d, u) <= alpha, and
      // angle(d, d0) <= 2 asin(rho / 2) < beta, so the wave skips rx_maybe when d0 . u < cos(alpha + beta),
      // bounded below by cos(alpha) (1 - beta^2 / 2) - sin(alpha) beta
      if (use_wave && !a.rx_all0) {
        const float beta = fmaf(rho * rho * rho, 1.0f / 12.0f, fmaf(rho, 1.001f, 1e-3f));  // > 2 asin(rho / 2)
        const float thr = fmaf(a.rx_cos, fmaf(-0.5f * beta, beta, 1.0f), -a.rx_sin * beta) - 1e-5f;
        rx_wave0 = !(fmaf(d0.x, a.rx_u[0], fmaf(d0.y, a.rx_u[1], d0.z * a.rx_u[2])) < thr);
      }
    }
    // every lane runs the bounce loop (an invalid lane as a dead ray, storing nothing), so the wave-wide
    // steps (wave_boxes) see the whole wave
    float3 dir = dir0;
    float3 pos = make_float3(a.tx[0], a.tx[1], a.tx[2]);
    float path[P][3];
#pragma unroll
    for (int i = 0; i < P; ++i) path[i][0] = path[i][1] = path[i][2] = qnan;
    path[0][0] = pos.x;
    path[0][1] = pos.y;
    path[0][2] = pos.z;
    int last_rx = -1;
    bool alive = valid;
#pragma unroll
    for (int b = 0; b < B; ++b) {
      int kind = 0, face = -1;
      uint64_t box_cand = 0;
      bool rx_wave = true;  // can any lane of the wave reach the receiver ball (wave-uniform)
      if (use_box && b > 0) {
        box_cand = wave_boxes(box, a.env_nf, alive, pos, dir);
        if (a.env_nf < 64) {
          rx_wave = (box_cand >> a.env_nf) & 1;
          box_cand &= (1ull << a.env_nf) - 1;
        }
      } else if (b == 0) {
        rx_wave = rx_wave0;
      }
      if (alive) {
        const rt::Shear s = rt::make_shear(pos, dir);
        const rt::Hit he = (b == 0 && use_cone) ? query_cone(lds_tab, cone, a.env_nf, s, dir, wave_cand, use_wave)
                           : (use_box && b > 0) ? query_list(lds_tab, s, box_cand)
                                                : env_hit_query<USE_BVH>(a, lds_tab, s, pos, dir);
        const bool env_hit = he.face >= 0;
        rt::Hit hr;
        rt::hit_init(hr);
        if (rx_wave && a.rx_nf > 0 && rx_maybe(a, pos, dir, env_hit ? he.t : RT_MAX_T))
          hr = query_faces(a.rx_perm, a.rx_nf, s);
        const bool rx_hit = hr.face >= 0;
        if (rx_hit && (!env_hit || he.t > hr.t)) {  // kernel.py:85
          pos.x = fmaf(dir.x, hr.t, pos.x);
          pos.y = fmaf(dir.y, hr.t, pos.y);
          pos.z = fmaf(dir.z, hr.t, pos.z);
          path[b + 1][0] = pos.x;
          path[b + 1][1] = pos.y;
          path[b + 1][2] = pos.z;
          last_rx = b + 1;
          kind = 2;
          face = hr.face;
        } else if (env_hit) {  // kernel.py:93-96
          pos.x = fmaf(dir.x, he.t, pos.x);
          pos.y = fmaf(dir.y, he.t, pos.y);
          pos.z = fmaf(dir.z, he.t, pos.z);
          path[b + 1][0] = pos.x;
          path[b + 1][1] = pos.y;
          path[b + 1][2] = pos.z;
          const float4 n4 = a.env_nrm[he.face];
          const float3 n = make_float3(n4.x, n4.y, n4.z);
          const float sc = 2.0f * rt::dot3(dir, n);
          dir.x = fmaf(-sc, n.x, dir.x);
          dir.y = fmaf(-sc, n.y, dir.y);
          dir.z = fmaf(-sc, n.z, dir.z);
          kind = 1;
          face = he.face;
        } else {
          alive = false;  // kernel.py:97-98: every later iteration repeats this miss
        }
      }
      if (valid && a.hit_kind) a.hit_kind[row * B + b] = kind;
#if RT_DIAG_CAND  // diagnostics (tools/k2_cand_stats.py): the wave's candidate count, rx_wave, alive
      if (valid && a.hit_face)
        a.hit_face[row * B + b] = __popcll(b == 0 ? wave_cand : box_cand) | (rx_wave ? 256 : 0) | (alive ? 512 : 0);
#else
      if (valid && a.hit_face) a.hit_face[row * B + b] = face;
#endif
    }
    if (a.cost && (threadIdx.x & 63) == 0) atomicAdd(a.cost + chunk, (uint32_t)(wall_clock64() - t_begin));
    if (!valid) continue;  // block-uniform loop: the last chunk's spare lanes store nothing
    if (a.traced) store_row_fixed<P, false>(a.traced + row * (P * 3), path);
    // Direction-sorted launches: launch_trace fills received (NaN) and row_mask (0) in row order first, as the
    // reference does on the host (tracer.py:67-72), and only received rays store their row and
    // mask word here (kernel.py:89-91): a direction-sorted burst scatters its rows, and writing
    // every ray's NaN row and mask word cost ~0.2 GB of partial-line writes per K4 launch
    if (a.received && (!a.sparse_rx || last_rx >= 0)) {
      float rec[P][3];
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const bool keep = i <= last_rx;
        rec[i][0] = keep ? path[i][0] : qnan;
        rec[i][1] = keep ? path[i][1] : qnan;
        rec[i][2] = keep ? path[i][2] : qnan;
      }
      store_row_fixed<P, false>(a.received + row * (P * 3), rec);
    }
    if (a.mask && (!a.sparse_rx || last_rx >= 0)) a.mask[row] = last_rx >= 0 ? 1u : 0u;
    if (!USE_BVH && a.fused && last_rx >= 0) {  // list the received row under its own chunk (rare)
      const int64_t c = row >> 8;
      atomicAdd(a.fz.counts + c, 1);
      atomicAdd(a.fz.gcounts + (c >> 6), 1);
      atomicOr((unsigned long long*)a.fz.masks + c * 4 + ((row & 255) >> 6), 1ull << (row & 63));
    }
  }
}

// Active-ray compaction, measured and removed (round 5; last in commit 43de9a4):
// queueing each block's live rays in LDS between bounces on the brute force (K2 trace kernel 120.1
// vs 115.4 us: two block barriers per bounce and 25 KB of LDS per block), and a wavefront form of the
// BVH trace with one launch per bounce over the compacted live-ray list (K4 2353 vs 1333 us: the ray
// state's HBM round trips and three launches per bounce).  A direction-sorted wave's rays escape
// together, so whole waves retire early without a queue.

// brute-force kernels up to B = 3 are built for 7 waves per SIMD (72 VGPRs): with the face loop
// unrolled the K2 kernel took 73 VGPRs (6 waves); bounded, 164 vs 170 us per launch,
// bit-identical.  Longer paths keep their registers (their path points would spill).
template <int B, bool USE_BVH>
__global__ __launch_bounds__(256, (B <= 3 ? 7 : 1)) void k_trace_bf(TraceArgs a) {
  trace_body<B, USE_BVH>(a);
}
// BVH meshes: traversal is latency-bound (dependent node fetches), so the kernel is built for
// 4 waves per SIMD (128 VGPRs, no spills beyond the walk stack), which beat 6 (80 VGPRs, the path
// and walk state spilled inside the traversal loop): K4 1416 -> 1077 us per rt_trace with the
// 4-wide walk; 3 (132 VGPRs) measured 1141 us, 5 (96 VGPRs, 385 spilled) no better.
template <int B>
__global__ __launch_bounds__(256, 4) void k_trace_bvh(TraceArgs a) {
  trace_body<B, true>(a);
}

// Generic fallback for B beyond the register-resident instantiations: the path lives in
// the output rows themselves (same semantics, slower).
template <bool USE_BVH>
__global__ __launch_bounds__(256) void k_trace_bf_generic(TraceArgs a, int B) {
  extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
  stage_env<USE_BVH>(a, lds_tab);
  const int P = B + 1;
  const float qnan = __builtin_nanf("");
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t irow = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; irow < a.n; irow += stride) {
    const int64_t row = a.order ? (int64_t)a.order[irow] : irow;
    const int64_t gid = a.ray_offset + row;
    float3 dir = rt::ray_dir(gid);
    float3 pos = make_float3(a.tx[0], a.tx[1], a.tx[2]);
    float* tr = a.traced ? a.traced + row * (int64_t)(P * 3) : nullptr;
    float* rc = a.received ? a.received + row * (int64_t)(P * 3) : nullptr;
    for (int i = 0; i < 3 * P; ++i) {
      if (tr) tr[i] = qnan;
      if (rc) rc[i] = qnan;
    }
    if (tr) { tr[0] = pos.x; tr[1] = pos.y; tr[2] = pos.z; }
    int last_rx = -1;
    bool alive = true;
    for (int b = 0; b < B; ++b) {
      int kind = 0, face = -1;
      if (alive) {
        const rt::Shear s = rt::make_shear(pos, dir);
        const rt::Hit he = env_hit_query<USE_BVH>(a, lds_tab, s, pos, dir);
        const bool env_hit = he.face >= 0;
        rt::Hit hr;
        rt::hit_init(hr);
        if (a.rx_nf > 0 && rx_maybe(a, pos, dir, env_hit ? he.t : RT_MAX_T))
          hr = query_faces(a.rx_perm, a.rx_nf, s);
        const bool rx_hit = hr.face >= 0;
        if (rx_hit && (!env_hit || he.t > hr.t)) {
          pos.x = fmaf(dir.x, hr.t, pos.x);
          pos.y = fmaf(dir.y, hr.t, pos.y);
          pos.z = fmaf(dir.z, hr.t, pos.z);
          if (tr) { tr[3 * (b + 1)] = pos.x; tr[3 * (b + 1) + 1] = pos.y; tr[3 * (b + 1) + 2] = pos.z; }
          last_rx = b + 1;
          kind = 2;
          face = hr.face;
        } else if (env_hit) {
          pos.x = fmaf(dir.x, he.t, pos.x);
          pos.y = fmaf(dir.y, he.t, pos.y);
          pos.z = fmaf(dir.z, he.t, pos.z);
          if (tr) { tr[3 * (b + 1)] = pos.x; tr[3 * (b + 1) + 1] = pos.y; tr[3 * (b + 1) + 2] = pos.z; }
          const float4 n4 = a.env_nrm[he.face];
          const float3 n = make_float3(n4.x, n4.y, n4.z);
          const float sc = 2.0f * rt::dot3(dir, n);
          dir.x = fmaf(-sc, n.x, dir.x);
          dir.y = fmaf(-sc, n.y, dir.y);
          dir.z = fmaf(-sc, n.z, dir.z);
          kind = 1;
          face = he.face;
        } else {
          alive = false;
        }
        if (kind == 2 && rc) {  // kernel.py:89-90: copy the traced prefix
          if (tr) {
            for (int i = 0; i < 3 * (b + 2); ++i) rc[i] = tr[i];
          }
        }
      }
      if (a.hit_kind) a.hit_kind[row * B + b] = kind;
      if (a.hit_face) a.hit_face[row * B + b] = face;
    }
    if (a.mask) a.mask[row] = last_rx >= 0 ? 1u : 0u;
  }
}

// Sort key of a ray: the cell of its initial direction on a 256x256 octahedral map, in Morton
// order, so that rays traced by one wave start in nearly the same direction.  Only the order in
// which rows are processed changes; every row is computed exactly as before.
__device__ __forceinline__ uint16_t dir_cell(int64_t gid) {
  const float3 d = rt::ray_dir(gid);
  const float s = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
  float x = d.x / s, y = d.y / s;
  if (d.z < 0.0f) {
    const float ox = x;
    x = (1.0f - fabsf(y)) * (ox < 0.0f ? -1.0f : 1.0f);
    y = (1.0f - fabsf(ox)) * (y < 0.0f ? -1.0f : 1.0f);
  }
  const uint32_t cx = (uint32_t)fminf(fmaxf((x + 1.0f) * 128.0f, 0.0f), 255.0f);
  const uint32_t cy = (uint32_t)fminf(fmaxf((y + 1.0f) * 128.0f, 0.0f), 255.0f);
  uint32_t k = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b) k |= ((cx >> b) & 1u) << (2 * b) | ((cy >> b) & 1u) << (2 * b + 1);
  return (uint16_t)k;
}
constexpr int kZBandBits = rt::kZBands <= 1 ? 0 : 32 - __builtin_clz((unsigned)(rt::kZBands - 1));
// Coverage plans (dir_order_banded): the direction cell under a band of |d.z| (rt::kZBands bands, the most
// nearly horizontal first).  A terrain's grazing rays walk the longest BVH chains; issued first,
// their waves run beside the short ones instead of after them (a rank's trajectory pass is two
// rounds of the GPU's wave slots).  Only the processing order changes.
__global__ __launch_bounds__(256) void k_dir_keys_banded(int64_t ray_offset, int64_t n, uint32_t* keys, int32_t* rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float3 d = rt::ray_dir(ray_offset + i);
  const uint32_t band = (uint32_t)fminf(fabsf(d.z) * (float)rt::kZBands, (float)(rt::kZBands - 1));
  keys[i] = band << 16 | dir_cell(ray_offset + i);
  rows[i] = (int32_t)i;
}
// Sector shards (rt::sector_ray_ids): the azimuth of a ray's initial direction, 16 bits over
// [-pi, pi), and the banded key of a listed global id.  Only which rank traces a ray and in which
// order depend on them, never a result.
__global__ __launch_bounds__(256) void k_azimuth_keys(int64_t n, uint32_t* keys, int32_t* ids) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float3 d = rt::ray_dir(i);
  const float a = (atan2f(d.y, d.x) + 3.14159265f) * (65536.0f / 6.28318531f);
  keys[i] = (uint32_t)fminf(fmaxf(a, 0.0f), 65535.0f);
  ids[i] = (int32_t)i;
}
__global__ __launch_bounds__(256) void k_ids_keys_banded(const int32_t* ids, int64_t n, uint32_t* keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t gid = ids[i];
  const float3 d = rt::ray_dir(gid);
  const uint32_t band = (uint32_t)fminf(fabsf(d.z) * (float)rt::kZBands, (float)(rt::kZBands - 1));
  keys[i] = band << 16 | dir_cell(gid);
}
}  // namespace

// ------------------------------------------------------------------ launch (C++ side of rt_trace)
namespace rt {

constexpr int64_t kSortMinRays = 1 << 16;

// The stream-ordered workspaces below (hipMallocAsync / hipFreeAsync per launch) come from the
// device's default memory pool, whose release threshold is 0: every synchronize handed the memory
// back and the next launch allocated it afresh (~0.2 ms host gap per coverage rank-pass on the
// terrain, rocprofv3).  Keep freed blocks in the pool instead; once per device.
void keep_pool_memory() {
  static std::once_flag once[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
  std::call_once(once[dev], [dev] {
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
  });
}

// rays [ray_offset, ray_offset + n) by |d.z| band, then direction cell (k_dir_keys_banded); nullptr on failure
const int32_t* dir_order_banded(int64_t ray_offset, int64_t n, hipStream_t stream, void** ws) {
  size_t cub_bytes = 0;
  *ws = nullptr;
  keep_pool_memory();
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 16 + kZBandBits, stream) != hipSuccess) {
    set_error("dir_order_banded: hipcub sizing failed");
    return nullptr;
  }
  const size_t kb = ((size_t)n * 4 + 255) / 256 * 256;
  hipError_t e = hipMallocAsync(ws, 4 * kb + cub_bytes, stream);
  if (e != hipSuccess) {
    hip_fail(e, "dir_order_banded workspace");
    *ws = nullptr;
    return nullptr;
  }
  uint32_t* k_in = (uint32_t*)*ws;
  uint32_t* k_out = (uint32_t*)((char*)*ws + kb);
  int32_t* r_in = (int32_t*)((char*)*ws + 2 * kb);
  int32_t* r_out = (int32_t*)((char*)*ws + 3 * kb);
  void* tmp = (char*)*ws + 4 * kb;
  hipLaunchKernelGGL(k_dir_keys_banded, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, ray_offset, n, k_in,
                     r_in);
  e = hipcub::DeviceRadixSort::SortPairs(tmp, cub_bytes, k_in, k_out, r_in, r_out, (int)n, 0, 16 + kZBandBits, stream);
  if (e != hipSuccess) {
    hip_fail(e, "dir_order_banded sort");
    return nullptr;
  }
  return r_out;
}

// The rays of a sector shard of a burst of n_total rays (global ids 0..n_total-1): the burst sorted
// by the azimuth of the initial direction (stable, so equal keys stay in id order) and cut into
// world * slices equal pieces; rank takes pieces rank, rank + world, rank + 2 world, ... (slices = 1:
// one wedge of directions), then those ids in the banded order the trajectory kernels want.
// Written to out[sector_ray_count(...)]; synchronises `stream` (once per plan).
int64_t sector_ray_count(int64_t n_total, int rank, int world, int slices) {
  const int64_t P = (int64_t)world * slices;
  int64_t m = 0;
  for (int k = 0; k < slices; ++k) {
    const int64_t p = (int64_t)k * world + rank;
    m += (p + 1) * n_total / P - p * n_total / P;
  }
  return m;
}
int sector_ray_ids(int64_t n_total, int rank, int world, int slices, int32_t* out, hipStream_t stream) {
  if (n_total <= 0 || world < 1 || rank < 0 || rank >= world || slices < 1 || n_total > INT32_MAX ||
      (int64_t)world * slices > n_total) {
    set_error("sector_ray_ids: invalid arguments");
    return RT_EINVAL;
  }
  const int64_t m = sector_ray_count(n_total, rank, world, slices), P = (int64_t)world * slices;
  size_t b1 = 0, b2 = 0;
  RT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                            (int32_t*)nullptr, (int)n_total, 0, 16, stream));
  RT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                            (int32_t*)nullptr, (int)m, 0, 16 + kZBandBits, stream));
  const size_t kb = ((size_t)n_total * 4 + 255) / 256 * 256;
  char* ws = nullptr;
  RT_HIP(hipMalloc(&ws, 5 * kb + std::max(b1, b2)));
  uint32_t* k_in = (uint32_t*)ws;
  uint32_t* k_out = (uint32_t*)(ws + kb);
  int32_t* i_in = (int32_t*)(ws + 2 * kb);
  int32_t* i_out = (int32_t*)(ws + 3 * kb);
  int32_t* mine = (int32_t*)(ws + 4 * kb);
  void* tmp = ws + 5 * kb;
  hipError_t e = hipSuccess;
  hipLaunchKernelGGL(k_azimuth_keys, dim3((unsigned)((n_total + 255) / 256)), dim3(256), 0, stream, n_total, k_in, i_in);
  e = hipcub::DeviceRadixSort::SortPairs(tmp, b1, k_in, k_out, i_in, i_out, (int)n_total, 0, 16, stream);
  int64_t at = 0;
  for (int k = 0; k < slices && e == hipSuccess; ++k) {
    const int64_t p = (int64_t)k * world + rank, lo = p * n_total / P, hi = (p + 1) * n_total / P;
    e = hipMemcpyAsync(mine + at, i_out + lo, sizeof(int32_t) * (size_t)(hi - lo), hipMemcpyDeviceToDevice, stream);
    at += hi - lo;
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_ids_keys_banded, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, mine, m, k_in);
    e = hipcub::DeviceRadixSort::SortPairs(tmp, b2, k_in, k_out, mine, out, (int)m, 0, 16 + kZBandBits, stream);
  }
  if (e == hipSuccess) e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  (void)hipFree(ws);
  return e == hipSuccess ? RT_OK : hip_fail(e, "sector_ray_ids");
}

// The banded order of a burst depends only on (ray_offset, n): every call traces the same rays
// (kernel.py:51 seeds each ray with its id alone), so the order is computed once per device and
// (ray_offset, n) and kept.  rt_trace re-sorted the burst on every call before round 5 (K4: 0.14 ms
// of a 0.91 ms step).  A few entries per process, least recently used evicted; the first user's
// stream records an event that later users on other streams wait on.
namespace {
struct OrderEntry {
  int device = -1;
  int64_t ray_offset = 0, n = 0;
  int32_t* order = nullptr;
  hipEvent_t ready = nullptr;
  hipStream_t made_on = nullptr;
  uint64_t used = 0;
};
constexpr int kOrderCache = 8;
OrderEntry g_orders[kOrderCache];
uint64_t g_order_clock = 0;
std::mutex g_order_mu;
}  // namespace

const int32_t* dir_order_cached(int64_t ray_offset, int64_t n, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("dir_order_cached: hipGetDevice failed");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_order_mu);
  for (OrderEntry& e : g_orders)
    if (e.order && e.device == dev && e.ray_offset == ray_offset && e.n == n) {
      e.used = ++g_order_clock;
      if (e.made_on != stream && hipStreamWaitEvent(stream, e.ready, 0) != hipSuccess) {
        set_error("dir_order_cached: hipStreamWaitEvent failed");
        return nullptr;
      }
      return e.order;
    }
  OrderEntry* slot = &g_orders[0];
  for (OrderEntry& e : g_orders)
    if (!e.order) {
      slot = &e;
      break;
    } else if (e.used < slot->used) {
      slot = &e;
    }
  if (slot->order) {  // evict (hipFree waits for the device: nothing in flight still reads it)
    int cur = dev;
    if (slot->device != dev) (void)hipSetDevice(slot->device);
    (void)hipFree(slot->order);
    if (slot->ready) (void)hipEventDestroy(slot->ready);
    if (slot->device != cur) (void)hipSetDevice(cur);
    *slot = OrderEntry{};
  }
  void* ws = nullptr;
  const int32_t* o = dir_order_banded(ray_offset, n, stream, &ws);
  if (!o) return nullptr;
  int32_t* keep = nullptr;
  hipError_t e = hipMalloc(&keep, sizeof(int32_t) * (size_t)n);
  if (e == hipSuccess) e = hipMemcpyAsync(keep, o, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToDevice, stream);
  if (e == hipSuccess) e = hipFreeAsync(ws, stream);
  hipEvent_t ev = nullptr;
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(ev, stream);
  if (e != hipSuccess) {
    if (keep) (void)hipFree(keep);
    if (ev) (void)hipEventDestroy(ev);
    hip_fail(e, "dir_order_cached");
    return nullptr;
  }
  *slot = OrderEntry{dev, ray_offset, n, keep, ev, stream, ++g_order_clock};
  return keep;
}

void trace_mark(int i, hipStream_t s);
void trace_events(hipEvent_t* e0, hipEvent_t* e1);

// fused (optional, rt_trace_cir): the brute-force kernels list each chunk's received rows as they go
// and their last block finishes the CIR step; *fused_done tells whether they did (BVH and generic
// kernels: no, rt_trace_cir then launches k_chunk_counts + k_compact_cir)
// ------------------------------------------------------------------ chunk schedule (longest first)
// The chunks of a direction-sorted burst differ several-fold in cost (coherent strips against waves
// that straddle walls and corners), and the dispatcher starts blocks in chunk order: costly chunks
// at the end of the order leave the GPU draining a few slow blocks (K2: 132 us with the chunk order
// reversed against 104 forward, r5aw).  The first launch of a (device, rays, bounces, scene, TX)
// records each chunk's summed wave time (wall_clock64, one atomic per wave); k_chunk_schedule then
// orders the chunks by cost, longest first (LPT: 256 linear buckets of the largest cost, a counting
// sort in one block), and later launches run them in that order.  Any permutation traces the same
// rows with the same results; the schedule only moves the slow blocks to the front.
constexpr int kSchedBuckets = 256;
constexpr int64_t kSchedMaxChunks = 1 << 20;
__global__ __launch_bounds__(1024) void k_chunk_schedule(const uint32_t* cost, int64_t nch, int32_t* sched) {
  __shared__ uint32_t s_max;
  __shared__ int s_off[kSchedBuckets];
  if (threadIdx.x == 0) s_max = 0;
  for (int i = threadIdx.x; i < kSchedBuckets; i += blockDim.x) s_off[i] = 0;
  __syncthreads();
  uint32_t m = 0;
  for (int64_t c = threadIdx.x; c < nch; c += blockDim.x) m = max(m, cost[c]);
  atomicMax(&s_max, m);
  __syncthreads();
  const uint64_t top = (uint64_t)s_max + 1;
  auto bucket = [&](int64_t c) {  // costliest first
    return kSchedBuckets - 1 - (int)((uint64_t)cost[c] * kSchedBuckets / top);
  };
  for (int64_t c = threadIdx.x; c < nch; c += blockDim.x) atomicAdd(&s_off[bucket(c)], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int i = 0; i < kSchedBuckets; ++i) {
      const int k = s_off[i];
      s_off[i] = run;
      run += k;
    }
  }
  __syncthreads();
  for (int64_t c = threadIdx.x; c < nch; c += blockDim.x) sched[atomicAdd(&s_off[bucket(c)], 1)] = (int32_t)c;
}

namespace {
// One cached schedule.  An entry is published (added to the table) when its cost-recording launch
// is set up, but its `sched` buffer is only meaningful once k_chunk_schedule has run and `ready`
// has been recorded after it: `valid` says so, and is set under the mutex by finish_chunk_schedule.
// Lookups that find an entry that is not valid yet (another thread's launch in flight) trace in
// chunk order; a launch that fails between the two steps drops its entry (SchedClaim).
// Keys: the meshes' process-unique ids (rt_mesh::gen; a destroyed mesh's entries are evicted by
// rt_mesh_destroy), never their addresses, which a later mesh may reuse.
struct SchedEntry {
  int device = -1, B = 0;
  int64_t ray_offset = 0, n = 0;
  uint64_t env_gen = 0, rx_gen = 0;
  float tx[3] = {0, 0, 0};
  int32_t* sched = nullptr;
  uint32_t* cost = nullptr;
  hipEvent_t ready = nullptr;  // recorded after k_chunk_schedule
  hipStream_t made_on = nullptr;
  uint64_t used = 0;
  bool valid = false;
};
constexpr int kSchedCache = 8;
SchedEntry g_sched[kSchedCache];
uint64_t g_sched_clock = 0;
std::mutex g_sched_mu;

bool chunk_schedule_on() {  // RFRT_K2_LPT=0: chunks in order (A/B checks)
  static const bool v = [] {
    const char* e = getenv("RFRT_K2_LPT");
    return !(e && e[0] == '0');
  }();
  return v;
}

// caller holds g_sched_mu; hipFree waits for the device, so no launch still reads the buffers
void drop_entry(SchedEntry& e) {
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (e.device >= 0 && e.device != cur) (void)hipSetDevice(e.device);
  if (e.sched) (void)hipFree(e.sched);
  if (e.cost) (void)hipFree(e.cost);
  if (e.ready) (void)hipEventDestroy(e.ready);
  if (cur >= 0 && e.device != cur) (void)hipSetDevice(cur);
  e = SchedEntry{};
}

// Sets a.sched (schedule ready) or a.cost (this launch records the costs; *profile then names the
// entry whose schedule finish_chunk_schedule computes after the launch).  Errors leave both null.
void chunk_schedule(TraceArgs& a, int dev, const rt_mesh* env, const rt_mesh* rx, const float tx[3], int B,
                    int64_t ray_offset, int64_t n, hipStream_t stream, SchedEntry** profile) {
  *profile = nullptr;
  const int64_t nch = (n + 255) / 256;
  if (!chunk_schedule_on() || nch > kSchedMaxChunks) return;
  const uint64_t env_gen = env->gen, rx_gen = rx ? rx->gen : 0;
  std::lock_guard<std::mutex> lock(g_sched_mu);
  for (SchedEntry& e : g_sched)
    if (e.sched && e.device == dev && e.B == B && e.ray_offset == ray_offset && e.n == n && e.env_gen == env_gen &&
        e.rx_gen == rx_gen && e.tx[0] == tx[0] && e.tx[1] == tx[1] && e.tx[2] == tx[2]) {
      if (!e.valid) return;  // being computed by another launch: this one runs in chunk order
      e.used = ++g_sched_clock;
      if (e.made_on != stream && hipStreamWaitEvent(stream, e.ready, 0) != hipSuccess) return;
      a.sched = e.sched;
      return;
    }
  SchedEntry* slot = &g_sched[0];
  for (SchedEntry& e : g_sched)
    if (!e.sched) {
      slot = &e;
      break;
    } else if (e.used < slot->used) {
      slot = &e;
    }
  if (slot->sched) {
    if (!slot->valid) return;  // every entry in flight (8 threads at once): no schedule this time
    drop_entry(*slot);
  }
  SchedEntry e;
  e.device = dev;
  e.B = B;
  e.ray_offset = ray_offset;
  e.n = n;
  e.env_gen = env_gen;
  e.rx_gen = rx_gen;
  for (int k = 0; k < 3; ++k) e.tx[k] = tx[k];
  hipError_t err = hipMalloc(&e.sched, sizeof(int32_t) * (size_t)nch);
  if (err == hipSuccess) err = hipMalloc(&e.cost, sizeof(uint32_t) * (size_t)nch);
  if (err == hipSuccess) err = hipEventCreateWithFlags(&e.ready, hipEventDisableTiming);
  if (err == hipSuccess) err = hipMemsetAsync(e.cost, 0, sizeof(uint32_t) * (size_t)nch, stream);
  if (err != hipSuccess) {  // no schedule: chunks in order
    drop_entry(e);
    return;
  }
  e.made_on = stream;
  e.used = ++g_sched_clock;
  *slot = e;
  a.cost = slot->cost;
  *profile = slot;
}

// The entry a cost-recording launch claimed: finish() computes its schedule and publishes it as
// valid; any other way out of launch_trace (an error return between the two) drops it.
struct SchedClaim {
  SchedEntry* e = nullptr;
  int finish(int64_t n, hipStream_t stream) {
    if (!e) return 0;
    hipLaunchKernelGGL(k_chunk_schedule, dim3(1), dim3(1024), 0, stream, e->cost, (n + 255) / 256, e->sched);
    hipError_t err = hipGetLastError();
    if (err == hipSuccess) err = hipEventRecord(e->ready, stream);
    std::lock_guard<std::mutex> lock(g_sched_mu);
    if (err == hipSuccess) e->valid = true;
    else drop_entry(*e);
    e = nullptr;
    return err == hipSuccess ? 0 : hip_fail(err, "chunk schedule");
  }
  ~SchedClaim() {
    if (!e) return;
    std::lock_guard<std::mutex> lock(g_sched_mu);
    drop_entry(*e);
  }
};
}  // namespace

uint64_t next_mesh_gen() {
  static std::atomic<uint64_t> g{0};
  return ++g;
}

// rt_release_caches: every cached ray order and chunk schedule of every device (entries still in
// flight on another thread are left to finish).  hipFree waits for the device.
void release_trace_caches() {
  {
    std::lock_guard<std::mutex> lock(g_sched_mu);
    for (SchedEntry& e : g_sched)
      if (e.sched && e.valid) drop_entry(e);
  }
  std::lock_guard<std::mutex> lock(g_order_mu);
  int cur = -1;
  (void)hipGetDevice(&cur);
  for (OrderEntry& e : g_orders)
    if (e.order) {
      if (e.device != cur) (void)hipSetDevice(e.device);
      (void)hipFree(e.order);
      if (e.ready) (void)hipEventDestroy(e.ready);
      e = OrderEntry{};
    }
  if (cur >= 0) (void)hipSetDevice(cur);
}

void forget_mesh_schedules(uint64_t gen) {
  std::lock_guard<std::mutex> lock(g_sched_mu);
  for (SchedEntry& e : g_sched)
    // entries still in flight are left to finish: their ids never match again, LRU evicts them
    if (e.sched && e.valid && (e.env_gen == gen || e.rx_gen == gen)) drop_entry(e);
}

int launch_trace(const rt_mesh* env, const float tx[3], const rt_mesh* rx, int B, int64_t ray_offset, int64_t n,
                 float* traced, float* received, uint32_t* mask, int32_t* hit_kind, int32_t* hit_face,
                 hipStream_t stream, const TraceCirFused* fused, bool* fused_done) {
  if (fused_done) *fused_done = false;
  if (n == 0) return 0;
  TraceArgs a{};
  a.env_perm = env->perm;
  a.env_nrm = env->nrm;
  a.env_nf = (int)env->nf;
  a.env_bvh = rt::bvh_view(env);
  const bool bvh = env->nodes != nullptr;
  a.rx_perm = rx ? rx->perm : nullptr;
  a.rx_nf = rx ? (int)rx->nf : 0;
  for (int k = 0; k < 3; ++k) {
    a.rx_c[k] = rx ? rx->center[k] : 0.0f;
    a.tx[k] = tx[k];
  }
  a.rx_r2 = rx ? rx->radius * rx->radius : 0.0f;
  a.ray_offset = ray_offset;
  a.n = n;
  a.traced = traced;
  a.received = received;
  a.mask = mask;
  a.hit_kind = hit_kind;
  a.hit_face = hit_face;
  a.order = nullptr;
  a.fused = fused && !bvh && B <= 8;  // the register-resident brute-force kernels
  if (a.fused) a.fz = *fused;
  if (fused_done) *fused_done = a.fused;
  // brute force: the face table, then the bounce-0 cone normals (3 float4 per face, <= 64 faces)
  // then the bounce >= 1 face boxes (2 float4 per face, same meshes) and the receiver ball's box
  const size_t lds = bvh ? 0 : (size_t)(env->nf <= kConeMaxFaces ? env->nf * 23 + 2 : env->nf * 18) * sizeof(float4);
  {
    float amax = 0.0f;  // the environment's and the receiver's coordinates
    for (int k = 0; k < 3; ++k) amax = std::max(amax, std::max(std::fabs(env->lo[k]), std::fabs(env->hi[k])));
    for (int k = 0; rx && k < 3; ++k) amax = std::max(amax, std::max(std::fabs(rx->lo[k]), std::fabs(rx->hi[k])));
    a.env_pad = 1e-5f * (1.0f + amax);
  }
  static const bool box_cull = [] {  // RFRT_K2_BOX=0: every face at bounces >= 1 (A/B checks)
    const char* e = getenv("RFRT_K2_BOX");
    return !(e && e[0] == '0');
  }();
  a.box_cull = box_cull;
  // bounce-0 wave cones up to a spread of 0.3: 0.05 left half of K2's waves (banded order: a wave spans
  // a long strip of directions) on the per-lane cone loop; 0.3 takes nearly all, K2 rt_trace -7 us (r5aq)
  a.cone_rho_max = 0.3f;

  a.rx_all0 = true;
  if (rx) {  // the receiver ball seen from the TX (bounce 0 of the sorted brute-force kernels)
    const double dx = (double)rx->center[0] - tx[0], dy = (double)rx->center[1] - tx[1],
                 dz = (double)rx->center[2] - tx[2];
    const double dist = std::sqrt(dx * dx + dy * dy + dz * dz), r = (double)rx->radius * 1.001 + 1e-4;
    if (dist > 2.0 * r) {
      a.rx_all0 = false;
      a.rx_u[0] = (float)(dx / dist);
      a.rx_u[1] = (float)(dy / dist);
      a.rx_u[2] = (float)(dz / dist);
      const double sa = r / dist;
      a.rx_sin = (float)(sa * 1.001);
      a.rx_cos = (float)(std::sqrt(1.0 - sa * sa) * (1.0 - 1e-6));
    }
  }
  int dev_cu = 256;
  const int64_t want = (n + 255) / 256;
  const int64_t cap = (int64_t)dev_cu * 16;
  const int grid0 = (int)(want < cap ? want : cap);
  const dim3 blk(256);
  // a generic (non-generic-Warp) B>8 falls back to the row-resident kernel
  if (traced == nullptr && B > 8) {
    set_error("rt_trace: max_bounces > 8 requires the traced buffer (scratch rows)");
    return -1;
  }
  // Rows in direction-sorted order (the banded order, cached per (device, ray_offset, n)).  BVH
  // meshes: coherent traversal (K4: 2.98 -> 2.06 ms).  Brute force (register-resident
  // kernels): the lanes of a wave share their bounce-0 cone candidates and their branches, K2
  // rt_trace 143 -> 136 us (r5l); the rows are then stored like the BVH kernels' (no streaming
  // stores) and the fused CIR lists each received row under its own chunk.  (A cull of faces whose
  // corners all lie beyond the best t so far -- T / det is a convex combination of the corners'
  // sheared z -- was bit-identical and slower even on sorted rows, 138 us: in ascending face order a
  // wave reaches its last lane's hit face before it can skip anything.)
  if (g_poison >= 0) {
    const int rc = poison_pool((size_t)256 << 20, stream);
    if (rc) return rc;
  }
  const bool sort = (bvh || B <= 8) && n >= kSortMinRays && n <= INT32_MAX;
  SchedClaim sched_claim;
  if (sort) {
    trace_mark(0, stream);
    a.order = dir_order_cached(ray_offset, n, stream);
    if (!a.order) return -1;
    if (B <= 8) {
      int dev = 0;
      if (hipGetDevice(&dev) == hipSuccess) chunk_schedule(a, dev, env, rx, tx, B, ray_offset, n, stream, &sched_claim.e);
    }
    trace_mark(1, stream);
  }
  const int grid = grid0;
  // profiling: the kernel's own dispatch packet carries the start/stop timestamps
  // (hipExtLaunchKernelGGL), so timing adds no marker packets -- and no gaps -- to the stream
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  trace_events(&ev0, &ev1);
  // BVH kernels store only the received rows (trace_body): the fill comes first, inside the
  // profiled span (its start event, the trace kernel's stop event)
  // direction-sorted launches (BVH, and brute force since round 5: K2 rt_trace 130.7 -> 127.8 us,
  // r5aa) fill received / row_mask in row order first and store only the received rays' rows
  const bool fill = (bvh || a.order) && B <= 8 && (received || mask);
  a.sparse_rx = fill;
  if (fill) {
    const unsigned gf = (unsigned)std::min<int64_t>((n * (B + 1) * 3 / 4 + 255) / 256, 4096);
    if (ev0) hipExtLaunchKernelGGL(k_fill_received, dim3(gf), dim3(256), 0, stream, ev0, nullptr, 0, received,
                                   (int64_t)n * (B + 1) * 3, mask, n);
    else hipLaunchKernelGGL(k_fill_received, dim3(gf), dim3(256), 0, stream, received, (int64_t)n * (B + 1) * 3,
                            mask, n);
  }
  hipEvent_t ev_start = fill ? nullptr : ev0;
#define RT_LAUNCH(K, ...)                                                                                \
  do {                                                                                                   \
    if (ev0) hipExtLaunchKernelGGL(K, dim3(grid), blk, lds, stream, ev_start, ev1, 0, __VA_ARGS__);      \
    else hipLaunchKernelGGL(K, dim3(grid), blk, lds, stream, __VA_ARGS__);                              \
  } while (0)
  switch (B) {
#define RT_CASE(BB)                                                                                  \
  case BB:                                                                                           \
    if (bvh) {                                                                                       \
      RT_LAUNCH((k_trace_bvh<BB>), a);                                                               \
    } else {                                                                                         \
      if (lds > 48 * 1024) /* up to 192 faces: above the 48 KB default */                                       \
        RT_HIP(hipFuncSetAttribute((const void*)k_trace_bf<BB, false>,                              \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));           \
      RT_LAUNCH((k_trace_bf<BB, false>), a);                                                         \
    }                                                                                                \
    break;
    RT_CASE(1) RT_CASE(2) RT_CASE(3) RT_CASE(4) RT_CASE(5) RT_CASE(6) RT_CASE(7) RT_CASE(8)
#undef RT_CASE
    default:
      if (bvh) RT_LAUNCH(k_trace_bf_generic<true>, a, B);
      else RT_LAUNCH(k_trace_bf_generic<false>, a, B);
      break;
  }
#undef RT_LAUNCH
  {
    const int rc = sched_claim.finish(n, stream);
    if (rc) return rc;
  }
  if (a.fused) hipLaunchKernelGGL(k_trace_cir_tail, dim3(1), dim3(512), 0, stream, a.fz, n, received, B + 1);
  RT_HIP(hipGetLastError());
  return 0;
}

// rt_profile / rt_trace_last_profile / rt_trace_profile_stats: while profiling is on, every trace
// kernel launch (or every g_profile_every-th, rt_profile(k > 1)) records its start/stop in a ring of
// event pairs (through its dispatch packet), and BVH launches bracket their ray-order sort with
// markers.  Process-wide, for measurement; not thread-safe.
bool g_profile = false;
int g_profile_every = 1;
static int64_t g_launches = 0;
constexpr int kRing = 512;
static hipEvent_t g_ring[kRing][2] = {};
static int64_t g_ring_n = 0;
static hipEvent_t g_tev[2] = {};
static bool g_trec[2] = {};
void profile_reset() {
  g_ring_n = 0;
  g_launches = 0;
  g_trec[0] = g_trec[1] = false;
}
void trace_events(hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  if (!g_profile || g_launches++ % g_profile_every != 0) return;
  hipEvent_t* p = g_ring[g_ring_n % kRing];
  for (int i = 0; i < 2; ++i)
    if (!p[i] && hipEventCreate(&p[i]) != hipSuccess) return;
  *e0 = p[0];
  *e1 = p[1];
  ++g_ring_n;
}
void trace_mark(int i, hipStream_t s) {
  if (!g_profile) return;
  if (!g_tev[i] && hipEventCreate(&g_tev[i]) != hipSuccess) return;
  g_trec[i] = hipEventRecord(g_tev[i], s) == hipSuccess;
}
static double ring_ms(int64_t j) {
  float ms = 0.0f;
  hipEvent_t* p = g_ring[j % kRing];
  if (hipEventSynchronize(p[1]) != hipSuccess || hipEventElapsedTime(&ms, p[0], p[1]) != hipSuccess) return NAN;
  return (double)ms;
}
// out[0]: the last trace kernel (ms), out[1]: its ray-order sort (ms, BVH meshes; NaN otherwise)
int trace_last_profile(double* out, int n) {
  for (int i = 0; i < n; ++i) out[i] = NAN;
  if (n > 0 && g_ring_n > 0) out[0] = ring_ms(g_ring_n - 1);
  if (n > 1 && g_trec[0] && g_trec[1]) {
    float ms = 0.0f;
    if (hipEventSynchronize(g_tev[1]) == hipSuccess && hipEventElapsedTime(&ms, g_tev[0], g_tev[1]) == hipSuccess)
      out[1] = (double)ms;
  }
  return 0;
}
// over the trace kernels profiled since profiling was (re)enabled, at most the last 512:
// out = [launches, mean ms, min ms, max ms]
int trace_profile_stats(double* out, int n) {
  for (int i = 0; i < n; ++i) out[i] = NAN;
  const int64_t m = g_ring_n < kRing ? g_ring_n : kRing;
  if (n > 0) out[0] = (double)m;
  if (m == 0) return 0;
  double sum = 0.0, lo = INFINITY, hi = 0.0;
  for (int64_t j = g_ring_n - m; j < g_ring_n; ++j) {
    const double v = ring_ms(j);
    sum += v;
    lo = fmin(lo, v);
    hi = fmax(hi, v);
  }
  if (n > 1) out[1] = sum / (double)m;
  if (n > 2) out[2] = lo;
  if (n > 3) out[3] = hi;
  return 0;
}

}  // namespace rt

#if RT_COUNT_STEPS
// diagnostic builds only (RT_COUNT_STEPS=1, tools/walk_stats.py): the walk statistics of this file's
// kernels since the last reset -- out[0..3] = lane steps, wave iterations, queries, max steps
extern "C" int rt_debug_walk_stats(double* out, int reset) {
  unsigned long long h[16 * 4];
  if (hipDeviceSynchronize() != hipSuccess) return RT_EHIP;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(rt::g_walk_stats), sizeof h) != hipSuccess) return RT_EHIP;
  double a[4] = {0, 0, 0, 0};
  for (int i = 0; i < 16; ++i) {
    a[0] += (double)h[4 * i];
    a[1] += (double)h[4 * i + 1] / 65536.0;
    a[2] += (double)h[4 * i + 2];
    a[3] = std::max(a[3], (double)h[4 * i + 3]);
  }
  for (int k = 0; k < 4; ++k) out[k] = a[k];
  if (reset) {
    std::memset(h, 0, sizeof h);
    if (hipMemcpyToSymbol(HIP_SYMBOL(rt::g_walk_stats), h, sizeof h) != hipSuccess) return RT_EHIP;
  }
  return RT_OK;
}
#endif
