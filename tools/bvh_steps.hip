// bvh_steps.hip -- diagnostic (not shipped): per-ray BVH traversal step counts of the coverage
// trajectory pass (k_traj: B env-only bounces) on a librfrt mesh, for the sequential per-lane
// traversal of rt_bvh.h and for a simulated G-wide group traversal (G stack entries expanded per
// iteration).  Built by tools/bvh_steps.py against librfrt's internal mesh layout.
#include <hip/hip_runtime.h>

#include "../rf_ray_tracing_warp_amd/csrc/rt_bvh.h"
#include "../rf_ray_tracing_warp_amd/csrc/rt_internal.h"

namespace {
using namespace rt;

__device__ Hit query_seq(const BvhView& b, const Shear& s, float3 o, float3 d, int& iters, int& leaves) {
  Hit h;
  hit_init(h);
  const RayBox r = make_raybox(o, d);
  int stack[RT_BVH_STACK];
  float stackt[RT_BVH_STACK];
  int sp = 0, cur = 0;
  while (true) {
    ++iters;
    const float4 q0 = b.nodes[4 * cur + 0], q1 = b.nodes[4 * cur + 1];
    const float4 q2 = b.nodes[4 * cur + 2], q3 = b.nodes[4 * cur + 3];
    const int c0 = __float_as_int(q3.x), c1 = __float_as_int(q3.y);
    float t0 = slab(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
    float t1 = slab(r, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w);
    for (int side = 0; side < 2; ++side) {
      const int c = side ? c1 : c0;
      float& tt = side ? t1 : t0;
      if (c < 0 && tt <= h.t * 1.00001f + 1e-6f) {
        ++leaves;
        { const int2 lf = b.leaves[-1 - c]; leaf4(b, s, lf.x, lf.y, h); }
      }
      if (c < 0) tt = INFINITY;
    }
    const float lim = h.t * 1.00001f + 1e-6f;
    const bool h0 = t0 <= lim, h1 = t1 <= lim;
    if (h0 && h1) {
      const bool first0 = t0 <= t1;
      stack[sp] = first0 ? c1 : c0;
      stackt[sp] = first0 ? t1 : t0;
      ++sp;
      cur = first0 ? c0 : c1;
      continue;
    }
    if (h0) { cur = c0; continue; }
    if (h1) { cur = c1; continue; }
    bool found = false;
    while (sp > 0) {
      --sp;
      if (stackt[sp] <= h.t * 1.00001f + 1e-6f) { cur = stack[sp]; found = true; break; }
    }
    if (!found) break;
  }
  return h;
}

// G entries popped per iteration; their children pushed far-first; best shared after the iteration
__device__ int query_group_iters(const BvhView& b, const Shear& s, float3 o, float3 d, int G, Hit& out) {
  Hit h;
  hit_init(h);
  const RayBox r = make_raybox(o, d);
  int stack[256];
  float stackt[256];
  int sp = 1, iters = 0;
  stack[0] = 0;
  stackt[0] = 0.0f;
  while (sp > 0) {
    ++iters;
    const int m = sp < G ? sp : G;
    int pn[32];
    float pt[32];
    int np = 0;
    Hit hn = h;
    const float lim0 = h.t * 1.00001f + 1e-6f;
    for (int i = 0; i < m; ++i) {
      const int e = sp - 1 - i;
      if (stackt[e] > lim0) continue;
      const int cur = stack[e];
      const float4 q0 = b.nodes[4 * cur + 0], q1 = b.nodes[4 * cur + 1];
      const float4 q2 = b.nodes[4 * cur + 2], q3 = b.nodes[4 * cur + 3];
      const int c[2] = {__float_as_int(q3.x), __float_as_int(q3.y)};
      const float t[2] = {slab(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y), slab(r, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w)};
      for (int side = 0; side < 2; ++side) {
        if (!(t[side] <= lim0)) continue;
        if (c[side] < 0) {
          { const int2 lf = b.leaves[-1 - c[side]]; leaf4(b, s, lf.x, lf.y, hn); }
        } else if (np < 32) {
          pn[np] = c[side];
          pt[np] = t[side];
          ++np;
        }
      }
    }
    sp -= m;
    h = hn;
    // push far first (descending t) so the nearest ends on top
    for (int a = 0; a < np; ++a)
      for (int q = a + 1; q < np; ++q)
        if (pt[q] > pt[a]) {
          const float tt = pt[a]; pt[a] = pt[q]; pt[q] = tt;
          const int nn = pn[a]; pn[a] = pn[q]; pn[q] = nn;
        }
    for (int a = 0; a < np && sp < 256; ++a) {
      stack[sp] = pn[a];
      stackt[sp] = pt[a];
      ++sp;
    }
  }
  out = h;
  return iters;
}

__global__ void k_steps(BvhView bv, const float4* nrm, float tx, float ty, float tz, int64_t off, int64_t n, int B,
                        int G, int* iters_seq, int* leaves_seq, int* iters_grp, int* mismatch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float3 dir = ray_dir(off + i);
  float3 pos = make_float3(tx, ty, tz);
  for (int k = 0; k < B; ++k) {
    const Shear s = make_shear(pos, dir);
    int it = 0, lv = 0;
    const Hit h = query_seq(bv, s, pos, dir, it, lv);
    Hit hg;
    const int ig = G > 0 ? query_group_iters(bv, s, pos, dir, G, hg) : 0;
    if (G > 0 && (hg.face != h.face || hg.t != h.t)) atomicAdd(mismatch, 1);
    iters_seq[i * B + k] = it;
    leaves_seq[i * B + k] = lv;
    iters_grp[i * B + k] = ig;
    if (h.face < 0) {
      for (int q = k + 1; q < B; ++q) iters_seq[i * B + q] = leaves_seq[i * B + q] = iters_grp[i * B + q] = -1;
      break;
    }
    pos.x = fmaf(dir.x, h.t, pos.x);
    pos.y = fmaf(dir.y, h.t, pos.y);
    pos.z = fmaf(dir.z, h.t, pos.z);
    const float4 n4 = nrm[h.face];
    const float3 nn = make_float3(n4.x, n4.y, n4.z);
    const float sc = 2.0f * dot3(dir, nn);
    dir.x = fmaf(-sc, nn.x, dir.x);
    dir.y = fmaf(-sc, nn.y, dir.y);
    dir.z = fmaf(-sc, nn.z, dir.z);
  }
}

// ---- traversal variants (timing study) ------------------------------------------------------
// V1/V2: one flat loop, one step per iteration: pop (re-culled) and visit in the same step.
// PACKED: leaf (first, count) read from the node's q3.z / q3.w (first << 3 | count) instead of
// a dependent load of leaves[].  LDS: the stack lives in LDS (per-lane column, depth SD).
template <bool PACKED, bool LDS, int SD>
__device__ __forceinline__ Hit query_flat(const BvhView& b, int nf, const Shear& s, float3 o, float3 d, int* lds_n,
                                          float* lds_t) {
  Hit h;
  hit_init(h);
  const RayBox r = make_raybox(o, d);
  int stack[RT_BVH_STACK];
  float stackt[RT_BVH_STACK];
  const int lane = threadIdx.x;
  const int bd = blockDim.x;
  int sp = 0, cur = 0;
  bool active = true;
  while (active) {
    bool visit = true;
    if (cur < 0) {
      if (sp == 0) {
        active = false;
        visit = false;
      } else {
        --sp;
        const int nn = LDS ? lds_n[sp * bd + lane] : stack[sp];
        const float tt = LDS ? lds_t[sp * bd + lane] : stackt[sp];
        if (tt <= h.t * 1.00001f + 1e-6f) cur = nn;
        else visit = false;
      }
    }
    if (visit) {
      const float4 q0 = b.nodes[4 * cur + 0], q1 = b.nodes[4 * cur + 1];
      const float4 q2 = b.nodes[4 * cur + 2], q3 = b.nodes[4 * cur + 3];
      const int c0 = __float_as_int(q3.x), c1 = __float_as_int(q3.y);
      float t0 = slab(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
      float t1 = slab(r, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w);
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int c = side ? c1 : c0;
        float& tt = side ? t1 : t0;
        if (c < 0) {
          if (tt <= h.t * 1.00001f + 1e-6f) {
            int first, count;
            if (PACKED) {
              const int pk = __float_as_int(side ? q3.w : q3.z);
              first = pk >> 3;
              count = pk & 7;
            } else {
              const int2 lf = b.leaves[-1 - c];
              first = lf.x;
              count = lf.y;
            }
            leaf4(b, s, first, count, h);
          }
          tt = INFINITY;
        }
      }
      const float lim = h.t * 1.00001f + 1e-6f;
      const bool h0 = t0 <= lim, h1 = t1 <= lim;
      if (h0 && h1) {
        const bool first0 = t0 <= t1;
        if (sp < SD) {
          if (LDS) {
            lds_n[sp * bd + lane] = first0 ? c1 : c0;
            lds_t[sp * bd + lane] = first0 ? t1 : t0;
          } else {
            stack[sp] = first0 ? c1 : c0;
            stackt[sp] = first0 ? t1 : t0;
          }
          ++sp;
        }
        cur = first0 ? c0 : c1;
      } else if (h0) {
        cur = c0;
      } else if (h1) {
        cur = c1;
      } else {
        cur = -1;
      }
    }
  }
  return h;
}

__global__ void k_pack_leaves(float4* nodes, const int2* leaves, int64_t nnodes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnodes) return;
  float4 q3 = nodes[4 * i + 3];
  const int c0 = __float_as_int(q3.x), c1 = __float_as_int(q3.y);
  if (c0 < 0) { const int2 l = leaves[-1 - c0]; q3.z = __int_as_float(l.x << 3 | l.y); }
  if (c1 < 0) { const int2 l = leaves[-1 - c1]; q3.w = __int_as_float(l.x << 3 | l.y); }
  nodes[4 * i + 3] = q3;
}

template <int MODE>
__global__ void k_time(BvhView bv, int nf, const float4* nrm, float tx, float ty, float tz, const int64_t* ids, int64_t n,
                       int B, float* out, int* oface) {
  extern __shared__ int lds_stack[];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float3 dir = ray_dir(ids[i]);
  float3 pos = make_float3(tx, ty, tz);
  float acc = 0.0f;
  int fs = 0;
  int* ln = lds_stack;
  float* lt = (float*)(lds_stack + 24 * blockDim.x);
  for (int k = 0; k < B; ++k) {
    const Shear s = make_shear(pos, dir);
    Hit h;
    if (MODE == 0) h = bvh_query(bv, s, pos, dir);
    else if (MODE == 1) h = query_flat<false, false, RT_BVH_STACK>(bv, nf, s, pos, dir, ln, lt);
    else if (MODE == 2) h = query_flat<true, false, RT_BVH_STACK>(bv, nf, s, pos, dir, ln, lt);
    else h = query_flat<true, true, 24>(bv, nf, s, pos, dir, ln, lt);
    acc += h.t;
    fs = fs * 31 + h.face;
    if (h.face < 0) break;
    pos.x = fmaf(dir.x, h.t, pos.x);
    pos.y = fmaf(dir.y, h.t, pos.y);
    pos.z = fmaf(dir.z, h.t, pos.z);
    const float4 n4 = nrm[h.face];
    const float3 nn = make_float3(n4.x, n4.y, n4.z);
    const float sc = 2.0f * dot3(dir, nn);
    dir.x = fmaf(-sc, nn.x, dir.x);
    dir.y = fmaf(-sc, nn.y, dir.y);
    dir.z = fmaf(-sc, nn.z, dir.z);
  }
  out[i] = acc;
  oface[i] = fs;
}
}  // namespace

// time variant `mode` over rays ids[0..n) (B env bounces, as k_traj); out/oface: per-ray checksums
extern "C" float bvh_time(const rt_mesh* m, const float* tx, const int64_t* ids, int64_t n, int B, int reps, int mode,
                          int block, float* out, int* oface) {
  static float4* packed = nullptr;
  static const rt_mesh* packed_for = nullptr;
  if (packed_for != m) {
    if (packed) (void)hipFree(packed);
    (void)hipMalloc(&packed, sizeof(float4) * 4 * m->nnodes);
    (void)hipMemcpy(packed, m->nodes, sizeof(float4) * 4 * m->nnodes, hipMemcpyDeviceToDevice);
    hipLaunchKernelGGL(k_pack_leaves, dim3((unsigned)((m->nnodes + 255) / 256)), dim3(256), 0, 0, packed,
                       (const int2*)m->leaves, m->nnodes);
    packed_for = m;
  }
  const BvhView bv{mode >= 2 ? (const float4*)packed : (const float4*)m->nodes, (const int2*)m->leaves,
                   (const float4*)m->lcomp, (int)m->nf};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const size_t lds = mode == 3 ? (size_t)block * 24 * 8 : 0;
  auto launch = [&]() {
    const dim3 g((unsigned)((n + block - 1) / block)), t(block);
    if (mode == 0) hipLaunchKernelGGL(k_time<0>, g, t, lds, 0, bv, (int)m->nf, m->nrm, tx[0], tx[1], tx[2], ids, n, B, out, oface);
    else if (mode == 1) hipLaunchKernelGGL(k_time<1>, g, t, lds, 0, bv, (int)m->nf, m->nrm, tx[0], tx[1], tx[2], ids, n, B, out, oface);
    else if (mode == 2) hipLaunchKernelGGL(k_time<2>, g, t, lds, 0, bv, (int)m->nf, m->nrm, tx[0], tx[1], tx[2], ids, n, B, out, oface);
    else hipLaunchKernelGGL(k_time<3>, g, t, lds, 0, bv, (int)m->nf, m->nrm, tx[0], tx[1], tx[2], ids, n, B, out, oface);
  };
  launch();
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

extern "C" int bvh_steps(const rt_mesh* m, const float* tx, int64_t off, int64_t n, int B, int G, int* iters_seq,
                         int* leaves_seq, int* iters_grp, int* mismatch) {
  const BvhView bv{(const float4*)m->nodes, (const int2*)m->leaves, (const float4*)m->lcomp, (int)m->nf};
  hipLaunchKernelGGL(k_steps, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, bv, m->nrm, tx[0], tx[1], tx[2], off,
                     n, B, G, iters_seq, leaves_seq, iters_grp, mismatch);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
