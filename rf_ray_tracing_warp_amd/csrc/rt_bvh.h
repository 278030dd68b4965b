// rt_bvh.h -- BVH traversal for large environment meshes (the BVH behind wp.Mesh, tracer.py:24,
// and the traversal inside wp.mesh_query_ray, kernel.py:82).
//
// Layout (built on the host by bvh.hip, HBM-resident):
//   nodes  float4[nnodes][4]: child boxes c0 = (lo.xyz, hi.xyz), c1 = ..., then child ids:
//          q0 = (c0lo.x, c0lo.y, c0lo.z, c0hi.x)  q1 = (c0hi.y, c0hi.z, c1lo.x, c1lo.y)
//          q2 = (c1lo.z, c1hi.x, c1hi.y, c1hi.z)  q3 = (child0, child1, leaf0, leaf1) as int bits
//          child >= 0: internal node index;  child < 0: leaf -1-child into `leaves`, whose
//          (first, count) is also packed into leaf0/leaf1 as first << 3 | count (count <= 4) by
//          rt::pack_leaf_refs after either builder, so traversal never loads `leaves`
//   leaves int2[nleaves]: (first, count) into the leaf-ordered face table
//   lcomp  float4[nf][3]: faces in leaf order, un-permuted: (a.xyz b.x)(b.yz c.xy)(c.z, original
//          face id bits, -, -).  48 B per face, all of it used by every lane; the corners are
//          permuted to the lane's shear axes with selects.  (A leaf-ordered copy of the 288-B
//          six-case records of rt_mesh.perm measured 17% slower on K4: a lane reads only the
//          36 B of its case, so most of every fetched line is wasted.)
// Boxes are padded outward on the host so the f32 slab test below can never cull a face the
// watertight test would hit; the closest hit is the lexicographic (t, original face id) minimum,
// so traversal order cannot change a result (bit-exact vs the brute-force oracle).
#pragma once
#include "rt_device.h"

namespace rt {

struct BvhView {
  const float4* nodes;
  const int2* leaves;
  const float4* lcomp;
  int nf;  // faces in lcomp
  const float4* wide;  // 4-wide nodes (8 float4 each, see Walk4), collapsed from `nodes`
};

#define RT_BVH_STACK 64

struct RayBox {
  float ox, oy, oz, ix, iy, iz;  // origin and per-axis reciprocal direction (never 0/NaN)
};

__device__ __forceinline__ float safe_rcp(float d) {
  const float m = fabsf(d) < 1e-30f ? copysignf(1e-30f, d) : d;
  return 1.0f / m;
}

__device__ __forceinline__ RayBox make_raybox(float3 o, float3 d) {
  RayBox r;
  r.ox = o.x;
  r.oy = o.y;
  r.oz = o.z;
  r.ix = safe_rcp(d.x);
  r.iy = safe_rcp(d.y);
  r.iz = safe_rcp(d.z);
  return r;
}

// slab test, returns entry t (clamped at 0) or +inf on a miss; conservative slack on both ends
__device__ __forceinline__ float slab(const RayBox& r, float lx, float ly, float lz, float hx, float hy, float hz) {
  const float tx0 = (lx - r.ox) * r.ix, tx1 = (hx - r.ox) * r.ix;
  const float ty0 = (ly - r.oy) * r.iy, ty1 = (hy - r.oy) * r.iy;
  const float tz0 = (lz - r.oz) * r.iz, tz1 = (hz - r.oz) * r.iz;
  const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
  const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
  return tn <= tf * 1.00001f + 1e-6f ? tn : INFINITY;
}

// leaf faces [first, first + count), count <= 4: the four 48-B records are fetched together
// (indices clamped into the table, the results of q >= count ignored), so a leaf costs one
// memory latency instead of one per face
__device__ __forceinline__ void leaf4(const BvhView& b, const Shear& s, int first, int count, Hit& h) {
  float4 A[4], M[4], C[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = min(first + q, b.nf - 1);
    const float4* p = b.lcomp + (int64_t)j * 3;
    A[q] = p[0];
    M[q] = p[1];
    C[q] = p[2];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < count) {
      const float4 a = A[q], m = M[q], c = C[q];
      // corners A = (a.x a.y a.z), B = (a.w m.x m.y), C = (m.z m.w c.x) -> (kx, ky, kz) order
      const float4 q0 = make_float4(pick(a.x, a.y, a.z, s.kx), pick(a.x, a.y, a.z, s.ky), pick(a.x, a.y, a.z, s.kz),
                                    pick(a.w, m.x, m.y, s.kx));
      const float4 q1 = make_float4(pick(a.w, m.x, m.y, s.ky), pick(a.w, m.x, m.y, s.kz), pick(m.z, m.w, c.x, s.kx),
                                    pick(m.z, m.w, c.x, s.ky));
      const float c2 = pick(m.z, m.w, c.x, s.kz);
      float T, det;
      if (tri_test(s, q0, q1, c2, T, det)) hit_consider(h, T, det, __float_as_int(c.y));
    }
  }
}

__device__ __forceinline__ float cull_limit(const Hit& h, float tc) { return fminf(h.t, tc) * 1.00001f + 1e-6f; }

// Closest hit in a BVH mesh, the same result as brute force over all faces, as a resumable walk:
// init() for a ray, then step() until it returns false; h is then the (t, face) minimum.  One step
// = one flat-loop iteration for every lane (pop, re-culled against the best t, and visit in the
// same step; leaves tested on the spot from the (first, count) packed in their parent), so a wave
// iterates as often as its longest lane.  (The nested-loop form -- descend, inner pop loop, inner
// face loop -- made lanes wait for each other at every phase change: the slowest wave of a
// 125k-ray K5 burst took 2.2x longer.)  Callers either loop step() (bvh_query) or interleave
// steps of different rays and bounces in one loop (k_trace_pool).
//
// tcull < RT_MAX_T also culls boxes beyond tcull: every hit with t <= tcull is still found
// exactly, hits beyond it may be missed (callers that only compare against tcull use it).

// The (node, entry t) stack, kept apart from the walk's scalar state: inside one aggregate with
// the dynamically indexed arrays, the scalars went to scratch too (k_traj<true> 92 -> 102 VGPRs
// and +40 B scratch: cur, sp, the best hit and the ray box reloaded every step).
//
// The kLdsStack entries nearest the bottom of every lane's stack live in LDS (a [K][256] column per
// thread of the 256-thread block: lanes of a wave always hit distinct banks, whatever their stack
// pointers) and only deeper entries in the private array, so a walk that stays within K pending
// entries never touches scratch memory (K4 rt_trace 1825 -> 1328 us, K5 map 5.53 -> 4.74 ms against
// the all-private stack, profiles/r3b_*; 8 entries measured the same).
constexpr int kLdsStack = 16;
struct WalkStack {
  int* ln;    // this thread's LDS column: entry i at ln[256 * i]
  float* lt;
  int node[RT_BVH_STACK - kLdsStack];
  float t[RT_BVH_STACK - kLdsStack];
  __device__ __forceinline__ void set(int i, int c, float tt) {
    if (i < kLdsStack) {
      ln[256 * i] = c;
      lt[256 * i] = tt;
    } else {
      node[i - kLdsStack] = c;
      t[i - kLdsStack] = tt;
    }
  }
  __device__ __forceinline__ int get_node(int i) const { return i < kLdsStack ? ln[256 * i] : node[i - kLdsStack]; }
  __device__ __forceinline__ float get_t(int i) const { return i < kLdsStack ? lt[256 * i] : t[i - kLdsStack]; }
};
// every kernel that walks gets one [K][256] block of LDS (blocks of at most 256 threads)
__device__ __forceinline__ WalkStack make_stack() {
  __shared__ int s_node[kLdsStack * 256];
  __shared__ float s_t[kLdsStack * 256];
  WalkStack st;
  st.ln = s_node + threadIdx.x;
  st.lt = s_t + threadIdx.x;
  return st;
}
// 4-wide nodes (bvh_wide.hip collapses the binary tree, breadth first): 8 float4 = 128 B,
//   w[0] lo.x[4]  w[1] hi.x[4]  w[2] lo.y[4]  w[3] hi.y[4]  w[4] lo.z[4]  w[5] hi.z[4]
//   w[6] child refs (int bits): >= 0 wide node, -1 empty slot, <= -2 leaf ~(first << 3 | count)
// The child boxes are the binary tree's own (rounded outward and padded), so culling stays
// exactly as conservative as the binary tree's and the (t, face) minimum cannot depend on the tree.
// Per visit: four slab tests; the hit leaves tested on the spot, nearest first; the hit inner
// children sorted by entry t, the nearest visited next and the others pushed far to near.
// About half the dependent node fetches of the binary walk per query.  (The top 85 or 192 wide
// nodes staged in LDS per workgroup measured slower, 1575 / 1603 vs 1522 us on K4 with the same
// row mapping: every wave of a direction-sorted burst reads the same top nodes, which L1/L2 serve.)
// (Sorting packed keys instead -- the entry t's bits with the slot in the low 2 bits, two min/max
// per compare-exchange -- was bit-identical and slower: K4 rt_trace 731-735 vs 714-719 us, the
// slot decode and extra selects outweighing the cheaper exchanges; profiles/r6za_*, round 6.)
__device__ __forceinline__ void cas(float& ta, int& ra, float& tb, int& rb) {
  const bool sw = tb < ta;
  const float t0 = sw ? tb : ta, t1 = sw ? ta : tb;
  const int r0 = sw ? rb : ra, r1 = sw ? ra : rb;
  ta = t0;
  tb = t1;
  ra = r0;
  rb = r1;
}

struct Walk4 {
  Hit h;
  RayBox r;
  float tc;
  int cur, sp;

  __device__ __forceinline__ void init(float3 o, float3 d, float tcull = RT_MAX_T) {
    hit_init(h);
    tc = fminf(RT_MAX_T, tcull);
    r = make_raybox(o, d);
    cur = 0;
    sp = 0;
  }
  __device__ __forceinline__ void push(WalkStack& st, int c, float t) {
    if (sp < RT_BVH_STACK) {  // cannot overflow: bound checked on the host (build_wide)
      st.set(sp, c, t);
      ++sp;
    }
  }
  __device__ __forceinline__ bool step(const BvhView& b, const Shear& s, WalkStack& st) {
    bool visit = true;
    if (cur < 0) {  // pop
      if (sp == 0) return false;
      --sp;
      if (st.get_t(sp) <= cull_limit(h, tc)) cur = st.get_node(sp);
      else visit = false;
    }
    if (visit) {
    const float4* w = b.wide + 8 * (int64_t)cur;
    const float4 lx = w[0], hx = w[1], ly = w[2], hy = w[3], lz = w[4], hz = w[5];
    const float4 rf = w[6];
    int c0 = __float_as_int(rf.x), c1 = __float_as_int(rf.y), c2 = __float_as_int(rf.z), c3 = __float_as_int(rf.w);
    float t0 = slab(r, lx.x, ly.x, lz.x, hx.x, hy.x, hz.x);
    float t1 = slab(r, lx.y, ly.y, lz.y, hx.y, hy.y, hz.y);
    float t2 = slab(r, lx.z, ly.z, lz.z, hx.z, hy.z, hz.z);
    float t3 = slab(r, lx.w, ly.w, lz.w, hx.w, hy.w, hz.w);
    // leaves (and empty slots) leave the ordering; hit leaves are tested now, nearest first
    float l0 = c0 < -1 ? t0 : INFINITY, l1 = c1 < -1 ? t1 : INFINITY;
    float l2 = c2 < -1 ? t2 : INFINITY, l3 = c3 < -1 ? t3 : INFINITY;
    int p0 = ~c0, p1 = ~c1, p2 = ~c2, p3 = ~c3;
    t0 = c0 >= 0 ? t0 : INFINITY;
    t1 = c1 >= 0 ? t1 : INFINITY;
    t2 = c2 >= 0 ? t2 : INFINITY;
    t3 = c3 >= 0 ? t3 : INFINITY;
    cas(l0, p0, l1, p1);
    cas(l2, p2, l3, p3);
    cas(l0, p0, l2, p2);
    cas(l1, p1, l3, p3);
    cas(l1, p1, l2, p2);
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {  // one leaf4 body in the code; the sorted list shifts down
      if (!(l0 <= cull_limit(h, tc))) break;
      leaf4(b, s, p0 >> 3, p0 & 7, h);
      l0 = l1;
      l1 = l2;
      l2 = l3;
      l3 = INFINITY;
      p0 = p1;
      p1 = p2;
      p2 = p3;
    }
    cas(t0, c0, t1, c1);
    cas(t2, c2, t3, c3);
    cas(t0, c0, t2, c2);
    cas(t1, c1, t3, c3);
    cas(t1, c1, t2, c2);
    const float lim = cull_limit(h, tc);
    if (t0 <= lim) {  // far to near, so the nearest of the rest is popped first
      if (t3 <= lim) push(st, c3, t3);
      if (t2 <= lim) push(st, c2, t2);
      if (t1 <= lim) push(st, c1, t1);
      cur = c0;
    } else {
      cur = -1;
    }
    }
    return true;
  }
};

// Lane j (0..G-1) of a group of G lanes (G = 4 or 16) that trace ONE ray together.  G = 4: lane j
// walks the subtrees of grandchild slot j of every inner child of the root (and the root's leaf
// children c with c % 4 == j); G = 16: lane j walks grandchild slot j % 4 of root child j / 4 only
// (a leaf child c by lane 4c).  The group's (t, face) minimum (group_hit) is the ray's closest hit;
// each lane culls with the group's best t so far (group_min_t), exact for the same reason tcull is.
// Used where a burst is too small to fill the GPU (a ray-sharded rank traces 1/8 of the rays and the
// slowest ray's chain of dependent fetches sets the time).
template <int G>
__device__ __forceinline__ void split_init(Walk4& w, WalkStack& st, const BvhView& b, const Shear& s, float3 o,
                                           float3 d, int j, float tcull = RT_MAX_T) {
  static_assert(G == 4 || G == 16, "split over 4 or 16 lanes");
  w.init(o, d, tcull);
  w.cur = -1;
  const float4 rf = b.wide[6];
  const int rc[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
  const int gslot = j & 3;
#pragma unroll 1
  for (int c = 0; c < 4; ++c) {
    if (G == 16 && c != (j >> 2)) continue;
    const int ref = rc[c];
    if (ref < -1) {  // leaf child of the root
      if ((G == 4 && (c & 3) == j) || (G == 16 && gslot == 0)) {
        const int pk = ~ref;
        leaf4(b, s, pk >> 3, pk & 7, w.h);
      }
    } else if (ref >= 0) {  // inner child: its grandchild slot
      const float4* cw = b.wide + 8 * (int64_t)ref;
      const float4 lx = cw[0], hx = cw[1], ly = cw[2], hy = cw[3], lz = cw[4], hz = cw[5], cr = cw[6];
      const int q = gslot;
      const float sel_lx = q == 0 ? lx.x : q == 1 ? lx.y : q == 2 ? lx.z : lx.w;
      const float sel_ly = q == 0 ? ly.x : q == 1 ? ly.y : q == 2 ? ly.z : ly.w;
      const float sel_lz = q == 0 ? lz.x : q == 1 ? lz.y : q == 2 ? lz.z : lz.w;
      const float sel_hx = q == 0 ? hx.x : q == 1 ? hx.y : q == 2 ? hx.z : hx.w;
      const float sel_hy = q == 0 ? hy.x : q == 1 ? hy.y : q == 2 ? hy.z : hy.w;
      const float sel_hz = q == 0 ? hz.x : q == 1 ? hz.y : q == 2 ? hz.z : hz.w;
      const int g = __float_as_int(q == 0 ? cr.x : q == 1 ? cr.y : q == 2 ? cr.z : cr.w);
      const float t = slab(w.r, sel_lx, sel_ly, sel_lz, sel_hx, sel_hy, sel_hz);
      if (g < -1) {
        if (t <= cull_limit(w.h, w.tc)) {
          const int pk = ~g;
          leaf4(b, s, pk >> 3, pk & 7, w.h);
        }
      } else if (g >= 0 && t <= cull_limit(w.h, w.tc)) {
        w.push(st, g, t);
      }
    }
  }
}
// the group's best t so far (xor butterfly over the G lanes); every lane of the wave must call it
template <int G>
__device__ __forceinline__ float group_min_t(float t) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) t = fminf(t, __shfl_xor(t, o, 64));
  return t;
}
// lexicographic (t, face) minimum over the group; every lane of the wave must call it
template <int G>
__device__ __forceinline__ Hit group_hit(Hit h) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const float t2 = __shfl_xor(h.t, o, 64);
    const int f2 = __shfl_xor(h.face, o, 64);
    const bool better = f2 >= 0 && (h.face < 0 || t2 < h.t || (t2 == h.t && f2 < h.face));
    h.t = better ? t2 : h.t;
    h.face = better ? f2 : h.face;
  }
  return h;
}

// (Binary nodes (Walk2), compressed 8-wide nodes (Walk8), leaf faces fetched in pairs and a
// next-node prefetch were measured and removed in round 5; last in commit 43de9a4)
using Walk = Walk4;

// (Wave-packet walks -- all 64 lanes of a wave on one node sequence, node and leaf data read once
// per wave through the scalar cache, a wave stack in LDS of (node, lanes, smallest entry t) -- were
// bit-identical on every BVH parity test and 4-5x slower: K4 rt_trace 2974-2988 vs 719-720 us, K5
// trajectory pass 2.06 vs 0.395 ms (profiles/r6i_*_bvh_packet_ab.jsonl).  A direction-sorted wave's
// rays reach terrain points metres apart (and reflect apart), so the packet visits the
// union of 64 walks, and each visit is a chain of dependent scalar loads.  Removed in round 6.)

// RT_COUNT_STEPS (diagnostic builds only, tools/walk_stats.py): per query, the lane's walk steps and
// its share of the wave's loop iterations (1 / active lanes per iteration, so the shares of a wave
// add up to its iteration count), summed over 16 slots by block; the max steps of one query.
#ifndef RT_COUNT_STEPS
#define RT_COUNT_STEPS 0
#endif
#if RT_COUNT_STEPS
static __device__ unsigned long long g_walk_stats[16 * 4];  // steps, iterations * 2^16, queries, max steps
#endif

__device__ __forceinline__ Hit bvh_query(const BvhView& b, const Shear& s, float3 o, float3 d,
                                         float tcull = RT_MAX_T) {
  Walk w;
  WalkStack st = make_stack();
  w.init(o, d, tcull);
  bool active = true;
#if RT_COUNT_STEPS
  unsigned steps = 0;
  float iters = 0.0f;
  while (active) {
    iters += 1.0f / (float)__popcll(__ballot(1));
    ++steps;
    active = w.step(b, s, st);
  }
  unsigned long long* g = g_walk_stats + 4 * (blockIdx.x & 15);
  atomicAdd(g + 0, (unsigned long long)steps);
  atomicAdd(g + 1, (unsigned long long)(iters * 65536.0f + 0.5f));
  atomicAdd(g + 2, 1ull);
  atomicMax(g + 3, (unsigned long long)steps);
#else
  while (active) active = w.step(b, s, st);
#endif
  return w.h;
}

}  // namespace rt
