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

// closest hit in a BVH mesh (same result as brute force over all faces): near child first, far
// child on a per-lane (node, entry t) stack, popped entries re-culled against the best t.
// tcull < RT_MAX_T also culls boxes beyond tcull: every hit with t <= tcull is still found
// exactly, hits beyond it may be missed (callers that only compare against tcull use it).
//
// One flat loop, one step per iteration for every lane: pop (re-culled) and visit happen in the
// same step, leaves are tested on the spot from the (first, count) packed in their parent node,
// so a wave iterates as often as its longest lane.  (The nested-loop form -- descend, inner
// pop loop, inner face loop -- made lanes wait for each other at every phase change: the
// slowest wave of a 125k-ray K5 burst took 2.2x longer.)
__device__ __forceinline__ Hit bvh_query(const BvhView& b, const Shear& s, float3 o, float3 d,
                                         float tcull = RT_MAX_T) {
  Hit h;
  hit_init(h);
  const float tc = fminf(RT_MAX_T, tcull);
  const RayBox r = make_raybox(o, d);
  int stack[RT_BVH_STACK];
  float stackt[RT_BVH_STACK];
  int sp = 0, cur = 0;
  bool active = true;
  while (active) {
    bool visit = true;
    if (cur < 0) {  // pop
      if (sp == 0) {
        active = false;
        visit = false;
      } else {
        --sp;
        if (stackt[sp] <= fminf(h.t, tc) * 1.00001f + 1e-6f) cur = stack[sp];
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
        if (c < 0) {  // leaf child: test its faces now
          if (tt <= fminf(h.t, tc) * 1.00001f + 1e-6f) {
            const int pk = __float_as_int(side ? q3.w : q3.z);
            leaf4(b, s, pk >> 3, pk & 7, h);
          }
          tt = INFINITY;
        }
      }
      const float lim = fminf(h.t, tc) * 1.00001f + 1e-6f;
      const bool h0 = t0 <= lim, h1 = t1 <= lim;
      if (h0 && h1) {
        const bool first0 = t0 <= t1;
        if (sp < RT_BVH_STACK) {  // cannot overflow: tree depth <= RT_BVH_STACK - 4 (bvh.hip)
          stack[sp] = first0 ? c1 : c0;
          stackt[sp] = first0 ? t1 : t0;
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

}  // namespace rt
