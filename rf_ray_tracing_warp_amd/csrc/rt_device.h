// rt_device.h -- device arithmetic of the ray tracer (gfx950).
//
// Every function here restates one piece of the reference kernel and must agree bit for bit
// with the CPU oracle (oracle/rt_oracle.c), which restates the same contract independently.
// The build compiles this with -ffp-contract=off: the only fused multiply-adds are the
// explicit fmaf() calls, placed where nvcc's LLVM contraction puts them in Warp's CUDA build
// (pinned on the reference artifact web/scene.html, see DESIGN.md "Arithmetic contract").
//
//   ray generation   kernel.py:51-52  wp.rand_init(tid), wp.sample_unit_sphere_surface
//   closest hit      kernel.py:71,82  wp.mesh_query_ray -> watertight ray/triangle test
//   advance/reflect  kernel.py:87,94,96 and kernel.py:6-8
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_MAX_T 1.0e6f  // kernel.py:71,82 max_t

namespace rt {

// ------------------------------------------------------------------ ray generation
__device__ __forceinline__ uint32_t pcg(uint32_t s) {
  uint32_t b = s * 747796405u + 2891336453u;
  uint32_t c = ((b >> ((b >> 28u) + 4u)) ^ b) * 277803737u;
  return (c >> 22u) ^ c;
}

__device__ __forceinline__ float sin_poly(float r) {
  float z = r * r;
  float p = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
  p = fmaf(z, p, -1.6666654611e-1f);
  return fmaf(r * z, p, r);
}
__device__ __forceinline__ float cos_poly(float r) {
  float z = r * r;
  float p = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
  p = fmaf(z, p, 4.166664568298827e-2f);
  return fmaf(z * z, p, fmaf(-0.5f, z, 1.0f));
}
// Cody-Waite reduction by pi/2 (2-part constant; first step exact for |x| < 8)
__device__ __forceinline__ void sincos_rt(float x, float* s, float* c) {
  const float k = rintf(x * 0.636619746685028076171875f);
  float r = fmaf(-k, 1.57079637050628662109375f, x);
  r = fmaf(-k, -4.37113900018624283e-8f, r);
  const float sp = sin_poly(r), cp = cos_poly(r);
  const int q = ((int)k) & 3;
  const float ss = (q & 1) ? cp : sp;
  const float cc = (q & 1) ? sp : cp;
  *s = (q & 2) ? -ss : ss;
  *c = ((q + 1) & 2) ? -cc : cc;
}
__device__ __forceinline__ float asin_small(float x) {
  float z = x * x;
  float p = fmaf(4.2163199048e-2f, z, 2.4181311049e-2f);
  p = fmaf(p, z, 4.5470025998e-2f);
  p = fmaf(p, z, 7.4953002686e-2f);
  p = fmaf(p, z, 1.6666752422e-1f);
  return fmaf(p * z, x, x);
}
__device__ __forceinline__ float acos_rt(float x) {
  if (x < -0.5f) return 3.14159274101257324219f - 2.0f * asin_small(__builtin_sqrtf(0.5f * (1.0f + x)));
  if (x > 0.5f) return 2.0f * asin_small(__builtin_sqrtf(0.5f * (1.0f - x)));
  return 1.57079637050628662109375f - asin_small(x);
}

// wp.sample_unit_sphere_surface(wp.rand_init(gid)): phi from the first draw, theta from the second
__device__ __forceinline__ float3 ray_dir(int64_t gid) {
  uint32_t st = pcg((uint32_t)gid);
  st = pcg(st);
  const float u1 = (float)(st >> 8) * (1.0f / 16777216.0f);
  const float phi = acos_rt(1.0f - 2.0f * u1);
  st = pcg(st);
  const float u2 = (float)(st >> 8) * (1.0f / 16777216.0f);
  const float theta = 6.28318548202514648438f * u2;  // (2pi - 0) * u + 0
  float s_t, c_t, s_p, c_p;
  sincos_rt(theta, &s_t, &c_t);
  sincos_rt(phi, &s_p, &c_p);
  return make_float3(c_t * s_p, s_t * s_p, c_p);
}

// ------------------------------------------------------------------ vector helpers
__device__ __forceinline__ float dot3(float3 a, float3 b) {  // a.x*b.x + a.y*b.y + a.z*b.z, contracted
  return fmaf(a.z, b.z, fmaf(a.x, b.x, a.y * b.y));
}
__device__ __forceinline__ float comp(float3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

// ------------------------------------------------------------------ watertight test
// Per-ray precompute (Warp intersect_ray_tri_woop "precompute" block).  case = kz*2 + swap
// indexes the host-built permuted corner table, so the per-triangle permutation is a load.
struct Shear {
  float3 o;  // origin permuted to (o[kx], o[ky], o[kz])
  float Sx, Sy, Sz;
  int kcase;
  int kx, ky, kz;
};

// component k of (x, y, z) -- permutes un-permuted corners per lane (compact BVH leaves)
__device__ __forceinline__ float pick(float x, float y, float z, int k) { return k == 0 ? x : (k == 1 ? y : z); }

__device__ __forceinline__ Shear make_shear(float3 o, float3 d) {
  const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  const int kz = (ax > ay && ax > az) ? 0 : ((ay > az) ? 1 : 2);
  int kx = kz + 1;
  if (kx == 3) kx = 0;
  int ky = kx + 1;
  if (ky == 3) ky = 0;
  const float dkz = comp(d, kz);
  const int swap = dkz < 0.0f;
  if (swap) {
    const int t = kx;
    kx = ky;
    ky = t;
  }
  Shear s;
  s.o = make_float3(comp(o, kx), comp(o, ky), comp(o, kz));
  s.Sx = comp(d, kx) / dkz;
  s.Sy = comp(d, ky) / dkz;
  s.Sz = 1.0f / dkz;
  s.kcase = kz * 2 + swap;
  s.kx = kx;
  s.ky = ky;
  s.kz = kz;
  return s;
}

// One triangle given its permuted corners packed as q0 = (a0 a1 a2 b0), q1 = (b1 b2 c0 c1), c2
// (index 0 = [kx], 1 = [ky], 2 = [kz]); two ds_read_b128 + one ds_read_b32 per face.
// Returns true when the watertight test accepts; T and det give t = T * (1/det).
__device__ __forceinline__ bool tri_test(const Shear& s, float4 q0, float4 q1, float c2, float& T, float& det) {
  const float A0 = q0.x - s.o.x, A1 = q0.y - s.o.y, A2 = q0.z - s.o.z;
  const float B0 = q0.w - s.o.x, B1 = q1.x - s.o.y, B2 = q1.y - s.o.z;
  const float C0 = q1.z - s.o.x, C1 = q1.w - s.o.y, C2 = c2 - s.o.z;
  const float Ax = fmaf(-s.Sx, A2, A0), Ay = fmaf(-s.Sy, A2, A1);
  const float Bx = fmaf(-s.Sx, B2, B0), By = fmaf(-s.Sy, B2, B1);
  const float Cx = fmaf(-s.Sx, C2, C0), Cy = fmaf(-s.Sy, C2, C1);
  float U = fmaf(Cx, By, -(Cy * Bx));
  float V = fmaf(Ax, Cy, -(Ay * Cx));
  float W = fmaf(Bx, Ay, -(By * Ax));
  // any of U,V,W == 0 (min3 of magnitudes: one v_min3 + one compare; U,V,W are never NaN here)
  if (fminf(fminf(fabsf(U), fabsf(V)), fabsf(W)) == 0.0f) {  // edge/vertex case: recompute in double
    U = (float)((double)Cx * (double)By - (double)Cy * (double)Bx);
    V = (float)((double)Ax * (double)Cy - (double)Ay * (double)Cx);
    W = (float)((double)Bx * (double)Ay - (double)By * (double)Ax);
  }
  const bool anyneg = (U < 0.0f) | (V < 0.0f) | (W < 0.0f);
  const bool anypos = (U > 0.0f) | (V > 0.0f) | (W > 0.0f);
  det = U + V + W;
  const float Az = s.Sz * A2, Bz = s.Sz * B2, Cz = s.Sz * C2;
  T = fmaf(W, Cz, fmaf(U, Az, V * Bz));
  const float Ts = det < 0.0f ? -T : T;
  return !(anyneg & anypos) & (det != 0.0f) & !(Ts < 0.0f);
}

// Closest-hit state: lexicographic min of (t, face), t = T*(1/det) exactly as Warp computes it.
struct Hit {
  float t;
  int face;
};

__device__ __forceinline__ void hit_init(Hit& h) {
  h.t = RT_MAX_T;
  h.face = -1;
}
// Exact update: t = T*(1/det) with the correctly rounded reciprocal, as Warp computes it.
__device__ __forceinline__ void hit_update_exact(Hit& h, float T, float det, int face) {
  const float t = T * (1.0f / det);
  const bool better = (t < h.t) | ((t == h.t) & (face < h.face));
  if (better & (t >= 0.0f) & (t < RT_MAX_T)) {
    h.t = t;
    h.face = face;
  }
}
// Screened update: v_rcp_f32 (1 ulp) gives a = T*rcp(det) within 2^-21 of the exact t, so a
// candidate with a > h.t*(1+2^-16) cannot win and skips the ~12-instruction IEEE division.
// The decision (and so every output bit) is identical to hit_update_exact.
__device__ __forceinline__ void hit_consider(Hit& h, float T, float det, int face) {
  const float a = fabsf(T) * __builtin_amdgcn_rcpf(fabsf(det));
  if (!(a > h.t * 1.0000153f)) hit_update_exact(h, T, det, face);
}

// Closest hit over faces tested in ASCENDING face order (the brute-force loops), with the IEEE
// division deferred.  A later face can only win by a strictly smaller t (ties keep the lower face
// id, which came first), so the state is the best candidate's (T, det), its approximate t
// a = |T| * v_rcp(|det|) (within ~2^-21 of the exact T * (1/det) for normal values), and its face.
//   a > best.a * (1 + 2^-16)                  cannot win: skip (as hit_consider)
//   a < best.a * (1 - 2^-16), both normal     wins outright (exact t < exact best t); a self-hit
//                                             at T == 0 against a normal best also wins outright
//   otherwise (near tie, tiny, odd det)       the exact rule of hit_update_exact
// An accepted T == 0 is t = +-0, which no later face can beat, so the lane then skips the rest.
// lazy_finish computes the winner's t = T * (1/det) once per query: the decision and every output
// bit equal hit_update_exact's, with one division per query instead of one per competitive face.
struct LazyHit {
  float T, det, a;
  int face;
};
__device__ __forceinline__ void lazy_init(LazyHit& h) {
  h.T = RT_MAX_T;  // the "no hit" sentinel t = 1e6 * (1 / 1) = 1e6, face -1
  h.det = 1.0f;
  h.a = RT_MAX_T;
  h.face = -1;
}
__device__ __forceinline__ void lazy_consider(LazyHit& h, float T, float det, int face) {
  const float a = fabsf(T) * __builtin_amdgcn_rcpf(fabsf(det));
  if ((a > h.a * 1.0000153f) | (h.T == 0.0f)) return;
  bool take;
  if ((a < h.a * 0.9999847f) &
      ((a >= 1e-30f) | ((T == 0.0f) & (fabsf(det) >= 0x1p-125f) & (h.a >= 1e-30f)))) {
    take = true;
  } else {
    const float t = T * (1.0f / det), tb = h.T * (1.0f / h.det);
    take = (t < tb) & (t >= 0.0f) & (t < RT_MAX_T);
  }
  if (take) {
    h.T = T;
    h.det = det;
    h.a = a;
    h.face = face;
  }
}
__device__ __forceinline__ Hit lazy_finish(const LazyHit& h) {
  Hit r;
  r.t = h.T * (1.0f / h.det);
  r.face = h.face;
  return r;
}

}  // namespace rt
