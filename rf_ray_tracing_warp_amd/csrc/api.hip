// api.hip -- the C ABI of librfrt.so (declared in include/rfrt.h).
//
// Conventions: every entry point returns int status (0 ok, <0 error) and never throws; the
// message of the last error on the calling thread is rt_last_error().  Device pointers are
// caller-owned (PyTorch data_ptr()s); launches are asynchronous on the caller's hipStream_t.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/rfrt.h"
#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_internal.h"

namespace rt {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return RT_EHIP;
}
int build_bvh(rt_mesh* m, const std::vector<float>& tri);      // bvh.hip (host, binned SAH)
int build_bvh_gpu(rt_mesh* m, const std::vector<float>& tri);  // bvh_gpu.hip (device LBVH)

__global__ void k_pack_leaf_refs(float4* nodes, const int2* leaves, int64_t nnodes) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnodes; i += (int64_t)gridDim.x * blockDim.x) {
    float4 q3 = nodes[4 * i + 3];
    const int c0 = __float_as_int(q3.x), c1 = __float_as_int(q3.y);
    if (c0 < 0) {
      const int2 l = leaves[-1 - c0];
      q3.z = __int_as_float(l.x << 3 | l.y);
    }
    if (c1 < 0) {
      const int2 l = leaves[-1 - c1];
      q3.w = __int_as_float(l.x << 3 | l.y);
    }
    nodes[4 * i + 3] = q3;
  }
}

int g_poison = -1;
extern bool g_profile;                      // trace.hip
extern int g_profile_every;                 // trace.hip
int trace_last_profile(double* out, int n);  // trace.hip
int trace_profile_stats(double* out, int n);  // trace.hip
void profile_reset();                        // trace.hip
void keep_pool_memory();  // trace.hip

int poison_pool(size_t bytes, hipStream_t s) {
  keep_pool_memory();  // freed blocks stay in the pool, so the next allocations see the poison
  void* p = nullptr;
  RT_HIP(hipMallocAsync(&p, bytes, s));
  RT_HIP(hipMemsetAsync(p, g_poison & 0xFF, bytes, s));
  RT_HIP(hipFreeAsync(p, s));
  return RT_OK;
}

int pack_leaf_refs(rt_mesh* m) {
  if (m->nf >= ((int64_t)1 << 28) || m->bvh_max_leaf > 4) {
    set_error("rt_mesh_create: BVH leaves must hold <= 4 faces of a mesh below 2^28 faces");
    return RT_EINVAL;
  }
  hipLaunchKernelGGL(k_pack_leaf_refs, dim3((unsigned)std::min<int64_t>((m->nnodes + 255) / 256, 8192)), dim3(256), 0,
                     0, (float4*)m->nodes, (const int2*)m->leaves, m->nnodes);
  RT_HIP(hipGetLastError());
  RT_HIP(hipDeviceSynchronize());
  return RT_OK;
}
}  // namespace rt

extern "C" {

const char* rt_last_error(void) { return rt::g_err.c_str(); }

int rt_version(void) { return RFRT_VERSION; }

int rt_profile(int enable) {
  if (enable < 0) {
    rt::set_error("rt_profile: enable must be 0, 1 or a sampling period > 1");
    return RT_EINVAL;
  }
  if (enable && (!rt::g_profile || rt::g_profile_every != enable)) rt::profile_reset();
  rt::g_profile = enable != 0;
  rt::g_profile_every = enable > 1 ? enable : 1;
  return RT_OK;
}

int rt_trace_profile_stats(double* out, int n) {
  if (!out || n < 1) {
    rt::set_error("rt_trace_profile_stats: invalid arguments");
    return RT_EINVAL;
  }
  return rt::trace_profile_stats(out, n);
}

int rt_trace_last_profile(double* out, int n) {
  if (!out || n < 1) {
    rt::set_error("rt_trace_last_profile: invalid arguments");
    return RT_EINVAL;
  }
  return rt::trace_last_profile(out, n);
}

int rt_debug_poison(int byte) {
  if (byte > 255) {
    rt::set_error("rt_debug_poison: byte must be 0..255 (or < 0 to disable)");
    return RT_EINVAL;
  }
  rt::g_poison = byte < 0 ? -1 : byte;
  return RT_OK;
}

// same contraction as the device / oracle: a.x*b.x + a.y*b.y + a.z*b.z
static inline float h_dot(const float* a, const float* b) {
  return std::fmaf(a[2], b[2], std::fmaf(a[0], b[0], a[1] * b[1]));
}

int rt_mesh_create(int device, const float* vertices, int64_t nv, const int32_t* faces, int64_t nf, rt_mesh** out) {
  return rt_mesh_create_ex(device, vertices, nv, faces, nf, 0, out);
}

int rt_mesh_create_ex(int device, const float* vertices, int64_t nv, const int32_t* faces, int64_t nf, int flags,
                      rt_mesh** out) {
  if (!out || (nf > 0 && (!vertices || !faces)) || nv < 0 || nf < 0 || (flags & ~RT_MESH_BVH_GPU) != 0) {
    rt::set_error("rt_mesh_create: invalid arguments");
    return RT_EINVAL;
  }
  *out = nullptr;
  for (int64_t i = 0; i < 3 * nf; ++i) {
    if (faces[i] < 0 || faces[i] >= nv) {
      rt::set_error("rt_mesh_create: face index out of range");
      return RT_EINVAL;
    }
  }
  rt::DeviceGuard dg(device);
  RT_HIP(dg.err);
  // the permuted-corner table feeds the brute-force queries: environments of <= 192 faces
  // (staged in LDS) and receivers (read from HBM, rt_trace).  BVH environments read lcomp, so the
  // table (288 B/face) is skipped for meshes too large to serve as a brute-force receiver.
  const bool brute = nf <= RT_BRUTE_MAX_FACES;
  const bool want_perm = nf <= RT_PERM_MAX_FACES;
  std::vector<float> perm(want_perm ? (size_t)std::max<int64_t>(nf, 1) * 72 : 0, 0.0f);
  std::vector<float> nrm((size_t)std::max<int64_t>(nf, 1) * 4, 0.0f);
  std::vector<float> tri((size_t)std::max<int64_t>(nf, 1) * 9, 0.0f);
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t f = 0; f < nf; ++f) {
    const float* c[3] = {vertices + 3 * (int64_t)faces[3 * f], vertices + 3 * (int64_t)faces[3 * f + 1],
                         vertices + 3 * (int64_t)faces[3 * f + 2]};
    for (int v = 0; v < 3; ++v)
      for (int k = 0; k < 3; ++k) {
        tri[9 * f + 3 * v + k] = c[v][k];
        lo[k] = std::min(lo[k], (double)c[v][k]);
        hi[k] = std::max(hi[k], (double)c[v][k]);
      }
    for (int kz = 0; kz < 3 && want_perm; ++kz)
      for (int sw = 0; sw < 2; ++sw) {
        int kx = kz + 1;
        if (kx == 3) kx = 0;
        int ky = kx + 1;
        if (ky == 3) ky = 0;
        if (sw) std::swap(kx, ky);
        // (a0 a1 a2 b0)(b1 b2 c0 c1)(c2 0 0 0), component 0/1/2 = [kx]/[ky]/[kz]
        float* dst = perm.data() + 72 * f + 12 * (kz * 2 + sw);
        for (int v = 0; v < 3; ++v) {
          dst[3 * v + 0] = c[v][kx];
          dst[3 * v + 1] = c[v][ky];
          dst[3 * v + 2] = c[v][kz];
        }
        dst[9] = dst[10] = dst[11] = 0.0f;
      }
    // unit geometric normal: normalize(cross(q-p, r-p))   (warp mesh_query_ray normal)
    const float e1[3] = {c[1][0] - c[0][0], c[1][1] - c[0][1], c[1][2] - c[0][2]};
    const float e2[3] = {c[2][0] - c[0][0], c[2][1] - c[0][1], c[2][2] - c[0][2]};
    const float N[3] = {std::fmaf(e1[1], e2[2], -(e1[2] * e2[1])), std::fmaf(e1[2], e2[0], -(e1[0] * e2[2])),
                        std::fmaf(e1[0], e2[1], -(e1[1] * e2[0]))};
    const float len = std::sqrt(h_dot(N, N));
    for (int k = 0; k < 3; ++k) nrm[4 * f + k] = len > 0.0f ? N[k] / len : 0.0f;
  }
  rt_mesh* m = new rt_mesh();
  m->device = device;
  m->gen = rt::next_mesh_gen();
  m->nf = nf;
  // bounding sphere (double), padded so f32 rounding in the pre-test can never reject a hit
  double cen[3], rmax = 0.0, amax = 0.0;
  for (int k = 0; k < 3; ++k) cen[k] = nf > 0 ? 0.5 * (lo[k] + hi[k]) : 0.0;
  for (int64_t i = 0; i < 9 * nf; i += 3) {
    double d2 = 0;
    for (int k = 0; k < 3; ++k) {
      const double d = tri[i + k] - cen[k];
      d2 += d * d;
      amax = std::max(amax, std::fabs((double)tri[i + k]));
    }
    rmax = std::max(rmax, std::sqrt(d2));
  }
  for (int k = 0; k < 3; ++k) {
    m->center[k] = (float)cen[k];
    m->lo[k] = nf > 0 ? (float)lo[k] : 0.0f;
    m->hi[k] = nf > 0 ? (float)hi[k] : 0.0f;
  }
  m->radius = (float)(rmax * (1.0 + 1e-3) + 1e-5 * (1.0 + amax));
  hipError_t e = want_perm ? hipMalloc(&m->perm, perm.size() * sizeof(float)) : hipSuccess;
  if (e == hipSuccess) e = hipMalloc(&m->nrm, nrm.size() * sizeof(float));
  if (e == hipSuccess && want_perm)
    e = hipMemcpy(m->perm, perm.data(), perm.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(m->nrm, nrm.data(), nrm.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    rt_mesh_destroy(m);
    return rt::hip_fail(e, "rt_mesh_create upload");
  }
  if (!brute) {
    int rc = 1;
    if (flags & RT_MESH_BVH_GPU) rc = rt::build_bvh_gpu(m, tri);  // 1: too deep for the stack
    if (rc == 1) rc = rt::build_bvh(m, tri);
    if (!rc) rc = rt::pack_leaf_refs(m);
    if (!rc) rc = rt::build_wide(m);
    if (rc) {
      rt_mesh_destroy(m);
      return rc;
    }
  }
  *out = m;
  return RT_OK;
}

int rt_release_caches(void) {
  rt::release_trace_caches();
  return RT_OK;
}

int rt_mesh_destroy(rt_mesh* m) {
  if (!m) return RT_OK;
  rt::DeviceGuard dg(m->device);
  rt::forget_mesh_schedules(m->gen);
  if (m->perm) (void)hipFree(m->perm);
  if (m->nrm) (void)hipFree(m->nrm);
  if (m->nodes) (void)hipFree(m->nodes);
  if (m->leaves) (void)hipFree(m->leaves);
  if (m->lcomp) (void)hipFree(m->lcomp);
  if (m->wide) (void)hipFree(m->wide);
  delete m;
  return RT_OK;
}

int rt_mesh_info(const rt_mesh* m, int64_t* nf, float* bounds6, float* sphere4) {
  if (!m) {
    rt::set_error("rt_mesh_info: null mesh");
    return RT_EINVAL;
  }
  if (nf) *nf = m->nf;
  if (bounds6)
    for (int k = 0; k < 3; ++k) {
      bounds6[k] = m->lo[k];
      bounds6[3 + k] = m->hi[k];
    }
  if (sphere4) {
    for (int k = 0; k < 3; ++k) sphere4[k] = m->center[k];
    sphere4[3] = m->radius;
  }
  return RT_OK;
}

int rt_bvh_info(const rt_mesh* m, int64_t* info4) {
  if (!m || !info4) {
    rt::set_error("rt_bvh_info: null argument");
    return RT_EINVAL;
  }
  info4[0] = m->nnodes;
  info4[1] = m->nleaves;
  info4[2] = m->bvh_depth;
  info4[3] = m->bvh_max_leaf;
  return RT_OK;
}

int rt_trace(const rt_mesh* env, const float* tx_pos, const rt_mesh* rx, int max_bounces, int64_t ray_offset, int64_t n,
             float* traced, float* received, uint32_t* row_mask, int32_t* hit_kind, int32_t* hit_face, void* stream) {
  if (!env || !tx_pos || max_bounces < 0 || n < 0 || ray_offset < 0) {
    rt::set_error("rt_trace: invalid arguments");
    return RT_EINVAL;
  }
  if (rx && (rx->nf > RT_PERM_MAX_FACES || !rx->perm)) {
    rt::set_error("rt_trace: receiver mesh too large (max 65536 faces, queried by brute force)");
    return RT_EINVAL;
  }
  if (rx && rx->device != env->device) {
    rt::set_error("rt_trace: environment and receiver meshes live on different devices");
    return RT_EINVAL;
  }
  if (max_bounces == 0) return RT_OK;
  rt::DeviceGuard dg(env->device);
  RT_HIP(dg.err);
  return rt::launch_trace(env, tx_pos, rx, max_bounces, ray_offset, n, traced, received, row_mask, hit_kind, hit_face,
                          (hipStream_t)stream);
}

}  // extern "C"

// ------------------------------------------------------------------ self-test kernels (parity tests)
namespace {
__global__ void k_math(const float* x, int64_t n, float* out, int op) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  float s, c;
  switch (op) {
    case 0: out[i] = __builtin_sqrtf(v); break;
    case 1: out[i] = 1.0f / v; break;
    case 2: rt::sincos_rt(v, &s, &c); out[i] = s; break;
    case 3: rt::sincos_rt(v, &s, &c); out[i] = c; break;
    case 4: out[i] = rt::acos_rt(v); break;
    case 5: out[i] = x[i] / x[(i + 1) % n]; break;
    default: out[i] = v; break;
  }
}
__global__ void k_dirs(int64_t off, int64_t n, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float3 d = rt::ray_dir(off + i);
  out[3 * i] = d.x;
  out[3 * i + 1] = d.y;
  out[3 * i + 2] = d.z;
}
__global__ void k_query_bvh(rt::BvhView bv, const float* o, const float* d, int64_t n, float* t, int32_t* face) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float3 oo = make_float3(o[3 * i], o[3 * i + 1], o[3 * i + 2]);
  const float3 dd = make_float3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
  const rt::Shear s = rt::make_shear(oo, dd);
  const rt::Hit h = rt::bvh_query(bv, s, oo, dd);
  t[i] = h.face >= 0 ? h.t : __builtin_nanf("");
  face[i] = h.face;
}
__global__ void k_query(const float4* perm, int nf, const float* o, const float* d, int64_t n, float* t, int32_t* face) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float3 oo = make_float3(o[3 * i], o[3 * i + 1], o[3 * i + 2]);
  const float3 dd = make_float3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
  const rt::Shear s = rt::make_shear(oo, dd);
  rt::Hit h;
  rt::hit_init(h);
  for (int f = 0; f < nf; ++f) {
    float T, det;
    const float4* p = perm + f * 18 + s.kcase * 3;
    if (rt::tri_test(s, p[0], p[1], p[2].x, T, det)) rt::hit_consider(h, T, det, f);
  }
  t[i] = h.face >= 0 ? h.t : __builtin_nanf("");
  face[i] = h.face;
}
}  // namespace

extern "C" {
int rt_selftest_math(const float* x, int64_t n, float* out, int op, void* stream) {
  if (n <= 0) return RT_OK;
  hipLaunchKernelGGL(k_math, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n, out, op);
  RT_HIP(hipGetLastError());
  return RT_OK;
}
int rt_ray_dirs(int64_t ray_offset, int64_t n, float* out, void* stream) {
  if (n <= 0) return RT_OK;
  hipLaunchKernelGGL(k_dirs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ray_offset, n, out);
  RT_HIP(hipGetLastError());
  return RT_OK;
}
int rt_query(const rt_mesh* m, const float* o, const float* d, int64_t n, float* t, int32_t* face, void* stream) {
  if (!m || n < 0) {
    rt::set_error("rt_query: invalid arguments");
    return RT_EINVAL;
  }
  if (n == 0) return RT_OK;
  rt::DeviceGuard dg(m->device);
  RT_HIP(dg.err);
  if (m->nodes) {
    const rt::BvhView bv = rt::bvh_view(m);
    hipLaunchKernelGGL(k_query_bvh, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, bv, o, d, n,
                       t, face);
  } else {
    hipLaunchKernelGGL(k_query, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, m->perm,
                       (int)m->nf, o, d, n, t, face);
  }
  RT_HIP(hipGetLastError());
  return RT_OK;
}
}
