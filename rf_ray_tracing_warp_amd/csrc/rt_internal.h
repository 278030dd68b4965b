// rt_internal.h -- host-side structures shared by the librfrt translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "rt_bvh.h"

// Device-resident triangle mesh (the object wp.Mesh is in the reference, tracer.py:24,30).
//
// HBM layout (all float4, 16-byte aligned):
//   perm  [nf][6][3]  corners of face f permuted for shear case kz*2+swap, packed
//                     (p0 p1 p2 q0)(q1 q2 r0 r1)(r2 0 0 0) with 0/1/2 = [kx]/[ky]/[kz]
//                     -- 288 B per face, read as 2x ds_read_b128 + ds_read_b32
//   nrm   [nf]        unit geometric normal normalize(cross(q-p, r-p)), w = 0
//   bvh nodes (optional, large meshes): see rt_bvh.h
struct rt_mesh {
  int device = 0;
  uint64_t gen = 0;  // process-unique id (caches key on it, never on the handle's address)
  int64_t nf = 0;
  float4* perm = nullptr;
  float4* nrm = nullptr;
  // bounding sphere (centre, conservative radius) and box, computed on the host in double
  float center[3] = {0, 0, 0};
  float radius = 0.0f;
  float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  // BVH (built when nf > RT_BRUTE_MAX_FACES), layout in rt_bvh.h
  float* nodes = nullptr;  // [nnodes][16]
  int* leaves = nullptr;   // [nleaves][2] (first, count)
  float* lcomp = nullptr;  // leaf-ordered compact faces: 3 float4 (a.xyz b.x)(b.yz c.xy)(c.z, face bits, 0, 0)
  float* wide = nullptr;   // [nwide][32] 4-wide nodes collapsed from `nodes` (bvh_wide.hip)
  int64_t nnodes = 0, nleaves = 0, nwide = 0;
  int bvh_depth = 0, bvh_max_leaf = 0, wide_stack = 0;
};

namespace rt {
void set_error(const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// Scoped device switch for the ABI entry points: the calling thread's current device (which
// PyTorch also uses) is restored on every return path, including error returns and calls made
// from Python finalisers (DeviceMesh/Coverage __del__).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int device) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != device) err = hipSetDevice(device);
    else if (err != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// Debug poison (rt_debug_poison): when >= 0, every coverage plan buffer and a large block of the
// default memory pool are filled with this byte before each run, so a read of memory the run did
// not write shows up as a changed result instead of depending on what ran before.
extern int g_poison;
// fill `bytes` of a fresh stream-ordered allocation with the poison byte and free it back into the
// pool (whose release threshold keeps it), so the next hipMallocAsync returns poisoned memory
int poison_pool(size_t bytes, hipStream_t s);
// keep freed blocks of the device's default memory pool across synchronizes (trace.hip)
void keep_pool_memory();
// Row order for tracing rays [ray_offset, ray_offset+n) of one burst (trace.hip): bands of |d.z|
// (kZBands, a power of two <= 256, the most nearly horizontal first), then the initial direction's
// cell.  Stream-ordered workspace returned in *ws (hipFreeAsync it after the consumer).
constexpr int kZBands = 16;  // K4 rt_trace 1037 / 945 / 915 / 928 / 976 us at 4 / 8 / 16 / 32 / 64 (r4z7, r4z8)
const int32_t* dir_order_banded(int64_t ray_offset, int64_t n, hipStream_t stream, void** ws);
// The same order, computed once per (device, ray_offset, n) and kept by the library (the rays of a
// burst depend on their ids only); ready on `stream` when it returns.  nullptr on failure.
const int32_t* dir_order_cached(int64_t ray_offset, int64_t n, hipStream_t stream);
// Sector shards of a burst of n_total rays (trace.hip): the burst sorted by the azimuth of the
// initial direction, cut into world * slices equal pieces, rank taking every world-th piece from
// piece rank; written to out[sector_ray_count(...)] as global ids in the banded order
int64_t sector_ray_count(int64_t n_total, int rank, int world, int slices);
int sector_ray_ids(int64_t n_total, int rank, int world, int slices, int32_t* out, hipStream_t stream);
// Device view of a mesh's BVH for rt::bvh_query
inline BvhView bvh_view(const rt_mesh* m) {
  return BvhView{(const float4*)m->nodes, (const int2*)m->leaves, (const float4*)m->lcomp, (int)m->nf,
                 (const float4*)m->wide};
}
// After either builder: copy each leaf child's (first, count) into its parent node (q3.z/q3.w,
// first << 3 | count), the form bvh_query reads (api.hip)
int pack_leaf_refs(rt_mesh* m);
// After pack_leaf_refs: the 4-wide copy of the tree that rt::bvh4_query traverses (bvh_wide.hip)
int build_wide(rt_mesh* m);
// A new process-unique mesh id (rt_mesh_create), and the eviction of rt_trace's cached chunk
// schedules of a mesh that is being destroyed (trace.hip)
uint64_t next_mesh_gen();
void forget_mesh_schedules(uint64_t gen);
void release_trace_caches();
// rt_trace's launch (trace.hip).  fused (rt_trace_cir, optional): the brute-force kernels finish
// the CIR step in their last block (rt_cir.h); *fused_done tells whether this launch did.
struct TraceCirFused;
int launch_trace(const rt_mesh* env, const float tx[3], const rt_mesh* rx, int B, int64_t ray_offset, int64_t n,
                 float* traced, float* received, uint32_t* mask, int32_t* hit_kind, int32_t* hit_face,
                 hipStream_t stream, const TraceCirFused* fused = nullptr, bool* fused_done = nullptr);
}  // namespace rt

#define RT_HIP(call)                                                   \
  do {                                                                 \
    hipError_t _e = (call);                                            \
    if (_e != hipSuccess) return rt::hip_fail(_e, #call);              \
  } while (0)

// faces at or below this count are traced by the brute-force LDS kernel (whole mesh in LDS)
#define RT_BRUTE_MAX_FACES 192
#define RT_PERM_MAX_FACES (1 << 16)  // largest mesh given the permuted table (receivers are brute-forced)
