// cir.hip -- the host tail of Tracer.compute_cir (tracer.py:84-117) on the device.
//
//   rt_compact : row_mask -> ray ids of received rows in ray-id order (tracer.py:87)
//                3 kernels: per-tile counts, one-block exclusive scan, ordered scatter.
//   rt_cir     : per received row, the NaN strip (tracer.py:90-97), Fresnel product over the
//                interior vertices (tracer.py:106-111, _bounce_amplitude :34-61), float32 path
//                length and delay bin (tracer.py:112-115, NumPy 2 / NEP 50 semantics), then
//                impulse_response[bin] += amplitude (tracer.py:116-117).
//
// Exactness: the bin is computed with the reference's exact float32 operation sequence
// (np.dot on float32 = f32-rounded products summed in double, rounded once; norm = sqrtf of
// it), so bins match bit for bit.  The amplitude uses double acos/sin/asin/cos where the
// reference uses NumPy's float32 arccos and Python's math: agreement ~1e-7 relative.
// Accumulation is deterministic and in the reference's order: k_cir writes every path's (bin,
// amplitude) in ray order, then one workgroup applies impulse_response[bin] += amplitude chunk by
// chunk, each bin's additions by a single lane in ray order (tracer.py:116-117 exactly; a double
// atomic add gave run-to-run different last bits for bins with several paths).
#include <math.h>

#include <algorithm>

#include "../../include/rfrt.h"
#include "rt_cir.h"
#include "rt_internal.h"

namespace {

rt::CirConsts cir_consts(double amp0, double light_speed, double sample_rate, int flags, int64_t n_bins) {
  rt::CirConsts k;
  k.amp0 = amp0;
  k.c32 = (float)light_speed;
  k.fs32 = (float)sample_rate;
  k.c64 = light_speed;
  k.fs64 = sample_rate;
  k.flags = flags;
  k.n_bins = n_bins;
  return k;
}

constexpr int TILE = 2048;  // flags per compaction tile (256 threads x 8)

__global__ __launch_bounds__(256) void k_count(const uint32_t* mask, int64_t n, int64_t* tile_count) {
  __shared__ int wsum[4];
  const int64_t base = (int64_t)blockIdx.x * TILE;
  int c = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    c += (i < n && mask[i] != 0u) ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_count[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(1024) void k_scan(int64_t* tile_count, int64_t ntiles, int64_t* total) {
  // single block exclusive scan, in place, chunks of 1024
  __shared__ int64_t buf[1024];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < ntiles; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < ntiles ? tile_count[i] : 0;
    buf[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int64_t add = threadIdx.x >= (unsigned)o ? buf[threadIdx.x - o] : 0;
      __syncthreads();
      buf[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < ntiles) tile_count[i] = carry + buf[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += buf[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void k_scatter(const uint32_t* mask, int64_t n, const int64_t* tile_off,
                                                 int64_t* out_index) {
  __shared__ int wbase[4];
  const int64_t base = (int64_t)blockIdx.x * TILE;
  int64_t run = tile_off[blockIdx.x];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < 8; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    const bool f = i < n && mask[i] != 0u;
    const unsigned long long bal = __ballot(f);
    const int wc = __popcll(bal);
    if (lane == 0) wbase[w] = wc;
    __syncthreads();
    int before = 0;
    for (int j = 0; j < w; ++j) before += wbase[j];
    const int total = wbase[0] + wbase[1] + wbase[2] + wbase[3];
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    if (f) out_index[run + before + rank] = i;
    run += total;
    __syncthreads();
  }
}

// Scatter with the scan folded in, for up to kFusedTiles tiles: each block sums the counts of the
// tiles before it (at most a few KB, L2-resident) instead of waiting for a separate scan kernel; the
// last block writes the total.  Tiles without a flag return before touching the mask again.
constexpr int64_t kFusedTiles = 1024;
__global__ __launch_bounds__(256) void k_scatter_fused(const uint32_t* mask, int64_t n, const int64_t* tile_count,
                                                       int64_t ntiles, int64_t* out_index, int64_t* out_count) {
  __shared__ int64_t wpart[4];
  __shared__ int wbase[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t part = 0;
  for (int64_t j = threadIdx.x; j < (int64_t)blockIdx.x; j += 256) part += tile_count[j];
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if (lane == 0) wpart[w] = part;
  __syncthreads();
  int64_t run = wpart[0] + wpart[1] + wpart[2] + wpart[3];
  const int64_t mine = tile_count[blockIdx.x];
  if ((int64_t)blockIdx.x == ntiles - 1 && threadIdx.x == 0) *out_count = run + mine;
  if (mine == 0) return;  // uniform over the block
  const int64_t base = (int64_t)blockIdx.x * TILE;
  for (int k = 0; k < 8; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    const bool f = i < n && mask[i] != 0u;
    const unsigned long long bal = __ballot(f);
    const int wc = __popcll(bal);
    if (lane == 0) wbase[w] = wc;
    __syncthreads();
    int before = 0;
    for (int j = 0; j < w; ++j) before += wbase[j];
    const int total = wbase[0] + wbase[1] + wbase[2] + wbase[3];
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    if (f) out_index[run + before + rank] = i;
    run += total;
    __syncthreads();
  }
}

__device__ __forceinline__ void cir_one(const float* received, const int64_t* index, int64_t k, int P,
                                        const rt::CirConsts& kc, int32_t* out_bin, double* out_amp) {
  rt::cir_row(received + index[k] * (int64_t)(P * 3), P, kc, out_bin ? out_bin + k : nullptr,
              out_amp ? out_amp + k : nullptr);
}

__global__ __launch_bounds__(256) void k_cir(const float* received, const int64_t* index, const int64_t* count,
                                             int P, rt::CirConsts kc, int32_t* out_bin, double* out_amp) {
  const int64_t cnt = *count;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += (int64_t)gridDim.x * blockDim.x)
    cir_one(received, index, k, P, kc, out_bin, out_amp);
}

// impulse_response[bin] += amp for paths k = 0 .. count-1 in order (tracer.py:116-117): chunks of
// 1024 paths; in a chunk the first lane of each distinct bin adds that bin's amplitudes in path
// order (bins of different lanes are distinct, so no two lanes touch one bin)
__global__ __launch_bounds__(1024) void k_cir_accum(const int32_t* bins, const double* amps, const int64_t* count,
                                                    int64_t n_bins, double* ir) {
  __shared__ int32_t sb[1024];
  __shared__ double sa[1024];
  const int64_t cnt = *count;
  const int t = threadIdx.x;
  for (int64_t base = 0; base < cnt; base += 1024) {
    const int64_t k = base + t;
    const int32_t b = k < cnt ? bins[k] : -1;
    sb[t] = (b >= 0 && b < n_bins) ? b : -1;
    sa[t] = k < cnt ? amps[k] : 0.0;
    __syncthreads();
    const int32_t mb = sb[t];
    if (mb >= 0) {
      bool leader = true;
      for (int j = 0; j < t && leader; ++j) leader = sb[j] != mb;
      if (leader) {
        const int m = (int)(cnt - base < 1024 ? cnt - base : 1024);
        double v = ir[mb];
        for (int j = t; j < m; ++j)
          if (sb[j] == mb) v += sa[j];
        ir[mb] = v;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ fused compaction + CIR (rt_trace_cir)
// K2's step after the trace kernel was five launches of a few microseconds each (count, scatter,
// per-path CIR, ordered accumulation, impulse-response zeroing) for ~1 received row per 1M rays.
// Brute-force meshes: the trace kernel itself finishes the step (trace.hip, fused tail): it lists
// each 256-row chunk's received rows as it goes, and its last block to finish compacts them in
// order and accumulates the impulse response.  BVH meshes trace in direction-sorted order, so
// k_chunk_counts counts each chunk's rows from the mask and ONE launch of kFusedBlocks blocks does
// the rest:
//   block b owns chunks [b*C, (b+1)*C): the rows before them (a block reduction of the counts),
//   its chunks' offsets (an LDS scan), the ordered indices of its received rows (wave ballots),
//   and each of those rows' (bin, amplitude) -- computed by the lane that found the row;
//   the last block to finish (an agent-scope release by every block with rows, one atomic ticket)
//   zeroes the impulse response and adds the amplitudes in path order (tracer.py:116-117).
// Both leave the workspace's chunk counts zero and its ticket reset for the next call.
constexpr int kFusedBlocks = 64;
constexpr int kChunk = (int)rt::kCirChunk;

// received rows of every 256-row chunk from the mask (BVH / generic kernels, which do not count)
__global__ __launch_bounds__(256) void k_chunk_counts(const uint32_t* mask, int64_t n, int32_t* counts) {
  __shared__ int32_t w4[4];
  for (int64_t ch = blockIdx.x; ch * kChunk < n; ch += gridDim.x) {
    const int64_t i = ch * kChunk + threadIdx.x;
    const uint64_t m = __ballot(i < n && mask[i] != 0u);
    if ((threadIdx.x & 63) == 0) w4[threadIdx.x >> 6] = (int32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) counts[ch] = w4[0] + w4[1] + w4[2] + w4[3];
    __syncthreads();
  }
}

__device__ __forceinline__ int64_t block_sum_i64(int64_t v, int64_t* red) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const int64_t t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

struct CirArgs {
  const uint32_t* mask;
  int32_t* counts;
  int64_t nchunks, n, cpb;  // cpb: chunks per block (<= kFusedMaxCpb)
  const float* received;
  int P;
  rt::CirConsts k;
  double* ir;
  int64_t* index;
  int64_t* count;
  int32_t* pbin;
  double* pamp;
  unsigned* done;
};
constexpr int kFusedMaxCpb = (int)(rt::kCirMaxChunks / kFusedBlocks);  // up to 2^25 rows per call

__global__ __launch_bounds__(256) void k_compact_cir(CirArgs a) {
  __shared__ int32_t off[kFusedMaxCpb];
  __shared__ int64_t red[4];
  __shared__ int32_t wofs[4];
  __shared__ bool last;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * a.cpb;
  const int64_t c1 = c0 + a.cpb < a.nchunks ? c0 + a.cpb : a.nchunks;
  // rows received before this block's chunks
  int64_t before = 0;
#pragma unroll 8
  for (int64_t j = t; j < c0 && j < a.nchunks; j += 256) before += a.counts[j];
  const int64_t base = block_sum_i64(before, red);
  // exclusive scan of this block's chunk counts (serial over <= 2048 entries by thread 0 after a
  // parallel load: the counts are almost all zero and the block has little else to do)
  const int m = c1 > c0 ? (int)(c1 - c0) : 0;
  for (int j = t; j < m; j += 256) off[j] = a.counts[c0 + j];
  __syncthreads();
  __shared__ int32_t btotal;
  if (t == 0) {
    int32_t acc = 0;
    for (int j = 0; j < m; ++j) {
      const int32_t c = off[j];
      off[j] = acc;
      acc += c;
    }
    btotal = acc;
  }
  __syncthreads();
  for (int j = 0; j < m; ++j) {
    const int64_t ch = c0 + j;
    if ((j + 1 < m ? off[j + 1] : btotal) == off[j]) continue;  // block-uniform: no received row
    const int64_t i = ch * kChunk + t;
    const bool got = i < a.n && a.mask[i] != 0u;
    const uint64_t bm = __ballot(got);
    if (lane == 0) wofs[w] = (int32_t)__popcll(bm);
    __syncthreads();
    int32_t pre = 0;
    for (int q = 0; q < w; ++q) pre += wofs[q];
    __syncthreads();
    if (got) {
      const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
      const int64_t k = base + off[j] + pre + rank;
      a.index[k] = i;
      cir_one(a.received, a.index, k, a.P, a.k, a.pbin, a.pamp);
    }
  }
  // publish, then the last block accumulates.  Only blocks that wrote rows release them: an
  // agent-scope release writes back the XCD's whole L2, full of the trace kernel's dirty rows
  // (64 releases took the launch from ~5 to 18 us on K2, where ~1 block has a received row).
  if (btotal > 0) __threadfence();
  __syncthreads();
  if (t == 0) last = atomicAdd(a.done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  int64_t tot = 0;
  for (int64_t j = t; j < a.nchunks; j += 256) {
    tot += a.counts[j];
    a.counts[j] = 0;  // every block has read its counts (ticket): leave them zero for the next call
  }
  const int64_t cnt = block_sum_i64(tot, red);
  if (t == 0) {
    *a.count = cnt;
    *a.done = 0u;  // ready for the next call on this workspace
  }
  if (a.ir) rt::ir_accumulate_block(a.pbin, a.pamp, cnt, a.k.n_bins, a.ir);
}

}  // namespace

extern "C" {

int64_t rt_compact_workspace_bytes(int64_t n) { return (int64_t)(((n + TILE - 1) / TILE) + 1) * 8; }

int rt_compact(const uint32_t* row_mask, int64_t n, void* workspace, int64_t workspace_bytes, int64_t* out_index,
               int64_t* out_count, void* stream) {
  if (n < 0 || !out_count || (n > 0 && (!row_mask || !out_index || !workspace))) {
    rt::set_error("rt_compact: invalid arguments");
    return RT_EINVAL;
  }
  const int64_t ntiles = (n + TILE - 1) / TILE;
  if (workspace_bytes < rt_compact_workspace_bytes(n)) {
    rt::set_error("rt_compact: workspace too small");
    return RT_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    RT_HIP(hipMemsetAsync(out_count, 0, 8, s));
    return RT_OK;
  }
  int64_t* tiles = (int64_t*)workspace;
  hipLaunchKernelGGL(k_count, dim3((unsigned)ntiles), dim3(256), 0, s, row_mask, n, tiles);
  if (ntiles <= kFusedTiles) {  // up to 2M rows: two launches
    hipLaunchKernelGGL(k_scatter_fused, dim3((unsigned)ntiles), dim3(256), 0, s, row_mask, n, tiles, ntiles,
                       out_index, out_count);
  } else {  // the folded prefix would re-read O(ntiles^2) counts: separate scan
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, tiles, ntiles, out_count);
    hipLaunchKernelGGL(k_scatter, dim3((unsigned)ntiles), dim3(256), 0, s, row_mask, n, tiles, out_index);
  }
  RT_HIP(hipGetLastError());
  return RT_OK;
}

int64_t rt_trace_cir_workspace_bytes(int64_t n) {
  // ticket, chunk counts (fixed size), per-path amplitudes + bins, row within chunk; see rt_cir.h
  return rt::kCirAmpOff + (n > 0 ? n : 0) * 24 + 64;
}

int rt_cir(const float* received, const int64_t* index, const int64_t* count, int64_t max_count, int max_bounces,
           double amp0, double light_speed, double sample_rate, int flags, int64_t n_bins, double* impulse_response,
           int32_t* out_bin, double* out_amp, void* stream) {
  if (!received || !index || !count || max_count < 0 || max_bounces < 1 || n_bins < 0) {
    rt::set_error("rt_cir: invalid arguments");
    return RT_EINVAL;
  }
  if (max_count == 0) return RT_OK;
  hipStream_t s = (hipStream_t)stream;
  // per-path (bin, amplitude): the caller's diagnostic outputs, or stream-ordered pool scratch
  void* scratch = nullptr;
  int32_t* bins = out_bin;
  double* amps = out_amp;
  if (impulse_response && (!bins || !amps)) {
    rt::keep_pool_memory();
    RT_HIP(hipMallocAsync(&scratch, (size_t)max_count * 12 + 16, s));
    if (!amps) amps = (double*)scratch;
    if (!bins) bins = (int32_t*)((char*)scratch + (size_t)max_count * 8);
  }
  // the count is on the device and usually tiny (K2: ~1 row per 1M rays): one block per CU, a
  // grid-stride loop covers larger counts; empty blocks cost launch time, not work
  const int64_t want = (max_count + 255) / 256;
  const unsigned grid = (unsigned)(want < 256 ? want : 256);
  hipLaunchKernelGGL(k_cir, dim3(grid), dim3(256), 0, s, received, index, count, max_bounces + 1,
                     cir_consts(amp0, light_speed, sample_rate, flags, n_bins), bins, amps);
  if (impulse_response)
    hipLaunchKernelGGL(k_cir_accum, dim3(1), dim3(1024), 0, s, bins, amps, count, n_bins, impulse_response);
  RT_HIP(hipGetLastError());
  if (scratch) RT_HIP(hipFreeAsync(scratch, s));
  return RT_OK;
}


}  // extern "C"


extern "C" int rt_trace_cir(const rt_mesh* env, const float* tx_pos, const rt_mesh* rx, int max_bounces,
                            int64_t ray_offset, int64_t n, float* traced, float* received, uint32_t* row_mask,
                            double amp0, double light_speed, double sample_rate, int flags, int64_t n_bins,
                            double* impulse_response, int64_t* out_index, int64_t* out_count, void* workspace,
                            int64_t workspace_bytes, void* stream) {
  if (!env || !tx_pos || max_bounces < 1 || n < 0 || ray_offset < 0 || !received || !row_mask || !out_index ||
      !out_count || n_bins < 0 || (n_bins > 0 && !impulse_response) || !workspace) {
    rt::set_error("rt_trace_cir: invalid arguments");
    return RT_EINVAL;
  }
  if (workspace_bytes < rt_trace_cir_workspace_bytes(n) || ((uintptr_t)workspace & 7)) {
    rt::set_error("rt_trace_cir: workspace too small or misaligned (rt_trace_cir_workspace_bytes, 8-B aligned)");
    return RT_EINVAL;
  }
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const int64_t cpb = (nch + kFusedBlocks - 1) / kFusedBlocks;
  if (nch > rt::kCirMaxChunks || cpb > kFusedMaxCpb) {
    rt::set_error("rt_trace_cir: more than 2^25 rays per call; shard the burst");
    return RT_EINVAL;
  }
  if (rx && (rx->nf > RT_PERM_MAX_FACES || !rx->perm || rx->device != env->device)) {
    rt::set_error("rt_trace_cir: receiver mesh too large or on another device");
    return RT_EINVAL;
  }
  rt::DeviceGuard dg(env->device);
  RT_HIP(dg.err);
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    RT_HIP(hipMemsetAsync(out_count, 0, 8, s));
    if (n_bins > 0) RT_HIP(hipMemsetAsync(impulse_response, 0, n_bins * 8, s));
    return RT_OK;
  }
  // workspace (rt_cir.h): zero on entry -- the caller zero-fills it once, every call leaves the
  // ticket and the chunk counts zero again
  char* ws = (char*)workspace;
  rt::TraceCirFused fz;
  fz.done = (unsigned*)ws;
  fz.counts = (int32_t*)(ws + rt::kCirCountsOff);
  fz.pamp = (double*)(ws + rt::kCirAmpOff);
  fz.pbin = (int32_t*)(fz.pamp + n);
  fz.masks = (uint64_t*)(ws + rt::kCirMasksOff);
  fz.gcounts = (int32_t*)(ws + rt::kCirGroupCountsOff);
  fz.camp = (double*)(ws + rt::kCirAmpOff + ((n * 12 + 7) / 8) * 8);
  fz.cbin = (int32_t*)(fz.camp + n);
  fz.index = out_index;
  fz.count = out_count;
  fz.ir = n_bins > 0 ? impulse_response : nullptr;
  fz.k = cir_consts(amp0, light_speed, sample_rate, flags, n_bins);
  bool fused = false;
  int rc = rt::launch_trace(env, tx_pos, rx, max_bounces, ray_offset, n, traced, received, row_mask, nullptr, nullptr,
                            s, &fz, &fused);
  if (rc) return rc;
  if (fused) return RT_OK;  // the trace kernel and its tail kernel did the compaction and the CIR
  hipLaunchKernelGGL(k_chunk_counts, dim3((unsigned)std::min<int64_t>(nch, 4096)), dim3(256), 0, s, row_mask, n,
                     fz.counts);
  CirArgs a;
  a.mask = row_mask;
  a.counts = fz.counts;
  a.nchunks = nch;
  a.n = n;
  a.cpb = cpb;
  a.received = received;
  a.P = max_bounces + 1;
  a.k = fz.k;
  a.ir = fz.ir;
  a.index = out_index;
  a.count = out_count;
  a.pbin = fz.pbin;
  a.pamp = fz.pamp;
  a.done = fz.done;
  hipLaunchKernelGGL(k_compact_cir, dim3(kFusedBlocks), dim3(256), 0, s, a);
  RT_HIP(hipGetLastError());
  return RT_OK;
}
