// rt_cir.h -- per-path impulse-response arithmetic (tracer.py:84-117) shared by the compaction
// kernels (cir.hip) and the trace kernel's fused tail (trace.hip, rt_trace_cir).
//
// Exactness: the bin is computed with the reference's exact float32 operation sequence (np.dot on
// float32 = f32-rounded products summed in double, rounded once; norm = sqrtf of it), so bins
// match bit for bit.  The amplitude uses double acos/sin/asin/cos where the reference uses NumPy's
// float32 arccos and Python's math: agreement ~1e-7 relative.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/rfrt.h"

namespace rt {

// per-call constants of the CIR step (tracer.py:101-117)
struct CirConsts {
  double amp0;      // tx_power / n_rays
  float c32, fs32;  // light speed / sample rate as float32 (Python-float arguments, NEP 50)
  double c64, fs64;
  int flags;        // RT_CIR_C_F64 / RT_CIR_FS_F64: NumPy float64 scalars promote the delay to f64
  int64_t n_bins;
};

// np.dot(float32[3], float32[3]): f32 products, summed in double left to right, rounded once
__device__ __forceinline__ float npdot(const float* a, const float* b) {
  const float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2];
  return (float)(((double)p0 + (double)p1) + (double)p2);
}
__device__ __forceinline__ float npnorm(const float* a) { return sqrtf(npdot(a, a)); }

// Tracer._bounce_amplitude (tracer.py:34-61) for a float32 angle
__device__ __forceinline__ double bounce_amplitude(float angle) {
  if (isnan(angle)) return 0.0;
  const float theta32 = 1.57079637050628662109375f - angle / 2.0f;  // f32(pi/2) - angle/2 in f32
  const double theta = (double)theta32;
  const double theta_i = asin(sin(theta) / 5.0);
  const double num = cos(theta_i) - 5.0 * cos(theta);
  const double den = cos(theta_i) + 5.0 * cos(theta);
  const double q = num / den;
  double amp = -(q * q);
  if (amp < -1.0) amp = -1.0;
  if (isnan(amp)) return 0.0;
  return -amp;
}

// One received row of P points (tracer.py:87-115): NaN strip, Fresnel product over the interior
// vertices, float32 path length, delay bin (int() truncation, clamped to int32).
__device__ __forceinline__ void cir_row(const float* row, int P, const CirConsts& k, int32_t* bin_out,
                                        double* amp_out) {
  // tracer.py:90-97: cut at the first point with a NaN component
  int L = 0;
  while (L < P && !(isnan(row[3 * L]) || isnan(row[3 * L + 1]) || isnan(row[3 * L + 2]))) ++L;
  double amp = k.amp0;
  float dist = 0.0f;
  for (int j = 0; j + 2 < L; ++j) {
    const float* p1 = row + 3 * j;
    const float* p2 = p1 + 3;
    const float* p3 = p2 + 3;
    const float s1[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    const float s2[3] = {p3[0] - p2[0], p3[1] - p2[1], p3[2] - p2[2]};
    const float l1 = npnorm(s1);
    const float cosv = npdot(s1, s2) / (l1 * npnorm(s2));
    const float angle = (float)acos((double)cosv);
    amp *= bounce_amplitude(angle);
    dist += l1;
  }
  if (L >= 2) {
    const float* a = row + 3 * (L - 2);
    const float d[3] = {a[0] - a[3], a[1] - a[4], a[2] - a[5]};
    dist += npnorm(d);
  }
  // delay_samples = int((distance / light_speed_mps) * sample_rate_hz)   (tracer.py:115)
  double dl;
  if (k.flags & RT_CIR_C_F64) {
    const double q = (double)dist / k.c64;
    dl = q * k.fs64;
  } else {
    const float q = dist / k.c32;
    dl = (k.flags & RT_CIR_FS_F64) ? (double)q * k.fs64 : (double)(q * k.fs32);
  }
  const int64_t bin = (int64_t)dl;  // int() truncates toward zero
  if (bin_out) *bin_out = (int32_t)(bin < 2147483647 ? bin : 2147483647);
  if (amp_out) *amp_out = amp;
}

// One 256-thread block: ir[0 .. n_bins) = 0, then ir[bin] += amp for paths 0 .. cnt-1 in path order
// (tracer.py:116-117).  256 paths at a time; the first lane of each distinct bin adds that bin's
// amplitudes in path order, so no two lanes touch one bin and the result is order-exact.
__device__ __forceinline__ void ir_accumulate_block(const int32_t* pbin, const double* pamp, int64_t cnt,
                                                    int64_t n_bins, double* ir) {
  __shared__ int32_t sb[256];
  __shared__ double sa[256];
  const int t = threadIdx.x;
  for (int64_t b = t; b < n_bins; b += 256) ir[b] = 0.0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < cnt; b0 += 256) {
    const int64_t k = b0 + t;
    const int32_t bb = k < cnt ? pbin[k] : -1;
    sb[t] = (bb >= 0 && bb < n_bins) ? bb : -1;
    sa[t] = k < cnt ? pamp[k] : 0.0;
    __syncthreads();
    const int32_t mb = sb[t];
    if (mb >= 0) {
      bool leader = true;
      for (int j = 0; j < t && leader; ++j) leader = sb[j] != mb;
      if (leader) {
        const int mm = (int)(cnt - b0 < 256 ? cnt - b0 : 256);
        double v = b0 == 0 ? 0.0 : ir[mb];  // the first 256 paths add to the zeros just written
        for (int j = t; j < mm; ++j)
          if (sb[j] == mb) v += sa[j];
        ir[mb] = v;
      }
    }
    __syncthreads();
  }
}

// One wave (64 lanes), no block barriers: the same result as ir_accumulate_block, 64 paths at a
// time; a lane whose bin no earlier lane of the batch holds adds that bin's amplitudes in path
// order (through wave shuffles).
__device__ __forceinline__ void ir_accumulate_wave(const int32_t* pbin, const double* pamp, int64_t cnt,
                                                   int64_t n_bins, double* ir, bool zero = true) {
  const int lane = threadIdx.x & 63;
  if (zero)  // else the caller zeroed ir and synchronised
    for (int64_t b = lane; b < n_bins; b += 64) ir[b] = 0.0;
  for (int64_t b0 = 0; b0 < cnt; b0 += 64) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // this wave's earlier ir stores first
    const int64_t k = b0 + lane;
    const int32_t bb = k < cnt ? pbin[k] : -1;
    const int32_t mb = (bb >= 0 && bb < n_bins) ? bb : -1;
    const double am = k < cnt ? pamp[k] : 0.0;
    bool leader = mb >= 0;
    // wave-uniform trip counts (every lane takes part in the shuffles), only over this batch's
    // paths: each shuffle is a dependent LDS round trip, 2 x 64 of them took ~3 us for one path
    const int m = cnt - b0 < 64 ? (int)(cnt - b0) : 64;
    for (int j = 0; j < m; ++j) {
      const int32_t bj = __shfl(mb, j, 64);
      if (j < lane && bj == mb) leader = false;
    }
    double v = (leader && b0 > 0) ? ir[mb] : 0.0;  // the first 64 paths add to the zeros just written
    for (int j = 0; j < m; ++j) {
      const int32_t bj = __shfl(mb, j, 64);
      const double aj = __shfl(am, j, 64);
      if (j >= lane && bj == mb) v += aj;
    }
    if (leader) ir[mb] = v;
  }
}

// rt_trace_cir's workspace: [0, 64) done ticket | counts of received rows per 256-row chunk,
// kCirMaxChunks int32 | the same per group of 64 chunks | per chunk a 256-bit mask of its received rows, kCirMaxChunks x 4 u64 --
// both at fixed offsets and all zero between calls, whatever n the workspace was last used with |
// per path f64 amplitude [n] | per path int32 bin [n] (at the row's index when the trace kernel
// fills them, in path order otherwise) | the fused tail's path-ordered f64 amplitudes [n] and
// int32 bins [n]
constexpr int64_t kCirChunk = 256;
constexpr int64_t kCirMaxChunks = (int64_t)1 << 17;  // 2^25 rows per call
constexpr int64_t kCirCountsOff = 64;
constexpr int64_t kCirGroupCountsOff = kCirCountsOff + kCirMaxChunks * 4;  // per 64 chunks (fused tail)
constexpr int64_t kCirMasksOff = kCirGroupCountsOff + kCirMaxChunks / 64 * 4;
constexpr int64_t kCirAmpOff = kCirMasksOff + kCirMaxChunks * 32;

// The brute-force trace kernel's fused tail (trace.hip): set by rt_trace_cir, consumed by
// launch_trace when the kernel can count its chunks in row order
struct TraceCirFused {
  int32_t* counts;
  int32_t* gcounts;  // per 64 chunks
  double* pamp;
  int32_t* pbin;
  uint64_t* masks;
  double* camp;  // path order
  int32_t* cbin;
  unsigned* done;
  int64_t* index;
  int64_t* count;
  double* ir;  // null: no impulse response
  CirConsts k;
};

}  // namespace rt
