// os_sort_bench.hip -- stand-alone harness for the record sort planned to replace rocPRIM's Onesweep
// in the coverage reduction (DESIGN.md §9 "What is left, and the next step"); not part of librfrt.
//
// The sort: LSD radix over (u64 key, u64 value) pairs on the key's low `bits` bits (<= 48), digits
// of up to 12 bits (35-bit K5 keys in 3 passes where rocPRIM takes 4 of 10 bits), 4096-key tiles,
// one launch per pass with decoupled look-back between tiles, and ONE histogram launch for all
// passes.  Nothing is zeroed between sorts:
//   * every look-back state word carries the pass's 24-bit tag (another tag = "not published yet"),
//   * the tile counter only grows (the host passes the number of tiles issued before),
//   * the histogram kernel zeroes the other of two histogram buffers for the next sort.
// So a sort is 1 + P launches; rocPRIM's Onesweep is a fill, a histogram and a scan, then two fills
// and one sort launch per pass.  The look-back spin is bounded (kOsSpinLimit polls): a bug there ends
// the kernel with wrong output and an error count instead of a hung device.
//
// The harness checks the result bit for bit against rocPRIM's radix_sort_pairs (both are stable
// LSD sorts, so keys and values must agree exactly) and times both with HIP events.
// Keys: a fraction `hot` of the records falls on 4 keys in long runs (the transmitter cells of a
// coverage rank), the rest uniformly over `bits` bits.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/os_sort_bench.hip -o tools/os_sort_bench
//   timeout -k 10 60 tools/os_sort_bench [N=1048576] [bits=30] [hot=0.5]   (one JSON line)
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kOsThreads = 256, kOsItems = 16, kOsWaveItems = 64 * kOsItems, kOsTile = kOsThreads * kOsItems;
#ifndef OS_BITS
#define OS_BITS 12  // digit bits per pass (-DOS_BITS=8 / 10 for the narrower-digit variants)
#endif
constexpr int kOsMaxBits = OS_BITS, kOsMaxBins = 1 << kOsMaxBits, kOsMaxPasses = (48 + OS_BITS - 1) / OS_BITS;
constexpr uint64_t kOsAgg = 1ull << 38, kOsInc = 2ull << 38, kOsCount = (1ull << 38) - 1;
constexpr uint64_t kOsTagMask = ~(kOsInc | kOsAgg | kOsCount);
constexpr size_t kOsHistWords = (size_t)kOsMaxPasses * kOsMaxBins;  // u32 per histogram buffer
constexpr int kOsSpinLimit = 1 << 22;

// every pass's digit histogram (LDS per block, then one global add per nonzero bin); zeroes the
// other histogram buffer for the next sort
__global__ __launch_bounds__(256) void k_os_hist(const uint64_t* keys, int64_t n, int passes, int dbits, int end_bit,
                                                 uint32_t* hist, uint32_t* hist_next) {
  __shared__ uint32_t h[kOsMaxPasses * kOsMaxBins];
  for (int i = threadIdx.x; i < passes * kOsMaxBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    for (int p = 0; p < passes; ++p) {
      const int sh = p * dbits, nb = min(dbits, end_bit - sh);
      atomicAdd(&h[p * kOsMaxBins + (int)((k >> sh) & ((1ull << nb) - 1))], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * kOsMaxBins; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < kOsHistWords; i += (size_t)gridDim.x * blockDim.x)
    hist_next[i] = 0u;
}

// one LSD pass: stable ranks inside the tile (each wave ranks its 1024 keys in order, 64 at a time,
// the lanes with equal digits found by ballots), then per digit the tile's exclusive prefix over the
// tiles before it by decoupled look-back, then the scatter
__global__ __launch_bounds__(kOsThreads) void k_os_pass(const uint64_t* kin, const uint64_t* vin, uint64_t* kout,
                                                        uint64_t* vout, int64_t n, int shift, int nbits,
                                                        const uint32_t* ghist, uint64_t* states, uint64_t* tile_ctr,
                                                        uint64_t tile_base, uint64_t tag, unsigned* errors) {
  __shared__ uint16_t wc[4][kOsMaxBins];
  __shared__ uint32_t dbase[kOsMaxBins];
  __shared__ uint32_t part[kOsThreads];
  __shared__ uint32_t s_tile;
  const int B = 1 << nbits, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t mask = (uint64_t)B - 1;
  if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd((unsigned long long*)tile_ctr, 1ull) - tile_base);
  for (int d = threadIdx.x; d < B; d += kOsThreads) wc[0][d] = wc[1][d] = wc[2][d] = wc[3][d] = 0;
  // digit bases: exclusive scan of this pass's global histogram, B / 256 consecutive digits per thread
  const int per = (B + kOsThreads - 1) / kOsThreads, d0 = threadIdx.x * per;
  uint32_t acc = 0;
  for (int j = 0; j < per; ++j)
    if (d0 + j < B) acc += ghist[d0 + j];
  part[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {  // the 256 partial sums, 4 per lane of one wave
    uint32_t a[4], t = 0;
    for (int q = 0; q < 4; ++q) t += (a[q] = part[4 * threadIdx.x + q]);
    uint32_t x = t;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    uint32_t e = x - t;
    for (int q = 0; q < 4; ++q) {
      part[4 * threadIdx.x + q] = e;
      e += a[q];
    }
  }
  __syncthreads();
  {
    uint32_t e = part[threadIdx.x];
    for (int j = 0; j < per; ++j)
      if (d0 + j < B) {
        dbase[d0 + j] = e;
        e += ghist[d0 + j];
      }
  }
  const int64_t tile = s_tile;
  const int64_t base = tile * kOsTile + (int64_t)w * kOsWaveItems;
  uint64_t k[kOsItems], v[kOsItems];
  uint32_t r[kOsItems];
  const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const int64_t idx = base + i * 64 + lane;
    const bool valid = idx < n;
    k[i] = valid ? kin[idx] : 0;
    v[i] = valid ? vin[idx] : 0;
    const uint32_t d = (uint32_t)((k[i] >> shift) & mask);
    uint64_t m = __ballot(valid);
    for (int b = 0; b < nbits; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    // every lane reads its digit's count before the digit's lowest lane writes it (one wave: LDS
    // operations in program order)
    uint32_t prior = 0;
    if (valid) prior = wc[w][d];
    r[i] = prior + (uint32_t)__popcll(m & lt);
    if (valid && (m & lt) == 0) wc[w][d] = (uint16_t)(prior + (uint32_t)__popcll(m));
  }
  __syncthreads();
  // per digit: the waves' offsets inside the tile, the tile's count, its prefix over earlier tiles
  uint64_t* st = states + (size_t)tile * kOsMaxBins;
  for (int d = threadIdx.x; d < B; d += kOsThreads) {
    const uint32_t c0 = wc[0][d], c1 = wc[1][d], c2 = wc[2][d], c3 = wc[3][d];
    const uint32_t cnt = c0 + c1 + c2 + c3;
    wc[0][d] = 0;
    wc[1][d] = (uint16_t)c0;
    wc[2][d] = (uint16_t)(c0 + c1);
    wc[3][d] = (uint16_t)(c0 + c1 + c2);
    __hip_atomic_store(&st[d], tag | (tile == 0 ? kOsInc : kOsAgg) | cnt, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int d = threadIdx.x; d < B; d += kOsThreads) {
    uint64_t excl = 0;
    if (tile > 0) {
      int spins = 0;
      for (int64_t j = tile - 1; j >= 0;) {
        const uint64_t sv =
            __hip_atomic_load(&states[(size_t)j * kOsMaxBins + d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((sv & kOsTagMask) != tag) {  // not published yet
          if (++spins > kOsSpinLimit) {
            atomicAdd(errors, 1u);
            break;
          }
          continue;
        }
        excl += sv & kOsCount;
        if (sv & kOsInc) break;
        --j;
      }
      const uint64_t own = st[d] & kOsCount;
      __hip_atomic_store(&st[d], tag | kOsInc | (excl + own), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    dbase[d] += (uint32_t)excl;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const int64_t idx = base + i * 64 + lane;
    if (idx < n) {
      const uint32_t d = (uint32_t)((k[i] >> shift) & mask);
      const uint32_t pos = dbase[d] + wc[w][d] + r[i];
      if (pos < (uint32_t)n) {
        kout[pos] = k[i];
        vout[pos] = v[i];
      } else {
        atomicAdd(errors, 1u);
      }
    }
  }
}

struct OsSorter {
  int64_t cap = 0;
  uint64_t *tk = nullptr, *tv = nullptr, *states = nullptr, *aux = nullptr;  // aux: [tile counter | 2 histograms]
  unsigned* errors = nullptr;
  uint64_t tiles = 0, tag = 0;
  int flip = 0;
  void init(int64_t c) {
    cap = c;
    CK(hipMalloc(&tk, cap * 8));
    CK(hipMalloc(&tv, cap * 8));
    const size_t ns = (size_t)((cap + kOsTile - 1) / kOsTile) * kOsMaxBins;
    CK(hipMalloc(&states, ns * 8));
    CK(hipMemset(states, 0, ns * 8));
    CK(hipMalloc(&aux, 8 + 2 * kOsHistWords * 4));
    CK(hipMemset(aux, 0, 8 + 2 * kOsHistWords * 4));
    CK(hipMalloc(&errors, 4));
    CK(hipMemset(errors, 0, 4));
  }
  void sort(const uint64_t* kin, uint64_t* kout, const uint64_t* vin, uint64_t* vout, int64_t n, int end_bit,
            hipStream_t s) {
    const int passes = (end_bit + kOsMaxBits - 1) / kOsMaxBits;
    const int dbits = (end_bit + passes - 1) / passes;
    const int64_t ntiles = (n + kOsTile - 1) / kOsTile;
    uint32_t* h0 = reinterpret_cast<uint32_t*>(aux + 1);
    uint32_t* hist = h0 + (flip ? kOsHistWords : 0);
    uint32_t* hist_next = h0 + (flip ? 0 : kOsHistWords);
    flip ^= 1;
    const unsigned hblocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(n / 32768, 256));
    hipLaunchKernelGGL(k_os_hist, dim3(hblocks), dim3(256), 0, s, kin, n, passes, dbits, end_bit, hist, hist_next);
    const uint64_t* ki = kin;
    const uint64_t* vi = vin;
    for (int p = 0; p < passes; ++p) {
      const bool to_out = ((passes - 1 - p) & 1) == 0;  // the last pass writes kout / vout
      uint64_t* ko = to_out ? kout : tk;
      uint64_t* vo = to_out ? vout : tv;
      const int shift = p * dbits, nb = std::min(dbits, end_bit - shift);
      const uint64_t tg = (tag++ % 0xFFFFFEull + 1ull) << 40;
      hipLaunchKernelGGL(k_os_pass, dim3((unsigned)ntiles), dim3(kOsThreads), 0, s, ki, vi, ko, vo, n, shift, nb,
                         hist + (size_t)p * kOsMaxBins, states, aux, tiles, tg, errors);
      tiles += (uint64_t)ntiles;
      ki = ko;
      vi = vo;
    }
  }
};

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1048576;
  const int bits = argc > 2 ? atoi(argv[2]) : 30;
  const double hot = argc > 3 ? atof(argv[3]) : 0.5;
  if (n < 1 || n > (1ll << 30) || bits < 1 || bits > 48) {
    fprintf(stderr, "usage: os_sort_bench [N <= 2^30] [bits 1..48] [hot]\n");
    return 2;
  }
  std::mt19937_64 rng(42);
  const uint64_t km = bits == 64 ? ~0ull : ((1ull << bits) - 1);
  std::vector<uint64_t> hk(n), hv(n);
  uint64_t hot_keys[4];
  for (auto& x : hot_keys) x = rng() & km;
  for (int64_t i = 0; i < n; ++i) {
    const bool h = (double)(rng() >> 11) * (1.0 / 9007199254740992.0) < hot;
    hk[i] = h ? hot_keys[(i / 64) & 3] : (rng() & km);
    hv[i] = (uint64_t)i;
  }
  uint64_t *kin, *vin, *ko1, *vo1, *ko2, *vo2;
  for (uint64_t** p : {&kin, &vin, &ko1, &vo1, &ko2, &vo2}) CK(hipMalloc(p, n * 8));
  CK(hipMemcpy(kin, hk.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(vin, hv.data(), n * 8, hipMemcpyHostToDevice));
  size_t tb = 0;
  CK(rocprim::radix_sort_pairs(nullptr, tb, kin, ko1, vin, vo1, (unsigned)n, 0u, (unsigned)bits, 0));
  void* tmp;
  CK(hipMalloc(&tmp, tb));
  OsSorter os;
  os.init(n);
  hipStream_t s = 0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto fn) {
    for (int i = 0; i < 3; ++i) fn();
    CK(hipEventRecord(e0, s));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) fn();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1000.0 * ms / reps;
  };
  const double us_rocprim = timed([&] {
    size_t b = tb;
    CK(rocprim::radix_sort_pairs(tmp, b, kin, ko1, vin, vo1, (unsigned)n, 0u, (unsigned)bits, s));
  });
  const double us_os = timed([&] { os.sort(kin, ko2, vin, vo2, n, bits, s); });
  CK(hipDeviceSynchronize());
  unsigned errors = 0;
  CK(hipMemcpy(&errors, os.errors, 4, hipMemcpyDeviceToHost));
  std::vector<uint64_t> a(n), b(n), c(n), d(n);
  CK(hipMemcpy(a.data(), ko1, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), ko2, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), vo1, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(d.data(), vo2, n * 8, hipMemcpyDeviceToHost));
  const bool same = a == b && c == d;
  printf("{\"digit_bits\": %d, \"n\": %lld, \"bits\": %d, \"hot\": %.2f, \"passes\": %d, \"rocprim_us\": %.1f, \"os_us\": %.1f, "
         "\"bit_identical\": %s, \"spin_or_range_errors\": %u}\n",
         OS_BITS, (long long)n, bits, hot, (bits + kOsMaxBits - 1) / kOsMaxBits, us_rocprim, us_os, same ? "true" : "false",
         errors);
  return same && errors == 0 ? 0 : 1;
}
