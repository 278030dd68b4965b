// hash_bench.hip -- micro-benchmark behind the coverage reduction design: how fast
// does MI355X aggregate N (key, amplitude) records exactly?
//   sort   : rocPRIM radix sort of (u64 key, f64 value) pairs on the key's low `bits` bits (the
//            round-2 pipeline's first step, before its run sums)
//   insert : open-addressing hash, one returning 64-bit CAS per probe, then the amplitude as 32-bit
//            limbs added with no-return 64-bit atomics (2-3 per record)
//   cas    : the insert's CAS probes alone
//   scatter: plain 8-B stores to the same random slots (the memory system's floor for this pattern)
//   flush  : scan of the key array (what every consumer of the table pays)
// Keys: a fraction `hot` of the records falls on 4*66 "transmitter cell" keys in runs of 64 (as the
// replay emits them), the rest uniformly on U = N / 5 keys.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/hash_bench.hip -o tools/hash_bench
//   tools/hash_bench [N=1048576] [hot=0.5]
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr unsigned long long kEmpty = ~0ull;

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void k_insert(const uint64_t* keys, const double* amps, int64_t n, unsigned long long* tkey,
                         unsigned long long* tacc, uint64_t mask, int limbs, unsigned* overflow) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    uint64_t slot = mix(k) & mask;
    int probe = 0;
    for (; probe < 4096; ++probe) {
      const unsigned long long old = atomicCAS(tkey + slot, kEmpty, (unsigned long long)k);
      if (old == kEmpty || old == k) break;
      slot = (slot + 1) & mask;
    }
    if (probe == 4096) {
      atomicOr(overflow, 1u);
      continue;
    }
    if (limbs > 0) {
      // amplitude -> 53-bit mantissa at bit offset sh of the 2^-136 fixed point; 32-bit limbs
      const double a = amps[i];
      uint64_t bits;
      memcpy(&bits, &a, 8);
      const int e = (int)(bits >> 52) & 0x7ff;
      const uint64_t m = (bits & ((1ull << 52) - 1)) | (1ull << 52);
      const int sh = e - 939;
      const int l0 = sh >> 5, b = sh & 31;
      const uint64_t lo = m << b;                     // bits [32 l0, 32 l0 + 64)
      const uint64_t hi = b ? m >> (64 - b) : 0;      // bits above
      unsigned long long* acc = tacc + slot * 8;
      atomicAdd(acc + l0, lo & 0xffffffffull);
      atomicAdd(acc + l0 + 1, lo >> 32);
      if (hi) atomicAdd(acc + l0 + 2, hi);
    }
  }
}

__global__ void k_scatter(const uint64_t* keys, int64_t n, unsigned long long* tkey, uint64_t mask) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    tkey[mix(k) & mask] = k;
  }
}

__global__ void k_flush(const unsigned long long* tkey, int64_t cap, unsigned long long* out) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
    c += tkey[i] != kEmpty;
  for (int o = 32; o >= 1; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 20);
  const double hot = argc > 2 ? atof(argv[2]) : 0.5;
  const int64_t U = std::max<int64_t>(n / 5, 1);
  std::mt19937_64 rng(7);
  std::vector<uint64_t> hk(n);
  std::vector<double> ha(n);
  int64_t i = 0;
  while (i < n) {
    if (std::uniform_real_distribution<double>(0, 1)(rng) < hot) {  // a run of 64 hot records
      for (int j = 0; j < 64 && i < n; ++j, ++i) hk[i] = (uint64_t)(rng() % 264) * 7919 + 3;
    } else {
      hk[i++] = (uint64_t)(rng() % U) * 104729 + 1000003;
    }
  }
  std::lognormal_distribution<double> ld(-14.0, 2.0);
  for (auto& a : ha) a = std::min(ld(rng), 1.0);
  uint64_t *dk, *dks;
  double *da, *das;
  CK(hipMalloc(&dk, n * 8));
  CK(hipMalloc(&dks, n * 8));
  CK(hipMalloc(&da, n * 8));
  CK(hipMalloc(&das, n * 8));
  CK(hipMemcpy(dk, hk.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(da, ha.data(), n * 8, hipMemcpyHostToDevice));
  int64_t cap = 1;
  while (cap < 2 * n) cap <<= 1;
  unsigned long long *tkey, *tacc, *cnt;
  unsigned* ovf;
  CK(hipMalloc(&tkey, cap * 8));
  CK(hipMalloc(&tacc, cap * 64));
  CK(hipMalloc(&cnt, 8));
  CK(hipMalloc(&ovf, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto&& body, auto&& reset) {
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      reset();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      body();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    printf("{\"n\": %lld, \"hot\": %.2f, \"cap\": %lld, \"what\": \"%s\", \"us\": %.1f}\n", (long long)n, hot,
           (long long)cap, name, best * 1e3f);
  };
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  auto reset_table = [&] {
    CK(hipMemsetAsync(tkey, 0xFF, cap * 8));
    CK(hipMemsetAsync(tacc, 0, cap * 64));
    CK(hipMemsetAsync(ovf, 0, 4));
  };
  timeit("insert (CAS + 2-3 limb atomics)",
         [&] { hipLaunchKernelGGL(k_insert, dim3(grid), dim3(256), 0, 0, dk, da, n, tkey, tacc, cap - 1, 1, ovf); },
         reset_table);
  timeit("cas only", [&] { hipLaunchKernelGGL(k_insert, dim3(grid), dim3(256), 0, 0, dk, da, n, tkey, tacc, cap - 1, 0, ovf); },
         reset_table);
  timeit("scatter (plain 8-B stores)",
         [&] { hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(256), 0, 0, dk, n, tkey, cap - 1); }, reset_table);
  timeit("flush scan of the key array",
         [&] { hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, tkey, cap, cnt); }, [&] {});
  for (int bits : {31, 36, 57}) {
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, dk, dks, da, das, (unsigned)n, 0u, (unsigned)bits, 0));
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    char name[64];
    snprintf(name, sizeof name, "rocprim radix_sort_pairs u64/f64, %d bits", bits);
    timeit(name, [&] { CK(rocprim::radix_sort_pairs(tmp, tb, dk, dks, da, das, (unsigned)n, 0u, (unsigned)bits, 0)); },
           [&] {});
    CK(hipFree(tmp));
  }
  unsigned ov = 0;
  CK(hipMemcpy(&ov, ovf, 4, hipMemcpyDeviceToHost));
  if (ov) printf("overflow!\n");
  return 0;
}
