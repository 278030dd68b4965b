// Stress test: hipcub DeviceRadixSort::SortPairs on (cell << 32 | bin) keys with ~0 sentinels,
// checked against std::stable_sort on the host (keys and the values paired with them).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 100;
  std::mt19937_64 rng(7);
  int bad = 0;
  for (int rep = 0; rep < reps; ++rep) {
    const int n = 100 + (int)(rng() % 5000);
    const int cells = 1 + (int)(rng() % 200);
    std::vector<uint64_t> k(n);
    std::vector<double> v(n);
    for (int i = 0; i < n; ++i) {
      if (rng() % 8 == 0) k[i] = ~0ull;
      else k[i] = ((uint64_t)(rng() % cells) << 32) | (rng() % 20000);
      v[i] = (double)i + 0.25;
    }
    int cb = 0;
    while ((1ull << cb) < (uint64_t)cells) ++cb;
    for (int endbit : {32 + cb, 64}) {
      uint64_t *dk, *dko;
      double *dv, *dvo;
      hipMalloc(&dk, n * 8); hipMalloc(&dko, n * 8); hipMalloc(&dv, n * 8); hipMalloc(&dvo, n * 8);
      hipMemcpy(dk, k.data(), n * 8, hipMemcpyHostToDevice);
      hipMemcpy(dv, v.data(), n * 8, hipMemcpyHostToDevice);
      size_t tb = 0;
      hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dko, dv, dvo, n, 0, 64);
      void* tmp;
      hipMalloc(&tmp, tb);
      hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dko, dv, dvo, n, 0, endbit);
      std::vector<uint64_t> ko(n);
      std::vector<double> vo(n);
      hipMemcpy(ko.data(), dko, n * 8, hipMemcpyDeviceToHost);
      hipMemcpy(vo.data(), dvo, n * 8, hipMemcpyDeviceToHost);
      std::vector<int> idx(n);
      std::iota(idx.begin(), idx.end(), 0);
      const uint64_t mask = endbit >= 64 ? ~0ull : ((1ull << endbit) - 1);
      std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return (k[a] & mask) < (k[b] & mask); });
      int wrong = 0;
      for (int i = 0; i < n; ++i)
        if (ko[i] != k[idx[i]] || vo[i] != v[idx[i]]) ++wrong;
      if (wrong || e != hipSuccess) {
        ++bad;
        printf("rep %d n %d endbit %d: %d wrong (err %d)\n", rep, n, endbit, wrong, (int)e);
      }
      hipFree(dk); hipFree(dko); hipFree(dv); hipFree(dvo); hipFree(tmp);
    }
  }
  printf("sort_stress: %d bad of %d\n", bad, 2 * reps);
  return bad ? 1 : 0;
}
