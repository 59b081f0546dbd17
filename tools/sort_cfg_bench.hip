// rocPRIM onesweep configurations for the connecting-edge key sort
// (sort.hip): u64 keys on their 2*nb significant bits, at the sizes of the
// 128^3 headline's sorting steps (X = 2.17 M keys of 44 bits at step 14,
// 10.5 M of 46 bits at step 16).  Times each config with HIP events (median
// of 9) and checks the output against the default config's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o gpurun_out/sort_cfg tools/sort_cfg_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <rocprim/device/device_radix_sort.hpp>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

template <int BS, int IPT, int BITS>
using OneCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>, rocprim::kernel_config<BS, IPT>, BITS,
                                        rocprim::block_radix_rank_algorithm::match>,
    256 * 1024>;
using DefCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config,
                                          256 * 1024>;

template <class Cfg>
float run(const char* name, const uint64_t* src, uint64_t* a, uint64_t* b, size_t n, int bits,
          std::vector<uint64_t>* out) {
  size_t bytes = 0;
  rocprim::double_buffer<uint64_t> db0(a, b);
  CK(rocprim::radix_sort_keys<Cfg>(nullptr, bytes, db0, n, 0u, (unsigned)bits));
  void* scr = nullptr;
  CK(hipMalloc(&scr, bytes + 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  uint64_t* res = nullptr;
  for (int r = 0; r < 9; ++r) {
    CK(hipMemcpy(a, src, n * 8, hipMemcpyDeviceToDevice));
    rocprim::double_buffer<uint64_t> db(a, b);
    size_t bb = bytes;
    CK(hipEventRecord(e0));
    CK(rocprim::radix_sort_keys<Cfg>(scr, bb, db, n, 0u, (unsigned)bits));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms);
    res = db.current();
  }
  std::sort(t.begin(), t.end());
  std::vector<uint64_t> h(n);
  CK(hipMemcpy(h.data(), res, n * 8, hipMemcpyDeviceToHost));
  bool ok = true;
  if (out->empty())
    *out = h;
  else
    ok = (*out == h);
  printf("  %-28s n=%zu bits=%d  %.4f ms  %s\n", name, n, bits, t[4], ok ? "ok" : "MISMATCH");
  CK(hipFree(scr));
  return t[4];
}

int main() {
  const size_t sizes[2] = {2170351, 10549679};
  const int nbs[2] = {22, 23};
  for (int c = 0; c < 2; ++c) {
    const size_t n = sizes[c];
    const int nb = nbs[c];
    // unique (lo, hi) pairs, lo < hi < 2^nb, lo spread over the id range with
    // hi near lo (connecting edges join nearby vertices)
    std::mt19937_64 g(1234 + c);
    std::vector<uint64_t> k(n);
    const uint64_t NV = (1ull << nb) - 1000;
    for (size_t i = 0; i < n; ++i) {
      uint64_t lo = g() % (NV - 600);
      uint64_t hi = lo + 1 + g() % 512;
      k[i] = (lo << nb) | hi;
    }
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    std::shuffle(k.begin(), k.end(), g);
    const size_t m = k.size();
    uint64_t *src, *a, *b;
    CK(hipMalloc(&src, m * 8));
    CK(hipMalloc(&a, m * 8));
    CK(hipMalloc(&b, m * 8));
    CK(hipMemcpy(src, k.data(), m * 8, hipMemcpyHostToDevice));
    std::vector<uint64_t> ref;
    const int bits = 2 * nb;
    run<DefCfg>("default", src, a, b, m, bits, &ref);
    run<OneCfg<512, 12, 8>>("512x12 r8", src, a, b, m, bits, &ref);
    run<OneCfg<512, 16, 8>>("512x16 r8", src, a, b, m, bits, &ref);
    run<OneCfg<1024, 8, 8>>("1024x8 r8", src, a, b, m, bits, &ref);
    run<OneCfg<512, 12, 10>>("512x12 r10", src, a, b, m, bits, &ref);
    run<OneCfg<1024, 8, 10>>("1024x8 r10", src, a, b, m, bits, &ref);
    run<OneCfg<512, 16, 10>>("512x16 r10", src, a, b, m, bits, &ref);
    run<OneCfg<256, 16, 10>>("256x16 r10", src, a, b, m, bits, &ref);
    run<OneCfg<512, 12, 9>>("512x12 r9", src, a, b, m, bits, &ref);
    run<OneCfg<256, 12, 8>>("256x12 r8", src, a, b, m, bits, &ref);
    CK(hipFree(src));
    CK(hipFree(a));
    CK(hipFree(b));
  }
  return 0;
}
