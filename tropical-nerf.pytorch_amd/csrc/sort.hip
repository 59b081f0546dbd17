// Radix sorts: (1) cell bucketing of (cell, member) entries; (2) packed u64 keys (connecting edges lo << nb | hi)
// on their 2*nb significant bits: the lexicographic order of
// c_new.sort(-1).unique(dim=0) (subpoly.py:243-244) -- the keys are already
// unique, one per canonical cell.  rocPRIM's onesweep radix sort is the
// primitive; only the significant bits are visited.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"
#include "step.h"

// rocPRIM sorts up to 1 M keys by block sort + merge passes (a dozen launches
// for 2 M keys); the connecting-edge keys go to onesweep above this size
#ifndef TNP_SORT_MERGE_LIMIT
#define TNP_SORT_MERGE_LIMIT (256 * 1024)
#endif
// onesweep in 1024-thread blocks of 8 keys per thread: 0.43 -> 0.40 ms per
// 128^3 pass against rocPRIM's gfx950 default (512 x 12); 1024 x 6 measured
// the same, 1024 x 12 and 768 x 8 slower (tools/sort_cfg_bench.hip, A/B in
// the engine)
using KeySortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 8,
                                        rocprim::block_radix_rank_algorithm::match>,
    TNP_SORT_MERGE_LIMIT>;

size_t sort_scratch_bytes(int64_t n, int bits) {
  size_t bytes = 0;
  rocprim::double_buffer<uint64_t> db(nullptr, nullptr);
  if (rocprim::radix_sort_keys<KeySortCfg>(nullptr, bytes, db, (size_t)std::max<int64_t>(n, 1), 0u,
                                           (unsigned)bits) != hipSuccess)
    return 0;
  return bytes;
}

int sort_keys_u64(uint64_t* a, uint64_t* b, int64_t n, int bits, void* scratch, size_t scratch_bytes,
                  uint64_t** out, hipStream_t s) {
  *out = a;
  if (n <= 1) return 0;
  rocprim::double_buffer<uint64_t> db(a, b);
  size_t bytes = scratch_bytes;
  TNP_CHECK(rocprim::radix_sort_keys<KeySortCfg>(scratch, bytes, db, (size_t)n, 0u, (unsigned)bits, s));
  *out = db.current();
  return 0;
}

// ---------------------------------------------------------------------------
// Lexicographic (lo, hi) order in two stages.  A connecting-edge key is
// lo << nb | hi, and a vertex is the lower end of only a few connecting
// edges: sorting the lo half alone (onesweep on bits [nb, 2nb): 3 digit
// passes instead of 6, each with its two look-back resets) leaves short runs
// of equal lo whose hi are in emission order; one pass then puts every key of
// a run of <= R keys at run start + its rank in the run (keys are unique).
// Longer runs (a vertex joined to many others in one region) are listed by
// their first key's thread and sorted by k_lex_long, one workgroup per run.
// ---------------------------------------------------------------------------
namespace {

constexpr int LX_BLOCK = 256;
constexpr int LX_RMAX = 256;  // longest run the pass ranks (R is clamped to it)
// a block's keys and R + 2 on either side in LDS (dynamic: LX_BLOCK + 2R + 4)
__global__ void __launch_bounds__(LX_BLOCK)
k_lex_runs(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, int64_t n, int nb, int R,
           int64_t* __restrict__ longs, unsigned long long* __restrict__ nlong) {
  extern __shared__ uint64_t win[];
  const int64_t base = (int64_t)blockIdx.x * LX_BLOCK;
  const int64_t w0 = base - R - 2 > 0 ? base - R - 2 : 0;
  const int64_t w1 = base + LX_BLOCK + R + 2 < n ? base + LX_BLOCK + R + 2 : n;
  for (int64_t t = threadIdx.x; t < w1 - w0; t += LX_BLOCK) win[t] = src[w0 + t];
  __syncthreads();
  const int64_t i = base + threadIdx.x;
  if (i >= n) return;
  auto w = [&](int64_t j) -> uint64_t { return win[j - w0]; };  // src[j], j in [w0, w1)
  const uint64_t k = w(i);
  const uint64_t lo = k >> nb;
  int64_t s = i, e = i + 1;
  while (s > 0 && i - s <= R && (w(s - 1) >> nb) == lo) --s;
  while (e < n && e - s <= R && (w(e) >> nb) == lo) ++e;
  const bool sfound = s == 0 || (w(s - 1) >> nb) != lo;
  const bool efound = e == n || (w(e) >> nb) != lo;
  if (sfound && efound && e - s <= R) {
    int rank = 0;
    for (int64_t j = s; j < e; ++j) rank += w(j) < k;
    dst[s + rank] = k;
  } else if (sfound && i == s) {  // the first key of a long run lists it
    longs[atomicAdd(nlong, 1ull)] = s;
  }
}

// ascending bitonic sort of a[0, L) over the power of two P >= L (indices >= L
// are +inf: a pair reaching one is left alone), block-wide; a in LDS or global
// memory (one workgroup: its own stores are visible after the barrier)
template <int NT>
__device__ void block_bitonic(uint64_t* a, int64_t L, int64_t P) {
  for (int64_t k = 2; k <= P; k <<= 1)
    for (int64_t j = k >> 1; j > 0; j >>= 1) {
      for (int64_t t = threadIdx.x; t < (P >> 1); t += NT) {
        const int lj = __builtin_ctzll((unsigned long long)j);
        const int64_t i = ((t >> lj) << (lj + 1)) | (t & (j - 1));
        const int64_t p = (j == (k >> 1)) ? (i ^ (k - 1)) : (i + j);
        if (p < L) {
          const uint64_t x = a[i], y = a[p];
          if (x > y) {
            a[i] = y;
            a[p] = x;
          }
        }
      }
      __syncthreads();
    }
}

constexpr int LL_THREADS = 1024, LL_CAP = 8192;  // 64 KB of LDS keys
__global__ void __launch_bounds__(LL_THREADS)
k_lex_long(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, int64_t n, int nb,
           const int64_t* __restrict__ longs, const unsigned long long* __restrict__ nlong) {
  __shared__ uint64_t sk[LL_CAP];
  __shared__ unsigned long long se;
  const int64_t cnt = (int64_t)*nlong;
  for (int64_t r = blockIdx.x; r < cnt; r += gridDim.x) {
    const int64_t s = longs[r];
    const uint64_t lo = src[s] >> nb;
    if (threadIdx.x == 0) se = (unsigned long long)n;
    __syncthreads();
    for (int64_t c = s; c < n; c += LL_THREADS) {  // the run's end
      const int64_t j = c + threadIdx.x;
      if (j < n && (src[j] >> nb) != lo) atomicMin(&se, (unsigned long long)j);
      __syncthreads();
      const bool done = se < (unsigned long long)n;
      __syncthreads();
      if (done) break;
    }
    const int64_t L = (int64_t)se - s;
    int64_t P = 1;
    while (P < L) P <<= 1;
    if (P <= LL_CAP) {
      for (int64_t t = threadIdx.x; t < L; t += LL_THREADS) sk[t] = src[s + t];
      __syncthreads();
      block_bitonic<LL_THREADS>(sk, L, P);
      for (int64_t t = threadIdx.x; t < L; t += LL_THREADS) dst[s + t] = sk[t];
    } else {  // beyond the LDS: in place in dst
      for (int64_t t = threadIdx.x; t < L; t += LL_THREADS) dst[s + t] = src[s + t];
      __syncthreads();
      block_bitonic<LL_THREADS>(dst + s, L, P);
    }
    __syncthreads();
  }
}

// the lo-half sort's scratch, then the long-run count and list
size_t lex_sort_bytes(int64_t n, int nb) {
  size_t bytes = 0;
  rocprim::double_buffer<uint64_t> db(nullptr, nullptr);
  if (rocprim::radix_sort_keys<KeySortCfg>(nullptr, bytes, db, (size_t)std::max<int64_t>(n, 1), (unsigned)nb,
                                           (unsigned)(2 * nb)) != hipSuccess)
    return 0;
  return (bytes + 255) / 256 * 256;
}

}  // namespace

size_t sort_lex_scratch_bytes(int64_t n, int nb, int R) {
  R = std::min(R, LX_RMAX);
  if (R <= 0 || n <= TNP_SORT_MERGE_LIMIT) return sort_scratch_bytes(n, 2 * nb);
  return lex_sort_bytes(n, nb) + 256 + sizeof(int64_t) * (size_t)(n / (R + 1) + 1);
}

int sort_keys_lex(uint64_t* a, uint64_t* b, int64_t n, int nb, int R, void* scratch, size_t scratch_bytes,
                  uint64_t** out, hipStream_t s) {
  R = std::min(R, LX_RMAX);
  if (R <= 0 || n <= TNP_SORT_MERGE_LIMIT) return sort_keys_u64(a, b, n, 2 * nb, scratch, scratch_bytes, out, s);
  const size_t rb = lex_sort_bytes(n, nb);
  if (rb == 0 || scratch_bytes < sort_lex_scratch_bytes(n, nb, R)) {
    tnp_set_error("sort_keys_lex: scratch too small");
    return -1;
  }
  rocprim::double_buffer<uint64_t> db(a, b);
  size_t bytes = rb;
  TNP_CHECK(rocprim::radix_sort_keys<KeySortCfg>(scratch, bytes, db, (size_t)n, (unsigned)nb, (unsigned)(2 * nb), s));
  uint64_t* srt = db.current();
  uint64_t* fin = srt == a ? b : a;
  auto* nlong = reinterpret_cast<unsigned long long*>(static_cast<char*>(scratch) + rb);
  auto* longs = reinterpret_cast<int64_t*>(static_cast<char*>(scratch) + rb + 256);
  TNP_CHECK(hipMemsetAsync(nlong, 0, sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_lex_runs, dim3((unsigned)((n + LX_BLOCK - 1) / LX_BLOCK)), dim3(LX_BLOCK),
                     (LX_BLOCK + 2 * R + 4) * sizeof(uint64_t), s, srt, fin, n, nb, R, longs, nlong);
  hipLaunchKernelGGL(k_lex_long, dim3(256), dim3(LL_THREADS), 0, s, srt, fin, n, nb, longs, nlong);
  TNP_CHECK(hipGetLastError());
  *out = fin;
  return 0;
}

size_t sort_pairs_scratch_bytes(int64_t n, int bits) {
  size_t bytes = 0;
  rocprim::double_buffer<uint32_t> k(nullptr, nullptr);
  rocprim::double_buffer<int32_t> v(nullptr, nullptr);
  if (rocprim::radix_sort_pairs(nullptr, bytes, k, v, (size_t)std::max<int64_t>(n, 1), 0u,
                                (unsigned)bits) != hipSuccess)
    return 0;
  return bytes;
}

int sort_pairs_u32(uint32_t* ka, uint32_t* kb, int32_t* va, int32_t* vb, int64_t n, int bits,
                   void* scratch, size_t scratch_bytes, uint32_t** ko, int32_t** vo, hipStream_t s) {
  *ko = ka;
  *vo = va;
  if (n <= 1) return 0;
  rocprim::double_buffer<uint32_t> k(ka, kb);
  rocprim::double_buffer<int32_t> v(va, vb);
  size_t bytes = scratch_bytes;
  TNP_CHECK(rocprim::radix_sort_pairs(scratch, bytes, k, v, (size_t)n, 0u, (unsigned)bits, s));
  *ko = k.current();
  *vo = v.current();
  return 0;
}
