// Device-wide exclusive scan (reduce-then-scan, 3 launches) for int32
// counts -> int64 offsets.  HBM-bound: 4 B read twice + 8 B written per
// element.  Used for every order-preserving compaction keyed by counts
// (cell buckets, pair buckets, vertex renumbering).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int IPT = 16;
constexpr int TILE = TNP_BLOCK * IPT;

__global__ void __launch_bounds__(TNP_BLOCK)
k_tile_sums(const int32_t* __restrict__ in, int64_t n, int64_t* __restrict__ part) {
  __shared__ int64_t lds[TNP_WAVES];
  int64_t base = (int64_t)blockIdx.x * TILE;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    if (i < n) s += in[i];
  }
  s = tnp::wave_sum(s);
  if (tnp::lane() == 0) lds[tnp::wave()] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < TNP_WAVES; ++w) t += lds[w];
    part[blockIdx.x] = t;
  }
}

// single workgroup: exclusive scan of the tile sums in place, total -> *total
__global__ void __launch_bounds__(TNP_BLOCK)
k_scan_parts(int64_t* __restrict__ part, int64_t m, int64_t* __restrict__ total) {
  __shared__ int64_t lds[TNP_WAVES];
  int64_t carry = 0;
  for (int64_t base = 0; base < m; base += TNP_BLOCK) {
    int64_t i = base + threadIdx.x;
    int64_t v = i < m ? part[i] : 0;
    int64_t tot;
    int64_t ex = tnp::block_scan_excl(v, lds, tot);
    if (i < m) part[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

__global__ void __launch_bounds__(TNP_BLOCK)
k_tile_scan(const int32_t* __restrict__ in, int64_t n, const int64_t* __restrict__ part,
            int64_t* __restrict__ out) {
  __shared__ int64_t lds[TNP_WAVES];
  // thread t owns IPT consecutive elements -> local serial scan, block scan of sums
  int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * IPT;
  int32_t v[IPT];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + k;
    v[k] = i < n ? in[i] : 0;
    s += v[k];
  }
  int64_t tot;
  int64_t ex = tnp::block_scan_excl(s, lds, tot) + part[blockIdx.x];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + k;
    if (i < n) out[i] = ex;
    ex += v[k];
  }
}

}  // namespace

size_t scan_scratch_bytes(int64_t n) {
  return (size_t)((n + TILE - 1) / TILE + 1) * sizeof(int64_t);
}

int scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, int64_t* total, void* scratch,
                    size_t scratch_bytes, hipStream_t s) {
  if (n <= 0) {
    if (total) TNP_CHECK(hipMemsetAsync(total, 0, sizeof(int64_t), s));
    return 0;
  }
  int64_t tiles = (n + TILE - 1) / TILE;
  if ((size_t)tiles * sizeof(int64_t) > scratch_bytes) {
    tnp_set_error("scan scratch too small");
    return -1;
  }
  int64_t* part = static_cast<int64_t*>(scratch);
  hipLaunchKernelGGL(k_tile_sums, dim3((unsigned)tiles), dim3(TNP_BLOCK), 0, s, in, n, part);
  hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(TNP_BLOCK), 0, s, part, tiles, total);
  hipLaunchKernelGGL(k_tile_scan, dim3((unsigned)tiles), dim3(TNP_BLOCK), 0, s, in, n, part, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
