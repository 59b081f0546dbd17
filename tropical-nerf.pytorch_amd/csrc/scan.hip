// Device-wide exclusive scan (single pass, decoupled look-back) for int32
// counts -> int64 offsets.  HBM-bound: 4 B read + 8 B written per element.
// Used for every order-preserving compaction keyed by counts (cell buckets,
// pair buckets, vertex renumbering).
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int IPT = 32;
constexpr int TILE = TNP_BLOCK * IPT;

// single pass: tile = blockIdx (ticket-free look-back, common.h
// lb_prefix_rc), thread t owns IPT consecutive elements (local serial scan),
// block scan of the thread sums, decoupled look-back for the tile's offset;
// the last tile writes the total.
__global__ void __launch_bounds__(TNP_BLOCK)
k_scan_lb(const int32_t* __restrict__ in, int64_t n, int64_t ntiles, int64_t* __restrict__ out,
          int64_t* __restrict__ total, TnpLB lb) {
  __shared__ int64_t lds[TNP_WAVES];
  __shared__ int64_t slot;
  const int64_t tile = blockIdx.x;
  int64_t base = tile * TILE + (int64_t)threadIdx.x * IPT;
  int32_t v[IPT];
  int64_t s = 0;
  if (base + IPT <= n && ((reinterpret_cast<uintptr_t>(in) & 15) == 0)) {
    // full run: 16-byte loads, all in flight (a bounds branch per element
    // would serialise them)
    const int4* p4 = reinterpret_cast<const int4*>(in + base);
#pragma unroll
    for (int q = 0; q < IPT / 4; ++q) {
      const int4 x = p4[q];
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int64_t i = base + k;
      v[k] = i < n ? in[i] : 0;
    }
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) s += v[k];
  int64_t tot;
  int64_t ex = tnp::block_scan_excl(s, lds, tot);
  // a predecessor tile not yet published: its sum, one wave
  auto tile_agg = [&](int64_t t) -> int64_t {
    const int64_t b0 = t * TILE, b1 = b0 + TILE < n ? b0 + TILE : n;
    int64_t c = 0;
    for (int64_t j = b0 + tnp::lane(); j < b1; j += 64) c += in[j];
    return tnp::wave_sum(c);
  };
  const int64_t prefix = tnp::lb_prefix_rc(lb, tile, tot, &slot, tile_agg);
  ex += prefix;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + k;
    if (i < n) out[i] = ex;
    ex += v[k];
  }
  if (total && tile == ntiles - 1 && threadIdx.x == 0) *total = prefix + tot;
}

struct FillOps {
  FillOp op[FILL_MAX];
};
// blockIdx.y: the range; 16-B stores over the aligned body, bytes at the ends
__global__ void __launch_bounds__(TNP_BLOCK) k_fill(FillOps f) {
  const FillOp& o = f.op[blockIdx.y];
  uint8_t* p = static_cast<uint8_t*>(o.p);
  const uint64_t n = o.n;
  const uint32_t b = o.byte & 0xFFu;
  const uint32_t w = b * 0x01010101u;
  const uint64_t h0 = (16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15;
  const uint64_t head = h0 < n ? h0 : n;
  const uint64_t nb = (n - head) >> 4;  // 16-B words
  const uint64_t tail0 = head + (nb << 4);
  const uint64_t t = (uint64_t)blockIdx.x * TNP_BLOCK + threadIdx.x;
  if (t < head) p[t] = (uint8_t)b;
  if (t < n - tail0) p[tail0 + t] = (uint8_t)b;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  for (uint64_t i = t; i < nb; i += (uint64_t)gridDim.x * TNP_BLOCK) q[i] = make_uint4(w, w, w, w);
}

}  // namespace

int64_t scan_tiles(int64_t n) { return (n + TILE - 1) / TILE; }

int scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, int64_t* total, const TnpLB& lb,
                    hipStream_t s) {
  if (n <= 0) {
    if (total) TNP_CHECK(hipMemsetAsync(total, 0, sizeof(int64_t), s));
    return 0;
  }
  int64_t tiles = scan_tiles(n);
  hipLaunchKernelGGL(k_scan_lb, dim3((unsigned)tiles), dim3(TNP_BLOCK), 0, s, in, n, tiles, out,
                     total, lb);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_fill(const FillOp* ops, int n, hipStream_t s) {
  FillOps f{};
  uint64_t mx = 0;
  int k = 0;
  for (int i = 0; i < n; ++i) {
    if (!ops[i].p || ops[i].n == 0) continue;
    if (k == FILL_MAX) { tnp_set_error("launch_fill: more than %d ranges", FILL_MAX); return -1; }
    f.op[k++] = ops[i];
    mx = std::max<uint64_t>(mx, ops[i].n);
  }
  if (k == 0) return 0;
  const uint64_t words = (mx + 15) / 16;
  const unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(2048, (words + TNP_BLOCK - 1) / TNP_BLOCK));
  hipLaunchKernelGGL(k_fill, dim3(gx, k), dim3(TNP_BLOCK), 0, s, f);
  TNP_CHECK(hipGetLastError());
  return 0;
}
