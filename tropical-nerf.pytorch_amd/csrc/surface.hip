// extract_skeleton (tropical/subpoly.py:556-581): keep vertices on the zero
// level set of the last plane (|o1-o0| < eps, pre-tanh) inside [0,1]^3 after
// Net.preprocess, keep edges with both endpoints kept, compact in order.
#include "common.h"
#include "kernels.h"
#include "step.h"

namespace {

constexpr int IPT = 8;
constexpr int TILE = TNP_BLOCK * IPT;

__global__ void k_surface_flags(const float* __restrict__ xyz, const float* __restrict__ col,
                                int64_t V, float eps, int32_t* __restrict__ on) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  bool f = fabsf(col[v]) < eps;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float x = __fdiv_rn(__fadd_rn(xyz[3 * v + d], 1.0f), 2.0f);
    f = f && !(x > 1.0f) && !(x < 0.0f);
  }
  on[v] = f ? 1 : 0;
}

__global__ void __launch_bounds__(TNP_BLOCK)
k_surface_edges(const int32_t* __restrict__ edges, int64_t E, const int32_t* __restrict__ on,
                int32_t* __restrict__ blk, const int64_t* __restrict__ blkoff, int emit,
                int32_t* __restrict__ out, int32_t* __restrict__ used) {
  __shared__ int lds[TNP_WAVES];
  int64_t base = (int64_t)blockIdx.x * TILE;
  int64_t run = emit ? blkoff[blockIdx.x] : 0;
  int cnt = 0;
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    int a = 0, b = 0;
    bool f = false;
    if (i < E) {
      a = edges[2 * i];
      b = edges[2 * i + 1];
      f = on[a] && on[b];
    }
    if (emit) {
      int tot;
      int r = tnp::block_rank(f, lds, tot);
      if (f) {
        out[2 * (run + r)] = a;
        out[2 * (run + r) + 1] = b;
        used[a] = 1;
        used[b] = 1;
      }
      run += tot;
    } else {
      cnt += f;
    }
  }
  if (!emit) {
    cnt = tnp::wave_sum(cnt);
    if (tnp::lane() == 0) lds[tnp::wave()] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < TNP_WAVES; ++w) t += lds[w];
      blk[blockIdx.x] = t;
    }
  }
}

}  // namespace

int launch_surface_flags(const float* xyz, const float* col, int64_t V, float eps, int32_t* on,
                         hipStream_t s) {
  if (V <= 0) return 0;
  hipLaunchKernelGGL(k_surface_flags, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, xyz, col, V, eps, on);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_surface_edges(const int32_t* edges, int64_t E, const int32_t* on, int32_t* blk,
                         const int64_t* blkoff, int emit, int32_t* out, int32_t* used,
                         hipStream_t s) {
  if (E <= 0) return 0;
  hipLaunchKernelGGL(k_surface_edges, dim3((unsigned)((E + TILE - 1) / TILE)), dim3(TNP_BLOCK), 0, s,
                     edges, E, on, blk, blkoff, emit, out, used);
  TNP_CHECK(hipGetLastError());
  return 0;
}
