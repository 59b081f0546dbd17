// Net evaluation for gfx950: the eps-sign region vector, the packed sign keys
// and the new vertices' override; the level-count dispatch of the fused
// hash-grid encoding + ReLU MLP kernels (net_lv.hip, one translation unit per
// level count: forward, new-vertex forward, SDF + input gradient, encoding).
//
// Reference semantics:
//   Net.forward(x, gather=True)   tropical/stanford/model.py:52-76
//   TropicalHashGrid.forward      tropical/tropical.py:46-47 -> tcnn Grid/Hash
//   Net.region / grid region      model.py:90-103, tropical.py:227-236
//   Net.sdf / Net.normal          model.py:84-88, 105-123
//
// Bitwise contract with the PyTorch-CPU path (oracle/encoding.py,
// oracle/subdivide.py): the encoding uses the same non-fused op order, and
// every Linear layer is acc=0; acc=fma(x_k, W_jk, acc) for k ascending, then
// acc + b_j -- which is what x86 MKL sgemm (torch.nn.Linear on CPU) computes
// for these shapes (verified bitwise, tests/test_oracle_golden.py).  This
// file MUST be compiled with -ffp-contract=off; explicit __f*_rn intrinsics
// pin every rounding anyway.
//
// Roofline: one new vertex costs ~200 B of table gathers (L2/MALL resident:
// 70 kB-5 MB tables) + 12 B coords in + 4K B pre-activations out and
// ~2 kflop -- latency-bound on its dependent gathers.  k_forward_new runs the
// hidden layers of every >= 16-row call on v_mfma_f32_16x16x4_f32, which on
// gfx950 is bit for bit the sequential fma chain above (net_device.h
// mfma_layer); the small-batch schedules and the 2-output layer stay on VALU.
#include "common.h"
#include "kernels.h"
#include "net_device.h"
#include "step.h"

using namespace tnpnet;

namespace {

// the override itself (masked_fill_ of the shared planes, subpoly_debug.py:48)
// on what k_forward_new wrote; override_ < 0: the single-device predicate is
// still in ctr[CTR_FAIL]
template <int KW>
__global__ void k_override_new(int64_t n, int override_, const uint64_t* __restrict__ shared,
                               float* __restrict__ pre, int64_t ld, int keep_from, int64_t V,
                               const uint64_t* pos, const uint64_t* zero,
                               const int64_t* __restrict__ ctr, uint64_t* pz) {
  const bool ov = override_ < 0 ? ctr[CTR_FAIL] != 0 : override_ != 0;
  if (!ov) return;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const Key<KW> m = tnp::key_load<KW>(shared, r);
#pragma unroll
  for (int q = 0; q < KW; ++q)
    for (uint64_t t = m.w[q]; t; t &= t - 1) {
      const int p = 64 * q + __builtin_ctzll(t);
      if (p >= keep_from) pre[(int64_t)p * ld + V + r] = 0.f;
    }
  const Key<KW> p = tnp::vkey_load<KW>(pos, V + r) & ~m, z = tnp::vkey_load<KW>(zero, V + r) | m;
  tnp::pz_store(pz, V + r, p, z);  // (pos / zero: views of pz)
}

__global__ void k_region(NetDev net, const float* __restrict__ xyz,
                         const float* __restrict__ pre, int64_t ld, int64_t n, int K,
                         float eps, int64_t* __restrict__ m, int64_t* __restrict__ off) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[3];
  load_point(xyz, i, x);
  uint64_t g = grid_word(net.marks, net.n_marks, eps, x);
  const int C = 3 + K;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    m[i * C + d] = tnp::grid_zero(g, d) ? 0 : 1;
    off[i * 3 + d] = tnp::grid_off(g, d);
  }
  for (int p = 0; p < K; ++p) {
    float v = pre[(int64_t)p * ld + i];
    m[i * C + 3 + p] = (fabsf(v) <= eps) ? 0 : (v > 0.f ? 1 : -1);
  }
}

template <int KW>
__global__ void k_keys(NetDev net, const float* __restrict__ xyz, const float* __restrict__ pre,
                       int64_t ld, int64_t n, int K, uint64_t* __restrict__ pos,
                       uint64_t* __restrict__ zero, uint64_t* __restrict__ grid,
                       uint64_t* __restrict__ pz) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[3];
  load_point(xyz, i, x);
  grid[i] = grid_word(net.marks, net.n_marks, net.eps, x);
  Key<KW> ps = tnp::key_zero<KW>(), zs = tnp::key_zero<KW>();
  for (int p = 0; p < K; ++p) {
    float v = pre[(int64_t)p * ld + i];
    tnp::key_put(ps, p, v > net.eps);  // sign +1 ((output>0)*2-1 with |.|<=eps -> 0)
    tnp::key_put(zs, p, fabsf(v) <= net.eps);
  }
  tnp::pz_store(pz, i, ps, zs);  // (pos / zero: views of pz)
}

}  // namespace

int net_supported(const NetDev& n) {
  if (n.n_levels < 2 || n.n_levels > 8) return 0;
#define TNP_SHAPE_OK(H_, NL_) if (n.num_hidden == H_ && n.num_layers == NL_) return 1;
  TNP_ALL_SHAPES(TNP_SHAPE_OK)
#undef TNP_SHAPE_OK
  return 0;
}

int net_supported_full(const NetDev& n) {
  if (n.n_levels < 2 || n.n_levels > 8) return 0;
#define TNP_SHAPE_OK(H_, NL_) if (n.num_hidden == H_ && n.num_layers == NL_) return 1;
  TNP_NET_SHAPES(TNP_SHAPE_OK)
#undef TNP_SHAPE_OK
  return 0;
}

int launch_forward(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld,
                   int group, hipStream_t s, float* out2, uint64_t* pos, uint64_t* zero, uint64_t* grid,
                   uint64_t* pz) {
  if (n <= 0) return 0;
  if (!net_supported(net)) { tnp_set_error("unsupported net shape"); return -1; }
  if (group != 1 && (group != 8 || n % 8)) { tnp_set_error("group must be 1 or 8 (n%%8==0)"); return -1; }
  if (pos && net.n_marks > TNP_MAX_MARKS) { tnp_set_error("more than %d marks per axis", TNP_MAX_MARKS); return -1; }
  TNP_LV_SWITCH(net.n_levels, return lv_forward<L_>(net, xyz, n, pre, ld, group, s, out2, pos, zero, grid, pz));
  return 0;
}

int launch_forward_new(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld,
                       int64_t V, int keep_from, const int32_t* sa, const int32_t* sb, int idx,
                       const OwnBox& own, uint64_t* pos, uint64_t* zero, uint64_t* grid,
                       uint64_t* shared, int64_t* ctr, uint64_t* pz, const float* col, hipStream_t s) {
  if (n == 0) return 0;  // (n < 0: the count on the device, -n a bound)
  if (!net_supported(net)) { tnp_set_error("unsupported net shape"); return -1; }
  if (net.n_marks > TNP_MAX_MARKS) { tnp_set_error("more than %d marks per axis", TNP_MAX_MARKS); return -1; }
  TNP_LV_SWITCH(net.n_levels, return lv_forward_new<L_>(net, xyz, n, pre, ld, V, keep_from, sa, sb, idx, own, pos, zero, grid, shared, ctr, pz, col, s));
  return 0;
}

int launch_override_new(int64_t n, int override_, const uint64_t* shared, float* pre, int64_t ld,
                        int keep_from, int64_t V, uint64_t* pos, uint64_t* zero,
                        const int64_t* ctr, uint64_t* pz, int kw, hipStream_t s) {
  if (n <= 0 || override_ == 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_override_new<2>, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, n, override_, shared,
                       pre, ld, keep_from, V, pos, zero, ctr, pz);
  else
    hipLaunchKernelGGL(k_override_new<1>, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, n, override_, shared,
                       pre, ld, keep_from, V, pos, zero, ctr, pz);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_region(const NetDev& net, const float* xyz, const float* pre, int64_t ld, int64_t n,
                  float eps, int64_t* m, int64_t* off, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_region, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, pre, ld, n,
                     net_K(net), eps, m, off);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_keys(const NetDev& net, const float* xyz, const float* pre, int64_t ld, int64_t n,
                int K, uint64_t* pos, uint64_t* zero, uint64_t* grid, hipStream_t s, uint64_t* pz) {
  if (n <= 0) return 0;
  if (key_words(K) == 2)
    hipLaunchKernelGGL(k_keys<2>, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, pre, ld, n, K,
                       pos, zero, grid, pz);
  else
    hipLaunchKernelGGL(k_keys<1>, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, pre, ld, n, K,
                       pos, zero, grid, pz);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_sdf_grad(const NetDev& net, const float* xyz, int64_t n, float* sdf, float* grad,
                    hipStream_t s) {
  if (n <= 0) return 0;
  if (!net_supported(net)) { tnp_set_error("unsupported net shape"); return -1; }
  TNP_LV_SWITCH(net.n_levels, return lv_sdf_grad<L_>(net, xyz, n, sdf, grad, s));
  return 0;
}

int launch_encode(const NetDev& net, const float* x01, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return 0;
  TNP_LV_SWITCH(net.n_levels, return lv_encode<L_>(net, x01, n, out, s));
  return 0;
}
