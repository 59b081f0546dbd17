// Fused hash-grid encoding + ReLU MLP forward for gfx950, plus the eps-sign
// region vector, packed sign keys and the analytic SDF input gradient.
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
// ~2 kflop -- bandwidth-bound on the K*4 B store.  The MLP (8->16->16->2) is
// too narrow for MFMA tiles and its sequential-fma order is part of the
// parity contract, so it runs on VALU with weights broadcast from LDS.
#include "common.h"
#include "kernels.h"
#include "net_device.h"
#include "step.h"

using namespace tnpnet;

namespace {

// GROUPED: rows come in groups of 8 consecutive lanes (box corners); a
// hidden unit is active for the whole group iff corner 0 or corner 7 has a
// pre-activation > eps (model.py:67-70), else ReLU.
template <int LV, int H, int NL, bool GROUPED>
__global__ void __launch_bounds__(TNP_BLOCK)
k_forward(NetDev net, const float* __restrict__ xyz, int64_t n, float* __restrict__ pre,
          int64_t ld, float* __restrict__ out2, uint64_t* __restrict__ kpos, uint64_t* __restrict__ kzero,
          uint64_t* __restrict__ kgrid, ulonglong2* __restrict__ kpz) {
  constexpr int IN = 2 * LV;
  constexpr int NW = H * IN + H + (NL - 2) * (H * H + H) + 2 * H + 2;
  __shared__ float w[NW];
  __shared__ float mk[GROUPED ? 1 : TNP_MAX_MARKS];  // the marks for the grid words (keys)
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  if (!GROUPED && kpos)
    for (int i = threadIdx.x; i < net.n_marks; i += blockDim.x) mk[i] = net.marks[i];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n;
  float x[3] = {0.f, 0.f, 0.f};
  if (live) load_point(xyz, i, x);
  float h[H > IN ? H : IN];
  float a[H];
  encode<LV>(net, x, h);
  const float* W = w;
  int p = 0;
  const int mh = lin_mode(n, false), mo = lin_mode(n, true);
  uint64_t ps = 0, zs = 0;  // packed eps-sign keys (k_keys), when kpos is given
#pragma unroll
  for (int layer = 0; layer < NL - 1; ++layer) {
    if (layer == 0) {
      linear_mode<IN, H>(W, W + H * IN, h, a, mh);
      W += H * IN + H;
    } else {
      linear_mode<H, H>(W, W + H * H, h, a, mh);
      W += H * H + H;
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
      ps |= (uint64_t)(a[j] > net.eps) << (p + j);
      zs |= (uint64_t)(fabsf(a[j]) <= net.eps) << (p + j);
      if (live && pre) pre[(int64_t)(p + j) * ld + i] = a[j];
      if (GROUPED) {
        const int base = (threadIdx.x & 63) & ~7;
        float a_first = __shfl(a[j], base, 64);
        float a_last = __shfl(a[j], base + 7, 64);
        bool on = (a_first > net.eps) || (a_last > net.eps);
        h[j] = __fmul_rn(a[j], on ? 1.0f : 0.0f);
      } else {
        h[j] = fmaxf(a[j], 0.0f);
      }
    }
    p += H;
  }
  float o[2];
  linear_mode<H, 2>(W, W + 2 * H, h, o, mo);
  const float v = __fsub_rn(o[1], o[0]);
  if (live && pre) pre[(int64_t)p * ld + i] = v;
  if (live && out2) {
    out2[2 * i] = o[0];
    out2[2 * i + 1] = o[1];
  }
  if (!GROUPED && live && kpos) {  // the keys of k_keys, from the values in registers
    ps |= (uint64_t)(v > net.eps) << p;
    zs |= (uint64_t)(fabsf(v) <= net.eps) << p;
    kpos[i] = ps;
    kzero[i] = zs;
    kpz[i] = make_ulonglong2(ps, zs);
    kgrid[i] = grid_word(mk, net.n_marks, net.eps, x);
  }
}

// Forward of the S new vertices of a flat step with the step's epilogue
// fused (replaces forward -> fail_check -> keys -> finalize_new): the
// pre-activations of planes >= keep_from go straight into the cache
// (plane-major, slot V + r), the packed pos/zero/grid keys are written as if
// no override applies, and the failover predicate of subpoly_debug.py:35-49
// (a new vertex off one of its shared planes by more than eps) is ORed into
// ctr[CTR_FAIL]; shared[r] keeps the plane set for k_override_new.  Values
// and the MKL row-count schedule are those of k_forward (same n = S).
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK, 4)
k_forward_new(NetDev net, const float* xyz, int64_t n, float* __restrict__ pre,
              int64_t ld, int64_t V, int keep_from, const int32_t* __restrict__ sa,
              const int32_t* __restrict__ sb, int idx, int own_lo, int own_hi, uint64_t* pos,
              uint64_t* zero, uint64_t* __restrict__ grid, uint64_t* __restrict__ shared,
              int64_t* __restrict__ ctr, ulonglong2* __restrict__ pz, const float* __restrict__ scol) {
  constexpr int IN = 2 * LV;
  constexpr int NW = H * IN + H + (NL - 2) * (H * H + H) + 2 * H + 2;
  __shared__ float w[NW];
  __shared__ float mk[TNP_MAX_MARKS];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  for (int i = threadIdx.x; i < net.n_marks; i += blockDim.x) mk[i] = net.marks[i];
  __syncthreads();
  // XCD-contiguous chunks of the (edge-ordered, spatially coherent) splits:
  // the hash-table lines one XCD's splits touch then mostly fit its L2
  const int64_t i = tnp::xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const bool live = i < n;
  const float eps = net.eps;
  float x[3] = {0.f, 0.f, 0.f};
  uint64_t m = 0;
  if (live) {
    const int a = sa[i], b = sb[i];
    // every gather the endpoints need, issued before the first store (the
    // coordinate store could alias zero[] for the compiler)
    const uint64_t za = zero[a], zb = zero[b];
    if (scol) {
      // the split point itself (k_new_vertices, subpoly.py:113-117, 180), fused:
      // d = d/eps; w = |d0| / |d1 - d0|; v = e0*(1-w) + e1*w
      const float* base = xyz - 3 * V;  // xyz points at slot V
      const float c0 = scol[a], c1 = scol[b];
      float ea[3], eb[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        ea[d] = base[3 * (int64_t)a + d];
        eb[d] = base[3 * (int64_t)b + d];
      }
      const float d0 = __fdiv_rn(c0, eps), d1 = __fdiv_rn(c1, eps);
      const float w = __fdiv_rn(fabsf(d0), fabsf(__fsub_rn(d1, d0)));
      const float om = __fsub_rn(1.0f, w);
      float* out = const_cast<float*>(xyz) + 3 * i;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float v = __fadd_rn(__fmul_rn(ea[d], om), __fmul_rn(eb[d], w));
        out[d] = v;
        x[d] = __fmul_rn(__fadd_rn(v, 1.0f), 0.5f);  // Net.preprocess, as load_point (x/2 == x*0.5 exactly)
      }
    } else {
      load_point(xyz, i, x);
    }
    const uint64_t below = (idx >= 64) ? ~0ull : ((1ull << idx) - 1ull);
    m = (za & zb & below) | (1ull << idx);
  }
  float h[H > IN ? H : IN];
  float a[H];
  encode<LV>(net, x, h);
  const float* W = w;
  int p = 0;
  uint64_t ps = 0, zs = 0;
  bool bad = false;
  const int mh = lin_mode(n, false), mo = lin_mode(n, true);
  float* col = pre + V + i;
#pragma unroll
  for (int layer = 0; layer < NL - 1; ++layer) {
    if (layer == 0) {
      linear_mode<IN, H>(W, W + H * IN, h, a, mh);
      W += H * IN + H;
    } else {
      linear_mode<H, H>(W, W + H * H, h, a, mh);
      W += H * H + H;
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const float v = a[j];
      if (live && p + j >= keep_from) col[(int64_t)(p + j) * ld] = v;
      ps |= (uint64_t)(v > eps) << (p + j);
      zs |= (uint64_t)(fabsf(v) <= eps) << (p + j);
      bad |= ((m >> (p + j)) & 1) && fabsf(v) > eps;
      h[j] = fmaxf(v, 0.0f);
    }
    p += H;
  }
  float o[2];
  linear_mode<H, 2>(W, W + 2 * H, h, o, mo);
  const float v = __fsub_rn(o[1], o[0]);
  if (live) {
    if (p >= keep_from) col[(int64_t)p * ld] = v;
    ps |= (uint64_t)(v > eps) << p;
    zs |= (uint64_t)(fabsf(v) <= eps) << p;
    bad |= ((m >> p) & 1) && fabsf(v) > eps;
    pos[V + i] = ps;
    zero[V + i] = zs;
    pz[V + i] = make_ulonglong2(ps, zs);
    shared[i] = m;
  }
  // full lower_bound over the marks in LDS: cheaper than gathering the
  // endpoints' grid words to narrow it (measured at 128^3: 1.02 -> 0.90 ms
  // per pass for this kernel)
  const uint64_t g = grid_word(mk, net.n_marks, eps, x);
  if (live) grid[V + i] = g;
  if (__ballot(live && bad) && tnp::lane() == 0) tnp::or_sticky(&ctr[CTR_FAIL], 1ull);
  if (own_lo <= own_hi) {
    // x-slab ownership of the new vertex: on mark plane p -> owned iff
    // own_lo < p <= own_hi (plane 0 by the first shard); in the cell above
    // mark c -> owned iff own_lo <= c < own_hi
    const int c = tnp::grid_off(g, 0);
    const bool owned = tnp::grid_zero(g, 0) ? ((c > own_lo || (own_lo == 0 && c == 0)) && c <= own_hi)
                                            : (c >= own_lo && c < own_hi);
    const uint64_t halo = __ballot(live && !owned);
    if (halo && tnp::lane() == 0)
      atomicAdd((unsigned long long*)&ctr[CTR_DUP], (unsigned long long)__popcll(halo));
  }
}

// the override itself (masked_fill_ of the shared planes, subpoly_debug.py:48)
// on what k_forward_new wrote; override_ < 0: the single-device predicate is
// still in ctr[CTR_FAIL]
__global__ void k_override_new(int64_t n, int override_, const uint64_t* __restrict__ shared,
                               float* __restrict__ pre, int64_t ld, int keep_from, int64_t V,
                               uint64_t* __restrict__ pos, uint64_t* __restrict__ zero,
                               const int64_t* __restrict__ ctr, ulonglong2* __restrict__ pz) {
  const bool ov = override_ < 0 ? ctr[CTR_FAIL] != 0 : override_ != 0;
  if (!ov) return;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint64_t m = shared[r];
  for (uint64_t t = m; t; t &= t - 1) {
    const int p = __builtin_ctzll(t);
    if (p >= keep_from) pre[(int64_t)p * ld + V + r] = 0.f;
  }
  const uint64_t p = pos[V + r] & ~m, z = zero[V + r] | m;
  pos[V + r] = p;
  zero[V + r] = z;
  pz[V + r] = make_ulonglong2(p, z);
}

// TropicalHashGrid.forward: raw encoding of x already in [0,1]^3 -> [n][2L]
template <int LV>
__global__ void k_encode(NetDev net, const float* __restrict__ x01, int64_t n, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[3] = {x01[3 * i], x01[3 * i + 1], x01[3 * i + 2]};
  float f[2 * LV];
  encode<LV>(net, x, f);
#pragma unroll
  for (int k = 0; k < 2 * LV; ++k) out[i * 2 * LV + k] = f[k];
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

__global__ void k_keys(NetDev net, const float* __restrict__ xyz, const float* __restrict__ pre,
                       int64_t ld, int64_t n, int K, uint64_t* __restrict__ pos,
                       uint64_t* __restrict__ zero, uint64_t* __restrict__ grid,
                       ulonglong2* __restrict__ pz) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[3];
  load_point(xyz, i, x);
  grid[i] = grid_word(net.marks, net.n_marks, net.eps, x);
  uint64_t ps = 0, zs = 0;
  for (int p = 0; p < K; ++p) {
    float v = pre[(int64_t)p * ld + i];
    ps |= (uint64_t)(v > net.eps) << p;  // sign +1 ((output>0)*2-1 with |.|<=eps -> 0)
    zs |= (uint64_t)(fabsf(v) <= net.eps) << p;
  }
  pos[i] = ps;
  zero[i] = zs;
  if (pz) pz[i] = make_ulonglong2(ps, zs);
}

// SDF = tanh(o1 - o0) and its input gradient (Net.sdf / Net.normal).
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK)
k_sdf_grad(NetDev net, const float* __restrict__ xyz, int64_t n, float* __restrict__ sdf,
           float* __restrict__ grad) {
  static_assert(NL == 3, "gradient kernel instantiated for 3-layer nets");
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  __syncthreads();
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[3];
  load_point(xyz, i, x);
  float g[3];
  float y = sdf_grad<LV, H>(net, w, x, grad ? g : nullptr);
  sdf[i] = y;
  if (grad)
    for (int d = 0; d < 3; ++d) grad[3 * i + d] = g[d];
}

}  // namespace

#define TNP_DISPATCH(LV, BODY)                                      \
  switch (LV) {                                                     \
    case 2: { constexpr int L_ = 2; BODY; break; }                  \
    case 4: { constexpr int L_ = 4; BODY; break; }                  \
    default: tnp_set_error("n_levels=%d not instantiated", LV); return -1; \
  }

int net_supported(const NetDev& n) {
  return (n.n_levels == 2 || n.n_levels == 4) && n.num_hidden == 16 && n.num_layers == 3;
}

int launch_forward(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld,
                   int group, hipStream_t s, float* out2, uint64_t* pos, uint64_t* zero, uint64_t* grid,
                   uint64_t* pz) {
  if (n <= 0) return 0;
  if (!net_supported(net)) { tnp_set_error("unsupported net shape"); return -1; }
  if (group != 1 && (group != 8 || n % 8)) { tnp_set_error("group must be 1 or 8 (n%%8==0)"); return -1; }
  if (pos && net.n_marks > TNP_MAX_MARKS) { tnp_set_error("more than %d marks per axis", TNP_MAX_MARKS); return -1; }
  TNP_DISPATCH(net.n_levels, {
    if (group == 8)
      hipLaunchKernelGGL((k_forward<L_, 16, 3, true>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s,
                         net, xyz, n, pre, ld, out2, nullptr, nullptr, nullptr, nullptr);
    else
      hipLaunchKernelGGL((k_forward<L_, 16, 3, false>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s,
                         net, xyz, n, pre, ld, out2, pos, zero, grid,
                         reinterpret_cast<ulonglong2*>(pz));
  });
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_forward_new(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld,
                       int64_t V, int keep_from, const int32_t* sa, const int32_t* sb, int idx,
                       int own_lo, int own_hi, uint64_t* pos, uint64_t* zero, uint64_t* grid,
                       uint64_t* shared, int64_t* ctr, uint64_t* pz, const float* col, hipStream_t s) {
  if (n <= 0) return 0;
  if (!net_supported(net)) { tnp_set_error("unsupported net shape"); return -1; }
  if (net.n_marks > TNP_MAX_MARKS) { tnp_set_error("more than %d marks per axis", TNP_MAX_MARKS); return -1; }
  TNP_DISPATCH(net.n_levels, {
    hipLaunchKernelGGL((k_forward_new<L_, 16, 3>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net,
                       xyz, n, pre, ld, V, keep_from, sa, sb, idx, own_lo, own_hi, pos, zero, grid,
                       shared, ctr, reinterpret_cast<ulonglong2*>(pz), col);
  });
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_override_new(int64_t n, int override_, const uint64_t* shared, float* pre, int64_t ld,
                        int keep_from, int64_t V, uint64_t* pos, uint64_t* zero,
                        const int64_t* ctr, uint64_t* pz, hipStream_t s) {
  if (n <= 0 || override_ == 0) return 0;
  hipLaunchKernelGGL(k_override_new, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, n, override_, shared,
                     pre, ld, keep_from, V, pos, zero, ctr, reinterpret_cast<ulonglong2*>(pz));
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
  hipLaunchKernelGGL(k_keys, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, pre, ld, n, K,
                     pos, zero, grid, reinterpret_cast<ulonglong2*>(pz));
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_sdf_grad(const NetDev& net, const float* xyz, int64_t n, float* sdf, float* grad,
                    hipStream_t s) {
  if (n <= 0) return 0;
  if (!net_supported(net)) { tnp_set_error("unsupported net shape"); return -1; }
  TNP_DISPATCH(net.n_levels, {
    hipLaunchKernelGGL((k_sdf_grad<L_, 16, 3>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net,
                       xyz, n, sdf, grad);
  });
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_encode(const NetDev& net, const float* x01, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return 0;
  TNP_DISPATCH(net.n_levels, {
    hipLaunchKernelGGL((k_encode<L_>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, x01, n, out);
  });
  TNP_CHECK(hipGetLastError());
  return 0;
}
