// The net kernels of ONE level count (compiled once per level count,
// -DTNP_LV=2..8, so the shape instantiations build in parallel): the fused
// hash-grid encoding + ReLU MLP forward, the forward of a step's new
// vertices with its epilogue, the SDF with its input gradient, the raw
// encoding and the skeleton's tile evaluation, for every (hidden, layers)
// shape of TNP_NET_SHAPES.
//
// Reference semantics:
//   Net.forward(x, gather=True)   tropical/stanford/model.py:52-76 (any
//                                 num_layers / num_hidden, model.py:19-50)
//   TropicalHashGrid.forward      tropical/tropical.py:46-47 -> tcnn Grid/Hash
//   Net.sdf / Net.normal          model.py:84-88, 105-123
//   skeleton max_grad             tropical.py:188-197
//
// Bitwise contract with the PyTorch-CPU path: net.hip header; every Linear
// layer follows the MKL schedule of its shape and row count (net_device.h
// lin_mode / linear_mode).  Compiled with -ffp-contract=off.
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "net_device.h"
#include "step.h"
#include "descend.h"
#include "train_net.h"

#ifndef TNP_LV
#error "net_lv.hip is compiled once per level count: -DTNP_LV=<2..8>"
#endif

using namespace tnpnet;

namespace {

constexpr int LVC = TNP_LV;

// GROUPED: rows come in groups of 8 consecutive lanes (box corners); a
// hidden unit is active for the whole group iff corner 0 or corner 7 has a
// pre-activation > eps (model.py:67-70), else ReLU.
template <int LV, int H, int NL, bool GROUPED>
__global__ void __launch_bounds__(TNP_BLOCK)
k_forward(NetDev net, const float* __restrict__ xyz, int64_t n, float* __restrict__ pre,
          int64_t ld, float* __restrict__ out2, uint64_t* __restrict__ kpos, uint64_t* __restrict__ kzero,
          uint64_t* __restrict__ kgrid, uint64_t* __restrict__ kpz) {
  constexpr int IN = 2 * LV;
  constexpr int NW = NetShape<LV, H, NL>::NW;
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
  const int64_t ns = net.sched_rows > 0 ? net.sched_rows : n;  // the schedule's row count
  const int m0 = lin_mode<IN, H>(ns), mh = lin_mode<H, H>(ns), mo = lin_mode<H, 2>(ns);
  constexpr int KW = key_words((NL - 1) * H + 1);
  Key<KW> ps = tnp::key_zero<KW>(), zs = tnp::key_zero<KW>();  // packed eps-sign keys (k_keys), when kpos is given
#pragma unroll
  for (int layer = 0; layer < NL - 1; ++layer) {
    if (layer == 0) {
      linear_mode<IN, H>(W, W + H * IN, h, a, m0, i);
      W += H * IN + H;
    } else {
      linear_mode<H, H>(W, W + H * H, h, a, mh, i);
      W += H * H + H;
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
      tnp::key_put(ps, p + j, a[j] > net.eps);
      tnp::key_put(zs, p + j, fabsf(a[j]) <= net.eps);
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
  linear_mode<H, 2>(W, W + 2 * H, h, o, mo, i);
  const float v = __fsub_rn(o[1], o[0]);
  if (live && pre) pre[(int64_t)p * ld + i] = v;
  if (live && out2) {
    out2[2 * i] = o[0];
    out2[2 * i + 1] = o[1];
  }
  if (!GROUPED && live && kpos) {  // the keys of k_keys, from the values in registers
    tnp::key_put(ps, p, v > net.eps);
    tnp::key_put(zs, p, fabsf(v) <= net.eps);
    tnp::pz_store(kpz, i, ps, zs);  // (kpos / kzero: views of kpz)
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
// EXP (timing experiments only, -DTNP_FWD_SHADOW builds: a shadow launch
// before the real one, tools/fwd_shadow.py): 1 no stores (a checksum), 2
// endpoints read coalesced (slots i, i + 1), 4 no zero-key gathers, 8 no
// plane-value gathers, 16 no coordinate gathers, 32 no encoding; 64: the
// real kernel (its outputs rewritten by the real launch); 128 the grid word
// without the marks search (an arithmetic stand-in)
// k_forward_new's grid: one workgroup per 256 splits (n < 0: the count on
// the device, -n its bound)
inline unsigned fwd_new_grid(int64_t n) { return tnp_grid(n >= 0 ? n : -n); }
// Streaming stores of k_forward_new: what no later kernel of the step reads
// -- the cache planes (later steps' split tests), the coordinates (later
// steps' split points, the finish) and the shared planes (the failover
// override) -- go out non-temporal, keeping the L2 for the encoding tables
// and the endpoint gathers; the (pos, zero) keys (pz, the only copy since
// round 6) and the grid words are read by this step's grouping and stay
// cached.  128^3: 0.89 -> 0.84 ms per pass for this kernel.
template <typename T>
__device__ __forceinline__ void st_stream(T& dst, T v) {
  __builtin_nontemporal_store(v, &dst);
}
template <int KW>
__device__ __forceinline__ void key_store_stream(uint64_t* a, int64_t v, const Key<KW>& k) {
#pragma unroll
  for (int q = 0; q < KW; ++q) __builtin_nontemporal_store(k.w[q], &a[KW * v + q]);
}
#ifndef TNP_FWD_MINB  // workgroups per CU the register budget is cut for (4: 100 VGPRs, no spill)
#define TNP_FWD_MINB 4
#endif
template <int LV, int H, int NL, int EXP = 0>
__global__ void __launch_bounds__(TNP_BLOCK, TNP_FWD_MINB)
k_forward_new(NetDev net, const float* xyz, int64_t n_arg, float* __restrict__ pre,
              int64_t ld, int64_t V, int keep_from, const int32_t* __restrict__ sa,
              const int32_t* __restrict__ sb, int idx, OwnBox own, uint64_t* pos,
              uint64_t* zero, uint64_t* __restrict__ grid, uint64_t* __restrict__ shared,
              int64_t* __restrict__ ctr, uint64_t* pz, const float* __restrict__ scol,
              uint32_t* __restrict__ sink = nullptr) {
  constexpr bool NOST = (EXP & 1) != 0;
  uint32_t chk = 0;
  constexpr int IN = 2 * LV;
  constexpr int NW = NetShape<LV, H, NL>::NW;
  constexpr int KW = key_words((NL - 1) * H + 1);
  // n_arg < 0: the split count is on the device (ctr[CTR_S], the split just
  // launched ahead on the stream), the grid sized by a bound (launch_forward_new)
  const int64_t n = n_arg >= 0 ? n_arg : ctr[CTR_S];  // the batch: its MKL schedule
  // the rows this launch computes: a device count is capped by the host's
  // bound -n_arg, which sized the grid, the vertex set and the shared words
  // (engine.cpp early_bound: the largest split count seen, possibly below
  // this step's S -- the host then runs the whole forward again once S is
  // known; rows past the bound are never touched here)
  const int64_t nr = n_arg >= 0 ? n_arg : (n < -n_arg ? n : -n_arg);
  // XCD-contiguous chunks of the (edge-ordered, spatially coherent) splits:
  // the hash-table lines one XCD's splits touch then mostly fit its L2.  One
  // tile per workgroup (a loop over tiles spills this kernel's registers):
  // with a device count the grid covers the bound, the workgroups past the
  // count leave before any barrier
  const int64_t ntl = (nr + TNP_BLOCK - 1) / TNP_BLOCK;
  if ((int64_t)blockIdx.x >= ntl) return;
  __shared__ float w[NW];
  __shared__ float mk[TNP_MAX_MARKS];
  // MFMA path: each wave's LDS stage for the row <-> lane-layout transposes
  __shared__ float stg[(EXP == 0 && mfma_shape<H>()) ? TNP_WAVES * 16 * MST : 1];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  for (int i = threadIdx.x; i < net.n_marks; i += blockDim.x) mk[i] = net.marks[i];
  __syncthreads();
  const int64_t i = tnp::xcd_block(blockIdx.x, ntl) * TNP_BLOCK + threadIdx.x;
  const bool live = i < nr;
  const float eps = net.eps;      // Net.region: the keys
  const float eps_s = net.eps_s;  // subpoly_'s eps: split point, failover
  float x[3] = {0.f, 0.f, 0.f};
  Key<KW> m = tnp::key_zero<KW>();
  if (live) {
    int a = sa[i], b = sb[i];
    if constexpr ((EXP & 2) != 0) {
      a = (int)min<int64_t>(i, V - 1);
      b = (int)min<int64_t>(i + 1, V - 1);
    }
    // every gather the endpoints need, issued before the first store (the
    // coordinate store could alias zero[] for the compiler)
    const Key<KW> za = (EXP & 4) ? tnp::key_zero<KW>() : tnp::vkey_load<KW>(zero, a);
    const Key<KW> zb = (EXP & 4) ? tnp::key_zero<KW>() : tnp::vkey_load<KW>(zero, b);
    if (scol) {
      // the split point itself (k_new_vertices, subpoly.py:113-117, 180), fused:
      // d = d/eps; w = |d0| / |d1 - d0|; v = e0*(1-w) + e1*w
      const float* base = xyz - 3 * V;  // xyz points at slot V
      const float c0 = (EXP & 8) ? 1.0f : scol[a], c1 = (EXP & 8) ? -1.0f - (float)(i & 7) : scol[b];
      float ea[3], eb[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        ea[d] = (EXP & 16) ? (float)(i & 255) * 0.003f : base[3 * (int64_t)a + d];
        eb[d] = (EXP & 16) ? (float)(i & 127) * 0.002f : base[3 * (int64_t)b + d];
      }
      const float d0 = __fdiv_rn(c0, eps_s), d1 = __fdiv_rn(c1, eps_s);
      const float w = __fdiv_rn(fabsf(d0), fabsf(__fsub_rn(d1, d0)));
      const float om = __fsub_rn(1.0f, w);
      float* out = const_cast<float*>(xyz) + 3 * i;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float v = __fadd_rn(__fmul_rn(ea[d], om), __fmul_rn(eb[d], w));
        if constexpr (NOST) chk ^= __float_as_uint(v);
        else st_stream(out[d], v);
        x[d] = __fmul_rn(__fadd_rn(v, 1.0f), 0.5f);  // Net.preprocess, as load_point (x/2 == x*0.5 exactly)
      }
    } else {
      load_point(xyz, i, x);
    }
    m = (za & zb & tnp::key_below<KW>(idx)) | tnp::key_bit<KW>(idx);
  }
  float h[H > IN ? H : IN];
  float a[H];
  if constexpr ((EXP & 32) != 0) {
#pragma unroll
    for (int q = 0; q < IN; ++q) h[q] = x[q % 3] * (float)(q + 1);
  } else {
    encode<LV>(net, x, h);
  }
  const float* W = w;
  int p = 0;
  Key<KW> ps = tnp::key_zero<KW>(), zs = tnp::key_zero<KW>();
  bool bad = false;
  const int m0 = lin_mode<IN, H>(n), mh = lin_mode<H, H>(n), mo = lin_mode<H, 2>(n);
  float* col = pre + V + i;
  // one plane value of this row: the cache store, the keys, the failover test
  auto plane = [&](int pp, float v) {
    if (live && pp >= keep_from) st_stream(col[(int64_t)pp * ld], v);
    tnp::key_put(ps, pp, v > eps);
    tnp::key_put(zs, pp, fabsf(v) <= eps);
    bad |= tnp::key_test(m, pp) && fabsf(v) > eps_s;
  };
  bool on_mfma = false;
  if constexpr (EXP == 0 && mfma_shape<H>()) {
    // >= 16 rows: every hidden layer is the SEQ schedule (lin_mode) -> MFMA
    // (net_device.h mfma_layer); the wave's rows go through LDS twice per 16
    // planes: features in, pre-activations back out to one row per lane
    if (n >= 16) {
      on_mfma = true;
      constexpr int NG = H / 16;
      constexpr int S0 = (IN + 3) / 4, SH = H / 4;
      constexpr int SM = S0 > SH ? S0 : SH;
      const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15;
      float* st = stg + (threadIdx.x >> 6) * (16 * MST);
#pragma unroll
      for (int k = 0; k < IN; ++k) st[k * MST + lane] = h[k];
      wave_lds_sync();
      float act[4][SM];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int s = 0; s < S0; ++s) {
          const int k = 4 * s + q;
          act[b][s] = (IN % 4 == 0 || k < IN) ? st[k * MST + 16 * b + r] : 0.f;
        }
      }
      wave_lds_sync();
#pragma unroll
      for (int layer = 0; layer < NL - 1; ++layer) {
        mf4 acc[NG][4];
        if (layer == 0) mfma_layer<IN, NG, SM>(W, act, acc, q, r);
        else mfma_layer<H, NG, SM>(W, act, acc, q, r);
        const float* B = W + H * (layer == 0 ? IN : H);
        W = B + H;
#pragma unroll
        for (int G = 0; G < NG; ++G) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float bj = B[16 * G + 4 * g + q];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const float v = __fadd_rn(acc[G][b][g], bj);
              st[(4 * g + q) * MST + 16 * b + r] = v;
              act[b][4 * G + g] = fmaxf(v, 0.0f);
            }
          }
          wave_lds_sync();
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const float v = st[j * MST + lane];
            plane(p + 16 * G + j, v);
            h[16 * G + j] = fmaxf(v, 0.0f);
          }
          wave_lds_sync();
        }
        p += H;
      }
    }
  }
#ifndef TNP_FWD_VALU_PATH  // 0: timing experiments only (tools/build_lv_variant.sh): no VALU layers
#define TNP_FWD_VALU_PATH 1  // on MFMA shapes, so < 16-row batches compute nothing
#endif
  if (!on_mfma && (TNP_FWD_VALU_PATH || !mfma_shape<H>() || EXP != 0)) {
    // VALU: the small-batch schedules (ONE / FOLD, < 16 rows), 8-wide nets
#pragma unroll
    for (int layer = 0; layer < NL - 1; ++layer) {
      if (layer == 0) {
        linear_mode<IN, H>(W, W + H * IN, h, a, m0, i);
        W += H * IN + H;
      } else {
        linear_mode<H, H>(W, W + H * H, h, a, mh, i);
        W += H * H + H;
      }
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const float v = a[j];
        if constexpr (NOST) chk ^= __float_as_uint(v);
        else plane(p + j, v);
        if constexpr (NOST) {
          tnp::key_put(ps, p + j, v > eps);
          tnp::key_put(zs, p + j, fabsf(v) <= eps);
          bad |= tnp::key_test(m, p + j) && fabsf(v) > eps_s;
        }
        h[j] = fmaxf(v, 0.0f);
      }
      p += H;
    }
  }
  p = (NL - 1) * H;
  W = w + (NW - 2 * H - 2);  // the output layer
  float o[2];
  linear_mode<H, 2>(W, W + 2 * H, h, o, mo, i);
  const float v = __fsub_rn(o[1], o[0]);
  if (NOST) {
    tnp::key_put(ps, p, v > eps);
    tnp::key_put(zs, p, fabsf(v) <= eps);
    bad |= tnp::key_test(m, p) && fabsf(v) > eps_s;
    chk ^= __float_as_uint(v) ^ (uint32_t)tnp::key_pop(ps) ^ ((uint32_t)tnp::key_pop(zs) << 8) ^ (uint32_t)bad;
    const uint64_t g = grid_word(mk, net.n_marks, eps, x);
    chk ^= (uint32_t)g ^ (uint32_t)(g >> 32);
    if (chk == 0x9E3779B9u && i == 0x7FFFFFFF) sink[0] = chk;  // never: keeps the work
    return;
  }
  if (live) {
    if (p >= keep_from) st_stream(col[(int64_t)p * ld], v);
    tnp::key_put(ps, p, v > eps);
    tnp::key_put(zs, p, fabsf(v) <= eps);
    bad |= tnp::key_test(m, p) && fabsf(v) > eps_s;
    tnp::pz_store(pz, V + i, ps, zs);  // (pos / zero: views of pz)
    key_store_stream<KW>(shared, i, m);
  }
  // full lower_bound over the marks in LDS: cheaper than gathering the
  // endpoints' grid words to narrow it (measured at 128^3: 1.02 -> 0.90 ms
  // per pass for this kernel)
  // (EXP & 128: timing experiment -- an arithmetic stand-in for the marks search)
  const uint64_t g = (EXP & 128) ? (uint64_t)(uint32_t)(int)(x[0] * 127.f) | ((uint64_t)(uint32_t)(int)(x[1] * 127.f) << 16) |
                                       ((uint64_t)(uint32_t)(int)(x[2] * 127.f) << 32)
                                 : grid_word(mk, net.n_marks, eps, x);
  if (live) grid[V + i] = g;
  // a shard's failover predicate covers the new vertices it owns: their OR
  // over the shards is the whole batch's, while a halo vertex is another
  // shard's or -- near the halo's outer faces, which miss the cells beyond
  // -- may split an edge the whole complex does not have
  const bool owned = !tnp::own_any(own) || tnp::owned_by(own, g);
  if (__ballot(live && bad && owned) && tnp::lane() == 0) tnp::or_sticky(&ctr[CTR_FAIL], 1ull);
  if (tnp::own_any(own)) {
    // the shard's ownership of the new vertex (common.h OwnBox)
    const uint64_t halo = __ballot(live && !owned);
    if (halo && tnp::lane() == 0)
      atomicAdd((unsigned long long*)&ctr[CTR_DUP], (unsigned long long)__popcll(halo));
  }
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

// SDF = tanh(o1 - o0) and its input gradient (Net.sdf / Net.normal).
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK)
k_sdf_grad(NetDev net, const float* __restrict__ xyz, int64_t n, float* __restrict__ sdf,
           float* __restrict__ grad) {
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  __syncthreads();
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[3];
  load_point(xyz, i, x);
  float g[3];
  float y = sdf_grad<LV, H, NL>(net, w, x, grad ? g : nullptr);
  sdf[i] = y;
  if (grad)
    for (int d = 0; d < 3; ++d) grad[3 * i + d] = g[d];
}

// skeleton tile (tropical.py:186-197): |sdf| at every tile lattice point +
// the tile's max |grad sdf| (skeleton.hip has the rest)
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK)
k_skel_eval(NetDev net, int i0, int j0, int k0, int n0, int n1, int n2,
            float* __restrict__ dist, unsigned int* __restrict__ gmax_bits) {
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  __syncthreads();
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t n = (int64_t)n0 * n1 * n2;
  float gn = 0.f;
  if (t < n) {
    int k = (int)(t % n2), j = (int)((t / n2) % n1), i = (int)(t / ((int64_t)n1 * n2));
    int ix[3] = {i0 + i, j0 + j, k0 + k};
    float x[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      // vertex = marks*2-1 (preprocess_inverse), then preprocess (x+1)/2
      float v = __fsub_rn(__fmul_rn(net.marks[ix[d]], 2.0f), 1.0f);
      x[d] = __fmul_rn(__fadd_rn(v, 1.0f), 0.5f);  // x/2 == x*0.5 exactly
    }
    float g[3];
    float y = sdf_grad<LV, H, NL>(net, w, x, g);
    dist[t] = fabsf(y);
    gn = sqrtf(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]);
  }
  // non-negative floats order like their bit patterns
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) gn = fmaxf(gn, __shfl_xor(gn, o, 64));
  if (tnp::lane() == 0) atomicMax(gmax_bits, __float_as_uint(gn));
}

}  // namespace

// (hidden, layers) dispatch inside one level count
#define TNP_SHAPE_CASE(H_, NL_)                              \
  case H_ * 16 + NL_: {                                      \
    constexpr int H = H_, NL = NL_;                          \
    TNP_SHAPE_BODY;                                          \
    break;                                                   \
  }
#define TNP_SHAPE_SWITCH_OF(net, SHAPES)                                                            \
  switch ((net).num_hidden * 16 + (net).num_layers) {                                              \
    SHAPES(TNP_SHAPE_CASE)                                                                           \
    default:                                                                                         \
      tnp_set_error("net shape (hidden=%d, layers=%d) not instantiated for this operation",         \
                    (net).num_hidden, (net).num_layers);                                             \
      return -1;                                                                                     \
  }
// every shape / the K <= 63 shapes (curve descent, training, autograd)
#define TNP_SHAPE_SWITCH_ALL(net) TNP_SHAPE_SWITCH_OF(net, TNP_ALL_SHAPES)
#define TNP_SHAPE_SWITCH(net) TNP_SHAPE_SWITCH_OF(net, TNP_NET_SHAPES)

template <>
int lv_forward<LVC>(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld, int group,
                    hipStream_t s, float* out2, uint64_t* pos, uint64_t* zero, uint64_t* grid, uint64_t* pz) {
#define TNP_SHAPE_BODY                                                                                          \
  if (group == 8)                                                                                               \
    hipLaunchKernelGGL((k_forward<LVC, H, NL, true>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, n, pre, \
                       ld, out2, nullptr, nullptr, nullptr, nullptr);                                           \
  else                                                                                                          \
    hipLaunchKernelGGL((k_forward<LVC, H, NL, false>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, n,    \
                       pre, ld, out2, pos, zero, grid, pz);
  TNP_SHAPE_SWITCH_ALL(net)
#undef TNP_SHAPE_BODY
  TNP_CHECK(hipGetLastError());
  return 0;
}

template <>
int lv_forward_new<LVC>(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld, int64_t V,
                        int keep_from, const int32_t* sa, const int32_t* sb, int idx, const OwnBox& own,
                        uint64_t* pos, uint64_t* zero, uint64_t* grid, uint64_t* shared, int64_t* ctr, uint64_t* pz,
                        const float* col, hipStream_t s) {
#ifdef TNP_FWD_SHADOW
  // the shadow launch's own time (HIP events; it runs first, on the caches the
  // real launch would see), summed over the process and printed at exit
  static const int shadow = getenv("TNP_FWD_SHADOW") ? atoi(getenv("TNP_FWD_SHADOW")) : 0;
  static uint32_t* sink = nullptr;
  static hipEvent_t ev[2];
  static bool pending = false;
  static double total_ms = 0.0;
  static int64_t launches = 0;
  if (shadow && !sink) {
    (void)hipMalloc(&sink, 64);
    (void)hipEventCreate(&ev[0]);
    (void)hipEventCreate(&ev[1]);
    atexit([] { fprintf(stderr, "fwd_shadow mode %d: %.4f ms over %lld launches\n", shadow, total_ms, (long long)launches); });
  }
  if (pending) {
    float ms = 0.f;
    (void)hipEventSynchronize(ev[1]);
    (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
    total_ms += ms;
    ++launches;
    pending = false;
  }
  if (shadow) (void)hipEventRecord(ev[0], s);
#define TNP_SHADOW(M)                                                                                          \
  case M:                                                                                                      \
    hipLaunchKernelGGL((k_forward_new<LVC, H, NL, M>), dim3(fwd_new_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, n, pre, \
                       ld, V, keep_from, sa, sb, idx, own, pos, zero, grid, shared, ctr, pz, col, sink);       \
    break;
#define TNP_SHADOW_LAUNCH                                                                                      \
  switch (shadow) {                                                                                            \
    TNP_SHADOW(1) TNP_SHADOW(3) TNP_SHADOW(5) TNP_SHADOW(9) TNP_SHADOW(17) TNP_SHADOW(33) TNP_SHADOW(29)       \
    TNP_SHADOW(61) TNP_SHADOW(64) TNP_SHADOW(192) default: break;                                              \
  }                                                                                                            \
  if (shadow) {                                                                                                \
    (void)hipEventRecord(ev[1], s);                                                                            \
    pending = true;                                                                                            \
  }
#else
#define TNP_SHADOW_LAUNCH
#endif
#define TNP_SHAPE_BODY                                                                                   \
  TNP_SHADOW_LAUNCH                                                                                      \
  hipLaunchKernelGGL((k_forward_new<LVC, H, NL>), dim3(fwd_new_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, n, pre, ld, \
                     V, keep_from, sa, sb, idx, own, pos, zero, grid, shared, ctr, pz, col);
  TNP_SHAPE_SWITCH_ALL(net)
#undef TNP_SHAPE_BODY
  TNP_CHECK(hipGetLastError());
  return 0;
}

template <>
int lv_sdf_grad<LVC>(const NetDev& net, const float* xyz, int64_t n, float* sdf, float* grad, hipStream_t s) {
#define TNP_SHAPE_BODY \
  hipLaunchKernelGGL((k_sdf_grad<LVC, H, NL>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, n, sdf, grad);
  TNP_SHAPE_SWITCH_ALL(net)
#undef TNP_SHAPE_BODY
  TNP_CHECK(hipGetLastError());
  return 0;
}

template <>
int lv_skel_eval<LVC>(const NetDev& net, int i0, int j0, int k0, int n0, int n1, int n2, float* dist,
                      unsigned int* gmax_bits, hipStream_t s) {
  const int64_t n = (int64_t)n0 * n1 * n2;
#define TNP_SHAPE_BODY                                                                                         \
  hipLaunchKernelGGL((k_skel_eval<LVC, H, NL>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, i0, j0, k0, n0, \
                     n1, n2, dist, gmax_bits);
  TNP_SHAPE_SWITCH_ALL(net)
#undef TNP_SHAPE_BODY
  TNP_CHECK(hipGetLastError());
  return 0;
}

template <>
int lv_train<LVC>(const NetDev& net, const float* xyz, const float* gt, int64_t n, float T, float eik_w,
                  int64_t eik_batch, double* stats, float* g_table, float* g_w, const float* gout, const float* gJ,
                  float* g_x, hipStream_t s) {
  const bool train = !gout && !gJ;
#define TNP_SHAPE_BODY                                                                                            \
  if (train)                                                                                                      \
    hipLaunchKernelGGL((k_train_norms<LVC, H, NL>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, gt, n, T,  \
                       stats);                                                                                    \
  hipLaunchKernelGGL((k_train_grads<LVC, H, NL>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, gt, n, T,    \
                     eik_w, eik_batch, stats, g_table, g_w, gout, gJ, g_x);
  TNP_SHAPE_SWITCH(net)
#undef TNP_SHAPE_BODY
  TNP_CHECK(hipGetLastError());
  return 0;
}

template <>
int lv_forward_vjp<LVC>(const NetDev& net, const float* xyz, int64_t n, const float* gpl, int64_t ld,
                        const float* gout2, float* g_table, float* g_w, float* g_x, hipStream_t s) {
#define TNP_SHAPE_BODY                                                                                           \
  hipLaunchKernelGGL((k_forward_vjp<LVC, H, NL>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, n, gpl, ld, \
                     gout2, g_table, g_w, g_x);
  TNP_SHAPE_SWITCH(net)
#undef TNP_SHAPE_BODY
  TNP_CHECK(hipGetLastError());
  return 0;
}

template <>
int lv_descend<LVC>(const NetDev& net, int64_t G, const int32_t* glist, const int32_t* crow, const int32_t* sa,
                    const int32_t* sb, const float* xyz, const int32_t* plane, int idx, float eps, int iters,
                    int record, float* ints, float* d0s, float* d1s, unsigned long long* conv, bool per_thread,
                    hipStream_t s) {
#define TNP_SHAPE_BODY                                                                                           \
  if (per_thread)                                                                                                \
    hipLaunchKernelGGL((k_descend<LVC, H, NL>), dim3(tnp_grid(G)), dim3(TNP_BLOCK), 0, s, net, G, glist, crow, sa, \
                       sb, xyz, plane, idx, eps, iters, record, ints, d0s, d1s, conv);                          \
  else                                                                                                           \
    hipLaunchKernelGGL((k_descend_wave<LVC, H, NL>), dim3((unsigned)G), dim3(64), 0, s, net, G, glist, crow, sa, \
                       sb, xyz, plane, idx, eps, iters, record, ints, d0s, d1s, conv);
  TNP_SHAPE_SWITCH_ALL(net)
#undef TNP_SHAPE_BODY
  TNP_CHECK(hipGetLastError());
  return 0;
}

template <>
int lv_encode<LVC>(const NetDev& net, const float* x01, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL((k_encode<LVC>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, x01, n, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
