// Device-side building blocks of the net evaluation, shared by net.hip
// (forward / region / keys / gradient kernels) and skeleton.hip.
// Bitwise contract: see net.hip.
#pragma once
#include "common.h"
#include "kernels.h"

namespace tnpnet {

constexpr uint32_t P1 = 2654435761u;
constexpr uint32_t P2 = 805459861u;

// idx mod size, without an integer division when size is a power of two
// (every hashed level: 2^T; the branch is uniform)
__device__ __forceinline__ uint32_t wrap_index(uint32_t idx, uint32_t size) {
  return (size & (size - 1u)) == 0u ? (idx & (size - 1u)) : idx % size;
}

// float2 entry `idx` of level l in either table layout (NetDev::tied)
__device__ __forceinline__ float2 table_entry(const NetDev& net, int l, uint32_t idx) {
  const float2* tab = reinterpret_cast<const float2*>(net.table);
  return net.tied ? tab[(size_t)idx * net.n_levels + l] : tab[net.offsets[l] + idx];
}

// Tied levels: positions, weights and indices are those of level 0 for
// every level (same fp32 scale), the per-level sums keep the corner order
// of the untied path, so the features are bitwise the same.
template <int LV>
__device__ __forceinline__ void encode_tied(const NetDev& net, const float x[3], float* feat) {
  const float s = net.scales[0];
  float t[3];
  uint32_t g[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float pos = __fadd_rn(__fmul_rn(x[d], s), 0.5f);
    float fl = floorf(pos);
    t[d] = __fsub_rn(pos, fl);
    g[d] = (uint32_t)(int)fl;
  }
  const uint32_t res = (uint32_t)net.res[0];
  const uint32_t size = net.sizes[0];
  const bool dense = net.dense[0] != 0;
  const float4* tab = reinterpret_cast<const float4*>(net.table);
  float acc[2 * LV];
#pragma unroll
  for (int q = 0; q < 2 * LV; ++q) acc[q] = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float w = 1.0f;
    uint32_t gc[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      if ((c >> d) & 1) {
        w = __fmul_rn(w, t[d]);
        gc[d] = g[d] + 1u;
      } else {
        w = __fmul_rn(w, __fsub_rn(1.0f, t[d]));
        gc[d] = g[d];
      }
    }
    uint32_t idx = dense ? (gc[0] + gc[1] * res + gc[2] * (res * res))
                         : (gc[0] ^ (gc[1] * P1) ^ (gc[2] * P2));
    idx = wrap_index(idx, size);
#pragma unroll
    for (int q = 0; q < LV / 2; ++q) {
      const float4 v = tab[(size_t)idx * (LV / 2) + q];
      acc[4 * q + 0] = __fadd_rn(acc[4 * q + 0], __fmul_rn(w, v.x));
      acc[4 * q + 1] = __fadd_rn(acc[4 * q + 1], __fmul_rn(w, v.y));
      acc[4 * q + 2] = __fadd_rn(acc[4 * q + 2], __fmul_rn(w, v.z));
      acc[4 * q + 3] = __fadd_rn(acc[4 * q + 3], __fmul_rn(w, v.w));
    }
  }
#pragma unroll
  for (int q = 0; q < 2 * LV; ++q) feat[q] = acc[q];
}

template <int LV>
__device__ __forceinline__ void encode(const NetDev& net, const float x[3], float* feat) {
  if constexpr (LV % 2 == 0) {
    if (net.tied) {
      encode_tied<LV>(net, x, feat);
      return;
    }
  }
#pragma unroll
  for (int l = 0; l < LV; ++l) {
    const float s = net.scales[l];
    float t[3];
    uint32_t g[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float pos = __fadd_rn(__fmul_rn(x[d], s), 0.5f);
      float fl = floorf(pos);
      t[d] = __fsub_rn(pos, fl);
      g[d] = (uint32_t)(int)fl;
    }
    const uint32_t res = (uint32_t)net.res[l];
    const uint32_t size = net.sizes[l];
    const bool dense = net.dense[l] != 0;
    const float2* tab = reinterpret_cast<const float2*>(net.table) + net.offsets[l];
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float w = 1.0f;
      uint32_t gc[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        if ((c >> d) & 1) {
          w = __fmul_rn(w, t[d]);
          gc[d] = g[d] + 1u;
        } else {
          w = __fmul_rn(w, __fsub_rn(1.0f, t[d]));
          gc[d] = g[d];
        }
      }
      uint32_t idx = dense ? (gc[0] + gc[1] * res + gc[2] * (res * res))
                           : (gc[0] ^ (gc[1] * P1) ^ (gc[2] * P2));
      idx = wrap_index(idx, size);
      float2 v = tab[idx];
      a0 = __fadd_rn(a0, __fmul_rn(w, v.x));
      a1 = __fadd_rn(a1, __fmul_rn(w, v.y));
    }
    feat[2 * l] = a0;
    feat[2 * l + 1] = a1;
  }
}

__device__ __forceinline__ void load_point(const float* xyz, int64_t i, float x[3]) {
  // Net.preprocess: (x + 1) / 2   (model.py:78-79)
#pragma unroll
  for (int d = 0; d < 3; ++d) x[d] = __fmul_rn(__fadd_rn(xyz[3 * i + d], 1.0f), 0.5f);  // x/2 == x*0.5 exactly
}

template <int IN, int OUT>
__device__ __forceinline__ void linear(const float* __restrict__ W, const float* __restrict__ b,
                                       const float* in, float* out) {
#pragma unroll
  for (int j = 0; j < OUT; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < IN; ++k) acc = __fmaf_rn(in[k], W[j * IN + k], acc);
    out[j] = __fadd_rn(acc, b[j]);
  }
}

// lower_bound over the sorted marks: torch.searchsorted(marks, v) (left)
__device__ __forceinline__ int search_left(const float* marks, int M, float v) {
  int lo = 0, hi = M;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (marks[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint64_t grid_word(const float* marks, int M, float eps,
                                              const float x[3]) {
  uint64_t g = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    int off = search_left(marks, M, __fadd_rn(x[d], eps)) - 1;
    float mk = marks[off < 0 ? off + M : off];
    bool zero = !(fabsf(__fsub_rn(mk, x[d])) > eps);
    g |= (uint64_t)(uint32_t)(off + 2) << (16 * d);
    g |= (uint64_t)(zero ? 1 : 0) << (48 + d);
  }
  return g;
}


// SDF = tanh(o1 - o0) and d SDF / d x (input gradient through ReLU masks and
// the trilinear encoding; floor() has zero gradient so the cell on the right
// is used on grid lines, as autograd through tcnn does).  w: packed weights
// of an NL-layer net (NL - 1 hidden layers of H).
template <int LV, int H, int NL>
__device__ __forceinline__ float sdf_grad(const NetDev& net, const float* w, const float x[3],
                                          float* grad) {
  constexpr int IN = 2 * LV;
  constexpr int NH = NL - 1;  // hidden layers
  float f[IN], a[NH][H], h[H], o[2];
  encode<LV>(net, x, f);
  const float* Wl[NH];
  Wl[0] = w;
#pragma unroll
  for (int l = 1; l < NH; ++l) Wl[l] = Wl[l - 1] + (l == 1 ? H * IN + H : H * H + H);
  const float* WL = Wl[NH - 1] + (NH == 1 ? H * IN + H : H * H + H);
  linear<IN, H>(Wl[0], Wl[0] + H * IN, f, a[0]);
#pragma unroll
  for (int j = 0; j < H; ++j) h[j] = fmaxf(a[0][j], 0.f);
#pragma unroll
  for (int l = 1; l < NH; ++l) {
    linear<H, H>(Wl[l], Wl[l] + H * H, h, a[l]);
#pragma unroll
    for (int j = 0; j < H; ++j) h[j] = fmaxf(a[l][j], 0.f);
  }
  linear<H, 2>(WL, WL + 2 * H, h, o);
  float y = tanhf(o[1] - o[0]);
  if (grad == nullptr) return y;
  float gz = 1.f - y * y;
  float d[H], df[IN];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float v = gz * WL[H + j] - gz * WL[j];
    d[j] = a[NH - 1][j] > 0.f ? v : 0.f;
  }
#pragma unroll
  for (int l = NH - 1; l >= 1; --l) {
    float dp[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < H; ++j) v += d[j] * Wl[l][j * H + k];
      dp[k] = a[l - 1][k] > 0.f ? v : 0.f;
    }
#pragma unroll
    for (int k = 0; k < H; ++k) d[k] = dp[k];
  }
  const float* W0 = Wl[0];
#pragma unroll
  for (int m = 0; m < IN; ++m) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < H; ++k) v += d[k] * W0[k * IN + m];
    df[m] = v;
  }
  float gx[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < LV; ++l) {
    const float s = net.scales[l];
    float t[3];
    uint32_t g[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float pos = x[d] * s + 0.5f;
      float fl = floorf(pos);
      t[d] = pos - fl;
      g[d] = (uint32_t)(int)fl;
    }
    const uint32_t res = (uint32_t)net.res[l];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float fc[3];
      uint32_t gc[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        bool up = (c >> d) & 1;
        fc[d] = up ? t[d] : 1.f - t[d];
        gc[d] = g[d] + (up ? 1u : 0u);
      }
      uint32_t idx = net.dense[l] ? (gc[0] + gc[1] * res + gc[2] * (res * res))
                                  : (gc[0] ^ (gc[1] * P1) ^ (gc[2] * P2));
      idx = wrap_index(idx, net.sizes[l]);
      float2 v = table_entry(net, l, idx);
      float dv = v.x * df[2 * l] + v.y * df[2 * l + 1];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        float sg = ((c >> d) & 1) ? 1.f : -1.f;
        gx[d] += sg * fc[(d + 1) % 3] * fc[(d + 2) % 3] * dv * s;
      }
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) grad[d] = gx[d] * 0.5f;  // d/dx of (x+1)/2
  return y;
}

// Batch-size-dependent summation schedules of x86 MKL sgemm (what
// torch.nn.Linear computes on CPU in the reference), reverse-engineered
// bitwise for every layer shape of the supported nets (IN = 2 x levels or
// H inputs, OUT = H or 2 outputs; oracle/subdivide.py::linear_seqfma,
// tools/mkl_order_probe.py).  With p_k = x_k*W_jk rounded and the lanes of a
// WD-wide vector (WD = next power of two >= IN, zero-padded; 16 lanes a
// register: inputs 16..31 are fma'd onto lanes 0..15 first):
//   SEQ   acc = 0; acc = fma(x_k, W_jk, acc); acc + b_j
//   ONE   (a 1-row call) lanes {0, fma(x1,W_j1,p0), p2, ...}, halving fold,
//         + b_j; the 2-output layer adds p0 after the fold of {0, p1, p2, ...}
//   FOLD  (2-output layer, 2..15 rows; 8-output layer of <= 8 inputs, 2..7
//         rows) halving fold of the p_k, + b_j; 32 inputs: lane i = p_i +
//         p_{i+16} on even rows, fma(x_{i+16}, W, p_i) on odd rows
enum LinMode { LIN_SEQ = 0, LIN_ONE = 1, LIN_FOLD = 2 };

__host__ __device__ constexpr int next_pow2(int k) { return k <= 1 ? 1 : 2 * next_pow2((k + 1) / 2); }

template <int IN>
__device__ __forceinline__ float fold_lanes(float* l) {
#pragma unroll
  for (int h = IN / 2; h >= 1; h /= 2) {
#pragma unroll
    for (int i = 0; i < h; ++i) l[i] = __fadd_rn(l[i], l[i + h]);
  }
  return l[0];
}

// output j of linear_mode<IN, OUT> (the same ops, one output); row: the
// row's index in the call (its parity picks the 32-input FOLD variant)
template <int IN, int OUT>
__device__ __forceinline__ float neuron_mode(const float* __restrict__ W, const float* __restrict__ b,
                                             const float* in, int j, int mode, int64_t row = 0) {
  if (mode == LIN_SEQ) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < IN; ++k) acc = __fmaf_rn(in[k], W[j * IN + k], acc);
    return __fadd_rn(acc, b[j]);
  }
  constexpr int WD = next_pow2(IN);
  constexpr int LN = WD < 16 ? WD : 16;
  static_assert(WD <= 32, "layers of at most 32 inputs");
  const float* Wj = W + j * IN;
  if constexpr (IN == 32 && OUT == 32) {
    // the 32 -> 32 hidden layer's 1-row call (mode ONE; FOLD never applies):
    // MKL's tree, probed bitwise (tools/mkl_order_probe.py tree32): inputs
    // 0..16 as one block, then 17 by fma, then 25, 21 + 29 and
    // 19/23/27/31 in turn, the even inputs 18..30 as one block, bias last
    if (mode == LIN_ONE) {
      auto p = [&](int k) { return __fmul_rn(in[k], Wj[k]); };
      auto s = [](float u, float v) { return __fadd_rn(u, v); };
      const float a1 = s(s(__fmaf_rn(in[1], Wj[1], p(0)), p(9)), s(p(5), p(13)));
      const float a2 = s(s(p(3), p(11)), s(p(7), p(15)));
      const float bl = s(s(s(p(2), p(10)), s(p(6), p(14))), s(s(p(4), p(12)), s(p(8), p(16))));
      float t = __fmaf_rn(in[17], Wj[17], s(s(a1, a2), bl));
      t = s(t, p(25));
      t = s(t, s(p(21), p(29)));
      t = s(t, s(s(p(19), p(27)), s(p(23), p(31))));
      const float ev = s(s(s(p(18), p(26)), s(p(22), p(30))), s(s(p(20), p(28)), p(24)));
      return s(s(t, ev), b[j]);
    }
  }
  float l[LN];
  float r;
  if (mode == LIN_FOLD) {
    if constexpr (WD <= 16) {
#pragma unroll
      for (int k = 0; k < WD; ++k) l[k] = k < IN ? __fmul_rn(in[k], Wj[k]) : 0.f;
    } else {
      const bool odd = row & 1;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __fmul_rn(in[i], Wj[i]);
        l[i] = odd ? __fmaf_rn(in[i + 16], Wj[i + 16], p) : __fadd_rn(p, __fmul_rn(in[i + 16], Wj[i + 16]));
      }
    }
    r = fold_lanes<LN>(l);
  } else {
    float base[WD];
#pragma unroll
    for (int k = 0; k < WD; ++k) base[k] = k < IN ? __fmul_rn(in[k], Wj[k]) : 0.f;
    const float p0 = base[0];
    if (OUT != 2) base[1] = __fmaf_rn(in[1], Wj[1], p0);
    base[0] = 0.f;
#pragma unroll
    for (int i = 0; i < LN; ++i) l[i] = (WD > 16 && i + 16 < IN) ? __fmaf_rn(in[i + 16], Wj[i + 16], base[i]) : base[i];
    r = fold_lanes<LN>(l);
    if (OUT == 2) r = __fadd_rn(p0, r);
  }
  return __fadd_rn(r, b[j]);
}

template <int IN, int OUT>
__device__ __forceinline__ void linear_mode(const float* __restrict__ W, const float* __restrict__ b,
                                            const float* in, float* out, int mode, int64_t row = 0) {
  if (mode == LIN_SEQ) {
    linear<IN, OUT>(W, b, in, out);
    return;
  }
#pragma unroll
  for (int j = 0; j < OUT; ++j) out[j] = neuron_mode<IN, OUT>(W, b, in, j, mode, row);
}

// the schedule of an n-row call of an IN -> OUT layer
template <int IN, int OUT>
__host__ __device__ __forceinline__ int lin_mode(int64_t n) {
  if (n == 1) return LIN_ONE;
  if (n >= 16) return LIN_SEQ;
  if (OUT == 2 || (OUT == 8 && IN <= 8 && n <= 7)) return LIN_FOLD;
  return LIN_SEQ;
}

// ---------------------------------------------------------------------------
// The SEQ schedule on the matrix cores.  On gfx950 v_mfma_f32_16x16x4_f32 is
// bit for bit the k-ordered fp32 fma chain D = fma(a_k3, b_k3, ... fma(a_k0,
// b_k0, C)), one rounding per product (cdna_hip_programming.md "FP32-input
// MFMA"; tools/mfma_probe.hip checks it on the box: 41 M outputs, zeros,
// negative zeros and denormals included, 0 mismatches).  So a 16-output
// slice of an IN -> H layer over 16 rows, K-blocks of 4 chained in ascending
// order from C = 0 and the bias added after, IS acc = fma(x_k, W_jk, acc),
// + b_j -- the LIN_SEQ schedule of every call of >= 16 rows.
//
// The layer is computed transposed, D = W' . X^T (16 neurons x 16 rows), so
// a wave's 64 rows are 4 row blocks b of 16 and lane (q = lane >> 4, r =
// lane & 15) holds, in accumulator register g of block b, the neuron
// 4g + q (+ 16 G for output group G) of row 16 b + r: the A operand's row i
// is neuron perm(i) = 4 (i & 3) + (i >> 2).  That is exactly the B operand
// layout of the next layer's K-block s = 4 G + g (input 4 s + q of row r),
// so activations never leave the registers between layers.  An input count
// that is not a multiple of 4 is padded with weight -0 and activation 0:
// fma(-0, 0, acc) = acc for every acc, so the chain is unchanged.
// ---------------------------------------------------------------------------
typedef float mf4 __attribute__((ext_vector_type(4)));
constexpr int MST = 80;  // LDS stage: floats per plane (64 rows + 16: conflict-free transposes)

// LDS hand-over between lanes of ONE wave: every DS op of the wave retires
// in order, so a wait on this wave's own DS ops (and no compiler motion of
// memory ops across it) suffices -- no workgroup barrier
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// acc[G][b] = D of output group G, row block b; act[b][s]: K-block s of row
// block b (B operand); Wl: the layer's weights [16 NG][KI] (row-major, LDS)
template <int KI, int NG, int SMAX>
__device__ __forceinline__ void mfma_layer(const float* Wl, const float (&act)[4][SMAX], mf4 (&acc)[NG][4],
                                           int q, int r) {
  constexpr int S = (KI + 3) / 4;
  static_assert(S <= SMAX, "K-blocks");
#pragma unroll
  for (int G = 0; G < NG; ++G) {
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[G][b] = mf4{0.f, 0.f, 0.f, 0.f};
    const int j = 16 * G + 4 * (r & 3) + (r >> 2);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int k = 4 * s + q;
      const float a = (KI % 4 == 0 || k < KI) ? Wl[j * KI + k] : -0.0f;
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[G][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, act[b][s], acc[G][b], 0, 0, 0);
    }
  }
}

// the layers of an NL-layer net that run on MFMA: hidden widths of 16 or 32
// (TNP_FWD_MFMA=0: variant builds for A/B, every layer on VALU as round 5)
#ifndef TNP_FWD_MFMA
#define TNP_FWD_MFMA 1
#endif
template <int H>
__host__ __device__ constexpr bool mfma_shape() { return TNP_FWD_MFMA && H % 16 == 0; }

template <int LV, int H, int NL>
struct NetShape {
  static constexpr int IN = 2 * LV;
  static constexpr int NW = H * IN + H + (NL - 2) * (H * H + H) + 2 * H + 2;
};

// the net shapes with kernels: levels 2..8 (one translation unit each,
// net_lv.hip), (hidden, layers) below -- K = (layers - 1) hidden + 1 <= 63
// planes fit the 64-bit sign keys
#ifdef TNP_SHAPES_BENCH_ONLY  // experiment builds (tools/): the bench net's shape only, fast to compile
#define TNP_NET_SHAPES(X) X(16, 3)
#define TNP_WIDE_SHAPES(X)
#else
#define TNP_NET_SHAPES(X) X(8, 2) X(8, 3) X(8, 4) X(16, 2) X(16, 3) X(16, 4) X(32, 2)
// wide shapes: K = 65 or 97 planes, two-word sign keys (common.h Key<2>).
// They run everything the K <= 63 shapes run -- the flat and curve subpoly
// paths (the descent included), sharding, faces, Net.forward / sdf / normal
// and the skeleton -- except the training / autograd kernels, which stay
// with TNP_NET_SHAPES
#define TNP_WIDE_SHAPES(X) X(16, 5) X(32, 3) X(32, 4)
#endif
#define TNP_ALL_SHAPES(X) TNP_NET_SHAPES(X) TNP_WIDE_SHAPES(X)
// sign-key words of a net of K planes
__host__ __device__ constexpr int key_words(int K) { return K <= 63 ? 1 : 2; }

}  // namespace tnpnet
