// The curve branch's gradient-descent fallback (deal_with_gradient_descent,
// subpoly_debug.py:121-165): per descending row, 500 iterations of the
// forward at the row's point on its edge, the gradient of d0^2 + d1^2 by
// torch autograd's CPU schedules, a normalised step.  Included by net_lv.hip
// (one translation unit per level count, every hidden/layer shape of
// TNP_ALL_SHAPES: lv_descend), launched by curve.hip launch_descend.
#pragma once
#include "common.h"
#include "kernels.h"
#include "net_device.h"

namespace {

using namespace tnpnet;

// The 1-row products of the descent's backward, mm(g[1 x K], W[K x M])
// (AddmmBackward, subpoly_debug.py:143-148) as x86 MKL sgemm sums them on
// CPU (tools/mkl_backward_probe.py, bitwise against torch.mm): with M a
// multiple of 16 the K = 8 k inputs go through this tree, pr(a, b) =
// fma(x_a, w_a, x_b * w_b):
//   ((pr(0,2) + pr(1,3)) + (pr(4,6) + pr(5,7))), then per further block of
//   8 at s: fma x_{s+6}, fma x_{s+4}, + pr(s+5, s+7), + (pr(s,s+2) + pr(s+1,s+3));
// any other M, and every multi-row call, is a sequential fma chain from 0.
template <int K>
__device__ __forceinline__ float mm1_tree(const float* x, const float* W, int ld, int k) {
  static_assert(K % 8 == 0, "the tree takes blocks of 8 inputs");
  auto pr = [&](int a, int b) {  // fma(x_a, w_a, x_b * w_b)
    return __fmaf_rn(x[a], W[a * ld + k], __fmul_rn(x[b], W[b * ld + k]));
  };
  float v = __fadd_rn(__fadd_rn(pr(0, 2), pr(1, 3)), __fadd_rn(pr(4, 6), pr(5, 7)));
#pragma unroll
  for (int s = 8; s < K; s += 8) {
    v = __fmaf_rn(x[s + 6], W[(s + 6) * ld + k], v);
    v = __fmaf_rn(x[s + 4], W[(s + 4) * ld + k], v);
    v = __fadd_rn(v, pr(s + 5, s + 7));
    v = __fadd_rn(v, __fadd_rn(pr(s, s + 2), pr(s + 1, s + 3)));
  }
  return v;
}
// column k of mm(g[rows x K], W[K x M]) (W row-major, leading dimension M)
template <int K, int M>
__device__ __forceinline__ float mm_col(const float* x, const float* W, int k, bool one_row) {
  if constexpr (M % 16 == 0 && K % 8 == 0)
    if (one_row) return mm1_tree<K>(x, W, M, k);
  float v = 0.f;
#pragma unroll
  for (int j = 0; j < K; ++j) v = __fmaf_rn(x[j], W[j * M + k], v);
  return v;
}

// pre-activations of planes j0, j1 at u (preprocessed) and d(d0^2 + d1^2)/du
// exactly as torch autograd computes it on CPU for a G-row batch
// (subpoly_debug.py:143-148): forward with MKL's G-row schedules, backward
// through AddmmBackward (mm(grad, W): mm_col), threshold_backward, and the
// encoding's input gradient (oracle/encoding.py _GridFn.backward op order).
template <int LV, int H, int NL>
__device__ __forceinline__ void plane_pair_grad(const NetDev& net, const float* w, const float u[3],
                                                int j0, int j1, int m0, int mh, int mo, bool one_row,
                                                int64_t row, float& d0, float& d1, float gu[3]) {
  constexpr int IN = 2 * LV;
  constexpr int NH = NL - 1;
  float f[IN], a[NH][H], h[H], o[2];
  encode<LV>(net, u, f);
  const float* Wl[NH];
  Wl[0] = w;
#pragma unroll
  for (int l = 1; l < NH; ++l) Wl[l] = Wl[l - 1] + (l == 1 ? H * IN + H : H * H + H);
  const float* WL = Wl[NH - 1] + (NH == 1 ? H * IN + H : H * H + H);
  // row: the row's index in the batch (the 32-input FOLD schedule's parity)
  linear_mode<IN, H>(Wl[0], Wl[0] + H * IN, f, a[0], m0, row);
#pragma unroll
  for (int j = 0; j < H; ++j) h[j] = fmaxf(a[0][j], 0.f);
#pragma unroll
  for (int l = 1; l < NH; ++l) {
    linear_mode<H, H>(Wl[l], Wl[l] + H * H, h, a[l], mh, row);
#pragma unroll
    for (int j = 0; j < H; ++j) h[j] = fmaxf(a[l][j], 0.f);
  }
  linear_mode<H, 2>(WL, WL + 2 * H, h, o, mo, row);
  float last = __fsub_rn(o[1], o[0]);
  d0 = last;
  d1 = last;
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int k = 0; k < H; ++k) {
      if (j0 == l * H + k) d0 = a[l][k];
      if (j1 == l * H + k) d1 = a[l][k];
    }
  // seeds of y = d0^2 + d1^2 on the gathered pre-activations (2 d, exact)
  float g[NH][H], go = 0.f;
#pragma unroll
  for (int l = 0; l < NH; ++l)
#pragma unroll
    for (int k = 0; k < H; ++k) g[l][k] = 0.f;
  const int js[2] = {j0, j1};
  const float ds[2] = {d0, d1};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float gs = __fmul_rn(2.f, ds[s]);
    int j = js[s];
#pragma unroll
    for (int l = 0; l < NH; ++l)
#pragma unroll
      for (int k = 0; k < H; ++k)
        if (j == l * H + k) g[l][k] = __fadd_rn(g[l][k], gs);
    if (j == NH * H) go = __fadd_rn(go, gs);
  }
  // last layer (o1 - o0): mm([-go, go], W), K = 2 sequential fma; ReLU
#pragma unroll
  for (int k = 0; k < H; ++k) {
    float v = __fmaf_rn(go, WL[H + k], __fmul_rn(-go, WL[k]));
    if (a[NH - 1][k] > 0.f) g[NH - 1][k] = __fadd_rn(g[NH - 1][k], v);
  }
  // hidden H x H layers, top down: mm(g_a, W) ; ReLU
#pragma unroll
  for (int l = NH - 1; l >= 1; --l) {
    float gp[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      const float v = mm_col<H, H>(g[l], Wl[l], k, one_row);
      gp[k] = a[l - 1][k] > 0.f ? __fadd_rn(g[l - 1][k], v) : g[l - 1][k];
    }
#pragma unroll
    for (int k = 0; k < H; ++k) g[l - 1][k] = gp[k];
  }
  // first layer: mm(g_a0, W0)
  const float* W0 = Wl[0];
  float df[IN];
#pragma unroll
  for (int m = 0; m < IN; ++m) df[m] = mm_col<H, IN>(g[0], W0, m, one_row);
  // encoding input gradient: per level, per corner, per dim
  //   gx_d += (((sgn * f_e0) * f_e1) * dv) * scale,  dv = val . g_feat
  float gx[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < LV; ++l) {
    const float sc = net.scales[l];
    float t[3];
    uint32_t gi[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float pos = __fadd_rn(__fmul_rn(u[d], sc), 0.5f);
      float fl = floorf(pos);
      t[d] = __fsub_rn(pos, fl);
      gi[d] = (uint32_t)(int)fl;
    }
    const uint32_t res = (uint32_t)net.res[l];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float fc[3];
      uint32_t gc[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        bool up = (c >> d) & 1;
        fc[d] = up ? t[d] : __fsub_rn(1.f, t[d]);
        gc[d] = gi[d] + (up ? 1u : 0u);
      }
      uint32_t id = net.dense[l] ? (gc[0] + gc[1] * res + gc[2] * (res * res))
                                 : (gc[0] ^ (gc[1] * P1) ^ (gc[2] * P2));
      id = wrap_index(id, net.sizes[l]);
      float2 v = table_entry(net, l, id);
      float dv = __fadd_rn(__fmul_rn(v.x, df[2 * l]), __fmul_rn(v.y, df[2 * l + 1]));
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        float sg = ((c >> d) & 1) ? 1.f : -1.f;
        float fa = fc[d == 0 ? 1 : 0], fb = fc[d == 2 ? 1 : 2];
        gx[d] = __fadd_rn(gx[d], __fmul_rn(__fmul_rn(__fmul_rn(__fmul_rn(sg, fa), fb), dv), sc));
      }
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) gu[d] = gx[d];
}

// deal_with_gradient_descent (subpoly_debug.py:121-165), one thread per row.
// record != 0: AND this row's per-iteration "both residuals <= eps" bits into
// conv[0..7] (iteration i -> bit i) so the host finds the common stop.
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK)
k_descend(NetDev net, int64_t G, const int32_t* __restrict__ glist,
          const int32_t* __restrict__ crow, const int32_t* __restrict__ sa,
          const int32_t* __restrict__ sb, const float* __restrict__ xyz,
          const int32_t* __restrict__ plane, int idx, float eps, int iters, int record,
          float* __restrict__ ints, float* __restrict__ d0s, float* __restrict__ d1s,
          unsigned long long* __restrict__ conv) {
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  __syncthreads();
  int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  int b = glist[g];
  int r = crow[b];
  float e0[3], de[3], x[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    e0[d] = xyz[3 * (int64_t)sa[r] + d];
    de[d] = __fsub_rn(xyz[3 * (int64_t)sb[r] + d], e0[d]);
    x[d] = ints[3 * b + d];
  }
  const int j0 = plane[b];
  const int64_t Gs = net.sched_rows > 0 ? net.sched_rows : G;  // the schedule's row count (sharded: global)
  const int m0 = lin_mode<2 * LV, H>(Gs), mh = lin_mode<H, H>(Gs), mo = lin_mode<H, 2>(Gs);
  uint64_t bits[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float d0 = 1.f, d1 = 1.f;
  for (int it = 0; it < iters; ++it) {
    float u[3], gu[3];
#pragma unroll
    for (int d = 0; d < 3; ++d)
      u[d] = __fmul_rn(__fadd_rn(__fadd_rn(e0[d], __fmul_rn(x[d], de[d])), 1.0f), 0.5f);  // x/2 == x*0.5
    plane_pair_grad<LV, H, NL>(net, w, u, j0, idx, m0, mh, mo, Gs == 1, g, d0, d1, gu);
    float gx[3], nn = 0.f;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      gx[d] = __fmul_rn(__fmul_rn(gu[d], 0.5f), de[d]);
      nn = __fmaf_rn(gx[d], gx[d], nn);
    }
    float den = fmaxf(sqrtf(nn), 1e-12f);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float v = __fsub_rn(x[d], __fmul_rn(1e-2f, __fdiv_rn(gx[d], den)));
      x[d] = fminf(fmaxf(v, 0.f), 1.f);
    }
    if (record && fabsf(d0) <= eps && fabsf(d1) <= eps) bits[it >> 6] |= 1ull << (it & 63);
  }
  if (record)
    for (int k = 0; k < 8; ++k) atomicAnd(&conv[k], (unsigned long long)bits[k]);
#pragma unroll
  for (int d = 0; d < 3; ++d) ints[3 * b + d] = x[d];
  d0s[b] = d0;
  d1s[b] = d1;
}

__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// every lane's v -> out[0..N) in every lane, through LDS (one wave per
// workgroup: its LDS accesses complete in program order, so no barrier; the
// slot array's aliasing keeps the compiler's order).  Replaces N v_readlane
// round trips (each with its SGPR hazard wait, and the SGPRs they fill
// spilled to VGPR lanes) by one store and N/4 broadcast loads.
template <int N>
__device__ __forceinline__ void wave_bcast(float v, float (&out)[N], float* slot) {
  slot[threadIdx.x] = v;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < N; ++j) out[j] = slot[j];
  __builtin_amdgcn_wave_barrier();
}

// The same descent with ONE WAVE PER ROW: the 500 iterations are strictly
// sequential, so a row's latency per iteration is the whole cost (one thread
// per row left a lone wave issuing ~4k dependent instructions per
// iteration).  Here lane q holds hash-grid corner q & 7 of level q >> 3 (its
// table entry is gathered once per iteration and reused by the backward
// pass) and lane j < H neuron j of each layer; every sum keeps the
// single-thread order above -- corner sums, sequential fma chains, the
// 1-row 16 x 16 tree -- over operands broadcast through LDS (wave_bcast), so
// the result is bitwise that of k_descend.
template <int LV, int H, int NL>
__global__ void __launch_bounds__(64)
k_descend_wave(NetDev net, int64_t G, const int32_t* __restrict__ glist,
               const int32_t* __restrict__ crow, const int32_t* __restrict__ sa,
               const int32_t* __restrict__ sb, const float* __restrict__ xyz,
               const int32_t* __restrict__ plane, int idx, float eps, int iters, int record,
               float* __restrict__ ints, float* __restrict__ d0s, float* __restrict__ d1s,
               unsigned long long* __restrict__ conv) {
  static_assert(LV * 8 <= 64 && H <= 64, "one wave holds every corner and neuron");
  constexpr int IN = 2 * LV;
  constexpr int NH = NL - 1;
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  __syncthreads();
  const int64_t g = blockIdx.x;
  if (g >= G) return;
  const int lane = threadIdx.x;
  const int b = glist[g];
  const int r = crow[b];
  float e0[3], de[3], x[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    e0[d] = xyz[3 * (int64_t)sa[r] + d];
    de[d] = __fsub_rn(xyz[3 * (int64_t)sb[r] + d], e0[d]);
    x[d] = ints[3 * b + d];
  }
  const int j0 = plane[b];
  const int64_t Gs = net.sched_rows > 0 ? net.sched_rows : G;  // the schedule's row count (sharded: global)
  const int m0 = lin_mode<IN, H>(Gs), mh = lin_mode<H, H>(Gs), mo = lin_mode<H, 2>(Gs);
  const bool one_row = Gs == 1;
  // lane roles
  const int nj = lane & (H - 1);                      // neuron
  const int lc = min(lane >> 3, LV - 1), c = lane & 7;  // corner c of level lc
  float sc = 0.f;
  uint32_t res = 0, size = 1;
  bool dense = false;
#pragma unroll
  for (int l = 0; l < LV; ++l)
    if (l == lc) {
      sc = net.scales[l];
      res = (uint32_t)net.res[l];
      size = net.sizes[l];
      dense = net.dense[l] != 0;
    }
  const float* Wl[NH];
  Wl[0] = w;
#pragma unroll
  for (int l = 1; l < NH; ++l) Wl[l] = Wl[l - 1] + (l == 1 ? H * IN + H : H * H + H);
  const float* WL = Wl[NH - 1] + (NH == 1 ? H * IN + H : H * H + H);
  // broadcast slots (wave_bcast): rows 0..2 the corner / gradient sums, rows
  // 3..3+NH-1 the hidden layers' pre-activations (read again for d0 / d1),
  // row 3+NH the two outputs
  __shared__ __attribute__((aligned(16))) float bc[4 + NH][64];
  uint64_t word = 0;  // convergence bits of iterations [64 k, 64 k + 64)
  float d0 = 1.f, d1 = 1.f;
  // this lane's table entry of the last iteration: the point moves by ~1e-2
  // of its edge per iteration, so its corners mostly stay those of the
  // iteration before -- a lane gathers only when its corner id changes, and
  // a wave whose lanes all hit skips the iteration's one dependent memory
  // round trip (same values: the table is constant over the descent)
  uint32_t cid = 0xFFFFFFFFu;  // (wrap_index < size <= 2^31: never an id)
  float2 cv = make_float2(0.f, 0.f);
  for (int it = 0; it < iters; ++it) {
    float u[3];
#pragma unroll
    for (int d = 0; d < 3; ++d)
      u[d] = __fmul_rn(__fadd_rn(__fadd_rn(e0[d], __fmul_rn(x[d], de[d])), 1.0f), 0.5f);  // x/2 == x*0.5
    // this lane's corner (encode's op order)
    float t[3];
    uint32_t gc[3];
    float wc = 1.0f;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float pos = __fadd_rn(__fmul_rn(u[d], sc), 0.5f);
      const float fl = floorf(pos);
      t[d] = __fsub_rn(pos, fl);
      const uint32_t gi = (uint32_t)(int)fl;
      if ((c >> d) & 1) {
        wc = __fmul_rn(wc, t[d]);
        gc[d] = gi + 1u;
      } else {
        wc = __fmul_rn(wc, __fsub_rn(1.0f, t[d]));
        gc[d] = gi;
      }
    }
    uint32_t id = dense ? (gc[0] + gc[1] * res + gc[2] * (res * res)) : (gc[0] ^ (gc[1] * P1) ^ (gc[2] * P2));
    id = wrap_index(id, size);
    if (id != cid) {
      cv = table_entry(net, lc, id);
      cid = id;
    }
    const float2 v = cv;
    const float px = __fmul_rn(wc, v.x), py = __fmul_rn(wc, v.y);
    float f[IN];
    {
      float cx[8 * LV], cy[8 * LV];
      wave_bcast<8 * LV>(px, cx, bc[0]);
      wave_bcast<8 * LV>(py, cy, bc[1]);
#pragma unroll
      for (int l = 0; l < LV; ++l) {
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          a0 = __fadd_rn(a0, cx[8 * l + k]);
          a1 = __fadd_rn(a1, cy[8 * l + k]);
        }
        f[2 * l] = a0;
        f[2 * l + 1] = a1;
      }
    }
    // forward, neuron nj per lane; a[l]: this lane's neuron of hidden layer l
    // (ab[l]: layer l's H pre-activations, in every lane)
    float a[NH];
    float ab[NH][H];
    float hh[H];
    a[0] = neuron_mode<IN, H>(Wl[0], Wl[0] + H * IN, f, nj, m0, g);
#pragma unroll
    for (int l = 1; l < NH; ++l) {
      wave_bcast<H>(a[l - 1], ab[l - 1], bc[3 + l - 1]);
#pragma unroll
      for (int j = 0; j < H; ++j) hh[j] = fmaxf(ab[l - 1][j], 0.f);
      a[l] = neuron_mode<H, H>(Wl[l], Wl[l] + H * H, hh, nj, mh, g);
    }
    wave_bcast<H>(a[NH - 1], ab[NH - 1], bc[3 + NH - 1]);
#pragma unroll
    for (int j = 0; j < H; ++j) hh[j] = fmaxf(ab[NH - 1][j], 0.f);
    const float o = neuron_mode<H, 2>(WL, WL + 2 * H, hh, lane & 1, mo, g);
    float ob[2];
    wave_bcast<2>(o, ob, bc[3 + NH]);
    const float last = __fsub_rn(ob[1], ob[0]);
    // the two planes' values: a hidden pre-activation (row 3 + layer, slot
    // neuron; uniform indices) or the output
    d0 = j0 < NH * H ? bc[3 + j0 / H][j0 % H] : last;
    d1 = idx < NH * H ? bc[3 + idx / H][idx % H] : last;
    // backward: seeds of d0^2 + d1^2, neuron nj per lane
    float gl[NH], go = 0.f;
#pragma unroll
    for (int l = 0; l < NH; ++l) gl[l] = 0.f;
    {
      const int js[2] = {j0, idx};
      const float ds[2] = {d0, d1};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float gs = __fmul_rn(2.f, ds[s]);
#pragma unroll
        for (int l = 0; l < NH; ++l)
          if (js[s] == l * H + nj) gl[l] = __fadd_rn(gl[l], gs);
        if (js[s] == NH * H) go = __fadd_rn(go, gs);
      }
    }
    const float v3 = __fmaf_rn(go, WL[H + nj], __fmul_rn(-go, WL[nj]));
    if (a[NH - 1] > 0.f) gl[NH - 1] = __fadd_rn(gl[NH - 1], v3);
#pragma unroll
    for (int l = NH - 1; l >= 1; --l) {
      float gu_[H];
      wave_bcast<H>(gl[l], gu_, bc[0]);
      const float v2 = mm_col<H, H>(gu_, Wl[l], nj, one_row);
      gl[l - 1] = a[l - 1] > 0.f ? __fadd_rn(gl[l - 1], v2) : gl[l - 1];
    }
    float ga1u[H];
    wave_bcast<H>(gl[0], ga1u, bc[2]);  // (rows 0 / 2 alternate: a row is rewritten only after its reads)
    const float* W0 = Wl[0];
    const int m = lane % IN;
    const float dfm = mm_col<H, IN>(ga1u, W0, m, one_row);
    // encoding input gradient, this lane's corner; sums in (level, corner) order
    float dfa, dfb;
    bc[1][lane] = dfm;  // (this lane's level lc: its two input gradients)
    __builtin_amdgcn_wave_barrier();
    dfa = bc[1][2 * lc];
    dfb = bc[1][2 * lc + 1];
    __builtin_amdgcn_wave_barrier();
    const float dv = __fadd_rn(__fmul_rn(v.x, dfa), __fmul_rn(v.y, dfb));
    float fc[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) fc[d] = ((c >> d) & 1) ? t[d] : __fsub_rn(1.f, t[d]);
    float term[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float sg = ((c >> d) & 1) ? 1.f : -1.f;
      const float fa = fc[d == 0 ? 1 : 0], fb = fc[d == 2 ? 1 : 2];
      term[d] = __fmul_rn(__fmul_rn(__fmul_rn(__fmul_rn(sg, fa), fb), dv), sc);
    }
    float gx[3], nn = 0.f;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float tq[8 * LV];
      wave_bcast<8 * LV>(term[d], tq, bc[d]);
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < 8 * LV; ++q) acc = __fadd_rn(acc, tq[q]);
      gx[d] = __fmul_rn(__fmul_rn(acc, 0.5f), de[d]);
      nn = __fmaf_rn(gx[d], gx[d], nn);
    }
    const float den = fmaxf(sqrtf(nn), 1e-12f);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float vv = __fsub_rn(x[d], __fmul_rn(1e-2f, __fdiv_rn(gx[d], den)));
      x[d] = fminf(fmaxf(vv, 0.f), 1.f);
    }
    if (record && fabsf(d0) <= eps && fabsf(d1) <= eps) word |= 1ull << (it & 63);
    if ((it & 63) == 63 || it == iters - 1) {
      if (record && lane == 0) atomicAnd(&conv[it >> 6], (unsigned long long)word);
      word = 0;
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < 3; ++d) ints[3 * b + d] = x[d];
    d0s[b] = d0;
    d1s[b] = d1;
  }
}


}  // namespace
