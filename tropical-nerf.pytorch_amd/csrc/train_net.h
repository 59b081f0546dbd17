// Parameter gradients of the net for training and autograd, every
// instantiated shape (TNP_NET_SHAPES x levels 2..8): included by net_lv.hip
// (one translation unit per level count: lv_train, lv_forward_vjp).
//
// Loss of one training batch of n points x (train.py:181-201, Net.sdf =
// tanh(o1 - o0), model.py:84-87):
//   L1  = mean_i |clamp(y_i) - clamp(gt_i)|,   clamp to [-T, T] (T = 0.2)
//   Eik = w_e (||J||_F - 1)^2 / B,   J_i = d y_i / d x_i   (w_e = 1e-2, B = BATCH_SIZE)
// The reference gets dEik/dtheta by double backward through tcnn; here it is
// written out.  With z = o1 - o0, g = dz/dx, y = tanh z and an upstream
// v_i = dL/dJ_i (the eikonal's w_e 2 (||J|| - 1) / (B ||J||) J_i, or any
// caller's for Net.normal(create_graph=True)):
//   v.J = (1 - y^2) q,  q = v.g = u . a,
//   u = dz/de (the encoding's output), a = (1/2) sum_c T_c (grad w_c . v)
// -- q is the derivative of z along the direction a in feature space, so its
// parameter gradient is a forward-mode pass along a (the ReLU net is
// piecewise linear: no second-order term), and every parameter's gradient is
//   kappa dz/dtheta + mu dq/dtheta,   kappa = (1 - y^2)(rho - 2 y q),
//   mu = 1 - y^2,   rho = dL/dy of the other terms (L1: sign(clamp y - clamp gt) / n):
//   W_l += delta_l (kappa h_{l-1} + mu h'_{l-1})^T,  b_l += kappa delta_l
//   (h_{-1} = e, h'_{-1} = a; delta_l = dz/d(pre-activation of layer l);
//   h'_l = D_l W_l h'_{l-1}; the output layer: W[1] = -W[0] += kappa h + mu h')
//   T[l, c, f] += u_{l,f} (kappa w_c + mu (1/2) grad w_c . v)
// Summation order is not part of the bitwise contract here (training and
// autograd are held to a float64 oracle, oracle/train.py): MLP terms are
// reduced per wave, then per block in LDS, one global atomic per parameter
// per block; table terms are global float atomics.
#pragma once
#include "common.h"
#include "kernels.h"
#include "net_device.h"

namespace {

using namespace tnpnet;

// trilinear corner c of level l at x' (preprocessed, [0,1]^3): weight,
// weight gradient d w_c / d x' and the float2 entry index
struct TCorner {
  float w;
  float dw[3];
  float f[3];  // the per-axis factors (up ? t : 1 - t)
  uint32_t idx;
};

__device__ __forceinline__ TCorner tcorner_of(const NetDev& net, int l, const float t[3], const uint32_t g[3],
                                              int c) {
  const float s = net.scales[l];
  uint32_t gc[3];
  TCorner r;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const bool up = (c >> d) & 1;
    r.f[d] = up ? t[d] : 1.f - t[d];
    gc[d] = g[d] + (up ? 1u : 0u);
  }
  r.w = r.f[0] * r.f[1] * r.f[2];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float sg = ((c >> d) & 1) ? 1.f : -1.f;
    r.dw[d] = sg * r.f[(d + 1) % 3] * r.f[(d + 2) % 3] * s;
  }
  const uint32_t res = (uint32_t)net.res[l];
  uint32_t idx = net.dense[l] ? (gc[0] + gc[1] * res + gc[2] * (res * res)) : (gc[0] ^ (gc[1] * P1) ^ (gc[2] * P2));
  r.idx = net.offsets[l] + wrap_index(idx, net.sizes[l]);
  return r;
}

__device__ __forceinline__ void tcell_of(const NetDev& net, int l, const float x[3], float t[3], uint32_t g[3]) {
  const float s = net.scales[l];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float pos = x[d] * s + 0.5f;
    const float fl = floorf(pos);
    t[d] = pos - fl;
    g[d] = (uint32_t)(int)fl;
  }
}

// packed weights of layer l (NetShape layout: W0, b0, W1, b1, ..., WL, bL)
template <int LV, int H, int NL>
__device__ __forceinline__ const float* layer_w(const float* w, int l) {
  constexpr int IN = 2 * LV;
  return l == 0 ? w : w + H * IN + H + (l - 1) * (H * H + H);
}

// the forward of one point and dz/d(pre-activations), dz/de, dz/dx
template <int LV, int H, int NL>
struct TPass {
  static constexpr int IN = 2 * LV;
  static constexpr int NH = NL - 1;  // hidden layers
  float e[IN], a[NH][H], d[NH][H], u[IN];
  float z, y;
  float gz[3];  // dz/dx (x in [-1, 1]: the (x + 1) / 2 preprocess halves it)

  __device__ __forceinline__ float h(int l, int j) const { return fmaxf(a[l][j], 0.f); }

  __device__ __forceinline__ void run(const NetDev& net, const float* w, const float x[3]) {
    const float2* tab = reinterpret_cast<const float2*>(net.table);
#pragma unroll
    for (int l = 0; l < LV; ++l) {
      float t[3];
      uint32_t g[3];
      tcell_of(net, l, x, t, g);
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const TCorner k = tcorner_of(net, l, t, g, c);
        const float2 v = tab[k.idx];
        s0 += k.w * v.x;
        s1 += k.w * v.y;
      }
      e[2 * l] = s0;
      e[2 * l + 1] = s1;
    }
    linear<IN, H>(w, w + H * IN, e, a[0]);
#pragma unroll
    for (int l = 1; l < NH; ++l) {
      const float* Wl = layer_w<LV, H, NL>(w, l);
      float hp[H];
#pragma unroll
      for (int k = 0; k < H; ++k) hp[k] = h(l - 1, k);
      linear<H, H>(Wl, Wl + H * H, hp, a[l]);
    }
    const float* WL = layer_w<LV, H, NL>(w, NH);
    float hl[H], o[2];
#pragma unroll
    for (int k = 0; k < H; ++k) hl[k] = h(NH - 1, k);
    linear<H, 2>(WL, WL + 2 * H, hl, o);
    z = o[1] - o[0];
    y = tanhf(z);
#pragma unroll
    for (int j = 0; j < H; ++j) d[NH - 1][j] = a[NH - 1][j] > 0.f ? WL[H + j] - WL[j] : 0.f;
#pragma unroll
    for (int l = NH - 1; l >= 1; --l) {
      const float* Wl = layer_w<LV, H, NL>(w, l);
#pragma unroll
      for (int k = 0; k < H; ++k) {
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < H; ++j) v += d[l][j] * Wl[j * H + k];
        d[l - 1][k] = a[l - 1][k] > 0.f ? v : 0.f;
      }
    }
#pragma unroll
    for (int m = 0; m < IN; ++m) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < H; ++k) v += d[0][k] * w[k * IN + m];
      u[m] = v;
    }
    gz[0] = gz[1] = gz[2] = 0.f;
#pragma unroll
    for (int l = 0; l < LV; ++l) {
      float t[3];
      uint32_t g[3];
      tcell_of(net, l, x, t, g);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const TCorner k = tcorner_of(net, l, t, g, c);
        const float2 v = tab[k.idx];
        const float dv = v.x * u[2 * l] + v.y * u[2 * l + 1];
#pragma unroll
        for (int q = 0; q < 3; ++q) gz[q] += k.dw[q] * dv;
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) gz[q] *= 0.5f;
  }
};

__device__ __forceinline__ float clamp_t(float v, float T) { return fminf(fmaxf(v, -T), T); }

// one parameter's per-lane terms: wave sum, then the block's LDS slot
__device__ __forceinline__ void acc_param(float* lds_g, int p, float v) {
  v = tnp::wave_sum(v);
  if (tnp::lane() == 0 && v != 0.f) atomicAdd(&lds_g[p], v);
}

// training pass 1: sum_i |clamp(y_i) - clamp(gt_i)| -> stats[0], sum_i ||J_i||^2 -> stats[1]
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK)
k_train_norms(NetDev net, const float* __restrict__ xyz, const float* __restrict__ gt, int64_t n, float T,
              double* __restrict__ stats) {
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double l1 = 0.0, j2 = 0.0;
  if (i < n) {
    float x[3];
    load_point(xyz, i, x);
    TPass<LV, H, NL> p;
    p.run(net, w, x);
    const float ty = 1.f - p.y * p.y;
    l1 = fabsf(clamp_t(p.y, T) - clamp_t(gt[i], T));
#pragma unroll
    for (int d = 0; d < 3; ++d) j2 += (double)(ty * p.gz[d]) * (ty * p.gz[d]);
  }
  l1 = tnp::wave_sum(l1);
  j2 = tnp::wave_sum(j2);
  if (tnp::lane() == 0) {
    atomicAdd(&stats[0], l1);
    atomicAdd(&stats[1], j2);
  }
}

// The parameter gradient (header comment), three modes:
//   training   (gout, gJ null): the L1 + eikonal terms of one batch (stats: pass 1)
//   sdf VJP    (gout):  sum_i gout_i d y_i / d theta            (kappa = (1 - y^2) gout_i, mu = 0)
//   normal VJP (gJ):    sum_i gJ_i . d J_i / d theta            (v_i = gJ_i, rho = 0)
//                       and, with g_x, sum_i gJ_i . d J_i / d x_i (the Hessian of y along gJ_i)
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK)
k_train_grads(NetDev net, const float* __restrict__ xyz, const float* __restrict__ gt, int64_t n, float T,
              float eik_w, int64_t eik_batch, const double* __restrict__ stats, float* __restrict__ g_table,
              float* __restrict__ g_w, const float* __restrict__ gout, const float* __restrict__ gJ,
              float* __restrict__ g_x) {
  constexpr int IN = 2 * LV;
  constexpr int NH = NL - 1;
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  __shared__ float gw[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) {
    w[i] = net.weights[i];
    gw[i] = 0.f;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n;
  float x[3] = {0.5f, 0.5f, 0.5f};
  if (live) load_point(xyz, i, x);
  TPass<LV, H, NL> p;
  p.run(net, w, x);
  const float ty = 1.f - p.y * p.y;
  float v[3] = {0.f, 0.f, 0.f};
  if (gJ) {
    if (live)
#pragma unroll
      for (int d = 0; d < 3; ++d) v[d] = gJ[3 * i + d];
  } else if (!gout) {
    // v_i = c J_i, c = w_e 2 (||J|| - 1) / (B ||J||), B = BATCH_SIZE (train.py:197;
    // the L1 mean below divides by the actual n)   (torch: a zero norm has a zero gradient)
    const double nj = sqrt(stats[1]);
    const float c = nj > 0.0 ? (float)(eik_w * 2.0 * (nj - 1.0) / ((double)eik_batch * nj)) : 0.f;
#pragma unroll
    for (int d = 0; d < 3; ++d) v[d] = c * ty * p.gz[d];
  }
  const float q = v[0] * p.gz[0] + v[1] * p.gz[1] + v[2] * p.gz[2];
  float rho = 0.f;
  if (!gout && !gJ && live && p.y >= -T && p.y <= T) {
    const float r = clamp_t(p.y, T) - clamp_t(gt[i], T);
    rho = (r > 0.f ? 1.f : (r < 0.f ? -1.f : 0.f)) / (float)n;
  }
  const float kappa = !live ? 0.f : (gout ? ty * gout[i] : ty * (rho - 2.f * p.y * q));
  const float mu = (live && !gout) ? ty : 0.f;
  // direction a = (1/2) sum_c T_c (grad w_c . v), the table terms, and (g_x)
  // the Hessian of z along v: 1/4 sum_c (T_c . u) (grad^2 w_c) v
  const float2* tab = reinterpret_cast<const float2*>(net.table);
  float a[IN];
  float hz[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < LV; ++l) {
    float t[3];
    uint32_t g[3];
    tcell_of(net, l, x, t, g);
    const float s = net.scales[l];
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      const TCorner k = tcorner_of(net, l, t, g, cc);
      const float gv = 0.5f * (k.dw[0] * v[0] + k.dw[1] * v[1] + k.dw[2] * v[2]);
      const float2 e2 = tab[k.idx];
      s0 += e2.x * gv;
      s1 += e2.y * gv;
      const float coef = kappa * k.w + mu * gv;
      if (live && coef != 0.f) {
        if (p.u[2 * l] != 0.f) unsafeAtomicAdd(&g_table[2 * (size_t)k.idx], p.u[2 * l] * coef);
        if (p.u[2 * l + 1] != 0.f) unsafeAtomicAdd(&g_table[2 * (size_t)k.idx + 1], p.u[2 * l + 1] * coef);
      }
      if (g_x) {
        // d^2 w_c / dx'_q dx'_r = sg_q sg_r s^2 f_other (q != r), 0 on the diagonal
        const float tu = e2.x * p.u[2 * l] + e2.y * p.u[2 * l + 1];
#pragma unroll
        for (int qd = 0; qd < 3; ++qd) {
          float hv = 0.f;
#pragma unroll
          for (int rd = 0; rd < 3; ++rd) {
            if (rd == qd) continue;
            const int od = 3 - qd - rd;
            const float sq = ((cc >> qd) & 1) ? 1.f : -1.f, sr = ((cc >> rd) & 1) ? 1.f : -1.f;
            hv += sq * sr * s * s * k.f[od] * v[rd];
          }
          hz[qd] += tu * hv;
        }
      }
    }
    a[2 * l] = s0;
    a[2 * l + 1] = s1;
  }
  if (g_x && live) {
    // d (v . J) / dx = (1 - y^2) (H_z v) - 2 y (1 - y^2) (g . v) g,  H_z = 1/4 (d^2 z / dx'^2)
#pragma unroll
    for (int d = 0; d < 3; ++d) g_x[3 * i + d] += ty * 0.25f * hz[d] - 2.f * p.y * ty * q * p.gz[d];
  }
  // tangent activations along a: hd[l] = D_l W_l hd[l - 1], hd[-1] = a
  float hd[NH][H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < IN; ++m) s += w[k * IN + m] * a[m];
    hd[0][k] = p.a[0][k] > 0.f ? s : 0.f;
  }
#pragma unroll
  for (int l = 1; l < NH; ++l) {
    const float* Wl = layer_w<LV, H, NL>(w, l);
#pragma unroll
    for (int j = 0; j < H; ++j) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < H; ++k) s += Wl[j * H + k] * hd[l - 1][k];
      hd[l][j] = p.a[l][j] > 0.f ? s : 0.f;
    }
  }
  // packed gradient layout = packed weight layout (fc.0.weight, fc.0.bias, ...)
  int o = 0;
#pragma unroll
  for (int k = 0; k < H; ++k)
#pragma unroll
    for (int m = 0; m < IN; ++m) acc_param(gw, o + k * IN + m, p.d[0][k] * (kappa * p.e[m] + mu * a[m]));
  o += H * IN;
#pragma unroll
  for (int k = 0; k < H; ++k) acc_param(gw, o + k, kappa * p.d[0][k]);
  o += H;
#pragma unroll
  for (int l = 1; l < NH; ++l) {
#pragma unroll
    for (int j = 0; j < H; ++j)
#pragma unroll
      for (int k = 0; k < H; ++k)
        acc_param(gw, o + j * H + k, p.d[l][j] * (kappa * p.h(l - 1, k) + mu * hd[l - 1][k]));
    o += H * H;
#pragma unroll
    for (int j = 0; j < H; ++j) acc_param(gw, o + j, kappa * p.d[l][j]);
    o += H;
  }
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const float r = kappa * p.h(NH - 1, j) + mu * hd[NH - 1][j];
    acc_param(gw, o + j, -r);
    acc_param(gw, o + H + j, r);
  }
  o += 2 * H;
  acc_param(gw, o, -kappa);
  acc_param(gw, o + 1, kappa);
  __syncthreads();
  for (int k = threadIdx.x; k < NW; k += blockDim.x)
    if (gw[k] != 0.f) unsafeAtomicAdd(&g_w[k], gw[k]);
}

// VJP of Net.forward(x, gather=True) (model.py:52-76): upstream gradients of
// the gathered pre-activations (plane-major gpl[K][ld]: the hidden layers'
// pre-activations, then o1 - o0) and of the output gout2[n][2] (either may
// be null) -> the table, the packed fc parameters and (g_x) the points
template <int LV, int H, int NL>
__global__ void __launch_bounds__(TNP_BLOCK)
k_forward_vjp(NetDev net, const float* __restrict__ xyz, int64_t n, const float* __restrict__ gpl, int64_t ld,
              const float* __restrict__ gout2, float* __restrict__ g_table, float* __restrict__ g_w,
              float* __restrict__ g_x) {
  constexpr int IN = 2 * LV;
  constexpr int NH = NL - 1;
  constexpr int NW = NetShape<LV, H, NL>::NW;
  __shared__ float w[NW];
  __shared__ float gw[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) {
    w[i] = net.weights[i];
    gw[i] = 0.f;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n;
  float x[3] = {0.5f, 0.5f, 0.5f};
  if (live) load_point(xyz, i, x);
  TPass<LV, H, NL> p;
  p.run(net, w, x);  // (its z-backward is not used: the upstream here is general)
  auto up = [&](int plane) { return (live && gpl) ? gpl[(int64_t)plane * ld + i] : 0.f; };
  // output layer: o = WL h + bL; the gathered o1 - o0 adds (-g, +g)
  const float gl = up(NH * H);
  float go[2] = {-gl, gl};
  if (live && gout2) {
    go[0] += gout2[2 * i];
    go[1] += gout2[2 * i + 1];
  }
  if (!live) go[0] = go[1] = 0.f;
  const float* WL = layer_w<LV, H, NL>(w, NH);
  float da[NH][H];  // dL / d(pre-activation of hidden layer l)
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const float dh = go[0] * WL[j] + go[1] * WL[H + j];
    da[NH - 1][j] = up((NH - 1) * H + j) + (p.a[NH - 1][j] > 0.f ? dh : 0.f);
  }
#pragma unroll
  for (int l = NH - 1; l >= 1; --l) {
    const float* Wl = layer_w<LV, H, NL>(w, l);
#pragma unroll
    for (int k = 0; k < H; ++k) {
      float dh = 0.f;
#pragma unroll
      for (int j = 0; j < H; ++j) dh += da[l][j] * Wl[j * H + k];
      da[l - 1][k] = up((l - 1) * H + k) + (p.a[l - 1][k] > 0.f ? dh : 0.f);
    }
  }
  float de[IN];
#pragma unroll
  for (int m = 0; m < IN; ++m) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < H; ++k) s += da[0][k] * w[k * IN + m];
    de[m] = s;
  }
  // the encoding: table terms and d/dx
  const float2* tab = reinterpret_cast<const float2*>(net.table);
  float gxd[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < LV; ++l) {
    float t[3];
    uint32_t g[3];
    tcell_of(net, l, x, t, g);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const TCorner k = tcorner_of(net, l, t, g, c);
      if (live && k.w != 0.f) {
        if (de[2 * l] != 0.f) unsafeAtomicAdd(&g_table[2 * (size_t)k.idx], k.w * de[2 * l]);
        if (de[2 * l + 1] != 0.f) unsafeAtomicAdd(&g_table[2 * (size_t)k.idx + 1], k.w * de[2 * l + 1]);
      }
      const float2 v = tab[k.idx];
      const float dv = v.x * de[2 * l] + v.y * de[2 * l + 1];
#pragma unroll
      for (int q = 0; q < 3; ++q) gxd[q] += k.dw[q] * dv;
    }
  }
  if (g_x && live)
#pragma unroll
    for (int q = 0; q < 3; ++q) g_x[3 * i + q] += 0.5f * gxd[q];
  // parameters
  int o = 0;
#pragma unroll
  for (int k = 0; k < H; ++k)
#pragma unroll
    for (int m = 0; m < IN; ++m) acc_param(gw, o + k * IN + m, da[0][k] * p.e[m]);
  o += H * IN;
#pragma unroll
  for (int k = 0; k < H; ++k) acc_param(gw, o + k, da[0][k]);
  o += H;
#pragma unroll
  for (int l = 1; l < NH; ++l) {
#pragma unroll
    for (int j = 0; j < H; ++j)
#pragma unroll
      for (int k = 0; k < H; ++k) acc_param(gw, o + j * H + k, da[l][j] * p.h(l - 1, k));
    o += H * H;
#pragma unroll
    for (int j = 0; j < H; ++j) acc_param(gw, o + j, da[l][j]);
    o += H;
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int j = 0; j < H; ++j) acc_param(gw, o + c * H + j, go[c] * p.h(NH - 1, j));
  o += 2 * H;
  acc_param(gw, o, go[0]);
  acc_param(gw, o + 1, go[1]);
  __syncthreads();
  for (int k = threadIdx.x; k < NW; k += blockDim.x)
    if (gw[k] != 0.f) unsafeAtomicAdd(&g_w[k], gw[k]);
}

}  // namespace
