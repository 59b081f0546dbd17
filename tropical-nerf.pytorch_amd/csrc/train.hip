// SDF training on the device (reference train.py:169-224,
// dataset.py:80-96): the batch gradient of the reference's loss in closed
// form, and the mesh signed distances its dataset samples.
//
// Loss of one batch of n points x (train.py:181-201, Net.sdf = tanh(o1 - o0),
// model.py:84-87):
//   L1  = mean_i |clamp(y_i) - clamp(gt_i)|,   clamp to [-T, T] (T = 0.2)
//   Eik = w_e (||J||_F - 1)^2 / B,   J_i = d y_i / d x_i   (w_e = 1e-2, B = BATCH_SIZE)
// (the weight-norm term needs only the fc weights: the caller's).  The
// reference gets dEik/dtheta by double backward (autograd.grad with
// create_graph through tcnn); here it is written out.  With z = o1 - o0,
// g = dz/dx, y = tanh z, v_i = dEik/dJ_i = w_e 2 (||J|| - 1) / (B ||J||) J_i:
//   v.J = (1 - y^2) q,  q = v.g = u . a,
//   u = dz/de (the encoding's output), a = (1/2) sum_c T_c (grad w_c . v)
// -- q is the derivative of z along the direction a in feature space, so
// its weight gradient is a forward-mode pass (a1' = W0 a, h1' = D1 a1',
// a2' = W1 h1', h2' = D2 a2') and every parameter's gradient is
//   kappa dz/dtheta + mu dq/dtheta,   kappa = (1 - y^2)(rho - 2 y q),
//   mu = 1 - y^2,   rho = dL1/dy = sign(clamp y - clamp gt) [|y| <= T] / n:
//   W0 += delta1 (kappa e + mu a)^T      b0 += kappa delta1
//   W1 += delta2 (kappa h1 + mu h1')^T   b1 += kappa delta2
//   W2[1] = -W2[0] += kappa h2 + mu h2'   b2 += kappa (-1, 1)
//   T[l, c, f] += u_{l,f} (kappa w_c + mu (1/2) grad w_c . v)
// (delta2 = D2 (W2[1] - W2[0]), delta1 = D1 W1^T delta2, u = W0^T delta1).
// Two passes: the first reduces ||J||^2 (the global norm every v_i needs)
// and the L1 sum; the second accumulates the gradients -- MLP terms reduced
// per wave, then per block in LDS, one global atomic per parameter per
// block; table terms as global float atomics (summation order is not
// fixed: training is not part of the bitwise contract).
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "net_device.h"

namespace {

using namespace tnpnet;

// trilinear corner c of level l at x' (preprocessed, [0,1]^3): weight,
// weight gradient d w_c / d x' and the float2 entry index
struct Corner {
  float w;
  float dw[3];
  uint32_t idx;
};

__device__ __forceinline__ Corner corner_of(const NetDev& net, int l, const float t[3], const uint32_t g[3],
                                            int c) {
  const float s = net.scales[l];
  float f[3];
  uint32_t gc[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const bool up = (c >> d) & 1;
    f[d] = up ? t[d] : 1.f - t[d];
    gc[d] = g[d] + (up ? 1u : 0u);
  }
  Corner r;
  r.w = f[0] * f[1] * f[2];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float sg = ((c >> d) & 1) ? 1.f : -1.f;
    r.dw[d] = sg * f[(d + 1) % 3] * f[(d + 2) % 3] * s;
  }
  const uint32_t res = (uint32_t)net.res[l];
  uint32_t idx = net.dense[l] ? (gc[0] + gc[1] * res + gc[2] * (res * res)) : (gc[0] ^ (gc[1] * P1) ^ (gc[2] * P2));
  r.idx = net.offsets[l] + wrap_index(idx, net.sizes[l]);
  return r;
}

__device__ __forceinline__ void cell_of(const NetDev& net, int l, const float x[3], float t[3], uint32_t g[3]) {
  const float s = net.scales[l];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float pos = x[d] * s + 0.5f;
    const float fl = floorf(pos);
    t[d] = pos - fl;
    g[d] = (uint32_t)(int)fl;
  }
}

// the forward and dz/d(activations) of one point
template <int LV, int H>
struct Pass {
  static constexpr int IN = 2 * LV;
  float e[IN], a1[H], h1[H], a2[H], h2[H];
  float d1[H], d2[H], u[IN];
  float z, y;
  float gz[3];  // dz/dx (x in [-1, 1]: the (x + 1) / 2 preprocess halves it)

  __device__ __forceinline__ void run(const NetDev& net, const float* w, const float x[3]) {
    const float2* tab = reinterpret_cast<const float2*>(net.table);
#pragma unroll
    for (int l = 0; l < LV; ++l) {
      float t[3];
      uint32_t g[3];
      cell_of(net, l, x, t, g);
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const Corner k = corner_of(net, l, t, g, c);
        const float2 v = tab[k.idx];
        s0 += k.w * v.x;
        s1 += k.w * v.y;
      }
      e[2 * l] = s0;
      e[2 * l + 1] = s1;
    }
    const float* W0 = w;
    const float* W1 = W0 + H * IN + H;
    const float* W2 = W1 + H * H + H;
    linear<IN, H>(W0, W0 + H * IN, e, a1);
#pragma unroll
    for (int j = 0; j < H; ++j) h1[j] = fmaxf(a1[j], 0.f);
    linear<H, H>(W1, W1 + H * H, h1, a2);
#pragma unroll
    for (int j = 0; j < H; ++j) h2[j] = fmaxf(a2[j], 0.f);
    float o[2];
    linear<H, 2>(W2, W2 + 2 * H, h2, o);
    z = o[1] - o[0];
    y = tanhf(z);
#pragma unroll
    for (int j = 0; j < H; ++j) d2[j] = a2[j] > 0.f ? W2[H + j] - W2[j] : 0.f;
#pragma unroll
    for (int k = 0; k < H; ++k) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < H; ++j) v += d2[j] * W1[j * H + k];
      d1[k] = a1[k] > 0.f ? v : 0.f;
    }
#pragma unroll
    for (int m = 0; m < IN; ++m) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < H; ++k) v += d1[k] * W0[k * IN + m];
      u[m] = v;
    }
    gz[0] = gz[1] = gz[2] = 0.f;
#pragma unroll
    for (int l = 0; l < LV; ++l) {
      float t[3];
      uint32_t g[3];
      cell_of(net, l, x, t, g);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const Corner k = corner_of(net, l, t, g, c);
        const float2 v = tab[k.idx];
        const float dv = v.x * u[2 * l] + v.y * u[2 * l + 1];
#pragma unroll
        for (int d = 0; d < 3; ++d) gz[d] += k.dw[d] * dv;
      }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) gz[d] *= 0.5f;
  }
};

__device__ __forceinline__ float clampf(float v, float T) { return fminf(fmaxf(v, -T), T); }

// pass 1: sum_i |clamp(y_i) - clamp(gt_i)| -> stats[0], sum_i ||J_i||^2 -> stats[1]
template <int LV, int H>
__global__ void __launch_bounds__(TNP_BLOCK)
k_train_norms(NetDev net, const float* __restrict__ xyz, const float* __restrict__ gt, int64_t n, float T,
              double* __restrict__ stats) {
  constexpr int NW = NetShape<LV, H, 3>::NW;
  __shared__ float w[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) w[i] = net.weights[i];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double l1 = 0.0, j2 = 0.0;
  if (i < n) {
    float x[3];
    load_point(xyz, i, x);
    Pass<LV, H> p;
    p.run(net, w, x);
    const float ty = 1.f - p.y * p.y;
    l1 = fabsf(clampf(p.y, T) - clampf(gt[i], T));
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

// one parameter's per-lane terms: wave sum, then the block's LDS slot
__device__ __forceinline__ void acc_param(float* lds_g, int p, float v) {
  v = tnp::wave_sum(v);
  if (tnp::lane() == 0 && v != 0.f) atomicAdd(&lds_g[p], v);
}

// pass 2: the gradients (header comment)
template <int LV, int H>
__global__ void __launch_bounds__(TNP_BLOCK)
k_train_grads(NetDev net, const float* __restrict__ xyz, const float* __restrict__ gt, int64_t n, float T,
              float eik_w, int64_t eik_batch, const double* __restrict__ stats, float* __restrict__ g_table,
              float* __restrict__ g_w, const float* __restrict__ gout) {
  constexpr int IN = 2 * LV;
  constexpr int NW = NetShape<LV, H, 3>::NW;
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
  Pass<LV, H> p;
  p.run(net, w, x);
  // v_i = c J_i, c = w_e 2 (||J|| - 1) / (B ||J||), B = BATCH_SIZE (train.py:197;
  // the L1 mean below divides by the actual n)   (torch: a zero norm has a zero gradient)
  // gout != null: the vector-Jacobian product sum_i gout_i d sdf_i / d theta
  // instead (autograd through Net.sdf): kappa = gout (1 - y^2), mu = 0
  const double nj = gout ? 0.0 : sqrt(stats[1]);
  const float c = nj > 0.0 ? (float)(eik_w * 2.0 * (nj - 1.0) / ((double)eik_batch * nj)) : 0.f;
  const float ty = 1.f - p.y * p.y;
  float v[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) v[d] = c * ty * p.gz[d];
  const float q = v[0] * p.gz[0] + v[1] * p.gz[1] + v[2] * p.gz[2];
  float rho = 0.f;
  if (!gout && live && p.y >= -T && p.y <= T) {
    const float r = clampf(p.y, T) - clampf(gt[i], T);
    rho = (r > 0.f ? 1.f : (r < 0.f ? -1.f : 0.f)) / (float)n;
  }
  const float kappa = !live ? 0.f : (gout ? ty * gout[i] : ty * (rho - 2.f * p.y * q));
  const float mu = (live && !gout) ? ty : 0.f;
  // direction a = (1/2) sum_c T_c (grad w_c . v), and the table terms
  const float2* tab = reinterpret_cast<const float2*>(net.table);
  float a[IN];
#pragma unroll
  for (int l = 0; l < LV; ++l) {
    float t[3];
    uint32_t g[3];
    cell_of(net, l, x, t, g);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      const Corner k = corner_of(net, l, t, g, cc);
      const float gv = 0.5f * (k.dw[0] * v[0] + k.dw[1] * v[1] + k.dw[2] * v[2]);
      const float2 e2 = tab[k.idx];
      s0 += e2.x * gv;
      s1 += e2.y * gv;
      const float coef = kappa * k.w + mu * gv;
      if (live && coef != 0.f) {
        if (p.u[2 * l] != 0.f) unsafeAtomicAdd(&g_table[2 * (size_t)k.idx], p.u[2 * l] * coef);
        if (p.u[2 * l + 1] != 0.f) unsafeAtomicAdd(&g_table[2 * (size_t)k.idx + 1], p.u[2 * l + 1] * coef);
      }
    }
    a[2 * l] = s0;
    a[2 * l + 1] = s1;
  }
  const float* W0 = w;
  const float* W1 = W0 + H * IN + H;
  float h1d[H], h2d[H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < IN; ++m) s += W0[k * IN + m] * a[m];
    h1d[k] = p.a1[k] > 0.f ? s : 0.f;
  }
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < H; ++k) s += W1[j * H + k] * h1d[k];
    h2d[j] = p.a2[j] > 0.f ? s : 0.f;
  }
  // packed gradient layout = packed weight layout (fc.0.weight, fc.0.bias, ...)
  int o = 0;
#pragma unroll
  for (int k = 0; k < H; ++k)
#pragma unroll
    for (int m = 0; m < IN; ++m) acc_param(gw, o + k * IN + m, p.d1[k] * (kappa * p.e[m] + mu * a[m]));
  o += H * IN;
#pragma unroll
  for (int k = 0; k < H; ++k) acc_param(gw, o + k, kappa * p.d1[k]);
  o += H;
#pragma unroll
  for (int j = 0; j < H; ++j)
#pragma unroll
    for (int k = 0; k < H; ++k) acc_param(gw, o + j * H + k, p.d2[j] * (kappa * p.h1[k] + mu * h1d[k]));
  o += H * H;
#pragma unroll
  for (int j = 0; j < H; ++j) acc_param(gw, o + j, kappa * p.d2[j]);
  o += H;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const float r = kappa * p.h2[j] + mu * h2d[j];
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

// ---------------------------------------------------------------------------
// mesh signed distance (cubvh signed_distance, dataset.py:77, 92): exact
// closest-point distance to every triangle, sign from the generalized
// winding number.  Grid (point tiles) x (triangle chunks); a chunk's
// triangles go through LDS 256 at a time; per point, atomicMin of the
// squared distance bits (non-negative floats order as integers) and an
// atomic sum of the solid angles.
// ---------------------------------------------------------------------------

// squared distance from p to triangle (a, b, c): closest point by Voronoi
// region of the triangle (vertex, edge or face)
__device__ __forceinline__ float tri_dist2(const float p[3], const float* a, const float* b, const float* c) {
  float ab[3], ac[3], ap[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    ab[d] = b[d] - a[d];
    ac[d] = c[d] - a[d];
    ap[d] = p[d] - a[d];
  }
  auto dot = [](const float* u, const float* w) { return u[0] * w[0] + u[1] * w[1] + u[2] * w[2]; };
  float q[3];
  const float d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.f && d2 <= 0.f) {
    for (int d = 0; d < 3; ++d) q[d] = a[d];
  } else {
    float bp[3];
    for (int d = 0; d < 3; ++d) bp[d] = p[d] - b[d];
    const float d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0.f && d4 <= d3) {
      for (int d = 0; d < 3; ++d) q[d] = b[d];
    } else {
      const float vc = d1 * d4 - d3 * d2;
      if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
        const float t = d1 / (d1 - d3);
        for (int d = 0; d < 3; ++d) q[d] = a[d] + t * ab[d];
      } else {
        float cp[3];
        for (int d = 0; d < 3; ++d) cp[d] = p[d] - c[d];
        const float d5 = dot(ab, cp), d6 = dot(ac, cp);
        if (d6 >= 0.f && d5 <= d6) {
          for (int d = 0; d < 3; ++d) q[d] = c[d];
        } else {
          const float vb = d5 * d2 - d1 * d6;
          if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
            const float t = d2 / (d2 - d6);
            for (int d = 0; d < 3; ++d) q[d] = a[d] + t * ac[d];
          } else {
            const float va = d3 * d6 - d5 * d4;
            if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
              const float t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
              for (int d = 0; d < 3; ++d) q[d] = b[d] + t * (c[d] - b[d]);
            } else {
              const float den = 1.f / (va + vb + vc);
              const float vv = vb * den, ww = vc * den;
              for (int d = 0; d < 3; ++d) q[d] = a[d] + ab[d] * vv + ac[d] * ww;
            }
          }
        }
      }
    }
  }
  float r = 0.f;
#pragma unroll
  for (int d = 0; d < 3; ++d) r += (p[d] - q[d]) * (p[d] - q[d]);
  return r;
}

// signed solid angle of triangle (a, b, c) seen from p (Van Oosterom &
// Strackee), over 4 pi
__device__ __forceinline__ float tri_winding(const float p[3], const float* a, const float* b, const float* c) {
  float u[3], v[3], w[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    u[d] = a[d] - p[d];
    v[d] = b[d] - p[d];
    w[d] = c[d] - p[d];
  }
  const float lu = sqrtf(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  const float lv = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  const float lw = sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const float det = u[0] * (v[1] * w[2] - v[2] * w[1]) - u[1] * (v[0] * w[2] - v[2] * w[0]) +
                    u[2] * (v[0] * w[1] - v[1] * w[0]);
  const float den = lu * lv * lw + (u[0] * v[0] + u[1] * v[1] + u[2] * v[2]) * lw +
                    (u[0] * w[0] + u[1] * w[1] + u[2] * w[2]) * lv + (v[0] * w[0] + v[1] * w[1] + v[2] * w[2]) * lu;
  return atan2f(det, den) * (float)(0.5 / 3.14159265358979323846);  // 2 atan2 / (4 pi)
}

constexpr int SD_TILE = 256;

__global__ void __launch_bounds__(TNP_BLOCK)
k_mesh_sd(const float* __restrict__ V, int64_t nV, const int32_t* __restrict__ F, int64_t nF, int64_t chunk,
          const float* __restrict__ P, int64_t n, uint32_t* __restrict__ d2bits, float* __restrict__ wind) {
  __shared__ float tri[SD_TILE][9];
  const int64_t i = (int64_t)blockIdx.x * TNP_BLOCK + threadIdx.x;
  float p[3] = {0.f, 0.f, 0.f};
  if (i < n)
    for (int d = 0; d < 3; ++d) p[d] = P[3 * i + d];
  const int64_t f0 = (int64_t)blockIdx.y * chunk;
  const int64_t f1 = f0 + chunk < nF ? f0 + chunk : nF;
  float best = __int_as_float(0x7f800000);
  float wsum = 0.f;
  for (int64_t t0 = f0; t0 < f1; t0 += SD_TILE) {
    const int64_t f = t0 + threadIdx.x;
    if (f < f1) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        int64_t vi = F[3 * f + k];
        vi = (vi < 0 || vi >= nV) ? 0 : vi;  // the host checks the indices; never read past V
#pragma unroll
        for (int d = 0; d < 3; ++d) tri[threadIdx.x][3 * k + d] = V[3 * (int64_t)vi + d];
      }
    }
    __syncthreads();
    const int m = (int)(f1 - t0 < SD_TILE ? f1 - t0 : SD_TILE);
    for (int k = 0; k < m; ++k) {
      const float* t = tri[k];
      best = fminf(best, tri_dist2(p, t, t + 3, t + 6));
      wsum += tri_winding(p, t, t + 3, t + 6);
    }
    __syncthreads();
  }
  if (i < n) {
    atomicMin(&d2bits[i], __float_as_uint(best));
    unsafeAtomicAdd(&wind[i], wsum);
  }
}

__global__ void k_mesh_sd_finish(const uint32_t* __restrict__ d2bits, const float* __restrict__ wind, int64_t n,
                                 float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float d = sqrtf(__uint_as_float(d2bits[i]));
  out[i] = fabsf(wind[i]) > 0.5f ? d : -d;  // inside is positive (dataset.py:96)
}

__global__ void k_fill_u32(uint32_t* __restrict__ p, int64_t n, uint32_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

}  // namespace

#define TNP_TRAIN_DISPATCH(LV, BODY)                                \
  switch (LV) {                                                     \
    case 2: { constexpr int L_ = 2; BODY; break; }                  \
    case 4: { constexpr int L_ = 4; BODY; break; }                  \
    default: tnp_set_error("n_levels=%d not instantiated", LV); return -1; \
  }

int launch_train_grad(const NetDev& net, const float* xyz, const float* gt, int64_t n, float clamp_t, float eik_w,
                      int64_t eik_batch, float* g_table, float* g_w, double* stats, hipStream_t s) {
  if (!net_supported(net) || net.tied || net.num_hidden != 16 || net.num_layers != 3) {
    tnp_set_error("train: the closed-form gradient is written for 3-layer, 16-hidden nets (this net: %d layers, "
                  "%d hidden, %d levels)", net.num_layers, net.num_hidden, net.n_levels);
    return -1;
  }
  TNP_CHECK(hipMemsetAsync(stats, 0, 2 * sizeof(double), s));
  if (n <= 0) return 0;
  TNP_TRAIN_DISPATCH(net.n_levels, {
    hipLaunchKernelGGL((k_train_norms<L_, 16>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, gt, n, clamp_t,
                       stats);
    hipLaunchKernelGGL((k_train_grads<L_, 16>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, gt, n, clamp_t,
                       eik_w, eik_batch, stats, g_table, g_w, nullptr);
  });
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_sdf_vjp(const NetDev& net, const float* xyz, const float* gout, int64_t n, float* g_table, float* g_w,
                   hipStream_t s) {
  if (!net_supported(net) || net.tied || net.num_hidden != 16 || net.num_layers != 3) {
    tnp_set_error("sdf_vjp: the parameter gradient is written for 3-layer, 16-hidden nets (this net: %d layers, "
                  "%d hidden, %d levels)", net.num_layers, net.num_hidden, net.n_levels);
    return -1;
  }
  if (n <= 0) return 0;
  TNP_TRAIN_DISPATCH(net.n_levels, {
    hipLaunchKernelGGL((k_train_grads<L_, 16>), dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, net, xyz, nullptr, n, 0.f,
                       0.f, (int64_t)1, nullptr, g_table, g_w, gout);
  });
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_mesh_sd(const float* V, int64_t nV, const int32_t* F, int64_t nF, const float* P, int64_t n, float* work,
                   float* out, hipStream_t s) {
  if (n <= 0) return 0;
  if (nF <= 0 || nV <= 0) { tnp_set_error("mesh_signed_distance: empty mesh"); return -1; }
  uint32_t* d2 = reinterpret_cast<uint32_t*>(work);
  float* wind = work + n;
  hipLaunchKernelGGL(k_fill_u32, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, d2, n, 0x7f800000u);
  TNP_CHECK(hipMemsetAsync(wind, 0, n * sizeof(float), s));
  // enough workgroups for the chip: split the triangles when the points alone
  // give fewer than ~4 per CU
  const int64_t bx = tnp_grid(n);
  int64_t by = std::max<int64_t>(1, std::min<int64_t>((nF + SD_TILE - 1) / SD_TILE, (2048 + bx - 1) / bx));
  const int64_t chunk = ((nF + by - 1) / by + SD_TILE - 1) / SD_TILE * SD_TILE;
  by = (nF + chunk - 1) / chunk;
  if (by > 65535) { tnp_set_error("mesh_signed_distance: too many triangle chunks"); return -1; }
  hipLaunchKernelGGL(k_mesh_sd, dim3((unsigned)bx, (unsigned)by), dim3(TNP_BLOCK), 0, s, V, nV, F, nF, chunk, P, n, d2,
                     wind);
  hipLaunchKernelGGL(k_mesh_sd_finish, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, d2, wind, n, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
