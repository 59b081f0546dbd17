// SDF training on the device (reference train.py:169-224,
// dataset.py:80-96): the launchers of the closed-form batch gradient and the
// autograd VJPs (kernels in train_net.h, one translation unit per level count
// through net_lv.hip), and the mesh signed distances the dataset samples.
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "net_device.h"

namespace {

using namespace tnpnet;

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

static int train_net_ok(const NetDev& net, const char* what) {
  if (!net_supported_full(net) || net.tied) {
    tnp_set_error("%s: net shape (levels=%d, layers=%d, hidden=%d) not instantiated", what, net.n_levels,
                  net.num_layers, net.num_hidden);
    return -1;
  }
  return 0;
}

int launch_train_grad(const NetDev& net, const float* xyz, const float* gt, int64_t n, float clamp_t, float eik_w,
                      int64_t eik_batch, float* g_table, float* g_w, double* stats, hipStream_t s) {
  if (train_net_ok(net, "train")) return -1;
  TNP_CHECK(hipMemsetAsync(stats, 0, 2 * sizeof(double), s));
  if (n <= 0) return 0;
  TNP_LV_SWITCH(net.n_levels, return lv_train<L_>(net, xyz, gt, n, clamp_t, eik_w, eik_batch, stats, g_table, g_w,
                                                   nullptr, nullptr, nullptr, s));
  return 0;
}

int launch_sdf_vjp(const NetDev& net, const float* xyz, const float* gout, int64_t n, float* g_table, float* g_w,
                   hipStream_t s) {
  if (train_net_ok(net, "sdf_vjp")) return -1;
  if (n <= 0) return 0;
  TNP_LV_SWITCH(net.n_levels, return lv_train<L_>(net, xyz, nullptr, n, 0.f, 0.f, 1, nullptr, g_table, g_w, gout,
                                                   nullptr, nullptr, s));
  return 0;
}

int launch_normal_vjp(const NetDev& net, const float* xyz, const float* gJ, int64_t n, float* g_table, float* g_w,
                      float* g_x, hipStream_t s) {
  if (train_net_ok(net, "normal_vjp")) return -1;
  if (n <= 0) return 0;
  TNP_LV_SWITCH(net.n_levels, return lv_train<L_>(net, xyz, nullptr, n, 0.f, 0.f, 1, nullptr, g_table, g_w, nullptr,
                                                   gJ, g_x, s));
  return 0;
}

int launch_forward_vjp(const NetDev& net, const float* xyz, int64_t n, const float* gpl, int64_t ld,
                       const float* gout2, float* g_table, float* g_w, float* g_x, hipStream_t s) {
  if (train_net_ok(net, "forward_vjp")) return -1;
  if (n <= 0) return 0;
  TNP_LV_SWITCH(net.n_levels, return lv_forward_vjp<L_>(net, xyz, n, gpl, ld, gout2, g_table, g_w, g_x, s));
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
