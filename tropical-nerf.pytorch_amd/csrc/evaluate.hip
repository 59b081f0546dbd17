// The `-e` evaluation stack of tropical.stanford.train (train.py:275-354) on
// gfx950, replacing the reference's third-party CUDA/C++ helpers:
//
//   mcubes.marching_cubes     -> tnp_mc_count / tnp_mc_emit (procedural case
//                                table, tropical/utils/mc_table.py)
//   cubvh.cuBVH(...).ray_trace -> tnp_raycaster_* (uniform-grid traversal,
//                                Moller-Trumbore, nearest hit)
//   sklearn NearestNeighbors   -> tnp_nn_min_dist (exact brute force, LDS
//                                tiles; chamfer_distance.py:39-48)
//
// Bandwidth notes: marching cubes is a streaming pass over the volume (4 B
// per sample read twice + 8 B offsets per lattice edge and cube); the ray
// caster and the NN search are compute/L2-bound (triangle and point tiles
// stay cache-resident).
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "common.h"
#include "kernels.h"

namespace {

// ---------------------------------------------------------------------------
// marching cubes
// ---------------------------------------------------------------------------
struct Dims {
  int n0, n1, n2;
};

__device__ __forceinline__ int64_t pidx(const Dims& d, int i, int j, int k) {
  return ((int64_t)i * d.n1 + j) * d.n2 + k;
}

// crossed lattice edges: flag per (point, axis), inside = value < iso
__global__ void k_mc_edge_flags(const float* __restrict__ vol, Dims d, float iso,
                                int64_t* __restrict__ flag) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t N = (int64_t)d.n0 * d.n1 * d.n2;
  if (p >= N) return;
  const int k = (int)(p % d.n2), j = (int)((p / d.n2) % d.n1), i = (int)(p / ((int64_t)d.n1 * d.n2));
  const bool in0 = vol[p] < iso;
  flag[3 * p + 0] = (i + 1 < d.n0) && ((vol[pidx(d, i + 1, j, k)] < iso) != in0);
  flag[3 * p + 1] = (j + 1 < d.n1) && ((vol[pidx(d, i, j + 1, k)] < iso) != in0);
  flag[3 * p + 2] = (k + 1 < d.n2) && ((vol[pidx(d, i, j, k + 1)] < iso) != in0);
}

__device__ __forceinline__ int cube_case(const float* __restrict__ vol, const Dims& d, int i, int j,
                                         int k, float iso) {
  int c = 0;
  c |= (vol[pidx(d, i, j, k)] < iso) << 0;
  c |= (vol[pidx(d, i + 1, j, k)] < iso) << 1;
  c |= (vol[pidx(d, i + 1, j + 1, k)] < iso) << 2;
  c |= (vol[pidx(d, i, j + 1, k)] < iso) << 3;
  c |= (vol[pidx(d, i, j, k + 1)] < iso) << 4;
  c |= (vol[pidx(d, i + 1, j, k + 1)] < iso) << 5;
  c |= (vol[pidx(d, i + 1, j + 1, k + 1)] < iso) << 6;
  c |= (vol[pidx(d, i, j + 1, k + 1)] < iso) << 7;
  return c;
}

// triangles per cube (cube index = (i, j, k) over [0, n-1)^3, x slowest)
__global__ void k_mc_cube_counts(const float* __restrict__ vol, Dims d, float iso,
                                 const int8_t* __restrict__ table, int64_t* __restrict__ cnt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int m0 = d.n0 - 1, m1 = d.n1 - 1, m2 = d.n2 - 1;
  if (c >= (int64_t)m0 * m1 * m2) return;
  const int k = (int)(c % m2), j = (int)((c / m2) % m1), i = (int)(c / ((int64_t)m1 * m2));
  const int cs = cube_case(vol, d, i, j, k, iso);
  int n = 0;
  while (n < 5 && table[cs * 16 + 3 * n] >= 0) ++n;
  cnt[c] = n;
}

__global__ void k_mc_vertices(const float* __restrict__ vol, Dims d, float iso,
                              const int64_t* __restrict__ eoff, double* __restrict__ verts) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t N = (int64_t)d.n0 * d.n1 * d.n2;
  if (p >= N) return;
  const int k = (int)(p % d.n2), j = (int)((p / d.n2) % d.n1), i = (int)(p / ((int64_t)d.n1 * d.n2));
  const double v0 = vol[p];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int64_t e = 3 * p + a;
    if (eoff[e + 1] == eoff[e]) continue;  // not crossed
    const int64_t q = pidx(d, i + (a == 0), j + (a == 1), k + (a == 2));
    // in double, as PyMCubes interpolates: an fp32 i + t snaps every t below
    // half an ulp of i onto the lattice point, and two such vertices of one
    // triangle make it degenerate (a zero normal in the -e angular distance)
    const double t = __ddiv_rn(__dsub_rn((double)iso, v0), __dsub_rn((double)vol[q], v0));
    double* o = verts + 3 * eoff[e];
    o[0] = (double)i;
    o[1] = (double)j;
    o[2] = (double)k;
    o[a] = __dadd_rn(o[a], t);
  }
}

// cube edge -> (di, dj, dk, axis) of its lattice edge
__constant__ int8_t c_edge_lat[12][4] = {
    {0, 0, 0, 0}, {1, 0, 0, 1}, {0, 1, 0, 0}, {0, 0, 0, 1}, {0, 0, 1, 0}, {1, 0, 1, 1},
    {0, 1, 1, 0}, {0, 0, 1, 1}, {0, 0, 0, 2}, {1, 0, 0, 2}, {1, 1, 0, 2}, {0, 1, 0, 2}};

__global__ void k_mc_triangles(const float* __restrict__ vol, Dims d, float iso,
                               const int8_t* __restrict__ table, const int64_t* __restrict__ eoff,
                               const int64_t* __restrict__ coff, int64_t* __restrict__ tris) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int m0 = d.n0 - 1, m1 = d.n1 - 1, m2 = d.n2 - 1;
  if (c >= (int64_t)m0 * m1 * m2) return;
  int64_t t0 = coff[c];
  const int nt = (int)(coff[c + 1] - t0);
  if (nt == 0) return;
  const int k = (int)(c % m2), j = (int)((c / m2) % m1), i = (int)(c / ((int64_t)m1 * m2));
  const int cs = cube_case(vol, d, i, j, k, iso);
  for (int q = 0; q < 3 * nt; ++q) {
    const int e = table[cs * 16 + q];
    const int8_t* L = c_edge_lat[e];
    const int64_t lid = 3 * pidx(d, i + L[0], j + L[1], k + L[2]) + L[3];
    tris[3 * t0 + q] = eoff[lid];
  }
}

template <typename T>
int excl_scan_inplace(T* buf, int64_t n, hipStream_t s) {
  // exclusive scan of buf[0, n) into buf[0, n] (buf[n] = total; caller sized n + 1)
  size_t tmp = 0;
  TNP_CHECK(rocprim::exclusive_scan(nullptr, tmp, buf, buf, (T)0, (size_t)(n + 1),
                                    rocprim::plus<T>(), s));
  void* scratch = nullptr;
  TNP_CHECK(hipMallocAsync(&scratch, std::max<size_t>(tmp, 16), s));
  hipError_t err = rocprim::exclusive_scan(scratch, tmp, buf, buf, (T)0, (size_t)(n + 1),
                                           rocprim::plus<T>(), s);
  TNP_CHECK(hipFreeAsync(scratch, s));
  TNP_CHECK(err);
  return 0;
}

// ---------------------------------------------------------------------------
// ray caster: uniform grid over the mesh bounding box
// ---------------------------------------------------------------------------
struct Grid {
  float lo[3], cell[3];
  int res[3];
};

__device__ __forceinline__ void tri_bounds(const float* V, const int32_t* F, int64_t f, float mn[3],
                                           float mx[3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    mn[d] = FLT_MAX;
    mx[d] = -FLT_MAX;
  }
  for (int q = 0; q < 3; ++q) {
    const float* p = V + 3 * (int64_t)F[3 * f + q];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      mn[d] = fminf(mn[d], p[d]);
      mx[d] = fmaxf(mx[d], p[d]);
    }
  }
}

__device__ __forceinline__ int cell_of(const Grid& g, float x, int d) {
  int c = (int)floorf((x - g.lo[d]) / g.cell[d]);
  return c < 0 ? 0 : (c >= g.res[d] ? g.res[d] - 1 : c);
}

template <bool FILL>
__global__ void k_grid_bin(const float* __restrict__ V, const int32_t* __restrict__ F, int64_t nF,
                           Grid g, int32_t* __restrict__ cnt, const int64_t* __restrict__ off,
                           int32_t* __restrict__ cur, int32_t* __restrict__ items) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nF) return;
  float mn[3], mx[3];
  tri_bounds(V, F, f, mn, mx);
  int a[3], b[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    a[d] = cell_of(g, mn[d], d);
    b[d] = cell_of(g, mx[d], d);
  }
  for (int x = a[0]; x <= b[0]; ++x)
    for (int y = a[1]; y <= b[1]; ++y)
      for (int z = a[2]; z <= b[2]; ++z) {
        const int64_t c = ((int64_t)x * g.res[1] + y) * g.res[2] + z;
        if (FILL) items[off[c] + atomicAdd(&cur[c], 1)] = (int32_t)f;
        else atomicAdd(&cnt[c], 1);
      }
}

// Moller-Trumbore; t of the hit or +inf
__device__ __forceinline__ float ray_tri(const float o[3], const float dir[3], const float* a,
                                         const float* b, const float* c) {
  const float e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const float e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  const float p[3] = {dir[1] * e2[2] - dir[2] * e2[1], dir[2] * e2[0] - dir[0] * e2[2],
                      dir[0] * e2[1] - dir[1] * e2[0]};
  const float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
  if (fabsf(det) < 1e-12f) return INFINITY;
  const float inv = 1.0f / det;
  const float s[3] = {o[0] - a[0], o[1] - a[1], o[2] - a[2]};
  const float u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * inv;
  if (u < 0.f || u > 1.f) return INFINITY;
  const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2],
                      s[0] * e1[1] - s[1] * e1[0]};
  const float v = (dir[0] * q[0] + dir[1] * q[1] + dir[2] * q[2]) * inv;
  if (v < 0.f || u + v > 1.f) return INFINITY;
  const float t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
  return t > 0.f ? t : INFINITY;
}

// 3D DDA through the grid; the nearest hit inside the current cell's t range
// ends the walk (a triangle spanning several cells is tested in each)
__global__ void k_ray_cast(const float* __restrict__ V, const int32_t* __restrict__ F, Grid g,
                           const int64_t* __restrict__ off, const int32_t* __restrict__ items,
                           const float* __restrict__ ro, const float* __restrict__ rd, int64_t nR,
                           float* __restrict__ tout, int32_t* __restrict__ fout) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nR) return;
  const float o[3] = {ro[3 * r], ro[3 * r + 1], ro[3 * r + 2]};
  const float d[3] = {rd[3 * r], rd[3 * r + 1], rd[3 * r + 2]};
  float t0 = 0.f, t1 = INFINITY;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float lo = g.lo[a], hi = g.lo[a] + g.cell[a] * g.res[a];
    if (fabsf(d[a]) < 1e-20f) {
      if (o[a] < lo || o[a] > hi) t1 = -1.f;
    } else {
      float ta = (lo - o[a]) / d[a], tb = (hi - o[a]) / d[a];
      if (ta > tb) { const float x = ta; ta = tb; tb = x; }
      t0 = fmaxf(t0, ta);
      t1 = fminf(t1, tb);
    }
  }
  float best = INFINITY;
  int bestf = -1;
  if (t0 <= t1) {
    int c[3], step[3];
    float tmax[3], tdelta[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float x = o[a] + t0 * d[a];
      c[a] = cell_of(g, x, a);
      if (d[a] > 0.f) {
        step[a] = 1;
        tmax[a] = (g.lo[a] + (c[a] + 1) * g.cell[a] - o[a]) / d[a];
        tdelta[a] = g.cell[a] / d[a];
      } else if (d[a] < 0.f) {
        step[a] = -1;
        tmax[a] = (g.lo[a] + c[a] * g.cell[a] - o[a]) / d[a];
        tdelta[a] = -g.cell[a] / d[a];
      } else {
        step[a] = 0;
        tmax[a] = INFINITY;
        tdelta[a] = INFINITY;
      }
    }
    while (true) {
      const int64_t cid = ((int64_t)c[0] * g.res[1] + c[1]) * g.res[2] + c[2];
      for (int64_t q = off[cid]; q < off[cid + 1]; ++q) {
        const int f = items[q];
        const float t = ray_tri(o, d, V + 3 * (int64_t)F[3 * f], V + 3 * (int64_t)F[3 * f + 1],
                                V + 3 * (int64_t)F[3 * f + 2]);
        if (t < best || (t == best && f < bestf)) {
          best = t;
          bestf = f;
        }
      }
      const float texit = fminf(tmax[0], fminf(tmax[1], tmax[2]));
      if (best <= texit) break;
      const int a = (tmax[0] <= tmax[1] && tmax[0] <= tmax[2]) ? 0 : (tmax[1] <= tmax[2] ? 1 : 2);
      c[a] += step[a];
      if (c[a] < 0 || c[a] >= g.res[a]) break;
      tmax[a] += tdelta[a];
    }
  }
  tout[r] = best;
  fout[r] = bestf;
}

// ---------------------------------------------------------------------------
// exact nearest-neighbour distance, brute force over LDS tiles of b
// ---------------------------------------------------------------------------
constexpr int NN_TILE = 1024;

__global__ void __launch_bounds__(TNP_BLOCK)
k_nn_min_dist(const float* __restrict__ a, int64_t na, const float* __restrict__ b, int64_t nb,
              float* __restrict__ out) {
  __shared__ float tb[3 * NN_TILE];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float q[3] = {0.f, 0.f, 0.f};
  if (i < na) {
    q[0] = a[3 * i];
    q[1] = a[3 * i + 1];
    q[2] = a[3 * i + 2];
  }
  float best = INFINITY;
  for (int64_t base = 0; base < nb; base += NN_TILE) {
    const int n = (int)std::min<int64_t>(NN_TILE, nb - base);
    __syncthreads();
    for (int t = threadIdx.x; t < 3 * n; t += blockDim.x) tb[t] = b[3 * base + t];
    __syncthreads();
    for (int t = 0; t < n; ++t) {
      const float dx = q[0] - tb[3 * t], dy = q[1] - tb[3 * t + 1], dz = q[2] - tb[3 * t + 2];
      best = fminf(best, dx * dx + dy * dy + dz * dz);
    }
  }
  if (i < na) out[i] = sqrtf(best);
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" int tnp_mc_count(const float* d_vol, int n0, int n1, int n2, float iso,
                            const int8_t* d_table, int64_t* d_eoff, int64_t* d_coff,
                            int64_t* n_verts, int64_t* n_tris, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n0 < 2 || n1 < 2 || n2 < 2) { tnp_set_error("marching cubes needs >= 2 samples per axis"); return -1; }
  const Dims d{n0, n1, n2};
  const int64_t N = (int64_t)n0 * n1 * n2, C = (int64_t)(n0 - 1) * (n1 - 1) * (n2 - 1);
  hipLaunchKernelGGL(k_mc_edge_flags, dim3(tnp_grid(N)), dim3(TNP_BLOCK), 0, s, d_vol, d, iso, d_eoff);
  hipLaunchKernelGGL(k_mc_cube_counts, dim3(tnp_grid(C)), dim3(TNP_BLOCK), 0, s, d_vol, d, iso, d_table,
                     d_coff);
  TNP_CHECK(hipGetLastError());
  if (excl_scan_inplace(d_eoff, 3 * N, s)) return -1;
  if (excl_scan_inplace(d_coff, C, s)) return -1;
  TNP_CHECK(hipMemcpyAsync(n_verts, d_eoff + 3 * N, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TNP_CHECK(hipMemcpyAsync(n_tris, d_coff + C, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TNP_CHECK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int tnp_mc_emit(const float* d_vol, int n0, int n1, int n2, float iso,
                           const int8_t* d_table, const int64_t* d_eoff, const int64_t* d_coff,
                           double* d_verts, int64_t* d_tris, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const Dims d{n0, n1, n2};
  const int64_t N = (int64_t)n0 * n1 * n2, C = (int64_t)(n0 - 1) * (n1 - 1) * (n2 - 1);
  hipLaunchKernelGGL(k_mc_vertices, dim3(tnp_grid(N)), dim3(TNP_BLOCK), 0, s, d_vol, d, iso, d_eoff,
                     d_verts);
  hipLaunchKernelGGL(k_mc_triangles, dim3(tnp_grid(C)), dim3(TNP_BLOCK), 0, s, d_vol, d, iso, d_table,
                     d_eoff, d_coff, d_tris);
  TNP_CHECK(hipGetLastError());
  return 0;
}

struct tnp_raycaster {
  int device = 0;
  Grid g{};
  const float* V = nullptr;
  const int32_t* F = nullptr;
  int64_t nF = 0;
  int64_t* off = nullptr;
  int32_t* items = nullptr;
};

extern "C" int tnp_raycaster_create(tnp_raycaster** out, int device) {
  TNP_CHECK(hipSetDevice(device));
  tnp_raycaster* r = new tnp_raycaster();
  r->device = device;
  *out = r;
  return 0;
}

extern "C" void tnp_raycaster_destroy(tnp_raycaster* r) {
  if (!r) return;
  (void)hipSetDevice(r->device);
  if (r->off) (void)hipFree(r->off);
  if (r->items) (void)hipFree(r->items);
  delete r;
}

extern "C" int tnp_raycaster_build(tnp_raycaster* r, const float* d_V, int64_t nV, const int32_t* d_F,
                                   int64_t nF, const float* bbox_lo, const float* bbox_hi,
                                   void* stream) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(r->device));
  (void)nV;
  if (r->off) { TNP_CHECK(hipFree(r->off)); r->off = nullptr; }
  if (r->items) { TNP_CHECK(hipFree(r->items)); r->items = nullptr; }
  // ~2 triangles per cell, cubic cells over the box
  float ext[3], mx = 0.f;
  for (int d = 0; d < 3; ++d) {
    ext[d] = std::max(bbox_hi[d] - bbox_lo[d], 1e-6f);
    mx = std::max(mx, ext[d]);
  }
  const double target = std::max<double>(1.0, nF / 2.0);
  const double vol = (double)ext[0] * ext[1] * ext[2];
  const float h = (float)std::cbrt(vol / target);
  Grid g{};
  int64_t ncell = 1;
  for (int d = 0; d < 3; ++d) {
    g.res[d] = (int)std::min(512.0, std::max(1.0, std::ceil((double)ext[d] / h)));
    g.cell[d] = ext[d] / g.res[d] * 1.0001f;
    g.lo[d] = bbox_lo[d] - 1e-5f * mx;
    ncell *= g.res[d];
  }
  int32_t *cnt = nullptr, *cur = nullptr;
  TNP_CHECK(hipMalloc(&r->off, (ncell + 1) * sizeof(int64_t)));
  TNP_CHECK(hipMalloc(&cnt, (ncell + 1) * sizeof(int32_t)));
  TNP_CHECK(hipMalloc(&cur, ncell * sizeof(int32_t)));
  TNP_CHECK(hipMemsetAsync(cnt, 0, (ncell + 1) * sizeof(int32_t), s));
  TNP_CHECK(hipMemsetAsync(cur, 0, ncell * sizeof(int32_t), s));
  if (nF > 0)
    hipLaunchKernelGGL(k_grid_bin<false>, dim3(tnp_grid(nF)), dim3(TNP_BLOCK), 0, s, d_V, d_F, nF, g,
                       cnt, nullptr, nullptr, nullptr);
  // widen to int64 offsets
  {
    size_t tmp = 0;
    TNP_CHECK(rocprim::exclusive_scan(nullptr, tmp, cnt, r->off, (int64_t)0, (size_t)(ncell + 1),
                                      rocprim::plus<int64_t>(), s));
    void* scratch = nullptr;
    TNP_CHECK(hipMallocAsync(&scratch, std::max<size_t>(tmp, 16), s));
    TNP_CHECK(rocprim::exclusive_scan(scratch, tmp, cnt, r->off, (int64_t)0, (size_t)(ncell + 1),
                                      rocprim::plus<int64_t>(), s));
    TNP_CHECK(hipFreeAsync(scratch, s));
  }
  int64_t total = 0;
  TNP_CHECK(hipMemcpyAsync(&total, r->off + ncell, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TNP_CHECK(hipStreamSynchronize(s));
  TNP_CHECK(hipMalloc(&r->items, std::max<int64_t>(total, 1) * sizeof(int32_t)));
  if (nF > 0)
    hipLaunchKernelGGL(k_grid_bin<true>, dim3(tnp_grid(nF)), dim3(TNP_BLOCK), 0, s, d_V, d_F, nF, g,
                       nullptr, r->off, cur, r->items);
  TNP_CHECK(hipGetLastError());
  TNP_CHECK(hipStreamSynchronize(s));
  TNP_CHECK(hipFree(cnt));
  TNP_CHECK(hipFree(cur));
  r->g = g;
  r->V = d_V;
  r->F = d_F;
  r->nF = nF;
  return 0;
}

extern "C" int tnp_raycaster_cast(tnp_raycaster* r, const float* d_o, const float* d_d, int64_t nR,
                                  float* d_t, int32_t* d_face, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(r->device));
  if (!r->off) { tnp_set_error("raycaster not built"); return -1; }
  if (nR <= 0) return 0;
  hipLaunchKernelGGL(k_ray_cast, dim3(tnp_grid(nR)), dim3(TNP_BLOCK), 0, s, r->V, r->F, r->g, r->off,
                     r->items, d_o, d_d, nR, d_t, d_face);
  TNP_CHECK(hipGetLastError());
  return 0;
}

extern "C" int tnp_nn_min_dist(const float* d_a, int64_t na, const float* d_b, int64_t nb,
                               float* d_out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (na <= 0) return 0;
  if (nb <= 0) { tnp_set_error("nearest neighbour against an empty set"); return -1; }
  hipLaunchKernelGGL(k_nn_min_dist, dim3(tnp_grid(na)), dim3(TNP_BLOCK), 0, s, d_a, na, d_b, nb, d_out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
