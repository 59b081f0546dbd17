// TropicalHashGrid.skeleton(net, unit=128) (tropical/tropical.py:158-225) on
// the device, both pruning modes of the reference:
//   "distance" (PRUNING_MODE's value there, _skeleton_dist, tropical.py:111-136)
//   "sign"     (the dormant branch, tropical.py:198-202 -> _skeleton,
//               tropical.py:80-109: an edge is kept iff its endpoints' eps-sign
//               vectors over all planes differ)
//
// Per reference tile (starts range(0, L, unit-1), 1-mark overlap):
//   skel_eval   : |sdf| at every tile lattice point + tile max |grad sdf|
//                 (sign mode: skel_points + the forward with packed keys)
//   skel_edges  : axis edges (hi, lo) with both |sdf| <= sqrt(3)*2*dmax*gmax
//                 (sign mode: keys differ), x then y then z, meshgrid-ij order
//                 (count -> scan -> emit)
// then squeeze: used global ids p2v(i,j,k) -> dense ranks (sorted unique),
// vertices = marks[v2p(id)]*2-1 with the reference's float32 v2p division.
// Duplicate edges on tile overlaps are kept, as in the reference.
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "net_device.h"
#include "skeleton.h"

using namespace tnpnet;

namespace {

constexpr int IPT = 8;
constexpr int TILE = TNP_BLOCK * IPT;

// k_skel_eval (|sdf| + the tile max |grad sdf|) lives in net_lv.hip

struct TileGeom {
  int i0, j0, k0, n0, n1, n2, L;
  int64_t nx, ny, nz;
  int kw;  // sign mode: sign-key words (the keys are (pos, zero) pairs of kw words each)
};

// the tile's lattice points as vertices (marks * 2 - 1, preprocess_inverse)
__global__ void k_skel_points(int i0, int j0, int k0, int n0, int n1, int n2, const float* __restrict__ marks,
                              float* __restrict__ xyz) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n0 * n1 * n2) return;
  const int k = (int)(t % n2), j = (int)((t / n2) % n1), i = (int)(t / ((int64_t)n1 * n2));
  const int ix[3] = {i0 + i, j0 + j, k0 + k};
#pragma unroll
  for (int d = 0; d < 3; ++d) xyz[3 * t + d] = __fsub_rn(__fmul_rn(marks[ix[d]], 2.0f), 1.0f);
}

// keys != null: sign mode (keep iff the endpoints' (pos, zero) keys differ)
__device__ __forceinline__ bool skel_edge(const TileGeom& g, const float* dist, const ulonglong2* keys,
                                          float thr, int64_t c, int& hi, int& lo) {
  int a0, a1, a2, b0, b1, b2;  // lo (a) and hi (b) local coords
  if (c < g.nx) {              // shape (n0-1, n1, n2)
    a2 = (int)(c % g.n2); a1 = (int)((c / g.n2) % g.n1); a0 = (int)(c / ((int64_t)g.n1 * g.n2));
    b0 = a0 + 1; b1 = a1; b2 = a2;
  } else if (c < g.nx + g.ny) {  // shape (n0, n1-1, n2)
    int64_t r = c - g.nx;
    a2 = (int)(r % g.n2); a1 = (int)((r / g.n2) % (g.n1 - 1)); a0 = (int)(r / ((int64_t)(g.n1 - 1) * g.n2));
    b0 = a0; b1 = a1 + 1; b2 = a2;
  } else {                       // shape (n0, n1, n2-1)
    int64_t r = c - g.nx - g.ny;
    a2 = (int)(r % (g.n2 - 1)); a1 = (int)((r / (g.n2 - 1)) % g.n1); a0 = (int)(r / ((int64_t)g.n1 * (g.n2 - 1)));
    b0 = a0; b1 = a1; b2 = a2 + 1;
  }
  const int64_t ia = ((int64_t)a0 * g.n1 + a1) * g.n2 + a2, ib = ((int64_t)b0 * g.n1 + b1) * g.n2 + b2;
  const int64_t LL = (int64_t)g.L * g.L;
  lo = (int)((g.i0 + a0) * LL + (int64_t)(g.j0 + a1) * g.L + (g.k0 + a2));
  hi = (int)((g.i0 + b0) * LL + (int64_t)(g.j0 + b1) * g.L + (g.k0 + b2));
  if (keys) {
    bool d = false;
    for (int q = 0; q < g.kw; ++q) {  // the point's kw (pos, zero) word pairs (common.h pz_store)
      const ulonglong2 ka = keys[g.kw * ia + q], kb = keys[g.kw * ib + q];
      d |= ka.x != kb.x || ka.y != kb.y;
    }
    return d;
  }
  return (dist[ib] <= thr) && (dist[ia] <= thr);
}

__device__ __forceinline__ float skel_threshold(float dmax, const unsigned int* gmax_bits) {
  // sqrt(tensor(3.0)) * 2 * len_max * max_grad, left to right in fp32
  float t = __fmul_rn(sqrtf(3.0f), 2.0f);
  t = __fmul_rn(t, dmax);
  return __fmul_rn(t, __uint_as_float(*gmax_bits));
}

__global__ void __launch_bounds__(TNP_BLOCK)
k_skel_count(TileGeom g, const float* __restrict__ dist, const ulonglong2* __restrict__ keys, float dmax,
             const unsigned int* __restrict__ gmax_bits, int32_t* __restrict__ blk) {
  __shared__ int lds[TNP_WAVES];
  const float thr = keys ? 0.f : skel_threshold(dmax, gmax_bits);
  const int64_t N = g.nx + g.ny + g.nz;
  int64_t base = (int64_t)blockIdx.x * TILE;
  int c = 0;
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    int hi, lo;
    if (i < N) c += skel_edge(g, dist, keys, thr, i, hi, lo);
  }
  c = tnp::wave_sum(c);
  if (tnp::lane() == 0) lds[tnp::wave()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < TNP_WAVES; ++w) t += lds[w];
    blk[blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(TNP_BLOCK)
k_skel_emit(TileGeom g, const float* __restrict__ dist, const ulonglong2* __restrict__ keys, float dmax,
            const unsigned int* __restrict__ gmax_bits, const int64_t* __restrict__ blkoff,
            int64_t out_base, int32_t* __restrict__ out, int32_t* __restrict__ used) {
  __shared__ int lds[TNP_WAVES];
  const float thr = keys ? 0.f : skel_threshold(dmax, gmax_bits);
  const int64_t N = g.nx + g.ny + g.nz;
  int64_t base = (int64_t)blockIdx.x * TILE;
  int64_t run = out_base + blkoff[blockIdx.x];
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    int hi = 0, lo = 0;
    bool f = (i < N) && skel_edge(g, dist, keys, thr, i, hi, lo);
    int tot;
    int r = tnp::block_rank(f, lds, tot);
    if (f) {
      out[2 * (run + r)] = hi;
      out[2 * (run + r) + 1] = lo;
      used[hi] = 1;
      used[lo] = 1;
    }
    run += tot;
  }
}

// the skeleton's load per mark plane (sharded subpoly: the cuts' balance):
// per axis d, load[d * L + m] += the tile's points on plane m of axis d with
// |sdf| under the tile's edge threshold (the candidates of its edges)
__global__ void __launch_bounds__(TNP_BLOCK)
k_skel_load(TileGeom g, const float* __restrict__ dist, float dmax, const unsigned int* __restrict__ gmax_bits,
            unsigned long long* __restrict__ load) {
  extern __shared__ unsigned int hist[];  // [3][L]
  const int L = g.L;
  for (int i = threadIdx.x; i < 3 * L; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const float thr = skel_threshold(dmax, gmax_bits);
  const int64_t n = (int64_t)g.n0 * g.n1 * g.n2;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    if (!(dist[t] <= thr)) continue;
    const int k = (int)(t % g.n2), j = (int)((t / g.n2) % g.n1), i = (int)(t / ((int64_t)g.n1 * g.n2));
    atomicAdd(&hist[g.i0 + i], 1u);
    atomicAdd(&hist[L + g.j0 + j], 1u);
    atomicAdd(&hist[2 * L + g.k0 + k], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * L; i += blockDim.x)
    if (hist[i]) atomicAdd(&load[i], (unsigned long long)hist[i]);
}

__global__ void k_skel_vertices(const int32_t* __restrict__ used, const int64_t* __restrict__ nid,
                                int64_t n, int L, const float* __restrict__ marks,
                                float* __restrict__ xyz) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n || !used[v]) return;
  int64_t r = v;
  int p[3];
  const int64_t Lp[3] = {(int64_t)L * L, (int64_t)L, 1};
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    // v_idx.div(L**i).floor().long(): int64 -> float32 true division
    float q = floorf(__fdiv_rn((float)r, (float)Lp[d]));
    int64_t qi = (int64_t)q;
    p[d] = (int)qi;
    r -= qi * Lp[d];
  }
  int64_t o = nid[v];
#pragma unroll
  for (int d = 0; d < 3; ++d) xyz[3 * o + d] = __fsub_rn(__fmul_rn(marks[p[d]], 2.0f), 1.0f);
}

__global__ void k_remap(int32_t* __restrict__ e, int64_t n, const int64_t* __restrict__ nid) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) e[i] = (int32_t)nid[e[i]];
}

}  // namespace

int launch_skel_eval(const NetDev& net, int i0, int j0, int k0, int n0, int n1, int n2,
                     float* dist, unsigned int* gmax_bits, hipStream_t s) {
  int64_t n = (int64_t)n0 * n1 * n2;
  if (n <= 0) return 0;
  if (!net_supported(net)) { tnp_set_error("unsupported net shape"); return -1; }
  TNP_LV_SWITCH(net.n_levels, return lv_skel_eval<L_>(net, i0, j0, k0, n0, n1, n2, dist, gmax_bits, s));
  return 0;
}

int64_t skel_candidates(int n0, int n1, int n2) {
  return (int64_t)(n0 - 1) * n1 * n2 + (int64_t)n0 * (n1 - 1) * n2 + (int64_t)n0 * n1 * (n2 - 1);
}

int64_t skel_tiles(int64_t n) { return (n + TILE - 1) / TILE; }

static TileGeom geom(int i0, int j0, int k0, int n0, int n1, int n2, int L) {
  TileGeom g{i0, j0, k0, n0, n1, n2, L, (int64_t)(n0 - 1) * n1 * n2,
             (int64_t)n0 * (n1 - 1) * n2, (int64_t)n0 * n1 * (n2 - 1), 1};
  return g;
}

int launch_skel_points(int i0, int j0, int k0, int n0, int n1, int n2, const float* marks, float* xyz,
                       hipStream_t s) {
  const int64_t n = (int64_t)n0 * n1 * n2;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_skel_points, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, i0, j0, k0, n0, n1, n2, marks,
                     xyz);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_skel_edges(bool emit, int i0, int j0, int k0, int n0, int n1, int n2, int L,
                      const float* dist, const uint64_t* keys, float dmax, const unsigned int* gmax_bits,
                      int32_t* blk, const int64_t* blkoff, int64_t out_base, int32_t* out, int32_t* used,
                      hipStream_t s, int kw) {
  TileGeom g = geom(i0, j0, k0, n0, n1, n2, L);
  g.kw = kw;
  int64_t N = g.nx + g.ny + g.nz;
  if (N <= 0) return 0;
  const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(keys);
  if (emit)
    hipLaunchKernelGGL(k_skel_emit, dim3((unsigned)skel_tiles(N)), dim3(TNP_BLOCK), 0, s, g, dist, k2, dmax,
                       gmax_bits, blkoff, out_base, out, used);
  else
    hipLaunchKernelGGL(k_skel_count, dim3((unsigned)skel_tiles(N)), dim3(TNP_BLOCK), 0, s, g, dist, k2,
                       dmax, gmax_bits, blk);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_skel_load(int i0, int j0, int k0, int n0, int n1, int n2, int L, const float* dist, float dmax,
                     const unsigned int* gmax_bits, int64_t* load, hipStream_t s) {
  const int64_t n = (int64_t)n0 * n1 * n2;
  if (n <= 0) return 0;
  if (L > 4096) { tnp_set_error("skeleton load: more than 4096 marks"); return -1; }
  TileGeom g = geom(i0, j0, k0, n0, n1, n2, L);
  const unsigned grid = (unsigned)std::min<int64_t>((n + TNP_BLOCK * 16 - 1) / (TNP_BLOCK * 16), 1024);
  hipLaunchKernelGGL(k_skel_load, dim3(grid), dim3(TNP_BLOCK), 3 * L * sizeof(unsigned int), s, g, dist, dmax,
                     gmax_bits, reinterpret_cast<unsigned long long*>(load));
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_skel_vertices(const int32_t* used, const int64_t* nid, int64_t n, int L,
                         const float* marks, float* xyz, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_skel_vertices, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, used, nid, n, L, marks,
                     xyz);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_remap_i32(int32_t* e, int64_t n, const int64_t* nid, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_remap, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, e, n, nid);
  TNP_CHECK(hipGetLastError());
  return 0;
}
