// extract_faces (tropical/subpoly.py:584-728, tropical/geometry.py:483-556)
// on the device.
//
//  F1 regions  : every surface vertex with k zeros among (3 grid + K-1 plane)
//                sign columns spans 2^k sign-resolved regions
//                (regions_to_vertices, subpoly.py:281-340).  Each (cell,
//                signs) key -- two words: the 30-bit cell, the plane signs
//                (up to 62 planes) -- is hashed into an open-addressing
//                table (the signs word claimed by CAS, the cell word
//                published behind it); the slot is the region id.  Only ids
//                are hashed -- no output order comes from the table.
//  F2 rows     : regions with >= 3 members (mean_points_with_valid) keep
//                their member list sorted by (k, vertex id) = the stable
//                argsort order of r_idx_as_tensor (subpoly.py:357).
//  F3 unique   : rows sorted lexicographically with -1 padding and
//                de-duplicated (v_indices.unique(dim=0), subpoly.py:620):
//                counting sort by first vertex, then a per-bucket sort.
//  F4 polygons : normal = grad sdf at the row mean; members ordered by
//                s = cos * sgn(d) + 2[d<0] descending, d = (u0 x u) . n
//                (sort_polygon_vertices_batch, geometry.py:483-525).
//  F5 fans     : (v0, v_t+1, v_t+2) emitted fan-position-major
//                (tensor_to_triangle_faces, subpoly.py:700-728): triangle
//                (t, row r) lands at sum_{t'<t} n_t' + #rows<r with c>=t+3,
//                from one t-major histogram scan.
#include "common.h"
#include "faces.h"
#include "kernels.h"
#include <algorithm>
#include <cstdlib>

namespace {

constexpr uint64_t EMPTY = ~0ull;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

template <int KW>
struct VKey {
  int k;        // zeros among the region columns
  int zc[3];    // grid zero dims
  int nzg;      // number of grid zeros
  Key<KW> pz;   // plane zeros (planes < nplanes)
  Key<KW> ps;   // plane positive signs
  int off[3];
};

template <int KW>
__device__ __forceinline__ VKey<KW> vkey(uint64_t g, const Key<KW>& pos, const Key<KW>& zero, const Key<KW>& pmask) {
  VKey<KW> r;
  r.nzg = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    r.off[d] = tnp::grid_off(g, d);
    if (tnp::grid_zero(g, d)) r.zc[r.nzg++] = d;
  }
  r.pz = zero & pmask;
  r.ps = pos & pmask;
  r.k = r.nzg + tnp::key_pop(r.pz);
  return r;
}
template <int KW>
__device__ __forceinline__ VKey<KW> vkey_of(int64_t v, const uint64_t* grid, const uint64_t* pos,
                                            const uint64_t* zero, const Key<KW>& pmask) {
  return vkey<KW>(grid[v], tnp::vkey_load<KW>(pos, v), tnp::vkey_load<KW>(zero, v), pmask);
}

// a region key: cell word (3 x 10-bit cell coordinates + 2, never 0) and the
// plane-sign words (bit j: plane j positive).  One-word nets: planes < K - 1
// <= 62, so the sign word is never all ones (the table's EMPTY claim word)
template <int KW>
struct RKey {
  uint64_t cell;
  Key<KW> signs;
};
constexpr uint64_t NO_CELL = 0ull;

// augmented key of pattern p (torch.cartesian_prod order: the first zero
// column is the most significant pattern bit; 0 -> -1, 1 -> +1)
template <int KW>
__device__ __forceinline__ RKey<KW> aug_key(const VKey<KW>& v, uint32_t p) {
  int cell[3] = {v.off[0], v.off[1], v.off[2]};
  int j = 0;
  for (int i = 0; i < v.nzg; ++i, ++j) {
    int b = (p >> (v.k - 1 - j)) & 1;
    cell[v.zc[i]] = b ? v.off[v.zc[i]] : v.off[v.zc[i]] - 1;
  }
  Key<KW> signs = v.ps;
#pragma unroll
  for (int q = 0; q < KW; ++q)
    for (uint64_t t = v.pz.w[q]; t; t &= t - 1, ++j) {
      int pl = __builtin_ctzll(t);
      int b = (p >> (v.k - 1 - j)) & 1;
      if (b) signs.w[q] |= 1ull << pl;
    }
  return RKey<KW>{((uint64_t)(cell[0] + 2) << 20) | ((uint64_t)(cell[1] + 2) << 10) | (uint64_t)(cell[2] + 2),
                  signs};
}

template <int KW>
__global__ void k_face_count(int64_t V, const uint64_t* __restrict__ grid, const uint64_t* __restrict__ pos,
                             const uint64_t* __restrict__ zero, Key<KW> pmask, int64_t* __restrict__ ctr) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t a = 0;
  int kmax = 0;
  if (v < V) {
    VKey<KW> k = vkey_of<KW>(v, grid, pos, zero, pmask);
    a = 1ll << k.k;
    kmax = k.k;
  }
  a = tnp::wave_sum(a);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o, 64));
  if (tnp::lane() == 0) {
    atomicAdd((unsigned long long*)&ctr[0], (unsigned long long)a);
    atomicMax((unsigned long long*)&ctr[1], (unsigned long long)kmax);
  }
}

// One-word table: [cap] sign words (EMPTY: free) then [cap] cell words
// (NO_CELL: not yet published).  A slot is claimed by CAS on its sign word and the
// claiming lane publishes the cell word in the same loop round; a lane that
// found the same sign word reads the cell word once per round (no inner
// wait: every lane advances one step per round, so a lane never waits on a
// store its own wave has not yet issued).
// Two-word table (K > 63: a sign word may be all ones): [cap] cell words
// (NO_CELL: free, claimed by CAS), [cap] low and [cap] high sign words,
// [cap] ready words (release-stored by the claimer behind its sign words),
// the same one-step-per-round loop.
__device__ __forceinline__ uint64_t rkey_hash(const RKey<1>& k) { return mix64(k.signs.w[0] ^ mix64(k.cell)); }
__device__ __forceinline__ uint64_t rkey_hash(const RKey<2>& k) {
  return mix64(k.signs.w[1] ^ mix64(k.signs.w[0] ^ mix64(k.cell)));
}

__device__ __forceinline__ uint64_t probe_insert(uint64_t* table, uint64_t mask, const RKey<1>& key) {
  uint64_t* cells = table + mask + 1;
  uint64_t h = rkey_hash(key) & mask;
  bool polling = false;  // slot h holds our signs; its cell word was not published yet
  while (true) {
    if (!polling) {
      const uint64_t prev = atomicCAS((unsigned long long*)&table[h], (unsigned long long)EMPTY,
                                      (unsigned long long)key.signs.w[0]);
      if (prev == EMPTY) {
        tnp::st_agent(cells + h, key.cell);
        return h;
      }
      if (prev != key.signs.w[0]) {
        h = (h + 1) & mask;
        continue;
      }
    }
    const uint64_t c = tnp::ld_agent(cells + h);
    polling = c == NO_CELL;
    if (polling) continue;
    if (c == key.cell) return h;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ uint64_t probe_insert(uint64_t* table, uint64_t mask, const RKey<2>& key) {
  const uint64_t cap = mask + 1;
  uint64_t* s0 = table + cap;
  uint64_t* s1 = table + 2 * cap;
  uint64_t* ready = table + 3 * cap;
  uint64_t h = rkey_hash(key) & mask;
  bool polling = false;  // slot h holds our cell; its sign words were not published yet
  while (true) {
    if (!polling) {
      const uint64_t prev = atomicCAS((unsigned long long*)&table[h], (unsigned long long)NO_CELL,
                                      (unsigned long long)key.cell);
      if (prev == NO_CELL) {
        tnp::st_agent(s0 + h, key.signs.w[0]);
        tnp::st_agent(s1 + h, key.signs.w[1]);
        __hip_atomic_store(ready + h, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return h;
      }
      if (prev != key.cell) {
        h = (h + 1) & mask;
        continue;
      }
    }
    const uint64_t r = __hip_atomic_load(ready + h, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    polling = r == 0;
    if (polling) continue;
    if (tnp::ld_agent(s0 + h) == key.signs.w[0] && tnp::ld_agent(s1 + h) == key.signs.w[1]) return h;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ uint64_t probe_find(const uint64_t* table, uint64_t mask, const RKey<1>& key) {
  const uint64_t* cells = table + mask + 1;
  uint64_t h = rkey_hash(key) & mask;
  while (table[h] != key.signs.w[0] || cells[h] != key.cell) h = (h + 1) & mask;
  return h;
}
__device__ __forceinline__ uint64_t probe_find(const uint64_t* table, uint64_t mask, const RKey<2>& key) {
  const uint64_t cap = mask + 1;
  uint64_t h = rkey_hash(key) & mask;
  while (table[h] != key.cell || table[cap + h] != key.signs.w[0] || table[2 * cap + h] != key.signs.w[1])
    h = (h + 1) & mask;
  return h;
}

template <int KW>
__global__ void k_face_insert(int64_t V, const uint64_t* __restrict__ grid, const uint64_t* __restrict__ pos,
                              const uint64_t* __restrict__ zero, Key<KW> pmask, uint64_t* __restrict__ table,
                              uint64_t tmask, int32_t* __restrict__ cnt) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  VKey<KW> k = vkey_of<KW>(v, grid, pos, zero, pmask);
  for (uint32_t p = 0; p < (1u << k.k); ++p) {
    uint64_t s = probe_insert(table, tmask, aug_key<KW>(k, p));
    atomicAdd(&cnt[s], 1);
  }
}

__global__ void k_keep_counts(const int32_t* __restrict__ cnt, int64_t n, int32_t* __restrict__ kc,
                              int32_t* __restrict__ kf) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int c = cnt[i];
  kc[i] = c >= 3 ? c : 0;
  kf[i] = c >= 3 ? 1 : 0;
}

template <int KW>
__global__ void k_face_scatter(int64_t V, const uint64_t* __restrict__ grid, const uint64_t* __restrict__ pos,
                               const uint64_t* __restrict__ zero, Key<KW> pmask,
                               const uint64_t* __restrict__ table, uint64_t tmask,
                               const int32_t* __restrict__ cnt, const int64_t* __restrict__ memoff,
                               int32_t* __restrict__ cur, uint64_t* __restrict__ mem) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  VKey<KW> k = vkey_of<KW>(v, grid, pos, zero, pmask);
  for (uint32_t p = 0; p < (1u << k.k); ++p) {
    uint64_t s = probe_find(table, tmask, aug_key<KW>(k, p));
    if (cnt[s] < 3) continue;
    int64_t at = memoff[s] + atomicAdd(&cur[s], 1);
    mem[at] = ((uint64_t)(uint32_t)k.k << 32) | (uint64_t)(uint32_t)v;
  }
}

template <typename T>
__device__ __forceinline__ void shell_sort(T* a, int n) {
  int gap = 1;
  while (gap < n / 3) gap = 3 * gap + 1;
  for (; gap > 0; gap /= 3)
    for (int i = gap; i < n; ++i) {
      T x = a[i];
      int j = i;
      while (j >= gap && a[j - gap] > x) {
        a[j] = a[j - gap];
        j -= gap;
      }
      a[j] = x;
    }
}

// per kept slot: region id, member range; members sorted by (k, v)
__global__ void k_region_finalize(int64_t n, const int32_t* __restrict__ kf, const int64_t* __restrict__ rid,
                                  const int32_t* __restrict__ cnt, const int64_t* __restrict__ memoff,
                                  uint64_t* __restrict__ mem, int64_t* __restrict__ roff,
                                  int32_t* __restrict__ rcnt) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n || !kf[s]) return;
  int64_t r = rid[s];
  int c = cnt[s];
  roff[r] = memoff[s];
  rcnt[r] = c;
  shell_sort(mem + memoff[s], c);
}

__device__ __forceinline__ int row_v(const uint64_t* mem, int64_t off, int i) {
  return (int)(uint32_t)mem[off + i];
}

// lexicographic compare of two member lists with -1 padding: <0, 0, >0
__device__ __forceinline__ int row_cmp(const uint64_t* mem, const int64_t* roff, const int32_t* rcnt,
                                       int a, int b) {
  int na = rcnt[a], nb = rcnt[b];
  int n = na < nb ? na : nb;
  for (int i = 0; i < n; ++i) {
    int x = row_v(mem, roff[a], i), y = row_v(mem, roff[b], i);
    if (x != y) return x < y ? -1 : 1;
  }
  return na == nb ? 0 : (na < nb ? -1 : 1);  // a shorter prefix has -1 (smaller) next
}

__global__ void k_row_bucket_count(int64_t R, const uint64_t* __restrict__ mem, const int64_t* __restrict__ roff,
                                   int32_t* __restrict__ bcnt) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) atomicAdd(&bcnt[row_v(mem, roff[r], 0)], 1);
}

__global__ void k_row_bucket_scatter(int64_t R, const uint64_t* __restrict__ mem, const int64_t* __restrict__ roff,
                                     const int64_t* __restrict__ boff, int32_t* __restrict__ bcur,
                                     int32_t* __restrict__ rows) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  int v0 = row_v(mem, roff[r], 0);
  rows[boff[v0] + atomicAdd(&bcur[v0], 1)] = (int32_t)r;
}

__global__ void k_row_bucket_sort(int64_t V, const int64_t* __restrict__ boff, const int32_t* __restrict__ bcnt,
                                  int32_t* __restrict__ rows, const uint64_t* __restrict__ mem,
                                  const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt,
                                  int32_t* __restrict__ keep) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  int n = bcnt[v];
  if (n == 0) return;
  int32_t* a = rows + boff[v];
  int gap = 1;
  while (gap < n / 3) gap = 3 * gap + 1;
  for (; gap > 0; gap /= 3)
    for (int i = gap; i < n; ++i) {
      int32_t x = a[i];
      int j = i;
      while (j >= gap && row_cmp(mem, roff, rcnt, a[j - gap], x) > 0) {
        a[j] = a[j - gap];
        j -= gap;
      }
      a[j] = x;
    }
  int32_t* kp = keep + boff[v];
  kp[0] = 1;
  for (int i = 1; i < n; ++i) kp[i] = row_cmp(mem, roff, rcnt, a[i - 1], a[i]) != 0;
}

__global__ void k_compact_rows(int64_t n, const int32_t* __restrict__ keep, const int64_t* __restrict__ koff,
                               const int32_t* __restrict__ rows, int32_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && keep[i]) out[koff[i]] = rows[i];
}

// ---------------------------------------------------------------------------
// torch CPU float semantics the polygon sort depends on (pinned by probes in
// tools/torch_cpu_semantics.py):
//  * Tensor.sum over the padded row width M (dim=-2): ATen cascade row_sum
//    with 4 interleaved lanes, tail into lane 0, lanes added in order
//  * torch.cross (CPU): out0 = fma(a1, b2, -(a2*b1)) (gcc-contracted)
//  * linalg.vector_norm: sqrt_rn(fma(z,z, fma(y,y, x*x)))
//  * bmm of a 3-vector: (c0*n0 + c1*n1) + c2*n2, no fma
//  * cosine_similarity: (a/max(|a|,1e-8)) * (b/max(|b|,1e-8)), summed in order
// ---------------------------------------------------------------------------
__device__ __forceinline__ int ceil_log2(int64_t x) {
  if (x <= 2) return 1;
  return 64 - __builtin_clzll((uint64_t)(x - 1));
}

// row_sum of coordinate d over positions [0, M) of a row whose first c
// positions hold members (the rest are zero padding)
__device__ float torch_row_sum(const uint64_t* mem, int64_t off, int c, int M, int d,
                               const float* xyz) {
  auto X = [&](int64_t p) -> float {
    if (p >= c) return 0.f;
    int v = (int)(uint32_t)mem[off + p];
    return xyz[3 * (int64_t)v + d];
  };
  const int64_t size = M / 4;
  float acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[j][k] = 0.f;
  const int level_power = max(4, ceil_log2(size) / 4);
  const int64_t level_step = 1ll << level_power;
  const int64_t level_mask = level_step - 1;
  int64_t i = 0;
  for (; i + level_step <= size;) {
    for (int64_t j = 0; j < level_step; ++j, ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[0][k] = __fadd_rn(acc[0][k], X(i * 4 + k));
    for (int j = 1; j < 4; ++j) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[j][k] = __fadd_rn(acc[j][k], acc[j - 1][k]);
        acc[j - 1][k] = 0.f;
      }
      if ((i & (level_mask << (j * level_power))) != 0) break;
    }
  }
  for (; i < size; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[0][k] = __fadd_rn(acc[0][k], X(i * 4 + k));
  for (int j = 1; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[0][k] = __fadd_rn(acc[0][k], acc[j][k]);
  for (int64_t p = size * 4; p < M; ++p) acc[0][0] = __fadd_rn(acc[0][0], X(p));
  float r = acc[0][0];
  r = __fadd_rn(r, acc[0][1]);
  r = __fadd_rn(r, acc[0][2]);
  r = __fadd_rn(r, acc[0][3]);
  return r;
}

__device__ __forceinline__ bool nonzero3(const float* p) {
  return p[0] != 0.f || p[1] != 0.f || p[2] != 0.f;
}

// mean_points_with_valid: points.sum(dim=1) / Z (subpoly.py:669-678)
__global__ void k_row_mean(int64_t F, const int32_t* __restrict__ frow, const uint64_t* __restrict__ mem,
                           const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt, int M,
                           const float* __restrict__ xyz, float* __restrict__ mean) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  int r = frow[f];
  int c = rcnt[r];
#pragma unroll
  for (int d = 0; d < 3; ++d)
    mean[3 * f + d] = __fdiv_rn(torch_row_sum(mem, roff[r], c, M, d, xyz), (float)c);
}

// centroid of sort_polygon_vertices_batch: v.sum(dim=-2) / max(#{|v|>0}, 1)
__device__ __forceinline__ void row_centroid(const uint64_t* mem, int64_t off, int c, int M,
                                             const float* xyz, float cen[3]) {
  int k = 0;
  for (int i = 0; i < c; ++i) {
    int v = (int)(uint32_t)mem[off + i];
    k += nonzero3(xyz + 3 * (int64_t)v);
  }
  if (k == 0) k = 1;
#pragma unroll
  for (int d = 0; d < 3; ++d) cen[d] = __fdiv_rn(torch_row_sum(mem, off, c, M, d, xyz), (float)k);
}

__device__ __forceinline__ void cross3(const float a[3], const float b[3], float o[3]) {
  o[0] = __fmaf_rn(a[1], b[2], -__fmul_rn(a[2], b[1]));
  o[1] = __fmaf_rn(a[2], b[0], -__fmul_rn(a[0], b[2]));
  o[2] = __fmaf_rn(a[0], b[1], -__fmul_rn(a[1], b[0]));
}

__device__ __forceinline__ float vnorm3(const float a[3]) {
  // sqrtf, not __fsqrt_rn: on gfx950 only sqrtf is correctly rounded (tools/diag_ops.py)
  return sqrtf(__fmaf_rn(a[2], a[2], __fmaf_rn(a[1], a[1], __fmul_rn(a[0], a[0]))));
}

__device__ __forceinline__ float cosine(const float a[3], const float b[3]) {
  float na = fmaxf(vnorm3(a), 1e-8f), nb = fmaxf(vnorm3(b), 1e-8f);
  float p0 = __fmul_rn(__fdiv_rn(a[0], na), __fdiv_rn(b[0], nb));
  float p1 = __fmul_rn(__fdiv_rn(a[1], na), __fdiv_rn(b[1], nb));
  float p2 = __fmul_rn(__fdiv_rn(a[2], na), __fdiv_rn(b[2], nb));
  return __fadd_rn(__fadd_rn(p0, p1), p2);
}

__device__ __forceinline__ float dot3_bmm(const float c[3], const float n[3]) {
  return __fadd_rn(__fadd_rn(__fmul_rn(c[0], n[0]), __fmul_rn(c[1], n[1])), __fmul_rn(c[2], n[2]));
}

// F4a: angular score of every entry of every final row's PADDED row (width
// M = the largest region; pads are the zero point), exactly as
// sort_polygon_vertices_batch evaluates it -- the pads matter because the
// reference sorts them together with the members (an unstable sort, so
// their positions steer how exact ties among members resolve).
// quirk3: torch.cross without dim= picks dim 0 when there are exactly 3 rows
// (geometry.py:500).
__global__ void k_row_score(int64_t F, const int32_t* __restrict__ frow, const uint64_t* __restrict__ mem,
                            const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt, int M,
                            const float* __restrict__ xyz, const float* __restrict__ nrm, int quirk3,
                            float* __restrict__ skey, int32_t* __restrict__ sidx, int32_t* __restrict__ cnt_all,
                            int32_t* __restrict__ cnt_nz, const int32_t* __restrict__ slow) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F || (slow && !slow[f])) return;
  const int r = frow[f];
  const int c = rcnt[r];
  const int64_t off = roff[r];
  float cen[3];
  row_centroid(mem, off, c, M, xyz, cen);
  const int v0 = row_v(mem, off, 0);
  float u0[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) u0[d] = __fsub_rn(xyz[3 * (int64_t)v0 + d], cen[d]);
  const float n[3] = {nrm[3 * f], nrm[3 * f + 1], nrm[3 * f + 2]};
  float U0[3][3], CEN[3][3];
  int RC[3] = {0, 0, 0};
  int64_t ROFF[3] = {0, 0, 0};
  if (quirk3) {
    for (int q = 0; q < 3; ++q) {
      int rq = frow[q];
      RC[q] = rcnt[rq];
      ROFF[q] = roff[rq];
      row_centroid(mem, ROFF[q], RC[q], M, xyz, CEN[q]);
      int bq = row_v(mem, ROFF[q], 0);
      for (int d = 0; d < 3; ++d) U0[q][d] = __fsub_rn(xyz[3 * (int64_t)bq + d], CEN[q][d]);
    }
  }
  int nz = 0;
  float* key = skey + f * (int64_t)M;
  int32_t* idx = sidx + f * (int64_t)M;
  for (int i = 0; i < M; ++i) {
    float p[3] = {0.f, 0.f, 0.f};
    if (i < c) {
      int v = row_v(mem, off, i);
      p[0] = xyz[3 * (int64_t)v];
      p[1] = xyz[3 * (int64_t)v + 1];
      p[2] = xyz[3 * (int64_t)v + 2];
      nz += nonzero3(p);
    }
    float u[3] = {__fsub_rn(p[0], cen[0]), __fsub_rn(p[1], cen[1]), __fsub_rn(p[2], cen[2])};
    float dd = 0.f;
    if (!quirk3) {
      float cr[3];
      cross3(u0, u, cr);
      dd = dot3_bmm(cr, n);
    } else {
      // D[q][m][c] = (a x b)[q] with a = (u_q[0][c])_q, b = (u_q[m][c])_q
      float col[3];
      for (int cc = 0; cc < 3; ++cc) {
        float av[3], bv[3], o[3];
        for (int q = 0; q < 3; ++q) {
          av[q] = U0[q][cc];
          float pq = 0.f;
          if (i < RC[q]) pq = xyz[3 * (int64_t)row_v(mem, ROFF[q], i) + cc];
          bv[q] = __fsub_rn(pq, CEN[q][cc]);
        }
        cross3(av, bv, o);
        col[cc] = o[f];
      }
      dd = dot3_bmm(col, n);
    }
    float cs = cosine(u0, u);
    key[i] = __fadd_rn(__fmul_rn(cs, dd >= 0.f ? 1.f : -1.f), dd < 0.f ? 2.f : 0.f);
    idx[i] = i;
  }
  cnt_all[f] = c;
  cnt_nz[f] = nz;
}

// F4 fast path.  The pads of a padded row are all the zero point, so they
// share one key; the sort is unstable, but when no two of the c member keys
// and the pad key are equal (and none is NaN), every member's place is its
// rank in descending key order whatever the introsort does with the pads --
// so such a row is ordered in registers, without the padded M-entry sort.
// Rows with an exact tie (or more than FAST_MAX members, or the 3-row cross
// quirk) are flagged for k_row_score + k_row_sort.  Same keys as k_row_score.
constexpr int FAST_MAX = 16;
__global__ void __launch_bounds__(TNP_BLOCK)
k_row_fast(int64_t F, const int32_t* __restrict__ frow, const uint64_t* __restrict__ mem,
           const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt, int M,
           const float* __restrict__ xyz, const float* __restrict__ nrm, int32_t* __restrict__ ordv,
           int32_t* __restrict__ cnt_all, int32_t* __restrict__ cnt_nz, int32_t* __restrict__ slow) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  const int r = frow[f];
  const int c = rcnt[r];
  const int64_t off = roff[r];
  if (c > FAST_MAX) {
    slow[f] = 1;
    return;
  }
  float cen[3];
  row_centroid(mem, off, c, M, xyz, cen);
  const int v0 = row_v(mem, off, 0);
  float u0[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) u0[d] = __fsub_rn(xyz[3 * (int64_t)v0 + d], cen[d]);
  const float n[3] = {nrm[3 * f], nrm[3 * f + 1], nrm[3 * f + 2]};
  auto score = [&](const float p[3]) {
    const float u[3] = {__fsub_rn(p[0], cen[0]), __fsub_rn(p[1], cen[1]), __fsub_rn(p[2], cen[2])};
    float cr[3];
    cross3(u0, u, cr);
    const float dd = dot3_bmm(cr, n);
    const float cs = cosine(u0, u);
    return __fadd_rn(__fmul_rn(cs, dd >= 0.f ? 1.f : -1.f), dd < 0.f ? 2.f : 0.f);
  };
  float key[FAST_MAX];
  int id[FAST_MAX];
  int nz = 0;
  bool tie = false;
  for (int i = 0; i < c; ++i) {
    const int v = row_v(mem, off, i);
    const float p[3] = {xyz[3 * (int64_t)v], xyz[3 * (int64_t)v + 1], xyz[3 * (int64_t)v + 2]};
    nz += nonzero3(p);
    key[i] = score(p);
    id[i] = v;
    tie |= isnan(key[i]);
  }
  if (c < M) {
    const float z[3] = {0.f, 0.f, 0.f};
    const float kp = score(z);
    tie |= isnan(kp);
    for (int i = 0; i < c; ++i) tie |= key[i] == kp;
  }
  for (int i = 1; i < c && !tie; ++i) {  // insertion sort, descending; an equal key is a tie
    const float k = key[i];
    const int v = id[i];
    int j = i - 1;
    while (j >= 0 && key[j] < k) {
      key[j + 1] = key[j];
      id[j + 1] = id[j];
      --j;
    }
    tie |= j >= 0 && key[j] == k;
    key[j + 1] = k;
    id[j + 1] = v;
  }
  slow[f] = tie ? 1 : 0;
  if (tie) return;
  for (int i = 0; i < c; ++i) ordv[off + i] = id[i];
  cnt_all[f] = c;
  cnt_nz[f] = nz;
}

// ---- libstdc++ std::sort (introsort) with torch's KeyValueCompDesc ----------
// torch.sort(descending=True, stable=False) on CPU (ATen SortingKernel) runs
// std::sort over (value, index) pairs comparing values only; emulated step by
// step so that exact ties land where the reference puts them.
struct KV {
  float k;
  int32_t v;
};

__device__ __forceinline__ bool kv_less(const KV& a, const KV& b) {  // "comes first"
  return (isnan(a.k) && !isnan(b.k)) || (a.k > b.k);
}
__device__ __forceinline__ void kv_swap(KV* a, KV* b) {
  KV t = *a;
  *a = *b;
  *b = t;
}
__device__ void unguarded_linear_insert(KV* last) {
  KV val = *last;
  KV* next = last - 1;
  while (kv_less(val, *next)) {
    *last = *next;
    last = next;
    --next;
  }
  *last = val;
}
__device__ void insertion_sort(KV* first, KV* last) {
  if (first == last) return;
  for (KV* i = first + 1; i != last; ++i) {
    if (kv_less(*i, *first)) {
      KV val = *i;
      for (KV* p = i; p != first; --p) *p = *(p - 1);
      *first = val;
    } else {
      unguarded_linear_insert(i);
    }
  }
}
__device__ void move_median_to_first(KV* result, KV* a, KV* b, KV* c) {
  if (kv_less(*a, *b)) {
    if (kv_less(*b, *c)) kv_swap(result, b);
    else if (kv_less(*a, *c)) kv_swap(result, c);
    else kv_swap(result, a);
  } else if (kv_less(*a, *c)) {
    kv_swap(result, a);
  } else if (kv_less(*b, *c)) {
    kv_swap(result, c);
  } else {
    kv_swap(result, b);
  }
}
__device__ KV* unguarded_partition(KV* first, KV* last, KV* pivot) {
  while (true) {
    while (kv_less(*first, *pivot)) ++first;
    --last;
    while (kv_less(*pivot, *last)) --last;
    if (!(first < last)) return first;
    kv_swap(first, last);
    ++first;
  }
}
__device__ void push_heap_(KV* first, int64_t hole, int64_t top, KV value) {
  int64_t parent = (hole - 1) / 2;
  while (hole > top && kv_less(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}
__device__ void adjust_heap(KV* first, int64_t hole, int64_t len, KV value) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (kv_less(first[child], first[child - 1])) child--;
    first[hole] = first[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = first[child - 1];
    hole = child - 1;
  }
  push_heap_(first, hole, top, value);
}
__device__ void heap_sort(KV* first, KV* last) {  // std::__partial_sort(first, last, last)
  int64_t len = last - first;
  if (len >= 2) {
    for (int64_t parent = (len - 2) / 2;; --parent) {
      adjust_heap(first, parent, len, first[parent]);
      if (parent == 0) break;
    }
  }
  while (last - first > 1) {
    --last;
    KV value = *last;
    *last = *first;
    adjust_heap(first, 0, last - first, value);
  }
}
__device__ void std_sort(KV* first, KV* last) {
  const int64_t n = last - first;
  if (n <= 1) return;
  int depth0 = 2 * (63 - __builtin_clzll((uint64_t)n));
  // introsort loop; sub-ranges are independent, so an explicit stack
  // visits them in a different order with identical results
  struct Rng { KV* f; KV* l; int d; };
  Rng stack[64];
  int sp = 0;
  stack[sp++] = {first, last, depth0};
  while (sp) {
    Rng g = stack[--sp];
    KV* f = g.f;
    KV* l = g.l;
    int depth = g.d;
    while (l - f > 16) {
      if (depth == 0) {
        heap_sort(f, l);
        l = f;
        break;
      }
      --depth;
      KV* mid = f + (l - f) / 2;
      move_median_to_first(f, f + 1, mid, l - 1);
      KV* cut = unguarded_partition(f + 1, l, f);
      stack[sp++] = {cut, l, depth};
      l = cut;
    }
  }
  if (n > 16) {
    insertion_sort(first, first + 16);
    for (KV* i = first + 16; i != last; ++i) unguarded_linear_insert(i);
  } else {
    insertion_sort(first, last);
  }
}

// F4b: sort each padded row and write the members' ids in sorted order
// (slow != null: only the rows k_row_fast left to this path)
__global__ void k_row_sort(int64_t F, const int32_t* __restrict__ frow, const uint64_t* __restrict__ mem,
                           const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt, int M,
                           KV* __restrict__ kv, const float* __restrict__ skey, const int32_t* __restrict__ sidx,
                           int32_t* __restrict__ ordv, const int32_t* __restrict__ slow) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F || (slow && !slow[f])) return;
  const int r = frow[f];
  const int c = rcnt[r];
  const int64_t off = roff[r];
  KV* a = kv + f * (int64_t)M;
  for (int i = 0; i < M; ++i) a[i] = KV{skey[f * (int64_t)M + i], sidx[f * (int64_t)M + i]};
  std_sort(a, a + M);
  int j = 0;
  for (int i = 0; i < M; ++i)
    if (a[i].v < c) ordv[off + j++] = row_v(mem, off, a[i].v);
}

// the largest v over the block (every thread calls it; two barriers)
__device__ __forceinline__ int block_max(int v, int* lds) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  if (tnp::lane() == 0) lds[tnp::wave()] = v;
  __syncthreads();
  int m = lds[0];
#pragma unroll
  for (int w = 1; w < TNP_WAVES; ++w) m = max(m, lds[w]);
  __syncthreads();
  return m;
}

// F5: per block of rows, how many rows have c >= t+3, t-major layout
__global__ void __launch_bounds__(TNP_BLOCK)
k_fan_hist(int64_t F, const int32_t* __restrict__ cnt, int T, int64_t nb, int32_t* __restrict__ hist) {
  __shared__ int lds[TNP_WAVES];
  int64_t f = (int64_t)blockIdx.x * TNP_BLOCK + threadIdx.x;
  int c = f < F ? cnt[f] : 0;
  // fan positions past this block's largest row hold none of its rows (T is
  // the largest row over all rows): ranked only up to the block's own
  const int tb = min(T, block_max(c, lds) - 2);
  for (int t = 0; t < tb; ++t) {
    int tot;
    (void)tnp::block_rank(c >= t + 3, lds, tot);
    if (threadIdx.x == 0) hist[(int64_t)t * nb + blockIdx.x] = tot;
  }
  for (int t = max(tb, 0) + threadIdx.x; t < T; t += TNP_BLOCK) hist[(int64_t)t * nb + blockIdx.x] = 0;
}

// i-th ordered member with a non-zero position (the float faces' mask m)
__device__ __forceinline__ int nz_member(const int32_t* a, int c, int i, const float* xyz) {
  for (int j = 0; j < c; ++j) {
    int v = a[j];
    bool nzv = xyz[3 * (int64_t)v] != 0.f || xyz[3 * (int64_t)v + 1] != 0.f || xyz[3 * (int64_t)v + 2] != 0.f;
    if (nzv && i-- == 0) return v;
  }
  return a[0];
}

__global__ void __launch_bounds__(TNP_BLOCK)
k_fan_emit(int64_t F, const int32_t* __restrict__ frow, const int32_t* __restrict__ ordv,
           const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt, const int32_t* __restrict__ cnt,
           int T, int64_t nb, const int64_t* __restrict__ base, int floats, const float* __restrict__ xyz,
           int64_t* __restrict__ tri, float* __restrict__ fc) {
  __shared__ int lds[TNP_WAVES];
  int64_t f = (int64_t)blockIdx.x * TNP_BLOCK + threadIdx.x;
  int c = 0, rc = 0;
  const int32_t* a = nullptr;
  if (f < F) {
    int r = frow[f];
    c = cnt[f];
    rc = rcnt[r];
    a = ordv + roff[r];
  }
  const int tb = min(T, block_max(c, lds) - 2);  // (as k_fan_hist)
  // floats: c counts the row's members off the origin; a row with none at
  // the origin (c == rc, all but a vertex exactly at 0) takes its i-th
  // member directly instead of scanning the row for it per triangle
  const bool clean = c == rc;
  for (int t = 0; t < tb; ++t) {
    bool on = c >= t + 3;
    int tot;
    int rk = tnp::block_rank(on, lds, tot);
    if (!on) continue;
    int64_t at = base[(int64_t)t * nb + blockIdx.x] + rk;
    if (!floats) {
      tri[3 * at + 0] = a[0];
      tri[3 * at + 1] = a[t + 1];
      tri[3 * at + 2] = a[t + 2];
    } else {
      const int ids[3] = {0, t + 1, t + 2};
      for (int q = 0; q < 3; ++q) {
        int v = clean ? a[ids[q]] : nz_member(a, rc, ids[q], xyz);
        for (int d = 0; d < 3; ++d) fc[9 * at + 3 * q + d] = xyz[3 * (int64_t)v + d];
      }
    }
  }
}

}  // namespace

// ----------------------------------------------------------------------------
int launch_face_count(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                      int K, int64_t* ctr2, hipStream_t s) {
  if (V <= 0) return 0;
  if (K > 63)
    hipLaunchKernelGGL(k_face_count<2>, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero,
                       tnp::key_below<2>(K - 1), ctr2);
  else
    hipLaunchKernelGGL(k_face_count<1>, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero,
                       tnp::key_below<1>(K - 1), ctr2);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_face_insert(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                       int K, uint64_t* table, uint64_t tmask, int32_t* cnt, hipStream_t s) {
  if (V <= 0) return 0;
  if (K > 63)
    hipLaunchKernelGGL(k_face_insert<2>, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero,
                       tnp::key_below<2>(K - 1), table, tmask, cnt);
  else
    hipLaunchKernelGGL(k_face_insert<1>, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero,
                       tnp::key_below<1>(K - 1), table, tmask, cnt);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_keep_counts(const int32_t* cnt, int64_t n, int32_t* kc, int32_t* kf, hipStream_t s) {
  hipLaunchKernelGGL(k_keep_counts, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, cnt, n, kc, kf);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_face_scatter(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                        int K, const uint64_t* table, uint64_t tmask, const int32_t* cnt,
                        const int64_t* memoff, int32_t* cur, uint64_t* mem, hipStream_t s) {
  if (V <= 0) return 0;
  if (K > 63)
    hipLaunchKernelGGL(k_face_scatter<2>, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero,
                       tnp::key_below<2>(K - 1), table, tmask, cnt, memoff, cur, mem);
  else
    hipLaunchKernelGGL(k_face_scatter<1>, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero,
                       tnp::key_below<1>(K - 1), table, tmask, cnt, memoff, cur, mem);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_region_finalize(int64_t n, const int32_t* kf, const int64_t* rid, const int32_t* cnt,
                           const int64_t* memoff, uint64_t* mem, int64_t* roff, int32_t* rcnt,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_region_finalize, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, n, kf, rid, cnt, memoff,
                     mem, roff, rcnt);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_row_buckets(int64_t R, int64_t V, const uint64_t* mem, const int64_t* roff, const int32_t* rcnt,
                       int32_t* bcnt, int64_t* boff, int32_t* bcur, int32_t* rows, int32_t* keep, int phase,
                       hipStream_t s) {
  if (phase == 0)
    hipLaunchKernelGGL(k_row_bucket_count, dim3(tnp_grid(R)), dim3(TNP_BLOCK), 0, s, R, mem, roff, bcnt);
  else if (phase == 1)
    hipLaunchKernelGGL(k_row_bucket_scatter, dim3(tnp_grid(R)), dim3(TNP_BLOCK), 0, s, R, mem, roff, boff,
                       bcur, rows);
  else
    hipLaunchKernelGGL(k_row_bucket_sort, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, boff, bcnt, rows, mem,
                       roff, rcnt, keep);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_compact_rows(int64_t n, const int32_t* keep, const int64_t* koff, const int32_t* rows,
                        int32_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_compact_rows, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, n, keep, koff, rows, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_row_mean(int64_t F, const int32_t* frow, const uint64_t* mem, const int64_t* roff,
                    const int32_t* rcnt, int M, const float* xyz, float* mean, hipStream_t s) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(k_row_mean, dim3(tnp_grid(F)), dim3(TNP_BLOCK), 0, s, F, frow, mem, roff, rcnt, M, xyz,
                     mean);
  TNP_CHECK(hipGetLastError());
  return 0;
}
size_t row_order_scratch(int64_t F, int M) { return (size_t)F * M * (sizeof(float) + 4 + sizeof(KV)) + F * 4; }

int launch_row_order(int64_t F, const int32_t* frow, const uint64_t* mem, const int64_t* roff,
                     const int32_t* rcnt, int M, const float* xyz, const float* nrm, int quirk3, void* scratch,
                     int32_t* ordv, int32_t* cnt_all, int32_t* cnt_nz, hipStream_t s) {
  if (F <= 0) return 0;
  float* skey = static_cast<float*>(scratch);
  int32_t* sidx = reinterpret_cast<int32_t*>(skey + F * (int64_t)M);
  KV* kv = reinterpret_cast<KV*>(sidx + F * (int64_t)M);
  // the 3-row quirk (and TNP_ROW_SORT_FULL=1, tests) sorts every padded row
  const char* full = getenv("TNP_ROW_SORT_FULL");
  const bool s_full = full && full[0] == '1';
  int32_t* slow = (quirk3 || s_full) ? nullptr : reinterpret_cast<int32_t*>(kv + F * (int64_t)M);
  if (slow)
    hipLaunchKernelGGL(k_row_fast, dim3(tnp_grid(F)), dim3(TNP_BLOCK), 0, s, F, frow, mem, roff, rcnt, M, xyz, nrm,
                       ordv, cnt_all, cnt_nz, slow);
  hipLaunchKernelGGL(k_row_score, dim3(tnp_grid(F)), dim3(TNP_BLOCK), 0, s, F, frow, mem, roff, rcnt, M, xyz,
                     nrm, quirk3, skey, sidx, cnt_all, cnt_nz, slow);
  hipLaunchKernelGGL(k_row_sort, dim3(tnp_grid(F)), dim3(TNP_BLOCK), 0, s, F, frow, mem, roff, rcnt, M, kv, skey,
                     sidx, ordv, slow);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int64_t fan_blocks(int64_t F) { return (F + TNP_BLOCK - 1) / TNP_BLOCK; }
int launch_fan_hist(int64_t F, const int32_t* cnt, int T, int32_t* hist, hipStream_t s) {
  if (F <= 0 || T <= 0) return 0;
  int64_t nb = fan_blocks(F);
  hipLaunchKernelGGL(k_fan_hist, dim3((unsigned)nb), dim3(TNP_BLOCK), 0, s, F, cnt, T, nb, hist);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_fan_emit(int64_t F, const int32_t* frow, const int32_t* ordv, const int64_t* roff,
                    const int32_t* rcnt, const int32_t* cnt, int T, const int64_t* base, int floats,
                    const float* xyz, int64_t* tri, float* fc, hipStream_t s) {
  if (F <= 0 || T <= 0) return 0;
  int64_t nb = fan_blocks(F);
  hipLaunchKernelGGL(k_fan_emit, dim3((unsigned)nb), dim3(TNP_BLOCK), 0, s, F, frow, ordv, roff, rcnt, cnt, T, nb,
                     base, floats, xyz, tri, fc);
  TNP_CHECK(hipGetLastError());
  return 0;
}

namespace {
// max of a[0..n) -> *out and (b != null) of b[0..n) -> *out_b: the waves
// reduce in LDS, one atomic per workgroup and array on a grid of at most 256
// (one per wave on one word serialised ~4,000 atomics: ~50 us per call)
__global__ void __launch_bounds__(TNP_BLOCK)
k_max_i32(const int32_t* __restrict__ a, const int32_t* __restrict__ b, int64_t n, int64_t* __restrict__ out,
          int64_t* __restrict__ out_b) {
  __shared__ int lds[2][TNP_WAVES];
  int m = 0, mb = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    m = max(m, a[i]);
    if (b) mb = max(mb, b[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m = max(m, __shfl_xor(m, o, 64));
    mb = max(mb, __shfl_xor(mb, o, 64));
  }
  if (tnp::lane() == 0) {
    lds[0][tnp::wave()] = m;
    lds[1][tnp::wave()] = mb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < TNP_WAVES; ++w) {
      m = max(m, lds[0][w]);
      mb = max(mb, lds[1][w]);
    }
    atomicMax((unsigned long long*)out, (unsigned long long)m);
    if (b) atomicMax((unsigned long long*)out_b, (unsigned long long)mb);
  }
}
}  // namespace

int launch_max_i32(const int32_t* a, int64_t n, int64_t* out, hipStream_t s, const int32_t* b, int64_t* out_b) {
  if (n <= 0) return 0;
  unsigned g = (unsigned)std::min<int64_t>(tnp_grid(n), 256);
  hipLaunchKernelGGL(k_max_i32, dim3(g), dim3(TNP_BLOCK), 0, s, a, b, n, out, out_b);
  TNP_CHECK(hipGetLastError());
  return 0;
}
