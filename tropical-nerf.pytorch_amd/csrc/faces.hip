// extract_faces (tropical/subpoly.py:584-728, tropical/geometry.py:483-556)
// on the device.
//
//  F1 regions  : every surface vertex with k zeros among (3 grid + K-1 plane)
//                sign columns spans 2^k sign-resolved regions
//                (regions_to_vertices, subpoly.py:281-340).  Each (cell,
//                signs) key is hashed into an open-addressing table (u64
//                CAS); the slot is the region id.  Only ids are hashed --
//                no output order comes from the table.
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

struct VKey {
  int k;        // zeros among the region columns
  int zc[3];    // grid zero dims
  int nzg;      // number of grid zeros
  uint64_t pz;  // plane zeros (planes < nplanes)
  uint64_t ps;  // plane positive signs
  int off[3];
};

__device__ __forceinline__ VKey vkey(uint64_t g, uint64_t pos, uint64_t zero, uint64_t pmask) {
  VKey r;
  r.nzg = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    r.off[d] = tnp::grid_off(g, d);
    if (tnp::grid_zero(g, d)) r.zc[r.nzg++] = d;
  }
  r.pz = zero & pmask;
  r.ps = pos & pmask;
  r.k = r.nzg + __popcll(r.pz);
  return r;
}

// augmented key of pattern p (torch.cartesian_prod order: the first zero
// column is the most significant pattern bit; 0 -> -1, 1 -> +1)
__device__ __forceinline__ uint64_t aug_key(const VKey& v, uint32_t p) {
  int cell[3] = {v.off[0], v.off[1], v.off[2]};
  int j = 0;
  for (int i = 0; i < v.nzg; ++i, ++j) {
    int b = (p >> (v.k - 1 - j)) & 1;
    cell[v.zc[i]] = b ? v.off[v.zc[i]] : v.off[v.zc[i]] - 1;
  }
  uint64_t signs = v.ps;
  for (uint64_t t = v.pz; t; t &= t - 1, ++j) {
    int pl = __builtin_ctzll(t);
    int b = (p >> (v.k - 1 - j)) & 1;
    if (b) signs |= 1ull << pl;
  }
  return ((uint64_t)(cell[0] + 2) << 54) | ((uint64_t)(cell[1] + 2) << 44) |
         ((uint64_t)(cell[2] + 2) << 34) | signs;
}

__global__ void k_face_count(int64_t V, const uint64_t* __restrict__ grid, const uint64_t* __restrict__ pos,
                             const uint64_t* __restrict__ zero, uint64_t pmask, int64_t* __restrict__ ctr) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t a = 0;
  int kmax = 0;
  if (v < V) {
    VKey k = vkey(grid[v], pos[v], zero[v], pmask);
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

__device__ __forceinline__ uint64_t probe_insert(uint64_t* table, uint64_t mask, uint64_t key) {
  uint64_t h = mix64(key) & mask;
  while (true) {
    uint64_t prev = atomicCAS((unsigned long long*)&table[h], (unsigned long long)EMPTY,
                              (unsigned long long)key);
    if (prev == EMPTY || prev == key) return h;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ uint64_t probe_find(const uint64_t* table, uint64_t mask, uint64_t key) {
  uint64_t h = mix64(key) & mask;
  while (table[h] != key) h = (h + 1) & mask;
  return h;
}

__global__ void k_face_insert(int64_t V, const uint64_t* __restrict__ grid, const uint64_t* __restrict__ pos,
                              const uint64_t* __restrict__ zero, uint64_t pmask, uint64_t* __restrict__ table,
                              uint64_t tmask, int32_t* __restrict__ cnt) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  VKey k = vkey(grid[v], pos[v], zero[v], pmask);
  for (uint32_t p = 0; p < (1u << k.k); ++p) {
    uint64_t s = probe_insert(table, tmask, aug_key(k, p));
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

__global__ void k_face_scatter(int64_t V, const uint64_t* __restrict__ grid, const uint64_t* __restrict__ pos,
                               const uint64_t* __restrict__ zero, uint64_t pmask,
                               const uint64_t* __restrict__ table, uint64_t tmask,
                               const int32_t* __restrict__ cnt, const int64_t* __restrict__ memoff,
                               int32_t* __restrict__ cur, uint64_t* __restrict__ mem) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  VKey k = vkey(grid[v], pos[v], zero[v], pmask);
  for (uint32_t p = 0; p < (1u << k.k); ++p) {
    uint64_t s = probe_find(table, tmask, aug_key(k, p));
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

// mean point of each final row (mean_points_with_valid: sum / #members)
__global__ void k_row_mean(int64_t F, const int32_t* __restrict__ frow, const uint64_t* __restrict__ mem,
                           const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt,
                           const float* __restrict__ xyz, float* __restrict__ mean) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  int r = frow[f];
  int c = rcnt[r];
  float s[3] = {0.f, 0.f, 0.f};
  for (int i = 0; i < c; ++i) {
    int v = row_v(mem, roff[r], i);
#pragma unroll
    for (int d = 0; d < 3; ++d) s[d] += xyz[3 * (int64_t)v + d];
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) mean[3 * f + d] = s[d] / (float)c;
}

__device__ __forceinline__ void row_centroid(const uint64_t* mem, int64_t off, int c, const float* xyz,
                                             float cen[3]) {
  float s[3] = {0.f, 0.f, 0.f};
  int k = 0;
  for (int i = 0; i < c; ++i) {
    int v = row_v(mem, off, i);
    float p[3] = {xyz[3 * (int64_t)v], xyz[3 * (int64_t)v + 1], xyz[3 * (int64_t)v + 2]};
    s[0] += p[0];
    s[1] += p[1];
    s[2] += p[2];
    k += (p[0] != 0.f || p[1] != 0.f || p[2] != 0.f);  // norm > 0
  }
  if (k == 0) k = 1;
#pragma unroll
  for (int d = 0; d < 3; ++d) cen[d] = s[d] / (float)k;
}

__device__ __forceinline__ void cross3(const float a[3], const float b[3], float o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// F.cosine_similarity: (x1/max(|x1|,eps)) . (x2/max(|x2|,eps)), eps=1e-8
__device__ __forceinline__ float cosine(const float a[3], const float b[3]) {
  float na = fmaxf(sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]), 1e-8f);
  float nb = fmaxf(sqrtf(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]), 1e-8f);
  return (a[0] / na) * (b[0] / nb) + (a[1] / na) * (b[1] / nb) + (a[2] / na) * (b[2] / nb);
}

// F4a: angular score of every member of every final row (no in-place
// writes, so the exactly-3-rows quirk can read the other rows).  quirk3:
// torch.cross without dim= picks dim 0 when there are exactly 3 rows
// (geometry.py:500).  key = (descending score << 32) | position.
__global__ void k_row_score(int64_t F, const int32_t* __restrict__ frow, const uint64_t* __restrict__ mem,
                            const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt,
                            const float* __restrict__ xyz, const float* __restrict__ nrm, int quirk3,
                            uint64_t* __restrict__ key, int32_t* __restrict__ cnt_all,
                            int32_t* __restrict__ cnt_nz) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  const int r = frow[f];
  const int c = rcnt[r];
  const int64_t off = roff[r];
  float cen[3];
  row_centroid(mem, off, c, xyz, cen);
  const int v0 = row_v(mem, off, 0);
  float u0[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) u0[d] = xyz[3 * (int64_t)v0 + d] - cen[d];
  const float n[3] = {nrm[3 * f], nrm[3 * f + 1], nrm[3 * f + 2]};
  float U0[3][3], CEN[3][3];
  int RC[3] = {0, 0, 0};
  int64_t ROFF[3] = {0, 0, 0};
  if (quirk3) {
    for (int q = 0; q < 3; ++q) {
      int rq = frow[q];
      RC[q] = rcnt[rq];
      ROFF[q] = roff[rq];
      row_centroid(mem, ROFF[q], RC[q], xyz, CEN[q]);
      int bq = row_v(mem, ROFF[q], 0);
      for (int d = 0; d < 3; ++d) U0[q][d] = xyz[3 * (int64_t)bq + d] - CEN[q][d];
    }
  }
  int nz = 0;
  for (int i = 0; i < c; ++i) {
    int v = row_v(mem, off, i);
    float p[3] = {xyz[3 * (int64_t)v], xyz[3 * (int64_t)v + 1], xyz[3 * (int64_t)v + 2]};
    nz += (p[0] != 0.f || p[1] != 0.f || p[2] != 0.f);
    float u[3] = {p[0] - cen[0], p[1] - cen[1], p[2] - cen[2]};
    float dd = 0.f;
    if (!quirk3) {
      float cr[3];
      cross3(u0, u, cr);
      dd = cr[0] * n[0] + cr[1] * n[1] + cr[2] * n[2];
    } else {
      // D[q][m][c] = (a x b)[q] with a = (u_q[0][c])_q, b = (u_q[m][c])_q
      for (int cc = 0; cc < 3; ++cc) {
        float av[3], bv[3], o[3];
        for (int q = 0; q < 3; ++q) {
          av[q] = U0[q][cc];
          if (i < RC[q]) {
            int vq = row_v(mem, ROFF[q], i);
            bv[q] = xyz[3 * (int64_t)vq + cc] - CEN[q][cc];
          } else {
            bv[q] = -CEN[q][cc];  // padding entry: the zero point minus the centroid
          }
        }
        cross3(av, bv, o);
        dd += o[f] * n[cc];
      }
    }
    float cs = cosine(u0, u);
    float sc = cs * (dd >= 0.f ? 1.f : -1.f) + (dd < 0.f ? 2.f : 0.f);
    uint32_t sb = __float_as_uint(sc);
    sb = (sb & 0x80000000u) ? ~sb : (sb | 0x80000000u);  // ascending-orderable bits
    key[off + i] = ((uint64_t)(~sb) << 32) | (uint64_t)(uint32_t)i;  // descending score
  }
  cnt_all[f] = c;
  cnt_nz[f] = nz;
}

// F4b: sort each row's keys (descending score, then position) and write the
// ordered vertex ids
__global__ void k_row_sort(int64_t F, const int32_t* __restrict__ frow, const uint64_t* __restrict__ mem,
                           const int64_t* __restrict__ roff, const int32_t* __restrict__ rcnt,
                           uint64_t* __restrict__ key, int32_t* __restrict__ ordv) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  const int r = frow[f];
  const int c = rcnt[r];
  const int64_t off = roff[r];
  shell_sort(key + off, c);
  for (int j = 0; j < c; ++j) ordv[off + j] = row_v(mem, off, (int)(uint32_t)key[off + j]);
}

// F5: per block of rows, how many rows have c >= t+3, t-major layout
__global__ void __launch_bounds__(TNP_BLOCK)
k_fan_hist(int64_t F, const int32_t* __restrict__ cnt, int T, int64_t nb, int32_t* __restrict__ hist) {
  __shared__ int lds[TNP_WAVES];
  int64_t f = (int64_t)blockIdx.x * TNP_BLOCK + threadIdx.x;
  int c = f < F ? cnt[f] : 0;
  for (int t = 0; t < T; ++t) {
    int tot;
    (void)tnp::block_rank(c >= t + 3, lds, tot);
    if (threadIdx.x == 0) hist[(int64_t)t * nb + blockIdx.x] = tot;
  }
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
  for (int t = 0; t < T; ++t) {
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
        int v = nz_member(a, rc, ids[q], xyz);
        for (int d = 0; d < 3; ++d) fc[9 * at + 3 * q + d] = xyz[3 * (int64_t)v + d];
      }
    }
  }
}

}  // namespace

// ----------------------------------------------------------------------------
int launch_face_count(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                      uint64_t pmask, int64_t* ctr2, hipStream_t s) {
  if (V <= 0) return 0;
  hipLaunchKernelGGL(k_face_count, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero, pmask, ctr2);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_face_insert(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                       uint64_t pmask, uint64_t* table, uint64_t tmask, int32_t* cnt, hipStream_t s) {
  if (V <= 0) return 0;
  hipLaunchKernelGGL(k_face_insert, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero, pmask,
                     table, tmask, cnt);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_keep_counts(const int32_t* cnt, int64_t n, int32_t* kc, int32_t* kf, hipStream_t s) {
  hipLaunchKernelGGL(k_keep_counts, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, cnt, n, kc, kf);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_face_scatter(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                        uint64_t pmask, const uint64_t* table, uint64_t tmask, const int32_t* cnt,
                        const int64_t* memoff, int32_t* cur, uint64_t* mem, hipStream_t s) {
  if (V <= 0) return 0;
  hipLaunchKernelGGL(k_face_scatter, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, V, grid, pos, zero, pmask,
                     table, tmask, cnt, memoff, cur, mem);
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
                    const int32_t* rcnt, const float* xyz, float* mean, hipStream_t s) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(k_row_mean, dim3(tnp_grid(F)), dim3(TNP_BLOCK), 0, s, F, frow, mem, roff, rcnt, xyz, mean);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_row_order(int64_t F, const int32_t* frow, const uint64_t* mem, const int64_t* roff,
                     const int32_t* rcnt, const float* xyz, const float* nrm, int quirk3, uint64_t* key,
                     int32_t* ordv, int32_t* cnt_all, int32_t* cnt_nz, hipStream_t s) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(k_row_score, dim3(tnp_grid(F)), dim3(TNP_BLOCK), 0, s, F, frow, mem, roff, rcnt, xyz, nrm,
                     quirk3, key, cnt_all, cnt_nz);
  hipLaunchKernelGGL(k_row_sort, dim3(tnp_grid(F)), dim3(TNP_BLOCK), 0, s, F, frow, mem, roff, rcnt, key, ordv);
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
__global__ void k_max_i32(const int32_t* __restrict__ a, int64_t n, int64_t* __restrict__ out) {
  int m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, a[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
  if (tnp::lane() == 0) atomicMax((unsigned long long*)out, (unsigned long long)m);
}
}  // namespace

int launch_max_i32(const int32_t* a, int64_t n, int64_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  unsigned g = (unsigned)std::min<int64_t>(tnp_grid(n), 1024);
  hipLaunchKernelGGL(k_max_i32, dim3(g), dim3(TNP_BLOCK), 0, s, a, n, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
