// One hyperplane step of the subdivision (tropical/subpoly.py:90-279, flat
// branch) as gfx950 kernels.  Launch order per active step (engine.cpp):
//
//   split_count -> scan -> split_emit            order-preserving split
//   new_vertices -> forward(stage) -> fail_check   coords, MLP, override test
//   [host: S, global override flag]
//   finalize_new                                 override + packed keys
//   hit_count -> scan -> hit_emit                 old vertices on the plane
//   cell_count -> scan -> cell_scatter            members bucketed by grid cell
//   cell_tcnt -> scan -> connect -> radix sort    connecting edges c_new
//   prune_count -> scan -> prune_emit             future-key pruning
//   scan(used) -> gather_vertices, remap_edges    vertex compaction
//
// Layouts: xyz fp32 [V][3]; pre fp32 plane-major [K][ld]; packed keys per
// vertex: pos/zero u64 (bit p = plane p), grid u64 (common.h); edges int32
// [E][2].  Everything that fixes an output ORDER is a scan in input order
// (the reference's masked_scatter_ / sorted unique semantics); atomics only
// produce counts, bucket membership and append slots, and every appended
// set is sorted before it is used, so results are deterministic and
// bitwise reproducible.
#include "common.h"
#include "kernels.h"
#include "step.h"
#include "connect.h"

#include <algorithm>

namespace {

// per-edge high plane h = 1 + the highest plane on which the endpoint keys
// differ (0: equal keys); the pruning of step idx keeps an edge iff h > idx
constexpr uint8_t EDGE_STALE = 0xFF;  // rewired edge: recompute from the endpoint keys
__device__ __forceinline__ uint8_t high_plane(uint64_t dm) {
  return (uint8_t)(dm ? 64 - __clzll(dm) : 0);
}
// per-edge first split plane ef: the lowest plane >= the next step that
// splits the edge (endpoints non-zero with opposite signs, exactly the split
// test of subpoly.py:104-105); EDGE_NOSPLIT: none.  An edge splits at most
// once more as it stands: at plane ef it is replaced by its two halves,
// whose planes come from the new keys, so one byte per edge carries every
// future split test (instead of the 64-bit mask of all its split planes)
constexpr uint8_t EDGE_NOSPLIT = 0xFF;
// lazily deleted edge (high-plane byte; its first split plane is
// EDGE_NOSPLIT): the pruning of a step marks the edges it removes instead of
// compacting the list (k_prune_lazy); every edge pass skips them and the
// compacting passes drop them
constexpr uint8_t EDGE_DEAD = 0xFE;
__device__ __forceinline__ uint8_t first_plane(uint64_t m) {
  return (uint8_t)(m ? __builtin_ctzll(m) : EDGE_NOSPLIT);
}
// an edge's high plane byte d and first split plane byte m (planes of amask)
// from its endpoint keys (pz, KW words per key)
template <int KW>
__device__ __forceinline__ void edge_bytes(const uint64_t* __restrict__ pz, int a, int b, const Key<KW>& amask,
                                           uint32_t& d, uint32_t& m) {
  Key<KW> pa, za, pb, zb;
  tnp::pz_load(pz, a, pa, za);
  tnp::pz_load(pz, b, pb, zb);
  d = (uint32_t)tnp::key_high((pa ^ pb) | (za ^ zb));
  const int f = tnp::key_first((pa ^ pb) & ~za & ~zb & amask);
  m = f < 0 ? EDGE_NOSPLIT : (uint32_t)f;
}
// a plane set folded into an active-plane word (common.h act_bit)
template <int KW>
__device__ __forceinline__ uint64_t act_word(const Key<KW>& k) {
  if constexpr (KW == 1) return k.w[0];
  else return k.w[0] | (k.w[1] ? (1ull << 63) : 0ull);
}
constexpr int IPT = 8;                  // items per thread per tile
constexpr int TILE = TNP_BLOCK * IPT;   // tile of a compaction pass
// single-pass (look-back) compactions: items per thread of the split / hit
// pass (SIPT) and of the prune pass (LIPT); every item's loads are issued
// before any is used
// split / hit passes: 32 items per thread on large inputs (more loads in
// flight), 8 on small ones (more tiles to spread over the CUs)
#ifndef TNP_SIPT_BIG
#define TNP_SIPT_BIG 32
#endif
constexpr int SIPT_BIG = TNP_SIPT_BIG, SIPT_SMALL = 8;
constexpr int64_t SIPT_BIG_FROM = 1 << 20;
__host__ __device__ constexpr int split_ipt(int64_t n) { return n >= SIPT_BIG_FROM ? SIPT_BIG : SIPT_SMALL; }
constexpr int SIPT = 16;  // the radix path's run-start pass
constexpr int STILE = TNP_BLOCK * SIPT;
#ifndef TNP_LIPT
#define TNP_LIPT 16  // 16: half the look-back tickets of 8 (one returning atomic per tile on one word)
#endif
constexpr int LIPT = TNP_LIPT;
#ifndef TNP_SPLIT_SPIN  // look-back polls before recomputing (0: recompute at once; tests)
#define TNP_SPLIT_SPIN 64
#endif
#ifndef TNP_PRUNE_SPIN
#define TNP_PRUNE_SPIN 1024
#endif
constexpr int LTILE = TNP_BLOCK * LIPT;

constexpr int HIPT = 16;                    // slots per thread per chunk
constexpr int HCHUNK = TNP_BLOCK * HIPT;    // slots per chunk
constexpr int HBUF = 2 * HCHUNK;            // LDS hit buffer (a chunk always fits after a flush)
constexpr int HIT_GRID = HIT_WORKERS_MAX;

__device__ __forceinline__ void hit_body(int64_t bid, int64_t nblk, const float* __restrict__ col,
                                         const uint8_t* __restrict__ alive, int64_t V, float eps,
                                         int32_t* __restrict__ out, int64_t* __restrict__ ctr,
                                         int64_t* __restrict__ hpart);
// ---------------------------------------------------------------------------
// split test: subpoly.py:102-105
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool split_test(const float* __restrict__ col, const int32_t* e,
                                           float eps) {
  float d0 = col[e[0]], d1 = col[e[1]];
  return (__fmul_rn(d0, d1) < 0.f) && (fabsf(d0) > eps) && (fabsf(d1) > eps);
}

// single pass (replaces split_count -> scan -> split_emit): tile by ticket,
// decoupled look-back for the tile's first new-vertex id; the last tile
// writes S to ctr[CTR_S].  sa/sb/eidx need capacity E.  Loads are issued
// unconditionally (clamped index) in two batches -- the edge pairs, then the
// plane-column gathers -- so a thread has SIPT * 2 loads in flight instead
// of a bounds branch serialising every item.
template <int SI>
__global__ void __launch_bounds__(TNP_BLOCK)
k_split_lb(int32_t* __restrict__ edges, int64_t E, int64_t ntiles, const uint8_t* __restrict__ ef,
           uint8_t* __restrict__ dm, int idx, int64_t V, int32_t* __restrict__ sa,
           int32_t* __restrict__ sb, int64_t* __restrict__ ctr, int32_t* __restrict__ eidx, TnpLB lb,
           HitArgs ha) {
  if ((int64_t)blockIdx.x >= ntiles) {
    // the plane's hit vertices (k_hit_append's work) in the same dispatch:
    // workgroups past the split tiles (they wait on nothing)
    hit_body((int64_t)blockIdx.x - ntiles, (int64_t)gridDim.x - ntiles, ha.col, ha.alive, ha.V, ha.eps, ha.out,
             ctr, ha.hpart);
    return;
  }
  __shared__ int cnt[SI][TNP_WAVES];
  __shared__ int64_t slot;
  const int64_t tile = blockIdx.x;  // ticket-free look-back (lb_prefix_rc)
  const int64_t base = tile * (TNP_BLOCK * SI);
  uint64_t bal[SI];
  uint32_t fp[SI];
#pragma unroll
  for (int k = 0; k < SI; ++k) {  // coalesced, unconditional (clamped) loads
    const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    fp[k] = ef[i < E ? i : E - 1];
  }
  bool missed = false;
#pragma unroll
  for (int k = 0; k < SI; ++k) {
    const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    bal[k] = __ballot((i < E) && fp[k] == (uint32_t)idx);
    missed |= (i < E) && fp[k] < (uint32_t)idx;
    if (tnp::lane() == 0) cnt[k][tnp::wave()] = __popcll(bal[k]);
  }
  if (__ballot(missed) && tnp::lane() == 0) tnp::or_sticky(&ctr[CTR_MISSED], 1ull);
  __syncthreads();
  int64_t agg = 0;
#pragma unroll
  for (int k = 0; k < SI; ++k)
#pragma unroll
    for (int w = 0; w < TNP_WAVES; ++w) agg += cnt[k][w];
  // a predecessor tile not yet published: count its split edges (ef == idx)
  // four bytes per load; tiles start on multiples of TNP_BLOCK * SI
  const uint32_t rep = (uint32_t)idx * 0x01010101u;
  auto tile_agg = [&](int64_t t) -> int64_t {
    const int64_t b0 = t * (TNP_BLOCK * SI), b1 = b0 + TNP_BLOCK * SI < E ? b0 + TNP_BLOCK * SI : E;
    int c = 0;
    for (int64_t j = b0 + 4 * tnp::lane(); j < b1; j += 256) {
      if (j + 4 <= b1) {
        const uint32_t x = *reinterpret_cast<const uint32_t*>(ef + j) ^ rep;
        c += ((x & 0xFFu) == 0) + ((x & 0xFF00u) == 0) + ((x & 0xFF0000u) == 0) + ((x >> 24) == 0);
      } else {
        for (int64_t q = j; q < b1; ++q) c += ef[q] == (uint8_t)idx;
      }
    }
    return tnp::wave_sum((int64_t)c);
  };
  const int64_t prefix = tnp::lb_prefix_rc(lb, tile, agg, &slot, tile_agg, TNP_SPLIT_SPIN);
  int64_t run = prefix;
#pragma unroll
  for (int k = 0; k < SI; ++k) {
    int64_t off = run;
    int tot = 0;
#pragma unroll
    for (int w = 0; w < TNP_WAVES; ++w) {
      const int c = cnt[k][w];
      off += (w < tnp::wave()) ? c : 0;
      tot += c;
    }
    if ((bal[k] >> tnp::lane()) & 1) {
      const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
      const int64_t id = off + tnp::mbcnt(bal[k]);
      const int2 ab = reinterpret_cast<const int2*>(edges)[i];
      sa[id] = ab.x;
      sb[id] = ab.y;
      if (eidx) {
        eidx[id] = (int32_t)i;
      } else {
        edges[2 * i + 1] = (int32_t)(V + id);
        dm[i] = EDGE_STALE;  // rewired: the prune recomputes its masks
      }
    }
    run += tot;
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) ctr[CTR_S] = prefix + agg;
}

// ---------------------------------------------------------------------------
// new vertices: subpoly.py:113-117, 180
//   d = d/eps; w = |d0| / |d1 - d0|; v = e0*(1-w) + e1*w
// ---------------------------------------------------------------------------
__global__ void k_new_vertices(const int32_t* __restrict__ sa, const int32_t* __restrict__ sb,
                               int64_t S, const float* __restrict__ col, float eps,
                               float* __restrict__ xyz, int64_t V) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= S) return;
  int a = sa[r], b = sb[r];
  float d0 = __fdiv_rn(col[a], eps), d1 = __fdiv_rn(col[b], eps);
  float w = __fdiv_rn(fabsf(d0), fabsf(__fsub_rn(d1, d0)));
  float om = __fsub_rn(1.0f, w);
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float e0 = xyz[3 * (int64_t)a + d], e1 = xyz[3 * (int64_t)b + d];
    xyz[3 * (V + r) + d] = __fadd_rn(__fmul_rn(e0, om), __fmul_rn(e1, w));
  }
}

// shared planes (subpoly_debug.py:35-42): planes j < idx where both
// endpoints are eps-zero, plus the current plane idx.  Any new vertex off one
// of its shared planes by more than eps -> global override flag.  On a shard
// (own_any(own)) only the new vertices it owns vote (grid_new: their grid
// words), as k_forward_new on the flat path: a halo vertex near the halo's
// outer faces may belong to an edge the whole complex does not have.
template <int KW>
__global__ void k_fail_check(const int32_t* __restrict__ sa, const int32_t* __restrict__ sb,
                             int64_t S, int idx, const uint64_t* __restrict__ zero,
                             const float* __restrict__ stage, float eps,
                             uint64_t* __restrict__ shared, int64_t* __restrict__ ctr,
                             const uint64_t* __restrict__ grid_new, OwnBox own) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (r < S) {
    const Key<KW> m = (tnp::vkey_load<KW>(zero, sa[r]) & tnp::vkey_load<KW>(zero, sb[r]) & tnp::key_below<KW>(idx)) |
                      tnp::key_bit<KW>(idx);
    tnp::key_store(shared, r, m);
#pragma unroll
    for (int q = 0; q < KW; ++q)
      for (uint64_t t = m.w[q]; t; t &= t - 1) {
        const int p = 64 * q + __builtin_ctzll(t);
        bad |= fabsf(stage[(int64_t)p * S + r]) > eps;
      }
    if (tnp::own_any(own)) bad &= tnp::owned_by(own, grid_new[r]);
  }
  if (__ballot(bad) && tnp::lane() == 0) tnp::or_sticky(&ctr[CTR_FAIL], 1ull);
}

// override (masked_fill_ on the shared planes, subpoly_debug.py:48), packed
// keys of the final pre-activations, live planes copied into the cache.
// override_ < 0: the (single-device) predicate is still in ctr[CTR_FAIL]
template <int KW>
__global__ void k_finalize_new(int64_t S, int K, int override_, const uint64_t* __restrict__ shared,
                               float* __restrict__ stage, float eps, float* __restrict__ pre,
                               int64_t ld, int keep_from, int64_t V, uint64_t* __restrict__ pos,
                               uint64_t* __restrict__ zero, const int64_t* __restrict__ ctr,
                               uint64_t* __restrict__ pz) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= S) return;
  const bool ov = override_ < 0 ? ctr[CTR_FAIL] != 0 : override_ != 0;
  const Key<KW> m = ov ? tnp::key_load<KW>(shared, r) : tnp::key_zero<KW>();
  Key<KW> ps = tnp::key_zero<KW>(), zs = tnp::key_zero<KW>();
  for (int p = 0; p < K; ++p) {
    float v = stage[(int64_t)p * S + r];
    if (tnp::key_test(m, p)) v = 0.f;
    tnp::key_put(ps, p, v > eps);  // sign +1  (pos & zero == 0)
    tnp::key_put(zs, p, fabsf(v) <= eps);
    if (p >= keep_from) pre[(int64_t)p * ld + V + r] = v;
  }
  tnp::pz_store(pz, V + r, ps, zs);  // (pos / zero: views of pz)
}

// ---------------------------------------------------------------------------
// hit vertices: |outputs_[:, idx]| < eps (subpoly.py:233)
// ---------------------------------------------------------------------------
// live vertices on the plane, appended after the S new members in no
// particular order (every consumer is order-free: the bucket / cell grouping
// keeps arbitrary in-cell order and the emitted edges are sorted), count ->
// ctr[CTR_H] (zero on entry).  A fixed grid of workgroups walks the slots in
// chunks, collects its hits in LDS and appends them with one device atomic
// per flush: no tickets, no look-back (one returning atomic per workgroup on
// one word serialises chip-wide).  alive: the live-slot flags of the lazily
// compacted vertex set.

// one hit worker (block bid of nblk): hits appended to out[ctr[CTR_H]++]
__device__ __forceinline__ void hit_body(int64_t bid, int64_t nblk, const float* __restrict__ col,
                                         const uint8_t* __restrict__ alive, int64_t V, float eps,
                                         int32_t* __restrict__ out, int64_t* __restrict__ ctr,
                                         int64_t* __restrict__ hpart) {
  __shared__ int32_t hb[HBUF];
  __shared__ int hn;
  __shared__ int64_t hbase;
  __shared__ int64_t lcnt[TNP_WAVES];
  int64_t nlive = 0;  // (hpart) live slots this thread read
  if (threadIdx.x == 0) hn = 0;
  __syncthreads();
  auto flush = [&]() {
    const int n = hn;
    if (n == 0) return;
    if (threadIdx.x == 0) hbase = (int64_t)atomicAdd((unsigned long long*)&ctr[CTR_H], (unsigned long long)n);
    __syncthreads();
    for (int q = threadIdx.x; q < n; q += TNP_BLOCK) out[hbase + q] = hb[q];
    __syncthreads();
    if (threadIdx.x == 0) hn = 0;
    __syncthreads();
  };
  for (int64_t base = bid * HCHUNK; base < V; base += nblk * HCHUNK) {
    float c[HIPT];
    uint8_t al[HIPT];
#pragma unroll
    for (int k = 0; k < HIPT; ++k) {  // unconditional (clamped) loads, all in flight
      const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
      const int64_t ic = i < V ? i : V - 1;
      c[k] = col[ic];
      al[k] = alive[ic];
    }
#pragma unroll
    for (int k = 0; k < HIPT; ++k) {
      const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
      nlive += (i < V) && al[k];
      const bool h = (i < V) && (fabsf(c[k]) < eps) && al[k];
      const uint64_t b = __ballot(h);
      if (b) {
        int w0 = 0;
        if (tnp::lane() == 0) w0 = atomicAdd(&hn, __popcll(b));  // LDS
        w0 = __shfl(w0, 0, 64);
        if (h) hb[w0 + tnp::mbcnt(b)] = (int32_t)i;
      }
    }
    __syncthreads();
    if (hn > HBUF - HCHUNK) flush();
  }
  __syncthreads();
  flush();
  if (hpart) {
    nlive = tnp::wave_sum(nlive);
    if (tnp::lane() == 0) lcnt[tnp::wave()] = nlive;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t t = 0;
      for (int w = 0; w < TNP_WAVES; ++w) t += lcnt[w];
      hpart[bid] = t;
    }
  }
}

__global__ void __launch_bounds__(TNP_BLOCK)
k_hit_append(const float* __restrict__ col, const uint8_t* __restrict__ alive, int64_t V, float eps,
             int32_t* __restrict__ members, int64_t S_arg, int64_t* __restrict__ ctr) {
  // S_arg < 0: launched right behind the split, whose count is on the device
  const int64_t S = S_arg < 0 ? ctr[CTR_S] : S_arg;
  hit_body(blockIdx.x, gridDim.x, col, alive, V, eps, members + S, ctr, nullptr);
}

// new vertices outside this shard's owned box (the flat path counts
// them in k_forward_new) -> ctr[CTR_DUP]: a kept curve-branch split on a
// halo cell or on the shared boundary plane is another shard's
__global__ void k_count_unowned(const uint64_t* __restrict__ grid, int64_t n, OwnBox own,
                                int64_t* __restrict__ ctr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool halo = i < n && !tnp::owned_by(own, grid[i]);
  const uint64_t hb = __ballot(halo);
  if (hb && tnp::lane() == 0) atomicAdd((unsigned long long*)&ctr[CTR_DUP], (unsigned long long)__popcll(hb));
}

__global__ void k_new_members(int32_t* __restrict__ members, int64_t S, int64_t V) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < S) members[r] = (int32_t)(V + r);
}

// ---------------------------------------------------------------------------
// grid cells spanned by a member: per dim {off-1, off} on a mark else {off}
// (the grid part of regions_to_vertices' augmentation, subpoly.py:327-332)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cell_span(uint64_t g, int lo[3], int n[3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    int o = tnp::grid_off(g, d);
    bool z = tnp::grid_zero(g, d);
    lo[d] = z ? o - 1 : o;
    n[d] = z ? 2 : 1;
  }
}

__device__ __forceinline__ int64_t cell_id(int cx, int cy, int cz, int NC) {
  return ((int64_t)(cx + 2) * NC + (cy + 2)) * NC + (cz + 2);
}

// ---- sort-based cell bucketing ---------------------------------------------
// entries (cell, member) are generated per member in span order, radix-sorted
// by cell; segment bounds give each cell's member list.  No per-entry
// atomics (the atomic counting sort they replace serialised on the spatially
// coherent members of a wave).
__device__ __forceinline__ int span_cells(uint64_t g, int lo[3], int n[3]) {
  cell_span(g, lo, n);
  return n[0] * n[1] * n[2];
}

// entries per member; per-block sums of the reference's augmented rows (A)
template <int KW>
__global__ void __launch_bounds__(TNP_BLOCK)
k_span_count(const int32_t* __restrict__ members, int64_t S, int64_t Mcap,
             const uint64_t* __restrict__ grid, const uint64_t* __restrict__ zero, int idx,
             int32_t* __restrict__ cnt, int64_t* __restrict__ part, int64_t* __restrict__ ctr) {
  __shared__ int64_t lds[TNP_WAVES];
  const int64_t M = S + ctr[CTR_H];  // members = splits ++ hits (device count)
  int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t aug = 0;
  bool k0 = false;
  if (m < Mcap) cnt[m] = 0;
  if (m < M) {
    int v = members[m];
    int lo[3], n[3];
    cnt[m] = span_cells(grid[v], lo, n);
    const int kz = tnp::key_pop(tnp::vkey_load<KW>(zero, v) & tnp::key_below<KW>(idx)) + (n[0] - 1) + (n[1] - 1) +
                   (n[2] - 1);
    aug = 1ll << kz;
    k0 = kz == 0;
  }
  if (__ballot(k0) && tnp::lane() == 0) atomicOr((unsigned long long*)&ctr[CTR_K0], 1ull);
  int64_t tot;
  tnp::block_scan_excl(aug, lds, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(TNP_BLOCK)
k_sum_parts(const int64_t* __restrict__ part, int64_t n, int64_t* __restrict__ ctr, int slot) {
  int64_t a = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) a += part[i];
  a = tnp::wave_sum(a);
  if (tnp::lane() == 0 && a) atomicAdd((unsigned long long*)&ctr[slot], (unsigned long long)a);
}

__global__ void k_span_emit(const int32_t* __restrict__ members, int64_t S,
                            const uint64_t* __restrict__ grid, int NC,
                            const int64_t* __restrict__ eoff, uint32_t* __restrict__ ekey,
                            int32_t* __restrict__ eval, const int64_t* __restrict__ ctr) {
  const int64_t M = S + ctr[CTR_H];
  int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  int v = members[m];
  int lo[3], n[3];
  cell_span(grid[v], lo, n);
  int64_t p = eoff[m];
  for (int i = 0; i < n[0]; ++i)
    for (int j = 0; j < n[1]; ++j)
      for (int k = 0; k < n[2]; ++k) {
        ekey[p] = (uint32_t)cell_id(lo[0] + i, lo[1] + j, lo[2] + k, NC);
        eval[p] = v;
        ++p;
      }
}

// Pair cells straight from the cell-sorted entries (no dense cell grid):
// a run of equal keys is one cell's member list.
// (1) run starts, compacted in entry order (single pass, lane-interleaved
//     items, decoupled look-back); the last tile closes the list with T.
__global__ void __launch_bounds__(TNP_BLOCK)
k_run_starts_lb(const uint32_t* __restrict__ key, int64_t T, int64_t ntiles,
                int32_t* __restrict__ rstart, int64_t* __restrict__ ctr, TnpLB lb) {
  __shared__ int cnt[SIPT][TNP_WAVES];
  __shared__ int64_t slot;
  const int64_t tile = tnp::lb_tile(lb, &slot);
  const int64_t base = tile * STILE;
  uint32_t kc[SIPT], kp[SIPT];
#pragma unroll
  for (int k = 0; k < SIPT; ++k) {  // unconditional (clamped) loads, all in flight
    const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    const int64_t ic = i < T ? i : T - 1;
    kc[k] = key[ic];
    kp[k] = key[ic > 0 ? ic - 1 : 0];
  }
  uint64_t bal[SIPT];
#pragma unroll
  for (int k = 0; k < SIPT; ++k) {
    const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    bal[k] = __ballot(i < T && (i == 0 || kp[k] != kc[k]));
    if (tnp::lane() == 0) cnt[k][tnp::wave()] = __popcll(bal[k]);
  }
  __syncthreads();
  int64_t agg = 0;
#pragma unroll
  for (int k = 0; k < SIPT; ++k)
#pragma unroll
    for (int w = 0; w < TNP_WAVES; ++w) agg += cnt[k][w];
  const int64_t prefix = tnp::lb_prefix(lb, tile, agg, &slot);
  int64_t run = prefix;
#pragma unroll
  for (int k = 0; k < SIPT; ++k) {
    int64_t off = run;
    int tot = 0;
#pragma unroll
    for (int w = 0; w < TNP_WAVES; ++w) {
      const int cc = cnt[k][w];
      off += (w < tnp::wave()) ? cc : 0;
      tot += cc;
    }
    if ((bal[k] >> tnp::lane()) & 1)
      rstart[off + tnp::mbcnt(bal[k])] = (int32_t)(base + (int64_t)k * TNP_BLOCK + threadIdx.x);
    run += tot;
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) {
    rstart[prefix + agg] = (int32_t)T;
    ctr[CTR_RUNS] = prefix + agg;
  }
}

// (2) runs with >= 2 members, compacted in cell order with their flattened
// pair offsets: thread-contiguous groups of PIPT runs, two decoupled
// look-back chains (rank, pair offset).  Launched over an upper bound of
// tiles; the blocks past the device-side run count leave at once.  A cell above 65535 members flags CTR_BIG
// (one linear region that large is the degenerate case the host refuses).
constexpr int PIPT = 16;
constexpr int PTILE = TNP_BLOCK * PIPT;

__global__ void __launch_bounds__(TNP_BLOCK)
k_pair_runs_lb(const uint32_t* __restrict__ key, const int32_t* __restrict__ rstart,
               int32_t* __restrict__ pcell, int32_t* __restrict__ pent, int32_t* __restrict__ pn,
               int64_t* __restrict__ ptoff, int64_t* __restrict__ ctr, TnpLB lbr, TnpLB lbp) {
  __shared__ int64_t lds[TNP_WAVES];
  __shared__ int64_t slot;
  const int64_t R = ctr[CTR_RUNS];
  const int64_t ntiles = (R + PTILE - 1) / PTILE;
  // exactly ntiles blocks take a ticket (the ticket is one same-address
  // atomic per block: the surplus blocks must not queue on it).  The host
  // advanced its ticket base by gridDim.x, so the surplus is added in one
  // step: by the last tile (every ticket is taken by then), or by block 0
  // when there is no tile at all.
  if ((int64_t)blockIdx.x >= ntiles) {
    if (ntiles == 0 && blockIdx.x == 0 && threadIdx.x == 0)
      atomicAdd(lbr.ticket, (unsigned long long)gridDim.x);
    return;
  }
  const int64_t tile = tnp::lb_tile(lbr, &slot);
  if (tile == ntiles - 1 && threadIdx.x == 0 && (int64_t)gridDim.x > ntiles)
    atomicAdd(lbr.ticket, (unsigned long long)(gridDim.x - ntiles));
  const int64_t base = tile * PTILE + (int64_t)threadIdx.x * PIPT;
  int32_t st[PIPT + 1];
#pragma unroll
  for (int g = 0; g <= PIPT; ++g) st[g] = rstart[base + g <= R ? base + g : R];
  int32_t n[PIPT];
  int64_t nr = 0, np = 0;
  bool big = false;
#pragma unroll
  for (int g = 0; g < PIPT; ++g) {
    const int32_t m = base + g < R ? st[g + 1] - st[g] : 0;
    big |= m > 65535;
    n[g] = m > 65535 ? 0 : m;
    nr += n[g] >= 2;
    np += (int64_t)n[g] * (n[g] - 1) / 2;
  }
  if (__ballot(big) && tnp::lane() == 0) atomicOr((unsigned long long*)&ctr[CTR_BIG], 1ull);
  int64_t tr, tp;
  int64_t er = tnp::block_scan_excl(nr, lds, tr);
  int64_t ep = tnp::block_scan_excl(np, lds, tp);
  er += tnp::lb_prefix(lbr, tile, tr, &slot);
  const int64_t pp = tnp::lb_prefix(lbp, tile, tp, &slot);
  ep += pp;
#pragma unroll
  for (int g = 0; g < PIPT; ++g) {
    if (n[g] >= 2) {
      pcell[er] = (int32_t)key[st[g]];
      pent[er] = st[g];
      pn[er] = n[g];
      ptoff[er] = ep;
      ++er;
      ep += (int64_t)n[g] * (n[g] - 1) / 2;
    }
  }
  if (tile == ntiles - 1 && threadIdx.x == TNP_BLOCK - 1) {
    ctr[CTR_R] = er;
    ctr[CTR_TESTS] = ep;
  }
}

// entry-aligned records of the cell-sorted (cell, member) entries (radix
// path): the member's keys and its cell flags in that cell
template <int KW>
__global__ void k_entry_keys(const int32_t* __restrict__ ent_v, const uint32_t* __restrict__ ekey, int NC,
                             int64_t T, const uint64_t* __restrict__ grid,
                             const uint64_t* __restrict__ pz, CellEntT<KW>* __restrict__ ent) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T) return;
  const int v = ent_v[i];
  const uint32_t c = ekey[i];
  CellEntT<KW> r;
  {
    Key<KW> p, z;
    tnp::pz_load(pz, v, p, z);  // pos and zero in one 16-byte gather (per word pair)
    ent_set_keys(r, p, z);
  }
  r.v = v;
  r.f = cell_flags(grid[v], (int)(c / ((uint32_t)NC * NC)), (int)((c / NC) % NC), (int)(c % NC));
  r.tag = 0x80000000u;  // radix path: every cell goes through k_connect
  r.pad = 0;
  ent[i] = r;
}

// first index in [lo, hi) with a[i] > x (hi if none)
__device__ __forceinline__ int64_t upper_bound_i64(const int64_t* __restrict__ a, int64_t lo,
                                                   int64_t hi, int64_t x) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

#ifndef TNP_CONNECT_CIPT
#define TNP_CONNECT_CIPT 8
#endif
constexpr int CIPT = TNP_CONNECT_CIPT;  // consecutive pair indices per thread
constexpr int CONNECT_CELLS = TNP_BLOCK * CIPT + 2;  // >= pair cells a chunk can touch
constexpr int CCH = TNP_BLOCK * CIPT;   // pair indices per block
#ifndef TNP_CONNECT_CB
#define TNP_CONNECT_CB 1
#endif
constexpr int CONNECT_CB = TNP_CONNECT_CB;  // pairs whose record loads are in flight together
static_assert(CONNECT_CB == 0 || CIPT % CONNECT_CB == 0, "connect batches");

__device__ __forceinline__ void cell_coords(int64_t cell, int NC, int cc[3]) {
  cc[2] = (int)(cell % NC) - 2;
  cc[1] = (int)((cell / NC) % NC) - 2;
  cc[0] = (int)(cell / ((int64_t)NC * NC)) - 2;
}

// The flattened pair-index space of all cells (cell-major, then (i, j<i)
// within the cell's member list) split evenly over threads: every thread
// tests CIPT consecutive pairs, so a cell of 10^4 members costs the same per
// thread as 10^4 cells of 2.  Member keys come from the entry-aligned copies
// written by cell_scatter (contiguous per cell: L1/L2 hits).  Emitted pairs
// are packed (lo << nb | hi) and appended block-contiguously through ONE
// atomic per block; their order is restored by the radix sort that follows,
// so the appended order never reaches the output.
// chunk b of the pair space starts in cell bcell[b] (written per cell: no
// host round trip for the pair count)
__global__ void k_chunk_cells(const int64_t* __restrict__ ptoff, const int32_t* __restrict__ pn,
                              int64_t rcap,
                              int32_t* __restrict__ bcell, int64_t cap, int64_t* __restrict__ ctr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rcap || r >= ctr[CTR_R]) return;
  const int64_t m = pn[r];
  const int64_t n = m * (m - 1) / 2;
  const int64_t lo = ptoff[r];
  int64_t b0 = (lo + CCH - 1) / CCH, b1 = (lo + n + CCH - 1) / CCH;
  if (b1 > cap) atomicOr((unsigned long long*)&ctr[CTR_BOVF], 1ull);
  for (int64_t b = b0; b < b1 && b < cap; ++b) bcell[b] = (int32_t)r;
}

// Persistent over the chunks of the pair space (count read on the device);
// stops at once if the complex is degenerate (pairs above the limit) or the
// chunk table overflowed -- the host reports either after the fact.
// row i and column j (j < i) of in-cell pair q (q = i (i - 1) / 2 + j);
// q < 2^31 (a cell holds <= 65535 members), so 32-bit unsigned arithmetic
__device__ __forceinline__ void pair_row(int q, int& i, int& j) {
  const uint32_t uq = (uint32_t)q;
  uint32_t r = (uint32_t)((1.0f + sqrtf(1.0f + 8.0f * (float)q)) * 0.5f);
  while (r * (r - 1) / 2 > uq) --r;
  while ((r + 1) * r / 2 <= uq) ++r;
  i = (int)r;
  j = (int)(uq - r * (r - 1) / 2);
}

// Lane-interleaved enumeration: the 64 lanes of a wave take 64 CONSECUTIVE
// pairs per step, so within a cell row they share the row entry (broadcast)
// and read consecutive column entries (coalesced 32-byte records); a wave
// walks CIPT such steps.  The chunk's pair cells (offset, id, member count,
// first entry) sit in LDS, so locating a pair is an LDS walk.
template <int KW>
__global__ void __launch_bounds__(TNP_BLOCK)
k_connect(const int64_t* __restrict__ ptoff, const int32_t* __restrict__ pcell,
          const int32_t* __restrict__ pn, const int32_t* __restrict__ pent, int NC,
          int64_t max_tests, const int32_t* __restrict__ bcell, const CellEntT<KW>* __restrict__ ent,
          int idx, int nb, Key<KW> fmask, uint64_t* __restrict__ keys, int64_t cap,
          int64_t* __restrict__ xs, int64_t* __restrict__ ctr, const int64_t* __restrict__ bstat,
          int nbstat) {
  __shared__ int64_t lds[TNP_WAVES];
  __shared__ int64_t s_base;
  if (bstat && blockIdx.x == 0) {
    // the grouping kernel's per-bucket statistics (small grids) -> ctr
    int64_t v[4] = {0, 0, 0, 0};
    for (int i = threadIdx.x; i < nbstat; i += TNP_BLOCK)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += bstat[4 * (int64_t)i + q];
    constexpr int slot[4] = {CTR_COMPAT, CTR_P, CTR_X, CTR_SPAIRS};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int64_t tot;
      tnp::block_scan_excl(v[q], lds, tot);
      if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long*)&ctr[slot[q]], (unsigned long long)tot);
    }
  }
  __shared__ int32_t s_off[CONNECT_CELLS];  // first pair of the cell - chunk start
  __shared__ int32_t s_n[CONNECT_CELLS];
  __shared__ int32_t s_ent[CONNECT_CELLS];  // first entry of the cell
  // the bucket path's atomically allocated list (cells | pairs << 24), else
  // the radix path's scans
  const int64_t pk = ctr[CTR_PCK];
  const int64_t TT = pk ? (pk >> 24) : ctr[CTR_TESTS];
  const int64_t R = pk ? (pk & (PCK_CELLS - 1)) : ctr[CTR_R];
  if (TT > max_tests || ctr[CTR_BOVF] || ctr[CTR_BIG]) return;
  const int64_t nblk = (TT + CCH - 1) / CCH;
  const Key<KW> below = tnp::key_below<KW>(idx);
  const bool filt = tnp::key_any(fmask);
  int64_t n_compat = 0, n_reg = 0, n_conn = 0;
  for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
  const int64_t pb = b * (int64_t)CCH;
  const int64_t r0 = bcell[b];
  const int64_t r_end = (b + 1 < nblk) ? (int64_t)bcell[b + 1] + 1 : R;
  const int nr = (int)(r_end - r0);  // <= CCH + 1: every pair cell holds >= 1 pair
  __syncthreads();  // the previous chunk is done with the cell window
  for (int t = threadIdx.x; t < nr; t += blockDim.x) {
    s_off[t] = (int32_t)(ptoff[r0 + t] - pb);  // > -2^31: a cell holds < 2^31 pairs
    s_n[t] = pn[r0 + t];
    s_ent[t] = pent[r0 + t];
  }
  __syncthreads();
  const int64_t pw = pb + (int64_t)tnp::wave() * 64 * CIPT + tnp::lane();
  uint64_t kk[CIPT];
  int ne = 0;
  int lc = 0;
  {  // the lane's first cell: binary search, then a forward walk per step
    const int64_t x = pw - pb;
    int lo = 0, hi = nr;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_off[mid] <= x) lo = mid + 1;
      else hi = mid;
    }
    lc = lo > 0 ? lo - 1 : 0;
  }
#if TNP_CONNECT_CB == 0
#pragma unroll
  for (int k = 0; k < CIPT; ++k) {
    const int64_t p = pw + 64 * k;
    if (p < TT) {
      const int x = (int)(p - pb);
      while (lc + 1 < nr && s_off[lc + 1] <= x) ++lc;
      int i, j;
      pair_row(x - s_off[lc], i, j);
      const int64_t base = s_ent[lc];
      const CellEntT<KW> eu = ent[base + i];
      const CellEntT<KW> ev = ent[base + j];
      const Key<KW> pu = ent_p(eu), zu = ent_z(eu), pv = ent_p(ev), zv = ent_z(ev);
      PairTest t = pair_test(below, eu.f, pu, zu, ev.f, pv, zv);
      if (t.compat) {
        n_compat++;
        n_reg += t.regions;
        n_conn += t.emit;
        // the step's pruning drops it anyway (keep_edge): never appended
        if (t.emit && (!filt || tnp::key_any(((pu ^ pv) | (zu ^ zv)) & fmask))) {
          const uint32_t vu = (uint32_t)eu.v, vv = (uint32_t)ev.v;
          const uint32_t lo = vu < vv ? vu : vv, hi = vu < vv ? vv : vu;
          kk[ne++] = ((uint64_t)lo << nb) | hi;
        }
      }
    }
  }
#else
  // CB pairs at a time: locate them (LDS only), issue all 4·CB record loads
  // (unconditional: an out-of-range pair reads entry 0 of its cell), then
  // test -- CB loads in flight per lane instead of one dependent pair
#pragma unroll
  for (int k0 = 0; k0 < CIPT; k0 += CONNECT_CB) {
    int iu[CONNECT_CB], iv[CONNECT_CB];
    bool ok[CONNECT_CB];
#pragma unroll
    for (int kb = 0; kb < CONNECT_CB; ++kb) {
      const int64_t p = pw + 64 * (k0 + kb);
      ok[kb] = p < TT;
      int i = 0, j = 0;
      if (ok[kb]) {
        const int x = (int)(p - pb);
        while (lc + 1 < nr && s_off[lc + 1] <= x) ++lc;
        pair_row(x - s_off[lc], i, j);
      }
      const int base = s_ent[lc];
      iu[kb] = base + i;
      iv[kb] = base + j;
    }
    // a record is RW 8-byte words: the KW pos words, the KW zero words, then (v, f)
    constexpr int RW = sizeof(CellEntT<KW>) / 8;
    Key<KW> pua[CONNECT_CB], zua[CONNECT_CB], pva[CONNECT_CB], zva[CONNECT_CB];
    uint2 fua[CONNECT_CB], fva[CONNECT_CB];
    const ulonglong2* er = reinterpret_cast<const ulonglong2*>(ent);
    const uint2* ef = reinterpret_cast<const uint2*>(ent);
#pragma unroll
    for (int kb = 0; kb < CONNECT_CB; ++kb) {
      if constexpr (KW == 1) {
        const ulonglong2 ua = er[2 * (int64_t)iu[kb]], va = er[2 * (int64_t)iv[kb]];  // (p, z)
        pua[kb].w[0] = ua.x;
        zua[kb].w[0] = ua.y;
        pva[kb].w[0] = va.x;
        zva[kb].w[0] = va.y;
      } else {
        const ulonglong2 up = er[(RW / 2) * (int64_t)iu[kb]], uz = er[(RW / 2) * (int64_t)iu[kb] + 1];
        const ulonglong2 vp = er[(RW / 2) * (int64_t)iv[kb]], vz = er[(RW / 2) * (int64_t)iv[kb] + 1];
        pua[kb].w[0] = up.x;
        pua[kb].w[1] = up.y;
        zua[kb].w[0] = uz.x;
        zua[kb].w[1] = uz.y;
        pva[kb].w[0] = vp.x;
        pva[kb].w[1] = vp.y;
        zva[kb].w[0] = vz.x;
        zva[kb].w[1] = vz.y;
      }
      fua[kb] = ef[RW * (int64_t)iu[kb] + 2 * KW];  // (v, f)
      fva[kb] = ef[RW * (int64_t)iv[kb] + 2 * KW];
    }
#pragma unroll
    for (int kb = 0; kb < CONNECT_CB; ++kb) {
      if (!ok[kb]) continue;
      const Key<KW> pu = pua[kb], zu = zua[kb];
      const Key<KW> pv = pva[kb], zv = zva[kb];
      PairTest t = pair_test(below, fua[kb].y, pu, zu, fva[kb].y, pv, zv);
      if (t.compat) {
        n_compat++;
        n_reg += t.regions;
        n_conn += t.emit;
        // the step's pruning drops it anyway (keep_edge): never appended
        if (t.emit && (!filt || tnp::key_any(((pu ^ pv) | (zu ^ zv)) & fmask))) {
          const uint32_t vu = fua[kb].x, vv = fva[kb].x;
          const uint32_t lo = vu < vv ? vu : vv, hi = vu < vv ? vv : vu;
          kk[ne++] = ((uint64_t)lo << nb) | hi;
        }
      }
    }
  }
#endif
  int64_t tot;
  int64_t off = tnp::block_scan_excl((int64_t)ne, lds, tot);
  const int sh = xs ? blockIdx.x % XS_N : 0;
  const int64_t rc = xs ? cap / XS_N : cap;
  if (threadIdx.x == 0)
    s_base = tot ? (int64_t)atomicAdd((unsigned long long*)sink_word(xs, ctr, XS_KEYS), (unsigned long long)tot) : 0;
  __syncthreads();
  const int64_t w0 = s_base + off;
  for (int k = 0; k < ne; ++k)
    if (w0 + k < rc) keys[sh * rc + w0 + k] = kk[k];
  }
  add_pair_stats(n_compat, n_reg, n_conn, lds, xs, ctr);
}

// the window pass over every cell-contiguous entry (connect.h window_pass);
// the bucket path runs it inside its grouping kernel instead
__global__ void __launch_bounds__(TNP_BLOCK)
k_connect_win(const CellEnt* __restrict__ ent, int idx, int nb, uint64_t fmask,
              uint64_t* __restrict__ keys, int64_t cap, int64_t* __restrict__ xs, int64_t* __restrict__ ctr) {
  __shared__ WinLds W;
  __shared__ int64_t lds[TNP_WAVES];
  const int64_t T = ctr[CTR_T];
  WinAcc a;
  const uint64_t below = (idx >= 64) ? ~0ull : ((1ull << idx) - 1ull);
  window_pass(ent, 0, T, (int64_t)blockIdx.x * TNP_WAVES + tnp::wave(), (int64_t)gridDim.x * TNP_WAVES,
              below, nb, fmask, keys, cap, xs, ctr, W, a);
  window_flush(keys, cap, xs, ctr, W, a);
  add_pair_stats(a.n_compat, a.n_reg, a.n_conn, lds, xs, ctr);
}

// the shards -> ctr and the regions' output offsets; shards zeroed for the
// next step (one wave)
__global__ void k_keys_finish(int64_t* __restrict__ xs, int64_t cap, int64_t* __restrict__ ctr) {
  const int L = threadIdx.x;
  const int64_t rc = cap / XS_N;
  const int64_t c = L < XS_N ? xs[xs_word(XS_KEYS, L)] : 0;
  const int64_t incl = tnp::wave_scan_incl(c);
  if (L <= XS_N) xs[XS_OFF + L] = incl - c;  // lane XS_N: the total
  int64_t mx = c;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
  const int64_t total = __shfl(incl, 63, 64);
  int64_t st[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) st[q] = tnp::wave_sum(L < XS_N ? xs[xs_word(XS_COMPAT + q, L)] : (int64_t)0);
  if (L == 0) {
    ctr[CTR_XK] = mx > rc ? mx * XS_N : total;  // overflow: the capacity every region needs
    ctr[CTR_COMPAT] = st[0];
    ctr[CTR_P] = st[1];
    ctr[CTR_X] = st[2];
    if (st[3]) ctr[CTR_SPAIRS] = st[3];  // (the bucket path's window-pass pairs)
  }
  for (int q = L; q < XS_N * XS_STATS; q += 64) xs[xs_word(q / XS_N, q % XS_N)] = 0;
}

// out[i] = the i-th key of the regions in shard order
__global__ void k_keys_compact(const uint64_t* __restrict__ keys, int64_t cap, const int64_t* __restrict__ xs,
                               int64_t X, uint64_t* __restrict__ out) {
  const int64_t rc = cap / XS_N;
  int64_t off[XS_N];
#pragma unroll
  for (int r = 0; r < XS_N; ++r) off[r] = xs[XS_OFF + r];
  for (int64_t i = (int64_t)blockIdx.x * TNP_BLOCK + threadIdx.x; i < X; i += (int64_t)gridDim.x * TNP_BLOCK) {
    int r = 0;
#pragma unroll
    for (int q = 1; q < XS_N; ++q) r += off[q] <= i;
    out[i] = keys[r * rc + (i - off[r])];
  }
}

// ---------------------------------------------------------------------------
// pruning: keep an edge iff its endpoints' future sign keys (planes >= idx)
// differ (subpoly.py:252-265).  The candidate list is the concatenation
// [edges (split ones already rewired); e_new; c_new].
// ---------------------------------------------------------------------------
struct EdgeSrc {
  const int32_t* edges;  int64_t E;
  const int32_t* sb;     int64_t S;  int64_t V;
  const uint64_t* ckeys;  int nb;      int64_t X;   // packed (lo << nb | hi)
};

__device__ __forceinline__ void fetch_edge(const EdgeSrc& s, int64_t i, int& a, int& b) {
  if (i < s.E) {
    a = s.edges[2 * i];
    b = s.edges[2 * i + 1];
  } else if (i < s.E + s.S) {
    int64_t r = i - s.E;
    a = s.sb[r];
    b = (int)(s.V + r);
  } else {
    uint64_t k = s.ckeys[i - s.E - s.S];
    a = (int)(k >> s.nb);
    b = (int)(k & ((1ull << s.nb) - 1ull));
  }
}

template <int KW>
__device__ __forceinline__ bool keep_edge(int a, int b, const Key<KW>& fmask, const uint64_t* pos,
                                          const uint64_t* zero) {
  return tnp::key_any(((tnp::vkey_load<KW>(pos, a) ^ tnp::vkey_load<KW>(pos, b)) |
                       (tnp::vkey_load<KW>(zero, a) ^ tnp::vkey_load<KW>(zero, b))) & fmask);
}


// emits kept edges in order, flags used vertices and ORs the next-active
// plane mask: planes > idx on which a kept edge has non-zero opposite signs
// (exactly the split test of that future step, subpoly.py:104-105).
template <int KW>
__global__ void __launch_bounds__(TNP_BLOCK)
k_prune_emit(EdgeSrc src, int64_t N, Key<KW> fmask, Key<KW> amask,
             const uint64_t* __restrict__ pos, const uint64_t* __restrict__ zero,
             const int64_t* __restrict__ blkoff, int prune, int32_t* __restrict__ out,
             int32_t* __restrict__ used, int64_t* __restrict__ ctr) {
  __shared__ int lds[TNP_WAVES];
  int64_t base = (int64_t)blockIdx.x * TILE;
  int64_t run = prune ? blkoff[blockIdx.x] : base;
  uint64_t act = 0;
  for (int k = 0; k < IPT; ++k) {
    int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    int a = 0, b = 0;
    bool f = false;
    if (i < N) {
      fetch_edge(src, i, a, b);
      f = !prune || keep_edge<KW>(a, b, fmask, pos, zero);
    }
    if (prune) {
      int tot;
      int r = tnp::block_rank(f, lds, tot);
      if (f) {
        out[2 * (run + r)] = a;
        out[2 * (run + r) + 1] = b;
      }
      run += tot;
    } else if (f) {
      out[2 * i] = a;
      out[2 * i + 1] = b;
    }
    if (f) {
      if (used) {
        used[a] = 1;
        used[b] = 1;
      }
      const Key<KW> za = tnp::vkey_load<KW>(zero, a), zb = tnp::vkey_load<KW>(zero, b);
      act |= act_word((tnp::vkey_load<KW>(pos, a) ^ tnp::vkey_load<KW>(pos, b)) & ~za & ~zb & amask);
    }
  }
  act = tnp::wave_or(act);
  if (tnp::lane() == 0) tnp::or_sticky(&ctr[CTR_ACTIVE], act);
}

// single-pass pruning (replaces prune_count -> scan -> prune_emit): tile by
// ticket, keep flags per item kept in registers, decoupled look-back for the
// tile's output offset, then the ordered emit (k-major, then thread, as
// prune_emit), used flags and the next-active plane mask.  The last tile
// writes the kept count to ctr[CTR_E].
// Per-edge key bytes travel with the edges: dm = the high plane of the
// endpoint keys' difference ((pos ^ pos') | (zero ^ zero')) and ef = the
// first plane above idx that splits the edge ((pos ^ pos') & ~zero & ~zero':
// both non-zero, opposite signs -- exactly the split test of
// subpoly.py:104-105).  Vertex keys never change after
// creation, so an edge's masks change only when the edge does: the prune
// reads them coalesced for the old edges and gathers the endpoint keys only
// for rewired (dm == EDGE_STALE), e_new and c_new edges.
template <int KW>
__global__ void __launch_bounds__(TNP_BLOCK, 4)
k_prune_lb(EdgeSrc src, int64_t N, int64_t ntiles, int idx, Key<KW> amask,
           const uint64_t* __restrict__ pz, const uint8_t* __restrict__ dm,
           const uint8_t* __restrict__ ef, int32_t* __restrict__ out, uint8_t* __restrict__ odm,
           uint8_t* __restrict__ oef, uint8_t* __restrict__ used, int count_live,
           int64_t* __restrict__ ctr, TnpLB lb) {
  __shared__ int cnt[LIPT][TNP_WAVES];
  __shared__ int64_t slot;
  __shared__ uint64_t acts[TNP_WAVES];
  const int64_t tile = blockIdx.x;  // ticket-free look-back (lb_prefix_rc)
  const int64_t base = tile * LTILE;
  const int64_t last = (base + LTILE < N ? base + LTILE : N) - 1;  // last item of the tile
  // block-uniform source of the tile: all old edges / all e_new / all c_new
  // (straight-line loads) or a tile straddling two segments (per-item branch)
  const int64_t ES = src.E + src.S;
  const int kind = last < src.E ? 0 : (base >= src.E && last < ES) ? 1 : (base >= ES ? 2 : 3);
  int a[LIPT], b[LIPT];
  uint32_t d[LIPT], m[LIPT];  // high plane, first split plane
  if (kind == 0) {
    const int2* e2 = reinterpret_cast<const int2*>(src.edges);
#pragma unroll
    for (int k = 0; k < LIPT; ++k) {
      const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
      const int64_t ic = i < last ? i : last;
      const int2 ab = e2[ic];
      a[k] = ab.x;
      b[k] = ab.y;
      d[k] = dm[ic];
      m[k] = ef[ic];
    }
  } else {
    if (kind == 1) {
#pragma unroll
      for (int k = 0; k < LIPT; ++k) {
        const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
        const int64_t r = (i < last ? i : last) - src.E;
        a[k] = src.sb[r];
        b[k] = (int)(src.V + r);
      }
    } else if (kind == 2) {
      const uint64_t lo_mask = (1ull << src.nb) - 1ull;
#pragma unroll
      for (int k = 0; k < LIPT; ++k) {
        const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
        const uint64_t key = src.ckeys[(i < last ? i : last) - ES];
        a[k] = (int)(key >> src.nb);
        b[k] = (int)(key & lo_mask);
      }
    } else {
#pragma unroll
      for (int k = 0; k < LIPT; ++k) {
        const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
        fetch_edge(src, i < last ? i : last, a[k], b[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < LIPT; ++k) {
      const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
      d[k] = (i < src.E) ? dm[i] : EDGE_STALE;  // mixed tile: old edges keep theirs
      m[k] = (i < src.E) ? ef[i] : EDGE_NOSPLIT;
    }
  }
#pragma unroll
  for (int k = 0; k < LIPT; ++k) {
    if (d[k] == EDGE_STALE)  // new or rewired edge: masks from the endpoint keys
      edge_bytes<KW>(pz, a[k], b[k], amask, d[k], m[k]);
  }
  uint64_t bal[LIPT];
  uint64_t act = 0;
#pragma unroll
  for (int k = 0; k < LIPT; ++k) {
    const int64_t i = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    const bool f = (i <= last) && ((int)d[k] > idx) && d[k] != EDGE_DEAD;
    // (an old edge's first split plane is above idx: else it would have split)
    if (f && m[k] != EDGE_NOSPLIT) act |= tnp::act_bit((int)m[k]);
    bal[k] = __ballot(f);
    if (tnp::lane() == 0) cnt[k][tnp::wave()] = __popcll(bal[k]);
  }
  __syncthreads();
  int64_t agg = 0;
#pragma unroll
  for (int k = 0; k < LIPT; ++k)
#pragma unroll
    for (int w = 0; w < TNP_WAVES; ++w) agg += cnt[k][w];
  // a predecessor tile not yet published: count its kept edges item by item
  auto tile_agg = [&](int64_t t) -> int64_t {
    const int64_t b0 = t * LTILE, b1 = b0 + LTILE < N ? b0 + LTILE : N;
    int c = 0;
    for (int64_t i = b0 + tnp::lane(); i < b1; i += 64) {
      uint32_t dd = (i < src.E) ? dm[i] : EDGE_STALE;
      if (dd == EDGE_STALE) {
        int ea, eb;
        fetch_edge(src, i, ea, eb);
        uint32_t mm;
        edge_bytes<KW>(pz, ea, eb, amask, dd, mm);
      }
      c += (int)dd > idx && dd != EDGE_DEAD;
    }
    return tnp::wave_sum((int64_t)c);
  };
  // (its tiles publish tens of µs after dispatch: poll long before recomputing)
  const int64_t prefix = tnp::lb_prefix_rc(lb, tile, agg, &slot, tile_agg, TNP_PRUNE_SPIN);
  int64_t run = prefix;
  int newly = 0;  // count_live: endpoints this thread marked live first
#pragma unroll
  for (int k = 0; k < LIPT; ++k) {
    int64_t off = run;
    int tot = 0;
#pragma unroll
    for (int w = 0; w < TNP_WAVES; ++w) {
      const int c = cnt[k][w];
      off += (w < tnp::wave()) ? c : 0;
      tot += c;
    }
    if ((bal[k] >> tnp::lane()) & 1) {
      const int64_t o = off + tnp::mbcnt(bal[k]);
      // (the kept list is read again a whole step later: streamed out)
      __builtin_nontemporal_store((uint64_t)(uint32_t)a[k] | ((uint64_t)(uint32_t)b[k] << 32),
                                  reinterpret_cast<uint64_t*>(out) + o);  // (int2 {a, b})
      odm[o] = (uint8_t)d[k];
      oef[o] = (uint8_t)m[k];
      if (count_live) {
        // small complexes: the distinct live count without a counting pass
        // (a word-wide atomic OR tells who set each byte first)
        unsigned* w4 = reinterpret_cast<unsigned*>(used);
        const int ab[2] = {a[k], b[k]};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const unsigned sh = 8u * (unsigned)(ab[q] & 3);
          newly += ((atomicOr(w4 + (ab[q] >> 2), 1u << sh) >> sh) & 0xFFu) == 0u;
        }
      } else {
        used[a[k]] = 1;
        used[b[k]] = 1;
      }
    }
    run += tot;
  }
  if (count_live) {
    const int wn = tnp::wave_sum(newly);
    if (tnp::lane() == 0 && wn) atomicAdd((unsigned long long*)&ctr[CTR_V], (unsigned long long)wn);
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) ctr[CTR_E] = prefix + agg;
  act = tnp::wave_or(act);
  if (tnp::lane() == 0) acts[tnp::wave()] = act;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < TNP_WAVES; ++w) t |= acts[w];
    tnp::or_sticky(&ctr[CTR_ACTIVE], t);
  }
}

// Lazy pruning (no compaction).  The old edges stay in their slots: a
// removed one is marked EDGE_DEAD, a rewired one (EDGE_STALE) gets its
// recomputed bytes, a kept one is not rewritten; e_new / c_new go behind
// them to slots E + r (removed ones marked dead).  The live edges so keep
// the order of the reference's `edges[p_idx]` (subpoly.py:246-263) with no
// look-back and no rewrite of the kept edges: a step that splits few edges
// but removes many costs one byte per old edge plus the kept edges' endpoint
// reads (live flags).  Kept count per workgroup -> part[blockIdx.x] (folded
// by the counting pass, launch_count_flags), next-active mask -> ctr.
constexpr int LZ_IPT = 4;
template <int KW>
__global__ void __launch_bounds__(TNP_BLOCK)
k_prune_lazy(EdgeSrc src, int64_t i0, int64_t N, int idx, Key<KW> amask, const uint64_t* __restrict__ pz,
             int32_t* __restrict__ edges, uint8_t* __restrict__ dm, uint8_t* __restrict__ ef,
             uint8_t* __restrict__ used, int64_t* __restrict__ part, int64_t* __restrict__ ctr) {
  __shared__ int64_t lds[TNP_WAVES];
  __shared__ uint64_t acts[TNP_WAVES];
  int2* const e2 = reinterpret_cast<int2*>(edges);
  const uint64_t lo_mask = (1ull << src.nb) - 1ull;
  const int64_t ES = src.E + src.S;
  int64_t kept = 0;
  uint64_t act = 0;
  for (int64_t t0 = i0 + (int64_t)blockIdx.x * TNP_BLOCK * LZ_IPT; t0 < N;
       t0 += (int64_t)gridDim.x * TNP_BLOCK * LZ_IPT) {
    uint32_t d[LZ_IPT], m[LZ_IPT];
    int a[LZ_IPT], b[LZ_IPT];
    bool need[LZ_IPT];  // endpoints needed (kept or stale old edge, or a new edge)
#pragma unroll
    for (int k = 0; k < LZ_IPT; ++k) {
      const int64_t i = t0 + (int64_t)k * TNP_BLOCK + threadIdx.x;
      d[k] = i < src.E ? dm[i] : (i < N ? EDGE_STALE : EDGE_DEAD);
      m[k] = i < src.E ? ef[i] : EDGE_NOSPLIT;
    }
#pragma unroll
    for (int k = 0; k < LZ_IPT; ++k) {
      const int64_t i = t0 + (int64_t)k * TNP_BLOCK + threadIdx.x;
      need[k] = d[k] == EDGE_STALE || (d[k] != EDGE_DEAD && (int)d[k] > idx);
      a[k] = b[k] = 0;
      if (!need[k]) continue;
      if (i < src.E) {
        const int2 ab = e2[i];
        a[k] = ab.x;
        b[k] = ab.y;
      } else if (i < ES) {
        a[k] = src.sb[i - src.E];
        b[k] = (int)(src.V + (i - src.E));
      } else {
        const uint64_t key = src.ckeys[i - ES];
        a[k] = (int)(key >> src.nb);
        b[k] = (int)(key & lo_mask);
      }
    }
#pragma unroll
    for (int k = 0; k < LZ_IPT; ++k) {
      const int64_t i = t0 + (int64_t)k * TNP_BLOCK + threadIdx.x;
      if (i >= N) continue;
      const bool stale = d[k] == EDGE_STALE;
      if (stale)  // rewired or new: bytes from the endpoint keys
        edge_bytes<KW>(pz, a[k], b[k], amask, d[k], m[k]);
      const bool keep = need[k] && (int)d[k] > idx;
      if (i >= src.E)  // (int2 {a, b}, streamed: read again a step later)
        __builtin_nontemporal_store((uint64_t)(uint32_t)a[k] | ((uint64_t)(uint32_t)b[k] << 32),
                                    reinterpret_cast<uint64_t*>(edges) + i);
      if (i >= src.E || stale || (!keep && d[k] != EDGE_DEAD)) {
        dm[i] = keep ? (uint8_t)d[k] : EDGE_DEAD;
        ef[i] = keep ? (uint8_t)m[k] : EDGE_NOSPLIT;
      }
      if (keep) {
        used[a[k]] = 1;
        used[b[k]] = 1;
        ++kept;
        if (m[k] != EDGE_NOSPLIT) act |= tnp::act_bit((int)m[k]);
      }
    }
  }
  kept = tnp::wave_sum(kept);
  act = tnp::wave_or(act);
  if (tnp::lane() == 0) {
    lds[tnp::wave()] = kept;
    acts[tnp::wave()] = act;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t k = 0;
    uint64_t t = 0;
    for (int w = 0; w < TNP_WAVES; ++w) {
      k += lds[w];
      t |= acts[w];
    }
    part[blockIdx.x] = k;
    tnp::or_sticky(&ctr[CTR_ACTIVE], t);
  }
}

// Split-eps mode (subpoly's eps argument != Net.eps, subpoly.py:24): the
// first split plane >= from of every live edge at the step's eps -- the
// sign test of subpoly.py:104-105 on the cached plane values of both
// endpoints (the mode keeps every plane cached) -- instead of the one the
// Net.eps keys give; OR of them -> ctr[CTR_ACTIVE] when ctr != null
__global__ void __launch_bounds__(TNP_BLOCK)
k_ef_cache(const int32_t* __restrict__ edges, int64_t E, const uint8_t* __restrict__ dm,
           uint8_t* __restrict__ ef, const float* __restrict__ pre, int64_t ld, int from, int K,
           float eps_s, int64_t* __restrict__ ctr) {
  __shared__ uint64_t lds[TNP_WAVES];
  uint64_t act = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (dm[i] == EDGE_DEAD) continue;
    const int2 ab = reinterpret_cast<const int2*>(edges)[i];
    uint8_t f = EDGE_NOSPLIT;
    for (int p = from; p < K; ++p) {
      const float d0 = pre[(int64_t)p * ld + ab.x], d1 = pre[(int64_t)p * ld + ab.y];
      if ((__fmul_rn(d0, d1) < 0.f) && (fabsf(d0) > eps_s) && (fabsf(d1) > eps_s)) {
        f = (uint8_t)p;
        break;
      }
    }
    ef[i] = f;
    if (f != EDGE_NOSPLIT) act |= 1ull << f;
  }
  if (!ctr) return;
  act = tnp::wave_or(act);
  if (tnp::lane() == 0) lds[tnp::wave()] = act;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < TNP_WAVES; ++w) t |= lds[w];
    tnp::or_sticky(&ctr[CTR_ACTIVE], t);
  }
}

// masks of every edge from the endpoint keys (after a load, or when the
// curve path rewired edges); OR of the split masks on planes of amask into
// ctr[CTR_ACTIVE] when ctr != null
template <int KW>
__global__ void __launch_bounds__(TNP_BLOCK)
k_edge_masks(const int32_t* __restrict__ edges, int64_t E, const uint64_t* __restrict__ pz,
             uint8_t* __restrict__ dm, uint8_t* __restrict__ ef, Key<KW> amask,
             int keep_dead, int64_t* __restrict__ ctr) {
  __shared__ uint64_t lds[TNP_WAVES];
  uint64_t act = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (keep_dead && dm[i] == EDGE_DEAD) continue;  // stays deleted
    const int2 ab = reinterpret_cast<const int2*>(edges)[i];
    uint32_t d, f;
    edge_bytes<KW>(pz, ab.x, ab.y, amask, d, f);
    dm[i] = (uint8_t)d;
    ef[i] = (uint8_t)f;
    if (f != EDGE_NOSPLIT) act |= tnp::act_bit((int)f);
  }
  if (!ctr) return;
  act = tnp::wave_or(act);
  if (tnp::lane() == 0) lds[tnp::wave()] = act;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < TNP_WAVES; ++w) t |= lds[w];
    tnp::or_sticky(&ctr[CTR_ACTIVE], t);
  }
}

// number of set byte flags -> ctr[slot] (+=, one atomic per block)
__global__ void __launch_bounds__(TNP_BLOCK)
k_count_flags(const uint8_t* __restrict__ f, int64_t n, int64_t* __restrict__ ctr, int slot,
              const int64_t* __restrict__ part, int nparts, int pslot) {
  __shared__ int lds[TNP_WAVES];
  __shared__ int64_t lds64[TNP_WAVES];
  if (part && blockIdx.x == 0) {  // the lazy prune's per-workgroup kept counts
    int64_t p = 0;
    for (int i = threadIdx.x; i < nparts; i += TNP_BLOCK) p += part[i];
    p = tnp::wave_sum(p);
    if (tnp::lane() == 0) lds64[tnp::wave()] = p;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t t = 0;
      for (int w = 0; w < TNP_WAVES; ++w) t += lds64[w];
      ctr[pslot] = t;
    }
  }
  int c = 0;
  const int64_t i0 = ((int64_t)blockIdx.x * TNP_BLOCK + threadIdx.x) * 16;
  const int64_t stride = (int64_t)gridDim.x * TNP_BLOCK * 16;
  for (int64_t i = i0; i < n; i += stride) {
    if (i + 15 < n) {
      const uint4 v = *reinterpret_cast<const uint4*>(f + i);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q)  // bytes are 0/1
        c += __popc(w[q] & 0x01010101u);
    } else {
      for (int64_t j = i; j < n; ++j) c += f[j] != 0;
    }
  }
  c = tnp::wave_sum(c);
  if (tnp::lane() == 0) lds[tnp::wave()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < TNP_WAVES; ++w) t += lds[w];
    if (t) atomicAdd((unsigned long long*)&ctr[slot], (unsigned long long)t);
  }
}

// byte flags -> int32 flags (the compaction scan's input)
__global__ void k_widen_flags(const uint8_t* __restrict__ f, int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = f[i];
}

template <int KW>
__global__ void k_gather_vertices(const int32_t* __restrict__ used, const int64_t* __restrict__ nid,
                                  int64_t NV, int K, int keep_from,
                                  const float* __restrict__ xyz, const float* __restrict__ pre,
                                  int64_t ld, const uint64_t* __restrict__ pos,
                                  const uint64_t* __restrict__ zero, const uint64_t* __restrict__ grid,
                                  float* __restrict__ xyz2, float* __restrict__ pre2, int64_t ld2,
                                  uint64_t* __restrict__ pos2, uint64_t* __restrict__ zero2,
                                  uint64_t* __restrict__ grid2, uint64_t* __restrict__ pz2) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= NV || !used[v]) return;
  int64_t n = nid[v];
#pragma unroll
  for (int d = 0; d < 3; ++d) xyz2[3 * n + d] = xyz[3 * v + d];
  for (int p = keep_from; p < K; ++p) pre2[(int64_t)p * ld2 + n] = pre[(int64_t)p * ld + v];
  const Key<KW> p = tnp::vkey_load<KW>(pos, v), z = tnp::vkey_load<KW>(zero, v);
  tnp::pz_store(pz2, n, p, z);  // (pos2 / zero2: views of pz2)
  grid2[n] = grid[v];
}

__global__ void k_remap_edges(int32_t* __restrict__ edges, int64_t E, const int64_t* __restrict__ nid) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * E) return;
  edges[i] = (int32_t)nid[edges[i]];
}


// per-step counter readback: every lane stores its own word (the block is
// tiny), the sequence word last, after a system-scope fence
__global__ void k_publish(int64_t* __restrict__ ctr, volatile int64_t* host, int64_t seq, int clear) {
  const int t = threadIdx.x;
  const int64_t v = t < 32 ? ctr[t] : 0;
  if (t < CTR_N) host[t] = v;
  if (clear && t < 32) ctr[t] = 0;  // (the word this lane read: program order)
  __threadfence_system();
  __syncthreads();
  if (t == 31) host[t] = seq;
}
// k_publish with the deferred live counts summed in: PS_THREADS threads, each
// chunk's loads all in flight before any is added (a one-wave loop over the
// ~1.5 K part words waited for each load in turn: 9-12 us per launch)
constexpr int PS_THREADS = 256, PS_IPT = 4;
__global__ void __launch_bounds__(PS_THREADS)
k_publish_sums(const int64_t* __restrict__ ctr, volatile int64_t* host, int64_t seq,
               const int64_t* __restrict__ vpart, int nv, const int64_t* __restrict__ epart, int ne) {
  __shared__ int64_t red[2][PS_THREADS / 64];
  const int t = threadIdx.x;
  int64_t v = 0, e = 0;
  for (int b = 0; b < nv || b < ne; b += PS_THREADS * PS_IPT) {
    int64_t pv[PS_IPT], pe[PS_IPT];
#pragma unroll
    for (int k = 0; k < PS_IPT; ++k) {
      const int i = b + k * PS_THREADS + t;
      pv[k] = i < nv ? vpart[i] : 0;
      pe[k] = i < ne ? epart[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < PS_IPT; ++k) {
      v += pv[k];
      e += pe[k];
    }
  }
  v = tnp::wave_sum(v);
  e = tnp::wave_sum(e);
  if (tnp::lane() == 0) {
    red[0][tnp::wave()] = v;
    red[1][tnp::wave()] = e;
  }
  __syncthreads();
  if (t < 64) {
    v = e = 0;
#pragma unroll
    for (int w = 0; w < PS_THREADS / 64; ++w) {
      v += red[0][w];
      e += red[1][w];
    }
    if (t < CTR_N) host[t] = t == CTR_V ? v : (t == CTR_E && ne > 0) ? e : ctr[t];
    __threadfence_system();
  }
  __syncthreads();
  if (t == 31) host[t] = seq;
}

}  // namespace

// ----------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------
int64_t step_tiles(int64_t n) { return (n + TILE - 1) / TILE; }
int64_t lb_tiles(int64_t n) { return (n + LTILE - 1) / LTILE; }
int split_hit_workers(int64_t V) {
  return V > 0 ? (int)std::min<int64_t>(HIT_GRID, (V + HCHUNK - 1) / HCHUNK) : 0;
}
int64_t split_tiles(int64_t n) {
  const int64_t t = (int64_t)TNP_BLOCK * split_ipt(n);
  return (n + t - 1) / t;
}
int64_t run_tiles(int64_t n) { return (n + STILE - 1) / STILE; }

int launch_split_lb(int32_t* edges, int64_t E, const uint8_t* sm, uint8_t* dm, int idx, int64_t V,
                    int32_t* sa, int32_t* sb, int64_t* ctr, int32_t* eidx, const TnpLB& lb,
                    hipStream_t s, const HitArgs* hits) {
  const int64_t tiles = split_tiles(E);
  HitArgs ha{nullptr, nullptr, 0, 0.f, nullptr, nullptr};
  int64_t hg = 0;
  if (hits && hits->V > 0) {
    ha = *hits;
    hg = split_hit_workers(hits->V);
  }
  const unsigned grid = (unsigned)(tiles + hg);
  if (split_ipt(E) == SIPT_BIG)
    hipLaunchKernelGGL(k_split_lb<SIPT_BIG>, dim3(grid), dim3(TNP_BLOCK), 0, s, edges, E, tiles, sm,
                       dm, idx, V, sa, sb, ctr, eidx, lb, ha);
  else
    hipLaunchKernelGGL(k_split_lb<SIPT_SMALL>, dim3(grid), dim3(TNP_BLOCK), 0, s, edges, E, tiles,
                       sm, dm, idx, V, sa, sb, ctr, eidx, lb, ha);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_new_vertices(const int32_t* sa, const int32_t* sb, int64_t S, const float* col,
                        float eps, float* xyz, int64_t V, hipStream_t s) {
  if (S <= 0) return 0;
  hipLaunchKernelGGL(k_new_vertices, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, sa, sb, S, col, eps,
                     xyz, V);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_fail_check(const int32_t* sa, const int32_t* sb, int64_t S, int idx,
                      const uint64_t* zero, const float* stage, float eps, uint64_t* shared,
                      int64_t* ctr, const uint64_t* grid_new, const OwnBox& own, int kw, hipStream_t s) {
  if (S <= 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_fail_check<2>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, sa, sb, S, idx, zero,
                       stage, eps, shared, ctr, grid_new, own);
  else
    hipLaunchKernelGGL(k_fail_check<1>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, sa, sb, S, idx, zero,
                       stage, eps, shared, ctr, grid_new, own);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_finalize_new(int64_t S, int K, int override_, const uint64_t* shared, float* stage,
                        float eps, float* pre, int64_t ld, int keep_from, int64_t V, uint64_t* pos,
                        uint64_t* zero, const int64_t* ctr, uint64_t* pz, int kw, hipStream_t s) {
  if (S <= 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_finalize_new<2>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, S, K, override_,
                       shared, stage, eps, pre, ld, keep_from, V, pos, zero, ctr, pz);
  else
    hipLaunchKernelGGL(k_finalize_new<1>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, S, K, override_,
                       shared, stage, eps, pre, ld, keep_from, V, pos, zero, ctr, pz);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_hits(const float* col, const uint8_t* alive, int64_t V, float eps, int32_t* members,
                int64_t S, int64_t* ctr, hipStream_t s) {
  if (V > 0) {
    const unsigned g = (unsigned)std::min<int64_t>(HIT_GRID, (V + HCHUNK - 1) / HCHUNK);
    hipLaunchKernelGGL(k_hit_append, dim3(g), dim3(TNP_BLOCK), 0, s, col, alive, V, eps, members, S, ctr);
  }
  if (S > 0) return launch_new_members(members, S, V, s);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_count_unowned(const uint64_t* grid, int64_t n, const OwnBox& own, int64_t* ctr, hipStream_t s) {
  if (n <= 0 || !tnp::own_any(own)) return 0;
  hipLaunchKernelGGL(k_count_unowned, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, grid, n, own, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_new_members(int32_t* members, int64_t S, int64_t V, hipStream_t s) {
  if (S <= 0) return 0;
  hipLaunchKernelGGL(k_new_members, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, members, S, V);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_span_count(const int32_t* members, int64_t S, int64_t M, const uint64_t* grid,
                      const uint64_t* zero, int idx, int32_t* cnt, int64_t* part, int64_t* ctr,
                      int kw, hipStream_t s) {
  if (M <= 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_span_count<2>, dim3(tnp_grid(M)), dim3(TNP_BLOCK), 0, s, members, S, M, grid,
                       zero, idx, cnt, part, ctr);
  else
    hipLaunchKernelGGL(k_span_count<1>, dim3(tnp_grid(M)), dim3(TNP_BLOCK), 0, s, members, S, M, grid,
                       zero, idx, cnt, part, ctr);
  hipLaunchKernelGGL(k_sum_parts, dim3(1), dim3(TNP_BLOCK), 0, s, part, (int64_t)tnp_grid(M), ctr,
                     (int)CTR_A);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_span_emit(const int32_t* members, int64_t S, int64_t M, const uint64_t* grid, int NC,
                     const int64_t* eoff, uint32_t* ekey, int32_t* eval, const int64_t* ctr,
                     hipStream_t s) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(k_span_emit, dim3(tnp_grid(M)), dim3(TNP_BLOCK), 0, s, members, S, grid, NC,
                     eoff, ekey, eval, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int64_t pair_run_tiles(int64_t T) { return (T + PTILE - 1) / PTILE; }
int launch_run_starts(const uint32_t* key, int64_t T, int32_t* rstart, int64_t* ctr, const TnpLB& lb,
                      hipStream_t s) {
  if (T <= 0) return 0;
  const int64_t tiles = run_tiles(T);
  hipLaunchKernelGGL(k_run_starts_lb, dim3((unsigned)tiles), dim3(TNP_BLOCK), 0, s, key, T, tiles,
                     rstart, ctr, lb);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_pair_runs(const uint32_t* key, const int32_t* rstart, int64_t T, int32_t* pcell,
                     int32_t* pent, int32_t* pn, int64_t* ptoff, int64_t* ctr, const TnpLB& lb_rank,
                     const TnpLB& lb_pairs, hipStream_t s) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(k_pair_runs_lb, dim3((unsigned)pair_run_tiles(T)), dim3(TNP_BLOCK), 0, s, key,
                     rstart, pcell, pent, pn, ptoff, ctr, lb_rank, lb_pairs);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_entry_keys(const int32_t* ent_v, const uint32_t* ekey, int NC, int64_t T,
                      const uint64_t* grid, const uint64_t* pz, void* ent, int kw, hipStream_t s) {
  if (T <= 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_entry_keys<2>, dim3(tnp_grid(T)), dim3(TNP_BLOCK), 0, s, ent_v, ekey, NC, T, grid, pz,
                       static_cast<CellEntT<2>*>(ent));
  else
    hipLaunchKernelGGL(k_entry_keys<1>, dim3(tnp_grid(T)), dim3(TNP_BLOCK), 0, s, ent_v, ekey, NC, T, grid, pz,
                       static_cast<CellEnt*>(ent));
  TNP_CHECK(hipGetLastError());
  return 0;
}
// persistent blocks: exactly the resident ones (occupancy x CUs), so the
// static chunk stride never leaves a second, late wave of blocks as a tail
// (cached per device: one process may drive several devices)
template <typename K>
static int resident_grid(K kernel, int slot) {
  static int cache[2][64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 2048;
  int& g = cache[slot][dev];
  if (!g) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, TNP_BLOCK, 0) != hipSuccess ||
        cus <= 0 || per_cu <= 0)
      g = 2048;
    else
      g = cus * per_cu;
  }
  return g;
}
static int connect_grid_size() {
  return std::max(resident_grid(k_connect<1>, 0), resident_grid(k_connect_win, 1));
}
int64_t connect_chunks(int64_t TT) { return (TT + CCH - 1) / CCH; }
int64_t connect_chunk_pairs() { return CCH; }
int launch_chunk_cells(const int64_t* ptoff, const int32_t* pn, int64_t rcap, int32_t* bcell,
                       int64_t cap, int64_t* ctr, hipStream_t s) {
  hipLaunchKernelGGL(k_chunk_cells, dim3(tnp_grid(rcap)), dim3(TNP_BLOCK), 0, s, ptoff, pn, rcap,
                     bcell, cap, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_connect(const int64_t* ptoff, const int32_t* pcell, const int32_t* pn,
                   const int32_t* pent, int NC, int64_t max_tests, const int32_t* bcell,
                   const void* ent, int idx, int nb, int filt_last, int kw, uint64_t* keys,
                   int64_t cap, int64_t* xs, int64_t* ctr, hipStream_t s, const int64_t* bstat, int nbstat) {
  static_assert(CONNECT_CELLS >= CCH + 2, "chunk cell window");
  const int grid = connect_grid_size();
  // the pruning filter: planes [idx, filt_last] (filt_last < 0: none)
  if (kw == 2)
    hipLaunchKernelGGL(k_connect<2>, dim3(grid), dim3(TNP_BLOCK), 0, s, ptoff, pcell, pn, pent, NC, max_tests, bcell,
                       static_cast<const CellEntT<2>*>(ent), idx, nb,
                       filt_last >= 0 ? tnp::key_range<2>(idx, filt_last) : tnp::key_zero<2>(), keys, cap, xs, ctr,
                       bstat, nbstat);
  else
    hipLaunchKernelGGL(k_connect<1>, dim3(grid), dim3(TNP_BLOCK), 0, s, ptoff, pcell, pn, pent, NC, max_tests, bcell,
                       static_cast<const CellEnt*>(ent), idx, nb,
                       filt_last >= 0 ? tnp::key_range<1>(idx, filt_last) : tnp::key_zero<1>(), keys, cap, xs, ctr,
                       bstat, nbstat);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_connect_win(const CellEnt* ent, int idx, int nb, uint64_t fmask, uint64_t* keys, int64_t cap,
                       int64_t* xs, int64_t* ctr, hipStream_t s) {
  const int grid = connect_grid_size();
  hipLaunchKernelGGL(k_connect_win, dim3(grid), dim3(TNP_BLOCK), 0, s, ent, idx, nb, fmask, keys, cap, xs, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_keys_finish(int64_t* xs, int64_t cap, int64_t* ctr, hipStream_t s) {
  hipLaunchKernelGGL(k_keys_finish, dim3(1), dim3(64), 0, s, xs, cap, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_keys_compact(const uint64_t* keys, int64_t cap, const int64_t* xs, int64_t X, uint64_t* out,
                        hipStream_t s) {
  if (X <= 0) return 0;
  const unsigned g = (unsigned)std::min<int64_t>(tnp_grid(X), 4096);
  hipLaunchKernelGGL(k_keys_compact, dim3(g), dim3(TNP_BLOCK), 0, s, keys, cap, xs, X, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int64_t connect_grid() { return connect_grid_size(); }
uint64_t prune_mask(int idx, int last_plane) {
  uint64_t fmask = (idx >= 64) ? 0ull : (~0ull << idx);
  if (last_plane < 63) fmask &= (1ull << (last_plane + 1)) - 1ull;
  return fmask;
}
// the planes [lo, last_plane] (lo clamped at 0) as a KW-word key
template <int KW>
static Key<KW> plane_mask(int lo, int last_plane) {
  return tnp::key_range<KW>(lo < 0 ? 0 : lo, last_plane);
}
// the key words of a net whose last plane is last_plane
static int kw_of(int last_plane) { return last_plane + 1 <= 63 ? 1 : 2; }
int launch_prune(bool emit, const int32_t* edges, int64_t E, const int32_t* sb, int64_t S,
                 int64_t V, const uint64_t* ckeys, int nb, int64_t X, int idx,
                 int prune, int last_plane, const uint64_t* pos, const uint64_t* zero,
                 int32_t* blk, const int64_t* blkoff, int32_t* out, int32_t* used, int64_t* ctr,
                 hipStream_t s) {
  EdgeSrc src{edges, E, sb, S, V, ckeys, nb, X};
  int64_t N = E + S + X;
  if (N <= 0) return 0;
  (void)emit;
  (void)blk;
  if (kw_of(last_plane) == 2)
    hipLaunchKernelGGL(k_prune_emit<2>, dim3((unsigned)step_tiles(N)), dim3(TNP_BLOCK), 0, s, src, N,
                       plane_mask<2>(idx, last_plane), plane_mask<2>(idx + 1, last_plane), pos, zero, blkoff, prune,
                       out, used, ctr);
  else
    hipLaunchKernelGGL(k_prune_emit<1>, dim3((unsigned)step_tiles(N)), dim3(TNP_BLOCK), 0, s, src, N,
                       plane_mask<1>(idx, last_plane), plane_mask<1>(idx + 1, last_plane), pos, zero, blkoff, prune,
                       out, used, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_prune_lb(const int32_t* edges, int64_t E, const int32_t* sb, int64_t S, int64_t V,
                    const uint64_t* ckeys, int nb, int64_t X, int idx, int last_plane,
                    const uint64_t* pz, const uint8_t* dm, const uint8_t* ef, int32_t* out,
                    uint8_t* odm, uint8_t* oef, uint8_t* used, bool count_live, int64_t* ctr,
                    const TnpLB& lb, hipStream_t s) {
  EdgeSrc src{edges, E, sb, S, V, ckeys, nb, X};
  const int64_t N = E + S + X;
  if (N <= 0) {
    TNP_CHECK(hipMemsetAsync(ctr + CTR_E, 0, sizeof(int64_t), s));
    return 0;
  }
  const int64_t tiles = lb_tiles(N);
  if (kw_of(last_plane) == 2)
    hipLaunchKernelGGL(k_prune_lb<2>, dim3((unsigned)tiles), dim3(TNP_BLOCK), 0, s, src, N, tiles, idx,
                       plane_mask<2>(idx + 1, last_plane), pz, dm, ef, out, odm, oef, used, count_live ? 1 : 0, ctr,
                       lb);
  else
    hipLaunchKernelGGL(k_prune_lb<1>, dim3((unsigned)tiles), dim3(TNP_BLOCK), 0, s, src, N, tiles, idx,
                       plane_mask<1>(idx + 1, last_plane), pz, dm, ef, out, odm, oef, used, count_live ? 1 : 0, ctr,
                       lb);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int prune_lazy_blocks(int64_t N) {
  static const int64_t s_max = [] {  // TNP_PL_BLOCKS: the grid cap (experiments)
    const char* v = getenv("TNP_PL_BLOCKS");
    const int64_t b = v ? atoll(v) : PRUNE_LAZY_MAX_BLOCKS;
    return b > 0 ? b : (int64_t)PRUNE_LAZY_MAX_BLOCKS;
  }();
  return (int)std::max<int64_t>(1, std::min<int64_t>(s_max, (N + TNP_BLOCK * LZ_IPT - 1) / (TNP_BLOCK * LZ_IPT)));
}
int launch_prune_lazy(int32_t* edges, int64_t E, const int32_t* sb, int64_t S, int64_t V, const uint64_t* ckeys,
                      int nb, int64_t X, int idx, int last_plane, const uint64_t* pz, uint8_t* dm, uint8_t* ef,
                      uint8_t* used, int64_t* part, int64_t* ctr, hipStream_t s, int64_t i0, int64_t i1) {
  EdgeSrc src{edges, E, sb, S, V, ckeys, nb, X};
  if (i0 < 0 || i1 < i0 || i1 > E + S + X) {
    tnp_set_error("prune range [%lld, %lld) outside the %lld slots", (long long)i0, (long long)i1,
                  (long long)(E + S + X));
    return -1;
  }
  const int g = prune_lazy_blocks(i1 - i0);
  if (kw_of(last_plane) == 2)
    hipLaunchKernelGGL(k_prune_lazy<2>, dim3(g), dim3(TNP_BLOCK), 0, s, src, i0, i1, idx,
                       plane_mask<2>(idx + 1, last_plane), pz, edges, dm, ef, used, part, ctr);
  else
    hipLaunchKernelGGL(k_prune_lazy<1>, dim3(g), dim3(TNP_BLOCK), 0, s, src, i0, i1, idx,
                       plane_mask<1>(idx + 1, last_plane), pz, edges, dm, ef, used, part, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_ef_cache(const int32_t* edges, int64_t E, const uint8_t* dm, uint8_t* ef, const float* pre, int64_t ld,
                    int from, int K, float eps_s, int64_t* ctr, hipStream_t s) {
  if (E <= 0) return 0;
  const unsigned g = (unsigned)std::min<int64_t>(4096, tnp_grid(E));
  hipLaunchKernelGGL(k_ef_cache, dim3(g), dim3(TNP_BLOCK), 0, s, edges, E, dm, ef, pre, ld, from, K, eps_s, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_widen_flags(const uint8_t* f, int64_t n, int32_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_widen_flags, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, s, f, n, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_publish(int64_t* ctr, int64_t* host, int64_t seq, hipStream_t s, bool clear) {
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, ctr, host, seq, clear ? 1 : 0);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_publish_sums(const int64_t* ctr, int64_t* host, int64_t seq, const int64_t* vpart, int nv,
                        const int64_t* epart, int ne, hipStream_t s) {
  hipLaunchKernelGGL(k_publish_sums, dim3(1), dim3(PS_THREADS), 0, s, ctr, host, seq, vpart, nv, epart, ne);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_count_flags(const uint8_t* f, int64_t n, int64_t* ctr, int slot, hipStream_t s,
                       const int64_t* part, int nparts, int pslot) {
  if (n <= 0 && !part) return 0;
  // one device-scope atomic per workgroup on one word: they serialise at
  // ~11 ns each (MI355X_MICROARCH.md fan-in), so few workgroups that loop
  const unsigned g = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>(256, (n + 16 * TNP_BLOCK - 1) / (16 * TNP_BLOCK)));
  hipLaunchKernelGGL(k_count_flags, dim3(g), dim3(TNP_BLOCK), 0, s, f, n, ctr, slot, part, nparts, pslot);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_edge_masks(const int32_t* edges, int64_t E, const uint64_t* pz, uint8_t* dm,
                      uint8_t* sm, int from, int last_plane, bool keep_dead, int64_t* ctr, hipStream_t s) {
  if (E <= 0) return 0;
  const unsigned g = (unsigned)std::min<int64_t>(4096, tnp_grid(E));
  if (kw_of(last_plane) == 2)
    hipLaunchKernelGGL(k_edge_masks<2>, dim3(g), dim3(TNP_BLOCK), 0, s, edges, E, pz, dm, sm,
                       plane_mask<2>(from, last_plane), keep_dead ? 1 : 0, ctr);
  else
    hipLaunchKernelGGL(k_edge_masks<1>, dim3(g), dim3(TNP_BLOCK), 0, s, edges, E, pz, dm, sm,
                       plane_mask<1>(from, last_plane), keep_dead ? 1 : 0, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_gather_vertices(const int32_t* used, const int64_t* nid, int64_t NV, int K,
                           int keep_from, const float* xyz, const float* pre, int64_t ld,
                           const uint64_t* pos, const uint64_t* zero, const uint64_t* grid,
                           float* xyz2, float* pre2, int64_t ld2, uint64_t* pos2, uint64_t* zero2,
                           uint64_t* grid2, uint64_t* pz2, hipStream_t s) {
  if (NV <= 0) return 0;
  if (kw_of(K - 1) == 2)
    hipLaunchKernelGGL(k_gather_vertices<2>, dim3(tnp_grid(NV)), dim3(TNP_BLOCK), 0, s, used, nid, NV,
                       K, keep_from, xyz, pre, ld, pos, zero, grid, xyz2, pre2, ld2, pos2, zero2, grid2, pz2);
  else
    hipLaunchKernelGGL(k_gather_vertices<1>, dim3(tnp_grid(NV)), dim3(TNP_BLOCK), 0, s, used, nid, NV,
                       K, keep_from, xyz, pre, ld, pos, zero, grid, xyz2, pre2, ld2, pos2, zero2, grid2, pz2);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_remap_edges(int32_t* edges, int64_t E, const int64_t* nid, hipStream_t s) {
  if (E <= 0) return 0;
  hipLaunchKernelGGL(k_remap_edges, dim3(tnp_grid(2 * E)), dim3(TNP_BLOCK), 0, s, edges, E, nid);
  TNP_CHECK(hipGetLastError());
  return 0;
}
