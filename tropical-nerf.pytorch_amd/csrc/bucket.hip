// Grouping of a step's region members by grid cell without a global sort
// (the bucketing behind regions_to_vertices / r_idx_as_tensor /
// extract_every_valid_edge, subpoly.py:281-370, 484-535).
//
// A member (new vertex or hit vertex) belongs to every grid cell its
// eps-region spans: 1 cell per axis, 2 when it lies on a mark plane
// (subpoly.py:327-332).  The pair test needs, per cell, the contiguous list
// of its members.  Instead of radix-sorting every (cell, member) entry over
// the whole cell-id range (3 global passes), cells are grouped in spatial
// BUCKETS of (2^sh)^3 cells:
//
//   bucket_count    member -> its entries' buckets: LDS histogram per block,
//                   one global add per non-empty bin (+ the reference's
//                   augmented-row count A, the k=0 guard)
//   bucket_scan     bucket bases (one block)
//   bucket_scatter  (local cell, vertex) entries into their bucket's range
//   bucket_group    one block per bucket: LDS counting sort by local cell,
//                   the 32-byte pair-test records written cell-contiguous,
//                   the bucket's pair cells (>= 2 members) in local cell
//                   order with their local pair offsets
//   pair_scan       per-bucket pair-cell / pair totals -> global offsets
//   pair_gather     the global pair-cell list (cell, first entry, members,
//                   first pair) that k_connect walks
//
// Every count the host needs stays on the device (no readback between the
// split and the connect kernel).  Within a cell the entry order is whatever
// the atomics produce: nothing downstream depends on it (the pair test is
// symmetric, the emitted edges are sorted), so results stay bitwise
// deterministic.  Traffic per entry: 8 B scatter write + 8 B read + 24 B key
// gather + 32 B record write, against ~70 B for three 8-bit radix passes.
#include <algorithm>
#include <cstdlib>
#include <cstdio>

#include "common.h"
#include "step.h"
#include "connect.h"

namespace {

#ifndef TNP_BK_IPT
#define TNP_BK_IPT 4
#endif
constexpr int BK_IPT = TNP_BK_IPT;  // members per thread in the member passes
// grids up to this many workgroups finish their scans in the last workgroup
// (one launch less); larger ones pay more in every workgroup's tail
// (measured at 128^3: 4,913 buckets +0.26 ms per pass) and scan in a launch
// of their own
constexpr unsigned FUSE_MAX_BLOCKS = 512;
static_assert(FUSE_MAX_BLOCKS <= 512, "engine.cpp sizes the parts buffer for at least 512 workgroups");

// member m of a step: the S new vertices are slots V + m (no list needed),
// the hit vertices follow in members[S..]
__device__ __forceinline__ int member_of(const int32_t* members, int64_t S, int64_t V, int64_t m) {
  return m < S ? (int)(V + m) : members[m];
}

using BGeom = BucketGeom;

// TNP_BG_PHASES=1 (diagnostic builds, tools/build_variant.sh): per-phase
// shader-clock totals of k_bucket_group, printed per launch to stderr
#ifndef TNP_BG_PHASES
#define TNP_BG_PHASES 0
#endif
#if TNP_BG_PHASES
__device__ unsigned long long g_bg_ph[8 * 8];
#define BG_PH(k) \
  do {           \
    if (threadIdx.x == 0) tph[k] = __builtin_readcyclecounter(); \
  } while (0)
#else
#define BG_PH(k) \
  do {           \
  } while (0)
#endif

// the window pass the grouping kernel runs over each bucket (keys == null:
// none; the engine then launches k_connect_win)
struct WinArgs {
  int idx, nb;
  uint64_t fmask;
  uint64_t* keys;
  int64_t cap;
  int64_t* xs;  // per-XCD shards of the appends and pair statistics (step.h); null: ctr
  // small grids (no shards): per-bucket pair statistics [NB][4] (compatible
  // pairs, shared regions, connecting edges, window-pass pairs), plain
  // stores that k_connect's first workgroup sums -- instead of 4 atomics per
  // bucket on the counter block's words (~11 ns each, serialised)
  int64_t* bstat;
  int packed;  // the LDS-record path stages packed records (connect.h packed_ok)
};

// a bucket's pair statistics -> its bstat row, or the counter block / shards
__device__ __forceinline__ void bucket_stats_out(const WinArgs& wa, int b, int64_t c, int64_t g, int64_t x,
                                                 int64_t sp, int64_t* __restrict__ ctr) {
  if (wa.bstat) {
    int64_t* r = wa.bstat + 4 * (int64_t)b;
    r[0] = c;
    r[1] = g;
    r[2] = x;
    r[3] = sp;
    return;
  }
  if (c) atomicAdd((unsigned long long*)sink_word(wa.xs, ctr, XS_COMPAT), (unsigned long long)c);
  if (g) atomicAdd((unsigned long long*)sink_word(wa.xs, ctr, XS_P), (unsigned long long)g);
  if (x) atomicAdd((unsigned long long*)sink_word(wa.xs, ctr, XS_X), (unsigned long long)x);
  if (sp) atomicAdd((unsigned long long*)sink_word(wa.xs, ctr, XS_SP), (unsigned long long)sp);
}

// the global pair-cell list (k_connect's) and the bucket counters
struct PairLists {
  int32_t *pcell, *pent, *pn;
  int64_t* ptoff;
  int32_t* bcell;
  int64_t bcap, chunk;
  int32_t *bcount, *bcur;
  int32_t* perm;  // LDS-record path: every bucket's entries in cell order (entry indices; null: off)
};

// the new vertices' failover override, applied by the bucket count
// (k_override_new's work; shared == null: not here)
struct Override {
  int flag;  // < 0: the device predicate ctr[CTR_FAIL]; else the host's decision
  const uint64_t* shared;
  float* pre;
  int64_t ld;
  int keep_from;
  const uint64_t* pos;  // (pos / zero: views of pz, common.h vkey_load)
  const uint64_t* zero;
  ulonglong2* pz;
};

__device__ __forceinline__ void span_of(uint64_t g, int lo[3], int n[3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int o = tnp::grid_off(g, d);
    const bool z = tnp::grid_zero(g, d);
    lo[d] = (z ? o - 1 : o) + 2;  // cell coordinate + 2 (cell_id convention)
    n[d] = z ? 2 : 1;
  }
}

__device__ __forceinline__ int bucket_of(const BGeom& G, int cx, int cy, int cz) {
  return (((cx - G.xorg) >> G.sh) * G.NBy + ((cy - G.yorg) >> G.sh)) * G.NBz + ((cz - G.zorg) >> G.sh);
}

__device__ __forceinline__ int local_of(const BGeom& G, int cx, int cy, int cz) {
  const int m = (1 << G.sh) - 1;
  return (((cx - G.xorg) & m) << (2 * G.sh)) | (((cy - G.yorg) & m) << G.sh) | ((cz - G.zorg) & m);
}

// every cell of the span inside the buckets' box (else the member is
// skipped and flagged: the complex left the span the engine was told of)
__device__ __forceinline__ bool span_inside(const BGeom& G, const int lo[3], const int n[3]) {
  return ((unsigned)(lo[0] - G.xorg) <= (unsigned)(G.xn - n[0])) &
         ((unsigned)(lo[1] - G.yorg) <= (unsigned)(G.yn - n[1])) &
         ((unsigned)(lo[2] - G.zorg) <= (unsigned)(G.zn - n[2]));
}

// exclusive scan of n counts another workgroup of this launch handed over
// (tnp::last_block; sc1 loads) -> out[0..n] (out[n] = total); one workgroup
template <typename T>
__device__ __forceinline__ int64_t scan_handed(const T* cnt, int n, int64_t* out, int64_t* lds) {
  constexpr int PER = (BUCKET_MAX + TNP_BLOCK - 1) / TNP_BLOCK;  // n <= BUCKET_MAX
  const int b0 = threadIdx.x * PER;
  int64_t v[PER];
  if constexpr (sizeof(T) == 4) {
    // int32 counts as 8-B pairs (cnt holds n + 1 slots, PER is even): the
    // compiler keeps 4-B sc1 loads one at a time, 8-B ones in flight together
    static_assert(PER % 2 == 0, "pairs");
    const int64_t* c2 = reinterpret_cast<const int64_t*>(cnt);
#pragma unroll
    for (int k = 0; k < PER; k += 2) {
      const int64_t w = b0 + k < n ? tnp::ld_agent(c2 + (b0 + k) / 2) : 0;
      v[k] = (int32_t)(uint32_t)w;
      v[k + 1] = b0 + k + 1 < n ? (int64_t)(int32_t)(uint32_t)(w >> 32) : 0;
    }
  } else {
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = b0 + k < n ? (int64_t)tnp::ld_agent(cnt + b0 + k) : 0;  // all in flight
  }
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) s += v[k];
  int64_t tot;
  int64_t run = tnp::block_scan_excl(s, lds, tot);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (b0 + k < n) out[b0 + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) out[n] = tot;
  return tot;
}

// (1) per-bucket entry counts; per-block augmented-row sums -> part[]; the
// workgroup finishing last scans the counts into the bucket bases (-> T)
// and sums the parts (-> A).  live (prune steps): the next live-flag set is
// zeroed here, after the hit pass has read it.
__global__ void __launch_bounds__(TNP_BLOCK)
k_bucket_count(const int32_t* __restrict__ members, int64_t S, int64_t V, int64_t M,
               const uint64_t* __restrict__ grid,
               const uint64_t* zero, int idx, BGeom G, int NB,
               int32_t* __restrict__ bcount, int64_t* __restrict__ part, int64_t* __restrict__ bbase,
               uint8_t* __restrict__ live, int64_t nlive, int fuse, Override ov,
               int64_t* __restrict__ ctr) {
  extern __shared__ int hist[];  // NB bins (dynamic: the geometry's count)
  __shared__ int64_t lds[TNP_WAVES];
  __shared__ int last;
  if (live) {
    const int64_t n16 = nlive >> 4;
    uint4* l4 = reinterpret_cast<uint4*>(live);
    for (int64_t i = (int64_t)blockIdx.x * TNP_BLOCK + threadIdx.x; i < n16; i += (int64_t)gridDim.x * TNP_BLOCK)
      l4[i] = make_uint4(0, 0, 0, 0);
    if (blockIdx.x == 0 && threadIdx.x < (nlive & 15)) live[(n16 << 4) + threadIdx.x] = 0;
  }
  const uint64_t below = (idx >= 64) ? ~0ull : ((1ull << idx) - 1ull);
  const int64_t base = (int64_t)blockIdx.x * TNP_BLOCK * BK_IPT;
  // workgroups past the members only zero live flags: no histogram to clear
  // or flush (a near-empty step's grid is sized by the live-flag zeroing)
  const bool counts = base < M;
  if (counts) {
    for (int i = threadIdx.x; i < NB; i += TNP_BLOCK) hist[i] = 0;
    __syncthreads();
  }
  int64_t aug = 0;
  bool k0 = false;
  // every item's loads in flight before any is used
  int vv[BK_IPT];
  uint64_t gg[BK_IPT], zz[BK_IPT];
#pragma unroll
  for (int k = 0; k < BK_IPT; ++k) {
    const int64_t m = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    vv[k] = m < M ? member_of(members, S, V, m) : -1;
  }
#pragma unroll
  for (int k = 0; k < BK_IPT; ++k) {
    const int v = vv[k] >= 0 ? vv[k] : 0;
    gg[k] = grid[v];
    zz[k] = zero[2 * (int64_t)v];  // (a view of pz: 2 words per vertex)
  }
  // the failover override of the new vertices (masked_fill_ of their shared
  // planes, subpoly_debug.py:48), fused here: new members are slots V + m
  if (ov.shared && (ov.flag < 0 ? ctr[CTR_FAIL] != 0 : ov.flag != 0)) {
    uint64_t sh[BK_IPT], ps[BK_IPT];
#pragma unroll
    for (int k = 0; k < BK_IPT; ++k) {  // loads first (the stores below could alias them)
      const int64_t m = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
      const int64_t mc = m < S ? m : 0;
      sh[k] = ov.shared[mc];
      ps[k] = ov.pos[2 * (V + mc)];
    }
#pragma unroll
    for (int k = 0; k < BK_IPT; ++k) {
      const int64_t m = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
      if (m >= S) continue;
      for (uint64_t t = sh[k]; t; t &= t - 1) {
        const int p = __builtin_ctzll(t);
        if (p >= ov.keep_from) ov.pre[(int64_t)p * ov.ld + V + m] = 0.f;
      }
      const uint64_t pp = ps[k] & ~sh[k], z = zz[k] | sh[k];
      ov.pz[V + m] = make_ulonglong2(pp, z);
      zz[k] = z;
    }
  }
  bool outside = false;
#pragma unroll
  for (int k = 0; k < BK_IPT; ++k) {
    if (vv[k] < 0) continue;
    int lo[3], n[3];
    span_of(gg[k], lo, n);
    if (!span_inside(G, lo, n)) {
      outside = true;
      continue;
    }
    for (int i = 0; i < n[0]; ++i)
      for (int j = 0; j < n[1]; ++j)
        for (int q = 0; q < n[2]; ++q) atomicAdd(&hist[bucket_of(G, lo[0] + i, lo[1] + j, lo[2] + q)], 1);
    const int kz = __popcll(zz[k] & below) + (n[0] - 1) + (n[1] - 1) + (n[2] - 1);
    aug += 1ll << kz;
    k0 |= kz == 0;
  }
  if (__ballot(k0) && tnp::lane() == 0) atomicOr((unsigned long long*)&ctr[CTR_K0], 1ull);
  if (__ballot(outside) && tnp::lane() == 0) atomicOr((unsigned long long*)&ctr[CTR_K0], 2ull);
  if (counts) {
    __syncthreads();
    for (int i = threadIdx.x; i < NB; i += TNP_BLOCK)
      if (hist[i]) atomicAdd(&bcount[i], hist[i]);
  }
  int64_t tot;
  tnp::block_scan_excl(aug, lds, tot);
  if (threadIdx.x == 0) tnp::st_agent(part + blockIdx.x, tot);
  if (!fuse || !tnp::last_block(&ctr[CTR_TK0], &last)) return;
  int64_t a = 0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += TNP_BLOCK) a += tnp::ld_agent(part + i);
  int64_t atot;
  tnp::block_scan_excl(a, lds, atot);
  const int64_t T = scan_handed(bcount, NB, bbase, lds);
  if (threadIdx.x == 0) {
    ctr[CTR_A] = atot;
    ctr[CTR_T] = T;
  }
}

// (1') bunny-scale steps: the member passes of a step with few members in
// ONE workgroup -- counts, the bucket scan and the scatter through LDS: no
// global bucket counters, no second launch and no last-workgroup hand-off
// (the two-launch path costs ~19 us per step at bunny scale, most of it
// global-atomic and hand-off latency)
constexpr int SB_THREADS = 1024;
constexpr int SB_IPT = 8;
constexpr int SB_WAVES = SB_THREADS / 64;
constexpr int64_t SB_MAX_M = (int64_t)SB_THREADS * SB_IPT;  // members
constexpr int64_t SB_MAX_LIVE = 1 << 18;                      // live-flag bytes it zeroes
constexpr int SB_PER = (BUCKET_MAX + SB_THREADS - 1) / SB_THREADS;

__device__ __forceinline__ int64_t sb_scan_excl(int64_t v, int64_t* lds, int64_t& total) {
  const int64_t inc = tnp::wave_scan_incl(v);
  if (tnp::lane() == 63) lds[threadIdx.x >> 6] = inc;
  __syncthreads();
  int64_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < SB_WAVES; ++i) {
    const int64_t c = lds[i];
    off += (i < (int)(threadIdx.x >> 6)) ? c : 0;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return off + inc - v;
}

__global__ void __launch_bounds__(SB_THREADS)
k_bucket_small(const int32_t* __restrict__ members, int64_t S, int64_t V, int64_t M,
               const uint64_t* __restrict__ grid, const uint64_t* zero, int idx, BGeom G, int NB,
               int64_t* __restrict__ bbase, uint64_t* __restrict__ ekv, uint8_t* __restrict__ live,
               int64_t nlive, Override ov, int64_t* __restrict__ ctr) {
  extern __shared__ int hist[];  // NB bins
  __shared__ int64_t lds[SB_WAVES];
  const int t = threadIdx.x;
  if (live) {  // the next live-flag set (k_bucket_count's zeroing)
    const int64_t n16 = nlive >> 4;
    uint4* l4 = reinterpret_cast<uint4*>(live);
    for (int64_t i = t; i < n16; i += SB_THREADS) l4[i] = make_uint4(0, 0, 0, 0);
    if (t < (nlive & 15)) live[(n16 << 4) + t] = 0;
  }
  for (int i = t; i < NB; i += SB_THREADS) hist[i] = 0;
  const uint64_t below = (idx >= 64) ? ~0ull : ((1ull << idx) - 1ull);
  int vv[SB_IPT];
  uint64_t gg[SB_IPT], zz[SB_IPT];
#pragma unroll
  for (int k = 0; k < SB_IPT; ++k) {
    const int64_t m = (int64_t)k * SB_THREADS + t;
    vv[k] = m < M ? member_of(members, S, V, m) : -1;
  }
#pragma unroll
  for (int k = 0; k < SB_IPT; ++k) {
    const int v = vv[k] >= 0 ? vv[k] : 0;
    gg[k] = grid[v];
    zz[k] = zero[2 * (int64_t)v];  // (a view of pz: 2 words per vertex)
  }
  if (ov.shared && (ov.flag < 0 ? ctr[CTR_FAIL] != 0 : ov.flag != 0)) {
    // the new vertices' failover override (as k_bucket_count)
    uint64_t sh[SB_IPT], ps[SB_IPT];
#pragma unroll
    for (int k = 0; k < SB_IPT; ++k) {
      const int64_t m = (int64_t)k * SB_THREADS + t;
      const int64_t mc = m < S ? m : 0;
      sh[k] = ov.shared[mc];
      ps[k] = ov.pos[2 * (V + mc)];
    }
#pragma unroll
    for (int k = 0; k < SB_IPT; ++k) {
      const int64_t m = (int64_t)k * SB_THREADS + t;
      if (m >= S) continue;
      for (uint64_t q = sh[k]; q; q &= q - 1) {
        const int p = __builtin_ctzll(q);
        if (p >= ov.keep_from) ov.pre[(int64_t)p * ov.ld + V + m] = 0.f;
      }
      const uint64_t pp = ps[k] & ~sh[k], z = zz[k] | sh[k];
      ov.pz[V + m] = make_ulonglong2(pp, z);
      zz[k] = z;
    }
  }
  __syncthreads();  // hist zeroed
  int64_t aug = 0;
  bool k0 = false, outside = false;
#pragma unroll
  for (int k = 0; k < SB_IPT; ++k) {
    if (vv[k] < 0) continue;
    int lo[3], n[3];
    span_of(gg[k], lo, n);
    if (!span_inside(G, lo, n)) {
      outside = true;
      vv[k] = -1;
      continue;
    }
    for (int i = 0; i < n[0]; ++i)
      for (int j = 0; j < n[1]; ++j)
        for (int q = 0; q < n[2]; ++q) atomicAdd(&hist[bucket_of(G, lo[0] + i, lo[1] + j, lo[2] + q)], 1);
    const int kz = __popcll(zz[k] & below) + (n[0] - 1) + (n[1] - 1) + (n[2] - 1);
    aug += 1ll << kz;
    k0 |= kz == 0;
  }
  if (__ballot(k0) && tnp::lane() == 0) atomicOr((unsigned long long*)&ctr[CTR_K0], 1ull);
  if (__ballot(outside) && tnp::lane() == 0) atomicOr((unsigned long long*)&ctr[CTR_K0], 2ull);
  __syncthreads();  // counts complete
  // bucket bases: a contiguous chunk of bins per thread
  {
    const int b0 = t * SB_PER;
    int c[SB_PER];
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < SB_PER; ++k) {
      c[k] = b0 + k < NB ? hist[b0 + k] : 0;
      s += c[k];
    }
    int64_t T;
    int64_t run = sb_scan_excl(s, lds, T);
#pragma unroll
    for (int k = 0; k < SB_PER; ++k) {
      if (b0 + k < NB) {
        bbase[b0 + k] = run;
        hist[b0 + k] = (int)run;  // cursor
      }
      run += c[k];
    }
    if (t == 0) {
      bbase[NB] = T;
      ctr[CTR_T] = T;
    }
  }
  int64_t atot;
  sb_scan_excl(aug, lds, atot);  // (its barriers also publish the cursors)
  if (t == 0) ctr[CTR_A] = atot;
#pragma unroll
  for (int k = 0; k < SB_IPT; ++k) {
    if (vv[k] < 0) continue;
    int lo[3], n[3];
    span_of(gg[k], lo, n);
    for (int i = 0; i < n[0]; ++i)
      for (int j = 0; j < n[1]; ++j)
        for (int q = 0; q < n[2]; ++q) {
          const int cx = lo[0] + i, cy = lo[1] + j, cz = lo[2] + q;
          const int pos = atomicAdd(&hist[bucket_of(G, cx, cy, cz)], 1);
          const uint32_t f = (uint32_t)(i == 0) | ((uint32_t)(j == 0) << 1) | ((uint32_t)(q == 0) << 2) |
                             ((uint32_t)(n[0] - 1) << 3) | ((uint32_t)(n[1] - 1) << 4) |
                             ((uint32_t)(n[2] - 1) << 5);
          ekv[pos] = ((uint64_t)local_of(G, cx, cy, cz) << 40) | ((uint64_t)f << 32) | (uint32_t)vv[k];
        }
  }
}

// (2) the same scans as a launch of their own, for grids too large for the
// last-workgroup hand-off to pay (every workgroup's tail then waits for its
// stores and a contended ticket): blockIdx.y picks (cnt, out, slot) set y;
// part != null: set 0 also sums the member pass's per-block parts -> pslot
struct ScanSet {
  const void* cnt;
  int wide;  // 1: int64 counts, 0: int32
  int64_t* out;
  int slot;
};
__global__ void __launch_bounds__(TNP_BLOCK)
k_scan_sets(ScanSet s0, ScanSet s1, ScanSet s2, int n, const int64_t* __restrict__ part, int64_t nparts,
            int pslot, int64_t* __restrict__ ctr) {
  __shared__ int64_t lds[TNP_WAVES];
  const ScanSet& q = blockIdx.y == 0 ? s0 : (blockIdx.y == 1 ? s1 : s2);
  const int64_t t = q.wide ? scan_handed(static_cast<const int64_t*>(q.cnt), n, q.out, lds)
                           : scan_handed(static_cast<const int32_t*>(q.cnt), n, q.out, lds);
  if (threadIdx.x == 0) ctr[q.slot] = t;
  if (part && blockIdx.y == 0) {
    int64_t a = 0;
    for (int64_t i = threadIdx.x; i < nparts; i += TNP_BLOCK) a += part[i];
    int64_t atot;
    tnp::block_scan_excl(a, lds, atot);
    if (threadIdx.x == 0) ctr[pslot] = atot;
  }
}

// (3) entries into their bucket ranges: a block reserves one range per
// non-empty bin (one global add), then places its entries inside it
__global__ void __launch_bounds__(TNP_BLOCK)
k_bucket_scatter(const int32_t* __restrict__ members, int64_t S, int64_t V, int64_t M,
                 const uint64_t* __restrict__ grid,
                 BGeom G, int NB, const int64_t* __restrict__ bbase, int32_t* __restrict__ bcur,
                 uint64_t* __restrict__ ekv) {
  extern __shared__ int hist[];  // NB bins, then rel[NB] (dynamic)
  int* const rel = hist + NB;
  for (int i = threadIdx.x; i < NB; i += TNP_BLOCK) hist[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TNP_BLOCK * BK_IPT;
  int vv[BK_IPT];
  uint64_t gg[BK_IPT];
#pragma unroll
  for (int k = 0; k < BK_IPT; ++k) {
    const int64_t m = base + (int64_t)k * TNP_BLOCK + threadIdx.x;
    vv[k] = m < M ? member_of(members, S, V, m) : -1;
  }
#pragma unroll
  for (int k = 0; k < BK_IPT; ++k) gg[k] = grid[vv[k] >= 0 ? vv[k] : 0];
#pragma unroll
  for (int k = 0; k < BK_IPT; ++k) {
    if (vv[k] < 0) continue;
    int lo[3], n[3];
    span_of(gg[k], lo, n);
    if (!span_inside(G, lo, n)) {  // flagged by the count pass
      vv[k] = -1;
      continue;
    }
    for (int i = 0; i < n[0]; ++i)
      for (int j = 0; j < n[1]; ++j)
        for (int q = 0; q < n[2]; ++q) atomicAdd(&hist[bucket_of(G, lo[0] + i, lo[1] + j, lo[2] + q)], 1);
  }
  __syncthreads();
  {
    // one range per non-empty bin; every returning atomic of the thread in
    // flight together (a runtime-bound loop would wait for each in turn)
    constexpr int PB = (BUCKET_MAX + TNP_BLOCK - 1) / TNP_BLOCK;
    int c[PB], r[PB];
#pragma unroll
    for (int k = 0; k < PB; ++k) {
      const int i = k * TNP_BLOCK + threadIdx.x;
      c[k] = i < NB ? hist[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < PB; ++k) r[k] = c[k] ? atomicAdd(&bcur[k * TNP_BLOCK + threadIdx.x], c[k]) : 0;
#pragma unroll
    for (int k = 0; k < PB; ++k) {
      const int i = k * TNP_BLOCK + threadIdx.x;
      if (i < NB) {
        rel[i] = r[k];
        hist[i] = 0;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < BK_IPT; ++k) {
    if (vv[k] < 0) continue;
    int lo[3], n[3];
    span_of(gg[k], lo, n);
    for (int i = 0; i < n[0]; ++i)
      for (int j = 0; j < n[1]; ++j)
        for (int q = 0; q < n[2]; ++q) {
          const int cx = lo[0] + i, cy = lo[1] + j, cz = lo[2] + q;
          const int b = bucket_of(G, cx, cy, cz);
          const int64_t pos = bbase[b] + rel[b] + atomicAdd(&hist[b], 1);
          // cell flags (CellEnt::f): the member's lowest cell along d is
          // this one iff it is the first of its span there
          const uint32_t f = (uint32_t)(i == 0) | ((uint32_t)(j == 0) << 1) | ((uint32_t)(q == 0) << 2) |
                             ((uint32_t)(n[0] - 1) << 3) | ((uint32_t)(n[1] - 1) << 4) |
                             ((uint32_t)(n[2] - 1) << 5);
          ekv[pos] = ((uint64_t)local_of(G, cx, cy, cz) << 40) | ((uint64_t)f << 32) | (uint32_t)vv[k];
        }
  }
}

// (3') sub geometries: each 16^3-cell bucket's entries regrouped by octant
// (8^3 cells), the group buckets 8 b + o.  One workgroup per bucket; each
// wave takes a contiguous quarter of the bucket's entries and walks it twice:
// octant counts (wave ballots, counts in scalar registers), then placement
// at wave-private cursors (the waves' octant counts scanned in LDS) -- no
// atomics.  The order inside an octant is free (as inside a bucket: nothing
// downstream depends on it)
constexpr int RF_U = 8;  // entries per lane in flight
// (1024-thread workgroups, 16 shorter walks per bucket: 7x slower, spilled)
constexpr int RF_THREADS = 256;
constexpr int RF_WAVES = RF_THREADS / 64;
__device__ __forceinline__ int refine_octant(uint64_t w) {
  const uint32_t lc = (uint32_t)(w >> 40);  // 16^3 local cell: x bits 8..11, y 4..7, z 0..3
  return (int)(((lc >> 9) & 4u) | ((lc >> 6) & 2u) | ((lc >> 3) & 1u));
}
__global__ void __launch_bounds__(RF_THREADS)
k_bucket_refine(int NB, const int64_t* __restrict__ bbase, const uint64_t* __restrict__ ekv,
                int64_t* __restrict__ bbase2, uint64_t* __restrict__ ekv2, int32_t* __restrict__ bcount,
                int32_t* __restrict__ bcur) {
  __shared__ int64_t wc[RF_WAVES][8];
  const int b = blockIdx.x, t = threadIdx.x, L = tnp::lane(), wv = tnp::wave();
  const int64_t base = bbase[b], n = bbase[b + 1] - base;
  if (t == 0) {  // the member passes' counters, clean for the next step
    bcount[b] = 0;
    bcur[b] = 0;
    if (b == NB - 1) bbase2[8 * (int64_t)NB] = bbase[NB];
  }
  const int64_t r0 = base + n * wv / RF_WAVES, r1 = base + n * (wv + 1) / RF_WAVES;
  int64_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t e0 = r0; e0 < r1; e0 += 64 * RF_U) {
    uint64_t w[RF_U];
#pragma unroll
    for (int k = 0; k < RF_U; ++k) {
      const int64_t e = e0 + 64 * k + L;
      w[k] = e < r1 ? ekv[e] : ~0ull;
    }
#pragma unroll
    for (int k = 0; k < RF_U; ++k) {
      const int o = w[k] != ~0ull ? refine_octant(w[k]) : 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) c[q] += __popcll(__ballot(o == q));
    }
  }
  if (L == 0)
#pragma unroll
    for (int q = 0; q < 8; ++q) wc[wv][q] = c[q];
  __syncthreads();
  // this wave's cursors: the bucket base, the earlier octants, the earlier
  // waves' share of this octant
  int64_t cur[8];
  {
    int64_t off = base;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int64_t tot = 0, before = 0;
#pragma unroll
      for (int w = 0; w < RF_WAVES; ++w) {
        tot += wc[w][q];
        before += w < wv ? wc[w][q] : 0;
      }
      if (wv == 0 && L == q) bbase2[8 * (int64_t)b + q] = off;
      cur[q] = off + before;
      off += tot;
    }
  }
  for (int64_t e0 = r0; e0 < r1; e0 += 64 * RF_U) {
    uint64_t w[RF_U];
#pragma unroll
    for (int k = 0; k < RF_U; ++k) {
      const int64_t e = e0 + 64 * k + L;
      w[k] = e < r1 ? ekv[e] : ~0ull;
    }
#pragma unroll
    for (int k = 0; k < RF_U; ++k) {
      const bool live = w[k] != ~0ull;
      const int o = live ? refine_octant(w[k]) : 8;
      int64_t pos = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t m = __ballot(o == q);
        if (o == q) pos = cur[q] + tnp::mbcnt(m);
        cur[q] += __popcll(m);
      }
      if (live) {
        const uint32_t lc = (uint32_t)(w[k] >> 40);
        const uint64_t l3 = ((lc >> 2) & 0x1C0u) | ((lc >> 1) & 0x38u) | (lc & 7u);
        ekv2[pos] = (l3 << 40) | (w[k] & 0xFFFFFFFFFFull);
      }
    }
  }
}

// (4) one block per bucket: counting sort by local cell in LDS, records,
// the bucket's pair cells.  Pair-cell lists are written to the bucket's own
// area [bbase / 2, bbase / 2 + n / 2] (a pair cell holds >= 2 entries).
// Entries go through in batches of GIPT per thread, every batch's loads in
// flight together (a bucket can hold 10^5 entries: a block walking them one
// dependent load -> atomic -> store chain at a time is latency-bound).
#ifndef TNP_GIPT
#define TNP_GIPT 8
#endif
constexpr int GIPT = TNP_GIPT;
// SW: the grouping writes the bucket's entry words in cell order (8 B per
// entry) for the LDS-record pass, one dependent gather less than the entry
// indices (4 B)
#ifndef TNP_SORTED_WORDS
#define TNP_SORTED_WORDS 1
#endif
constexpr bool SW = TNP_SORTED_WORDS;

// pair cell o of the global list (cell id, first entry, m members, first
// pair lo) and its chunks in k_connect's chunk table
__device__ __forceinline__ void put_pair_cell(int64_t o, int64_t lo, int32_t cell, int32_t ent, int m,
                                              const PairLists& pl, int64_t* __restrict__ ctr) {
  pl.pcell[o] = cell;
  pl.pent[o] = ent;
  pl.pn[o] = m;
  pl.ptoff[o] = lo;
  // k_connect's chunk table (k_chunk_cells): chunk q starts in pair cell o
  const int64_t n = (int64_t)m * (m - 1) / 2;
  const int64_t b0 = (lo + pl.chunk - 1) / pl.chunk, b1 = (lo + n + pl.chunk - 1) / pl.chunk;
  if (b1 > pl.bcap) atomicOr((unsigned long long*)&ctr[CTR_BOVF], 1ull);
  for (int64_t q = b0; q < b1 && q < pl.bcap; ++q) pl.bcell[q] = (int32_t)o;
}

// the first cell (+2 coordinates) of group bucket b: a member-pass bucket,
// or (sub geometries) octant b & 7 of member-pass bucket b >> 3
__device__ __forceinline__ void group_origin(const BGeom& G, int b, int& ox, int& oy, int& oz) {
  const int B = G.sub ? b >> 3 : b;
  const int bz = B % G.NBz, by = (B / G.NBz) % G.NBy, bx = B / (G.NBy * G.NBz);
  ox = G.xorg + (bx << G.sh);
  oy = G.yorg + (by << G.sh);
  oz = G.zorg + (bz << G.sh);
  if (G.sub) {
    ox += ((b >> 2) & 1) << 3;
    oy += ((b >> 1) & 1) << 3;
    oz += (b & 1) << 3;
  }
}

// the grouping of one bucket of n >= 2 entries (k_bucket_group)
template <int SH>
__device__ __forceinline__ void group_bucket(const BGeom& G, int b, int64_t base, int64_t n,
                                             const uint64_t* __restrict__ ekv,
                                             const ulonglong2* __restrict__ pz, CellEnt* __restrict__ ents,
                                             const PairLists& pl, int64_t* __restrict__ ctr, int* cnt,
                                             int* cur, int64_t* lds, int64_t* lds3, int64_t* s_pk,
                                             int64_t* s_sp, unsigned long long* tph, void* order) {
  (void)tph;
  constexpr int LC = 1 << (3 * SH);
  for (int i = threadIdx.x; i < LC; i += TNP_BLOCK) cnt[i] = 0;
  __syncthreads();
  const uint64_t* kv = ekv + base;
  for (int64_t e0 = 0; e0 < n; e0 += TNP_BLOCK * GIPT) {
    uint64_t w[GIPT];
#pragma unroll
    for (int k = 0; k < GIPT; ++k) {
      const int64_t e = e0 + k * TNP_BLOCK + threadIdx.x;
      w[k] = e < n ? kv[e] : ~0ull;
    }
#pragma unroll
    for (int k = 0; k < GIPT; ++k)
      if (w[k] != ~0ull) atomicAdd(&cnt[(int)(w[k] >> 40)], 1);
  }
  __syncthreads();
  BG_PH(1);
  // exclusive scan of cnt into cur (contiguous chunk per thread)
  constexpr int per = LC / TNP_BLOCK > 0 ? LC / TNP_BLOCK : 1;
  const int c0 = threadIdx.x * per;
  int64_t s = 0;
  for (int i = c0; i < c0 + per && i < LC; ++i) s += cnt[i];
  int64_t tot;
  int64_t run = tnp::block_scan_excl(s, lds, tot);
  for (int i = c0; i < c0 + per && i < LC; ++i) {
    cur[i] = (int)run;
    run += cnt[i];
  }
  __syncthreads();
  BG_PH(2);
  // records, cell-contiguous: the member keys gathered here (the members of
  // one bucket are spatially close: their slots cluster).  perm != null
  // (the LDS-record path): the entries' cell order goes to perm[] instead,
  // records are written only for the cells k_connect takes
  for (int64_t e0 = 0; e0 < n; e0 += TNP_BLOCK * GIPT) {
    uint64_t w[GIPT];
    int pos[GIPT];
    ulonglong2 k2[GIPT];
#pragma unroll
    for (int k = 0; k < GIPT; ++k) {
      const int64_t e = e0 + k * TNP_BLOCK + threadIdx.x;
      w[k] = e < n ? kv[e] : ~0ull;
    }
#pragma unroll
    for (int k = 0; k < GIPT; ++k) {
      pos[k] = w[k] != ~0ull ? atomicAdd(&cur[(int)(w[k] >> 40)], 1) : 0;
      const bool rec = w[k] != ~0ull && (!order || cnt[(int)(w[k] >> 40)] > WCELL);
      k2[k] = pz[rec ? (uint32_t)w[k] : 0u];
    }
#pragma unroll
    for (int k = 0; k < GIPT; ++k) {
      if (w[k] == ~0ull) continue;
      const int lc = (int)(w[k] >> 40);
      if (order) {
        if (SW)
          static_cast<uint64_t*>(order)[pos[k]] = w[k];
        else
          static_cast<int32_t*>(order)[pos[k]] = (int32_t)(e0 + k * TNP_BLOCK + threadIdx.x);
        if (cnt[lc] <= WCELL) continue;
      }
      CellEnt r;
      r.p = k2[k].x;
      r.z = k2[k].y;
      r.v = (int32_t)(uint32_t)w[k];
      r.f = (uint32_t)(w[k] >> 32) & 63u;
      // the cell's tag for the window pass; cells above WCELL members are
      // flagged: the flattened pair-space pass (k_connect) takes them
      r.tag = ((uint32_t)b * (uint32_t)LC + (uint32_t)lc) | (cnt[lc] > WCELL ? 0x80000000u : 0u);
      r.pad = 0;
      ents[base + pos[k]] = r;
    }
  }
  __syncthreads();
  BG_PH(3);
  // pair cells above WCELL members in local-cell order (cur[i] now = end
  // of cell i); the pairs of the smaller cells are the window pass's
  int npc = 0;
  int64_t np = 0, nsp = 0;
  bool big = false;
  for (int i = c0; i < c0 + per && i < LC; ++i) {
    const int m = cnt[i];
    big |= m > 65535;
    if (m > WCELL && m <= 65535) {
      ++npc;
      np += (int64_t)m * (m - 1) / 2;
    } else if (m >= 2 && m <= WCELL) {
      nsp += (int64_t)m * (m - 1) / 2;
    }
  }
  if (__ballot(big) && tnp::lane() == 0) atomicOr((unsigned long long*)&ctr[CTR_BIG], 1ull);
  // the three scans share one barrier pair (lds3: 3 * TNP_WAVES)
  int64_t tpc = 0, tp = 0, tsp = 0;
  int64_t opc = 0, op = 0;
  {
    const int64_t i0 = tnp::wave_scan_incl((int64_t)npc), i1 = tnp::wave_scan_incl(np),
                  i2 = tnp::wave_scan_incl(nsp);
    if (tnp::lane() == 63) {
      lds3[tnp::wave()] = i0;
      lds3[TNP_WAVES + tnp::wave()] = i1;
      lds3[2 * TNP_WAVES + tnp::wave()] = i2;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < TNP_WAVES; ++w) {
      const int64_t c0 = lds3[w], c1 = lds3[TNP_WAVES + w], c2 = lds3[2 * TNP_WAVES + w];
      if (w < tnp::wave()) {
        opc += c0;
        op += c1;
      }
      tpc += c0;
      tp += c1;
      tsp += c2;
    }
    __syncthreads();
    opc += i0 - npc;
    op += i1 - np;
  }
  // the bucket's cells and pairs in the global list: one atomic reserves
  // both (same order), then every thread writes its cells
  if (threadIdx.x == 0) {
    int64_t pk = 0;
    if (tpc) {
      pk = (int64_t)atomicAdd((unsigned long long*)&ctr[CTR_PCK], (unsigned long long)(tp << 24 | tpc));
      if ((pk & (PCK_CELLS - 1)) + tpc >= PCK_CELLS) atomicOr((unsigned long long*)&ctr[CTR_BIG], 1ull);
    }
    *s_pk = pk;
    *s_sp = tsp;  // (reported with the window pass's statistics)
  }
  if (tpc == 0) return;  // (block-uniform)
  __syncthreads();
  const int64_t o0 = (*s_pk & (PCK_CELLS - 1)) + opc, p0 = (*s_pk >> 24) + op;
  opc = 0;
  op = 0;
  constexpr int m_ = (1 << SH) - 1;
  int ox, oy, oz;
  group_origin(G, b, ox, oy, oz);
  for (int i = c0; i < c0 + per && i < LC; ++i) {
    const int m = cnt[i];
    if (m > WCELL && m <= 65535) {
      const int cx = ox + (i >> (2 * SH));
      const int cy = oy + ((i >> SH) & m_);
      const int cz = oz + (i & m_);
      put_pair_cell(o0 + opc, p0 + op, (int32_t)((cx * G.NC + cy) * G.NC + cz), (int32_t)(base + cur[i] - m), m,
                    pl, ctr);
      ++opc;
      op += (int64_t)m * (m - 1) / 2;
    }
  }
}

// Packed windows of one bucket (one wave builds the list): greedy over the
// bucket's cells in local-cell order, a window takes whole consecutive
// cells while they fit in 64 records and none holds more than WCELL members
// (those are k_connect's; they only end windows).  cnt[c] / cur[c]: member
// count and end offset of cell c (group_bucket's LDS); the list (start |
// end << 16, bucket-relative) overwrites cnt[0..nwin) -- a window is
// written only after every count it could overwrite was read.  Returns the
// window count (valid in lane 0).  n must be < 65536.
template <int LC>
__device__ __forceinline__ int build_windows(int* cnt, const int* cur) {
  const int L = tnp::lane();
  int nwin = 0;
  int so = -1;  // start offset of the open window (-1: none)
  for (int c0 = 0; c0 < LC; c0 += 64) {
    const int c = c0 + L;
    const int len = cnt[c], end = cur[c];
    const int start = end - len;
    const bool big = len > WCELL;
    __builtin_amdgcn_wave_barrier();
    int lo = 0;  // first lane of this chunk not yet placed in a window
    while (lo < 64) {
      const uint64_t rest = ~0ull << lo;
      if (so < 0) {
        // open a window at the first non-empty small cell from lane lo
        const uint64_t cand = __ballot(len > 0 && !big) & rest;
        if (!cand) break;
        const int f = __builtin_ctzll(cand);
        so = __shfl(start, f, 64);
        lo = f;
        continue;
      }
      // the window [so, ...) closes before the first cell that does not fit
      // or is big
      const uint64_t stop = __ballot((len > 0) && (big || end > so + 64)) & rest;
      if (!stop) break;  // every remaining cell of the chunk fits: carry on
      const int f = __builtin_ctzll(stop);
      const int eo = __shfl(start, f, 64);  // the window ends where cell f starts
      if (eo > so) {
        if (L == 0) cnt[nwin] = so | (eo << 16);
        ++nwin;
      }
      so = -1;
      lo = __shfl(big ? 1 : 0, f, 64) ? f + 1 : f;  // a big cell is skipped
    }
  }
  if (so >= 0) {
    const int eo = cur[LC - 1];
    if (eo > so) {
      if (L == 0) cnt[nwin] = so | (eo << 16);
      ++nwin;
    }
  }
  return nwin;
}

// build_windows over the cells [c_lo, c_hi) only (one wave's share of the
// bucket, bucket_group's per-wave path): the list goes to cnt[c_lo ...]
// (still written only after every count it could overwrite was read).
// Returns the window count (every lane).
__device__ __forceinline__ int build_windows_range(int* cnt, const int* cur, int c_lo, int c_hi) {
  const int L = tnp::lane();
  int nwin = 0;
  int so = -1;  // start offset of the open window (-1: none)
  for (int c0 = c_lo; c0 < c_hi; c0 += 64) {
    const int c = c0 + L;
    const bool in = c < c_hi;
    const int len = in ? cnt[c] : 0, end = in ? cur[c] : 0;
    const int start = end - len;
    const bool big = len > WCELL;
    __builtin_amdgcn_wave_barrier();
    int lo = 0;  // first lane of this chunk not yet placed in a window
    while (lo < 64) {
      const uint64_t rest = ~0ull << lo;
      if (so < 0) {
        const uint64_t cand = __ballot(len > 0 && !big) & rest;
        if (!cand) break;
        const int f = __builtin_ctzll(cand);
        so = __shfl(start, f, 64);
        lo = f;
        continue;
      }
      const uint64_t stop = __ballot((len > 0) && (big || end > so + 64)) & rest;
      if (!stop) break;
      const int f = __builtin_ctzll(stop);
      const int eo = __shfl(start, f, 64);
      if (eo > so) {
        if (L == 0) cnt[c_lo + nwin] = so | (eo << 16);
        ++nwin;
      }
      so = -1;
      lo = __shfl(big ? 1 : 0, f, 64) ? f + 1 : f;
    }
  }
  if (so >= 0 && c_hi > c_lo) {
    const int eo = cur[c_hi - 1];
    if (eo > so) {
      if (L == 0) cnt[c_lo + nwin] = so | (eo << 16);
      ++nwin;
    }
  }
  __builtin_amdgcn_wave_barrier();
  return nwin;
}

// the first cell whose records start at or after offset `target` (cells in
// local order; starts non-decreasing): a wave's share of the bucket
template <int LC>
__device__ __forceinline__ int first_cell_from(const int* cnt, const int* cur, int target) {
  int lo = 0, hi = LC;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cur[mid] - cnt[mid] >= target) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// A small bucket (2..64 entries, the bunny-scale nets' buckets hold tens):
// ONE wave groups it and tests all its pairs in a single window, with no
// barrier and no trip of the records through memory.  The wave ranks its
// entries by (local cell, lane) with v_readlane (the records land
// cell-contiguous in the window's LDS slot), and every same-cell pair --
// also of a cell above WCELL members, at most 64 * 63 / 2 tests -- is tested
// once by window_tests; the bucket lists no pair cell for k_connect.
#ifndef TNP_SMALL_BUCKET
#define TNP_SMALL_BUCKET 1
#endif
template <int SH>
__device__ __forceinline__ void group_small(int b, int64_t base, int n, const uint64_t* __restrict__ ekv,
                                            const ulonglong2* __restrict__ pz, const WinArgs& wa, uint64_t below,
                                            int64_t* __restrict__ ctr, WinLds& W) {
  constexpr int LC = 1 << (3 * SH);
  const int L = tnp::lane();
  const bool valid = L < n;
  const uint64_t w = valid ? ekv[base + L] : 0ull;
  const ulonglong2 k = pz[valid ? (uint32_t)w : 0u];
  const uint32_t lc = valid ? (uint32_t)(w >> 40) : (uint32_t)LC;  // invalid lanes rank last
  const uint32_t key = (lc << 6) | (uint32_t)L;
  int rank = 0;
  for (int q = 0; q < 64; ++q) rank += (uint32_t)__builtin_amdgcn_readlane((int)key, q) < key;
  CellEnt r;
  r.p = valid ? k.x : 0ull;
  r.z = valid ? k.y : 0ull;
  r.v = valid ? (int32_t)(uint32_t)w : 0;
  r.f = valid ? ((uint32_t)(w >> 32) & 63u) : 0u;
  r.tag = valid ? (uint32_t)b * (uint32_t)LC + lc : 0xFFFFFFFFu;  // invalid: matches nothing
  r.pad = 0;
  const int wv = tnp::wave();
  W.st[wv][rank] = r;
  lds_fence();
  // lane L now takes position L of the window
  const uint32_t tag = W.st[wv][L].tag;
  const uint32_t nxt = __shfl_down(tag, 1, 64);
  const uint64_t bm = __ballot(L == 63 || nxt != tag);
  const int last = L + __builtin_ctzll(bm >> L);
  const uint32_t prv = __shfl_up(tag, 1, 64);
  const bool first = L < n && (L == 0 || prv != tag);
  const int64_t m = first ? (int64_t)(last - L + 1) : 0;  // this cell's members (at its first position)
  const int64_t pairs = tnp::wave_sum(m * (m - 1) / 2);
  WinAcc a;
  window_tests(W.st[wv], L < n ? last - L : 0, below, wa.nb, wa.fmask, wa.keys, wa.cap, wa.xs, ctr, W, a);
  window_flush(wa.keys, wa.cap, wa.xs, ctr, W, a);
  const int64_t c = tnp::wave_sum(a.n_compat), g = tnp::wave_sum(a.n_reg), x = tnp::wave_sum(a.n_conn);
  if (L == 0) bucket_stats_out(wa, b, c, g, x, pairs, ctr);
}

// The same windows built by the whole workgroup (sh = 3).  The greedy
// packing is a chain c0 -> J(c0) -> ... over window-opening cells: a window
// opened at cell c closes before the first non-empty cell after c that is
// big or ends beyond s_c + 64 (a binary search over the cells' end
// offsets), and the next one opens there (after a big cell: at the next
// non-empty cell of <= WCELL members).  With every cell's J known, the
// chain is enumerated by pointer doubling (J^(2^k) tables) -- the serial
// walk of one wave (build_windows) was ~26 % of the grouping kernel's
// workgroup time at 128^3.  Bit for bit the windows of build_windows.
// scratch: (NJ + 3) * (LC + 1) uint16 + 8 int of LDS not otherwise in use.
#ifndef TNP_PAR_WIN
#define TNP_PAR_WIN 1
#endif
constexpr int PW_NJ = 10;  // J^(2^k), k < PW_NJ: chains of up to 1024 windows
// below this many entries the serial walk is shorter than the builder's
// fixed ~40 barrier-separated steps (bunny-scale buckets hold ~100)
constexpr int PW_MIN = 512;
template <int LC>
__device__ __forceinline__ int build_windows_par(int* cnt, const int* cur, uint16_t* scratch) {
  static_assert(LC + 1 <= 65535 && LC <= (1 << PW_NJ), "cell indices in 16 bits, chains in the tables");
  constexpr int W1 = LC + 1;  // cell index LC: none
  uint16_t* opn = scratch;    // first non-empty cell of <= WCELL members at or after c
  uint16_t* nbg = opn + W1;   // first big cell at or after c
  uint16_t* wend = nbg + W1;  // end offset of the window opened at c
  uint16_t* J = wend + W1;    // J[k * W1 + c] = J^(2^k)(c)
  int* red = reinterpret_cast<int*>(J + PW_NJ * W1 + (PW_NJ * W1 + 3 * W1) % 2);  // 8 ints
  const int t = threadIdx.x, L = tnp::lane(), wv = tnp::wave();
  constexpr int per = LC / TNP_BLOCK > 0 ? LC / TNP_BLOCK : 1;
  const int c0 = t * per;
  // (1) suffix minima: per-thread chunk, then over the lanes, then the waves
  int mo = LC, mb = LC;
  for (int i = c0 + per - 1; i >= c0; --i) {
    if (i >= LC) continue;
    const int m = cnt[i];
    if (m > 0 && m <= WCELL) mo = i;
    if (m > WCELL) mb = i;
  }
  int so = mo, sb = mb;  // minima over lanes >= L of this wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int a = __shfl_down(so, d, 64), b = __shfl_down(sb, d, 64);
    if (L + d < 64) {
      so = min(so, a);
      sb = min(sb, b);
    }
  }
  if (L == 0) {
    red[wv] = so;
    red[TNP_WAVES + wv] = sb;
  }
  __syncthreads();
  // carry: the minima of the chunks after this thread's
  int co = __shfl_down(so, 1, 64), cb = __shfl_down(sb, 1, 64);
  if (L == 63) co = cb = LC;
  for (int w = wv + 1; w < TNP_WAVES; ++w) {
    co = min(co, red[w]);
    cb = min(cb, red[TNP_WAVES + w]);
  }
  for (int i = c0 + per - 1; i >= c0; --i) {
    if (i >= LC) continue;
    const int m = cnt[i];
    if (m > 0 && m <= WCELL) co = i;
    if (m > WCELL) cb = i;
    opn[i] = (uint16_t)co;
    nbg[i] = (uint16_t)cb;
  }
  if (t == 0) {
    opn[LC] = LC;
    nbg[LC] = LC;
  }
  __syncthreads();
  // (2) J and the window end of every window-opening cell
  const int total = cur[LC - 1];
  for (int i = c0; i < c0 + per && i < LC; ++i) {
    const int m = cnt[i];
    int j = LC, e = total;
    if (m > 0 && m <= WCELL) {
      const int lim = cur[i] - m + 64;  // the window [s, s + 64)
      int lo = i + 1, hi = LC;  // first cell after i ending beyond it (ends never decrease)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cur[mid] > lim) hi = mid;
        else lo = mid + 1;
      }
      const int stop = min(lo, (int)nbg[i + 1]);
      if (stop < LC) {
        e = cur[stop] - cnt[stop];  // the window ends where the stopping cell starts
        j = cnt[stop] > WCELL ? opn[stop + 1] : stop;
      }
    }
    J[i] = (uint16_t)j;
    wend[i] = (uint16_t)e;
  }
  if (t == 0) J[LC] = LC;
  __syncthreads();
  for (int k = 1; k < PW_NJ; ++k) {
    const uint16_t* A = J + (k - 1) * W1;
    uint16_t* B = J + k * W1;
    for (int i = t; i < W1; i += TNP_BLOCK) B[i] = A[A[i]];
    __syncthreads();
  }
  // (3) window w opens at J^w(opn[0])
  const int first = opn[0];
  constexpr int NR = (1 << PW_NJ) / TNP_BLOCK;
  uint32_t ent[NR];
  int n = 0;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int w = t + r * TNP_BLOCK;
    int c = first;
#pragma unroll
    for (int k = 0; k < PW_NJ; ++k)
      if (((w >> k) & 1) && c < LC) c = J[k * W1 + c];
    ent[r] = c < LC ? ((uint32_t)(cur[c] - cnt[c]) | ((uint32_t)wend[c] << 16)) : 0xFFFFFFFFu;
    if (c < LC) n = w + 1;
  }
  // (windows are a prefix of w: the count is the largest valid w + 1)
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) n = max(n, __shfl_xor(n, d, 64));
  __syncthreads();  // every read of cnt[] is done: the list overwrites it
  if (L == 0) red[wv] = n;
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (ent[r] != 0xFFFFFFFFu) cnt[t + r * TNP_BLOCK] = (int)ent[r];
  __syncthreads();
  int nw = 0;
  for (int w = 0; w < TNP_WAVES; ++w) nw = max(nw, red[w]);
  return nw;
}

// 8^3-cell buckets: 5 workgroups per CU (LDS allows 5; the LDS-record
// path's pipeline registers would otherwise cost one: 105 VGPRs -> 4 waves
// per SIMD, bucket_group 0.92 vs 1.04 ms per 128^3 pass at 5)
#ifndef TNP_BG_MINB
#define TNP_BG_MINB 5
#endif
#ifndef TNP_PACKED_WIN  // 0: the 32-stride window pass (A/B variant)
#define TNP_PACKED_WIN 1
#endif
// LDS-record path (pl.perm != null): a bucket's records never go through
// memory -- its cell order goes to pl.perm (4 B per entry), chunks of
// TNP_LREC_CH record positions (+ 64 for the windows that start near a
// chunk's end) are gathered into LDS (over the window stage and behind it)
// and the windows starting in the chunk are tested there.  Only the cells
// above WCELL members (k_connect's) get records in memory.
#ifndef TNP_BG_WAVEWIN  // 1: per-wave windows (no workgroup barriers in the pass); 0: shared chunks
#define TNP_BG_WAVEWIN 1
#endif
#ifndef TNP_BG_LDS_MIN  // buckets above this many entries skip the records in memory
#define TNP_BG_LDS_MIN LREC_N
#endif
#ifndef TNP_LREC_CH
#define TNP_LREC_CH 192  // (256 records: the window stage's own LDS, occupancy unchanged)
#endif
constexpr int LREC_N = TNP_LREC_CH + 64;
constexpr size_t WL_ST = offsetof(WinLds, st);
constexpr size_t WL_RAW = WL_ST + (sizeof(WinLds) - WL_ST > LREC_N * sizeof(CellEnt) ? sizeof(WinLds) - WL_ST
                                                                                     : LREC_N * sizeof(CellEnt));
constexpr int LREC_R = (LREC_N + TNP_BLOCK - 1) / TNP_BLOCK;  // records per thread per chunk

// PK: packed records (steps with packed_ok)
template <int SH, bool PK>
__global__ void __launch_bounds__(TNP_BLOCK, SH == 3 ? TNP_BG_MINB : 1)
k_bucket_group(BGeom G, const int64_t* __restrict__ bbase, const uint64_t* __restrict__ ekv,
               const ulonglong2* __restrict__ pz, CellEnt* __restrict__ ents, WinArgs wa, PairLists pl,
               int64_t* __restrict__ ctr) {
  constexpr int LC = 1 << (3 * SH);
  __shared__ int cnt[LC];
  __shared__ int cur[LC];
  __shared__ int64_t lds[TNP_WAVES];
  __shared__ int64_t lds3[3 * TNP_WAVES];
  __shared__ int64_t s_pk, s_sp;
  __shared__ int nwin_s;
  constexpr bool LREC = TNP_PACKED_WIN;
  __shared__ __attribute__((aligned(32))) unsigned char wraw[LREC ? WL_RAW : sizeof(WinLds)];
  WinLds& W = *reinterpret_cast<WinLds*>(wraw);
  CellEnt* const lrec = reinterpret_cast<CellEnt*>(wraw + WL_ST);
  const int b = blockIdx.x;
  const int64_t base = bbase[b];
  const int64_t n = bbase[b + 1] - base;
  if (threadIdx.x == 0 && !G.sub) {  // the bucket counters are clean for the next step (read by the member
    pl.bcount[b] = 0;                 // passes; sub geometries: the refine pass zeroes them)
    pl.bcur[b] = 0;
  }
  if (n < 2) {
    if (threadIdx.x == 0 && wa.bstat) bucket_stats_out(wa, b, 0, 0, 0, 0, ctr);
    if (n == 1 && threadIdx.x == 0) {  // a lone entry: a record the window pass can read
      const uint64_t w = ekv[base];
      const ulonglong2 k = pz[(uint32_t)w];
      CellEnt r;
      r.p = k.x;
      r.z = k.y;
      r.v = (int32_t)(uint32_t)w;
      r.f = (uint32_t)(w >> 32) & 63u;
      r.tag = (uint32_t)b * (uint32_t)LC + (uint32_t)(w >> 40);
      r.pad = 0;
      ents[base] = r;
    }
  } else if (TNP_SMALL_BUCKET && wa.keys && n <= 64) {
    if (tnp::wave() == 0) {
      const uint64_t below = (wa.idx >= 64) ? ~0ull : ((1ull << wa.idx) - 1ull);
      group_small<SH>(b, base, (int)n, ekv, pz, wa, below, ctr, W);
    }
  } else {
    unsigned long long tph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    BG_PH(0);
    // (a bucket of one chunk gains nothing from it: bunny-scale buckets)
    const bool in_lds = LREC && wa.keys && pl.perm && n > TNP_BG_LDS_MIN && n < 65536;
    void* const order = !in_lds ? nullptr
                                : SW ? static_cast<void*>(reinterpret_cast<uint64_t*>(pl.perm) + base)
                                     : static_cast<void*>(pl.perm + base);
    group_bucket<SH>(G, b, base, n, ekv, pz, ents, pl, ctr, cnt, cur, lds, lds3, &s_pk, &s_sp, tph, order);
    BG_PH(4);
    if (wa.keys) {
      // the window pass over this bucket's records, right behind their
      // stores (the workgroup's own stores: visible after the barrier)
      __syncthreads();
      WinAcc a;
      const uint64_t below = (wa.idx >= 64) ? ~0ull : ((1ull << wa.idx) - 1ull);
      const bool wave_lists = in_lds && SW && TNP_BG_WAVEWIN;
      if (wave_lists) {
        // each wave takes the cells whose records start in its quarter of the
        // bucket, packs them into windows of whole cells itself (the serial
        // walk of build_windows over a quarter of the cells) and walks its
        // windows through a private 64-record stage in LDS: no workgroup
        // barrier from the grouping to the statistics.  A window's records
        // are built from the bucket's entry words in cell order and the
        // member keys, software-pipelined (the keys of the next window and the
        // words of the one after are in flight while a window is tested).
        // Round 4 built one list for the bucket (the whole workgroup,
        // pointer doubling) and tested it in shared chunks, each waiting for
        // its slowest window.
        const uint64_t* sw = static_cast<const uint64_t*>(order);
        const int L = tnp::lane(), wv = tnp::wave();
        const int nn = (int)n;
        const int c_lo = wv == 0 ? 0 : first_cell_from<LC>(cnt, cur, (int)((int64_t)nn * wv / TNP_WAVES));
        const int c_hi = wv == TNP_WAVES - 1 ? LC
                                             : first_cell_from<LC>(cnt, cur, (int)((int64_t)nn * (wv + 1) / TNP_WAVES));
        // (every wave has read the cells it bounds by before any list is written)
        __syncthreads();
        const int nw = uniform(build_windows_range(cnt, cur, c_lo, c_hi));
        BG_PH(5);
        const uint32_t* wl = reinterpret_cast<const uint32_t*>(cnt) + c_lo;
        auto span = [&](int k, int& s, int& m) {
          if (k >= nw) { s = 0; m = 0; return; }
          const uint32_t se = (uint32_t)uniform((int)wl[k]);
          s = (int)(se & 0xFFFFu);
          m = (int)(se >> 16) - s;
        };
        int s0, m0, s1, m1;
        span(0, s0, m0);
        span(1, s1, m1);
        uint64_t w0 = L < m0 ? sw[s0 + L] : 0ull;
        uint64_t w1 = L < m1 ? sw[s1 + L] : 0ull;
        ulonglong2 k0 = L < m0 ? pz[(uint32_t)w0] : make_ulonglong2(0ull, 0ull);
        // this wave's packed stage (64 records), laid over its W.st slots
        uint64_t* const ptw = reinterpret_cast<uint64_t*>(&W.st[wv][0]);
        uint64_t* const paw = ptw + 64;
        uint32_t* const pvv = reinterpret_cast<uint32_t*>(paw + 64);
        static_assert(64 * (8 + 8 + 4) <= sizeof(W.st[0]), "a wave's packed stage fits its record slots");
        const PackedRecs PR{ptw, paw, pvv, nullptr};
        uint64_t amask = 0;
        if (PK && wa.fmask) {
          const uint64_t lo = (uint32_t)(wa.fmask >> wa.idx);
          amask = lo | (lo << 32);
        }
        for (int k = 0; k < nw; ++k) {
          // in flight behind this window: the keys of the next, the words of the one after
          int s2, m2;
          span(k + 2, s2, m2);
          const ulonglong2 k1 = L < m1 ? pz[(uint32_t)w1] : make_ulonglong2(0ull, 0ull);
          const uint64_t w2 = L < m2 ? sw[s2 + L] : 0ull;
          const bool valid = L < m0;
          uint32_t tag;
          if constexpr (PK) {
            if (valid) {
              ptw[L] = packed_test_word(k0.x, k0.y, (uint32_t)(w0 >> 32) & 63u, below);
              paw[L] = packed_above_word(k0.x, k0.y, wa.idx);
              pvv[L] = (uint32_t)w0;
            }
            tag = valid ? (uint32_t)(w0 >> 40) : 0xFFFFFFFFu;
          } else {
            CellEnt e;
            e.p = k0.x;
            e.z = k0.y;
            e.v = (int32_t)(uint32_t)w0;
            e.f = (uint32_t)(w0 >> 32) & 63u;
            e.tag = valid ? (uint32_t)b * (uint32_t)LC + (uint32_t)(w0 >> 40) : 0xFFFFFFFFu;
            e.pad = 0;
            if (valid) W.st[wv][L] = e;
            tag = e.tag;
          }
          lds_fence();
          // last lane of my cell in the window (the window holds whole cells)
          const uint32_t nxt = __shfl_down(tag, 1, 64);
          const uint64_t bm = __ballot(L >= m0 - 1 || nxt != tag);
          const int last = L + __builtin_ctzll(bm >> L);
          const int rounds = valid ? last - L : 0;
          if constexpr (PK)
            window_tests_packed(PR, 0, rounds, (uint32_t)below, wa.nb, amask, wa.keys, wa.cap, wa.xs, ctr, W, a);
          else
            window_tests(W.st[wv], rounds, below, wa.nb, wa.fmask, wa.keys, wa.cap, wa.xs, ctr, W, a);
          w0 = w1;
          k0 = k1;
          m0 = m1;
          w1 = w2;
          m1 = m2;
        }
      } else if (TNP_PACKED_WIN && n < 65536) {
        // packed windows of whole cells (the list overwrites cnt[]): built by
        // the whole workgroup for 8^3-cell buckets (their scratch fits the
        // window pass's LDS, unused until the pass), by wave 0 for 16^3
        bool par = false;
        if constexpr (TNP_PAR_WIN && LC == 512) {
          static_assert(sizeof(WinLds) >= (PW_NJ + 3) * (LC + 1) * sizeof(uint16_t) + 12 * sizeof(int),
                        "window-builder scratch");
          par = n >= PW_MIN;
          if (par) {
            const int nw = build_windows_par<LC>(cnt, cur, reinterpret_cast<uint16_t*>(&W));
            if (threadIdx.x == 0) nwin_s = nw;
          }
        }
        if (!par && tnp::wave() == 0) {
          const int nw = build_windows<LC>(cnt, cur);
          if (tnp::lane() == 0) nwin_s = nw;
        }
        __syncthreads();
        BG_PH(5);
        if (in_lds) {
          // chunks of TNP_LREC_CH record positions gathered into LDS, then the
          // windows that start there tested.  Software-pipelined: SW (the
          // bucket's entry words written in cell order by the grouping): the
          // words of chunk j + 2 and the member keys of chunk j + 1 are in
          // flight while chunk j is tested; else (cell order as entry
          // indices) the order of j + 3, the words of j + 2, the keys of j + 1
          const uint64_t* kv = ekv + base;
          const int nn = (int)n;
          constexpr int CH = TNP_LREC_CH;
          int kw = tnp::wave();  // this wave's next window (windows kw, kw + TNP_WAVES, ...)
          int ia[LREC_R], ib[LREC_R];
          uint64_t wa0[LREC_R], wb[LREC_R];
          ulonglong2 ka[LREC_R], kb[LREC_R];
          auto in_chunk = [&](int q0, int r) {
            const int q = q0 + r * TNP_BLOCK + threadIdx.x;
            return q < q0 + LREC_N && q < nn;
          };
          auto load_i = [&](int q0, int (&ix)[LREC_R]) {
            const int32_t* perm = static_cast<const int32_t*>(order);
#pragma unroll
            for (int r = 0; r < LREC_R; ++r) ix[r] = in_chunk(q0, r) ? perm[q0 + r * TNP_BLOCK + threadIdx.x] : -1;
          };
          auto load_w = [&](const int (&ix)[LREC_R], uint64_t (&w)[LREC_R]) {
#pragma unroll
            for (int r = 0; r < LREC_R; ++r) w[r] = ix[r] >= 0 ? kv[ix[r]] : 0ull;
          };
          auto load_sw = [&](int q0, uint64_t (&w)[LREC_R]) {
            const uint64_t* sw = static_cast<const uint64_t*>(order);
#pragma unroll
            for (int r = 0; r < LREC_R; ++r) w[r] = in_chunk(q0, r) ? sw[q0 + r * TNP_BLOCK + threadIdx.x] : 0ull;
          };
          auto load_k = [&](const uint64_t (&w)[LREC_R], ulonglong2 (&k)[LREC_R]) {
#pragma unroll
            for (int r = 0; r < LREC_R; ++r) k[r] = pz[(uint32_t)w[r]];
          };
          if constexpr (SW) {
            load_sw(0, wa0);
            load_k(wa0, ka);
            if (CH < nn) load_sw(CH, wb);
          } else {
            load_i(0, ia);
            load_w(ia, wa0);
            load_k(wa0, ka);
            if (CH < nn) {
              load_i(CH, ia);
              load_w(ia, wb);
            }
            if (2 * CH < nn) load_i(2 * CH, ib);
          }
          // packed records (PK: steps with packed_ok): SoA over the same LDS
          uint64_t* const ptw = reinterpret_cast<uint64_t*>(wraw + WL_ST);
          uint64_t* const paw = ptw + LREC_N;
          uint32_t* const pvv = reinterpret_cast<uint32_t*>(paw + LREC_N);
          uint16_t* const ptg = reinterpret_cast<uint16_t*>(pvv + LREC_N);
          static_assert(LREC_N * (8 + 8 + 4 + 2) <= WL_RAW - WL_ST, "packed records fit the record chunk");
          const PackedRecs PR{ptw, paw, pvv, ptg};
          uint64_t amask = 0;
          if (PK && wa.fmask) {
            const uint64_t lo = (uint32_t)(wa.fmask >> wa.idx);
            amask = lo | (lo << 32);
          }
          for (int p0 = 0; p0 < nn; p0 += CH) {
            const int p1 = min(nn, p0 + LREC_N);
#pragma unroll
            for (int r = 0; r < LREC_R; ++r) {
              const int q = p0 + r * TNP_BLOCK + threadIdx.x;
              if (q >= p1) continue;
              if constexpr (PK) {
                ptw[q - p0] = packed_test_word(ka[r].x, ka[r].y, (uint32_t)(wa0[r] >> 32) & 63u, below);
                paw[q - p0] = packed_above_word(ka[r].x, ka[r].y, wa.idx);
                pvv[q - p0] = (uint32_t)wa0[r];
                ptg[q - p0] = (uint16_t)(wa0[r] >> 40);
              } else {
                CellEnt e;
                e.p = ka[r].x;
                e.z = ka[r].y;
                e.v = (int32_t)(uint32_t)wa0[r];
                e.f = (uint32_t)(wa0[r] >> 32) & 63u;
                e.tag = (uint32_t)b * (uint32_t)LC + (uint32_t)(wa0[r] >> 40);
                e.pad = 0;
                lrec[q - p0] = e;
              }
            }
            __syncthreads();
            uint64_t wc[LREC_R];
            if (p0 + CH < nn) load_k(wb, kb);
            if constexpr (SW) {
              if (p0 + 2 * CH < nn) load_sw(p0 + 2 * CH, wc);
            } else {
              if (p0 + 2 * CH < nn) load_w(ib, wc);
              if (p0 + 3 * CH < nn) load_i(p0 + 3 * CH, ib);
            }
            if constexpr (PK)
              window_pass_packed_lds(PR, p0, p0 + CH, reinterpret_cast<const uint32_t*>(cnt), nwin_s, &kw,
                                     TNP_WAVES, (uint32_t)below, wa.nb, amask, wa.keys, wa.cap, wa.xs, ctr, W, a);
            else
              window_pass_lds(lrec, p0, p0 + CH, reinterpret_cast<const uint32_t*>(cnt), nwin_s, &kw, TNP_WAVES,
                              below, wa.nb, wa.fmask, wa.keys, wa.cap, wa.xs, ctr, W, a);
            __syncthreads();  // (the next chunk overwrites the records)
#pragma unroll
            for (int r = 0; r < LREC_R; ++r) {
              wa0[r] = wb[r];
              ka[r] = kb[r];
              wb[r] = wc[r];
            }
          }
        } else {
          window_pass_packed(ents, base, reinterpret_cast<const uint32_t*>(cnt), nwin_s, tnp::wave(), TNP_WAVES,
                             below, wa.nb, wa.fmask, wa.keys, wa.cap, wa.xs, ctr, W, a);
        }
      } else {
        window_pass(ents, base, base + n, tnp::wave(), TNP_WAVES, below, wa.nb, wa.fmask, wa.keys, wa.cap,
                    wa.xs, ctr, W, a);
      }
      BG_PH(6);
      fold_wave_counts(a);
      window_flush(wa.keys, wa.cap, wa.xs, ctr, W, a);
      int64_t tc, tr, tx;
      tnp::block_scan_excl(a.n_compat, lds, tc);
      tnp::block_scan_excl(a.n_reg, lds, tr);
      tnp::block_scan_excl(a.n_conn, lds, tx);
      if (threadIdx.x == 0) bucket_stats_out(wa, b, tc, tr, tx, s_sp, ctr);
      BG_PH(7);
    }
#if TNP_BG_PHASES
    if (threadIdx.x == 0)
      for (int k = 0; k < 7; ++k)
        if (tph[k + 1] > tph[k] && tph[k])
          atomicAdd(&g_bg_ph[k * 8 + (blockIdx.x & 7)], tph[k + 1] - tph[k]);
#endif
  }
}

}  // namespace

int bucket_geometry(int n_marks, const int lo[3], const int hi[3], BucketGeom* g) {
  const int NC = n_marks + 2;
  // cells of a complex inside the mark planes [lo, hi] of an axis: offsets
  // lo - 1 (a vertex within eps of plane lo spans the cell below) to hi,
  // i.e. cell coordinates lo + 1 .. hi + 2; one more on each side
  int clo[3], cn[3];
  for (int d = 0; d < 3; ++d) {
    clo[d] = std::max(0, lo[d]);
    cn[d] = std::min(NC - 1, hi[d] + 3) - clo[d] + 1;
  }
  static const int s_env = [] {  // TNP_BUCKET_SH=3|4: force the bucket edge (experiments)
    const char* v = getenv("TNP_BUCKET_SH");
    return v ? atoi(v) : 0;
  }();
  static const int s_sub = [] {  // TNP_BUCKET_SUB=0: never two-level, 1: always (experiments)
    const char* v = getenv("TNP_BUCKET_SUB");
    return v ? atoi(v) : -1;
  }();
  for (int s = (s_env == 4 || s_sub == 1 ? 4 : 3); s <= 4; ++s) {
    int nbs[3];
    for (int d = 0; d < 3; ++d) nbs[d] = (cn[d] + (1 << s) - 1) >> s;
    const int64_t nb = (int64_t)nbs[0] * nbs[1] * nbs[2];
    if (nb > BUCKET_MAX) continue;
    // 16^3-cell member buckets are refined into 8^3-cell group buckets
    // unless TNP_BUCKET_SH=4 asks for the 16^3-cell grouping kernel
    const int sub = s == 4 && s_env != 4 && s_sub != 0;
    *g = BucketGeom{NC,          s,           nbs[0],      nbs[1],   nbs[2],   clo[0],
                    clo[1],      clo[2],      nbs[0] << s, nbs[1] << s, nbs[2] << s, (int)nb,
                    sub,         sub ? 8 * (int)nb : (int)nb};
    return 0;
  }
  return -1;
}

int64_t bucket_member_blocks(int64_t M) {
  const int64_t per = (int64_t)TNP_BLOCK * BK_IPT;
  return std::max<int64_t>((M + per - 1) / per, 1);
}
int launch_bucket_entries(const int32_t* members, int64_t S, int64_t V, int64_t M, const uint64_t* keys,
                          const uint64_t* zero, int idx, const BucketGeom& G, int32_t* bcount, int32_t* bcur,
                          int64_t* bbase, int64_t* part, uint64_t* ekv, bool clean, uint8_t* live,
                          int64_t nlive, const NewOverride* ovr, int64_t* ctr, hipStream_t s) {
  const int NB = G.NB;
  Override ov{0, nullptr, nullptr, 0, 0, nullptr, nullptr, nullptr};
  if (ovr)
    ov = Override{ovr->flag, ovr->shared, ovr->pre, ovr->ld, ovr->keep_from, ovr->pos, ovr->zero,
                  reinterpret_cast<ulonglong2*>(ovr->pz)};
  static const bool s_small = [] {  // TNP_SMALL_ENTRIES=0: always the two-launch path (A/B)
    const char* v = getenv("TNP_SMALL_ENTRIES");
    return !(v && v[0] == '0');
  }();
  if (s_small && M <= SB_MAX_M && (!live || nlive <= SB_MAX_LIVE)) {
    // bcount / bcur stay untouched (the grouping kernel zeroes them anyway)
    hipLaunchKernelGGL(k_bucket_small, dim3(1), dim3(SB_THREADS), NB * sizeof(int), s, members, S, V, M, keys, zero,
                       idx, G, NB, bbase, ekv, live, nlive, ov, ctr);
    TNP_CHECK(hipGetLastError());
    return 0;
  }
  if (!clean) {  // else: zeroed by the previous step's grouping kernel
    TNP_CHECK(hipMemsetAsync(bcount, 0, NB * sizeof(int32_t), s));
    TNP_CHECK(hipMemsetAsync(bcur, 0, NB * sizeof(int32_t), s));
  }
  const unsigned nblk = (unsigned)bucket_member_blocks(M);
  // the live-flag zeroing rides along: a step with few members still gets
  // enough workgroups for it (64 B per thread; the extra ones count nothing)
  unsigned grid = nblk;
  if (live) {
    const int64_t nz = ((nlive >> 4) + 4 * TNP_BLOCK - 1) / (4 * TNP_BLOCK);
    grid = std::max<unsigned>(nblk, (unsigned)std::min<int64_t>(nz, FUSE_MAX_BLOCKS));
  }
  const int fuse = grid <= FUSE_MAX_BLOCKS;
  hipLaunchKernelGGL(k_bucket_count, dim3(grid), dim3(TNP_BLOCK), NB * sizeof(int), s, members, S, V, M, keys, zero, idx,
                     G, NB, bcount, part, bbase, live, nlive, fuse, ov, ctr);
  if (!fuse)
    hipLaunchKernelGGL(k_scan_sets, dim3(1, 1), dim3(TNP_BLOCK), 0, s, ScanSet{bcount, 0, bbase, CTR_T},
                       ScanSet{}, ScanSet{}, NB, part, (int64_t)grid, (int)CTR_A, ctr);
  if (M > 0)
    hipLaunchKernelGGL(k_bucket_scatter, dim3(nblk), dim3(TNP_BLOCK), 2 * NB * sizeof(int), s, members, S, V, M, keys, G, NB,
                       bbase, bcur, ekv);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_bucket_refine(const BucketGeom& G, const int64_t* bbase, const uint64_t* ekv, int64_t* bbase2,
                         uint64_t* ekv2, int32_t* bcount, int32_t* bcur, hipStream_t s) {
  if (!G.sub || G.sh != 4) {
    tnp_set_error("bucket refine: not a two-level geometry");
    return -1;
  }
  hipLaunchKernelGGL(k_bucket_refine, dim3(G.NB), dim3(RF_THREADS), 0, s, G.NB, bbase, ekv, bbase2, ekv2, bcount,
                     bcur);
  TNP_CHECK(hipGetLastError());
  return 0;
}

int launch_bucket_pairs(const BucketGeom& G, const int64_t* bbase, const uint64_t* ekv, const uint64_t* pz,
                        CellEnt* ents, int32_t* pcell, int32_t* pent, int32_t* pn, int64_t* ptoff, int32_t* bcell,
                        int64_t bcap, int32_t* bcount, int32_t* bcur, const ConnectWin* win, int64_t* ctr,
                        hipStream_t s, int32_t* perm) {
  const int NB = G.NG, sh = G.sub ? 3 : G.sh;
  const PairLists pl{pcell, pent, pn, ptoff, bcell, bcap, connect_chunk_pairs(), bcount, bcur, perm};
  WinArgs wa{0, 0, 0ull, nullptr, 0, nullptr, nullptr, 0};
  if (win) wa = WinArgs{win->idx, win->nb, win->fmask, win->keys, win->cap, win->xs, win->bstat, win->packed};
  const ulonglong2* pz2 = reinterpret_cast<const ulonglong2*>(pz);
  if (sh == 3 && wa.packed)
    hipLaunchKernelGGL((k_bucket_group<3, true>), dim3(NB), dim3(TNP_BLOCK), 0, s, G, bbase, ekv, pz2, ents, wa, pl,
                       ctr);
  else if (sh == 3)
    hipLaunchKernelGGL((k_bucket_group<3, false>), dim3(NB), dim3(TNP_BLOCK), 0, s, G, bbase, ekv, pz2, ents, wa,
                       pl, ctr);
  else
    hipLaunchKernelGGL((k_bucket_group<4, false>), dim3(NB), dim3(TNP_BLOCK), 0, s, G, bbase, ekv, pz2, ents, wa,
                       pl, ctr);
#if TNP_BG_PHASES
  {
    unsigned long long h[64];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bg_ph), sizeof(h));
    unsigned long long t[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 7; ++k)
      for (int x = 0; x < 8; ++x) t[k] += h[k * 8 + x];
    fprintf(stderr, "bg_phases count %llu scan %llu records %llu paircells %llu windows %llu pass %llu flush %llu\n",
            t[0], t[1], t[2], t[3], t[4], t[5], t[6]);
    for (auto& v : h) v = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bg_ph), h, sizeof(h));
  }
#endif
  TNP_CHECK(hipGetLastError());
  return 0;
}
