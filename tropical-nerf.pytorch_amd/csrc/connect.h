// Connecting-edge pair test and the window pass over cell-contiguous entry
// records (subpoly.py:484-535), shared by step.hip (k_connect, k_connect_win)
// and bucket.hip (the grouping kernel runs the window pass over its own
// bucket).
#pragma once
#include "common.h"
#include "step.h"

namespace {

// ---------------------------------------------------------------------------
// connecting-edge pair test (subpoly.py:484-535 in closed form).
// Two members share an augmented region iff, per coordinate, their augmented
// value sets intersect: grid dim d -> their cell spans overlap; plane
// j < idx -> not (both non-zero with opposite signs).  The reference keeps
// the pair iff they share >= 1 zero plane (grid zeros only on the SAME mark
// plane).  Each pair is emitted once, in the canonical cell (per-dim max of
// the two span lows).  In terms of the entries' cell flags (CellEnt::f) for
// the cell under test, which both spans contain:
//   canonical       <=> per axis, one of the two spans starts here
//   same mark plane <=> both on a plane of the axis and both spans start here
// and the shared regions double per same-plane axis and per common zero plane.
// ---------------------------------------------------------------------------
struct PairTest {
  bool emit;
  bool compat;
  int64_t regions;  // shared regions (for the reference's candidate count P)
};

__device__ __forceinline__ PairTest pair_test(uint64_t below, uint32_t fu, uint64_t pu, uint64_t zu,
                                              uint32_t fv, uint64_t pv, uint64_t zv) {
  PairTest t{false, false, 0};
  if (((fu | fv) & 7u) != 7u) return t;  // not the canonical cell
  if (((pu ^ pv) & ~zu & ~zv & below) != 0) return t;
  const uint32_t a = fu & fv;
  const uint32_t sp = a & (a >> 3) & 7u;  // axes where both lie on the same mark plane
  const uint64_t zz = zu & zv & below;
  t.compat = true;
  t.regions = (int64_t)1 << (__popc(sp) + __popcll(zz));
  t.emit = sp != 0 || zz != 0;
  return t;
}

// the same test on KW-word keys (k_connect)
template <int KW>
__device__ __forceinline__ PairTest pair_test(const Key<KW>& below, uint32_t fu, const Key<KW>& pu,
                                              const Key<KW>& zu, uint32_t fv, const Key<KW>& pv,
                                              const Key<KW>& zv) {
  PairTest t{false, false, 0};
  if (((fu | fv) & 7u) != 7u) return t;  // not the canonical cell
  if (tnp::key_any((pu ^ pv) & ~zu & ~zv & below)) return t;
  const uint32_t a = fu & fv;
  const uint32_t sp = a & (a >> 3) & 7u;  // axes where both lie on the same mark plane
  const Key<KW> zz = zu & zv & below;
  t.compat = true;
  t.regions = (int64_t)1 << (__popc(sp) + tnp::key_pop(zz));
  t.emit = sp != 0 || tnp::key_any(zz);
  return t;
}

// where the connect phase counts its appended keys and pair statistics:
// this workgroup's XCD shard (xs != null: large grids, k_keys_finish folds
// the shards into ctr) or the counter block itself (small grids: a few
// hundred workgroups, no fold or concatenation launches)
__device__ __forceinline__ int64_t* sink_word(int64_t* xs, int64_t* ctr, int stat) {
  constexpr int slot[5] = {CTR_XK, CTR_COMPAT, CTR_P, CTR_X, CTR_SPAIRS};
  return xs ? &xs[xs_word(stat, blockIdx.x % XS_N)] : &ctr[slot[stat]];
}

// a block's (compatible pairs, shared regions, connecting edges) totals
//   -> ctr[CTR_COMPAT], ctr[CTR_P], ctr[CTR_X] (or their shards)
__device__ __forceinline__ void add_pair_stats(int64_t a, int64_t r, int64_t x, int64_t* lds,
                                               int64_t* __restrict__ xs, int64_t* __restrict__ ctr) {
  int64_t ta, tr, tx;
  tnp::block_scan_excl(a, lds, ta);
  tnp::block_scan_excl(r, lds, tr);
  tnp::block_scan_excl(x, lds, tx);
  if (threadIdx.x == 0) {
    if (ta) atomicAdd((unsigned long long*)sink_word(xs, ctr, XS_COMPAT), (unsigned long long)ta);
    if (tr) atomicAdd((unsigned long long*)sink_word(xs, ctr, XS_P), (unsigned long long)tr);
    if (tx) atomicAdd((unsigned long long*)sink_word(xs, ctr, XS_X), (unsigned long long)tx);
  }
}

// ---------------------------------------------------------------------------
// Window pass: the pairs of every cell of <= WCELL members.  The entries are
// cell-contiguous; a wave stages the 64 records of window w (entries
// [lo + S w, lo + S w + 64) of [lo, hi), S = WSTRIDE) in LDS; each of its first S
// entries j is tested against the later entries of its cell, the (j,
// partner) tests flattened over the 64 lanes (a wave scan of the per-entry
// counts; a test finds its pair in a per-window LDS table the initiators
// fill, or by a 6-step search past WOWN tests): a pair (j < i) of such a cell is
// tested exactly once, in window floor(j / S) (i - j <= 64 - S).  Each record
// is read once from memory per window; emitted keys go through a per-wave LDS
// buffer, one global append per WKEYS.
// ---------------------------------------------------------------------------
#ifndef TNP_WKEYS
#define TNP_WKEYS 256  // (round 6: 384 -> 256, its LDS to the 1,024-test table; bucket_group -1 %)
#endif
constexpr int WKEYS = TNP_WKEYS;


__device__ __forceinline__ void lds_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

#ifndef TNP_WOWN
#define TNP_WOWN 1024  // >= the most tests a window of cells <= WCELL members holds: no search
#endif
constexpr int WOWN = TNP_WOWN;  // tests of one window resolved by table (more: binary search)

// st last: the grouping kernel's LDS-record path lays its record chunk over
// st and the space behind it (bucket.hip k_bucket_group)
struct WinLds {
  int exc[TNP_WAVES][64];
  uint16_t own[TNP_WAVES][WOWN];  // test t -> initiator | partner << 8
  uint64_t kb[TNP_WAVES][WKEYS];
  CellEnt st[TNP_WAVES][64];
};
struct WinAcc {
  int kn = 0;  // wave-uniform fill of this wave's key buffer
  int64_t n_compat = 0, n_reg = 0, n_conn = 0;
  // (packed path) wave-uniform counts from the tests' ballots, scalar
  // registers instead of a per-lane 64-bit add per test; folded into lane 0's
  // n_compat / n_conn by fold_wave_counts before the block sums
  int64_t w_compat = 0, w_conn = 0;
};
__device__ __forceinline__ void fold_wave_counts(WinAcc& a) {
  if (tnp::lane() == 0) {
    a.n_compat += a.w_compat;
    a.n_conn += a.w_conn;
  }
  a.w_compat = a.w_conn = 0;
}
// a value every lane holds alike, as a scalar (wave-uniform branches and loop
// bounds instead of exec-mask juggling)
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// this wave's buffered keys -> its XCD shard's key region (xs != null) or
// the one key array, counted there
__device__ __forceinline__ void window_flush(uint64_t* __restrict__ keys, int64_t cap,
                                             int64_t* __restrict__ xs, int64_t* __restrict__ ctr, WinLds& W,
                                             WinAcc& a) {
  if (a.kn == 0) return;
  const int wv = tnp::wave(), L = tnp::lane();
  const int sh = xs ? blockIdx.x % XS_N : 0;
  const int64_t rc = xs ? cap / XS_N : cap;
  int64_t base = 0;
  if (L == 0) base = (int64_t)atomicAdd((unsigned long long*)sink_word(xs, ctr, XS_KEYS), (unsigned long long)a.kn);
  base = __shfl(base, 0, 64);
  uint64_t* dst = keys + sh * rc;
  for (int i = L; i < a.kn; i += 64)
    if (base + i < rc) dst[base + i] = W.kb[wv][i];
  lds_fence();
  a.kn = 0;
}

// the pair tests of one staged window (st[0..63], LDS): lane L initiates
// `rounds` tests, against the next `rounds` records of its cell
__device__ __forceinline__ void window_tests(const CellEnt* st, int rounds, uint64_t below, int nb, uint64_t fmask,
                                             uint64_t* __restrict__ keys, int64_t cap, int64_t* __restrict__ xs,
                                             int64_t* __restrict__ ctr, WinLds& W, WinAcc& a);

// windows w = w0, w0 + dw, ... of the records [lo, hi); one wave each
__device__ __forceinline__ void window_pass(const CellEnt* __restrict__ ent, int64_t lo, int64_t hi,
                                            int64_t w0, int64_t dw, uint64_t below, int nb, uint64_t fmask,
                                            uint64_t* __restrict__ keys, int64_t cap,
                                            int64_t* __restrict__ xs, int64_t* __restrict__ ctr, WinLds& W,
                                            WinAcc& a) {
  const int wv = tnp::wave(), L = tnp::lane();
  const int64_t nwin = (hi - lo + WSTRIDE - 1) / WSTRIDE;
  for (int64_t w = w0; w < nwin; w += dw) {
    const int64_t e = lo + w * WSTRIDE + L;
    const bool valid = e < hi;
    CellEnt r;
    if (valid) {
      r = ent[e];
    } else {
      r.p = r.z = 0;
      r.v = 0;
      r.f = 0;
      r.tag = 0xFFFFFFFFu;  // no cell: matches nothing, never initiates
      r.pad = 0;
    }
    W.st[wv][L] = r;
    lds_fence();
    // last lane of my cell inside the window (lane 63 always closes one)
    const uint32_t nxt = __shfl_down(r.tag, 1, 64);
    const uint64_t bm = __ballot(L == 63 || nxt != r.tag);
    const int last = L + __builtin_ctzll(bm >> L);
    const bool init = valid && L < WSTRIDE && !(r.tag & 0x80000000u);
    window_tests(W.st[wv], init ? last - L : 0, below, nb, fmask, keys, cap, xs, ctr, W, a);
  }
}

// Packed windows (the bucket path): window k holds the WHOLE cells
// [s_k, e_k) (at most 64 records, cells of <= WCELL members, chosen by the
// grouping kernel), so every record is staged once and every record
// initiates -- half the windows of the 32-stride pass above.
__device__ __forceinline__ void window_pass_packed(const CellEnt* __restrict__ ent, int64_t base,
                                                   const uint32_t* __restrict__ wl, int nwin, int w0, int dw,
                                                   uint64_t below, int nb, uint64_t fmask,
                                                   uint64_t* __restrict__ keys, int64_t cap,
                                                   int64_t* __restrict__ xs, int64_t* __restrict__ ctr,
                                                   WinLds& W, WinAcc& a) {
  const int wv = tnp::wave(), L = tnp::lane();
  for (int w = w0; w < nwin; w += dw) {
    const uint32_t se = (uint32_t)uniform((int)wl[w]);
    const int s = (int)(se & 0xFFFFu), n = (int)(se >> 16) - s;
    const bool valid = L < n;
    CellEnt r;
    if (valid) {
      r = ent[base + s + L];
    } else {
      r.p = r.z = 0;
      r.v = 0;
      r.f = 0;
      r.tag = 0xFFFFFFFFu;  // no cell: matches nothing, never initiates
      r.pad = 0;
    }
    W.st[wv][L] = r;
    lds_fence();
    const uint32_t nxt = __shfl_down(r.tag, 1, 64);
    const uint64_t bm = __ballot(L == 63 || nxt != r.tag);
    const int last = L + __builtin_ctzll(bm >> L);
    const bool init = valid && !(r.tag & 0x80000000u);  // (windows hold no big cell; defensive)
    window_tests(W.st[wv], init ? last - L : 0, below, nb, fmask, keys, cap, xs, ctr, W, a);
  }
}

// Packed windows over records already in LDS (the grouping kernel's record
// chunk: rec[p - p0] holds the bucket's record p): the windows of wl[] from
// this wave's cursor *k (windows k, k + dw, ...) that start before p_end
__device__ __forceinline__ void window_pass_lds(const CellEnt* rec, int p0, int p_end, const uint32_t* wl, int nwin,
                                                int* k, int dw, uint64_t below, int nb, uint64_t fmask,
                                                uint64_t* __restrict__ keys, int64_t cap,
                                                int64_t* __restrict__ xs, int64_t* __restrict__ ctr,
                                                WinLds& W, WinAcc& a) {
  const int L = tnp::lane();
  for (; *k < nwin; *k += dw) {
    const uint32_t se = (uint32_t)uniform((int)wl[*k]);
    const int s = (int)(se & 0xFFFFu), n = (int)(se >> 16) - s;
    if (s >= p_end) break;
    const CellEnt* st = rec + (s - p0);
    const bool valid = L < n;
    const uint32_t tag = valid ? st[L].tag : 0xFFFFFFFFu;
    const uint32_t nxt = __shfl_down(tag, 1, 64);
    const uint64_t bm = __ballot(L >= n - 1 || nxt != tag);  // (the window holds whole cells)
    const int last = L + __builtin_ctzll(bm >> L);
    window_tests(st, valid ? last - L : 0, below, nb, fmask, keys, cap, xs, ctr, W, a);
  }
}

// ---------------------------------------------------------------------------
// Packed records (the grouping kernel's LDS-record path, steps with
// 1 <= idx <= 29 and K - idx <= 32).  The pair test reads only the planes
// below idx and the 6 cell flags: one u64 TEST word per record,
//   low  32: (pos & below)   | span-start flags (bits 0..2 of f) << 29
//   high 32: (~zero & below) | on-plane flags   (bits 3..5 of f) << 29
// (pu ^ pv) & ~zu & ~zv & below  = (lo_u ^ lo_v) & hi_u & hi_v   (plane bits)
// zu & zv & below                = below & ~(hi_u | hi_v)
// canonical <=> (lo_u | lo_v) >> 29 == 7; sp = (lo_u & lo_v & hi_u & hi_v) >> 29.
// The pruning filter of the emitted pairs reads an ABOVE word (pos >> idx |
// zero >> idx << 32: planes idx .. K-1), the key the vertex slots.
// ---------------------------------------------------------------------------
struct PackedRecs {
  const uint64_t* tw;  // test words
  const uint64_t* aw;  // above words
  const uint32_t* vv;  // vertex slots
  const uint16_t* tg;  // local cell
};
constexpr int PK_FLAG_SHIFT = 29;
constexpr uint32_t PK_PLANES = (1u << PK_FLAG_SHIFT) - 1u;
__device__ __forceinline__ uint64_t packed_test_word(uint64_t p, uint64_t z, uint32_t f, uint64_t below) {
  const uint32_t lo = (uint32_t)(p & below) | ((f & 7u) << PK_FLAG_SHIFT);
  const uint32_t hi = (uint32_t)(~z & below) | (((f >> 3) & 7u) << PK_FLAG_SHIFT);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t packed_above_word(uint64_t p, uint64_t z, int idx) {
  return ((uint64_t)(uint32_t)(z >> idx) << 32) | (uint32_t)(p >> idx);
}

// the tests of one staged window of packed records (rec + s: its first
// record); lane L initiates `rounds` tests against the next records of its
// cell.  Same flattening, emission rules and counters as window_tests.
// amask: the pruning filter on the above words (0: every emitted pair kept)
__device__ __forceinline__ void window_tests_packed(const PackedRecs& R, int s, int rounds, uint32_t below,
                                                    int nb, uint64_t amask, uint64_t* __restrict__ keys,
                                                    int64_t cap, int64_t* __restrict__ xs,
                                                    int64_t* __restrict__ ctr, WinLds& W, WinAcc& a) {
  const int wv = tnp::wave(), L = tnp::lane();
  const int incl = tnp::wave_scan_incl(rounds);
  const int total = uniform(__shfl(incl, 63, 64));
  const bool table = total <= WOWN;
  W.exc[wv][L] = incl - rounds;
  if (table)
    for (int r = 0, t = incl - rounds; r < rounds; ++r, ++t) W.own[wv][t] = (uint16_t)(L | ((L + 1 + r) << 8));
  lds_fence();
  auto pair_of = [&](int t, int& j, int& i) {
    if (table) {
      const uint32_t o = W.own[wv][t];
      j = (int)(o & 0xFFu);
      i = (int)(o >> 8);
    } else {
      int lo2 = 0, hi2 = 62;
#pragma unroll
      for (int it = 0; it < 6; ++it) {
        const int mid = (lo2 + hi2 + 1) >> 1;
        if (W.exc[wv][mid] <= t) lo2 = mid;
        else hi2 = mid - 1;
      }
      j = lo2;
      i = j + 1 + (t - W.exc[wv][j]);
    }
  };
  // the test of records j, i (live == false counts nothing); true: append key
  auto test = [&](int j, int i, bool live, uint64_t& key) -> bool {
    // every LDS read of the test issued together (a read behind the emit
    // predicate would add a dependent round trip to nearly every batch)
    const uint64_t tu = R.tw[s + j], tv = R.tw[s + i];
    const uint64_t au = R.aw[s + j], av = R.aw[s + i];
    const uint32_t vu = R.vv[s + j], vq = R.vv[s + i];
    const uint32_t lu = (uint32_t)tu, hu = (uint32_t)(tu >> 32), lv = (uint32_t)tv, hv = (uint32_t)(tv >> 32);
    const uint32_t hh = hu & hv;
    const bool canon = ((lu | lv) >> PK_FLAG_SHIFT) == 7u;
    const uint32_t d = (lu ^ lv) & hh & PK_PLANES;
    const uint32_t sp = (lu & lv & hh) >> PK_FLAG_SHIFT;
    const uint32_t zz = below & ~(hu | hv);
    const bool compat = live & canon & (d == 0u);
    const bool emit = compat & ((sp | zz) != 0u);
    a.w_compat += __popcll(__ballot(compat));
    a.n_reg += compat ? ((int64_t)1 << (__popc(sp) + __popc(zz))) : 0;
    a.w_conn += __popcll(__ballot(emit));
    key = ((uint64_t)min(vu, vq) << nb) | max(vu, vq);
    // the step's pruning drops it anyway (keep_edge): never appended
    return emit & ((amask == 0) | (((au ^ av) & amask) != 0));
  };
  auto append = [&](bool em, uint64_t key) {
    const uint64_t eb = __ballot(em);
    if (em) W.kb[wv][a.kn + tnp::mbcnt(eb)] = key;
    a.kn += __popcll(eb);
  };
  int t0 = 0;
  for (; t0 + 64 < total; t0 += 128) {
    if (a.kn + 128 > WKEYS) window_flush(keys, cap, xs, ctr, W, a);
    const int ta = t0 + L, tb = t0 + 64 + L;
    const bool lb = tb < total;
    int ja, ia, jb, ib;
    pair_of(ta, ja, ia);
    pair_of(lb ? tb : ta, jb, ib);
    uint64_t ka = 0, kb = 0;
    const bool ema = test(ja, ia, true, ka);
    const bool emb = test(jb, ib, lb, kb);
    append(ema, ka);
    append(emb, kb);
  }
  for (; t0 < total; t0 += 64) {
    if (a.kn + 64 > WKEYS) window_flush(keys, cap, xs, ctr, W, a);
    const int t = t0 + L;
    const bool live = t < total;
    int j = 0, i = 0;
    pair_of(live ? t : 0, j, i);
    uint64_t key = 0;
    const bool em = test(j, i, live, key);
    append(em, key);
  }
  lds_fence();
}

// packed windows over the packed record chunk (records p0 .. of the bucket
// at R index p - p0): as window_pass_lds
__device__ __forceinline__ void window_pass_packed_lds(const PackedRecs& R, int p0, int p_end, const uint32_t* wl,
                                                       int nwin, int* k, int dw, uint32_t below, int nb,
                                                       uint64_t amask, uint64_t* __restrict__ keys, int64_t cap,
                                                       int64_t* __restrict__ xs, int64_t* __restrict__ ctr,
                                                       WinLds& W, WinAcc& a) {
  const int L = tnp::lane();
  for (; *k < nwin; *k += dw) {
    const uint32_t se = (uint32_t)uniform((int)wl[*k]);
    const int s = (int)(se & 0xFFFFu), n = (int)(se >> 16) - s;
    if (s >= p_end) break;
    const bool valid = L < n;
    const uint32_t tag = valid ? R.tg[s - p0 + L] : 0xFFFFFFFFu;
    const uint32_t nxt = __shfl_down(tag, 1, 64);
    const uint64_t bm = __ballot(L >= n - 1 || nxt != tag);  // (the window holds whole cells)
    const int last = L + __builtin_ctzll(bm >> L);
    window_tests_packed(R, s - p0, valid ? last - L : 0, below, nb, amask, keys, cap, xs, ctr, W, a);
  }
}

__device__ __forceinline__ void window_tests(const CellEnt* st, int rounds, uint64_t below, int nb, uint64_t fmask,
                                             uint64_t* __restrict__ keys, int64_t cap, int64_t* __restrict__ xs,
                                             int64_t* __restrict__ ctr, WinLds& W, WinAcc& a) {
  const int wv = tnp::wave(), L = tnp::lane();
  {
    // flatten the window's (initiator, partner) tests over the lanes: test t
    // belongs to the last initiator j with exc[j] <= t, partner j + 1 + t - exc[j]
    const int incl = tnp::wave_scan_incl(rounds);
    const int total = uniform(__shfl(incl, 63, 64));
    const bool table = total <= WOWN;
    W.exc[wv][L] = incl - rounds;
    if (table)  // each initiator lists its own tests (a few, mostly)
      for (int r = 0, t = incl - rounds; r < rounds; ++r, ++t) W.own[wv][t] = (uint16_t)(L | ((L + 1 + r) << 8));
    lds_fence();
    // test t -> (initiator j, partner i)
    auto pair_of = [&](int t, int& j, int& i) {
      if (table) {
        const uint32_t o = W.own[wv][t];
        j = (int)(o & 0xFFu);
        i = (int)(o >> 8);
      } else {
        int lo2 = 0, hi2 = 62;
#pragma unroll
        for (int it = 0; it < 6; ++it) {
          const int mid = (lo2 + hi2 + 1) >> 1;
          if (W.exc[wv][mid] <= t) lo2 = mid;
          else hi2 = mid - 1;
        }
        j = lo2;
        i = j + 1 + (t - W.exc[wv][j]);
      }
    };
    // pair_test without branches: both records are read once, every
    // predicate is a select (branches here cost exec-mask juggling and a
    // second dependent LDS round trip per test); live == false counts nothing
    auto test = [&](const CellEnt& u, const CellEnt& q, bool live, uint64_t& key) -> bool {
      const uint64_t d = (u.p ^ q.p) & ~u.z & ~q.z & below;
      const uint32_t af = u.f & q.f;
      const uint32_t sp = af & (af >> 3) & 7u;
      const uint64_t zz = u.z & q.z & below;
      const bool compat = live & (((u.f | q.f) & 7u) == 7u) & (d == 0);
      const bool emit = compat & ((sp != 0) | (zz != 0));
      a.n_compat += compat;
      a.n_reg += compat ? ((int64_t)1 << (__popc(sp) + __popcll(zz))) : 0;
      a.n_conn += emit;
      const uint32_t vu = (uint32_t)u.v, vv = (uint32_t)q.v;
      key = ((uint64_t)min(vu, vv) << nb) | max(vu, vv);
      // the step's pruning drops it anyway (keep_edge): never appended
      return emit & ((fmask == 0) | ((((u.p ^ q.p) | (u.z ^ q.z)) & fmask) != 0));
    };
    auto append = [&](bool em, uint64_t key) {
      const uint64_t eb = __ballot(em);
      if (em) W.kb[wv][a.kn + tnp::mbcnt(eb)] = key;
      a.kn += __popcll(eb);
    };
    int t0 = 0;
    // two batches of 64 tests per round while both hold tests: their LDS
    // reads in flight together (the chain own[] -> records -> test is
    // latency-bound one batch at a time)
    for (; t0 + 64 < total; t0 += 128) {
      if (a.kn + 128 > WKEYS) window_flush(keys, cap, xs, ctr, W, a);
      const int ta = t0 + L, tb = t0 + 64 + L;
      const bool lb = tb < total;
      int ja, ia, jb, ib;
      pair_of(ta, ja, ia);
      pair_of(lb ? tb : ta, jb, ib);
      const CellEnt ua = st[ja], qa = st[ia];
      const CellEnt ub = st[jb], qb = st[ib];
      uint64_t ka, kb;
      const bool ema = test(ua, qa, true, ka);
      const bool emb = test(ub, qb, lb, kb);
      append(ema, ka);
      append(emb, kb);
    }
    for (; t0 < total; t0 += 64) {
      if (a.kn + 64 > WKEYS) window_flush(keys, cap, xs, ctr, W, a);
      const int t = t0 + L;
      const bool live = t < total;
      int j = 0, i = 0;
      pair_of(live ? t : 0, j, i);
      const CellEnt u = st[j];
      const CellEnt q = st[i];
      uint64_t key;
      const bool em = test(u, q, live, key);
      append(em, key);
    }
    lds_fence();
  }
}

}  // namespace
