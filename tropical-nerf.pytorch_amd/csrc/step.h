// Internal: step-kernel launchers (step.hip) and device counter slots.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

// slots of the engine's int64 device counter block (one pinned readback)
enum {
  CTR_S = 0,        // split count (scan total)
  CTR_H = 1,        // hit vertices
  CTR_T = 2,        // cell entries
  CTR_X = 3,        // connecting edges
  CTR_E = 4,        // kept edges
  CTR_V = 5,        // kept vertices
  CTR_A = 6,        // augmented rows (reference regions_to_vertices size)
  CTR_P = 7,        // candidate pairs (reference extract_every_valid_edge size)
  CTR_COMPAT = 8,   // member pairs sharing >= 1 region
  CTR_TESTS = 9,    // member pairs tested
  CTR_FAIL = 10,    // local failover-override predicate
  CTR_K0 = 11,      // some member row has no zero (reference raises)
  CTR_ACTIVE = 12,  // next-active plane mask (u64 bits)
  CTR_TRI = 13,
  CTR_FACES = 14,
  CTR_AUX = 15,
  CTR_DUP = 16,     // splits on the slab's shared boundary plane
  CTR_BIG = 17,     // a cell with more than 65535 members
  CTR_B = 18,       // curve path: non-axis-aligned split edges
  CTR_G = 19,       // curve path: rows needing gradient descent
  CTR_NOPLANE = 20, // curve path: a c row with no shared plane below idx
  CTR_TIGHT = 21,   // curve path: a kept c row misses its edge plane by > eps
  CTR_KEEP = 22,    // curve path: splits surviving the strict filter
  CTR_BOVF = 23,    // pair-chunk table overflow
  CTR_XK = 24,      // connecting edges surviving this step's pruning (appended)
  CTR_R = 25,       // cells with at least one member pair
  CTR_RUNS = 26,    // occupied cells (runs of equal keys in the sorted entries)
  CTR_SPAIRS = 27,  // member pairs of the cells the window pass tests (<= WCELL members)
  CTR_TK0 = 28,     // last-workgroup ticket (tnp::last_block) of the fused bucket count
  CTR_PCK = 29,     // bucket path: pair cells (bits 0..23) | their pairs << 24, allocated by atomics
  CTR_MISSED = 30,  // split: an edge whose first split plane lies below the step (masks to redo)
  CTR_N = 31        // <= 31: the host-mapped mirror keeps its sequence word at [31]
};

int64_t step_tiles(int64_t n);
int64_t lb_tiles(int64_t n);     // tiles of the single-pass prune
int64_t split_tiles(int64_t n);  // tiles of the single-pass split and hit passes
int split_hit_workers(int64_t V);  // hit workers a split over V vertex slots runs (HitArgs::hpart entries)
int64_t run_tiles(int64_t n);    // tiles of the radix path's run-start pass
// single-pass split over split_tiles(E) look-back tiles (E > 0) from the
// edges' first split planes (ef == idx): S -> ctr[CTR_S]; an edge whose
// first split plane is below idx sets ctr[CTR_MISSED] (its masks are older
// than the caller's step order: redo them from idx); sa/sb (and eidx if
// given) need capacity E; without eidx the split edges are rewired in place
// and their masks marked stale
// hits != null: the plane's hit vertices in the same dispatch (workgroups
// past the split tiles): live slots v < hits->V with |col[v]| < eps ->
// hits->out[0, ctr[CTR_H]) (no dependence on S)
struct HitArgs {
  const float* col;
  const uint8_t* alive;
  int64_t V;
  float eps;
  int32_t* out;
  // != null: every hit worker also counts the live slots it reads -> hpart[w]
  // (the previous step's live vertex count, summed by launch_publish_sums:
  // the engine's run loop defers count_live into the next split)
  int64_t* hpart;
};
constexpr int HIT_WORKERS_MAX = 512;  // hit workers of one split (hpart entries)
int launch_split_lb(int32_t* edges, int64_t E, const uint8_t* ef, uint8_t* dm, int idx, int64_t V,
                    int32_t* sa, int32_t* sb, int64_t* ctr, int32_t* eidx, const TnpLB& lb,
                    hipStream_t s, const HitArgs* hits = nullptr);
// per-edge masks from the endpoint keys (pz): dm = 1 + highest plane where
// the keys differ (0: none), ef = the first plane in [from, last_plane] that
// splits the edge (EDGE_NOSPLIT: none); ctr != null: OR of those first
// planes -> CTR_ACTIVE
int launch_edge_masks(const int32_t* edges, int64_t E, const uint64_t* pz, uint8_t* dm,
                      uint8_t* sm, int from, int last_plane, bool keep_dead, int64_t* ctr, hipStream_t s);
int launch_new_vertices(const int32_t* sa, const int32_t* sb, int64_t S, const float* col,
                        float eps, float* xyz, int64_t V, hipStream_t s);
int launch_fail_check(const int32_t* sa, const int32_t* sb, int64_t S, int idx,
                      const uint64_t* zero, const float* stage, float eps, uint64_t* shared,
                      int64_t* ctr, const uint64_t* grid_new, const OwnBox& own, int kw, hipStream_t s);
int launch_finalize_new(int64_t S, int K, int override_, const uint64_t* shared, float* stage,
                        float eps, float* pre, int64_t ld, int keep_from, int64_t V, uint64_t* pos,
                        uint64_t* zero, const int64_t* ctr, uint64_t* pz, int kw, hipStream_t s);
// members = [V, V + S) ++ live vertices v < V with |col[v]| < eps (in no
// particular order: atomic appends); count -> ctr[CTR_H] (zero on entry).
// S < 0: the hits only, placed after ctr[CTR_S] members (launched behind
// the split kernel; launch_new_members fills [0, S) once S is known)
int launch_hits(const float* col, const uint8_t* alive, int64_t V, float eps, int32_t* members,
                int64_t S, int64_t* ctr, hipStream_t s);
int launch_new_members(int32_t* members, int64_t S, int64_t V, hipStream_t s);
// new vertices (grid words) outside the owned x range (lo, hi] -> ctr[CTR_DUP] (lo > hi: nothing)
int launch_count_unowned(const uint64_t* grid, int64_t n, const OwnBox& own, int64_t* ctr, hipStream_t s);
// sort-based cell bucketing: span counts (+ A), (cell, member) entries,
// segment bounds of the cell-sorted entries, per-cell counts, key copies
// M = capacity (S + V); the live member count S + ctr[CTR_H] is read on
// the device (no host round trip for the hit count)
int launch_span_count(const int32_t* members, int64_t S, int64_t M, const uint64_t* grid,
                      const uint64_t* zero, int idx, int32_t* cnt, int64_t* part, int64_t* ctr,
                      int kw, hipStream_t s);
int launch_span_emit(const int32_t* members, int64_t S, int64_t M, const uint64_t* grid, int NC,
                     const int64_t* eoff, uint32_t* ekey, int32_t* eval, const int64_t* ctr,
                     hipStream_t s);
// pair cells from the cell-sorted entry keys (runs of equal keys): the r-th
// cell with >= 2 members (cell order) -> pcell[r] = cell id, pent[r] = its
// first entry, pn[r] = its member count, ptoff[r] = its first pair in the
// flattened pair space; R -> ctr[CTR_R], pairs -> ctr[CTR_TESTS], a cell
// above 65535 members -> CTR_BIG.  Arrays sized >= T / 2 + 1.
// Two passes: run starts (rstart[r] = first entry of the r-th occupied
// cell, rstart[runs] = T, runs -> ctr[CTR_RUNS]; run_tiles(T) look-back
// tiles, rstart sized >= T + 1), then the runs with >= 2 entries
// (pair_run_tiles(T) look-back tiles for each of lb_rank / lb_pairs; the
// run count is read on the device).
int launch_run_starts(const uint32_t* key, int64_t T, int32_t* rstart, int64_t* ctr, const TnpLB& lb,
                      hipStream_t s);
int launch_pair_runs(const uint32_t* key, const int32_t* rstart, int64_t T, int32_t* pcell,
                     int32_t* pent, int32_t* pn, int64_t* ptoff, int64_t* ctr, const TnpLB& lb_rank,
                     const TnpLB& lb_pairs, hipStream_t s);
int64_t pair_run_tiles(int64_t T);
// one cell entry as the pair test reads it: the member's sign keys, its id
// and its grid relation to THIS cell in 6 bits (cell_flags): bit d = the
// member's lowest spanned cell along axis d is this cell, bit 3 + d = the
// member lies on a mark plane of axis d.  One 32-byte record per entry.
// tag: the cell's id for the window pass (bit 31: a cell above WCELL
// members, left to the flattened pair-space pass); 0 on the radix path
struct alignas(32) CellEnt {
  uint64_t p, z;
  int32_t v;
  uint32_t f;
  uint32_t tag, pad;
};
// the record of a two-word-key net (K > 63, radix path only): 48 bytes
struct alignas(16) CellEnt2 {
  uint64_t p[2], z[2];
  int32_t v;
  uint32_t f;
  uint32_t tag, pad;
};
template <int KW> struct CellEntOf { using type = CellEnt; };
template <> struct CellEntOf<2> { using type = CellEnt2; };
template <int KW> using CellEntT = typename CellEntOf<KW>::type;
__host__ __device__ inline size_t cell_ent_bytes(int kw) { return kw == 2 ? sizeof(CellEnt2) : sizeof(CellEnt); }
__device__ __forceinline__ Key<1> ent_p(const CellEnt& e) { return Key<1>{{e.p}}; }
__device__ __forceinline__ Key<1> ent_z(const CellEnt& e) { return Key<1>{{e.z}}; }
__device__ __forceinline__ Key<2> ent_p(const CellEnt2& e) { return Key<2>{{e.p[0], e.p[1]}}; }
__device__ __forceinline__ Key<2> ent_z(const CellEnt2& e) { return Key<2>{{e.z[0], e.z[1]}}; }
__device__ __forceinline__ void ent_set_keys(CellEnt& e, const Key<1>& p, const Key<1>& z) {
  e.p = p.w[0];
  e.z = z.w[0];
}
__device__ __forceinline__ void ent_set_keys(CellEnt2& e, const Key<2>& p, const Key<2>& z) {
  e.p[0] = p.w[0];
  e.p[1] = p.w[1];
  e.z[0] = z.w[0];
  e.z[1] = z.w[1];
}
// cells of at most WCELL members have their pairs tested by the window pass
// (k_connect_win): a pair (j < i) of such a cell lies in the 64-entry
// window starting at 32 * floor(j / 32)
#ifndef TNP_WSTRIDE
#define TNP_WSTRIDE 32
#endif
constexpr int WSTRIDE = TNP_WSTRIDE;  // window pass: windows of 64 records at this stride
constexpr int WCELL = 65 - WSTRIDE;    // a pair (j < i) of such a cell has i - j <= 64 - WSTRIDE
// cell_flags of a member (grid word g) in the cell with coordinates c (+2)
__device__ __forceinline__ uint32_t cell_flags(uint64_t g, int cx, int cy, int cz) {
  const int c[3] = {cx, cy, cz};
  uint32_t f = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int o = tnp::grid_off(g, d);
    const bool zd = tnp::grid_zero(g, d);
    const int lo = (zd ? o - 1 : o) + 2;
    f |= (uint32_t)(lo == c[d]) << d;
    f |= (uint32_t)zd << (3 + d);
  }
  return f;
}
// pz: the interleaved (pos, zero) copy of the vertex keys; ent: CellEntT<kw> records
int launch_entry_keys(const int32_t* ent_v, const uint32_t* ekey, int NC, int64_t T,
                      const uint64_t* grid, const uint64_t* pz, void* ent, int kw, hipStream_t s);

// connecting edges over the flattened pair space (pair cells in order, then
// (i, j<i) inside a cell); the pair count and R are read on the device.
// chunk_cells maps pair chunks to pair cells (capacity cap chunks, overflow
// -> CTR_BOVF); connect counts every connecting edge in ctr[CTR_X] and
// appends the packed keys (lo << nb | hi) of those the step's pruning keeps
// (fmask != 0: endpoint keys differ on the planes of fmask; fmask == 0: all)
// to keys[0, cap), counted in ctr[CTR_XK]; per block, the compatible pairs,
// shared regions and connecting edges are added to ctr[CTR_COMPAT],
// ctr[CTR_P], ctr[CTR_X].
int64_t connect_chunks(int64_t TT);
int64_t connect_grid();
int launch_chunk_cells(const int64_t* ptoff, const int32_t* pn, int64_t rcap, int32_t* bcell,
                       int64_t cap, int64_t* ctr, hipStream_t s);
// ent: CellEntT<kw> records; filt_last >= 0: the pruning filter is planes
// [idx, filt_last] (endpoint keys differing there), < 0: every pair kept
int launch_connect(const int64_t* ptoff, const int32_t* pcell, const int32_t* pn,
                   const int32_t* pent, int NC, int64_t max_tests, const int32_t* bcell,
                   const void* ent, int idx, int nb, int filt_last, int kw, uint64_t* keys,
                   int64_t cap, int64_t* xs, int64_t* ctr, hipStream_t s, const int64_t* bstat = nullptr,
                   int nbstat = 0);
// single-pass pruning over [edges; e_new; c_new] (lb_tiles(E + S + X)
// look-back tiles): kept edges in order -> out, used flags (zeroed by the
// caller), ctr[CTR_E], ctr[CTR_ACTIVE]
int launch_prune_lb(const int32_t* edges, int64_t E, const int32_t* sb, int64_t S, int64_t V,
                    const uint64_t* ckeys, int nb, int64_t X, int idx, int last_plane,
                    const uint64_t* pz, const uint8_t* dm, const uint8_t* ef, int32_t* out,
                    uint8_t* odm, uint8_t* oef, uint8_t* used, bool count_live, int64_t* ctr,
                    const TnpLB& lb, hipStream_t s);
// count_live: the distinct live endpoints are counted into ctr[CTR_V] on the
// way (word atomics; for small complexes, instead of launch_count_flags)
// ctr[slot] += number of set byte flags in f[0, n) (16-B aligned f, 0/1 bytes)
// part != null: also ctr[pslot] = sum of part[0, nparts) (the lazy prune's
// per-workgroup kept counts)
int launch_count_flags(const uint8_t* f, int64_t n, int64_t* ctr, int slot, hipStream_t s,
                       const int64_t* part = nullptr, int nparts = 0, int pslot = 0);
// lazy pruning of step idx over [edges; e_new; c_new] (N = E + S + X slots):
// old edges stay in place (removed ones marked EDGE_DEAD, rewired ones get
// their bytes), e_new / c_new written to slots E.. (edges, dm, ef need N
// entries); used flags; per-workgroup kept counts -> part (fold them with
// launch_count_flags), next-active planes -> ctr[CTR_ACTIVE]
// split-eps mode: first split planes >= from of the live edges at eps_s from
// the cached planes (pre plane-major, leading dimension ld, every plane
// cached); OR -> ctr[CTR_ACTIVE] when ctr != null
int launch_ef_cache(const int32_t* edges, int64_t E, const uint8_t* dm, uint8_t* ef, const float* pre, int64_t ld,
                    int from, int K, float eps_s, int64_t* ctr, hipStream_t s);
constexpr int PRUNE_LAZY_MAX_BLOCKS = 1024;
int prune_lazy_blocks(int64_t N);
// [i0, i1): the slots of [edges; e_new; c_new] this launch takes (the
// old edges and e_new need no c_new: the engine runs them while the connect
// counts travel to the host); prune_lazy_blocks(i1 - i0) parts
int launch_prune_lazy(int32_t* edges, int64_t E, const int32_t* sb, int64_t S, int64_t V, const uint64_t* ckeys,
                      int nb, int64_t X, int idx, int last_plane, const uint64_t* pz, uint8_t* dm, uint8_t* ef,
                      uint8_t* used, int64_t* part, int64_t* ctr, hipStream_t s, int64_t i0, int64_t i1);
// the counter block -> a host-mapped mirror, then the sequence word at [31]
// (the host spins on it instead of a copy + stream synchronise)
// clear: the counter words are zeroed once read (the next split's reset,
// without its memset: the run loop's last readback of a step)
int launch_publish(int64_t* ctr, int64_t* host, int64_t seq, hipStream_t s, bool clear = false);
// the same, publishing host[CTR_V] = sum(vpart[0..nv)) and (ne > 0)
// host[CTR_E] = sum(epart[0..ne)) instead of the device words (the deferred
// live counts of the previous step; the device words stay untouched)
int launch_publish_sums(const int64_t* ctr, int64_t* host, int64_t seq, const int64_t* vpart, int nv,
                        const int64_t* epart, int ne, hipStream_t s);
int launch_widen_flags(const uint8_t* f, int64_t n, int32_t* out, hipStream_t s);
// planes the pruning of step idx compares (idx .. last_plane)
uint64_t prune_mask(int idx, int last_plane);
// ---- bucket.hip: members grouped by grid cell in spatial buckets ----------
constexpr int BUCKET_MAX = 6144;        // member-pass buckets (17^3 lattice; 5 x 33 x 33 slab)
constexpr int BUCKET_LOCAL_MAX = 4096;  // cells per bucket (16^3)
// The buckets cover the cells (+2 coordinates) [xorg, xorg + xn) along x,
// and the same along y and z: a slab or block of a sharded complex buckets
// only its own cells (an 8-rank 256^3 x-slab: 5 x 33 x 33 buckets of 8^3
// cells instead of 17^3 buckets of 16^3, 82 % of them empty; a 2 x 2 x 2
// block: 17^3 buckets of 8^3 cells, the 128^3 lattice's geometry)
struct BucketGeom {
  int NC;    // cell coordinates per axis (n_marks + 2)
  int sh;    // log2 of the bucket edge in cells (the member passes' buckets)
  int NBx, NBy, NBz;     // buckets along x, y, z
  int xorg, yorg, zorg;  // first cell coordinate along each axis
  int xn, yn, zn;        // cells along each axis the buckets cover (NB. << sh)
  int NB;    // NBx * NBy * NBz
  // 1: two-level buckets.  The member passes bucket by 16^3 cells (sh = 4,
  // NB <= BUCKET_MAX bins in their LDS histograms); launch_bucket_refine
  // splits every bucket into its 8 octants of 8^3 cells, and the grouping
  // runs over those NG = 8 NB sub-buckets (group bucket 8 b + o) with the
  // 8^3-cell kernel -- grids above 17^3 buckets of 8^3 (~134 marks) keep
  // the small buckets the grouping is tuned for
  int sub;
  int NG;  // group buckets: NB, or 8 NB when sub
};
// the bucket geometry for a complex inside the mark planes [lo[d], hi[d]]:
// 8^3-cell buckets when their count fits BUCKET_MAX, else 16^3-cell member
// buckets refined into 8^3-cell group buckets (sub); -1: the grid is too
// fine for the bucket path (the radix-sort path takes it)
int bucket_geometry(int n_marks, const int lo[3], const int hi[3], BucketGeom* g);
// sub geometries: every 16^3-cell bucket's entries (bbase / ekv, the member
// passes' output) regrouped by octant into ekv2, bases of the 8 NB group
// buckets -> bbase2 [8 NB + 1]; entries keep their cell flags and vertex,
// their local cell becomes the 9-bit one of the octant.  Zeroes the member
// passes' bucket counters bcount / bcur for the next step
int launch_bucket_refine(const BucketGeom& g, const int64_t* bbase, const uint64_t* ekv, int64_t* bbase2,
                         uint64_t* ekv2, int32_t* bcount, int32_t* bcur, hipStream_t s);
// members -> (local cell, vertex) entries in bucket ranges; A -> ctr[CTR_A],
// T -> ctr[CTR_T], k=0 rows -> ctr[CTR_K0] bit 0, a member outside the
// geometry's x range -> bit 1 (skipped; the host raises).  bcount/bcur: NB int32,
// bbase: NB + 1, part: ceil(M / 2048) + 1 int64; ekey/ev: 8 M capacity
// ekv: the entries in bucket order, packed (local cell << 40 | cell flags
// << 32 | vertex) (8 M capacity)
// members: the step's S new vertices are slots V.. (not listed), the hits
// follow in members[S, M).  clean: bcount/bcur are known to be zero (the
// previous step's launch_bucket_pairs reset them).  live != null: nlive
// live flags zeroed on the way (the prune re-marks them).  Uses ctr[CTR_TK0].
// ovr != null: the new vertices' failover override (launch_override_new's
// work) applied on the way, before any key is read
struct NewOverride {
  int flag;  // < 0: the device predicate ctr[CTR_FAIL]; else the host's decision
  const uint64_t* shared;
  float* pre;
  int64_t ld;
  int keep_from;
  uint64_t* pos;
  uint64_t* zero;
  uint64_t* pz;
};
// workgroups of the member passes over M members (>= 1): the per-block parts buffer
// of launch_bucket_entries needs max(this, 512) entries
int64_t bucket_member_blocks(int64_t M);
int launch_bucket_entries(const int32_t* members, int64_t S, int64_t V, int64_t M, const uint64_t* grid,
                          const uint64_t* zero, int idx, const BucketGeom& g, int32_t* bcount, int32_t* bcur,
                          int64_t* bbase, int64_t* part, uint64_t* ekv, bool clean, uint8_t* live,
                          int64_t nlive, const NewOverride* ovr, int64_t* ctr, hipStream_t s);
// per bucket: cell-contiguous CellEnt records (ents, entry positions) and
// the bucket's cells above WCELL members, appended to the global pair-cell
// list (pcell, pent, pn, ptoff) that launch_connect walks: a workgroup
// reserves its cells and their pairs with ONE atomic on ctr[CTR_PCK] (cells
// | pairs << 24: cell slots and pair offsets in the same order, which the
// chunk walk needs; the list order is otherwise free -- the emitted keys are
// sorted), and fills k_connect's chunk table bcell (bcap chunks, overflow ->
// CTR_BOVF).  The pairs of the smaller cells -> ctr[CTR_SPAIRS].  Leaves
// bcount/bcur zeroed for the next step.  launch_connect unpacks CTR_PCK;
// the host reads R = CTR_PCK & 0xFFFFFF, pairs = CTR_PCK >> 24.
// win != null: the grouping kernel also runs the window pass (launch_connect_win's
// work) over each bucket's records
// Per-XCD shards of the connect phase's appends and pair statistics.  One
// device-scope atomic per workgroup (or per wave flush) on ONE word
// serialises at ~11 ns (MI355X_MICROARCH.md fan-in: ~88 per microsecond);
// shard x = blockIdx.x % 8 (the dispatcher's XCD) has a 128-B line per
// counter and its own key region keys[x * rc, (x + 1) * rc), rc = cap / 8.
// k_keys_finish folds the shards into ctr and the regions' output offsets;
// k_keys_compact concatenates the regions.
#ifndef TNP_XS_N
#define TNP_XS_N 8
#endif
constexpr int XS_N = TNP_XS_N;  // shards (<= 63: k_keys_finish folds them in one wave)
constexpr int XS_LINE = 16;  // int64 words per counter line
enum { XS_KEYS = 0, XS_COMPAT = 1, XS_P = 2, XS_X = 3, XS_SP = 4, XS_STATS = 5 };
__host__ __device__ constexpr int xs_word(int stat, int shard) { return (stat * XS_N + shard) * XS_LINE; }
constexpr int XS_OFF = XS_STATS * XS_N * XS_LINE;  // + [0, XS_N]: region output offsets
constexpr int XS_WORDS = XS_OFF + 64 + 1;  // + the XS_N + 1 offsets
// counts of the shards -> ctr[CTR_XK] (all keys, or XS_N x the largest
// region count when a region overflowed: the caller grows cap to it and
// redoes), ctr[CTR_COMPAT / CTR_P / CTR_X]; region offsets; shards zeroed
int launch_keys_finish(int64_t* xs, int64_t cap, int64_t* ctr, hipStream_t s);
// the X keys of the regions, concatenated in shard order -> out
int launch_keys_compact(const uint64_t* keys, int64_t cap, const int64_t* xs, int64_t X, uint64_t* out,
                        hipStream_t s);

// steps whose window pass can test packed records (connect.h): the planes
// below idx fit 29 bits beside 3 flag bits, the planes idx .. K-1 32 bits
__host__ __device__ inline bool packed_ok(int idx, int K) { return idx >= 1 && idx <= 29 && K - idx <= 32; }
struct ConnectWin {
  int idx, nb;
  uint64_t fmask;
  uint64_t* keys;
  int64_t cap;
  int64_t* xs;
  int64_t* bstat;  // small grids (xs == null): per-bucket statistics [NB][4] that launch_connect sums
  int packed;      // 1: the LDS-record path tests packed records (connect.h packed_ok(idx, K))
};
int launch_bucket_pairs(const BucketGeom& g, const int64_t* bbase, const uint64_t* ekv, const uint64_t* pz,
                        CellEnt* ents, int32_t* pcell, int32_t* pent, int32_t* pn, int64_t* ptoff, int32_t* bcell,
                        int64_t bcap, int32_t* bcount, int32_t* bcur, const ConnectWin* win, int64_t* ctr,
                        hipStream_t s, int32_t* perm = nullptr);  // perm: T int32 scratch (LDS-record path; null: off)
constexpr int64_t PCK_CELLS = 1 << 24;  // CTR_PCK: cell count field
// pair indices per k_connect chunk (its bcell table granularity)
int64_t connect_chunk_pairs();
// window pass over the cell-contiguous entries (count ctr[CTR_T]): every
// pair of a cell of <= WCELL members, same emission rules and counters as
// launch_connect
int launch_connect_win(const CellEnt* ent, int idx, int nb, uint64_t fmask, uint64_t* keys, int64_t cap,
                       int64_t* xs, int64_t* ctr, hipStream_t s);

// ---- sort.hip ----
// ascending LSD radix sort of n u64 keys on bits [0, bits); the sorted keys
// end in *out (== a or b)
size_t sort_scratch_bytes(int64_t n, int bits);
size_t sort_pairs_scratch_bytes(int64_t n, int bits);
// (u32 key, i32 value) pairs ascending by key bits [0, bits); stable; the
// sorted arrays end in *ko / *vo (== the a or b buffers)
int sort_pairs_u32(uint32_t* ka, uint32_t* kb, int32_t* va, int32_t* vb, int64_t n, int bits,
                   void* scratch, size_t scratch_bytes, uint32_t** ko, int32_t** vo, hipStream_t s);
int sort_keys_u64(uint64_t* a, uint64_t* b, int64_t n, int bits, void* scratch, size_t scratch_bytes,
                  uint64_t** out, hipStream_t s);
// connecting-edge keys lo << nb | hi in lexicographic order: the lo half
// radix-sorted, then each run of equal lo ordered by hi (runs of <= R keys
// in one pass, longer ones one workgroup each); R <= 0 or n within the merge
// sort's range: sort_keys_u64 on all 2 nb bits
size_t sort_lex_scratch_bytes(int64_t n, int nb, int R);
int sort_keys_lex(uint64_t* a, uint64_t* b, int64_t n, int nb, int R, void* scratch, size_t scratch_bytes,
                  uint64_t** out, hipStream_t s);
// the final (non-pruning) step's edge list [edges; e_new; c_new] with
// prune = 0 (emit must be true; the pruning steps use launch_prune_lb)
int launch_prune(bool emit, const int32_t* edges, int64_t E, const int32_t* sb, int64_t S,
                 int64_t V, const uint64_t* ckeys, int nb, int64_t X, int idx,
                 int prune, int last_plane, const uint64_t* pos, const uint64_t* zero,
                 int32_t* blk, const int64_t* blkoff, int32_t* out, int32_t* used, int64_t* ctr,
                 hipStream_t s);
int launch_gather_vertices(const int32_t* used, const int64_t* nid, int64_t NV, int K,
                           int keep_from, const float* xyz, const float* pre, int64_t ld,
                           const uint64_t* pos, const uint64_t* zero, const uint64_t* grid,
                           float* xyz2, float* pre2, int64_t ld2, uint64_t* pos2, uint64_t* zero2,
                           uint64_t* grid2, uint64_t* pz2, hipStream_t s);
int launch_remap_edges(int32_t* edges, int64_t E, const int64_t* nid, hipStream_t s);


// ---- surface.hip ----
int launch_surface_flags(const float* xyz, const float* col, int64_t V, float eps, int32_t* on,
                         hipStream_t s);
int launch_surface_edges(const int32_t* edges, int64_t E, const int32_t* on, int32_t* blk,
                         const int64_t* blkoff, int emit, int32_t* out, int32_t* used,
                         hipStream_t s);

// ---- curve.hip (force=False branch) ----
int launch_curve_flags(const int32_t* sa, const int32_t* sb, int64_t S, const float* xyz, float eps,
                       int32_t* cflag, hipStream_t s);
int launch_curve_rows(const int32_t* cflag, const int64_t* coff, int64_t S, int32_t* crow,
                      hipStream_t s);
int launch_curve_corners(const int32_t* crow, int64_t B, const int32_t* sa, const int32_t* sb,
                         const float* xyz, const uint64_t* zero, const uint64_t* grid, int idx, float* corners,
                         int32_t* plane, int64_t* ctr, int kw, hipStream_t s);
int launch_curve_solve(int64_t B, const float* stage_c, int64_t ldc, const int32_t* plane, int idx,
                       const int32_t* crow, const int32_t* sa, const int32_t* sb, const float* xyz,
                       float* ints, float* pts, hipStream_t s);
int launch_curve_dnew(int64_t B, const float* stage_p, int64_t ldp, const int32_t* plane, int idx,
                      const float* ints, float eps, float* d0s, float* d1s, int32_t* gg, int32_t* gd,
                      hipStream_t s);
int launch_gd_rows(const int32_t* gd, const int64_t* goff, int64_t B, int32_t* glist, hipStream_t s);
struct NetDev;
int launch_descend(const NetDev& net, int64_t G, const int32_t* glist, const int32_t* crow,
                   const int32_t* sa, const int32_t* sb, const float* xyz, const int32_t* plane,
                   int idx, float eps, int iters, int record, float* ints, float* d0s, float* d1s,
                   unsigned long long* conv, hipStream_t s);
int launch_curve_apply(int64_t B, const int32_t* crow, const int32_t* sa, const int32_t* sb,
                       float* xyz, int64_t V, const float* ints, const float* d0s, const int32_t* gg,
                       float eps, int32_t* cinfo, int64_t* ctr, hipStream_t s);
int launch_strict_keep(int64_t S, const int32_t* cinfo, const float* stage, int idx, int override_,
                       const uint64_t* shared, float eps, int tight, int strict, int32_t* keep, int kw, hipStream_t s);
int launch_compact_splits(int64_t S, int K, const int32_t* keep, const int64_t* nid,
                          const int32_t* eidx, int64_t V, const int32_t* sa, const int32_t* sb,
                          const uint64_t* shared, const float* stage, const float* xyz,
                          const uint64_t* grid, int64_t S2, int32_t* sa2, int32_t* sb2,
                          uint64_t* shared2, float* stage2, float* xyz2, uint64_t* grid2,
                          int32_t* edges, int kw, hipStream_t s);
