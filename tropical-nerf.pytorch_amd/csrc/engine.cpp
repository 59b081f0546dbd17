// Host side of the extraction engine: device-resident complex, buffer
// management and the per-step launch sequence (C ABI in
// include/tropical_hip.h).  One engine = one device = one HIP stream per
// call; all scratch is stream-ordered (hipMallocAsync) and reused across
// steps.  Host syncs per active step: split count, hit count, cell entries,
// pair count, final sizes (each one pinned readback of the counter block).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/tropical_hip.h"
#include "../../include/tropical_hip_debug.h"
#include "common.h"
#include "kernels.h"
#include "step.h"

static thread_local std::string g_err;

void tnp_set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

extern "C" const char* tnp_last_error(void) { return g_err.c_str(); }
extern "C" int tnp_abi_version(void) { return TNP_ABI_VERSION; }
extern "C" int tnp_device_count(int* n) {
  TNP_CHECK(hipGetDeviceCount(n));
  return 0;
}

// ---------------------------------------------------------------------------
// small utility kernels (layout conversion)
// ---------------------------------------------------------------------------
namespace {

__global__ void k_i64_to_i32(const int64_t* __restrict__ in, int32_t* __restrict__ out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)in[i];
}
__global__ void k_i32_to_i64(const int32_t* __restrict__ in, int64_t* __restrict__ out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i];
}
// row-major [n][K] <-> plane-major [K][ld]
__global__ void k_rows_to_planes(const float* __restrict__ in, int64_t n, int K, float* __restrict__ out,
                                 int64_t ld) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int p = 0; p < K; ++p) out[(int64_t)p * ld + i] = in[i * K + p];
}
__global__ void k_planes_to_rows(const float* __restrict__ in, int64_t ld, int64_t n, int K,
                                 float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int p = 0; p < K; ++p) out[i * K + p] = in[(int64_t)p * ld + i];
}

}  // namespace

// ---------------------------------------------------------------------------
// buffers
// ---------------------------------------------------------------------------
struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
};

// the capacity buf_ensure grows a buffer of `have` bytes to for a request of
// `bytes`: geometric (x1.5), in whole 256-B units
static size_t buf_grow_bytes(size_t have, size_t bytes) {
  const size_t nb = std::max(bytes, have + have / 2);
  return std::max<size_t>((nb + 255) & ~size_t(255), 256);
}

// the connect phase's key capacity (keys) for a step of M members, given the
// key buffer's current size: XS_N equal per-XCD regions.  The capacity the
// buffer already holds is rounded DOWN to the regions (so it never asks for
// more than the buffer has -- round 4's 1.5x-per-step growth to 44 GB came
// from rounding it up); only the floor of 4 M + 1024 keys is rounded up.
static int64_t connect_key_cap(size_t have_bytes, int64_t M, int xs_n) {
  const int64_t have = (int64_t)(have_bytes / sizeof(uint64_t)) / xs_n * xs_n;
  const int64_t floor = (4 * M + 1024 + xs_n - 1) / xs_n * xs_n;
  return std::max(have, floor);
}

static int buf_ensure(Buf& b, size_t bytes, hipStream_t s, bool keep = false) {
  if (bytes <= b.bytes && b.p) return 0;
  const size_t nb = buf_grow_bytes(b.bytes, bytes);
  void* p = nullptr;
  if (hipMallocAsync(&p, nb, s) != hipSuccess) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    tnp_set_error("hipMallocAsync of %zu bytes (buffer of %zu, %zu requested): out of memory, %zu of %zu free",
                  nb, b.bytes, bytes, fr, tot);
    return -1;
  }
  if (keep && b.p && b.bytes) TNP_CHECK(hipMemcpyAsync(p, b.p, b.bytes, hipMemcpyDeviceToDevice, s));
  if (b.p) TNP_CHECK(hipFreeAsync(b.p, s));
  b.p = p;
  b.bytes = nb;
  return 0;
}
static void buf_free(Buf& b, hipStream_t s) {
  if (b.p) (void)hipFreeAsync(b.p, s);
  b.p = nullptr;
  b.bytes = 0;
}

template <typename T>
static T* P(Buf& b) { return static_cast<T*>(b.p); }

struct VSet {
  Buf xyz, pre, grid;
  // the vertex keys, (pos, zero) interleaved: 2 kw words per vertex, one
  // gather for both; the kernels' pos / zero arrays are views of it (VP / VZ,
  // common.h vkey_load)
  Buf pz;
  int64_t cap = 0;  // rows; pre leading dimension == cap
  int K = 0;        // planes the pre buffer holds (the engine is reused across nets)
};
// the pos / zero key views of a vertex set from vertex `from` on
static uint64_t* VP(VSet& v, int kw, int64_t from = 0) { return static_cast<uint64_t*>(v.pz.p) + 2 * kw * from; }
static uint64_t* VZ(VSet& v, int kw, int64_t from = 0) { return VP(v, kw, from) + kw; }

struct KRec {
  const char* name;
  double bytes;
  hipEvent_t a, b;
};

// curve-path scratch (force=False branch, curve.hip)
enum {
  CV_EIDX, CV_CFLAG, CV_COFF, CV_CROW, CV_CORNERS, CV_PLANE, CV_STAGE_C, CV_INTS, CV_INTS0, CV_PTS,
  CV_STAGE_P, CV_D0, CV_D1, CV_GG, CV_GD, CV_GOFF, CV_GLIST, CV_CONV, CV_CINFO, CV_KEEP, CV_NID,
  CV_SA2, CV_SB2, CV_SHARED2, CV_STAGE2, CV_XYZ2, CV_GRID2, CV_N
};

struct tnp_engine {
  int device = 0;
  OwnBox own{{1, 1, 1}, {0, 0, 0}};  // owned box of a shard (common.h); uncut axes: all
  // mark planes the complex lies within, per axis (the spatial buckets cover
  // only those cells); sp_hi[d] < sp_lo[d]: the whole axis
  int sp_lo[3] = {0, 0, 0}, sp_hi[3] = {-1, -1, -1};
  int curve = 0;          // 1: subpoly_(force=False) semantics
  int strict = 1;         // curve path: subpoly_(strict=...) -- 0 keeps every split (subpoly.py:198-202)
  int shards = 1;         // >1: one x-slab of a sharded complex
  int pend_tight = 0;
  tnp_collective_fn coll_fn = nullptr;  // a sharded step's in-step decisions (tnp_engine_set_collective)
  void* coll_ctx = nullptr;
  bool coll_err = false;  // this shard failed: the next collective says so (coll_fail)
  int gd_iters = 500;     // subpoly_debug.py:141
  int64_t max_pair_tests = 20000000000LL;
  bool kt_on = false;
  std::vector<KRec> kt;
  std::vector<std::string> kt_names;
  std::vector<double> kt_ms, kt_bytes;
  std::vector<int64_t> kt_n;
  NetDev net{};
  int K = 0;
  int kw = 1;  // sign-key words per vertex key (net_kw: 2 when K > 63)
  bool has_net = false;
  VSet cur, alt;
  Buf edges, edges_alt;
  // per-edge key bytes (step.hip k_prune_lb): dm = 1 + the highest plane on
  // which the endpoint keys differ, ef = the first plane >= mask_from that
  // splits the edge (EDGE_NOSPLIT: none); valid when masks_valid
  Buf edm, eef, edm_alt, eef_alt;
  Buf lzpart;  // the lazy prune's per-workgroup kept counts
  Buf kse[3];  // split-eps faces: pos / zero / grid keys at subpoly's eps
  Buf xs;                // per-XCD shards of the connect phase (step.h XS_*)
  bool xs_clean = false;
  bool masks_valid = false;
  int mask_from = 0;       // plane the stored first split planes start at
  uint64_t act_bits = 0;   // OR of the edges' first split planes (bit p: plane p splits an edge)
  int64_t V = 0, E = 0;
  // E counts edge SLOTS: the pruning deletes lazily (EDGE_DEAD bytes, edges
  // keep their slots) and compacts only when most slots are dead or before
  // an export; E_live is the reference's edge count
  int64_t E_live = 0;
  int keep_all = 0;
  int valid_from = 0;  // pre planes [valid_from, K) are valid for every vertex
  int pend_keep = 0;   // the pending flat step's new vertices get planes [pend_keep, K) (new_keep_from)
  // Lazy compaction: during the hot loop vertex ids are SLOTS (V = slots in
  // use); pruned vertices stay in place, flagged dead in `used` (the live
  // flags).  Slot order == the reference's compacted id order (compaction
  // preserves ascending ids), so every id-ordered result is unchanged;
  // compact_now() renumbers once, before anything exports or reads ids.
  bool dirty = false;
  // a complex is loaded and consistent: a failed split / finish (an error
  // the reference raises mid-step, or a device failure) leaves the edges and
  // live flags half-updated, so the engine refuses to go on until a complex
  // is loaded again (tnp_engine_load / lattice / skeleton)
  bool valid = false;
  int64_t V_live = 0;
  Buf live;  // live-slot flags (uint8) of the lazily compacted vertex set
  // deferred live counts (tnp_engine_run_steps): a pruning step leaves
  // V_live (and, lazy prune, E_live) to the next split, whose hit workers read
  // every live flag anyway (HitArgs::hpart) and whose readback sums them
  // with the lazy prune's per-workgroup kept counts -- no count_live launch
  bool defer_counts = false;  // set by the run loop only
  bool cnt_pending = false;
  bool defer_ok = true;               // TNP_DEFER_COUNTS=0: count in the finish (A/B)
  bool early_forward = true;          // TNP_EARLY_FWD=0: k_forward_new after S is read back (A/B)
  // the early k_forward_new's row bound (early_bound): the largest split
  // count this engine has seen, not the edge-slot count E -- E counts the
  // lazily deleted slots too (up to ~2x the live edges), and the vertex set
  // and the shared-plane words keep whatever capacity the bound asks for
  int64_t max_split_seen = 0;
  int64_t n_early_redo = 0;  // steps whose S exceeded the early bound (forward run again)
  // side stream: the lazy prune of the old edges and e_new runs there, beside
  // the grouping kernel and the connect on the caller's stream (finish);
  // ev_s2[0]: the caller's stream reached the prune's inputs, ev_s2[1]: the
  // prune is done (the caller's stream waits on it before anything touches
  // the edge slots again: side_join)
  hipStream_t s2 = nullptr;
  hipEvent_t ev_s2[2] = {nullptr, nullptr};
  bool s2_pending = false;
  // TNP_SIDE_PRUNE=1 at creation: part A on the side stream.  Off: measured
  // no faster (profiles/r06_ab_side_prune.jsonl: 3.71-3.75 ms per 128^3 pass
  // either way -- the two kernels slow each other down as much as they
  // overlap: bucket_group 0.80 -> 1.08 ms, the prune 0.63 -> 1.03 ms)
  bool side_prune = false;
  bool early_bound_splits = true;  // TNP_EARLY_BOUND=0 at creation: the edge-slot bound E (round 5, A/B)
  // the connecting-edge sort: lo half + run pass for runs of <= sort_run keys
  // (sort.hip sort_keys_lex); 0: all 2 nb bits by onesweep.  TNP_SORT_RUN at creation
  int sort_run = 64;
  int64_t pend_lz_n = 0;              // lzpart entries holding E_live (0: E_live is known)
  tnp_step_stats* pend_st = nullptr;  // the step whose V_out / E_out wait for them
  Buf hpart;                          // the hit workers' live counts
  // step scratch
  Buf spcnt, spoff, part, ekey_a, ekey_b, eval_b, sort_scr2;
  // (pcell/ptoff: compacted pair cells and their first pair; ents: CellEnt
  // records in cell order; used/nid/flags: int32 scratch of compaction,
  // surface and skeleton)
  Buf blk, blkoff, scan_scr, sa, sb, stage, shared, members, pcn, pent, rstart, ent_v,
      ents, pcell, ptoff, bcell, ckeys_a, ckeys_b, sort_scr, flags, used, nid, ctr;
  uint64_t* ckeys = nullptr;  // sorted connecting edges of the current step
  int64_t* h_ctr = nullptr;  // host copy of ctr (the last readback)
  int64_t* h_map = nullptr;  // host-mapped mirror written by k_publish ([31]: sequence)
  int64_t* h_map_dev = nullptr;
  int64_t pub_seq = 0;
  // tnp_engine_run_steps: a step's last readback zeroes the counter words
  // (k_publish clear), and the next split skips its memset -- one host API
  // call less per step (hipMemsetAsync costs the host ~5-9 us, the
  // bunny-scale loop is launch-bound, profiles/r06_small_hip_trace.txt).
  // ctr_zero: the words are zero since the last publish; any other
  // publish, launch into the words or engine call in between clears it
  bool in_run = false;
  bool ctr_zero = false;
  // pending split
  int pend_idx = -1;
  int64_t pend_S = 0, pend_dup = 0;
  bool pend_hits = false;   // the pending split also found the plane's hit vertices
  int64_t pend_hoff = -1;   // ... at members[pend_hoff] (the split's E; -1: after the S new members)
  bool pend_fused = false;  // the pending split ran k_forward_new (flat path)
  // faces output
  Buf tri, faces;
  Buf tied_table;  // level-interleaved copy of the caller's table (NetDev::tied)
  int64_t n_tri = 0, n_faces = 0, dbg_F = 0, dbg_W = 0;
  // look-back states (a kernel may run two chains): [0] ticket counter,
  // [1..] tile status words; tickets issued so far; launch epoch
  Buf lb[2];
  uint64_t lb_tickets[2] = {0, 0};
  uint32_t lb_epoch[2] = {0, 0};
  int32_t lb_spin = -1;  // TNP_LB_SPIN: ticket-free look-back polls (0 forces the recompute path)
  Buf lbrc;              // look-back recompute counter (tnp_engine_debug_lb_recomputes)
  Buf fscr[12];
  Buf fscr2[32];
  Buf sents;                // bucket-ordered packed entries before the in-bucket grouping
  Buf sents2;               // ... regrouped by octant (two-level bucket geometries, bk[8]: their bases)
  Buf bk[14];               // bucket.hip scratch (per-bucket counts, bases, pair-cell areas)
  bool radix_cells = false; // TNP_RADIX_CELLS=1: the radix-sort bucketing path
  bool lazy_edges = true;   // TNP_LAZY_EDGES=0: every pruning step compacts the edge list
  bool lds_records = true;  // TNP_LDS_RECORDS=0: the grouping's records go through memory
  bool packed_records = true;  // TNP_PACKED_RECORDS=0: the LDS records stay 32-B CellEnt
  bool bk_clean = false;    // bucket counters (bk[0], bk[1]) are zero
  Buf cv[CV_N];
};

// the counter block is cleared as 32 words: a 248-byte memset takes two fill
// dispatches (aligned body + tail), 256 bytes one
constexpr size_t CTR_CLEAR_BYTES = 32 * sizeof(int64_t);
static_assert(CTR_N <= 32, "counter block");

// counter readback: k_publish writes the block into host-mapped memory and
// the host spins on its sequence word (measured on MI355X: 9.9 us per round
// trip against 15.7 us for a copy + stream synchronise); after 2 ms of
// spinning (long kernels) it blocks in the stream synchronise instead
// vpart != null: the published CTR_V (and CTR_E when ne > 0) are the sums of
// vpart[nv] / epart[ne] (the deferred live counts), not the device words
// (post_ctr enqueues the publish, wait_ctr takes it: work enqueued between
// the two runs on the GPU while the counters travel to the host)
static int post_ctr(tnp_engine* e, hipStream_t s, int64_t* seq_out, const int64_t* vpart = nullptr, int nv = 0,
                    const int64_t* epart = nullptr, int ne = 0, bool clear = false) {
  const int64_t seq = ++e->pub_seq;
  if (vpart ? launch_publish_sums(P<int64_t>(e->ctr), e->h_map_dev, seq, vpart, nv, epart, ne, s)
            : launch_publish(P<int64_t>(e->ctr), e->h_map_dev, seq, s, clear))
    return -1;
  e->ctr_zero = clear && !vpart;
  *seq_out = seq;
  return 0;
}
static int wait_ctr(tnp_engine* e, hipStream_t s, int64_t seq) {
  volatile int64_t* flag = e->h_map + 31;
  const auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  while (*flag != seq) {
    if ((++n & 255) == 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
      TNP_CHECK(hipStreamSynchronize(s));
      if (*flag != seq) { tnp_set_error("counter readback: no publish after the stream drained"); return -1; }
      break;
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  memcpy(e->h_ctr, (const void*)e->h_map, CTR_N * sizeof(int64_t));
  return 0;
}
static int read_ctr(tnp_engine* e, hipStream_t s, const int64_t* vpart = nullptr, int nv = 0,
                    const int64_t* epart = nullptr, int ne = 0, bool clear = false) {
  int64_t seq = 0;
  return post_ctr(e, s, &seq, vpart, nv, epart, ne, clear) || wait_ctr(e, s, seq) ? -1 : 0;
}

// the deferred live counts arrived (V_live, E_live; E_live < 0: unchanged)
static void apply_counts(tnp_engine* e, int64_t V_live, int64_t E_live) {
  e->V_live = V_live;
  if (e->pend_lz_n > 0) e->E_live = E_live;
  if (e->pend_st) {
    e->pend_st->V_out = e->V_live;
    e->pend_st->E_out = e->E_live;
  }
  e->cnt_pending = false;
  e->pend_lz_n = 0;
  e->pend_st = nullptr;
}

// the deferred counts now, by the counting pass (a split without hit
// workers, the end of the run loop, any other caller); the counter words
// CTR_V / CTR_E are still zero from the last split's reset
static int resolve_counts(tnp_engine* e, hipStream_t s) {
  if (!e->cnt_pending) return 0;
  int64_t* ctr = P<int64_t>(e->ctr);
  if (launch_count_flags(P<uint8_t>(e->live), e->V, ctr, CTR_V, s, e->pend_lz_n ? P<int64_t>(e->lzpart) : nullptr,
                         (int)e->pend_lz_n, CTR_E))
    return -1;
  if (read_ctr(e, s)) return -1;
  apply_counts(e, e->h_ctr[CTR_V], e->h_ctr[CTR_E]);
  return 0;
}

// ---- per-kernel HIP-event timer (bench.py's roofline leg) -----------------
static int ktimer_begin(tnp_engine* e, const char* name, double bytes, hipStream_t s) {
  if (!e->kt_on) return -1;
  KRec r;
  r.name = name;
  r.bytes = bytes;
  if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) return -1;
  (void)hipEventRecord(r.a, s);
  e->kt.push_back(r);
  return (int)e->kt.size() - 1;
}
// bytes of the encoding tables (2 fp32 features per entry)
static double table_bytes(const NetDev& n) {
  double b = 0;
  for (int l = 0; l < n.n_levels; ++l) b += 8.0 * n.sizes[l];
  return b;
}
// modelled bytes of the last timed launch, when they depend on its result
static void ktimer_set_bytes(tnp_engine* e, double bytes) {
  if (e->kt_on && !e->kt.empty()) e->kt.back().bytes = bytes;
}
// ... of the latest timed launch named `name` (counts read back later)
static void ktimer_set_bytes(tnp_engine* e, const char* name, double bytes) {
  if (!e->kt_on) return;
  for (size_t i = e->kt.size(); i-- > 0;)
    if (strcmp(e->kt[i].name, name) == 0) {
      e->kt[i].bytes = bytes;
      return;
    }
}
static void ktimer_end(tnp_engine* e, int t, hipStream_t s) {
  if (t >= 0) (void)hipEventRecord(e->kt[t].b, s);
}
#define TIMED(name, bytes, call)                                   \
  do {                                                             \
    int _t = ktimer_begin(e, name, (double)(bytes), s);            \
    if (call) return -1;                                           \
    ktimer_end(e, _t, s);                                          \
  } while (0)

// look-back state `w` for a single-pass launch of `tiles` tiles (common.h TnpLB)
// (`ticketed` false: the kernel numbers tiles by blockIdx and takes no ticket)
static int lb_begin(tnp_engine* e, int64_t tiles, hipStream_t s, TnpLB* out, int w = 0,
                    bool ticketed = true) {
  Buf& b = e->lb[w];
  size_t need = (size_t)(tiles + 1) * sizeof(uint64_t);
  if (need > b.bytes || !b.p) {
    if (buf_ensure(b, std::max(need, (size_t)64 << 10), s)) return -1;
    TNP_CHECK(hipMemsetAsync(b.p, 0, b.bytes, s));  // flag 0: no record
    e->lb_tickets[w] = 0;
  }
  e->lb_epoch[w] = (e->lb_epoch[w] + 1) & 0x3FFFFFu;
  if (e->lb_epoch[w] == 0) {  // wrapped: clear records that could carry a reused epoch
    TNP_CHECK(hipMemsetAsync(b.p, 0, b.bytes, s));
    e->lb_tickets[w] = 0;
    e->lb_epoch[w] = 1;
  }
  out->ticket = static_cast<unsigned long long*>(b.p);
  out->st = static_cast<uint64_t*>(b.p) + 1;
  out->tbase = e->lb_tickets[w];
  out->epoch = e->lb_epoch[w];
  out->spin = e->lb_spin;
  if (!e->lbrc.p) {
    if (buf_ensure(e->lbrc, sizeof(uint64_t), s)) return -1;
    TNP_CHECK(hipMemsetAsync(e->lbrc.p, 0, sizeof(uint64_t), s));
  }
  out->rc = static_cast<unsigned long long*>(e->lbrc.p);
  if (ticketed) e->lb_tickets[w] += (uint64_t)tiles;
  return 0;
}

static int scan_counts(tnp_engine* e, const int32_t* in, int64_t* out, int64_t n, int slot,
                       hipStream_t s) {
  TnpLB lb;
  if (n > 0 && lb_begin(e, scan_tiles(n), s, &lb, 0, false)) return -1;
  TIMED("scan", 12.0 * n, scan_i32_to_i64(in, out, n, P<int64_t>(e->ctr) + slot, lb, s));
  return 0;
}

// grow a vertex set to `rows` keeping [0, keep_rows)
static int vset_ensure(tnp_engine* e, VSet& v, int64_t rows, int64_t keep_rows, hipStream_t s) {
  if (rows <= v.cap && v.K == e->K) return 0;
  // another net: nothing of the old set is kept, and its capacity is no
  // growth history (alternating nets must not compound the 1.5x)
  const bool same = v.K == e->K;
  if (!same) keep_rows = 0;
  int64_t nc = same ? std::max<int64_t>(rows, v.cap + v.cap / 2) : rows;
  nc = (nc + 255) / 256 * 256;
  VSet n;
  n.cap = nc;
  n.K = e->K;
  if (buf_ensure(n.xyz, nc * 3 * sizeof(float), s)) return -1;
  if (buf_ensure(n.pre, (size_t)nc * e->K * sizeof(float), s)) return -1;
  const int64_t kb = 8 * e->kw;  // bytes per key
  if (buf_ensure(n.grid, nc * sizeof(uint64_t), s)) return -1;
  if (buf_ensure(n.pz, nc * 2 * kb, s)) return -1;
  if (keep_rows > 0 && v.cap > 0) {
    TNP_CHECK(hipMemcpyAsync(n.xyz.p, v.xyz.p, keep_rows * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
    TNP_CHECK(hipMemcpy2DAsync(n.pre.p, nc * sizeof(float), v.pre.p, v.cap * sizeof(float),
                               keep_rows * sizeof(float), e->K, hipMemcpyDeviceToDevice, s));
    TNP_CHECK(hipMemcpyAsync(n.grid.p, v.grid.p, keep_rows * 8, hipMemcpyDeviceToDevice, s));
    TNP_CHECK(hipMemcpyAsync(n.pz.p, v.pz.p, keep_rows * 2 * kb, hipMemcpyDeviceToDevice, s));
  }
  buf_free(v.xyz, s);
  buf_free(v.pre, s);
  buf_free(v.grid, s);
  buf_free(v.pz, s);
  v = n;
  return 0;
}

static int keys_for(tnp_engine* e, VSet& v, int64_t from, int64_t n, hipStream_t s) {
  return launch_keys(e->net, P<float>(v.xyz) + 3 * from, P<float>(v.pre) + from, v.cap, n, e->K,
                     VP(v, e->kw, from), VZ(v, e->kw, from), P<uint64_t>(v.grid) + from, s,
                     VP(v, e->kw, from));
}

// live flags of slots [from, from + n) := 1 (kept capacity: earlier flags stay)
static int set_alive(tnp_engine* e, int64_t from, int64_t n, hipStream_t s) {
  if (buf_ensure(e->live, std::max<int64_t>(from + n, 16), s, true)) return -1;
  const FillOp f{P<uint8_t>(e->live) + from, (uint64_t)std::max<int64_t>(n, 0), 1};
  if (launch_fill(&f, 1, s)) return -1;
  return 0;
}

// a freshly loaded complex: every slot live, ids dense, edge masks to compute
static int reset_live(tnp_engine* e, hipStream_t s, bool edges_changed = true) {
  if (edges_changed) e->masks_valid = false;
  e->valid = true;
  e->dirty = false;
  e->V_live = e->V;
  return set_alive(e, 0, e->V, s);
}

// the cell grouping runs on spatial buckets (bucket.hip) unless the grid is
// too fine for them or TNP_RADIX_CELLS=1; *bg: their geometry
static void span_all(tnp_engine* e) {
  for (int d = 0; d < 3; ++d) e->sp_lo[d] = 0, e->sp_hi[d] = -1;
}
// the span's mark planes along each axis (the whole axis where not narrowed)
static void span_of(const tnp_engine* e, int lo[3], int hi[3]) {
  for (int d = 0; d < 3; ++d) {
    const bool set = e->sp_hi[d] >= e->sp_lo[d];
    lo[d] = set ? e->sp_lo[d] : 0;
    hi[d] = set ? e->sp_hi[d] : e->net.n_marks - 1;
  }
}
static bool uses_buckets(const tnp_engine* e, BucketGeom* bg) {
  if (e->kw != 1) return false;  // two-word keys: the radix path's 48-B records
  int lo[3], hi[3];
  span_of(e, lo, hi);
  return !e->radix_cells && bucket_geometry(e->net.n_marks, lo, hi, bg) == 0;
}

// split-eps mode: subpoly's eps argument differs from Net.eps (tnp_engine_set_eps)
static bool eps2(const tnp_engine* e) { return e->net.eps_s != e->net.eps; }

// the cache planes a flat step at plane idx stores for its new vertices:
// those a later step, the surface (plane K - 1) or an export can read.  In the
// hot loop that is planes > idx (the step's pruning moves valid_from to
// idx + 1; the last plane always) -- not [valid_from, idx], dead the moment
// the step ends (up to 15 of 33 planes a split at 128^3).  A caller that
// hands outputs_ back (keep_all) or the split-eps mode keeps every plane.
static int new_keep_from(const tnp_engine* e, int idx) {
  if (e->keep_all || eps2(e)) return e->valid_from;
  return std::max(e->valid_from, std::min(idx + 1, e->K - 1));
}

// per-edge high plane and first split plane (>= from) from the endpoint
// keys; ctr != null: the OR of the first split planes -> ctr[CTR_ACTIVE]
static int compute_masks(tnp_engine* e, int from, int64_t* ctr, hipStream_t s) {
  const int64_t E1 = std::max<int64_t>(e->E, 1);
  if (buf_ensure(e->edm, E1 * sizeof(uint8_t), s)) return -1;
  if (buf_ensure(e->eef, E1 * sizeof(uint8_t), s)) return -1;
  TIMED("edge_masks", 42.0 * e->E,
        launch_edge_masks(P<int32_t>(e->edges), e->E, P<uint64_t>(e->cur.pz), P<uint8_t>(e->edm),
                          P<uint8_t>(e->eef), from, e->K - 1, e->cnt_pending || e->E != e->E_live, ctr, s));
  if (eps2(e)) {
    // first split planes at subpoly's eps from the cached planes (the mode
    // keeps them all): they replace the Net.eps ones and their OR
    if (e->valid_from > from) {
      tnp_set_error("split-eps masks from plane %d: planes below %d were dropped", from, e->valid_from);
      return -1;
    }
    if (ctr) TNP_CHECK(hipMemsetAsync(ctr + CTR_ACTIVE, 0, sizeof(int64_t), s));
    TIMED("edge_masks", 8.0 * e->E,
          launch_ef_cache(P<int32_t>(e->edges), e->E, P<uint8_t>(e->edm), P<uint8_t>(e->eef),
                          P<float>(e->cur.pre), e->cur.cap, from, e->K, e->net.eps_s, ctr, s));
  }
  e->masks_valid = true;
  e->mask_from = from;
  return 0;
}

// the masks a step at plane idx can use: the stored first split planes were
// taken from mask_from, so they are the ones of idx unless a plane in
// [mask_from, idx) still splits some edge (a step the caller skipped) --
// then they are recomputed from idx.  Returns 1 if recomputed (the OR of
// the first planes is then in ctr[CTR_ACTIVE], ctr zeroed by the caller).
// the active-plane word of the planes [lo, hi) (planes >= 63 share bit 63)
static uint64_t act_range(int lo, int hi) {
  uint64_t m = 0;
  for (int p = lo; p < hi && p < 63; ++p) m |= 1ull << p;
  if (hi > 63 && hi > lo) m |= 1ull << 63;
  return m;
}

static int ensure_masks(tnp_engine* e, int idx, hipStream_t s) {
  if (e->masks_valid && idx >= e->mask_from && (e->act_bits & act_range(e->mask_from, idx)) == 0) return 0;
  return compute_masks(e, idx, P<int64_t>(e->ctr), s) ? -1 : 1;
}

// drop the lazily deleted edges, live ones in order (the compacting prune
// keeping every live edge: idx = -1)
static int compact_edges(tnp_engine* e, hipStream_t s) {
  if (e->E == e->E_live) return 0;
  const int64_t E = e->E, E1 = std::max<int64_t>(E, 1);
  if (buf_ensure(e->edges_alt, E1 * 2 * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->edm_alt, E1 * sizeof(uint8_t), s)) return -1;
  if (buf_ensure(e->eef_alt, E1 * sizeof(uint8_t), s)) return -1;
  TnpLB lb;
  if (lb_begin(e, lb_tiles(E), s, &lb, 0, false)) return -1;
  TIMED("compact_edges", 12.0 * E,
        launch_prune_lb(P<int32_t>(e->edges), E, nullptr, 0, e->V, nullptr, 0, 0, -1, e->K - 1,
                        P<uint64_t>(e->cur.pz), P<uint8_t>(e->edm), P<uint8_t>(e->eef), P<int32_t>(e->edges_alt),
                        P<uint8_t>(e->edm_alt), P<uint8_t>(e->eef_alt), P<uint8_t>(e->live), false,
                        P<int64_t>(e->ctr), lb, s));
  std::swap(e->edges, e->edges_alt);
  std::swap(e->edm, e->edm_alt);
  std::swap(e->eef, e->eef_alt);
  if (read_ctr(e, s)) return -1;
  if (e->h_ctr[CTR_E] != e->E_live) {
    tnp_set_error("edge compaction: %lld live edges, %lld expected", (long long)e->h_ctr[CTR_E],
                  (long long)e->E_live);
    return -1;
  }
  e->E = e->E_live;
  return 0;
}

// renumber the live slots densely (the reference's per-step compaction,
// subpoly.py:266-277, done once): scan of the live flags, gather of the
// vertex rows (planes >= valid_from), edge remap
static int compact_now(tnp_engine* e, hipStream_t s) {
  if (e->cnt_pending) {  // (run_steps resolves them on every exit; V_live / E_live would read stale)
    tnp_set_error("compaction with the live counts of the last step still pending");
    return -1;
  }
  if (compact_edges(e, s)) return -1;
  if (!e->dirty) return 0;
  const int64_t NV = e->V;
  if (buf_ensure(e->nid, std::max<int64_t>(NV, 1) * sizeof(int64_t), s)) return -1;
  if (buf_ensure(e->used, std::max<int64_t>(NV, 1) * sizeof(int32_t), s)) return -1;
  if (launch_widen_flags(P<uint8_t>(e->live), NV, P<int32_t>(e->used), s)) return -1;
  if (scan_counts(e, P<int32_t>(e->used), P<int64_t>(e->nid), NV, CTR_AUX, s)) return -1;
  if (vset_ensure(e, e->alt, NV, 0, s)) return -1;
  VSet& c = e->cur;
  VSet& a = e->alt;
  TIMED("gather_vertices", 4.0 * NV + 2.0 * (12 + 4.0 * (e->K - e->valid_from) + 24) * e->V_live,
        launch_gather_vertices(P<int32_t>(e->used), P<int64_t>(e->nid), NV, e->K, e->valid_from,
                               P<float>(c.xyz), P<float>(c.pre), c.cap, VP(c, e->kw),
                               VZ(c, e->kw), P<uint64_t>(c.grid), P<float>(a.xyz),
                               P<float>(a.pre), a.cap, VP(a, e->kw), VZ(a, e->kw),
                               P<uint64_t>(a.grid), P<uint64_t>(a.pz), s));
  TIMED("remap_edges", 32.0 * e->E, launch_remap_edges(P<int32_t>(e->edges), e->E, P<int64_t>(e->nid), s));
  if (read_ctr(e, s)) return -1;
  const int64_t V2 = e->h_ctr[CTR_AUX];
  if (V2 != e->V_live) {
    tnp_set_error("compaction: %lld live slots, %lld expected", (long long)V2, (long long)e->V_live);
    return -1;
  }
  std::swap(e->cur, e->alt);
  e->V = V2;
  return reset_live(e, s, false);  // same edges, same order: masks stay valid
}

static int require_valid(const tnp_engine* e, const char* what) {
  if (e->valid) return 0;
  tnp_set_error("%s: no consistent complex (none loaded, or a failed step left it half-updated); "
                "load one first (tnp_engine_load / lattice / skeleton)", what);
  return -1;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" int tnp_engine_create(tnp_engine** out, int device) {
  TNP_CHECK(hipSetDevice(device));
  tnp_engine* e = new tnp_engine();
  e->device = device;
  if (const char* lim = getenv("TNP_MAX_PAIR_TESTS")) e->max_pair_tests = atoll(lim);
  if (const char* rc = getenv("TNP_RADIX_CELLS")) e->radix_cells = atoi(rc) != 0;
  if (const char* lz = getenv("TNP_LAZY_EDGES")) e->lazy_edges = atoi(lz) != 0;
  if (const char* lr = getenv("TNP_LDS_RECORDS")) e->lds_records = atoi(lr) != 0;
  if (const char* pr = getenv("TNP_PACKED_RECORDS")) e->packed_records = atoi(pr) != 0;
  if (const char* sp = getenv("TNP_LB_SPIN")) e->lb_spin = atoi(sp);
  if (const char* dc = getenv("TNP_DEFER_COUNTS")) e->defer_ok = atoi(dc) != 0;
  if (const char* ef = getenv("TNP_EARLY_FWD")) e->early_forward = atoi(ef) != 0;
  if (const char* eb = getenv("TNP_EARLY_BOUND")) e->early_bound_splits = atoi(eb) != 0;
  if (const char* sr = getenv("TNP_SORT_RUN")) e->sort_run = atoi(sr);
  if (const char* sp = getenv("TNP_SIDE_PRUNE")) e->side_prune = atoi(sp) != 0;
  if (hipHostMalloc((void**)&e->h_ctr, CTR_N * sizeof(int64_t), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&e->h_map, 32 * sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&e->h_map_dev, e->h_map, 0) != hipSuccess) {
    if (e->h_ctr) (void)hipHostFree(e->h_ctr);
    if (e->h_map) (void)hipHostFree(e->h_map);
    delete e;
    tnp_set_error("hipHostMalloc failed");
    return -1;
  }
  memset((void*)e->h_map, 0, 32 * sizeof(int64_t));
  *out = e;
  return 0;
}

// every device buffer the engine owns (destroy, tnp_engine_scratch_bytes)
template <typename F>
static void for_each_buf(tnp_engine* e, F&& f) {
  for (VSet* v : {&e->cur, &e->alt})
    for (Buf* b : {&v->xyz, &v->pre, &v->grid, &v->pz}) f(*b);
  Buf* bufs[] = {&e->edges, &e->edges_alt, &e->blk, &e->blkoff, &e->scan_scr, &e->sa, &e->sb,
                 &e->stage, &e->shared, &e->members, &e->pcn, &e->pent, &e->rstart,
                 &e->ent_v, &e->ents, &e->pcell, &e->ptoff, &e->bcell,
                 &e->ckeys_a, &e->ckeys_b, &e->sort_scr, &e->flags, &e->used, &e->nid,
                 &e->ctr, &e->tri, &e->faces, &e->lb[0], &e->lb[1], &e->edm, &e->eef,
                 &e->edm_alt, &e->eef_alt, &e->live, &e->tied_table, &e->xs, &e->lbrc, &e->lzpart,
                 &e->kse[0], &e->kse[1], &e->kse[2], &e->sents, &e->sents2,
                 &e->spcnt, &e->spoff, &e->part, &e->ekey_a, &e->ekey_b, &e->eval_b, &e->sort_scr2,
                 &e->hpart};
  for (Buf* b : bufs) f(*b);
  for (Buf& b : e->fscr) f(b);
  for (Buf& b : e->fscr2) f(b);
  for (Buf& b : e->bk) f(b);
  for (Buf& b : e->cv) f(b);
}

extern "C" void tnp_engine_destroy(tnp_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipDeviceSynchronize();
  if (e->s2) (void)hipStreamDestroy(e->s2);
  for (hipEvent_t ev : e->ev_s2)
    if (ev) (void)hipEventDestroy(ev);
  hipStream_t s = 0;
  for_each_buf(e, [&](Buf& b) { buf_free(b, s); });
  (void)hipDeviceSynchronize();
  if (e->h_ctr) (void)hipHostFree(e->h_ctr);
  delete e;
}

extern "C" int tnp_engine_scratch_bytes(tnp_engine* e, int64_t* bytes, int64_t* buffers, int64_t* key_bytes) {
  if (!e || !bytes) { tnp_set_error("tnp_engine_scratch_bytes: null argument"); return -1; }
  int64_t tot = 0, n = 0;
  for_each_buf(e, [&](Buf& b) { tot += (int64_t)b.bytes; n += b.p != nullptr; });
  *bytes = tot;
  if (buffers) *buffers = n;
  if (key_bytes) *key_bytes = (int64_t)e->ckeys_a.bytes;
  return 0;
}

extern "C" int tnp_engine_debug_vertex_capacity(tnp_engine* e, int64_t* rows, int64_t* early_redo) {
  if (!e || !rows || !early_redo) { tnp_set_error("tnp_engine_debug_vertex_capacity: null argument"); return -1; }
  *rows = e->cur.cap;
  *early_redo = e->n_early_redo;
  return 0;
}

extern "C" int tnp_debug_buf_growth(int64_t have_bytes, int64_t request_bytes, int64_t members, int xs_n,
                                    int64_t* grown_bytes, int64_t* key_cap) {
  if (have_bytes < 0 || request_bytes < 0 || members < 0 || xs_n < 1 || xs_n > 63) {
    tnp_set_error("tnp_debug_buf_growth: bad argument");
    return -1;
  }
  if (grown_bytes) *grown_bytes = (int64_t)buf_grow_bytes((size_t)have_bytes, (size_t)request_bytes);
  if (key_cap) *key_cap = connect_key_cap((size_t)have_bytes, members, xs_n);
  return 0;
}

static NetDev to_dev(const tnp_net* n) {
  NetDev d{};
  for (int l = 0; l < TNP_MAX_LEVELS; ++l) {
    d.scales[l] = n->scales[l];
    d.res[l] = n->res[l];
    d.sizes[l] = n->sizes[l];
    d.offsets[l] = n->offsets[l];
    d.dense[l] = n->dense[l];
  }
  d.table = n->d_table;
  d.weights = n->d_weights;
  d.marks = n->d_marks;
  d.n_levels = n->n_levels;
  d.num_layers = n->num_layers;
  d.num_hidden = n->num_hidden;
  d.n_marks = n->n_marks;
  d.eps = n->eps;
  d.eps_s = n->eps;
  return d;
}

static int check_net(const tnp_net* n) {
  if (!n) { tnp_set_error("null net"); return -1; }
  if (n->n_features != 2) { tnp_set_error("n_features must be 2"); return -1; }
  NetDev d = to_dev(n);
  if (!net_supported(d)) {
    tnp_set_error("net shape (levels=%d, layers=%d, hidden=%d) not instantiated", n->n_levels,
                  n->num_layers, n->num_hidden);
    return -1;
  }
  if (net_K(d) > 127) { tnp_set_error("more than 127 planes (two-word sign keys)"); return -1; }
  return 0;
}

// Levels with the same fp32 scale, resolution, table size and addressing
// (e.g. the synthetic lattice nets, r_min == r_max) share corner weights and
// hash indices: the engine keeps a level-interleaved copy of the table so a
// corner is one 16-B gather for two levels (net_device.h encode_tied).
static bool levels_tied(const tnp_net* n) {
  if (n->n_levels < 2 || n->n_levels % 2 != 0 || getenv("TNP_NO_TIED")) return false;
  for (int l = 1; l < n->n_levels; ++l)
    if (memcmp(&n->scales[l], &n->scales[0], sizeof(float)) != 0 || n->res[l] != n->res[0] ||
        n->sizes[l] != n->sizes[0] || n->dense[l] != n->dense[0])
      return false;
  return true;
}

extern "C" int tnp_engine_set_net(tnp_engine* e, const tnp_net* n) {
  if (check_net(n)) return -1;
  TNP_CHECK(hipSetDevice(e->device));
  e->net = to_dev(n);
  if (levels_tied(n)) {
    const int L = n->n_levels;
    const size_t entry = 2 * sizeof(float);
    if (buf_ensure(e->tied_table, (size_t)n->sizes[0] * L * entry, 0)) return -1;
    for (int l = 0; l < L; ++l)
      TNP_CHECK(hipMemcpy2DAsync(static_cast<char*>(e->tied_table.p) + l * entry, L * entry,
                                 n->d_table + 2 * (size_t)n->offsets[l], entry, entry, n->sizes[0],
                                 hipMemcpyDeviceToDevice, 0));
    TNP_CHECK(hipStreamSynchronize(0));
    e->net.table = P<float>(e->tied_table);
    e->net.tied = 1;
  }
  const int K = net_K(e->net);
  if (e->has_net && K != e->K) {
    // the resident complex's cache has the old net's planes (vset_ensure
    // reallocates the vertex sets for the new K): load a complex again
    e->valid = false;
    e->pend_idx = -1;
  }
  e->K = K;
  e->kw = net_kw(e->net);
  e->has_net = true;
  return 0;
}

extern "C" int tnp_forward(const tnp_net* n, const float* xyz, int64_t N, float* pre, int64_t ld,
                           float* out2, void* stream) {
  if (check_net(n)) return -1;
  return launch_forward(to_dev(n), xyz, N, pre, ld, 1, (hipStream_t)stream, out2);
}
extern "C" int tnp_encode(const tnp_net* n, const float* x01, int64_t N, float* out, void* stream) {
  if (check_net(n)) return -1;
  return launch_encode(to_dev(n), x01, N, out, (hipStream_t)stream);
}
extern "C" int tnp_forward_grouped(const tnp_net* n, const float* xyz, int64_t N, float* pre,
                                   int64_t ld, float* out2, void* stream) {
  if (check_net(n)) return -1;
  return launch_forward(to_dev(n), xyz, N, pre, ld, 8, (hipStream_t)stream, out2);
}
extern "C" int tnp_region(const tnp_net* n, const float* xyz, const float* pre, int64_t ld,
                          int64_t N, float eps, int64_t* m, int64_t* off, void* stream) {
  if (check_net(n)) return -1;
  return launch_region(to_dev(n), xyz, pre, ld, N, eps, m, off, (hipStream_t)stream);
}
extern "C" int tnp_sdf_grad(const tnp_net* n, const float* xyz, int64_t N, float* sdf, float* grad,
                            void* stream) {
  if (check_net(n)) return -1;
  return launch_sdf_grad(to_dev(n), xyz, N, sdf, grad, (hipStream_t)stream);
}

extern "C" int tnp_sdf_train_grad(const tnp_net* n, const float* xyz, const float* gt, int64_t N, float clamp_t,
                                  float eik_w, int64_t eik_batch, float* d_grad_table, float* d_grad_weights,
                                  double* d_stats, void* stream) {
  if (check_net(n)) return -1;
  if (N < 0 || !d_grad_table || !d_grad_weights || !d_stats) { tnp_set_error("sdf_train_grad: bad arguments"); return -1; }
  return launch_train_grad(to_dev(n), xyz, gt, N, clamp_t, eik_w, eik_batch > 0 ? eik_batch : N, d_grad_table, d_grad_weights, d_stats,
                           (hipStream_t)stream);
}

extern "C" int tnp_sdf_vjp(const tnp_net* n, const float* xyz, const float* gout, int64_t N, float* d_grad_table,
                           float* d_grad_weights, void* stream) {
  if (check_net(n)) return -1;
  if (N < 0 || !gout || !d_grad_table || !d_grad_weights) { tnp_set_error("sdf_vjp: bad arguments"); return -1; }
  return launch_sdf_vjp(to_dev(n), xyz, gout, N, d_grad_table, d_grad_weights, (hipStream_t)stream);
}

extern "C" int tnp_normal_vjp(const tnp_net* n, const float* xyz, const float* gJ, int64_t N, float* d_grad_table,
                              float* d_grad_weights, float* d_grad_x, void* stream) {
  if (check_net(n)) return -1;
  if (N < 0 || !gJ || !d_grad_table || !d_grad_weights) { tnp_set_error("normal_vjp: bad arguments"); return -1; }
  return launch_normal_vjp(to_dev(n), xyz, gJ, N, d_grad_table, d_grad_weights, d_grad_x, (hipStream_t)stream);
}

extern "C" int tnp_forward_vjp(const tnp_net* n, const float* xyz, int64_t N, const float* d_gpre, int64_t ld,
                               const float* d_gout, float* d_grad_table, float* d_grad_weights, float* d_grad_x,
                               void* stream) {
  if (check_net(n)) return -1;
  if (N < 0 || (!d_gpre && !d_gout) || (d_gpre && ld < N) || !d_grad_table || !d_grad_weights) {
    tnp_set_error("forward_vjp: bad arguments");
    return -1;
  }
  return launch_forward_vjp(to_dev(n), xyz, N, d_gpre, ld, d_gout, d_grad_table, d_grad_weights, d_grad_x,
                            (hipStream_t)stream);
}

extern "C" int tnp_mesh_signed_distance(const float* d_V, int64_t nV, const int32_t* d_F, int64_t nF,
                                        const float* d_p, int64_t n, float* d_work, float* d_dist, void* stream) {
  if (n < 0) { tnp_set_error("mesh_signed_distance: n < 0"); return -1; }
  return launch_mesh_sd(d_V, nV, d_F, nF, d_p, n, d_work, d_dist, (hipStream_t)stream);
}

static int set_edges_i64(tnp_engine* e, const int64_t* d_edges, int64_t E, hipStream_t s) {
  if (buf_ensure(e->edges, std::max<int64_t>(E, 1) * 2 * sizeof(int32_t), s)) return -1;
  if (E > 0)
    hipLaunchKernelGGL(k_i64_to_i32, dim3(tnp_grid(2 * E)), dim3(TNP_BLOCK), 0, s, d_edges,
                       P<int32_t>(e->edges), 2 * E);
  TNP_CHECK(hipGetLastError());
  e->E = E;
  e->E_live = E;
  return 0;
}

extern "C" int tnp_engine_load(tnp_engine* e, const float* d_xyz, int64_t V, const int64_t* d_edges,
                               int64_t E, const float* d_pre, int keep_all, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!e->has_net) { tnp_set_error("engine has no net"); return -1; }
  TNP_CHECK(hipSetDevice(e->device));
  span_all(e);  // anywhere (tnp_engine_set_span narrows it)
  if (buf_ensure(e->ctr, CTR_CLEAR_BYTES, s)) return -1;
  if (vset_ensure(e, e->cur, std::max<int64_t>(V, 1), 0, s)) return -1;
  if (V > 0)
    TNP_CHECK(hipMemcpyAsync(e->cur.xyz.p, d_xyz, V * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
  if (set_edges_i64(e, d_edges, E, s)) return -1;
  if (d_pre) {
    if (V > 0)
      hipLaunchKernelGGL(k_rows_to_planes, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, d_pre, V, e->K,
                         P<float>(e->cur.pre), e->cur.cap);
    TNP_CHECK(hipGetLastError());
  } else {
    if (launch_forward(e->net, P<float>(e->cur.xyz), V, P<float>(e->cur.pre), e->cur.cap, 1, s, nullptr,
                       VP(e->cur, e->kw), VZ(e->cur, e->kw), P<uint64_t>(e->cur.grid),
                       P<uint64_t>(e->cur.pz)))
      return -1;
  }
  if (d_pre && keys_for(e, e->cur, 0, V, s)) return -1;
  e->V = V;
  e->keep_all = keep_all;
  e->valid_from = 0;
  e->pend_idx = -1;
  return reset_live(e, s);
}

extern "C" int tnp_engine_sizes(tnp_engine* e, int64_t* V, int64_t* E) {
  if (e->cnt_pending) {  // (never a silent 0 from a deferred count)
    tnp_set_error("tnp_engine_sizes: the live counts of the last step are still pending");
    return -1;
  }
  *V = e->V_live;
  *E = e->E_live;
  return 0;
}

extern "C" int tnp_engine_active_planes(tnp_engine* e, int from, uint64_t* mask, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (require_valid(e, "active_planes")) return -1;
  if (buf_ensure(e->ctr, CTR_CLEAR_BYTES, s)) return -1;
  TNP_CHECK(hipMemsetAsync(P<int64_t>(e->ctr) + CTR_ACTIVE, 0, sizeof(int64_t), s));
  // the per-edge masks are (re)computed here and the OR of their first split
  // planes taken in the same pass: the planes the next steps must visit
  if (compute_masks(e, from, P<int64_t>(e->ctr), s)) return -1;
  if (read_ctr(e, s)) return -1;
  *mask = (uint64_t)e->h_ctr[CTR_ACTIVE];
  e->act_bits = *mask;
  return 0;
}

// ---------------------------------------------------------------------------
// curve path, phase 1 (subpoly.py:120-177, 204-207): correct the new vertices
// of non-axis-aligned split edges to the trilinear intersection, with the
// gradient-descent fallback; leaves per-split strict-filter inputs in cinfo.
// ---------------------------------------------------------------------------
// the shards' reduction of n words (tnp_engine_set_collective); one shard:
// none.  Every call carries one more word, this shard's failure flag
// (coll_fail), reduced with the same op: a shard that failed between two
// collectives joins the next one with the flag set, and every shard then
// fails at that same call -- none is left blocked in a collective its peer
// never reaches.
static int coll(tnp_engine* e, int64_t* v, int n, int op) {
  if (e->shards <= 1) return 0;
  if (!e->coll_fn) {
    tnp_set_error("curve path on %d shards: no collective for its whole-complex decisions "
                  "(tnp_engine_set_collective)", e->shards);
    return -1;
  }
  const bool all_ones = op == TNP_COLL_AND;  // AND: "no failure" is all ones
  std::vector<int64_t> w(v, v + n);
  w.push_back(e->coll_err ? (all_ones ? 0 : 1) : (all_ones ? -1 : 0));
  if (e->coll_fn(w.data(), n + 1, op, e->coll_ctx) != 0) {
    tnp_set_error("the shards' collective failed");
    return -1;
  }
  if (all_ones ? w[n] != -1 : w[n] != 0) {
    if (!e->coll_err) tnp_set_error("a peer shard failed in this sharded step (its own error names the cause)");
    e->coll_err = false;
    return -1;
  }
  std::copy(w.begin(), w.begin() + n, v);
  return 0;
}

// this shard failed before the step's next collective (n words, op): join
// it with the failure flag set, keep this shard's own error message
static int coll_fail(tnp_engine* e, int n, int op) {
  if (e->shards <= 1 || !e->coll_fn) return -1;
  const std::string msg = g_err;
  std::vector<int64_t> v(n, op == TNP_COLL_AND ? -1 : 0);
  e->coll_err = true;
  (void)coll(e, v.data(), n, op);
  e->coll_err = false;
  g_err = msg;
  return -1;
}

// curve path, phase 1 (subpoly.py:120-177, subpoly_debug.py:121-165).  On
// shards (e->shards > 1) every shard calls it for every split step, S == 0
// included, and takes the batch's decisions with the others: the curve rows'
// and descent rows' totals (MKL's row-count schedules of the corner, point
// and descent launches follow the whole batch) and the descent's stop (the
// AND of the shards' per-iteration convergence words).
// A sharded curve step whose batch -- the shards' total rows of one of its
// forwards -- is 2..15 rows on a 32-wide net: MKL's 32-input FOLD schedule
// of the 2-output layer depends on each row's parity in the WHOLE batch
// (net_device.h neuron_mode), the shards number their rows locally, and the
// batch's row order across shards is not defined.  Refused instead of left
// to halo_check; every shard sees the same total after the
// same collective, so every shard refuses at the same point.
static int fold32_sharded(const tnp_engine* e, int64_t rows, const char* what, int idx) {
  if (e->shards > 1 && e->net.num_hidden == 32 && rows >= 2 && rows <= 15) {
    tnp_set_error("plane %d: a sharded curve step of %lld %s on a 32-wide net (MKL's 2..15-row FOLD schedule "
                  "depends on each row's parity in the whole batch, which the shards do not share); run it "
                  "unsharded", idx, (long long)rows, what);
    return -1;
  }
  return 0;
}

static int curve_correct(tnp_engine* e, int idx, int64_t S, hipStream_t s) {
  const float eps = e->net.eps_s;  // subpoly_'s eps (subpoly.py:120-177)
  const int K = e->K;
  Buf* cv = e->cv;
  int64_t* ctr = P<int64_t>(e->ctr);
  const int32_t* sa = P<int32_t>(e->sa);
  const int32_t* sb = P<int32_t>(e->sb);
  float* xyz = P<float>(e->cur.xyz);
  // (sharded: a segment that fails joins the step's next collective with the
  // failure flag, coll_fail, so every shard stops at the same call)
  int64_t B = 0;
  auto seg_flags = [&]() -> int {
  if (S > 0) {
    if (buf_ensure(cv[CV_CFLAG], S * sizeof(int32_t), s)) return -1;
    if (buf_ensure(cv[CV_COFF], S * sizeof(int64_t), s)) return -1;
    if (buf_ensure(cv[CV_CINFO], S * sizeof(int32_t), s)) return -1;
    const FillOp f{cv[CV_CINFO].p, (uint64_t)S * sizeof(int32_t), 0};
    if (launch_fill(&f, 1, s)) return -1;
    TIMED("curve_flags", 32.0 * S,
          launch_curve_flags(sa, sb, S, xyz, eps, P<int32_t>(cv[CV_CFLAG]), s));
    if (scan_counts(e, P<int32_t>(cv[CV_CFLAG]), P<int64_t>(cv[CV_COFF]), S, CTR_B, s)) return -1;
    if (read_ctr(e, s)) return -1;
    B = e->h_ctr[CTR_B];
  }
  return 0;
  };
  if (seg_flags()) return coll_fail(e, 1, TNP_COLL_SUM);
  const bool sh = e->shards > 1;
  int64_t Bg = B;  // the batch's curve rows (r_edges, subpoly.py:120)
  if (coll(e, &Bg, 1, TNP_COLL_SUM)) return -1;
  if (Bg == 0) return 0;
  if (fold32_sharded(e, Bg, "curve rows", idx)) return -1;
  NetDev ns = e->net;  // sharded: the schedules of the whole batch
  int64_t G = 0;
  int32_t* crow = nullptr;
  int32_t* plane = nullptr;
  float* ints = nullptr;
  float* d0s = nullptr;
  float* d1s = nullptr;
  auto seg_rows = [&]() -> int {
  if (B > 0) {
  if (buf_ensure(cv[CV_CROW], B * sizeof(int32_t), s)) return -1;
  if (buf_ensure(cv[CV_CORNERS], 24 * B * sizeof(float), s)) return -1;
  if (buf_ensure(cv[CV_PLANE], B * sizeof(int32_t), s)) return -1;
  if (buf_ensure(cv[CV_STAGE_C], (size_t)8 * B * K * sizeof(float), s)) return -1;
  if (buf_ensure(cv[CV_INTS], 3 * B * sizeof(float), s)) return -1;
  if (buf_ensure(cv[CV_INTS0], 3 * B * sizeof(float), s)) return -1;
  if (buf_ensure(cv[CV_PTS], 3 * B * sizeof(float), s)) return -1;
  if (buf_ensure(cv[CV_STAGE_P], (size_t)B * K * sizeof(float), s)) return -1;
  for (int k : {CV_D0, CV_D1, CV_GG, CV_GD}) if (buf_ensure(cv[k], B * 4, s)) return -1;
  if (buf_ensure(cv[CV_GOFF], B * sizeof(int64_t), s)) return -1;
  crow = P<int32_t>(cv[CV_CROW]);
  plane = P<int32_t>(cv[CV_PLANE]);
  ints = P<float>(cv[CV_INTS]);
  d0s = P<float>(cv[CV_D0]);
  d1s = P<float>(cv[CV_D1]);
  if (launch_curve_rows(P<int32_t>(cv[CV_CFLAG]), P<int64_t>(cv[CV_COFF]), S, crow, s)) return -1;
  TIMED("curve_corners", 8.0 * B * 12 + 24.0 * B,
        launch_curve_corners(crow, B, sa, sb, xyz, VZ(e->cur, e->kw), P<uint64_t>(e->cur.grid), idx,
                             P<float>(cv[CV_CORNERS]), plane, ctr, e->kw, s));
  if (sh) ns.sched_rows = 8 * Bg;
  TIMED("curve_forward", 8.0 * B * (12 + 4.0 * K),
        launch_forward(ns, P<float>(cv[CV_CORNERS]), 8 * B, P<float>(cv[CV_STAGE_C]), 8 * B, 8, s));
  TIMED("curve_solve", 64.0 * B + 24.0 * B,
        launch_curve_solve(B, P<float>(cv[CV_STAGE_C]), 8 * B, plane, idx, crow, sa, sb, xyz, ints,
                           P<float>(cv[CV_PTS]), s));
  if (sh) ns.sched_rows = Bg;
  TIMED("curve_forward", B * (12 + 4.0 * K),
        launch_forward(ns, P<float>(cv[CV_PTS]), B, P<float>(cv[CV_STAGE_P]), B, 1, s));
  if (launch_curve_dnew(B, P<float>(cv[CV_STAGE_P]), B, plane, idx, ints, eps, d0s, d1s,
                        P<int32_t>(cv[CV_GG]), P<int32_t>(cv[CV_GD]), s)) return -1;
  if (scan_counts(e, P<int32_t>(cv[CV_GD]), P<int64_t>(cv[CV_GOFF]), B, CTR_G, s)) return -1;
  if (read_ctr(e, s)) return -1;
  if (e->h_ctr[CTR_NOPLANE] & 2) {
    tnp_set_error("curve path, plane %d: a split edge's endpoints share fewer than two zero columns (the "
                  "reference's check_new_vertices_on_two_planes then fails: AttributeError, "
                  "subpoly_debug.py:96-104)", idx);
    return -1;
  }
  if (e->h_ctr[CTR_NOPLANE]) {
    tnp_set_error("curve path: a split edge shares no plane below %d (the reference prints it and "
                  "exit()s, subpoly.py:141-148)", idx);
    return -1;
  }
  G = e->h_ctr[CTR_G];
  }  // B > 0
  return 0;
  };
  if (seg_rows()) return coll_fail(e, 1, TNP_COLL_SUM);
  int64_t Gg = G;  // the batch's descent rows
  if (coll(e, &Gg, 1, TNP_COLL_SUM)) return -1;
  if (fold32_sharded(e, Gg, "descent rows", idx)) return -1;
  if (Gg > 0) {
    if (sh) ns.sched_rows = Gg;
    uint64_t h_conv[8] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull};  // (no rows: converged)
    int32_t* glist = nullptr;
    unsigned long long* conv = nullptr;
    auto seg_desc = [&]() -> int {
    if (G > 0) {
      if (buf_ensure(cv[CV_GLIST], G * sizeof(int32_t), s)) return -1;
      if (buf_ensure(cv[CV_CONV], 8 * sizeof(uint64_t), s)) return -1;
      glist = P<int32_t>(cv[CV_GLIST]);
      conv = P<unsigned long long>(cv[CV_CONV]);
      if (launch_gd_rows(P<int32_t>(cv[CV_GD]), P<int64_t>(cv[CV_GOFF]), B, glist, s)) return -1;
      TNP_CHECK(hipMemcpyAsync(cv[CV_INTS0].p, ints, 3 * B * sizeof(float), hipMemcpyDeviceToDevice, s));
      TNP_CHECK(hipMemsetAsync(conv, 0xFF, 8 * sizeof(uint64_t), s));
      TIMED("descend", 0.0,
            launch_descend(ns, G, glist, crow, sa, sb, xyz, plane, idx, eps, e->gd_iters, 1, ints,
                           d0s, d1s, conv, s));
      TNP_CHECK(hipMemcpyAsync(h_conv, conv, sizeof(h_conv), hipMemcpyDeviceToHost, s));
      TNP_CHECK(hipStreamSynchronize(s));
    }
    return 0;
    };
    if (seg_desc()) return coll_fail(e, 8, TNP_COLL_AND);
    // the loop of subpoly_debug.py:141 stops when EVERY row of the batch met
    // both planes: the AND of the shards' per-iteration words
    if (coll(e, reinterpret_cast<int64_t*>(h_conv), 8, TNP_COLL_AND)) return -1;
    int stop = -1;  // first iteration after which every row met both planes (the replay below
                    // fails towards the step's next collective, the strict flag's OR)
    for (int i = 0; i < e->gd_iters && stop < 0; ++i)
      if ((h_conv[i >> 6] >> (i & 63)) & 1) stop = i;
    auto seg_replay = [&]() -> int {
    if (G > 0 && stop >= 0 && stop + 1 < e->gd_iters) {
      // the loop ends after iteration `stop`: replay
      TNP_CHECK(hipMemcpyAsync(ints, cv[CV_INTS0].p, 3 * B * sizeof(float), hipMemcpyDeviceToDevice, s));
      TIMED("descend", 0.0,
            launch_descend(ns, G, glist, crow, sa, sb, xyz, plane, idx, eps, stop + 1, 0, ints,
                           d0s, d1s, conv, s));
    }
    return 0;
    };
    if (seg_replay()) return coll_fail(e, 1, TNP_COLL_OR);
  }
  auto seg_apply = [&]() -> int {
  if (B > 0)
    TIMED("curve_apply", 60.0 * B,
          launch_curve_apply(B, crow, sa, sb, xyz, e->V, ints, d0s, P<int32_t>(cv[CV_GG]), eps,
                             P<int32_t>(cv[CV_CINFO]), ctr, s));
  return 0;
  };
  if (seg_apply()) return coll_fail(e, 1, TNP_COLL_OR);
  return 0;
}

// curve path, phase 2 (subpoly_debug.py:234-271): strict filter after the
// override; surviving splits get consecutive ids in edge order and rewire
// their edges (masked_scatter_ of the filtered mask, subpoly.py:201-212).
static int curve_filter(tnp_engine* e, int idx, int override_, hipStream_t s, int64_t* S_out) {
  const int64_t S = e->pend_S, V = e->V;
  const int K = e->K;
  Buf* cv = e->cv;
  if (S == 0) { *S_out = 0; return 0; }
  if (buf_ensure(cv[CV_KEEP], S * sizeof(int32_t), s)) return -1;
  if (buf_ensure(cv[CV_NID], S * sizeof(int64_t), s)) return -1;
  if (launch_strict_keep(S, P<int32_t>(cv[CV_CINFO]), P<float>(e->stage), idx, override_,
                         P<uint64_t>(e->shared), e->net.eps_s, e->pend_tight, e->strict, P<int32_t>(cv[CV_KEEP]),
                         e->kw, s))
    return -1;
  if (scan_counts(e, P<int32_t>(cv[CV_KEEP]), P<int64_t>(cv[CV_NID]), S, CTR_KEEP, s)) return -1;
  if (read_ctr(e, s)) return -1;
  const int64_t S2 = e->h_ctr[CTR_KEEP];
  const int64_t n = std::max<int64_t>(S2, 1);
  if (buf_ensure(cv[CV_SA2], n * sizeof(int32_t), s)) return -1;
  if (buf_ensure(cv[CV_SB2], n * sizeof(int32_t), s)) return -1;
  if (buf_ensure(cv[CV_SHARED2], n * sizeof(uint64_t) * e->kw, s)) return -1;
  if (buf_ensure(cv[CV_STAGE2], (size_t)n * K * sizeof(float), s)) return -1;
  if (buf_ensure(cv[CV_XYZ2], 3 * n * sizeof(float), s)) return -1;
  if (buf_ensure(cv[CV_GRID2], n * sizeof(uint64_t), s)) return -1;
  TIMED("compact_splits", (16.0 + 8.0 * K + 40.0) * S,
        launch_compact_splits(S, K, P<int32_t>(cv[CV_KEEP]), P<int64_t>(cv[CV_NID]),
                              P<int32_t>(cv[CV_EIDX]), V, P<int32_t>(e->sa), P<int32_t>(e->sb),
                              P<uint64_t>(e->shared), P<float>(e->stage), P<float>(e->cur.xyz),
                              P<uint64_t>(e->cur.grid), S2, P<int32_t>(cv[CV_SA2]),
                              P<int32_t>(cv[CV_SB2]), P<uint64_t>(cv[CV_SHARED2]),
                              P<float>(cv[CV_STAGE2]), P<float>(cv[CV_XYZ2]),
                              P<uint64_t>(cv[CV_GRID2]), P<int32_t>(e->edges), e->kw, s));
  if (S2 > 0) {
    TNP_CHECK(hipMemcpyAsync(P<float>(e->cur.xyz) + 3 * V, cv[CV_XYZ2].p, 3 * S2 * sizeof(float),
                             hipMemcpyDeviceToDevice, s));
    TNP_CHECK(hipMemcpyAsync(P<uint64_t>(e->cur.grid) + V, cv[CV_GRID2].p, S2 * sizeof(uint64_t),
                             hipMemcpyDeviceToDevice, s));
  }
  std::swap(e->sa, cv[CV_SA2]);
  std::swap(e->sb, cv[CV_SB2]);
  std::swap(e->shared, cv[CV_SHARED2]);
  std::swap(e->stage, cv[CV_STAGE2]);
  e->pend_S = S2;
  *S_out = S2;
  return 0;
}

extern "C" int tnp_engine_split_keep(tnp_engine* e, int32_t* d_keep, int64_t n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (!e->curve || n <= 0) return 0;
  if (e->cv[CV_KEEP].bytes < (size_t)n * sizeof(int32_t)) {
    tnp_set_error("split_keep: no strict filter ran for %lld splits", (long long)n);
    return -1;
  }
  TNP_CHECK(hipMemcpyAsync(d_keep, e->cv[CV_KEEP].p, n * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  return 0;
}

extern "C" int tnp_engine_set_shards(tnp_engine* e, int world) {
  e->shards = world < 1 ? 1 : world;
  return 0;
}

extern "C" int tnp_engine_set_curve(tnp_engine* e, int on) {
  e->curve = on ? 1 : 0;
  return 0;
}

extern "C" int tnp_engine_set_strict(tnp_engine* e, int on) {
  e->strict = on ? 1 : 0;
  return 0;
}

extern "C" int tnp_engine_set_collective(tnp_engine* e, tnp_collective_fn fn, void* ctx) {
  e->coll_fn = fn;
  e->coll_ctx = ctx;
  return 0;
}

// the flat step's new vertices: split points + forward + failover test +
// keys in one pass, straight into the cache (k_forward_new).  n < 0: S is
// still on the device (launched right behind the split, before the host
// reads S back: the readback's round trip overlaps this kernel), -n bounds
// it and sizes the vertex set and the shared-plane words.
static int64_t early_bound(const tnp_engine* e) {
  if (!e->early_bound_splits) return e->E;
  return std::min<int64_t>(e->E, e->max_split_seen + e->max_split_seen / 4 + 4096);
}

static int flat_forward_new(tnp_engine* e, int idx, int64_t n, hipStream_t s) {
  const int64_t bound = n >= 0 ? n : -n;
  if (vset_ensure(e, e->cur, e->V + bound, e->V, s)) return -1;
  if (buf_ensure(e->shared, bound * sizeof(uint64_t) * e->kw, s)) return -1;
  const float* col = P<float>(e->cur.pre) + (int64_t)idx * e->cur.cap;  // (after any move)
  e->pend_keep = new_keep_from(e, idx);
  // compulsory bytes per split: reads 8 B endpoint ids, 24 B endpoint
  // coordinates, 8 B endpoint plane values, 16 B endpoint zero keys; writes
  // 12 B coordinates, the cache planes >= keep_from, 32 B keys (pz: pos and
  // zero, the only copy since round 6; grid; shared); plus the encoding
  // tables once per launch (the 8
  // corners x L levels gathers are cache traffic).  (n < 0: set once S is known)
  TIMED("forward_new",
        (8.0 + 24.0 + 8.0 + 16.0 + 12.0 + 4.0 * (e->K - e->pend_keep) + 32.0) * std::max<int64_t>(n, 0) +
            table_bytes(e->net),
        launch_forward_new(e->net, P<float>(e->cur.xyz) + 3 * e->V, n, P<float>(e->cur.pre), e->cur.cap, e->V,
                           e->pend_keep, P<int32_t>(e->sa), P<int32_t>(e->sb), idx, e->own,
                           VP(e->cur, e->kw), VZ(e->cur, e->kw), P<uint64_t>(e->cur.grid),
                           P<uint64_t>(e->shared), P<int64_t>(e->ctr), P<uint64_t>(e->cur.pz), col, s));
  return 0;
}

extern "C" int tnp_engine_split(tnp_engine* e, int idx, void* stream, int64_t* S_out, int32_t* fail) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (idx < e->valid_from || idx >= e->K) {
    tnp_set_error("plane %d not cached (valid from %d)", idx, e->valid_from);
    return -1;
  }
  if (require_valid(e, "split")) return -1;
  e->valid = false;  // until this split has completed
  const float eps = e->net.eps_s;  // subpoly_'s eps: hits, split point, failover
  const float* col = P<float>(e->cur.pre) + (int64_t)idx * e->cur.cap;
  // curve branch on shards: the new vertices' forward follows the schedule
  // of the whole batch (the shards' total split count), and every shard
  // joins the branch's decisions (curve_correct) whatever its own count; a
  // shard failing between two of the step's collectives joins the next one
  // with its failure flag (coll_fail)
  const bool ccoll = e->curve && e->shards > 1;
  int64_t S = 0;
  bool early_fwd = false;  // k_forward_new already launched (device S)
  e->pend_hits = false;
  auto seg_split = [&]() -> int {
  // the last step's deferred live counts ride in this split's hit workers
  // (the flat bucket path); otherwise they are counted now, before the reset
  BucketGeom bgs{};
  const bool fused_hits = !e->curve && e->V > 0 && e->E > 0 && uses_buckets(e, &bgs);
  if (e->cnt_pending && !fused_hits && resolve_counts(e, s)) return -1;
  const bool take_counts = e->cnt_pending;
  if (!(e->in_run && e->ctr_zero)) TNP_CHECK(hipMemsetAsync(e->ctr.p, 0, CTR_CLEAR_BYTES, s));
  e->ctr_zero = false;
  if (e->E > 0) {
    // single pass; the id buffers hold the upper bound E (capacity is kept)
    if (buf_ensure(e->sa, e->E * sizeof(int32_t), s)) return -1;
    if (buf_ensure(e->sb, e->E * sizeof(int32_t), s)) return -1;
    if (e->curve && buf_ensure(e->cv[CV_EIDX], e->E * sizeof(int32_t), s)) return -1;
    const int fresh = ensure_masks(e, idx, s);
    if (fresh < 0) return -1;
    TnpLB lb;
    if (lb_begin(e, split_tiles(e->E), s, &lb, 0, false)) return -1;
    // flat path: the plane's hit vertices are found with the split (they
    // read only the cached column and the live flags), so one readback
    // returns S and H.  The bucket path reads them at members[E, E + H)
    // (S <= E) and they ride in the split's own dispatch; the radix path
    // wants them after the S new members (members[S, S + H)): launched
    // behind the split, which writes S
    const bool flat_hits = !e->curve && e->V > 0;
    if (flat_hits && buf_ensure(e->members, (e->E + e->V) * sizeof(int32_t), s)) return -1;
    if (take_counts && buf_ensure(e->hpart, HIT_WORKERS_MAX * sizeof(int64_t), s)) return -1;
    const HitArgs ha{col, P<uint8_t>(e->live), e->V, eps, P<int32_t>(e->members) + e->E,
                     take_counts ? P<int64_t>(e->hpart) : nullptr};
    // algorithmic bytes: 1 B first split plane per edge (+ 5 B per vertex
    // slot for fused hits); per split 8 B endpoints, 4 B rewired id, 1 B
    // stale mask (set once S is known)
    TIMED("split", 1.0 * e->E + (fused_hits ? 5.0 * e->V : 0.0),
          launch_split_lb(P<int32_t>(e->edges), e->E, P<uint8_t>(e->eef), P<uint8_t>(e->edm), idx,
                          e->V, P<int32_t>(e->sa), P<int32_t>(e->sb), P<int64_t>(e->ctr),
                          e->curve ? P<int32_t>(e->cv[CV_EIDX]) : nullptr, lb, s, fused_hits ? &ha : nullptr));
    if (flat_hits && !fused_hits)
      TIMED("hits", 5.0 * e->V,
            launch_hits(col, P<uint8_t>(e->live), e->V, eps, P<int32_t>(e->members), -1,
                        P<int64_t>(e->ctr), s));
    e->pend_hits = flat_hits;
    e->pend_hoff = fused_hits ? e->E : -1;
    // flat path: the new vertices' forward goes behind the split now, sized
    // by the bound S <= E, so the GPU runs it while S travels to the host
    early_fwd = !e->curve && e->early_forward;
    const int64_t eb = early_fwd ? early_bound(e) : 0;
    int64_t seq = 0;
    if (take_counts ? post_ctr(e, s, &seq, P<int64_t>(e->hpart), split_hit_workers(e->V),
                               e->pend_lz_n ? P<int64_t>(e->lzpart) : nullptr, (int)e->pend_lz_n)
                    : post_ctr(e, s, &seq))
      return -1;
    if (early_fwd && flat_forward_new(e, idx, -eb, s)) return -1;
    if (wait_ctr(e, s, seq)) return -1;
    if (take_counts) apply_counts(e, e->h_ctr[CTR_V], e->h_ctr[CTR_E]);
    S = e->h_ctr[CTR_S];
    e->max_split_seen = std::max(e->max_split_seen, S);
    if (early_fwd && S > eb) {
      // more splits than the early launch's bound: it processed rows [0, eb)
      // only; the whole forward runs again once S is known (the same values;
      // the failover OR is idempotent, the halo count is recounted)
      early_fwd = false;
      e->n_early_redo++;
      TNP_CHECK(hipMemsetAsync(P<int64_t>(e->ctr) + CTR_DUP, 0, sizeof(int64_t), s));
    }
    if (fresh) e->act_bits = (uint64_t)e->h_ctr[CTR_ACTIVE];
    if (e->h_ctr[CTR_MISSED]) {  // ensure_masks keeps this from happening
      tnp_set_error("plane %d: an edge's first split plane lies below the step (stale edge masks)", idx);
      return -1;
    }
    ktimer_set_bytes(e, "split", 1.0 * e->E + 13.0 * S + (e->pend_hoff >= 0 ? 5.0 * e->V : 0.0));
  }
  if (e->V + S >= (int64_t)INT32_MAX) {
    // slots (dead ones included: compaction is lazy) are int32 ids in sa/sb,
    // members, edges and the packed pair keys
    tnp_set_error("plane %d: %lld vertex slots + %lld splits exceed the int32 slot range", idx,
                  (long long)e->V, (long long)S);
    return -1;
  }
  return 0;
  };
  if (seg_split()) return ccoll ? coll_fail(e, 1, TNP_COLL_SUM) : -1;
  *fail = 0;
  int64_t Sg = S;
  if (ccoll && coll(e, &Sg, 1, TNP_COLL_SUM)) return -1;
  if (ccoll && fold32_sharded(e, Sg, "splits", idx)) return -1;
  if (ccoll && S == 0 && Sg > 0 && curve_correct(e, idx, 0, s)) return -1;
  if (S > 0) {
    auto seg_new = [&]() -> int {
    if (vset_ensure(e, e->cur, e->V + S, e->V, s)) return -1;
    col = P<float>(e->cur.pre) + (int64_t)idx * e->cur.cap;  // may have moved
    if (e->curve)
      TIMED("new_vertices", 52.0 * S,
            launch_new_vertices(P<int32_t>(e->sa), P<int32_t>(e->sb), S, col, eps, P<float>(e->cur.xyz),
                                e->V, s));
    return 0;
    };
    // (the curve branch's next collective: curve_correct's first)
    if (seg_new()) return ccoll ? coll_fail(e, 1, TNP_COLL_SUM) : -1;
    if (e->curve && curve_correct(e, idx, S, s)) return -1;
    auto seg_rest = [&]() -> int {
    e->pend_fused = !e->curve;
    if (e->pend_fused) {
      if (early_fwd)  // (launched behind the split; its modelled bytes now)
        ktimer_set_bytes(e, "forward_new",
                         (8.0 + 24.0 + 8.0 + 16.0 + 12.0 + 4.0 * (e->K - e->pend_keep) + 32.0) * S +
                             table_bytes(e->net));
      else if (flat_forward_new(e, idx, S, s))
        return -1;
    } else {
      if (buf_ensure(e->shared, S * sizeof(uint64_t) * e->kw, s)) return -1;
      if (buf_ensure(e->stage, (size_t)S * e->K * sizeof(float), s)) return -1;
      NetDev nf = e->net;
      if (ccoll) nf.sched_rows = Sg;
      TIMED("forward", (12.0 + 4.0 * e->K) * S,
            launch_forward(nf, P<float>(e->cur.xyz) + 3 * e->V, S, P<float>(e->stage), S, 1, s));
      // grid words of the new vertices (coordinates are final; the failover
      // test of a shard reads them: only owned vertices vote)
      if (launch_keys(e->net, P<float>(e->cur.xyz) + 3 * e->V, P<float>(e->stage), S, S, 0,
                      VP(e->cur, e->kw, e->V), VZ(e->cur, e->kw, e->V), P<uint64_t>(e->cur.grid) + e->V, s,
                      VP(e->cur, e->kw, e->V)))
        return -1;
      TIMED("fail_check", 48.0 * S,
            launch_fail_check(P<int32_t>(e->sa), P<int32_t>(e->sb), S, idx, VZ(e->cur, e->kw),
                              P<float>(e->stage), eps, P<uint64_t>(e->shared), P<int64_t>(e->ctr),
                              P<uint64_t>(e->cur.grid) + e->V, e->own, e->kw, s));
    }
    if (e->curve || e->shards > 1) {
      // the host takes the global override decision (all-reduce) / the curve
      // filter needs it: read it back
      if (read_ctr(e, s)) return -1;
      *fail = e->h_ctr[CTR_FAIL] ? 1 : 0;
    } else {
      *fail = -1;  // single device: the finish kernels read it in place
    }
    return 0;
    };
    // (then the strict filter flag's OR)
    if (seg_rest()) return ccoll ? coll_fail(e, 1, TNP_COLL_OR) : -1;
  }
  e->pend_dup = S > 0 ? e->h_ctr[CTR_DUP] : 0;
  e->pend_tight = (S > 0 && e->curve) ? (int)e->h_ctr[CTR_TIGHT] : 0;
  if (ccoll && Sg > 0) {  // the strict filter's flag is the batch's (subpoly_debug.py:253-257)
    int64_t t = e->pend_tight;
    if (coll(e, &t, 1, TNP_COLL_OR)) return -1;
    e->pend_tight = t != 0;
  }
  *S_out = S;
  e->pend_idx = idx;
  e->pend_S = S;
  e->valid = true;
  return 0;
}

// the side stream (created on first use, non-blocking: no implicit sync
// with the caller's stream) and its two events
static int side_stream(tnp_engine* e) {
  if (e->s2) return 0;
  TNP_CHECK(hipStreamCreateWithFlags(&e->s2, hipStreamNonBlocking));
  for (hipEvent_t& ev : e->ev_s2) TNP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  return 0;
}
// the caller's stream waits for the side stream's prune (every exit of a
// finish that launched one, errors included)
static void side_join(tnp_engine* e, hipStream_t s) {
  if (!e->s2_pending) return;
  (void)hipStreamWaitEvent(s, e->ev_s2[1], 0);
  e->s2_pending = false;
}
struct SideJoin {
  tnp_engine* e;
  hipStream_t s;
  ~SideJoin() { side_join(e, s); }
};

extern "C" int tnp_engine_finish(tnp_engine* e, int idx, int prune, int override_, void* stream,
                                 tnp_step_stats* st) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (e->pend_idx != idx) { tnp_set_error("finish(%d) without split(%d)", idx, idx); return -1; }
  if (require_valid(e, "finish")) return -1;
  if (e->cnt_pending) {  // (the split resolves them; a finish never sees them pending)
    tnp_set_error("finish(%d): live counts of the last step still pending", idx);
    return -1;
  }
  e->pend_idx = -1;
  e->valid = false;  // until this step has completed
  const SideJoin side_guard{e, s};
  const bool hits_done = e->pend_hits;
  const int64_t hoff = hits_done ? e->pend_hoff : -1;
  e->pend_hits = false;
  const float eps = e->net.eps;
  const int K = e->K;
  int64_t S_kept = e->pend_S;
  if (e->curve) {
    if (curve_filter(e, idx, override_, s, &S_kept)) return -1;
    e->masks_valid = false;  // the filter rewired the kept split edges
    // the kept splits another shard owns (read back with the connect
    // counters; the split's CTR_DUP count is the flat path's)
    TNP_CHECK(hipMemsetAsync(P<int64_t>(e->ctr) + CTR_DUP, 0, sizeof(int64_t), s));
    if (launch_count_unowned(P<uint64_t>(e->cur.grid) + e->V, S_kept, e->own, P<int64_t>(e->ctr), s))
      return -1;
  }
  const int64_t V = e->V, E = e->E, S = S_kept;
  const int64_t NV = V + S;
  VSet& c = e->cur;
  const float* col = P<float>(c.pre) + (int64_t)idx * c.cap;
  int64_t* ctr = P<int64_t>(e->ctr);
  uint64_t* pos = VP(c, e->kw);
  uint64_t* zero = VZ(c, e->kw);
  uint64_t* grid = P<uint64_t>(c.grid);

  BucketGeom bg{};
  int sp0[3], sp1[3];
  span_of(e, sp0, sp1);
  const bool buckets = uses_buckets(e, &bg);
  const int NB = buckets ? bg.NB : 0;
  // 1. override + keys of the new vertices (flat bucket path: the override
  //    runs inside the bucket count, below)
  if (e->pend_fused && buckets) {
  } else if (e->pend_fused) {
    TIMED("override_new", 8.0 * S,
          launch_override_new(S, override_, P<uint64_t>(e->shared), P<float>(c.pre), c.cap,
                              e->pend_keep, V, pos, zero, ctr, P<uint64_t>(c.pz), e->kw, s));
  } else {
    TIMED("finalize_new", (8.0 + 4.0 * K + 4.0 * (K - e->valid_from) + 16.0) * S,
          launch_finalize_new(S, K, override_, P<uint64_t>(e->shared), P<float>(e->stage), eps,
                              P<float>(c.pre), c.cap, e->valid_from, V, pos, zero, ctr,
                              P<uint64_t>(c.pz), e->kw, s));
  }

  // 2. members = new vertices ++ live hit vertices (any order); the bucket
  //    path reads the new vertices as slots V.. without a list
  if (buf_ensure(e->members, std::max<int64_t>(NV, 1) * sizeof(int32_t), s, hits_done)) return -1;
  if (hits_done) {
    if (!buckets && launch_new_members(P<int32_t>(e->members), S, V, s)) return -1;
  } else {
    TIMED("hits", 5.0 * V + 4.0 * S,
          launch_hits(col, P<uint8_t>(e->live), V, e->net.eps_s, P<int32_t>(e->members), S, ctr, s));
  }

  // 3. bucket members by grid cell (dense cell grid over the marks): one
  //    (cell, member) entry per spanned cell, radix-sorted by cell
  const int NC = e->net.n_marks + 2;
  if (NC > 1023) {  // connect packs cell coordinates in 10 bits each
    tnp_set_error("more than 1021 marks per axis");
    return -1;
  }
  const int64_t ncell = (int64_t)NC * NC * NC;
  // the live member count sizes the span pass and its scan (V counts every
  // slot, live or dead: sizing by it would scan ~V elements per step)
  if (!hits_done && read_ctr(e, s)) return -1;  // else: H came back with S
  const int64_t M = S + e->h_ctr[CTR_H];
  // a member spans <= 8 cells (2 per axis when on a mark plane): entry
  // buffers take the bound 8 M, so nothing waits for the entry count T
  const int64_t TB = std::max<int64_t>(8 * M, 1);
  const int64_t RC = TB / 2 + 1;  // a pair cell holds >= 2 entries
  if (buf_ensure(e->ents, TB * cell_ent_bytes(e->kw), s)) return -1;
  if (buf_ensure(e->pcell, RC * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->pent, RC * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->pcn, RC * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->ptoff, RC * sizeof(int64_t), s)) return -1;
  int64_t H = 0, T = 0;
  // k_connect's chunk table: its capacity is kept across steps (grown on
  // overflow and redone); the bucket path fills it in its pair-cell gather
  int64_t bcap = std::max<int64_t>(e->bcell.bytes / sizeof(int32_t), 4096);
  if (buf_ensure(e->bcell, bcap * sizeof(int32_t), s)) return -1;
  if (buckets) {
    // spatial buckets, every count on the device (bucket.hip)
    void* const bk0 = e->bk[0].p;
    void* const bk1 = e->bk[1].p;
    if (buf_ensure(e->bk[0], (NB + 1) * sizeof(int32_t), s)) return -1;  // counts (+1: read in pairs)
    if (buf_ensure(e->bk[1], NB * sizeof(int32_t), s)) return -1;        // cursors
    if (e->bk[0].p != bk0 || e->bk[1].p != bk1) e->bk_clean = false;     // fresh memory
    if (buf_ensure(e->bk[2], (NB + 1) * sizeof(int64_t), s)) return -1;  // bases
    // block parts: one per workgroup of the member passes (the grid is at least
    // FUSE_MAX_BLOCKS = 512 when the live-flag zeroing rides along)
    if (buf_ensure(e->bk[7], (std::max<int64_t>(bucket_member_blocks(M), 512) + 2) * sizeof(int64_t), s))
      return -1;
    if (buf_ensure(e->sents, TB * sizeof(uint64_t), s)) return -1;
    // a pruning step recomputes the live flags: zeroed by the bucket count
    // (after the hit pass read them), re-marked by the prune
    if (prune && buf_ensure(e->live, std::max<int64_t>(NV + 4, 16), s)) return -1;
    NewOverride nov{override_, P<uint64_t>(e->shared), P<float>(c.pre), c.cap, e->pend_keep, pos, zero,
                    P<uint64_t>(c.pz)};
    TIMED("bucket_entries", 16.0 * M,  // + 8 B per entry, set once T is known
          // (member m >= S is members[m]: the hits sit at hoff >= S when the split found them)
          launch_bucket_entries(P<int32_t>(e->members) + (hoff >= 0 ? hoff - S : 0), S, V, M, grid, zero, idx, bg,
                                P<int32_t>(e->bk[0]), P<int32_t>(e->bk[1]), P<int64_t>(e->bk[2]),
                                P<int64_t>(e->bk[7]), P<uint64_t>(e->sents), e->bk_clean,
                                prune ? P<uint8_t>(e->live) : nullptr, NV, e->pend_fused ? &nov : nullptr,
                                ctr, s));
    e->bk_clean = false;  // until the grouping's pair-cell gather has reset the counters
    if (bg.sub) {
      // two-level geometry: the 16^3-cell buckets split into their 8^3-cell
      // octants (the grouping's buckets); the refine resets the counters
      if (buf_ensure(e->bk[8], ((int64_t)bg.NG + 1) * sizeof(int64_t), s)) return -1;
      if (buf_ensure(e->sents2, TB * sizeof(uint64_t), s)) return -1;
      TIMED("bucket_refine", 24.0 * M,  // 8 B read twice + 8 B written per entry (set once T is known)
            launch_bucket_refine(bg, P<int64_t>(e->bk[2]), P<uint64_t>(e->sents), P<int64_t>(e->bk[8]),
                                 P<uint64_t>(e->sents2), P<int32_t>(e->bk[0]), P<int32_t>(e->bk[1]), s));
    }
  } else {
    // radix-sort path (grids finer than the bucket geometry, TNP_RADIX_CELLS=1)
    if (buf_ensure(e->spcnt, std::max<int64_t>(M, 1) * sizeof(int32_t), s)) return -1;
    if (buf_ensure(e->spoff, std::max<int64_t>(M, 1) * sizeof(int64_t), s)) return -1;
    if (buf_ensure(e->part, (int64_t)(tnp_grid(M) + 1) * sizeof(int64_t), s)) return -1;
    TIMED("span_count", 28.0 * M,
          launch_span_count(P<int32_t>(e->members), S, M, grid, zero, idx, P<int32_t>(e->spcnt),
                            P<int64_t>(e->part), ctr, e->kw, s));
    if (scan_counts(e, P<int32_t>(e->spcnt), P<int64_t>(e->spoff), M, CTR_T, s)) return -1;
    if (buf_ensure(e->ekey_a, TB * sizeof(uint32_t), s)) return -1;
    if (buf_ensure(e->ent_v, TB * sizeof(int32_t), s)) return -1;
    if (buf_ensure(e->ekey_b, TB * sizeof(uint32_t), s)) return -1;
    if (buf_ensure(e->eval_b, TB * sizeof(int32_t), s)) return -1;
    TIMED("span_emit", 28.0 * M,
          launch_span_emit(P<int32_t>(e->members), S, M, grid, NC, P<int64_t>(e->spoff),
                           P<uint32_t>(e->ekey_a), P<int32_t>(e->ent_v), ctr, s));
    if (read_ctr(e, s)) return -1;
    if (e->h_ctr[CTR_K0]) {
      // the reference builds torch.cartesian_prod() of zero tensors (subpoly.py:317)
      tnp_set_error("meshgrid expects a non-empty TensorList (a region row without zeros, plane %d)", idx);
      return -1;
    }
    H = e->h_ctr[CTR_H];
    T = e->h_ctr[CTR_T];
    const int64_t T1 = std::max<int64_t>(T, 1);
    ktimer_set_bytes(e, 20.0 * M + 8.0 * T);  // span_emit's bytes, known only now
    int cbits = 1;
    while (cbits < 32 && (1ll << cbits) < ncell) ++cbits;
    uint32_t* skey = nullptr;
    int32_t* sval = nullptr;
    {
      size_t need = sort_pairs_scratch_bytes(T, cbits);
      if (buf_ensure(e->sort_scr2, std::max<size_t>(need, 16), s)) return -1;
      TIMED("cell_sort", 16.0 * T * ((cbits + 7) / 8),
            sort_pairs_u32(P<uint32_t>(e->ekey_a), P<uint32_t>(e->ekey_b), P<int32_t>(e->ent_v),
                           P<int32_t>(e->eval_b), T, cbits, e->sort_scr2.p, e->sort_scr2.bytes, &skey,
                           &sval, s));
    }
    // cells holding member pairs straight from the runs of the sorted keys
    // (compacted, with their flattened pair space offsets; total = tests)
    {
      if (buf_ensure(e->rstart, (T1 + 1) * sizeof(int32_t), s)) return -1;
      if (T > 0) {
        TnpLB la, lr, lp;
        if (lb_begin(e, run_tiles(T), s, &la, 0)) return -1;
        TIMED("run_starts", 8.0 * T,
              launch_run_starts(skey, T, P<int32_t>(e->rstart), ctr, la, s));
        const int64_t pt = pair_run_tiles(T);
        if (lb_begin(e, pt, s, &lr, 0) || lb_begin(e, pt, s, &lp, 1)) return -1;
        TIMED("pair_cells", 0.0,
              launch_pair_runs(skey, P<int32_t>(e->rstart), T, P<int32_t>(e->pcell), P<int32_t>(e->pent),
                               P<int32_t>(e->pcn), P<int64_t>(e->ptoff), ctr, lr, lp, s));
      }
    }
    TIMED("entry_keys", 52.0 * T,
          launch_entry_keys(sval, skey, NC, T, grid, P<uint64_t>(c.pz), e->ents.p, e->kw, s));
  }
  // 4. connecting edges: test every in-cell member pair once, append the
  //    emitted ones, radix-sort them (lexicographic c_new, subpoly.py:243-244).
  //    The pair count stays on the device; the chunk table and the key buffer
  //    keep their capacity across steps and grow (then redo) on overflow.
  int nb = 1;
  while (nb < 31 && (1ll << nb) < NV) ++nb;
  // connecting edges this step's pruning drops are never appended (sorted,
  // re-tested): keep_edge() depends on the endpoints only
  const uint64_t cfmask = prune ? prune_mask(idx, K - 1) : 0ull;
  // the kept keys go to XS_N per-XCD regions of cap / XS_N keys (step.h) on
  // grids of many bucket workgroups; small grids count in ctr directly
  const int NG = buckets ? bg.NG : 0;  // grouping workgroups
  const bool shard = !buckets || NG > 512;
  if (shard && buf_ensure(e->xs, XS_WORDS * sizeof(int64_t), s)) return -1;
  int64_t* const xs = shard ? P<int64_t>(e->xs) : nullptr;
  // small bucket grids: per-bucket statistics rows (plain stores) that the
  // connect kernel sums, instead of counter-block atomics from every bucket
  if (buckets && !shard && buf_ensure(e->bk[3], (int64_t)NG * 4 * sizeof(int64_t), s)) return -1;
  int64_t* const bstat = (buckets && !shard) ? P<int64_t>(e->bk[3]) : nullptr;
  int64_t cap = connect_key_cap(e->ckeys_a.bytes, M, XS_N);
  int64_t X = 0, TT = 0;
  bool chunks_ok = false;  // (radix path) the chunk table matches the pair cells
  // lazy edge deletion (k_prune_lazy) unless the list is mostly dead edges
  // already: then the compacting prune drops them (and this step's)
  // (split-eps mode: always lazy -- its first split planes are recomputed
  // over the edge slots in place, k_ef_cache)
  const int64_t E_live_in = e->E_live;
  const bool lazy = prune && (eps2(e) || (e->lazy_edges && (E - E_live_in) <= E_live_in));
  // the lazy prune's old edges and e_new need no connecting edge: they are
  // pruned while the connect counts travel to the host (slots [0, E + S)),
  // c_new after the sort (part A's workgroup parts first in lzpart)
  const bool early_prune = lazy && buckets && e->early_forward && !eps2(e) && !e->curve && e->masks_valid;
  int part_a = 0;
  const int64_t ES = E + S;
  // part A (slots [0, E + S)) reads the edge slots, their bytes, the keys of
  // the new vertices (forward_new; their override came with the bucket
  // count) and writes the slots' bytes, e_new and the live flags the bucket
  // count zeroed -- nothing the grouping, the connect, the key sort or their
  // counters touch.  So it runs on the side stream from here, beside them
  // (the grouping kernel issue-bound, the prune memory-bound), and the
  // caller's stream waits for it before the pruning of c_new (side_join)
  const bool side = early_prune && e->side_prune;
  if (early_prune) {
    if (buf_ensure(e->live, std::max<int64_t>(NV + 4, 16), s)) return -1;  // (+4: word atomics)
    if (buf_ensure(e->edges, std::max<int64_t>(ES, 1) * 2 * sizeof(int32_t), s, true)) return -1;
    if (buf_ensure(e->edm, std::max<int64_t>(ES, 1) * sizeof(uint8_t), s, true)) return -1;
    if (buf_ensure(e->eef, std::max<int64_t>(ES, 1) * sizeof(uint8_t), s, true)) return -1;
    part_a = prune_lazy_blocks(ES);
    if (buf_ensure(e->lzpart, part_a * sizeof(int64_t), s)) return -1;
  }
  if (side) {
    if (side_stream(e)) return -1;
    TNP_CHECK(hipEventRecord(e->ev_s2[0], s));
    TNP_CHECK(hipStreamWaitEvent(e->s2, e->ev_s2[0], 0));
    const int t = ktimer_begin(e, "prune", 1.0 * E + 36.0 * S, e->s2);
    if (launch_prune_lazy(P<int32_t>(e->edges), E, P<int32_t>(e->sb), S, V, nullptr, nb, 0, idx, K - 1,
                          P<uint64_t>(c.pz), P<uint8_t>(e->edm), P<uint8_t>(e->eef), P<uint8_t>(e->live),
                          P<int64_t>(e->lzpart), ctr, e->s2, 0, ES))
      return -1;
    ktimer_end(e, t, e->s2);
    TNP_CHECK(hipEventRecord(e->ev_s2[1], e->s2));
    e->s2_pending = true;
  }
  for (int attempt = 0; attempt < 3; ++attempt) {
    if (buf_ensure(e->ckeys_a, std::max<int64_t>(cap, 1) * sizeof(uint64_t), s)) return -1;
    if (attempt > 0) {  // the split zeroed the whole counter block
      TNP_CHECK(hipMemsetAsync(ctr + CTR_X, 0, sizeof(int64_t), s));
      TNP_CHECK(hipMemsetAsync(ctr + CTR_XK, 0, sizeof(int64_t), s));
      TNP_CHECK(hipMemsetAsync(ctr + CTR_P, 0, 2 * sizeof(int64_t), s));  // CTR_P, CTR_COMPAT
      TNP_CHECK(hipMemsetAsync(ctr + CTR_BOVF, 0, sizeof(int64_t), s));
      TNP_CHECK(hipMemsetAsync(ctr + CTR_PCK, 0, sizeof(int64_t), s));
      TNP_CHECK(hipMemsetAsync(ctr + CTR_SPAIRS, 0, sizeof(int64_t), s));
    }
    // the shards are left zero by k_keys_finish; cleared here after an
    // aborted step or on fresh memory
    if (shard && !e->xs_clean) TNP_CHECK(hipMemsetAsync(e->xs.p, 0, XS_WORDS * sizeof(int64_t), s));
    if (shard) e->xs_clean = false;
    if (buckets) {
      // in-bucket grouping + the window pass over each bucket (cells of <=
      // WCELL members) + pair-cell lists and k_connect's chunk table (bcap)
      if (buf_ensure(e->bcell, bcap * sizeof(int32_t), s)) return -1;
      const ConnectWin cw{idx, nb, cfmask, P<uint64_t>(e->ckeys_a), cap, xs, bstat,
                          e->packed_records && packed_ok(idx, K) ? 1 : 0};
      // the LDS-record path's cell-order scratch (TNP_LDS_RECORDS=0: off)
      const bool lrec = e->lds_records;
      if (lrec && buf_ensure(e->bk[4], TB * sizeof(uint64_t), s)) return -1;  // (entry words or indices)
      TIMED("bucket_group", 0.0,
            launch_bucket_pairs(bg, P<int64_t>(e->bk[bg.sub ? 8 : 2]), P<uint64_t>(bg.sub ? e->sents2 : e->sents),
                                P<uint64_t>(c.pz), P<CellEnt>(e->ents), P<int32_t>(e->pcell),
                                P<int32_t>(e->pent), P<int32_t>(e->pcn), P<int64_t>(e->ptoff),
                                P<int32_t>(e->bcell), bcap, P<int32_t>(e->bk[0]), P<int32_t>(e->bk[1]),
                                &cw, ctr, s, lrec ? P<int32_t>(e->bk[4]) : nullptr));
      e->bk_clean = true;
    } else if (!chunks_ok) {
      if (buf_ensure(e->bcell, bcap * sizeof(int32_t), s)) return -1;
      if (launch_chunk_cells(P<int64_t>(e->ptoff), P<int32_t>(e->pcn), RC,
                             P<int32_t>(e->bcell), bcap, ctr, s)) return -1;
    }
    // cells above WCELL members: the flattened pair space (every cell on the
    // radix path); the others: the window pass
    TIMED("connect", 0.0,
          launch_connect(P<int64_t>(e->ptoff), P<int32_t>(e->pcell), P<int32_t>(e->pcn),
                         P<int32_t>(e->pent), NC, e->max_pair_tests, P<int32_t>(e->bcell),
                         e->ents.p, idx, nb, prune ? K - 1 : -1, e->kw, P<uint64_t>(e->ckeys_a), cap, xs, ctr, s,
                         bstat, NG));
    if (shard) {
      if (launch_keys_finish(xs, cap, ctr, s)) return -1;
      e->xs_clean = true;
    }
    int64_t seq = 0;
    if (post_ctr(e, s, &seq)) return -1;
    if (early_prune && attempt == 0 && !side) {  // (a redone connect leaves part A as it is)
      TIMED("prune", 1.0 * E + 36.0 * S,
            launch_prune_lazy(P<int32_t>(e->edges), E, P<int32_t>(e->sb), S, V, nullptr, nb, 0, idx, K - 1,
                              P<uint64_t>(c.pz), P<uint8_t>(e->edm), P<uint8_t>(e->eef), P<uint8_t>(e->live),
                              P<int64_t>(e->lzpart), ctr, s, 0, ES));
    }
    if (wait_ctr(e, s, seq)) return -1;
    if (buckets) {
      // the atomically allocated pair-cell list: cells | pairs << 24
      e->h_ctr[CTR_R] = e->h_ctr[CTR_PCK] & (PCK_CELLS - 1);
      e->h_ctr[CTR_TESTS] = e->h_ctr[CTR_PCK] >> 24;
      if (e->h_ctr[CTR_K0] & 2) {
        tnp_set_error("plane %d: a vertex outside the mark planes [%d, %d] x [%d, %d] x [%d, %d] the engine "
                      "was given (tnp_engine_set_span)", idx, sp0[0], sp1[0], sp0[1], sp1[1], sp0[2], sp1[2]);
        return -1;
      }
      if (e->h_ctr[CTR_K0]) {
        // the reference builds torch.cartesian_prod() of zero tensors (subpoly.py:317)
        tnp_set_error("meshgrid expects a non-empty TensorList (a region row without zeros, plane %d)",
                      idx);
        return -1;
      }
      H = e->h_ctr[CTR_H];
      T = e->h_ctr[CTR_T];
      // entries: written once by the scatter; the grouping reads them, gathers
      // 16 B of member keys and writes the 32 B record; the window pass reads
      // every record (once, algorithmically) and writes the kept keys
      ktimer_set_bytes(e, "bucket_entries", 16.0 * M + 8.0 * T);
      if (bg.sub) ktimer_set_bytes(e, "bucket_refine", 24.0 * T);
      // the window pass re-reads the records the same workgroup just wrote
      // (cache traffic): its compulsory bytes are the kept keys.  LDS-record
      // path: 8 B entry word + 16 B member keys + 4 + 4 B cell order (written,
      // read back) per entry, records in memory only for k_connect's cells
      // (not counted: an understatement)
      ktimer_set_bytes(e, "bucket_group", (e->lds_records ? 32.0 : 56.0) * T + 8.0 * e->h_ctr[CTR_XK]);
    }
    TT = e->h_ctr[CTR_TESTS];
    X = e->h_ctr[CTR_XK];
    ktimer_set_bytes(e, 32.0 * TT + 8.0 * T);  // known only now
    if (e->h_ctr[CTR_BIG] || TT > e->max_pair_tests) {
      // one linear region holding ~sqrt(2*tests) vertices: the reference would
      // materialise every in-region pair (subpoly.py:505-518) and run out of
      // memory long before; refuse instead of grinding for hours
      tnp_set_error("degenerate complex at plane %d: %lld in-cell vertex pairs exceed the limit %lld "
                    "(TNP_MAX_PAIR_TESTS)", idx, (long long)TT, (long long)e->max_pair_tests);
      return -1;
    }
    if (e->h_ctr[CTR_BOVF]) {  // chunk table too small: grow, remap, redo
      bcap = connect_chunks(TT) + 1;
      chunks_ok = false;
      continue;
    }
    chunks_ok = true;
    if (X <= cap) break;
    cap = (X + XS_N - 1) / XS_N * XS_N;  // appended beyond the buffer: grow and redo
  }
  if (e->h_ctr[CTR_BOVF] || X > cap) { tnp_set_error("connect: capacity retry failed"); return -1; }
  if (e->h_ctr[CTR_COMPAT] == 0 && e->shards <= 1) {
    // every region has a single member: extract_every_valid_edge cats an
    // empty list (subpoly.py:505-513)
    tnp_set_error("torch.cat(): expected a non-empty list of Tensors (no region with two vertices, plane %d)", idx);
    return -1;
  }
  if (buf_ensure(e->ckeys_b, std::max<int64_t>(X, 1) * sizeof(uint64_t), s)) return -1;
  // sharded: the regions concatenated (a, per-XCD -> b), then sorted (b <-> a)
  uint64_t* kin = P<uint64_t>(e->ckeys_a);
  uint64_t* kalt = P<uint64_t>(e->ckeys_b);
  if (shard) {
    TIMED("keys_compact", 16.0 * X, launch_keys_compact(kin, cap, xs, X, kalt, s));
    std::swap(kin, kalt);
  }
  {
    size_t need = sort_lex_scratch_bytes(X, nb, e->sort_run);
    if (buf_ensure(e->sort_scr, std::max<size_t>(need, 16), s)) return -1;
    TIMED("pair_sort", 16.0 * X * ((2 * nb + 7) / 8),
          sort_keys_lex(kin, kalt, X, nb, e->sort_run, e->sort_scr.p, e->sort_scr.bytes, &e->ckeys, s));
  }

  // 5. pruning over [edges; e_new; c_new] + vertex compaction (after the side
  // stream's part A: everything below may move or read the edge slots)
  side_join(e, s);
  const int64_t N = E + S + X;
  int64_t nt = step_tiles(N);
  if (buf_ensure(e->blk, (nt + 1) * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->blkoff, (nt + 1) * sizeof(int64_t), s)) return -1;
  // ctr[CTR_ACTIVE] and ctr[CTR_V] are still zero from the split's reset
  const int32_t* eg = P<int32_t>(e->edges);
  int64_t V2 = NV, E2 = N, E2_live = N;
  bool defer = false;  // the live counts left to the next split (tnp_engine_run_steps)
  int next_valid = e->valid_from;
  bool swap_edges = true;
  if (prune) {
    // live flags recomputed from the kept edges; no vertex moves (lazy
    // compaction): the distinct flagged count is the reference's V'
    if (buf_ensure(e->live, std::max<int64_t>(NV + 4, 16), s)) return -1;  // +4: word atomics
    if (!buckets) TNP_CHECK(hipMemsetAsync(e->live.p, 0, NV, s));  // else zeroed by the bucket count
    // (word-atomic live counting inside the prune measured slower than the
    // counting pass even at bunny scale: 0.25 vs 0.13 + 0.07 ms per subpoly)
    const bool count_in_prune = false;
    // the run loop leaves the live counts to the next split's hit workers
    // (not in the kernel-timer pass: the prune's modelled bytes want them)
    BucketGeom bgd{};
    defer = e->defer_counts && !e->kt_on && !e->curve && !eps2(e) && uses_buckets(e, &bgd);
    // (curve path: recomputed after the rewiring, first split planes above idx)
    if (!e->masks_valid && compute_masks(e, idx + 1, nullptr, s)) return -1;
    const int64_t N1 = std::max<int64_t>(N, 1);
    if (lazy) {
      // in place: the slots grow to N (kept contents), nothing is compacted
      if (buf_ensure(e->edges, N1 * 2 * sizeof(int32_t), s, true)) return -1;
      if (buf_ensure(e->edm, N1 * sizeof(uint8_t), s, true)) return -1;
      if (buf_ensure(e->eef, N1 * sizeof(uint8_t), s, true)) return -1;
      // old edges: 1 B high plane (+ 1 B first split plane, 8 B ids when
      // kept); e_new / c_new: 4 / 8 B ids + 32 B endpoint keys, 10 B written
      // (part_a > 0: the old edges and e_new were pruned behind the connect)
      const int64_t i0 = part_a ? E + S : 0;
      const int nparts = part_a + prune_lazy_blocks(N - i0);
      if (buf_ensure(e->lzpart, nparts * sizeof(int64_t), s, part_a > 0)) return -1;
      TIMED("prune", part_a ? 40.0 * X : 1.0 * E + 36.0 * S + 40.0 * X,
            launch_prune_lazy(P<int32_t>(e->edges), E, P<int32_t>(e->sb), S, V, e->ckeys, nb, X, idx, K - 1,
                              P<uint64_t>(c.pz), P<uint8_t>(e->edm), P<uint8_t>(e->eef), P<uint8_t>(e->live),
                              P<int64_t>(e->lzpart) + part_a, ctr, s, i0, N));
      if (eps2(e)) {  // the first split planes at subpoly's eps, and their OR
        TNP_CHECK(hipMemsetAsync(ctr + CTR_ACTIVE, 0, sizeof(int64_t), s));
        TIMED("edge_masks", 8.0 * N,
              launch_ef_cache(P<int32_t>(e->edges), N, P<uint8_t>(e->edm), P<uint8_t>(e->eef), P<float>(c.pre),
                              c.cap, idx + 1, K, e->net.eps_s, ctr, s));
      }
      if (defer)
        e->pend_lz_n = nparts;
      else
        TIMED("count_live", 1.0 * NV,
              launch_count_flags(P<uint8_t>(e->live), NV, ctr, CTR_V, s, P<int64_t>(e->lzpart), nparts, CTR_E));
      swap_edges = false;
    } else {
      if (buf_ensure(e->edges_alt, N1 * 2 * sizeof(int32_t), s)) return -1;
      if (buf_ensure(e->edm_alt, N1 * sizeof(uint8_t), s)) return -1;
      if (buf_ensure(e->eef_alt, N1 * sizeof(uint8_t), s)) return -1;
      TnpLB lb;
      if (lb_begin(e, lb_tiles(N), s, &lb, 0, false)) return -1;
      // old edges: 8 B ids + 1 B high plane + 1 B first split plane read; e_new /
      // c_new: 4 / 8 B ids + 32 B endpoint keys; kept edges: 10 B written + 2 B flags
      TIMED("prune", 10.0 * E + 36.0 * S + 40.0 * X,
            launch_prune_lb(eg, E, P<int32_t>(e->sb), S, V, e->ckeys, nb, X, idx, K - 1,
                            P<uint64_t>(c.pz), P<uint8_t>(e->edm), P<uint8_t>(e->eef),
                            P<int32_t>(e->edges_alt), P<uint8_t>(e->edm_alt), P<uint8_t>(e->eef_alt),
                            P<uint8_t>(e->live), count_in_prune, ctr, lb, s));
      std::swap(e->edm, e->edm_alt);
      std::swap(e->eef, e->eef_alt);
      if (defer)
        e->pend_lz_n = 0;  // (E_live: the compacting prune's own count, read back below)
      else if (!count_in_prune)
        TIMED("count_live", 1.0 * NV, launch_count_flags(P<uint8_t>(e->live), NV, ctr, CTR_V, s));
    }
    next_valid = (e->keep_all || eps2(e)) ? 0 : std::min(idx + 1, K - 1);
    if (read_ctr(e, s, nullptr, 0, nullptr, 0, e->in_run)) return -1;
    E2_live = (defer && lazy) ? E_live_in : e->h_ctr[CTR_E];  // (deferred: set by apply_counts)
    E2 = lazy ? N : E2_live;
    ktimer_set_bytes(e, "prune", lazy ? 1.0 * E + 36.0 * S + 40.0 * X + 9.0 * E2_live
                                      : 10.0 * E + 36.0 * S + 40.0 * X + 12.0 * E2_live);
    V2 = e->h_ctr[CTR_V];
    // the kept edges' first split planes are above idx now
    e->mask_from = idx + 1;
    e->act_bits = (uint64_t)e->h_ctr[CTR_ACTIVE];
    e->dirty = true;
  } else if (E != E_live_in) {
    // the last plane (no pruning) behind lazily deleted edges: the
    // concatenation drops them (the compacting prune keeping every live edge)
    const int64_t N1 = std::max<int64_t>(N, 1);
    if (buf_ensure(e->edges_alt, N1 * 2 * sizeof(int32_t), s)) return -1;
    if (buf_ensure(e->edm_alt, N1 * sizeof(uint8_t), s)) return -1;
    if (buf_ensure(e->eef_alt, N1 * sizeof(uint8_t), s)) return -1;
    // (the live flags grow to the new slots first: the pass marks endpoints)
    if (set_alive(e, V, S, s)) return -1;
    TnpLB lb;
    if (lb_begin(e, lb_tiles(N), s, &lb, 0, false)) return -1;
    if (launch_prune_lb(eg, E, P<int32_t>(e->sb), S, V, e->ckeys, nb, X, -1, K - 1, P<uint64_t>(c.pz),
                        P<uint8_t>(e->edm), P<uint8_t>(e->eef), P<int32_t>(e->edges_alt),
                        P<uint8_t>(e->edm_alt), P<uint8_t>(e->eef_alt), P<uint8_t>(e->live), false, ctr, lb, s))
      return -1;
    std::swap(e->edm, e->edm_alt);
    std::swap(e->eef, e->eef_alt);
    V2 = e->V_live + S;
    e->masks_valid = false;
    if (read_ctr(e, s)) return -1;
    E2 = E2_live = e->h_ctr[CTR_E];
  } else {
    if (buf_ensure(e->edges_alt, std::max<int64_t>(N, 1) * 2 * sizeof(int32_t), s)) return -1;
    if (launch_prune(true, eg, E, P<int32_t>(e->sb), S, V, e->ckeys, nb, X, idx, 0, K - 1, pos, zero, nullptr, nullptr,
                     P<int32_t>(e->edges_alt), nullptr, ctr, s))
      return -1;
    if (set_alive(e, V, S, s)) return -1;
    V2 = e->V_live + S;
    e->masks_valid = false;  // the concatenated edge list carries no masks
    if (read_ctr(e, s)) return -1;
  }
  if (swap_edges) std::swap(e->edges, e->edges_alt);
  // the new vertices hold planes >= pend_keep only: valid_from never claims
  // the planes below (a step order that could read them needs keep_all)
  if (e->pend_fused) next_valid = std::max(next_valid, e->pend_keep);
  const int64_t V_in_live = e->V_live;
  e->V = NV;  // slots
  e->V_live = V2;
  e->E = E2;
  e->E_live = E2_live;
  e->valid_from = next_valid;
  if (defer) {  // V_live (and the lazy prune's E_live) arrive with the next split
    e->cnt_pending = true;
    e->pend_st = st;
  }
  if (st) {
    st->idx = idx;
    st->V_in = V_in_live;
    st->E_in = E_live_in;
    st->S = S;
    st->H = H;
    st->X = e->h_ctr[CTR_X];  // all connecting edges (X kept ones were appended)
    st->V_out = V2;
    st->E_out = E2_live;
    st->A = e->h_ctr[CTR_A];
    st->P = e->h_ctr[CTR_P];
    st->pair_tests = (e->h_ctr[CTR_PCK] ? (e->h_ctr[CTR_PCK] >> 24) : e->h_ctr[CTR_TESTS]) + e->h_ctr[CTR_SPAIRS];
    st->override_applied = override_ < 0 ? (e->h_ctr[CTR_FAIL] != 0) : override_;
    st->next_active = (uint64_t)e->h_ctr[CTR_ACTIVE];
    st->S_dup = e->curve ? e->h_ctr[CTR_DUP] : e->pend_dup;
    st->T = T;
  }
  e->valid = true;
  return 0;
}

// the hyperplane loop of subpoly.py:58-69 on one device, in the library:
// the same split / finish calls the Python driver makes per step, without a
// host-language round trip per step (bunny-scale steps are tens of us)
extern "C" int tnp_engine_run_steps(tnp_engine* e, void* stream, tnp_step_stats* stats, int max_stats,
                                    int* n_steps) {
  *n_steps = 0;
  if (e->shards > 1) {
    tnp_set_error("run_steps: a sharded engine takes its global decisions between split and finish");
    return -1;
  }
  uint64_t mask = 0;
  if (tnp_engine_active_planes(e, 0, &mask, stream)) return -1;
  const int K = e->K;
  // a pruning step's live counts are taken by the next split (deferred);
  // every exit path below resolves the last ones
  tnp_step_stats spare{};
  auto done = [&](int rc) -> int {
    e->in_run = false;
    e->ctr_zero = false;
    e->defer_counts = false;
    if (resolve_counts(e, (hipStream_t)stream)) rc = -1;
    e->pend_st = nullptr;
    return rc;
  };
  e->defer_counts = e->defer_ok;
  e->in_run = true;
  e->ctr_zero = false;
  for (int idx = 0; idx < K; ++idx) {
    if (!tnp::act_test(mask, idx)) continue;
    int64_t S = 0;
    int32_t fail = 0;
    if (tnp_engine_split(e, idx, stream, &S, &fail)) return done(-1);
    if (S == 0) continue;
    const int prune = idx < K - 1;  // the last plane never prunes
    tnp_step_stats* st = *n_steps < max_stats ? &stats[*n_steps] : &spare;
    *st = tnp_step_stats{};
    if (tnp_engine_finish(e, idx, prune, fail, stream, st)) return done(-1);
    ++*n_steps;
    // (planes >= 63 share bit 63: after such a step only the next-active word counts)
    if (prune) mask = idx >= 62 ? ((mask & ((1ull << 63) - 1ull)) | st->next_active)
                                : ((mask & ((2ull << idx) - 1ull)) | st->next_active);
  }
  return done(0);
}

extern "C" int tnp_engine_export(tnp_engine* e, float* d_xyz, int64_t* d_edges, float* d_pre,
                                 void* stream) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (require_valid(e, "export")) return -1;
  if (compact_now(e, s)) return -1;
  if (d_xyz && e->V > 0)
    TNP_CHECK(hipMemcpyAsync(d_xyz, e->cur.xyz.p, e->V * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
  if (d_edges && e->E > 0)
    hipLaunchKernelGGL(k_i32_to_i64, dim3(tnp_grid(2 * e->E)), dim3(TNP_BLOCK), 0, s,
                       P<int32_t>(e->edges), d_edges, 2 * e->E);
  if (d_pre && e->V > 0) {
    if (e->valid_from != 0) {
      tnp_set_error("cached planes below %d were dropped (load with keep_all_planes=1)", e->valid_from);
      return -1;
    }
    hipLaunchKernelGGL(k_planes_to_rows, dim3(tnp_grid(e->V)), dim3(TNP_BLOCK), 0, s,
                       P<float>(e->cur.pre), e->cur.cap, e->V, e->K, d_pre);
  }
  TNP_CHECK(hipGetLastError());
  return 0;
}

// extract_skeleton (subpoly.py:556-581)
extern "C" int tnp_engine_surface(tnp_engine* e, void* stream, int64_t* V_out, int64_t* E_out) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (require_valid(e, "surface")) return -1;
  if (compact_now(e, s)) return -1;
  const int64_t V = e->V, E = e->E;
  VSet& c = e->cur;
  const float* col = P<float>(c.pre) + (int64_t)(e->K - 1) * c.cap;
  if (buf_ensure(e->used, std::max<int64_t>(V, 1) * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->flags, std::max<int64_t>(V, 1) * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->nid, std::max<int64_t>(V, 1) * sizeof(int64_t), s)) return -1;
  TNP_CHECK(hipMemsetAsync(e->ctr.p, 0, CTR_CLEAR_BYTES, s));
  int32_t* on = P<int32_t>(e->flags);
  if (launch_surface_flags(P<float>(c.xyz), col, V, e->net.eps_s, on, s)) return -1;
  if (scan_counts(e, on, P<int64_t>(e->nid), V, CTR_AUX, s)) return -1;
  if (read_ctr(e, s)) return -1;
  if (e->h_ctr[CTR_AUX] < 3) {
    e->V = 0;
    e->E = 0;
    e->E_live = 0;
    *V_out = 0;
    *E_out = 0;
    return reset_live(e, s);
  }
  int64_t nt = step_tiles(E);
  if (buf_ensure(e->blk, (nt + 1) * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->blkoff, (nt + 1) * sizeof(int64_t), s)) return -1;
  if (buf_ensure(e->edges_alt, std::max<int64_t>(E, 1) * 2 * sizeof(int32_t), s)) return -1;
  const FillOp fu{e->used.p, (uint64_t)V * sizeof(int32_t), 0};
  if (launch_fill(&fu, 1, s)) return -1;
  if (launch_surface_edges(P<int32_t>(e->edges), E, on, P<int32_t>(e->blk), nullptr, 0, nullptr,
                           nullptr, s))
    return -1;
  if (scan_counts(e, P<int32_t>(e->blk), P<int64_t>(e->blkoff), nt, CTR_E, s)) return -1;
  if (launch_surface_edges(P<int32_t>(e->edges), E, on, nullptr, P<int64_t>(e->blkoff), 1,
                           P<int32_t>(e->edges_alt), P<int32_t>(e->used), s))
    return -1;
  if (scan_counts(e, P<int32_t>(e->used), P<int64_t>(e->nid), V, CTR_V, s)) return -1;
  if (vset_ensure(e, e->alt, V, 0, s)) return -1;
  VSet& a = e->alt;
  int keep_from = e->valid_from;
  if (launch_gather_vertices(P<int32_t>(e->used), P<int64_t>(e->nid), V, e->K, keep_from,
                             P<float>(c.xyz), P<float>(c.pre), c.cap, VP(c, e->kw),
                             VZ(c, e->kw), P<uint64_t>(c.grid), P<float>(a.xyz),
                             P<float>(a.pre), a.cap, VP(a, e->kw), VZ(a, e->kw),
                             P<uint64_t>(a.grid), P<uint64_t>(a.pz), s))
    return -1;
  if (read_ctr(e, s)) return -1;
  int64_t E2 = e->h_ctr[CTR_E], V2 = e->h_ctr[CTR_V];
  if (launch_remap_edges(P<int32_t>(e->edges_alt), E2, P<int64_t>(e->nid), s)) return -1;
  std::swap(e->cur, e->alt);
  std::swap(e->edges, e->edges_alt);
  e->V = V2;
  e->E = E2;
  e->E_live = E2;
  *V_out = V2;
  *E_out = E2;
  return reset_live(e, s);
}

// ---------------------------------------------------------------------------
// full lattice over the marks, box [lo, hi] of mark indices per axis
// (tropical.py:103-109 layout: x-edges, then y, then z, each (hi, lo),
// meshgrid-ij order; the whole grid is the reference's lattice, an x-slab or
// a block of a sharded one keeps the same order within the box)
// ---------------------------------------------------------------------------
namespace {
__global__ void k_lattice_vertices(const float* __restrict__ marks, int x0, int y0, int z0, int nx, int ny,
                                   int nz, float* __restrict__ xyz) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t nv = (int64_t)nx * ny * nz;
  if (v >= nv) return;
  int k = (int)(v % nz) + z0, j = (int)((v / nz) % ny) + y0, i = (int)(v / ((int64_t)ny * nz)) + x0;
  // preprocess_inverse: x * 2 - 1 (model.py:81-82)
  xyz[3 * v + 0] = __fsub_rn(__fmul_rn(marks[i], 2.0f), 1.0f);
  xyz[3 * v + 1] = __fsub_rn(__fmul_rn(marks[j], 2.0f), 1.0f);
  xyz[3 * v + 2] = __fsub_rn(__fmul_rn(marks[k], 2.0f), 1.0f);
}
__global__ void k_lattice_edges(int nx, int ny, int nz, int32_t* __restrict__ edges) {
  const int64_t NN = (int64_t)ny * nz;
  const int64_t ex = (int64_t)(nx - 1) * NN;
  const int64_t ey = (int64_t)nx * (ny - 1) * nz;
  const int64_t ez = (int64_t)nx * ny * (nz - 1);
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t lo, hi;
  if (e < ex) {
    lo = e;
    hi = e + NN;
  } else if (e < ex + ey) {
    int64_t r = e - ex;  // shape (nx, ny-1, nz)
    int64_t k = r % nz, j = (r / nz) % (ny - 1), i = r / ((int64_t)(ny - 1) * nz);
    lo = i * NN + j * nz + k;
    hi = lo + nz;
  } else if (e < ex + ey + ez) {
    int64_t r = e - ex - ey;  // shape (nx, ny, nz-1)
    int64_t k = r % (nz - 1), j = (r / (nz - 1)) % ny, i = r / ((int64_t)ny * (nz - 1));
    lo = i * NN + j * nz + k;
    hi = lo + 1;
  } else {
    return;
  }
  edges[2 * e] = (int32_t)hi;
  edges[2 * e + 1] = (int32_t)lo;
}
}  // namespace

extern "C" int tnp_engine_lattice_box(tnp_engine* e, const int32_t* lo3, const int32_t* hi3, int keep_all,
                                      void* stream, int64_t* V_out, int64_t* E_out) {
  hipStream_t s = (hipStream_t)stream;
  if (!e->has_net) { tnp_set_error("engine has no net"); return -1; }
  TNP_CHECK(hipSetDevice(e->device));
  const int N = e->net.n_marks;
  int n[3];
  for (int d = 0; d < 3; ++d) {
    if (lo3[d] < 0 || hi3[d] >= N || hi3[d] < lo3[d]) {
      tnp_set_error("bad lattice box: axis %d marks [%d, %d] of %d", d, lo3[d], hi3[d], N);
      return -1;
    }
    n[d] = hi3[d] - lo3[d] + 1;
    e->sp_lo[d] = lo3[d];
    e->sp_hi[d] = hi3[d];
  }
  const int64_t V = (int64_t)n[0] * n[1] * n[2];
  const int64_t E = (int64_t)(n[0] - 1) * n[1] * n[2] + (int64_t)n[0] * (n[1] - 1) * n[2] +
                    (int64_t)n[0] * n[1] * (n[2] - 1);
  if (V >= (1LL << 31) || E >= (1LL << 31)) { tnp_set_error("lattice too large for int32 ids"); return -1; }
  if (buf_ensure(e->ctr, CTR_CLEAR_BYTES, s)) return -1;
  if (vset_ensure(e, e->cur, V, 0, s)) return -1;
  if (buf_ensure(e->edges, std::max<int64_t>(E, 1) * 2 * sizeof(int32_t), s)) return -1;
  hipLaunchKernelGGL(k_lattice_vertices, dim3(tnp_grid(V)), dim3(TNP_BLOCK), 0, s, e->net.marks, lo3[0], lo3[1],
                     lo3[2], n[0], n[1], n[2], P<float>(e->cur.xyz));
  hipLaunchKernelGGL(k_lattice_edges, dim3(tnp_grid(E)), dim3(TNP_BLOCK), 0, s, n[0], n[1], n[2],
                     P<int32_t>(e->edges));
  TNP_CHECK(hipGetLastError());
  // the lattice's full forward (12 B coordinates in; K planes, 40 B of keys out)
  TIMED("forward", (12.0 + 4.0 * e->K + 40.0) * V + table_bytes(e->net),
        launch_forward(e->net, P<float>(e->cur.xyz), V, P<float>(e->cur.pre), e->cur.cap, 1, s, nullptr,
                       VP(e->cur, e->kw), VZ(e->cur, e->kw), P<uint64_t>(e->cur.grid),
                       P<uint64_t>(e->cur.pz)));
  e->V = V;
  e->E = E;
  e->E_live = E;
  e->keep_all = keep_all;
  e->valid_from = 0;
  e->pend_idx = -1;
  *V_out = V;
  *E_out = E;
  return reset_live(e, s);
}

extern "C" int tnp_engine_lattice(tnp_engine* e, int x0, int x1, int keep_all, void* stream,
                                  int64_t* V_out, int64_t* E_out) {
  if (!e->has_net) { tnp_set_error("engine has no net"); return -1; }
  const int N = e->net.n_marks;
  if (x0 < 0 || x1 >= N || x1 < x0) { tnp_set_error("bad slab [%d, %d] of %d marks", x0, x1, N); return -1; }
  const int32_t lo[3] = {x0, 0, 0}, hi[3] = {x1, N - 1, N - 1};
  return tnp_engine_lattice_box(e, lo, hi, keep_all, stream, V_out, E_out);
}

// ---------------------------------------------------------------------------
// skeleton (tropical.py:158-225) + hypercube fallback (subpoly.py:51-52)
// ---------------------------------------------------------------------------
#include <vector>

#include "skeleton.h"

static int load_hypercube(tnp_engine* e, float size, hipStream_t s) {
  float x[2] = {-size, size};
  std::vector<float> v;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k < 2; ++k) {
        v.push_back(x[i]);
        v.push_back(x[j]);
        v.push_back(x[k]);
      }
  std::vector<int32_t> ed;
  for (int i = 0; i < 8; ++i)
    for (int j = i + 1; j < 8; ++j) {
      int neg = 0;
      for (int d = 0; d < 3; ++d) neg += (v[3 * i + d] * v[3 * j + d] < 0.f);
      if (neg == 1) {
        ed.push_back(i);
        ed.push_back(j);
      }
    }
  if (vset_ensure(e, e->cur, 8, 0, s)) return -1;
  if (buf_ensure(e->edges, ed.size() * sizeof(int32_t), s)) return -1;
  TNP_CHECK(hipMemcpyAsync(e->cur.xyz.p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice, s));
  TNP_CHECK(hipMemcpyAsync(e->edges.p, ed.data(), ed.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
  TNP_CHECK(hipStreamSynchronize(s));  // host vectors go out of scope
  e->V = 8;
  e->E = (int64_t)ed.size() / 2;
  e->E_live = (int64_t)ed.size() / 2;
  return 0;
}

extern "C" int tnp_engine_skeleton(tnp_engine* e, int unit, float size, void* stream, int64_t* V_out,
                                   int64_t* E_out) {
  return tnp_engine_skeleton_mode(e, unit, size, TNP_SKELETON_DISTANCE, stream, V_out, E_out);
}

// torch.diff(marks).max().item() (the skeleton's edge-length bound)
static int marks_dmax(tnp_engine* e, hipStream_t s, float* dmax) {
  const int L = e->net.n_marks;
  std::vector<float> mk(L);
  TNP_CHECK(hipMemcpyAsync(mk.data(), e->net.marks, L * sizeof(float), hipMemcpyDeviceToHost, s));
  TNP_CHECK(hipStreamSynchronize(s));
  float d = -INFINITY;
  for (int i = 0; i + 1 < L; ++i) d = std::max(d, mk[i + 1] - mk[i]);
  *dmax = d;
  return 0;
}

// the reference's skeleton tiles (tropical.py:176-181): starts range(0, L,
// unit - 1) per axis, unit marks each (1-mark overlap), x-major order
struct SkelTile {
  int o[3], n[3];
};
static std::vector<SkelTile> skeleton_tiles(int L, int unit) {
  std::vector<SkelTile> t;
  for (int i0 = 0; i0 < L; i0 += unit - 1)
    for (int j0 = 0; j0 < L; j0 += unit - 1)
      for (int k0 = 0; k0 < L; k0 += unit - 1)
        t.push_back(SkelTile{{i0, j0, k0},
                             {std::min(L, i0 + unit) - i0, std::min(L, j0 + unit) - j0, std::min(L, k0 + unit) - k0}});
  return t;
}

// TropicalHashGrid.skeleton on the device.  box_lo / box_hi (distance mode
// only): the part of the skeleton inside the mark box [lo, hi] -- every tile
// meeting the box evaluated on tile & box only, with its max |grad sdf| from
// tile_gmax (device, one word per tile: the whole tile's, tnp_engine_
// skeleton_gmax); the edges (both endpoints in the box) come out in the
// whole skeleton's order, so the result is box_restrict of the whole one.
static int skeleton_build(tnp_engine* e, int unit, float size, int mode, const int32_t* box_lo,
                          const int32_t* box_hi, const unsigned int* tile_gmax, hipStream_t s, int64_t* V_out,
                          int64_t* E_out) {
  if (!e->has_net) { tnp_set_error("engine has no net"); return -1; }
  if (unit < 2) { tnp_set_error("unit must be >= 2"); return -1; }
  TNP_CHECK(hipSetDevice(e->device));
  span_all(e);  // the whole grid
  const int L = e->net.n_marks;
  if ((int64_t)L * L * L >= (1LL << 31)) { tnp_set_error("too many marks for int32 ids"); return -1; }
  float dmax;
  if (marks_dmax(e, s, &dmax)) return -1;
  if (buf_ensure(e->ctr, CTR_CLEAR_BYTES, s)) return -1;
  const int64_t LLL = (int64_t)L * L * L;
  if (buf_ensure(e->used, LLL * sizeof(int32_t), s)) return -1;
  if (buf_ensure(e->nid, LLL * sizeof(int64_t), s)) return -1;
  const FillOp fu{e->used.p, (uint64_t)LLL * sizeof(int32_t), 0};
  if (launch_fill(&fu, 1, s)) return -1;
  if (mode != TNP_SKELETON_DISTANCE && mode != TNP_SKELETON_SIGN) {
    tnp_set_error("skeleton mode %d (0: distance, 1: sign)", mode);
    return -1;
  }
  const bool sign = mode == TNP_SKELETON_SIGN;
  const bool box = box_lo != nullptr;
  if (box && (sign || !tile_gmax)) {
    tnp_set_error("skeleton box: distance mode with the tiles' max |grad sdf| only");
    return -1;
  }
  int64_t tile_pts = (int64_t)std::min(unit, L) * std::min(unit, L) * std::min(unit, L);
  if (buf_ensure(e->stage, tile_pts * sizeof(float) * (sign ? e->K : 1), s)) return -1;
  // sign mode: the tile's points, their forward and packed keys (grid words;
  // pz: (pos, zero) interleaved, 2 kw words a point) in the curve path's
  // scratch slots
  Buf* sk = e->cv;
  if (sign) {
    if (buf_ensure(sk[CV_CORNERS], tile_pts * 3 * sizeof(float), s)) return -1;
    if (buf_ensure(sk[CV_GG], tile_pts * sizeof(uint64_t), s)) return -1;
    if (buf_ensure(sk[CV_STAGE_C], tile_pts * 2 * e->kw * sizeof(uint64_t), s)) return -1;
  }
  if (buf_ensure(e->shared, 16, s)) return -1;
  unsigned int* gmax = P<unsigned int>(e->shared);
  const std::vector<SkelTile> tiles = skeleton_tiles(L, unit);
  int64_t total = 0;
  for (size_t t = 0; t < tiles.size(); ++t) {
    int o[3], n[3];
    bool empty = false;
    for (int d = 0; d < 3; ++d) {
      o[d] = tiles[t].o[d];
      n[d] = tiles[t].n[d];
      if (box) {  // tile & box
        const int a = std::max(o[d], box_lo[d]), b = std::min(o[d] + n[d] - 1, box_hi[d]);
        empty |= b < a;
        o[d] = a;
        n[d] = b - a + 1;
      }
    }
    if (empty) continue;
    const int i0 = o[0], j0 = o[1], k0 = o[2], n0 = n[0], n1 = n[1], n2 = n[2];
    const uint64_t* keys = nullptr;
    const unsigned int* gm = box ? tile_gmax + t : gmax;
    if (sign) {
      // Net.region on the tile's vertices (tropical.py:199-201): the
      // forward of every point with its eps-sign keys
      const int64_t np_ = (int64_t)n0 * n1 * n2;
      if (launch_skel_points(i0, j0, k0, n0, n1, n2, e->net.marks, P<float>(sk[CV_CORNERS]), s)) return -1;
      if (launch_forward(e->net, P<float>(sk[CV_CORNERS]), np_, P<float>(e->stage), np_, 1, s, nullptr,
                         P<uint64_t>(sk[CV_STAGE_C]), P<uint64_t>(sk[CV_STAGE_C]) + e->kw,
                         P<uint64_t>(sk[CV_GG]), P<uint64_t>(sk[CV_STAGE_C])))
        return -1;
      keys = P<uint64_t>(sk[CV_STAGE_C]);
    } else {
      // (box: the sub-tile's |sdf|; its own gradient maximum is not used)
      TNP_CHECK(hipMemsetAsync(gmax, 0, sizeof(unsigned int), s));
      if (launch_skel_eval(e->net, i0, j0, k0, n0, n1, n2, P<float>(e->stage), gmax, s)) return -1;
    }
    int64_t N = skel_candidates(n0, n1, n2);
    int64_t nt = skel_tiles(N);
    if (nt == 0) continue;
    if (buf_ensure(e->blk, (nt + 1) * sizeof(int32_t), s)) return -1;
    if (buf_ensure(e->blkoff, (nt + 1) * sizeof(int64_t), s)) return -1;
    if (launch_skel_edges(false, i0, j0, k0, n0, n1, n2, L, P<float>(e->stage), keys, dmax, gm,
                          P<int32_t>(e->blk), nullptr, 0, nullptr, nullptr, s, e->kw))
      return -1;
    if (scan_counts(e, P<int32_t>(e->blk), P<int64_t>(e->blkoff), nt, CTR_AUX, s)) return -1;
    if (read_ctr(e, s)) return -1;
    int64_t cnt = e->h_ctr[CTR_AUX];
    if (cnt > 0) {
      if (buf_ensure(e->edges_alt, (total + cnt) * 2 * sizeof(int32_t), s, true)) return -1;
      if (launch_skel_edges(true, i0, j0, k0, n0, n1, n2, L, P<float>(e->stage), keys, dmax, gm,
                            nullptr, P<int64_t>(e->blkoff), total, P<int32_t>(e->edges_alt),
                            P<int32_t>(e->used), s, e->kw))
        return -1;
    }
    total += cnt;
  }
  e->pend_idx = -1;
  e->valid_from = 0;
  if (total == 0 && !box) {
    if (load_hypercube(e, size, s)) return -1;
  } else {
    // (box: a box without skeleton edges holds an empty complex -- the whole
    // skeleton's emptiness, the hypercube fallback, is the caller's check)
    if (scan_counts(e, P<int32_t>(e->used), P<int64_t>(e->nid), LLL, CTR_V, s)) return -1;
    if (read_ctr(e, s)) return -1;
    int64_t V = e->h_ctr[CTR_V];
    if (vset_ensure(e, e->cur, std::max<int64_t>(V, 1), 0, s)) return -1;
    if (launch_skel_vertices(P<int32_t>(e->used), P<int64_t>(e->nid), LLL, L, e->net.marks,
                             P<float>(e->cur.xyz), s))
      return -1;
    if (launch_remap_i32(P<int32_t>(e->edges_alt), 2 * total, P<int64_t>(e->nid), s)) return -1;
    if (total > 0) std::swap(e->edges, e->edges_alt);
    e->V = V;
    e->E = total;
    e->E_live = total;
  }
  if (launch_forward(e->net, P<float>(e->cur.xyz), e->V, P<float>(e->cur.pre), e->cur.cap, 1, s, nullptr,
                     VP(e->cur, e->kw), VZ(e->cur, e->kw), P<uint64_t>(e->cur.grid),
                     P<uint64_t>(e->cur.pz)))
    return -1;
  e->keep_all = 0;
  *V_out = e->V;
  *E_out = e->E;
  return reset_live(e, s);
}

extern "C" int tnp_engine_skeleton_mode(tnp_engine* e, int unit, float size, int mode, void* stream,
                                        int64_t* V_out, int64_t* E_out) {
  return skeleton_build(e, unit, size, mode, nullptr, nullptr, nullptr, (hipStream_t)stream, V_out, E_out);
}

extern "C" int tnp_engine_skeleton_gmax(tnp_engine* e, int unit, int rank, int world, uint32_t* h_gmax,
                                        int64_t* h_load, int cap, int* n_tiles, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!e->has_net) { tnp_set_error("engine has no net"); return -1; }
  if (unit < 2 || world < 1 || rank < 0 || rank >= world) {
    tnp_set_error("skeleton_gmax: unit %d, rank %d of %d", unit, rank, world);
    return -1;
  }
  TNP_CHECK(hipSetDevice(e->device));
  const int L = e->net.n_marks;
  const std::vector<SkelTile> tiles = skeleton_tiles(L, unit);
  *n_tiles = (int)tiles.size();
  if ((int)tiles.size() > cap) {
    tnp_set_error("skeleton_gmax: %d tiles, room for %d", (int)tiles.size(), cap);
    return -1;
  }
  float dmax;
  if (marks_dmax(e, s, &dmax)) return -1;
  const int64_t T = (int64_t)tiles.size();
  int64_t tile_pts = (int64_t)std::min(unit, L) * std::min(unit, L) * std::min(unit, L);
  if (buf_ensure(e->stage, tile_pts * sizeof(float), s)) return -1;
  // [T] gmax words, then [3][L] int64 load counts
  const size_t gbytes = (size_t)((T + 1) / 2 * 2) * sizeof(uint32_t);
  if (buf_ensure(e->fscr[0], gbytes + 3 * (size_t)L * sizeof(int64_t), s)) return -1;
  unsigned int* gm = P<unsigned int>(e->fscr[0]);
  int64_t* load = reinterpret_cast<int64_t*>(static_cast<char*>(e->fscr[0].p) + gbytes);
  TNP_CHECK(hipMemsetAsync(e->fscr[0].p, 0, gbytes + 3 * (size_t)L * sizeof(int64_t), s));
  for (int64_t t = rank; t < T; t += world) {
    const SkelTile& q = tiles[t];
    if (launch_skel_eval(e->net, q.o[0], q.o[1], q.o[2], q.n[0], q.n[1], q.n[2], P<float>(e->stage), gm + t, s))
      return -1;
    if (launch_skel_load(q.o[0], q.o[1], q.o[2], q.n[0], q.n[1], q.n[2], L, P<float>(e->stage), dmax, gm + t,
                         load, s))
      return -1;
  }
  TNP_CHECK(hipMemcpyAsync(h_gmax, gm, T * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (h_load) TNP_CHECK(hipMemcpyAsync(h_load, load, 3 * (size_t)L * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TNP_CHECK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int tnp_engine_skeleton_box(tnp_engine* e, int unit, const int32_t* lo, const int32_t* hi,
                                       const uint32_t* h_gmax, int n_tiles, void* stream, int64_t* V_out,
                                       int64_t* E_out) {
  hipStream_t s = (hipStream_t)stream;
  if (!e->has_net) { tnp_set_error("engine has no net"); return -1; }
  TNP_CHECK(hipSetDevice(e->device));
  const int L = e->net.n_marks;
  if ((int)skeleton_tiles(L, unit).size() != n_tiles) {
    tnp_set_error("skeleton_box: %d tile maxima for %d tiles", n_tiles, (int)skeleton_tiles(L, unit).size());
    return -1;
  }
  for (int d = 0; d < 3; ++d)
    if (lo[d] < 0 || hi[d] >= L || lo[d] > hi[d]) {
      tnp_set_error("skeleton_box: axis %d box [%d, %d] outside the %d marks", d, lo[d], hi[d], L);
      return -1;
    }
  if (buf_ensure(e->fscr[1], (size_t)std::max(n_tiles, 1) * sizeof(uint32_t), s)) return -1;
  TNP_CHECK(hipMemcpyAsync(e->fscr[1].p, h_gmax, n_tiles * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  return skeleton_build(e, unit, 0.f, TNP_SKELETON_DISTANCE, lo, hi, P<unsigned int>(e->fscr[1]), s, V_out, E_out);
}

// ---------------------------------------------------------------------------
// extract_faces (subpoly.py:584-728) on the current complex
// ---------------------------------------------------------------------------
#include "faces.h"

enum { FS_TABLE, FS_CNT, FS_KC, FS_KF, FS_MEMOFF, FS_RID, FS_MEM, FS_CUR, FS_ROFF, FS_RCNT,
       FS_BCNT, FS_BOFF, FS_BCUR, FS_ROWS, FS_KEEP, FS_KOFF, FS_FROW, FS_MEAN, FS_NRM, FS_SDF,
       FS_KEY, FS_ORDV, FS_CALL, FS_CNZ, FS_HIST, FS_BASE, FS_N };

extern "C" int tnp_engine_faces(tnp_engine* e, void* stream, int64_t* n_tri, int64_t* n_faces) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (require_valid(e, "faces")) return -1;
  if (compact_now(e, s)) return -1;
  static_assert(FS_N <= 32, "face scratch slots");
  Buf* fs = e->fscr2;
  const int64_t V = e->V;
  const int K = e->K;
  e->n_tri = e->n_faces = 0;
  *n_tri = *n_faces = 0;
  if (V == 0) return 0;
  if (e->net.n_marks + 2 >= 1024) {
    tnp_set_error("faces: region keys hold n_marks + 2 < 1024 cells per axis");
    return -1;
  }
  int64_t* ctr = P<int64_t>(e->ctr);
  const uint64_t* pos = VP(e->cur, e->kw);
  const uint64_t* zero = VZ(e->cur, e->kw);
  const uint64_t* grid = P<uint64_t>(e->cur.grid);
  const float* xyz = P<float>(e->cur.xyz);
  if (eps2(e)) {
    // extract_faces takes the regions at subpoly's eps (net.region(vertices,
    // outputs, eps), subpoly.py:606): keys of every plane from the cache
    if (e->valid_from != 0) { tnp_set_error("split-eps faces: cached planes were dropped"); return -1; }
    // kse[0]: the keys at subpoly's eps, (pos, zero) interleaved as pz; kse[2]: grid words
    for (int k = 0; k < 3; k += 2)
      if (buf_ensure(e->kse[k], V * sizeof(uint64_t) * (k == 0 ? 2 * e->kw : 1), s)) return -1;
    NetDev ns = e->net;
    ns.eps = ns.eps_s;
    if (launch_keys(ns, xyz, P<float>(e->cur.pre), e->cur.cap, V, K, P<uint64_t>(e->kse[0]),
                    P<uint64_t>(e->kse[0]) + e->kw, P<uint64_t>(e->kse[2]), s, P<uint64_t>(e->kse[0])))
      return -1;
    pos = P<uint64_t>(e->kse[0]);
    zero = P<uint64_t>(e->kse[0]) + e->kw;
    grid = P<uint64_t>(e->kse[2]);
  }
  TNP_CHECK(hipMemsetAsync(ctr, 0, CTR_CLEAR_BYTES, s));
  // F1: augmented-row count and region hash table
  TIMED("faces_count", 24.0 * V,
        launch_face_count(V, grid, pos, zero, K, ctr + CTR_AUX - 1, s));
  if (read_ctr(e, s)) return -1;
  const int64_t A = e->h_ctr[CTR_AUX - 1];
  if (e->h_ctr[CTR_AUX] > 30) { tnp_set_error("faces: a vertex lies on %lld planes", (long long)e->h_ctr[CTR_AUX]); return -1; }
  int64_t cap = 1024;
  while (cap < 2 * A) cap <<= 1;
  // region table: cap sign words + cap cell words (faces.hip probe_insert);
  // two-word keys: cap cell words + 2 cap sign words + cap ready words
  if (buf_ensure(fs[FS_TABLE], cap * 16 * e->kw, s) || buf_ensure(fs[FS_CNT], cap * 4, s) ||
      buf_ensure(fs[FS_KC], cap * 4, s) || buf_ensure(fs[FS_KF], cap * 4, s) ||
      buf_ensure(fs[FS_MEMOFF], cap * 8, s) || buf_ensure(fs[FS_RID], cap * 8, s) ||
      buf_ensure(fs[FS_CUR], cap * 4, s))
    return -1;
  if (e->kw == 1) {  // EMPTY signs, NO_CELL, counts, cursors: one dispatch
    const FillOp f[4] = {{fs[FS_TABLE].p, (uint64_t)cap * 8, 0xFF},
                         {static_cast<char*>(fs[FS_TABLE].p) + cap * 8, (uint64_t)cap * 8, 0},
                         {fs[FS_CNT].p, (uint64_t)cap * 4, 0},
                         {fs[FS_CUR].p, (uint64_t)cap * 4, 0}};
    if (launch_fill(f, 4, s)) return -1;
  } else {  // NO_CELL claim words and not-ready words (the sign words are written before use)
    const FillOp f[4] = {{fs[FS_TABLE].p, (uint64_t)cap * 8, 0},
                         {static_cast<char*>(fs[FS_TABLE].p) + cap * 24, (uint64_t)cap * 8, 0},
                         {fs[FS_CNT].p, (uint64_t)cap * 4, 0},
                         {fs[FS_CUR].p, (uint64_t)cap * 4, 0}};
    if (launch_fill(f, 4, s)) return -1;
  }
  TIMED("faces_insert", 24.0 * V + 16.0 * cap,
        launch_face_insert(V, grid, pos, zero, K, P<uint64_t>(fs[FS_TABLE]), (uint64_t)cap - 1,
                         P<int32_t>(fs[FS_CNT]), s));
  TIMED("faces_keep_counts", 12.0 * cap,
        launch_keep_counts(P<int32_t>(fs[FS_CNT]), cap, P<int32_t>(fs[FS_KC]), P<int32_t>(fs[FS_KF]), s));
  // padded width of r_idx_as_tensor = the largest region over ALL regions
  {
    const FillOp f{ctr + CTR_COMPAT, sizeof(int64_t), 0};
    if (launch_fill(&f, 1, s)) return -1;
  }
  TIMED("faces_width", 4.0 * cap,
        launch_max_i32(P<int32_t>(fs[FS_CNT]), cap, ctr + CTR_COMPAT, s));
  if (scan_counts(e, P<int32_t>(fs[FS_KC]), P<int64_t>(fs[FS_MEMOFF]), cap, CTR_T, s)) return -1;
  if (scan_counts(e, P<int32_t>(fs[FS_KF]), P<int64_t>(fs[FS_RID]), cap, CTR_X, s)) return -1;
  if (read_ctr(e, s)) return -1;
  const int64_t Mtot = e->h_ctr[CTR_T], R = e->h_ctr[CTR_X];
  const int width = (int)e->h_ctr[CTR_COMPAT];
  if (width > (1 << 16)) {
    tnp_set_error("faces: a region with %d vertices (degenerate complex)", width);
    return -1;
  }
  if (R == 0) return 0;
  // F2: member lists (k, v)-sorted
  if (buf_ensure(fs[FS_MEM], Mtot * 8, s) || buf_ensure(fs[FS_ROFF], R * 8, s) ||
      buf_ensure(fs[FS_RCNT], R * 4, s))
    return -1;
  TIMED("faces_scatter", 24.0 * V + 8.0 * Mtot,
        launch_face_scatter(V, grid, pos, zero, K, P<uint64_t>(fs[FS_TABLE]), (uint64_t)cap - 1,
                          P<int32_t>(fs[FS_CNT]), P<int64_t>(fs[FS_MEMOFF]), P<int32_t>(fs[FS_CUR]),
                          P<uint64_t>(fs[FS_MEM]), s));
  TIMED("faces_regions", 16.0 * cap + 12.0 * R,
        launch_region_finalize(cap, P<int32_t>(fs[FS_KF]), P<int64_t>(fs[FS_RID]), P<int32_t>(fs[FS_CNT]),
                             P<int64_t>(fs[FS_MEMOFF]), P<uint64_t>(fs[FS_MEM]), P<int64_t>(fs[FS_ROFF]),
                             P<int32_t>(fs[FS_RCNT]), s));
  // F3: lexicographic row order + unique
  if (buf_ensure(fs[FS_BCNT], V * 4, s) || buf_ensure(fs[FS_BOFF], V * 8, s) ||
      buf_ensure(fs[FS_BCUR], V * 4, s) || buf_ensure(fs[FS_ROWS], R * 4, s) ||
      buf_ensure(fs[FS_KEEP], R * 4, s) || buf_ensure(fs[FS_KOFF], R * 8, s))
    return -1;
  {
    const FillOp f[2] = {{fs[FS_BCNT].p, (uint64_t)V * 4, 0}, {fs[FS_BCUR].p, (uint64_t)V * 4, 0}};
    if (launch_fill(f, 2, s)) return -1;
  }
  const uint64_t* mem = P<uint64_t>(fs[FS_MEM]);
  const int64_t* roff = P<int64_t>(fs[FS_ROFF]);
  const int32_t* rcnt = P<int32_t>(fs[FS_RCNT]);
  TIMED("faces_row_count", 8.0 * Mtot + 12.0 * R,
        launch_row_buckets(R, V, mem, roff, rcnt, P<int32_t>(fs[FS_BCNT]), nullptr, nullptr, nullptr, nullptr, 0, s));
  if (scan_counts(e, P<int32_t>(fs[FS_BCNT]), P<int64_t>(fs[FS_BOFF]), V, CTR_AUX, s)) return -1;
  TIMED("faces_row_place", 8.0 * Mtot + 16.0 * R,
        launch_row_buckets(R, V, mem, roff, rcnt, nullptr, P<int64_t>(fs[FS_BOFF]), P<int32_t>(fs[FS_BCUR]),
                         P<int32_t>(fs[FS_ROWS]), nullptr, 1, s));
  TIMED("faces_row_unique", 8.0 * Mtot + 16.0 * R,
        launch_row_buckets(R, V, mem, roff, rcnt, P<int32_t>(fs[FS_BCNT]), P<int64_t>(fs[FS_BOFF]), nullptr,
                         P<int32_t>(fs[FS_ROWS]), P<int32_t>(fs[FS_KEEP]), 2, s));
  if (scan_counts(e, P<int32_t>(fs[FS_KEEP]), P<int64_t>(fs[FS_KOFF]), R, CTR_E, s)) return -1;
  if (read_ctr(e, s)) return -1;
  const int64_t F = e->h_ctr[CTR_E];
  if (buf_ensure(fs[FS_FROW], F * 4, s) || buf_ensure(fs[FS_MEAN], F * 12, s) ||
      buf_ensure(fs[FS_NRM], F * 12, s) || buf_ensure(fs[FS_SDF], F * 4, s) ||
      buf_ensure(fs[FS_KEY], row_order_scratch(F, width), s) || buf_ensure(fs[FS_ORDV], Mtot * 4, s) ||
      buf_ensure(fs[FS_CALL], F * 4, s) || buf_ensure(fs[FS_CNZ], F * 4, s))
    return -1;
  TIMED("faces_compact_rows", 16.0 * R,
        launch_compact_rows(R, P<int32_t>(fs[FS_KEEP]), P<int64_t>(fs[FS_KOFF]), P<int32_t>(fs[FS_ROWS]),
                          P<int32_t>(fs[FS_FROW]), s));
  const int32_t* frow = P<int32_t>(fs[FS_FROW]);
  e->dbg_F = F;
  e->dbg_W = width;
  // F4: normals at the row means, angular order
  TIMED("faces_row_mean", 20.0 * Mtot + 12.0 * F,
        launch_row_mean(F, frow, mem, roff, rcnt, width, xyz, P<float>(fs[FS_MEAN]), s));
  TIMED("faces_normals", 28.0 * F,
        launch_sdf_grad(e->net, P<float>(fs[FS_MEAN]), F, P<float>(fs[FS_SDF]), P<float>(fs[FS_NRM]), s));
  TIMED("faces_row_order", 20.0 * Mtot + 12.0 * F,
        launch_row_order(F, frow, mem, roff, rcnt, width, xyz, P<float>(fs[FS_NRM]), F == 3 ? 1 : 0,
                       fs[FS_KEY].p, P<int32_t>(fs[FS_ORDV]), P<int32_t>(fs[FS_CALL]),
                       P<int32_t>(fs[FS_CNZ]), s));
  {
    const FillOp f{ctr + CTR_TRI, 2 * sizeof(int64_t), 0};
    if (launch_fill(&f, 1, s)) return -1;
  }
  TIMED("faces_fan_width", 8.0 * F,
        launch_max_i32(P<int32_t>(fs[FS_CALL]), F, ctr + CTR_TRI, s, P<int32_t>(fs[FS_CNZ]), ctr + CTR_FACES));
  if (read_ctr(e, s)) return -1;
  // F5: fan triangles, fan-position-major
  const int64_t nb = fan_blocks(F);
  for (int floats = 0; floats < 2; ++floats) {
    const int32_t* cnt = P<int32_t>(fs[floats ? FS_CNZ : FS_CALL]);
    int T = (int)e->h_ctr[floats ? CTR_FACES : CTR_TRI] - 2;
    if (T <= 0) continue;
    if (buf_ensure(fs[FS_HIST], (int64_t)T * nb * 4, s) || buf_ensure(fs[FS_BASE], (int64_t)T * nb * 8, s))
      return -1;
    TIMED("faces_fan_hist", 4.0 * F,
        launch_fan_hist(F, cnt, T, P<int32_t>(fs[FS_HIST]), s));
    if (scan_counts(e, P<int32_t>(fs[FS_HIST]), P<int64_t>(fs[FS_BASE]), (int64_t)T * nb, CTR_AUX, s)) return -1;
    if (read_ctr(e, s)) return -1;
    int64_t n = e->h_ctr[CTR_AUX];
    if (floats) {
      if (buf_ensure(e->faces, std::max<int64_t>(n, 1) * 9 * sizeof(float), s)) return -1;
      e->n_faces = n;
    } else {
      if (buf_ensure(e->tri, std::max<int64_t>(n, 1) * 3 * sizeof(int64_t), s)) return -1;
      e->n_tri = n;
    }
    TIMED("faces_fan_emit", (floats ? 36.0 : 24.0) * n + 8.0 * F,
        launch_fan_emit(F, frow, P<int32_t>(fs[FS_ORDV]), roff, rcnt, cnt, T, P<int64_t>(fs[FS_BASE]), floats,
                        xyz, P<int64_t>(e->tri), P<float>(e->faces), s));
  }
  TNP_CHECK(hipStreamSynchronize(s));
  *n_tri = e->n_tri;
  *n_faces = e->n_faces;
  return 0;
}

extern "C" int tnp_engine_faces_export(tnp_engine* e, int64_t* d_tri, float* d_faces, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  if (d_tri && e->n_tri > 0)
    TNP_CHECK(hipMemcpyAsync(d_tri, e->tri.p, e->n_tri * 3 * sizeof(int64_t), hipMemcpyDefault, s));
  if (d_faces && e->n_faces > 0)  // (device or pinned host destinations: one DMA each)
    TNP_CHECK(hipMemcpyAsync(d_faces, e->faces.p, e->n_faces * 9 * sizeof(float), hipMemcpyDefault, s));
  return 0;
}

// ---------------------------------------------------------------------------
// slab boundary + kernel timer controls
// ---------------------------------------------------------------------------
extern "C" int tnp_engine_set_owned(tnp_engine* e, int lo, int hi) {
  e->own = OwnBox{{lo, 1, 1}, {hi, 0, 0}};
  return 0;
}

extern "C" int tnp_engine_set_owned_box(tnp_engine* e, const int32_t* lo3, const int32_t* hi3) {
  for (int d = 0; d < 3; ++d) e->own.lo[d] = lo3[d], e->own.hi[d] = hi3[d];
  return 0;
}

extern "C" int tnp_engine_set_eps(tnp_engine* e, float eps) {
  if (!e->has_net) { tnp_set_error("engine has no net"); return -1; }
  if (!(eps > 0.f)) { tnp_set_error("eps must be positive (got %g)", (double)eps); return -1; }
  if (eps != e->net.eps_s) {
    e->net.eps_s = eps;
    e->masks_valid = false;  // first split planes at the new eps
  }
  return 0;
}

extern "C" int tnp_engine_set_span(tnp_engine* e, const int32_t* lo3, const int32_t* hi3) {
  for (int d = 0; d < 3; ++d)
    if (hi3[d] >= lo3[d] && (lo3[d] < 0 || (e->has_net && hi3[d] >= e->net.n_marks))) {
      tnp_set_error("bad span: axis %d marks [%d, %d]", d, lo3[d], hi3[d]);
      return -1;
    }
  for (int d = 0; d < 3; ++d) e->sp_lo[d] = lo3[d], e->sp_hi[d] = hi3[d];
  return 0;
}

extern "C" int tnp_engine_set_xspan(tnp_engine* e, int x0, int x1) {
  const int32_t lo[3] = {x0, 0, 0}, hi[3] = {x1, -1, -1};
  return tnp_engine_set_span(e, lo, hi);
}

extern "C" int tnp_engine_kernel_timer(tnp_engine* e, int on, void* stream, int32_t* n_kernels) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  *n_kernels = 0;
  if (on) {
    e->kt.clear();
    e->kt_on = true;
    return 0;
  }
  e->kt_on = false;
  TNP_CHECK(hipStreamSynchronize(s));
  e->kt_names.clear();
  e->kt_ms.clear();
  e->kt_bytes.clear();
  e->kt_n.clear();
  for (KRec& r : e->kt) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
    size_t i = 0;
    for (; i < e->kt_names.size(); ++i)
      if (e->kt_names[i] == r.name) break;
    if (i == e->kt_names.size()) {
      e->kt_names.push_back(r.name);
      e->kt_ms.push_back(0);
      e->kt_bytes.push_back(0);
      e->kt_n.push_back(0);
    }
    e->kt_ms[i] += ms;
    e->kt_bytes[i] += r.bytes;
    e->kt_n[i] += 1;
  }
  e->kt.clear();
  *n_kernels = (int32_t)e->kt_names.size();
  return 0;
}

extern "C" int tnp_engine_kernel_stat(tnp_engine* e, int i, char* name, int cap, double* ms,
                                      int64_t* launches, double* bytes) {
  if (i < 0 || i >= (int)e->kt_names.size()) { tnp_set_error("kernel stat %d out of range", i); return -1; }
  snprintf(name, cap, "%s", e->kt_names[i].c_str());
  *ms = e->kt_ms[i];
  *launches = e->kt_n[i];
  *bytes = e->kt_bytes[i];
  return 0;
}

// diagnostics of the ticket-free look-back (common.h lb_prefix_rc): the poll
// count before a waiting wave recomputes an unpublished predecessor (< 0: the
// kernels' defaults; 0 forces the recompute on every unpublished one), and
// the number of recomputes since the last reset
extern "C" int tnp_engine_debug_set_lb_spin(tnp_engine* e, int spin) {
  e->lb_spin = spin;
  return 0;
}
extern "C" int tnp_engine_debug_set_lds_records(tnp_engine* e, int on) {
  e->lds_records = on != 0;
  return 0;
}
extern "C" int tnp_engine_debug_lb_recomputes(tnp_engine* e, int64_t* n, int reset, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  TNP_CHECK(hipSetDevice(e->device));
  *n = 0;
  if (!e->lbrc.p) return 0;
  uint64_t v = 0;
  TNP_CHECK(hipMemcpyAsync(&v, e->lbrc.p, sizeof(v), hipMemcpyDeviceToHost, s));
  TNP_CHECK(hipStreamSynchronize(s));
  if (reset) TNP_CHECK(hipMemsetAsync(e->lbrc.p, 0, sizeof(uint64_t), s));
  *n = (int64_t)v;
  return 0;
}

// debugging aid: the gradient-descent fallback on arbitrary rows
// (tropical_hip_debug.h; checked against the oracle's descent)
extern "C" int tnp_debug_descend(const tnp_net* n, const float* d_ends, float* d_x, const int32_t* d_plane,
                                 int64_t N, int idx, float eps, int iters, float* d_d0, float* d_d1, int per_thread,
                                 void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (check_net(n)) return -1;
  if (N <= 0) return 0;
  if (N > (1 << 20)) { tnp_set_error("debug_descend: at most 2^20 rows"); return -1; }
  NetDev net = to_dev(n);
  // the engine's operands for rows of a made-up complex: vertices 2r, 2r + 1
  // are the ends of split r, which is curve row r and descending row r
  std::vector<int32_t> h(4 * N);
  for (int64_t r = 0; r < N; ++r) {
    h[r] = (int32_t)(2 * r);          // sa
    h[N + r] = (int32_t)(2 * r + 1);  // sb
    h[2 * N + r] = (int32_t)r;        // crow
    h[3 * N + r] = (int32_t)r;        // glist
  }
  int32_t* d = nullptr;
  unsigned long long* conv = nullptr;
  TNP_CHECK(hipMalloc(&d, 4 * N * sizeof(int32_t)));
  TNP_CHECK(hipMalloc(&conv, 8 * sizeof(unsigned long long)));
  int rc = hipMemcpyAsync(d, h.data(), 4 * N * sizeof(int32_t), hipMemcpyHostToDevice, s) == hipSuccess ? 0 : -1;
  if (rc == 0) {
    const char* prev = getenv("TNP_DESCEND_THREAD");
    std::string keep = prev ? prev : "";
    setenv("TNP_DESCEND_THREAD", per_thread ? "1" : "0", 1);
    rc = launch_descend(net, N, d + 3 * N, d + 2 * N, d, d + N, d_ends, d_plane, idx, eps, iters, 0, d_x, d_d0,
                        d_d1, conv, s);
    if (prev) setenv("TNP_DESCEND_THREAD", keep.c_str(), 1);
    else unsetenv("TNP_DESCEND_THREAD");
  }
  if (hipStreamSynchronize(s) != hipSuccess && rc == 0) {
    tnp_set_error("debug_descend: stream synchronise failed");
    rc = -1;
  }
  (void)hipFree(d);
  (void)hipFree(conv);
  return rc;
}

// debugging aid: the padded angular scores of the last tnp_engine_faces call
// (F x width fp32, final-row order); returns F and width
extern "C" int tnp_engine_faces_debug(tnp_engine* e, float* d_scores, int64_t cap, int64_t* F, int64_t* width,
                                      void* stream) {
  hipStream_t s = (hipStream_t)stream;
  *F = e->dbg_F;
  *width = e->dbg_W;
  int64_t n = e->dbg_F * e->dbg_W;
  if (d_scores && n > 0 && n <= cap)
    TNP_CHECK(hipMemcpyAsync(d_scores, e->fscr2[FS_KEY].p, n * sizeof(float), hipMemcpyDeviceToDevice, s));
  return 0;
}
