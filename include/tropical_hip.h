/*
 * tropical_hip.h -- C ABI of the MI355X (gfx950) polyhedral-complex
 * extraction library (libtropical_hip.so).
 *
 * Every pointer named d_* is DEVICE memory on the engine's / caller's current
 * HIP device; `stream` is a hipStream_t passed as void* (0 = null stream).
 * No torch types cross this boundary.  All functions return 0 on success and
 * -1 on failure; tnp_last_error() then describes the failure (thread-local).
 *
 * The reference (seonghunn/tropical-nerf.pytorch) is pure Python/PyTorch and
 * has no FFI of its own; each entry point below names the reference
 * function (file:line under tropical/) whose semantics it implements.  The
 * Python host package (tropical-nerf.pytorch_amd/tropical) binds these with
 * ctypes behind the reference's own call surface.
 */
#ifndef TROPICAL_HIP_H
#define TROPICAL_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TNP_MAX_LEVELS 8
#define TNP_ABI_VERSION 1

/* Piecewise-trilinear SDF net: hash-grid encoding (tcnn Grid/Hash, 2
 * features/level, tropical.py:32-40) + ReLU MLP (model.py:38-50).
 * weights: fc.0.weight (H x 2L, row-major), fc.0.bias (H), fc.1.weight,
 * fc.1.bias, ..., fc.last.weight (2 x H), fc.last.bias (2), packed in that
 * order.  table: the flat `enc.module.params` (tcnn layout
 * params[(offset_l + index) * 2 + f]). */
typedef struct tnp_net {
  int32_t n_levels;   /* L  (2..8 are instantiated) */
  int32_t n_features; /* F  (must be 2) */
  int32_t num_layers; /* with num_hidden, one of the instantiated shapes */
  int32_t num_hidden; /* (layers, hidden): (2..4, 8) (2..4, 16) (2, 32) -- K <= 63 planes, every
                         operation; (5, 16) (3, 32) (4, 32) -- K = 65 / 97, two-word sign keys:
                         forward, region, sdf, skeleton and the flat single-device steps and
                         faces (no curve branch, sharding, training or autograd kernels) */
  int32_t n_marks;    /* len(TropicalHashGrid.marks) */
  float eps;          /* Net.eps (model.py:20) */
  float scales[TNP_MAX_LEVELS];    /* fp32 exp2(l*log2 b)*N_min - 1 */
  int32_t res[TNP_MAX_LEVELS];     /* ceil(scale)+1 */
  uint32_t sizes[TNP_MAX_LEVELS];  /* min(next_mult(res^3,8), 2^T) */
  uint32_t offsets[TNP_MAX_LEVELS];
  int32_t dense[TNP_MAX_LEVELS];   /* res^3 <= size */
  const float* d_table;
  const float* d_weights;
  const float* d_marks;
} tnp_net;

/* Per-step counters (the roofline model's inputs). */
typedef struct tnp_step_stats {
  int32_t idx;
  int64_t V_in, E_in, S, H, X, V_out, E_out;
  int64_t A;      /* augmented region rows the reference would build */
  int64_t P;      /* candidate in-region pairs the reference would build */
  int64_t pair_tests; /* member pairs this implementation tested */
  int32_t override_applied;
  uint64_t next_active; /* planes > idx a kept edge would split (pruning steps) */
  int64_t S_dup;        /* splits outside the owned slab (multi-GPU halo) */
  int64_t T;            /* (cell, member) entries of the pair test */
} tnp_step_stats;

const char* tnp_last_error(void);
int tnp_abi_version(void);
/* Hash of the sources the library was built from (csrc/build_id.sh); the
 * Python binding refuses a library whose id differs from its tree's. */
const char* tnp_build_id(void);
int tnp_device_count(int* n);

/* ---- stateless net ops -------------------------------------------------- */

/* Net.forward(x, gather=True)[1] concatenated (model.py:52-76): pre-
 * activations of every hidden neuron + (o1 - o0), written PLANE-MAJOR
 * d_pre[p * ld + i], p < K = (num_layers-1)*num_hidden + 1.  Bitwise equal
 * to the PyTorch-CPU reference (sequential-fma MLP, non-fused encoding). */
int tnp_forward(const tnp_net* net, const float* d_xyz, int64_t n,
                float* d_pre, int64_t ld, float* d_out2, void* stream);
/* d_out2 (nullable): the raw last-layer outputs [n][2] (Net.forward(x)
 * without gather).  d_pre may be null. */

/* TropicalHashGrid.forward(x) (tropical.py:46-47): x in [0,1]^3 (already
 * preprocessed), out [n][2L] fp32 (level-major, tcnn column order). */
int tnp_encode(const tnp_net* net, const float* d_x01, int64_t n, float* d_out,
               void* stream);

/* Net.forward(x, gather=True, group=8) (model.py:67-70): rows come in groups
 * of 8 box corners sharing one activation pattern. */
int tnp_forward_grouped(const tnp_net* net, const float* d_xyz, int64_t n,
                        float* d_pre, int64_t ld, float* d_out2, void* stream);

/* Net.region(v, output, eps) (model.py:90-103 + tropical.py:227-236):
 * d_m[n x (3+K)] int64 {grid mask 0/1, plane sign -1/0/1}, d_off[n x 3]
 * int64 offsets.  d_pre is plane-major with leading dimension ld. */
int tnp_region(const tnp_net* net, const float* d_xyz, const float* d_pre,
               int64_t ld, int64_t n, float eps, int64_t* d_m, int64_t* d_off,
               void* stream);

/* Net.sdf (model.py:84-88) and its input gradient (Net.normal,
 * model.py:105-123).  d_grad may be null. */
int tnp_sdf_grad(const tnp_net* net, const float* d_xyz, int64_t n,
                 float* d_sdf, float* d_grad, void* stream);

/* ---- stateful extraction engine ---------------------------------------- */

typedef struct tnp_engine tnp_engine;

int tnp_engine_create(tnp_engine** out, int device);
void tnp_engine_destroy(tnp_engine* eng);
int tnp_engine_set_net(tnp_engine* eng, const tnp_net* net);
/* Device memory the engine holds: *bytes = the sum of every scratch and
 * complex buffer (they grow geometrically and are reused across steps and
 * passes, so a repeated workload holds this constant after its first pass);
 * *buffers = buffers allocated; *key_bytes = the connect phase's key buffer
 * (the one round 4's growth bug inflated).  buffers / key_bytes may be null.
 * No reference counterpart (PyTorch's caching allocator there). */
int tnp_engine_scratch_bytes(tnp_engine* eng, int64_t* bytes, int64_t* buffers, int64_t* key_bytes);

/* Load a complex: vertices V x 3 fp32, edges E x 2 int64 (device).  d_pre:
 * optional cached outputs_ (V x K fp32, row-major as the reference keeps
 * them); null computes them (subpoly.py:92-93).  keep_all_planes=1 keeps
 * every cached column through compaction (needed to hand outputs_ back);
 * 0 keeps only the columns later steps read. */
int tnp_engine_load(tnp_engine* eng, const float* d_xyz, int64_t V,
                    const int64_t* d_edges, int64_t E, const float* d_pre,
                    int keep_all_planes, void* stream);

/* TropicalHashGrid.skeleton(net, unit) with PRUNING_MODE="distance"
 * (tropical.py:158-225) computed on the device and loaded as the complex;
 * falls back to get_hypercube(3, size) (subpoly.py:51-52, 731-750). */
int tnp_engine_skeleton(tnp_engine* eng, int unit, float size, void* stream,
                        int64_t* V, int64_t* E);
/* The same with the reference's pruning mode chosen (TropicalHashGrid.skeleton,
 * tropical/tropical.py:184-205: PRUNING_MODE is "distance" there; "sign" is
 * its dormant branch -> _skeleton, tropical.py:80-109, keeping an edge iff
 * the endpoints' eps-sign vectors over all planes differ). */
enum { TNP_SKELETON_DISTANCE = 0, TNP_SKELETON_SIGN = 1 };
int tnp_engine_skeleton_mode(tnp_engine* eng, int unit, float size, int mode, void* stream,
                             int64_t* n_vertices, int64_t* n_edges);
/* The distance-mode skeleton split over the ranks of a sharded extraction
 * (no reference counterpart: the reference runs one device).
 * skeleton_gmax: the tiles t of the reference's tile grid (tropical.py:
 * 176-181) with t % world == rank are evaluated whole; h_gmax[t] = the bits
 * of their max |grad sdf| (0 for the other tiles; the ranks' MAX is every
 * tile's), h_load[3][n_marks] (may be null) += per axis and mark plane the
 * points under the tile's edge threshold (the cuts' load balance; SUM over
 * the ranks).  *n_tiles = the tile count (<= cap).
 * skeleton_box: loads the part of the skeleton inside the mark box
 * [lo[d], hi[d]] -- exactly the whole skeleton with the vertices outside
 * the box and the edges leaving it dropped, order kept -- evaluating only
 * tile & box, with every tile's max |grad sdf| from h_gmax[n_tiles].  A box
 * the skeleton misses holds an empty complex (the whole skeleton's
 * emptiness, the hypercube fallback, is the caller's test). */
int tnp_engine_skeleton_gmax(tnp_engine* eng, int unit, int rank, int world, uint32_t* h_gmax,
                             int64_t* h_load, int cap, int* n_tiles, void* stream);
int tnp_engine_skeleton_box(tnp_engine* eng, int unit, const int32_t* lo, const int32_t* hi,
                            const uint32_t* h_gmax, int n_tiles, void* stream, int64_t* n_vertices,
                            int64_t* n_edges);

/* Load the full lattice over the marks restricted to the x-slab of mark
 * indices [x0, x1] (x0=0, x1=n_marks-1: the whole N^3 lattice) in the
 * layout of TropicalHashGrid._skeleton(..., pruning=False)
 * (tropical.py:103-109) with vertex ids (i-x0)*N^2 + j*N + k. */
int tnp_engine_lattice(tnp_engine* eng, int x0, int x1, int keep_all_planes,
                       void* stream, int64_t* V, int64_t* E);
/* The same lattice restricted to the box of mark indices [lo[d], hi[d]] per
 * axis (a block of a sharded lattice): vertex ids
 * (i-lo0)*ny*nz + (j-lo1)*nz + (k-lo2), edges in the same x / y / z order;
 * sets the span (tnp_engine_set_span) to the box. */
int tnp_engine_lattice_box(tnp_engine* eng, const int32_t* lo, const int32_t* hi, int keep_all_planes,
                           void* stream, int64_t* V, int64_t* E);

/* Bit p (p >= from) set iff some edge has endpoints with non-zero opposite
 * eps-signs on plane p, i.e. subpoly_ at idx=p would split (subpoly.py:104-110). */
int tnp_engine_active_planes(tnp_engine* eng, int from, uint64_t* mask,
                             void* stream);

/* subpoly_ phase 1 (subpoly.py:98-117, 180-189): sign test, order-preserving
 * split compaction, new vertices, their forward pass and the LOCAL
 * failover-override predicate.  Writes S (local split count) and fail
 * (0/1; -1 = left on the device -- single-device flat engines skip that
 * round trip; pass it on to tnp_engine_finish unchanged). */
int tnp_engine_split(tnp_engine* eng, int idx, void* stream, int64_t* S,
                     int32_t* fail);

/* subpoly_ phase 2 (subpoly.py:189-279): apply the override if `override`
 * (the GLOBAL predicate; -1: the device-resident local one), connecting edges, pruning (prune=1) and vertex
 * compaction.  Must follow tnp_engine_split on the same idx. */
int tnp_engine_finish(tnp_engine* eng, int idx, int prune, int override,
                      void* stream, tnp_step_stats* stats);

/* The whole hyperplane loop of subpoly.py:58-69 on one device: active
 * planes, then per active plane tnp_engine_split + tnp_engine_finish (prune
 * on every plane but the last), empty steps skipped (subpoly.py:110), the
 * next-active mask folded in after each pruning step -- the loop a host
 * driver would run, without a host round trip per step.  stats[0 ..
 * max_stats) receive the completed steps' stats, *n_steps their count.  Not
 * for a sharded engine (tnp_engine_set_shards > 1: its global decisions
 * fall between split and finish). */
int tnp_engine_run_steps(tnp_engine* eng, void* stream, tnp_step_stats* stats, int max_stats,
                         int* n_steps);

int tnp_engine_sizes(tnp_engine* eng, int64_t* V, int64_t* E);

/* Curve path: after tnp_engine_finish, the strict filter's keep flags
 * (int32 0/1) of the step's n candidate splits in edge order -- the mask
 * debug.strict_check returns (subpoly_debug.py:234-271) that the reference's
 * masked_scatter_ rewrites the caller's edges with (subpoly.py:209-212). */
int tnp_engine_split_keep(tnp_engine* eng, int32_t* d_keep, int64_t n, void* stream);

/* Copy the complex out: d_xyz V x 3, d_edges E x 2 int64, d_pre V x K
 * row-major (requires keep_all_planes, else may be null). */
int tnp_engine_export(tnp_engine* eng, float* d_xyz, int64_t* d_edges,
                      float* d_pre, void* stream);

/* extract_skeleton (subpoly.py:556-581) applied in place; writes the
 * surface sizes (0/0 when fewer than 3 surface vertices). */
int tnp_engine_surface(tnp_engine* eng, void* stream, int64_t* V, int64_t* E);

/* extract_faces (subpoly.py:584-728, geometry.py:483-556) on the current
 * (surface) complex: n_tri = rows of faces_with_indices, n_faces = rows of
 * the float faces (they differ only when a vertex sits exactly at the
 * origin, which the reference's norm>0 mask drops).  Read both with
 * tnp_engine_faces_export (d_tri n_tri x 3 int64, d_faces n_faces x 3 x 3;
 * device memory or pinned host memory -- the copies are asynchronous on
 * `stream`: synchronise it before reading host destinations). */
int tnp_engine_faces(tnp_engine* eng, void* stream, int64_t* n_tri, int64_t* n_faces);
int tnp_engine_faces_export(tnp_engine* eng, int64_t* d_tri, float* d_faces,
                            void* stream);

/* 1: subpoly_(..., force=False) -- the curve-approximation branch
 * (subpoly.py:120-177, 201-207; geometry.py:24-138, 259-299;
 * subpoly_debug.py:121-165, 234-271): new vertices of non-axis-aligned split
 * edges move to the intersection of the two trilinear level sets (largest
 * real root in [0,1] of the xz-plane quartic, gradient-descent fallback) and
 * the strict filter drops splits that miss their planes.  0: flat (default).
 * On x-slab shards the branch takes its whole-complex decisions through
 * the collective of tnp_engine_set_collective. */
int tnp_engine_set_curve(tnp_engine* eng, int on);

/* Collective for the decisions a sharded engine takes inside a step (the
 * curve branch: the curve rows' and descent rows' global counts, which pick
 * MKL's row-count schedules, the descent's stop iteration -- an AND over
 * the shards' per-iteration convergence words, subpoly_debug.py:141 -- and
 * the strict filter's "some kept c row misses its plane" flag,
 * subpoly_debug.py:253-257).  fn reduces n int64 words in place over the
 * shards (op: TNP_COLL_SUM, _MAX, _AND, _OR bitwise) and returns 0; the
 * engine calls it only with tnp_engine_set_shards(n > 1), every shard the
 * same calls in the same order.  fn == NULL: none (the branch then refuses
 * n > 1 shards).  Binds to the host language's all-reduce (the Python
 * driver: torch.distributed, tropical/_engine.py run_steps).  Every call
 * carries one word more than the decision it takes: the shard's failure
 * flag, so a shard that fails between two collectives still joins the next
 * one and every shard returns -1 from that same call (none waits on a
 * collective its peer never reaches). */
enum { TNP_COLL_SUM = 0, TNP_COLL_MAX = 1, TNP_COLL_AND = 2, TNP_COLL_OR = 3 };
typedef int (*tnp_collective_fn)(int64_t* vec, int n, int op, void* ctx);
int tnp_engine_set_collective(tnp_engine* eng, tnp_collective_fn fn, void* ctx);

/* Curve path: subpoly_(..., strict=...) (subpoly.py:198-203).  1 (default):
 * debug.strict_check drops splits that miss their planes
 * (subpoly_debug.py:234-271); 0: every split stays (the reference then only
 * prints a diagnostic). */
int tnp_engine_set_strict(tnp_engine* eng, int on);

/* Multi-GPU x-slabs, each extracted with a halo of cells on either side
 * (tropical/distributed.py; the halo width is the caller's, checked by
 * halo_check): this shard OWNS the mark planes
 * (lo, hi] (lo == 0: [0, hi]) and the cells between them; new vertices
 * outside (halo work, also computed by the neighbour that owns them) are
 * counted in tnp_step_stats.S_dup so the global split count counts each
 * split once.  lo > hi (default) = everything owned.  Flat path only. */
int tnp_engine_set_owned(tnp_engine* eng, int lo, int hi);
/* The same for a block of the mark grid (shards cut along several axes):
 * along axis d the shard owns the planes (lo[d], hi[d]] (plane 0 by the
 * shard with lo[d] == 0) and the cells between them; lo[d] > hi[d]: the
 * axis is not cut.  A vertex is owned iff it is owned along every cut axis. */
int tnp_engine_set_owned_box(tnp_engine* eng, const int32_t* lo, const int32_t* hi);

/* subpoly(net, d, size, eps) / subpoly_(..., eps, ...) with eps != Net.eps
 * (subpoly.py:24, 90): the following steps take the sign test, split point,
 * hit vertices and failover predicate at `eps` (subpoly.py:98-117, 233;
 * subpoly_debug.py:43), extract_skeleton and extract_faces too
 * (subpoly.py:556-606), while the region keys of the pair tests and the
 * pruning stay at Net.eps (Net.region without eps, subpoly.py:118, 184,
 * 256).  In this mode every cached plane is kept (first split planes come
 * from the plane values) and the pruning deletes edges lazily.  tnp_engine_set_net
 * resets it to Net.eps. */
int tnp_engine_set_eps(tnp_engine* eng, float eps);

/* The loaded complex lies between the x mark planes x0 and x1 (an x-slab
 * with its halo): the step's spatial buckets then cover only those cells.
 * tnp_engine_lattice sets it, tnp_engine_load / _skeleton reset it to the
 * whole grid (x1 < x0).  A vertex outside fails the step with an error.
 * Performance only: the results do not depend on it.  No reference
 * counterpart (multi-GPU sharding). */
int tnp_engine_set_xspan(tnp_engine* eng, int x0, int x1);
/* Per axis: the complex lies between the mark planes lo[d] and hi[d]
 * (hi[d] < lo[d]: anywhere along d) -- a block with its halo; x-slabs are
 * tnp_engine_set_xspan. */
int tnp_engine_set_span(tnp_engine* eng, const int32_t* lo, const int32_t* hi);

/* world > 1: this engine holds one x-slab of a complex sharded over `world`
 * devices.  A step the other shards split may leave this one without any
 * connecting pair; the reference's empty-torch.cat error (subpoly.py:505-513)
 * then only applies to the whole complex, not to a shard. */
int tnp_engine_set_shards(tnp_engine* eng, int world);

/* HIP-event timing of every engine kernel launch (on=1 clears and starts;
 * on=0 stops, synchronizes and aggregates per kernel name); read the
 * aggregates with tnp_engine_kernel_stat (ms, launches, modelled
 * algorithmic bytes). */
int tnp_engine_kernel_timer(tnp_engine* eng, int on, void* stream, int32_t* n_kernels);
int tnp_engine_kernel_stat(tnp_engine* eng, int i, char* name, int cap, double* ms,
                           int64_t* launches, double* bytes);

/* ---- single-node rank agreements (bench.py / tropical/distributed.py) ----
 * The per-step global decisions of the sharded loop (subpoly.py:110 "does
 * anything split", subpoly_debug.py:43-49 the failover override, and the OR
 * of the ranks' next-active plane masks) between the processes of ONE node
 * through a POSIX shared-memory segment: every rank writes <= 16 int64 words,
 * arrives on an atomic counter and spins until all have (no library
 * collective, no device copies).  Rank 0 creates the segment (create=1)
 * before the others open it; it can be unlinked once all have.  allreduce
 * op: TNP_SHM_MAX, TNP_SHM_OR (bitwise, 64-bit masks), TNP_SHM_SUM or
 * TNP_SHM_AND (bitwise). */
typedef struct tnp_shm tnp_shm;
enum { TNP_SHM_MAX = 0, TNP_SHM_OR = 1, TNP_SHM_SUM = 2, TNP_SHM_AND = 3 };
int tnp_shm_open(const char* name, int rank, int world, int create, tnp_shm** out);
int tnp_shm_unlink(const char* name);
void tnp_shm_close(tnp_shm* shm);
int tnp_shm_allreduce(tnp_shm* shm, const int64_t* in, int n, int op, int64_t* out);

/* ---- SDF training (train.py:169-224, dataset.py:80-96; csrc/train.hip) --
 * Gradient of one batch's loss (train.py:181-201) for the n points d_x
 * (n x 3 in [-1, 1]^3) with target distances d_gt (n):
 *   L = mean |clamp(sdf(x)) - clamp(gt)| + eik_w (||J||_F - 1)^2 / eik_batch,
 * clamp to [-clamp_t, clamp_t], sdf = tanh(o1 - o0) (model.py:84-87),
 * J = d sdf / d x (n x 3) -- the L1 and eikonal terms (eik_batch: the
 * reference's BATCH_SIZE constant, train.py:197, which equals n except for a
 * partial last batch; <= 0 takes n); the weight-norm term
 * (train.py:200-201) involves only the fc weights and is the caller's.  The
 * eikonal term's parameter gradient (the reference's double backward) is
 * written out in closed form.  ACCUMULATES into d_grad_table (the table's
 * own layout, params[(offset_l + idx) * 2 + f]) and d_grad_weights (the
 * packed weight layout of tnp_net); d_stats (2 doubles, device, zeroed by
 * the call) receives sum |clamp(sdf) - clamp(gt)| and sum ||J_i||^2.  Float
 * atomics: the summation order is not fixed.  Every instantiated net shape. */
int tnp_sdf_train_grad(const tnp_net* net, const float* d_x, const float* d_gt, int64_t n, float clamp_t,
                       float eik_w, int64_t eik_batch, float* d_grad_table, float* d_grad_weights,
                       double* d_stats, void* stream);

/* Autograd through Net.sdf (model.py:84-88): the vector-Jacobian product
 * sum_i d_gout[i] * d sdf(x_i) / d theta, ACCUMULATED into d_grad_table (the
 * table's own layout) and d_grad_weights (the packed weight layout) -- the
 * backward of a caller's net.sdf(x) w.r.t. the parameters (the input
 * gradient is tnp_sdf_grad's).  Float atomics; every instantiated net shape. */
int tnp_sdf_vjp(const tnp_net* net, const float* d_x, const float* d_gout, int64_t n, float* d_grad_table,
                float* d_grad_weights, void* stream);

/* Autograd through Net.normal(create_graph=True) (model.py:105-123: J =
 * d sdf / d x with a graph): the VJP sum_i d_gJ[i] . d J_i / d theta,
 * ACCUMULATED into d_grad_table / d_grad_weights, and (d_grad_x != null)
 * d_gJ[i] . d J_i / d x_i -- the Hessian of sdf along d_gJ[i] -- ACCUMULATED
 * into d_grad_x (n x 3).  Replaces the reference's double backward through
 * tcnn (train.py:196).  Float atomics. */
int tnp_normal_vjp(const tnp_net* net, const float* d_x, const float* d_gJ, int64_t n, float* d_grad_table,
                   float* d_grad_weights, float* d_grad_x, void* stream);

/* Autograd through Net.forward(x, gather=True) (model.py:52-76): upstream
 * gradients of the gathered planes (d_gpre, plane-major [K][ld] as
 * tnp_forward writes them: every hidden pre-activation, then o1 - o0) and
 * of the output (d_gout, n x 2); either may be null.  ACCUMULATES into
 * d_grad_table, d_grad_weights and (when given) d_grad_x (n x 3). */
int tnp_forward_vjp(const tnp_net* net, const float* d_x, int64_t n, const float* d_gpre, int64_t ld,
                    const float* d_gout, float* d_grad_table, float* d_grad_weights, float* d_grad_x, void* stream);

/* Signed distance of n points d_p (n x 3) to a closed triangle mesh (d_V
 * nV x 3 fp32, d_F nF x 3 int32, indices in [0, nV)): replaces
 * cubvh.cuBVH(V, F).signed_distance (dataset.py:77, 92).  Exact distance to
 * the closest triangle; the sign from the generalized winding number,
 * positive inside (dataset.py:96).  d_work: 2 n floats of scratch. */
int tnp_mesh_signed_distance(const float* d_V, int64_t nV, const int32_t* d_F, int64_t nF, const float* d_p,
                             int64_t n, float* d_work, float* d_dist, void* stream);

/* ---- `-e` evaluation stack (train.py:275-354; csrc/evaluate.hip) ------- */

/* Marching cubes over vol[n0][n1][n2] (x slowest), inside = value < iso,
 * case table int8 [256][16] (tropical/utils/mc_table.py).  Replaces
 * mcubes.marching_cubes (train.py:284).  Phase 1: d_eoff [3*n0*n1*n2 + 1]
 * int64 -> vertex id of every crossed lattice edge (point-major, axis
 * minor), d_coff [(n0-1)(n1-1)(n2-1) + 1] int64 -> first triangle of every
 * cube; returns the vertex and triangle counts.  Phase 2: vertices fp64
 * [n_verts][3] in index space (interpolated in double, as PyMCubes),
 * triangles int64 [n_tris][3]. */
int tnp_mc_count(const float* d_vol, int n0, int n1, int n2, float iso, const int8_t* d_table,
                 int64_t* d_eoff, int64_t* d_coff, int64_t* n_verts, int64_t* n_tris,
                 void* stream);
int tnp_mc_emit(const float* d_vol, int n0, int n1, int n2, float iso, const int8_t* d_table,
                const int64_t* d_eoff, const int64_t* d_coff, double* d_verts, int64_t* d_tris,
                void* stream);

/* Nearest-hit ray casting against a triangle mesh (replaces
 * cubvh.cuBVH(vertices, faces).ray_trace, chamfer_distance.py:184-212):
 * uniform-grid acceleration over the caller's bounding box; the mesh
 * buffers must outlive the caster.  cast: t (fp32, +inf on a miss) and face
 * id (-1 on a miss) per ray; rays are origins/directions fp32 [n][3]. */
typedef struct tnp_raycaster tnp_raycaster;
int tnp_raycaster_create(tnp_raycaster** out, int device);
void tnp_raycaster_destroy(tnp_raycaster* rc);
int tnp_raycaster_build(tnp_raycaster* rc, const float* d_V, int64_t nV, const int32_t* d_F,
                        int64_t nF, const float* bbox_lo, const float* bbox_hi, void* stream);
int tnp_raycaster_cast(tnp_raycaster* rc, const float* d_o, const float* d_d, int64_t nR,
                       float* d_t, int32_t* d_face, void* stream);

/* Exact nearest-neighbour L2 distance of every point of a [na][3] to the set
 * b [nb][3] (replaces sklearn NearestNeighbors in chamfer_distance.py:39-48). */
int tnp_nn_min_dist(const float* d_a, int64_t na, const float* d_b, int64_t nb, float* d_out,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TROPICAL_HIP_H */
