/*
 * tropical_hip_debug.h -- diagnostic entry points of libtropical_hip.so.
 *
 * Not part of the product surface (include/tropical_hip.h): self-checks and
 * intermediate dumps used by tests/ and tools/ only.  Same conventions as
 * tropical_hip.h (d_* device pointers, 0 / -1 returns, tnp_last_error()).
 */
#ifndef TROPICAL_HIP_DEBUG_H
#define TROPICAL_HIP_DEBUG_H

#include "tropical_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Self-check of the fp32 primitives the bitwise contract relies on:
 * out[8i..8i+7] = sqrt_rn(a), a/b (rn), fma(a,b,c), a*b, a+b, sqrtf(a),
 * a/b (default), tanhf(a). */
int tnp_debug_ops(const float* d_a, const float* d_b, const float* d_c, int64_t n,
                  float* d_out, void* stream);

/* Debug: padded angular scores (F x width fp32) of the last faces call. */
int tnp_engine_faces_debug(tnp_engine* eng, float* d_scores, int64_t cap, int64_t* F,
                           int64_t* width, void* stream);

/* Debug: the ticket-free look-back of the split, prune and count scans
 * (csrc/common.h lb_prefix_rc).  set_lb_spin: polls of an unpublished
 * predecessor tile before the waiting wave recomputes its aggregate (< 0: the
 * kernels' defaults, 0: recompute every unpublished predecessor -- the path
 * in-order dispatch makes rare).  lb_recomputes: recomputes since the last
 * reset (reset=1 zeroes the counter after reading it). */
int tnp_engine_debug_set_lb_spin(tnp_engine* eng, int spin);
int tnp_engine_debug_lb_recomputes(tnp_engine* eng, int64_t* n, int reset, void* stream);

/* Debug: the grouping kernel's LDS-record path (csrc/bucket.hip
 * k_bucket_group; on by default, TNP_LDS_RECORDS=0 at engine creation turns
 * it off): on = 0 sends every bucket's records through memory, as before. */
int tnp_engine_debug_set_lds_records(tnp_engine* eng, int on);

/* Debug: the vertex set's row capacity (the cache, coordinates and keys are
 * sized by it) and how often the early k_forward_new's row bound (the
 * largest split count seen, csrc/engine.cpp early_bound) was below a step's
 * split count, so that the forward ran again once the count was known. */
int tnp_engine_debug_vertex_capacity(tnp_engine* eng, int64_t* rows, int64_t* early_redo);

/* Debug: the engine's capacity arithmetic, host only (csrc/engine.cpp
 * buf_grow_bytes, connect_key_cap).  grown_bytes: the size a buffer of
 * have_bytes grows to for a request of request_bytes; key_cap: the connect
 * phase's key capacity (keys, a multiple of xs_n) for a step of `members`
 * bucket members when the key buffer holds have_bytes.  A steady workload
 * must never ask for more than the buffer holds: key_cap * 8 <= have_bytes
 * whenever have_bytes already covers the floor. */
int tnp_debug_buf_growth(int64_t have_bytes, int64_t request_bytes, int64_t members, int xs_n,
                         int64_t* grown_bytes, int64_t* key_cap);

/* Debug: the curve branch's gradient-descent fallback (descend.h, the
 * engine's launch) on n arbitrary rows: row r descends along the edge
 * d_ends[r] (e0 xyz, e1 xyz) from the box parameters d_x[r] (in/out) on
 * plane pair (d_plane[r], idx) for exactly `iters` iterations (<= 512);
 * d_d0 / d_d1: the distances evaluated before the last update.  The batch
 * is the n rows (MKL row-count schedules).  per_thread: the one-thread-per-
 * row kernel.  Checked against the oracle's descend (oracle/curve.py). */
int tnp_debug_descend(const tnp_net* net, const float* d_ends, float* d_x, const int32_t* d_plane, int64_t n,
                      int idx, float eps, int iters, float* d_d0, float* d_d1, int per_thread, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TROPICAL_HIP_DEBUG_H */
