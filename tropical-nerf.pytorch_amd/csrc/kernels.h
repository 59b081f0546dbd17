// Internal launcher interface between engine.cpp and the .hip kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tropical_hip.h"
#include "common.h"

// Net descriptor passed BY VALUE as a kernel argument (lives in SGPRs /
// the kernarg segment; every field is wave-uniform).
constexpr int TNP_MAX_MARKS = 1024;  // marks per axis (k_forward_new stages them in LDS)

struct NetDev {
  float scales[TNP_MAX_LEVELS];
  int32_t res[TNP_MAX_LEVELS];
  uint32_t sizes[TNP_MAX_LEVELS];
  uint32_t offsets[TNP_MAX_LEVELS];
  int32_t dense[TNP_MAX_LEVELS];
  const float* table;
  const float* weights;
  const float* marks;
  int32_t n_levels, num_layers, num_hidden, n_marks;
  float eps;
  // the eps argument of subpoly / subpoly_ (subpoly.py:24, 90): the steps'
  // sign test, split point and failover predicate use it, Net.region (the
  // keys) uses eps; equal unless tnp_engine_set_eps says otherwise
  float eps_s;
  // 1: every level has the same scale/res/size/dense, so one set of corner
  // weights and hash indices serves all levels, and `table` is the engine's
  // level-interleaved copy: entry idx of level l at float2 (idx * L + l) --
  // one 16-B gather per corner instead of L 8-B gathers in L cache lines
  int32_t tied;
  // > 0: the row count whose MKL schedule the forward / descent launches
  // follow (a sharded batch: the shards' total), else each launch's own
  int64_t sched_rows;
};

static inline int net_K(const NetDev& n) { return (n.num_layers - 1) * n.num_hidden + 1; }
int net_supported(const NetDev& n);       // 1 if forward / keys / the flat steps are instantiated
int net_supported_full(const NetDev& n);  // ... and the curve descent, training and autograd kernels
static inline int net_kw(const NetDev& n) { return net_K(n) <= 63 ? 1 : 2; }  // sign-key words

// ---- net_lv.hip: the kernels of one level count (one translation unit per
// level count 2..8, -DTNP_LV; explicit specializations, dispatched by the
// launch_* functions of net.hip / skeleton.hip) ----
template <int LV>
int lv_forward(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld, int group, hipStream_t s,
               float* out2, uint64_t* pos, uint64_t* zero, uint64_t* grid, uint64_t* pz);
template <int LV>
int lv_forward_new(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld, int64_t V,
                   int keep_from, const int32_t* sa, const int32_t* sb, int idx, const OwnBox& own,
                   uint64_t* pos, uint64_t* zero, uint64_t* grid, uint64_t* shared, int64_t* ctr, uint64_t* pz,
                   const float* col, hipStream_t s);
template <int LV>
int lv_sdf_grad(const NetDev& net, const float* xyz, int64_t n, float* sdf, float* grad, hipStream_t s);
template <int LV>
int lv_skel_eval(const NetDev& net, int i0, int j0, int k0, int n0, int n1, int n2, float* dist,
                 unsigned int* gmax_bits, hipStream_t s);
template <int LV>
int lv_encode(const NetDev& net, const float* x01, int64_t n, float* out, hipStream_t s);
// parameter gradients (train_net.h k_train_grads): training (gout, gJ null;
// stats zeroed by the caller), the sdf VJP (gout), the normal VJP (gJ, g_x)
template <int LV>
int lv_train(const NetDev& net, const float* xyz, const float* gt, int64_t n, float T, float eik_w, int64_t eik_batch,
             double* stats, float* g_table, float* g_w, const float* gout, const float* gJ, float* g_x, hipStream_t s);
// VJP of the forward's gathered planes / output (train_net.h k_forward_vjp)
template <int LV>
int lv_forward_vjp(const NetDev& net, const float* xyz, int64_t n, const float* gpl, int64_t ld, const float* gout2,
                   float* g_table, float* g_w, float* g_x, hipStream_t s);
// the curve branch's gradient descent (descend.h) for every shape of this
// level count; per_thread: one thread per row (else one wave per row)
template <int LV>
int lv_descend(const NetDev& net, int64_t G, const int32_t* glist, const int32_t* crow, const int32_t* sa,
               const int32_t* sb, const float* xyz, const int32_t* plane, int idx, float eps, int iters, int record,
               float* ints, float* d0s, float* d1s, unsigned long long* conv, bool per_thread, hipStream_t s);
#define TNP_LV_DECLARE(L)                                                                                   \
  template <> int lv_forward<L>(const NetDev&, const float*, int64_t, float*, int64_t, int, hipStream_t, float*, \
                                uint64_t*, uint64_t*, uint64_t*, uint64_t*);                                  \
  template <> int lv_forward_new<L>(const NetDev&, const float*, int64_t, float*, int64_t, int64_t, int,        \
                                    const int32_t*, const int32_t*, int, const OwnBox&, uint64_t*, uint64_t*, \
                                    uint64_t*, uint64_t*, int64_t*, uint64_t*, const float*, hipStream_t);    \
  template <> int lv_sdf_grad<L>(const NetDev&, const float*, int64_t, float*, float*, hipStream_t);           \
  template <> int lv_skel_eval<L>(const NetDev&, int, int, int, int, int, int, float*, unsigned int*,         \
                                  hipStream_t);                                                               \
  template <> int lv_encode<L>(const NetDev&, const float*, int64_t, float*, hipStream_t);                    \
  template <> int lv_train<L>(const NetDev&, const float*, const float*, int64_t, float, float, int64_t, double*, \
                              float*, float*, const float*, const float*, float*, hipStream_t);                  \
  template <> int lv_forward_vjp<L>(const NetDev&, const float*, int64_t, const float*, int64_t, const float*,   \
                                    float*, float*, float*, hipStream_t);                                         \
  template <> int lv_descend<L>(const NetDev&, int64_t, const int32_t*, const int32_t*, const int32_t*,        \
                                const int32_t*, const float*, const int32_t*, int, float, int, int, float*,    \
                                float*, float*, unsigned long long*, bool, hipStream_t);
TNP_LV_DECLARE(2)
TNP_LV_DECLARE(3)
TNP_LV_DECLARE(4)
TNP_LV_DECLARE(5)
TNP_LV_DECLARE(6)
TNP_LV_DECLARE(7)
TNP_LV_DECLARE(8)
#undef TNP_LV_DECLARE
// the level-count dispatch of the lv_* functions: BODY sees constexpr L_
#define TNP_LV_SWITCH(LV, BODY)                                                     \
  switch (LV) {                                                                     \
    case 2: { constexpr int L_ = 2; BODY; break; }                                  \
    case 3: { constexpr int L_ = 3; BODY; break; }                                  \
    case 4: { constexpr int L_ = 4; BODY; break; }                                  \
    case 5: { constexpr int L_ = 5; BODY; break; }                                  \
    case 6: { constexpr int L_ = 6; BODY; break; }                                  \
    case 7: { constexpr int L_ = 7; BODY; break; }                                  \
    case 8: { constexpr int L_ = 8; BODY; break; }                                  \
    default: tnp_set_error("n_levels=%d not instantiated (2..8)", (int)(LV)); return -1; \
  }

// ---- net.hip ----
// pre plane-major [K][ld]; rows [0, n)
// pos/zero/grid/pz (group 1 only): the packed keys of k_keys written by the
// same pass (pre must then hold every plane: keys cover planes [0, K))
int launch_forward(const NetDev& net, const float* xyz, int64_t n, float* pre,
                   int64_t ld, int group, hipStream_t s, float* out2 = nullptr,
                   uint64_t* pos = nullptr, uint64_t* zero = nullptr, uint64_t* grid = nullptr,
                   uint64_t* pz = nullptr);
// new vertices of a flat step, forward with the fused epilogue (net.hip
// k_forward_new); col != null: the split points are computed here too from
// the plane column (xyz = slot V: written); cache planes >= keep_from at
// slots V.., keys, shared
// planes, failover predicate -> ctr[CTR_FAIL], new vertices outside the
// owned box (common.h OwnBox) -> ctr[CTR_DUP]; then the override itself.
// n < 0: the split count is read from ctr[CTR_S] on the device (-n bounds
// it; buffers sized for the bound): launched behind the split, ahead of the
// host's readback of S
int launch_forward_new(const NetDev& net, const float* xyz, int64_t n, float* pre, int64_t ld,
                       int64_t V, int keep_from, const int32_t* sa, const int32_t* sb, int idx,
                       const OwnBox& own, uint64_t* pos, uint64_t* zero, uint64_t* grid,
                       uint64_t* shared, int64_t* ctr, uint64_t* pz, const float* col, hipStream_t s);
int launch_override_new(int64_t n, int override_, const uint64_t* shared, float* pre, int64_t ld,
                        int keep_from, int64_t V, uint64_t* pos, uint64_t* zero,
                        const int64_t* ctr, uint64_t* pz, int kw, hipStream_t s);
int launch_encode(const NetDev& net, const float* x01, int64_t n, float* out, hipStream_t s);
// pre plane-major; writes int64 m[n][3+K] and off[n][3] (Net.region)
int launch_region(const NetDev& net, const float* xyz, const float* pre, int64_t ld,
                  int64_t n, float eps, int64_t* m, int64_t* off, hipStream_t s);
// ---- train.hip ----
// SDF training gradients of one batch (train.py:181-201); stats: 2 doubles
int launch_train_grad(const NetDev& net, const float* xyz, const float* gt, int64_t n, float clamp_t, float eik_w,
                      int64_t eik_batch, float* g_table, float* g_w, double* stats, hipStream_t s);
// sum_i gout_i d sdf_i / d theta accumulated into g_table / g_w (autograd
// through Net.sdf)
int launch_sdf_vjp(const NetDev& net, const float* xyz, const float* gout, int64_t n, float* g_table, float* g_w,
                   hipStream_t s);
// sum_i gJ_i . d J_i / d theta (and d / d x_i into g_x when given), J = d sdf / d x
// (autograd through Net.normal(create_graph=True))
int launch_normal_vjp(const NetDev& net, const float* xyz, const float* gJ, int64_t n, float* g_table, float* g_w,
                      float* g_x, hipStream_t s);
// VJP of Net.forward(x, gather=True): upstream of the gathered planes (gpl
// plane-major [K][ld]) and of the output (gout2 [n][2]); either may be null
int launch_forward_vjp(const NetDev& net, const float* xyz, int64_t n, const float* gpl, int64_t ld,
                       const float* gout2, float* g_table, float* g_w, float* g_x, hipStream_t s);
// mesh signed distance (dataset.py:92); work: 2 n floats
int launch_mesh_sd(const float* V, int64_t nV, const int32_t* F, int64_t nF, const float* P, int64_t n, float* work,
                   float* out, hipStream_t s);
int launch_sdf_grad(const NetDev& net, const float* xyz, int64_t n, float* sdf,
                    float* grad, hipStream_t s);
// packed keys from pre (planes [0,K)) + grid word from coordinates
int launch_keys(const NetDev& net, const float* xyz, const float* pre, int64_t ld,
                int64_t n, int K, uint64_t* pos, uint64_t* zero, uint64_t* grid,
                hipStream_t s, uint64_t* pz = nullptr);  // pz: interleaved (pos, zero) copy

// ---- scan.hip ----
// exclusive scan of int32 counts into int64 offsets; *total (device) = sum.
// lb: look-back state prepared for scan_tiles(n) tiles (engine.cpp lb_begin)
int scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, int64_t* total, const TnpLB& lb,
                    hipStream_t s);
int64_t scan_tiles(int64_t n);
// Batched fill: up to FILL_MAX byte ranges set to a byte value in ONE
// dispatch (hipMemsetAsync takes one fill dispatch per range, two when the
// size is not 16-B aligned -- at bunny scale every dispatch costs ~4 us)
struct FillOp {
  void* p;
  uint64_t n;     // bytes
  uint32_t byte;  // value
};
constexpr int FILL_MAX = 4;
int launch_fill(const FillOp* ops, int n, hipStream_t s);
