// Internal: face-extraction launchers (faces.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// K: the net's planes (the regions' plane columns are planes < K - 1); K > 63:
// two-word keys, a table of 4 cap words (else 2 cap)
int launch_face_count(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                      int K, int64_t* ctr2, hipStream_t s);
int launch_face_insert(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                       int K, uint64_t* table, uint64_t tmask, int32_t* cnt, hipStream_t s);
int launch_keep_counts(const int32_t* cnt, int64_t n, int32_t* kc, int32_t* kf, hipStream_t s);
int launch_face_scatter(int64_t V, const uint64_t* grid, const uint64_t* pos, const uint64_t* zero,
                        int K, const uint64_t* table, uint64_t tmask, const int32_t* cnt,
                        const int64_t* memoff, int32_t* cur, uint64_t* mem, hipStream_t s);
int launch_region_finalize(int64_t n, const int32_t* kf, const int64_t* rid, const int32_t* cnt,
                           const int64_t* memoff, uint64_t* mem, int64_t* roff, int32_t* rcnt,
                           hipStream_t s);
int launch_row_buckets(int64_t R, int64_t V, const uint64_t* mem, const int64_t* roff, const int32_t* rcnt,
                       int32_t* bcnt, int64_t* boff, int32_t* bcur, int32_t* rows, int32_t* keep, int phase,
                       hipStream_t s);
int launch_compact_rows(int64_t n, const int32_t* keep, const int64_t* koff, const int32_t* rows,
                        int32_t* out, hipStream_t s);
int launch_row_mean(int64_t F, const int32_t* frow, const uint64_t* mem, const int64_t* roff,
                    const int32_t* rcnt, int M, const float* xyz, float* mean, hipStream_t s);
size_t row_order_scratch(int64_t F, int M);
int launch_row_order(int64_t F, const int32_t* frow, const uint64_t* mem, const int64_t* roff,
                     const int32_t* rcnt, int M, const float* xyz, const float* nrm, int quirk3, void* scratch,
                     int32_t* ordv, int32_t* cnt_all, int32_t* cnt_nz, hipStream_t s);
int64_t fan_blocks(int64_t F);
int launch_fan_hist(int64_t F, const int32_t* cnt, int T, int32_t* hist, hipStream_t s);
int launch_fan_emit(int64_t F, const int32_t* frow, const int32_t* ordv, const int64_t* roff,
                    const int32_t* rcnt, const int32_t* cnt, int T, const int64_t* base, int floats,
                    const float* xyz, int64_t* tri, float* fc, hipStream_t s);
// max of a (and of b, if given) over [0, n) -> *out (*out_b), zeroed by the caller
int launch_max_i32(const int32_t* a, int64_t n, int64_t* out, hipStream_t s, const int32_t* b = nullptr,
                   int64_t* out_b = nullptr);
