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

#ifdef __cplusplus
}
#endif

#endif /* TROPICAL_HIP_DEBUG_H */
