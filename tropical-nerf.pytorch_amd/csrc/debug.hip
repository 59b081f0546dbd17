// Arithmetic self-check: the bitwise contract assumes gfx950 fp32 ops round
// exactly like IEEE-754 / the host (tests/test_gpu_parity.py::test_fp32_ops).
#include "common.h"
#include "kernels.h"
#include "../../include/tropical_hip_debug.h"

namespace {
__global__ void k_ops(const float* a, const float* b, const float* c, int64_t n, float* o) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o[8 * i + 0] = sqrtf(a[i]);
  o[8 * i + 1] = __fdiv_rn(a[i], b[i]);
  o[8 * i + 2] = __fmaf_rn(a[i], b[i], c[i]);
  o[8 * i + 3] = __fmul_rn(a[i], b[i]);
  o[8 * i + 4] = __fadd_rn(a[i], b[i]);
  o[8 * i + 5] = sqrtf(a[i]);
  o[8 * i + 6] = a[i] / b[i];
  o[8 * i + 7] = tanhf(a[i]);
}
}  // namespace

extern "C" int tnp_debug_ops(const float* a, const float* b, const float* c, int64_t n, float* out,
                             void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_ops, dim3(tnp_grid(n)), dim3(TNP_BLOCK), 0, (hipStream_t)stream, a, b, c, n, out);
  TNP_CHECK(hipGetLastError());
  return 0;
}
