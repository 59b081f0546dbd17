// Calibration of rocprofv3's FETCH_SIZE for gather widths:
// MI355X_MICROARCH.md calibrates the x2 correction only for 16-B-per-lane
// streaming reads.  Each kernel below reads a KNOWN set of cache lines from
// a 2 GiB array (far past the 256 MiB Infinity Cache, so every line is a
// fabric fetch) in one access pattern of the extraction's kernels:
//   k_stream16   16 B per lane, coalesced (the guide's calibrated case)
//   k_gather4    4 B per lane, one random 128-B line per lane   (scol[a])
//   k_gather8    8 B per lane, one random line per lane          (zero[a])
//   k_gather12   12 B per lane at 12-B records (3 floats), random (xyz[a])
//   k_gather16   16 B per lane at 16-B records, random            (pz[a])
// Lines are drawn without repeats within a launch (a bijection of the line
// index), so the compulsory traffic is exactly lines x 128 B (+ the 12-B
// records that straddle two lines).
//   hipcc --offload-arch=gfx950 -O3 -o gpurun_out/gather_calib tools/gather_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d ... -- gpurun_out/gather_calib
// (tools/pmc_table.py GATHER_FACTOR records the result)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

constexpr size_t ARRAY_BYTES = size_t(2) << 30;  // 2 GiB
constexpr uint64_t LINES = ARRAY_BYTES / 128;     // 16 M lines
constexpr int64_t N = 4 << 20;                    // 4 M lanes (lines) per gather launch

// a bijection of [0, LINES) (LINES a power of two): odd multiplier, then a
// xor of high bits into low bits (invertible)
__device__ __forceinline__ uint64_t line_of(uint64_t i) {
  uint64_t x = (i * 0x9E3779B1ull) & (LINES - 1);
  return x ^ (x >> 13);
}

__global__ void k_stream16(const float4* __restrict__ a, int64_t n, float* __restrict__ out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}
__global__ void k_gather4(const float* __restrict__ a, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const float v = a[line_of(i) * 32];
  if (v == 1234.5f) out[0] = v;
}
__global__ void k_gather8(const uint64_t* __restrict__ a, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint64_t v = a[line_of(i) * 16];
  if (v == 12345) out[0] = (float)v;
}
// 12-B records as forward_new reads xyz[3 a .. 3 a + 2]: the first record
// starting in the chosen line, shifted by 0..7 records (a record straddles
// into the next line when it starts in the line's last 8 bytes)
__global__ void k_gather12(const float* __restrict__ a, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint64_t rec = (line_of(i) * 128 + 11) / 12 + (i & 7);
  const float x = a[3 * rec], y = a[3 * rec + 1], z = a[3 * rec + 2];
  if (x + y + z == 1234.5f) out[0] = x;
}
__global__ void k_gather16(const ulonglong2* __restrict__ a, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const ulonglong2 v = a[line_of(i) * 8];
  if (v.x == 12345) out[0] = (float)v.y;
}

int main() {
  void* buf = nullptr;
  float* out = nullptr;
  CK(hipMalloc(&buf, ARRAY_BYTES + 256));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, ARRAY_BYTES + 256));
  const int64_t n16 = (int64_t)(ARRAY_BYTES / 16 / 4);  // stream 512 MiB (known bytes)
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 g((unsigned)((N + 255) / 256)), blk(256);
  for (int rep = 0; rep < 2; ++rep) {
    float ms[5];
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_stream16, dim3(4096), blk, 0, 0, (const float4*)buf, n16, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms[0], a, b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_gather4, g, blk, 0, 0, (const float*)buf, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms[1], a, b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_gather8, g, blk, 0, 0, (const uint64_t*)buf, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms[2], a, b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_gather12, g, blk, 0, 0, (const float*)buf, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms[3], a, b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_gather16, g, blk, 0, 0, (const ulonglong2*)buf, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms[4], a, b));
    printf("rep %d: stream16 %lld B in %.3f ms; gathers of %lld lines (128 B each): 4B %.3f ms, 8B %.3f, 12B %.3f, "
           "16B %.3f\n",
           rep, (long long)(n16 * 16), ms[0], (long long)N, ms[1], ms[2], ms[3], ms[4]);
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
