// Host round-trip costs on one MI355X: what a per-step counter readback
// costs the engine (csrc/engine.cpp read_ctr) and the alternatives.
//   hipcc -O2 --offload-arch=gfx950 tools/readback_bench.hip -o tools/_readback_bench
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                          \
    }                                                                    \
  } while (0)

__global__ void k_tiny(int64_t* ctr, int64_t v) {
  if (threadIdx.x < 28) ctr[threadIdx.x] = v + threadIdx.x;
}

// counters -> host-mapped block, then the sequence word (vector stores only)
__global__ void k_publish(const int64_t* ctr, volatile int64_t* host, int64_t seq) {
  const int t = threadIdx.x;
  if (t < 28) host[t] = ctr[t];
  __threadfence_system();
  __syncthreads();
  if (t == 0) host[31] = seq;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int64_t* d;
  CK(hipMalloc(&d, 256));
  int64_t* h;
  CK(hipHostMalloc(&h, 256, hipHostMallocDefault));
  int64_t* hm;
  CK(hipHostMalloc(&hm, 256, hipHostMallocMapped | hipHostMallocCoherent));
  int64_t* hm_dev;
  CK(hipHostGetDevicePointer((void**)&hm_dev, hm, 0));
  const int N = 2000;
  for (int warm = 0; warm < 2; ++warm) {
    // (0) launch + stream sync, nothing copied
    double t0 = now_us();
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d, (int64_t)i);
      CK(hipStreamSynchronize(s));
    }
    double t1 = now_us();
    // (1) launch + D2H copy + stream sync (engine read_ctr)
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d, (int64_t)i);
      CK(hipMemcpyAsync(h, d, 224, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      if (h[0] != i) { printf("bad copy\n"); return 1; }
    }
    double t2 = now_us();
    // (2) launch + publish kernel + host spin on the sequence word
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d, (int64_t)i);
      hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, d, hm_dev, (int64_t)(i + 1 + warm * N));
      const int64_t want = i + 1 + warm * N;
      double ts = now_us();
      while (reinterpret_cast<volatile int64_t*>(hm)[31] != want) {
        if (now_us() - ts > 5e6) { printf("spin timeout\n"); return 1; }
      }
      std::atomic_thread_fence(std::memory_order_acquire);
      if (hm[0] != i) { printf("bad publish\n"); return 1; }
    }
    CK(hipStreamSynchronize(s));
    double t3 = now_us();
    // (3) back-to-back launches, one sync at the end
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d, (int64_t)i);
    CK(hipStreamSynchronize(s));
    double t4 = now_us();
    // (4) launch + memset + launch (a memset between kernels)
    for (int i = 0; i < N; ++i) {
      CK(hipMemsetAsync(d, 0, 224, s));
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d, (int64_t)i);
    }
    CK(hipStreamSynchronize(s));
    double t5 = now_us();
    // (5) launch + event record + event sync
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d, (int64_t)i);
      CK(hipMemcpyAsync(h, d, 224, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(ev, s));
      CK(hipEventSynchronize(ev));
    }
    double t6 = now_us();
    if (warm)
      printf("us per iteration: launch+sync %.2f | +D2H copy %.2f | publish+spin %.2f | "
             "back-to-back launch %.2f | memset+launch %.2f | copy+event sync %.2f\n",
             (t1 - t0) / N, (t2 - t1) / N, (t3 - t2) / N, (t4 - t3) / N, (t5 - t4) / N, (t6 - t5) / N);
  }
  return 0;
}
