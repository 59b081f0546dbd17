// Probe: is v_mfma_f32_16x16x4_f32, chained over K-blocks in ascending order
// from C = 0, bit-for-bit the sequential fmaf chain acc = fma(x_k, W_jk, acc)
// that the MKL SEQ schedule computes (net_device.h linear / neuron_mode
// LIN_SEQ)?  This is the premise of k_forward_new's MFMA layers.
//
// The layer is computed TRANSPOSED, as the kernel does: D[j'][r] =
// sum_k A[j'][k] B[k][r], A = the weights (row j' = neuron perm(j')), B = the
// activations of 16 data rows.  Inputs: random fp32 of wide exponent range,
// with zeros, negative zeros, denormals and exact cancellations mixed in.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/bin/mfma_probe tools/mfma_probe.hip
//   tools/bin/mfma_probe            (prints mismatches per K, exit 1 on any)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(2);                                                \
    }                                                         \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// one wave per problem: W [16][K], X [16 rows][K] -> out [16 rows][16]
template <int K>
__global__ void k_mfma(const float* __restrict__ W, const float* __restrict__ X, float* __restrict__ out, int nprob) {
  const int p = blockIdx.x;
  if (p >= nprob) return;
  const int l = threadIdx.x;
  const int q = l >> 4, r = l & 15;
  const float* w = W + (size_t)p * 16 * K;
  const float* x = X + (size_t)p * 16 * K;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < K / 4; ++s) {
    // A[i = l&15][k = l>>4]: neuron row perm(i) = 4*(i&3) + (i>>2)
    const int i = r, j = 4 * (i & 3) + (i >> 2);
    const float a = w[j * K + 4 * s + q];
    const float b = x[r * K + 4 * s + q];  // B[k = l>>4][col = l&15]
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  // D[row = 4q + g][col = r]: neuron perm(4q + g) = 4g + q of data row r
#pragma unroll
  for (int g = 0; g < 4; ++g) out[((size_t)p * 16 + r) * 16 + 4 * g + q] = acc[g];
}

template <int K>
__global__ void k_seq(const float* __restrict__ W, const float* __restrict__ X, float* __restrict__ out, int nprob) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nprob * 256) return;
  const int p = (int)(t >> 8), r = (int)((t >> 4) & 15), j = (int)(t & 15);
  const float* w = W + (size_t)p * 16 * K;
  const float* x = X + (size_t)p * 16 * K;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc = __fmaf_rn(x[r * K + k], w[j * K + k], acc);
  out[((size_t)p * 16 + r) * 16 + j] = acc;
}

static uint64_t rs = 0x243F6A8885A308D3ull;
static uint32_t rnd() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint32_t)(rs >> 16);
}
static float rval(int mode) {
  const uint32_t u = rnd();
  switch (u % 23) {
    case 0: return 0.f;
    case 1: return -0.f;
    case 2: {  // denormal
      uint32_t b = (rnd() & 0x007FFFFFu) | (rnd() & 0x80000000u);
      float f;
      memcpy(&f, &b, 4);
      return f;
    }
    default: break;
  }
  const float m = (float)(rnd() % 2000001) / 1000000.0f - 1.0f;
  const int e = mode ? (int)(rnd() % 60) - 30 : (int)(rnd() % 8) - 4;
  return ldexpf(m, e);
}

template <int K>
static int run(int nprob, int mode) {
  const size_t nw = (size_t)nprob * 16 * K;
  float *hW = (float*)malloc(nw * 4), *hX = (float*)malloc(nw * 4);
  for (size_t i = 0; i < nw; ++i) hW[i] = rval(mode);
  for (size_t i = 0; i < nw; ++i) hX[i] = rval(mode);
  // exact cancellations: some rows repeat a product with the opposite sign
  for (int p = 0; p < nprob; p += 7) hX[(size_t)p * 16 * K + 1] = -hX[(size_t)p * 16 * K];
  float *dW, *dX, *d1, *d2;
  const size_t no = (size_t)nprob * 256;
  CK(hipMalloc(&dW, nw * 4));
  CK(hipMalloc(&dX, nw * 4));
  CK(hipMalloc(&d1, no * 4));
  CK(hipMalloc(&d2, no * 4));
  CK(hipMemcpy(dW, hW, nw * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dX, hX, nw * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_mfma<K>, dim3(nprob), dim3(64), 0, 0, dW, dX, d1, nprob);
  hipLaunchKernelGGL(k_seq<K>, dim3((unsigned)((no + 255) / 256)), dim3(256), 0, 0, dW, dX, d2, nprob);
  CK(hipDeviceSynchronize());
  uint32_t *h1 = (uint32_t*)malloc(no * 4), *h2 = (uint32_t*)malloc(no * 4);
  CK(hipMemcpy(h1, d1, no * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2, d2, no * 4, hipMemcpyDeviceToHost));
  size_t bad = 0, zs = 0, dn = 0;
  for (size_t i = 0; i < no; ++i) {
    if (h1[i] != h2[i]) {
      if (bad < 4) fprintf(stderr, "K=%d mode=%d i=%zu mfma %08x seq %08x\n", K, mode, i, h1[i], h2[i]);
      ++bad;
    }
    zs += (h2[i] & 0x7FFFFFFFu) == 0;
    dn += (h2[i] & 0x7F800000u) == 0 && (h2[i] & 0x007FFFFFu) != 0;
  }
  printf("K=%2d mode=%d outputs=%zu mismatches=%zu (zeros %zu, denormal results %zu)\n", K, mode, no, bad, zs, dn);
  free(hW);
  free(hX);
  free(h1);
  free(h2);
  CK(hipFree(dW));
  CK(hipFree(dX));
  CK(hipFree(d1));
  CK(hipFree(d2));
  return bad != 0;
}

int main() {
  int bad = 0;
  for (int mode = 0; mode < 2; ++mode) {
    bad |= run<4>(20000, mode);
    bad |= run<8>(20000, mode);
    bad |= run<16>(20000, mode);
    bad |= run<32>(20000, mode);
  }
  printf(bad ? "MFMA != fma chain\n" : "MFMA == sequential fma chain, bitwise\n");
  return bad;
}
