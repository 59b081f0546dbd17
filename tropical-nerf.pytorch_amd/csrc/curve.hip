// Curve-approximation branch of a hyperplane step (subpoly_(..., force=False),
// tropical/subpoly.py:120-177, 201-207; tropical/geometry.py:24-138, 259-299,
// 350-372; tropical/subpoly_debug.py:121-165, 234-271) on gfx950.
//
// For every split edge that is not axis-aligned (c rows) the new vertex is
// the intersection of the two trilinear level sets it lies between -- the
// last plane below idx both endpoints are zero on (p) and the current plane
// (q) -- on the xz-diagonal plane of the edge's box:
//
//   curve_flags   c = more than one coordinate differs by > eps
//   curve_corners 8 box corners per c row (corner 4i+2j+k: x from endpoint
//                 k, y from j, z from i) + the shared plane p
//   forward(group=8) over the corners (one activation pattern per box)
//   curve_solve   quartic in x from the corner values, the last real root in
//                 [0,1] in LAPACK's eigenvalue order (sgeev restated for
//                 companions of degree 2..4), y from the quadratic ratio,
//                 bilinear boxes -> -1
//   forward over e0(1-t) + e1 t, curve_dnew  residuals on p and q
//   descend       normalised gradient descent of p^2 + q^2 (500 iterations
//                 max, all rows stop together: pass 1 records per-iteration
//                 convergence bits, pass 2 replays to the common stop)
//   curve_apply   v = e0 + t (e1 - e0); strict-filter inputs
//   (finish) strict_keep + compact_splits: dropped splits stay unsplit, new
//                 vertex ids follow the surviving edges' order
//
// Degree 2 reproduces MKL's sgeev bitwise; degree 3/4 follow reference
// LAPACK's fp32 algorithm (same eigenvalue order as MKL, values to fp32
// rounding), so vertices agree with the reference to ~1e-7, not bitwise
// (curve path tolerance 1e-5).
#include "common.h"
#include "kernels.h"
#include "net_device.h"
#include "step.h"

using namespace tnpnet;

namespace {

constexpr float ROOT_EPS = 1e-9f;  // geometry.py:259, 271

__global__ void k_curve_flags(const int32_t* __restrict__ sa, const int32_t* __restrict__ sb,
                              int64_t S, const float* __restrict__ xyz, float eps,
                              int32_t* __restrict__ cflag) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= S) return;
  int a = sa[r], b = sb[r], n = 0;
#pragma unroll
  for (int d = 0; d < 3; ++d)
    n += fabsf(__fsub_rn(xyz[3 * (int64_t)b + d], xyz[3 * (int64_t)a + d])) > eps;
  cflag[r] = n > 1;
}

__global__ void k_curve_rows(const int32_t* __restrict__ cflag, const int64_t* __restrict__ coff,
                             int64_t S, int32_t* __restrict__ crow) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < S && cflag[r]) crow[coff[r]] = (int32_t)r;
}

template <int KW>
__global__ void k_curve_corners(const int32_t* __restrict__ crow, int64_t B,
                                const int32_t* __restrict__ sa, const int32_t* __restrict__ sb,
                                const float* __restrict__ xyz, const uint64_t* __restrict__ zero,
                                const uint64_t* __restrict__ grid, int idx, float* __restrict__ corners,
                                int32_t* __restrict__ plane, int64_t* __restrict__ ctr) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 8 * B) return;
  int64_t b = t >> 3;
  int n = (int)(t & 7);
  int r = crow[b];
  int e[2] = {sa[r], sb[r]};
  int k = n & 1, j = (n >> 1) & 1, i = n >> 2;
  corners[3 * t + 0] = xyz[3 * (int64_t)e[k] + 0];
  corners[3 * t + 1] = xyz[3 * (int64_t)e[j] + 1];
  corners[3 * t + 2] = xyz[3 * (int64_t)e[i] + 2];
  if (n == 0) {
    // last plane j < idx both endpoints are eps-zero on (nonzero_last,
    // torch_ext.py:18-29); none -> the reference exit()s (subpoly.py:141-148)
    const Key<KW> zz = tnp::vkey_load<KW>(zero, e[0]) & tnp::vkey_load<KW>(zero, e[1]);
    const Key<KW> m = zz & tnp::key_below<KW>(idx);
    const int hi = tnp::key_high(m);
    plane[b] = hi ? hi - 1 : 0;
    if (!hi) atomicOr((unsigned long long*)&ctr[CTR_NOPLANE], 1ull);
    // check_new_vertices_on_two_planes (subpoly.py:134-135, subpoly_debug.py:
    // 96-104): the endpoints share fewer than two zero columns (every plane,
    // plus grid axes with both on the same mark) -> the reference's
    // diagnostic print fails (AttributeError: Tensor.astype)
    const uint64_t ga = grid[e[0]], gb = grid[e[1]];
    int shared = tnp::key_pop(zz);
#pragma unroll
    for (int d = 0; d < 3; ++d)
      shared += tnp::grid_zero(ga, d) && tnp::grid_zero(gb, d) && tnp::grid_off(ga, d) == tnp::grid_off(gb, d);
    if (shared < 2) atomicOr((unsigned long long*)&ctr[CTR_NOPLANE], 2ull);
  }
}

// ---- sgeev on a 2x2 real matrix, as x86 MKL computes it ---------------------
// (torch.linalg.eigvals on the quadratics' companion matrices -- 98% of the
// curve rows).  sgebal (permute + power-of-2 balance), slahqr's
// Ahues-Kressner deflation test on H(2,1), slanv2's standardisation; fp32
// with explicit roundings.  Reverse-engineered bitwise against torch on CPU
// (tools/lapack2x2_probe.py: 20000 random companions + every quadratic row
// of the golden nets).
__device__ __forceinline__ float fsign(float a, float b) { return b >= 0.f ? fabsf(a) : -fabsf(a); }

__device__ __forceinline__ float slapy2(float x, float y) {
  x = fabsf(x);
  y = fabsf(y);
  float w = fmaxf(x, y), z = fminf(x, y);
  if (z == 0.f || w > 3.4e38f) return w;
  float r = __fdiv_rn(z, w);
  return __fmul_rn(w, sqrtf(__fadd_rn(1.f, __fmul_rn(r, r))));
}

__device__ void slanv2(float a, float b, float c, float d, float wr[2], float wi[2]) {
  const float EPS = 1.1920928955078125e-07f;  // slamch('P')
  if (c == 0.f) {
  } else if (b == 0.f) {
    float t = d;
    d = a;
    a = t;
    b = -c;
    c = 0.f;
  } else if (__fsub_rn(a, d) == 0.f && ((b > 0.f) != (c > 0.f))) {
  } else {
    float temp = __fsub_rn(a, d);
    float p = __fmul_rn(0.5f, temp);
    float bcmax = fmaxf(fabsf(b), fabsf(c));
    float bcmis = __fmul_rn(__fmul_rn(fminf(fabsf(b), fabsf(c)), fsign(1.f, b)), fsign(1.f, c));
    float scale = fmaxf(fabsf(p), bcmax);
    float z = __fadd_rn(__fmul_rn(__fdiv_rn(p, scale), p), __fmul_rn(__fdiv_rn(bcmax, scale), bcmis));
    if (z >= 4.f * EPS) {
      z = __fadd_rn(p, fsign(__fmul_rn(sqrtf(scale), sqrtf(z)), p));
      a = __fadd_rn(d, z);
      d = __fsub_rn(d, __fmul_rn(__fdiv_rn(bcmax, z), bcmis));
      b = __fsub_rn(b, c);
      c = 0.f;
    } else {
      float sigma = __fadd_rn(b, c);
      float tau = slapy2(sigma, temp);
      float cs = sqrtf(__fmul_rn(0.5f, __fadd_rn(1.f, __fdiv_rn(fabsf(sigma), tau))));
      float sn = __fmul_rn(-__fdiv_rn(p, __fmul_rn(tau, cs)), fsign(1.f, sigma));
      float aa = __fadd_rn(__fmul_rn(a, cs), __fmul_rn(b, sn));
      float bb = __fadd_rn(__fmul_rn(-a, sn), __fmul_rn(b, cs));
      float cc = __fadd_rn(__fmul_rn(c, cs), __fmul_rn(d, sn));
      float dd = __fadd_rn(__fmul_rn(-c, sn), __fmul_rn(d, cs));
      a = __fadd_rn(__fmul_rn(aa, cs), __fmul_rn(cc, sn));
      b = __fadd_rn(__fmul_rn(bb, cs), __fmul_rn(dd, sn));
      c = __fadd_rn(__fmul_rn(-aa, sn), __fmul_rn(cc, cs));
      d = __fadd_rn(__fmul_rn(-bb, sn), __fmul_rn(dd, cs));
      temp = __fmul_rn(0.5f, __fadd_rn(a, d));
      a = d = temp;
      if (c != 0.f) {
        if (b != 0.f) {
          if ((b > 0.f) == (c > 0.f)) {
            float sab = sqrtf(fabsf(b)), sac = sqrtf(fabsf(c));
            p = fsign(__fmul_rn(sab, sac), c);
            a = __fadd_rn(temp, p);
            d = __fsub_rn(temp, p);
            b = __fsub_rn(b, c);
            c = 0.f;
          }
        } else {
          b = -c;
          c = 0.f;
        }
      }
    }
  }
  wr[0] = a;
  wr[1] = d;
  if (c == 0.f) {
    wi[0] = wi[1] = 0.f;
  } else {
    wi[0] = __fmul_rn(sqrtf(fabsf(b)), sqrtf(fabsf(c)));
    wi[1] = -wi[0];
  }
}

__device__ __forceinline__ float nrm2_2(float x, float y) {
  double s = (double)x * (double)x + (double)y * (double)y;
  return (float)sqrt(s);
}

__device__ void eig2x2(float A[2][2], float wr[2], float wi[2]) {
  // sgebal: permutations isolating eigenvalues
  int k = 0, l = 1;
  bool done = false;
  for (;;) {  // rows with zero off-diagonal (columns 0..l) pushed down
    int found = -1;
    for (int j = l; j >= 0; --j) {
      bool z = true;
      for (int i = 0; i <= l; ++i)
        if (i != j && A[j][i] != 0.f) z = false;
      if (z) { found = j; break; }
    }
    if (found < 0) break;
    if (found != l) {
      for (int r = 0; r < 2; ++r) { float t = A[r][found]; A[r][found] = A[r][l]; A[r][l] = t; }
      for (int c = 0; c < 2; ++c) { float t = A[found][c]; A[found][c] = A[l][c]; A[l][c] = t; }
    }
    if (l == 0) { done = true; break; }
    --l;
  }
  if (done) {
    wr[0] = A[0][0]; wr[1] = A[1][1]; wi[0] = wi[1] = 0.f;
    return;
  }
  for (;;) {  // columns with zero off-diagonal (rows k..l) pushed left
    int found = -1;
    for (int j = k; j <= l; ++j) {
      bool z = true;
      for (int i = k; i <= l; ++i)
        if (i != j && A[i][j] != 0.f) z = false;
      if (z) { found = j; break; }
    }
    if (found < 0) break;
    if (found != k) {
      for (int r = 0; r < 2; ++r) { float t = A[r][found]; A[r][found] = A[r][k]; A[r][k] = t; }
      for (int c = 0; c < 2; ++c) { float t = A[found][c]; A[found][c] = A[k][c]; A[k][c] = t; }
    }
    ++k;
  }
  if (k >= l) {  // at most one row left unisolated
    wr[0] = A[0][0]; wr[1] = A[1][1]; wi[0] = wi[1] = 0.f;
    return;
  }
  // power-of-2 balancing of rows/columns k..l (= 0..1 here)
  const float SAFMIN = 1.17549435e-38f, ULP = 1.1920928955078125e-07f;
  const float SFMIN1 = SAFMIN / ULP, SFMAX1 = 1.f / SFMIN1;
  const float SFMIN2 = SFMIN1 * 2.f, SFMAX2 = 1.f / SFMIN2;
  float scale[2] = {1.f, 1.f};
  for (int pass = 0; pass < 64; ++pass) {
    bool noconv = false;
    for (int i = 0; i < 2; ++i) {
      float c = nrm2_2(A[0][i], A[1][i]);
      float r = nrm2_2(A[i][0], A[i][1]);
      float ca = fmaxf(fabsf(A[0][i]), fabsf(A[1][i]));
      float ra = fmaxf(fabsf(A[i][0]), fabsf(A[i][1]));
      if (c == 0.f || r == 0.f) continue;
      float g = r / 2.f, f = 1.f, s = __fadd_rn(c, r);
      while (!(c >= g || fmaxf(f, fmaxf(c, ca)) >= SFMAX2 || fminf(r, fminf(g, ra)) <= SFMIN2)) {
        f *= 2.f; c *= 2.f; ca *= 2.f; r /= 2.f; g /= 2.f; ra /= 2.f;
      }
      g = c / 2.f;
      while (!(g < r || fmaxf(r, ra) >= SFMAX2 || fminf(fminf(f, c), fminf(g, ca)) <= SFMIN2)) {
        f /= 2.f; c /= 2.f; g /= 2.f; ca /= 2.f; r *= 2.f; ra *= 2.f;
      }
      if (__fadd_rn(c, r) >= __fmul_rn(0.95f, s)) continue;
      if (f < 1.f && scale[i] < 1.f && f * scale[i] <= SFMIN1) continue;
      if (f > 1.f && scale[i] > 1.f && scale[i] >= SFMAX1 / f) continue;
      float gi = 1.f / f;
      scale[i] *= f;
      noconv = true;
      A[i][0] *= gi; A[i][1] *= gi;
      A[0][i] *= f; A[1][i] *= f;
    }
    if (!noconv) break;
  }
  // slahqr: H(2,1) negligible (Ahues & Kressner) -> two 1x1 blocks
  const float SMLNUM = SAFMIN * (2.f / ULP);
  float h21 = fabsf(A[1][0]);
  bool defl = h21 <= SMLNUM;
  if (!defl) {
    float tst = __fadd_rn(fabsf(A[0][0]), fabsf(A[1][1]));
    if (h21 <= __fmul_rn(ULP, tst)) {
      float ab = fmaxf(h21, fabsf(A[0][1])), ba = fminf(h21, fabsf(A[0][1]));
      float dd = fabsf(__fsub_rn(A[0][0], A[1][1]));
      float aa = fmaxf(fabsf(A[1][1]), dd), bb = fminf(fabsf(A[1][1]), dd);
      float s = __fadd_rn(aa, ab);
      defl = __fmul_rn(ba, __fdiv_rn(ab, s)) <= fmaxf(SMLNUM, __fmul_rn(ULP, __fmul_rn(bb, __fdiv_rn(aa, s))));
    }
  }
  if (defl) {
    wr[0] = A[0][0]; wr[1] = A[1][1]; wi[0] = wi[1] = 0.f;
    return;
  }
  slanv2(A[0][0], A[0][1], A[1][0], A[1][1], wr, wi);
}

// ---- sgeev (eigenvalues only) on a 3x3 / 4x4 real matrix, reference LAPACK --
// sgebal('B') -> sgehd2 -> slahqr in fp32 with explicit roundings
// (tools/lapack_eig_port.py is the host restatement).  What the reference's
// "last real root in [0, 1]" (geometry.py:292-296) depends on is the ORDER
// of the eigenvalues: the restatement's order equals x86 MKL's
// (torch.linalg.eigvals) on every random companion checked; the values
// agree to fp32 rounding, ~1e-4 only for clustered (ill-conditioned) roots.
template <int N>
struct SmallEig {
  float H[N][N];
  float wr[N], wi[N];

  __device__ static float nrm(const float* v, int n, int stride) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += (double)v[i * stride] * (double)v[i * stride];
    return (float)sqrt(s);
  }
  // slarfg on (alpha, x[0..n1)): beta -> alpha, tau returned, x scaled
  __device__ static float slarfg(float& alpha, float* x, int n1) {
    if (n1 <= 0) return 0.f;
    double s = 0.0;
    for (int i = 0; i < n1; ++i) s += (double)x[i] * (double)x[i];
    const float xnorm = (float)sqrt(s);
    if (xnorm == 0.f) return 0.f;
    const float beta = -fsign(slapy2(alpha, xnorm), alpha);
    const float tau = __fdiv_rn(__fsub_rn(beta, alpha), beta);
    const float sc = __fdiv_rn(1.f, __fsub_rn(alpha, beta));
    for (int i = 0; i < n1; ++i) x[i] = __fmul_rn(x[i], sc);
    alpha = beta;
    return tau;
  }

  __device__ void balance(int& k, int& l) {
    k = 0;
    l = N - 1;
    for (;;) {  // rows with zero off-diagonal (columns 0..l) pushed down
      int found = -1;
      for (int j = l; j >= 0 && found < 0; --j) {
        bool z = true;
        for (int i = 0; i <= l; ++i)
          if (i != j && H[j][i] != 0.f) z = false;
        if (z) found = j;
      }
      if (found < 0) break;
      if (found != l) {
        for (int r = 0; r < N; ++r) { const float t = H[r][found]; H[r][found] = H[r][l]; H[r][l] = t; }
        for (int c = 0; c < N; ++c) { const float t = H[found][c]; H[found][c] = H[l][c]; H[l][c] = t; }
      }
      if (l == 0) { k = l = 0; return; }
      --l;
    }
    for (;;) {  // columns with zero off-diagonal (rows k..l) pushed left
      int found = -1;
      for (int j = k; j <= l && found < 0; ++j) {
        bool z = true;
        for (int i = k; i <= l; ++i)
          if (i != j && H[i][j] != 0.f) z = false;
        if (z) found = j;
      }
      if (found < 0) break;
      if (found != k) {
        for (int r = 0; r < N; ++r) { const float t = H[r][found]; H[r][found] = H[r][k]; H[r][k] = t; }
        for (int c = 0; c < N; ++c) { const float t = H[found][c]; H[found][c] = H[k][c]; H[k][c] = t; }
      }
      ++k;
    }
    if (k >= l) return;
    const float SAFMIN = 1.17549435e-38f, ULP = 1.1920928955078125e-07f;
    const float SFMIN1 = SAFMIN / ULP, SFMAX1 = 1.f / SFMIN1;
    const float SFMIN2 = SFMIN1 * 2.f, SFMAX2 = 1.f / SFMIN2;
    float scale[N];
    for (int i = 0; i < N; ++i) scale[i] = 1.f;
    for (int pass = 0; pass < 100; ++pass) {
      bool noconv = false;
      for (int i = k; i <= l; ++i) {
        float c = nrm(&H[k][i], l - k + 1, N);
        float r = nrm(&H[i][k], l - k + 1, 1);
        float ca = 0.f, ra = 0.f;
        for (int q = 0; q <= l; ++q) ca = fmaxf(ca, fabsf(H[q][i]));
        for (int q = k; q < N; ++q) ra = fmaxf(ra, fabsf(H[i][q]));
        if (c == 0.f || r == 0.f) continue;
        float g = r / 2.f, f = 1.f;
        const float s = __fadd_rn(c, r);
        while (!(c >= g || fmaxf(f, fmaxf(c, ca)) >= SFMAX2 || fminf(r, fminf(g, ra)) <= SFMIN2)) {
          f *= 2.f; c *= 2.f; ca *= 2.f; r /= 2.f; g /= 2.f; ra /= 2.f;
        }
        g = c / 2.f;
        while (!(g < r || fmaxf(r, ra) >= SFMAX2 || fminf(fminf(f, c), fminf(g, ca)) <= SFMIN2)) {
          f /= 2.f; c /= 2.f; g /= 2.f; ca /= 2.f; r *= 2.f; ra *= 2.f;
        }
        if (__fadd_rn(c, r) >= __fmul_rn(0.95f, s)) continue;
        if (f < 1.f && scale[i] < 1.f && f * scale[i] <= SFMIN1) continue;
        if (f > 1.f && scale[i] > 1.f && scale[i] >= SFMAX1 / f) continue;
        const float gi = 1.f / f;
        scale[i] *= f;
        noconv = true;
        for (int q = k; q < N; ++q) H[i][q] = __fmul_rn(H[i][q], gi);
        for (int q = 0; q <= l; ++q) H[q][i] = __fmul_rn(H[q][i], f);
      }
      if (!noconv) break;
    }
  }

  __device__ void hessenberg(int ilo, int ihi) {  // sgehd2
    for (int i = ilo; i < ihi; ++i) {
      float x[N];
      const int n1 = ihi - i - 1;
      for (int j = 0; j < n1; ++j) x[j] = H[i + 2 + j][i];
      float alpha = H[i + 1][i];
      const float tau = slarfg(alpha, x, n1);
      H[i + 1][i] = alpha;
      for (int j = 0; j < n1; ++j) H[i + 2 + j][i] = x[j];
      if (tau == 0.f) continue;
      float v[N];
      v[0] = 1.f;
      for (int j = 0; j < n1; ++j) v[j + 1] = x[j];
      const int nv = n1 + 1;
      for (int r = 0; r <= ihi; ++r) {  // right: C -= tau (C v) v^T
        float w = 0.f;
        for (int q = 0; q < nv; ++q) w = __fadd_rn(w, __fmul_rn(H[r][i + 1 + q], v[q]));
        for (int q = 0; q < nv; ++q) H[r][i + 1 + q] = __fsub_rn(H[r][i + 1 + q], __fmul_rn(__fmul_rn(tau, w), v[q]));
      }
      for (int c = i + 1; c < N; ++c) {  // left: C -= tau v (v^T C)
        float w = 0.f;
        for (int q = 0; q < nv; ++q) w = __fadd_rn(w, __fmul_rn(H[i + 1 + q][c], v[q]));
        for (int q = 0; q < nv; ++q) H[i + 1 + q][c] = __fsub_rn(H[i + 1 + q][c], __fmul_rn(__fmul_rn(tau, v[q]), w));
      }
    }
    for (int i = ilo; i < ihi; ++i)
      for (int j = i + 2; j < N; ++j) H[j][i] = 0.f;
  }

  // slahqr (WANTT = WANTZ = false); false if it did not converge
  __device__ bool qr(int ilo, int ihi) {
    const float SAFMIN = 1.17549435e-38f, ULP = 1.1920928955078125e-07f;
    for (int i = 0; i < N; ++i) { wr[i] = H[i][i]; wi[i] = 0.f; }
    if (ilo == ihi) return true;
    for (int j = ilo; j < ihi - 2; ++j) { H[j + 2][j] = 0.f; H[j + 3][j] = 0.f; }
    if (ilo <= ihi - 2) H[ihi][ihi - 2] = 0.f;
    const int nh = ihi - ilo + 1;
    const float smlnum = __fmul_rn(SAFMIN, __fdiv_rn((float)nh, ULP));
    const int itmax = 30 * (nh > 10 ? nh : 10);
    int kdefl = 0;
    int i = ihi;
    while (i >= ilo) {
      int l = ilo;
      bool conv = false;
      for (int its = 0; its <= itmax; ++its) {
        int k = i;
        for (; k > l; --k) {
          if (fabsf(H[k][k - 1]) <= smlnum) break;
          float tst = __fadd_rn(fabsf(H[k - 1][k - 1]), fabsf(H[k][k]));
          if (tst == 0.f) {
            if (k - 2 >= ilo) tst = __fadd_rn(tst, fabsf(H[k - 1][k - 2]));
            if (k + 1 <= ihi) tst = __fadd_rn(tst, fabsf(H[k + 1][k]));
          }
          if (fabsf(H[k][k - 1]) <= __fmul_rn(ULP, tst)) {
            const float ab = fmaxf(fabsf(H[k][k - 1]), fabsf(H[k - 1][k]));
            const float ba = fminf(fabsf(H[k][k - 1]), fabsf(H[k - 1][k]));
            const float dd = fabsf(__fsub_rn(H[k - 1][k - 1], H[k][k]));
            const float aa = fmaxf(fabsf(H[k][k]), dd), bb = fminf(fabsf(H[k][k]), dd);
            const float s = __fadd_rn(aa, ab);
            if (__fmul_rn(ba, __fdiv_rn(ab, s)) <= fmaxf(smlnum, __fmul_rn(ULP, __fmul_rn(bb, __fdiv_rn(aa, s)))))
              break;
          }
        }
        l = k;
        if (l > ilo) H[l][l - 1] = 0.f;
        if (l >= i - 1) { conv = true; break; }
        ++kdefl;
        const int i1 = l, i2 = i;
        float h11, h12, h21, h22;
        if (kdefl % 20 == 0) {
          const float s = __fadd_rn(fabsf(H[i][i - 1]), fabsf(H[i - 1][i - 2]));
          h11 = __fadd_rn(__fmul_rn(0.75f, s), H[i][i]); h12 = __fmul_rn(-0.4375f, s); h21 = s; h22 = h11;
        } else if (kdefl % 10 == 0) {
          const float s = __fadd_rn(fabsf(H[l + 1][l]), fabsf(H[l + 2][l + 1]));
          h11 = __fadd_rn(__fmul_rn(0.75f, s), H[l][l]); h12 = __fmul_rn(-0.4375f, s); h21 = s; h22 = h11;
        } else {
          h11 = H[i - 1][i - 1]; h21 = H[i][i - 1]; h12 = H[i - 1][i]; h22 = H[i][i];
        }
        float rt1r, rt1i, rt2r, rt2i;
        float s = __fadd_rn(__fadd_rn(__fadd_rn(fabsf(h11), fabsf(h12)), fabsf(h21)), fabsf(h22));
        if (s == 0.f) {
          rt1r = rt1i = rt2r = rt2i = 0.f;
        } else {
          h11 = __fdiv_rn(h11, s); h21 = __fdiv_rn(h21, s); h12 = __fdiv_rn(h12, s); h22 = __fdiv_rn(h22, s);
          const float tr = __fdiv_rn(__fadd_rn(h11, h22), 2.f);
          const float det = __fsub_rn(__fmul_rn(__fsub_rn(h11, tr), __fsub_rn(h22, tr)), __fmul_rn(h12, h21));
          const float rtdisc = sqrtf(fabsf(det));
          if (det >= 0.f) {
            rt1r = __fmul_rn(tr, s); rt2r = rt1r; rt1i = __fmul_rn(rtdisc, s); rt2i = -rt1i;
          } else {
            rt1r = __fadd_rn(tr, rtdisc); rt2r = __fsub_rn(tr, rtdisc);
            if (fabsf(__fsub_rn(rt1r, h22)) <= fabsf(__fsub_rn(rt2r, h22))) { rt1r = __fmul_rn(rt1r, s); rt2r = rt1r; }
            else { rt2r = __fmul_rn(rt2r, s); rt1r = rt2r; }
            rt1i = rt2i = 0.f;
          }
        }
        int m = i - 2;
        float v[3];
        for (;;) {
          float h21s = H[m + 1][m];
          s = __fadd_rn(__fadd_rn(fabsf(__fsub_rn(H[m][m], rt2r)), fabsf(rt2i)), fabsf(h21s));
          h21s = __fdiv_rn(H[m + 1][m], s);
          v[0] = __fsub_rn(__fadd_rn(__fmul_rn(h21s, H[m][m + 1]),
                                     __fmul_rn(__fsub_rn(H[m][m], rt1r), __fdiv_rn(__fsub_rn(H[m][m], rt2r), s))),
                           __fmul_rn(rt1i, __fdiv_rn(rt2i, s)));
          v[1] = __fmul_rn(h21s, __fsub_rn(__fsub_rn(__fadd_rn(H[m][m], H[m + 1][m + 1]), rt1r), rt2r));
          v[2] = __fmul_rn(h21s, H[m + 2][m + 1]);
          s = __fadd_rn(__fadd_rn(fabsf(v[0]), fabsf(v[1])), fabsf(v[2]));
          v[0] = __fdiv_rn(v[0], s); v[1] = __fdiv_rn(v[1], s); v[2] = __fdiv_rn(v[2], s);
          if (m == l) break;
          const float h00 = __fmul_rn(fabsf(H[m][m - 1]), __fadd_rn(fabsf(v[1]), fabsf(v[2])));
          const float h01 = __fmul_rn(__fmul_rn(ULP, fabsf(v[0])),
                                      __fadd_rn(__fadd_rn(fabsf(H[m - 1][m - 1]), fabsf(H[m][m])), fabsf(H[m + 1][m + 1])));
          if (h00 <= h01) break;
          --m;
        }
        for (int k2 = m; k2 < i; ++k2) {
          const int nr = (3 < i - k2 + 1) ? 3 : i - k2 + 1;
          if (k2 > m)
            for (int q = 0; q < nr; ++q) v[q] = H[k2 + q][k2 - 1];
          float alpha = v[0];
          const float t1 = slarfg(alpha, v + 1, nr - 1);
          v[0] = alpha;
          if (k2 > m) {
            H[k2][k2 - 1] = v[0];
            H[k2 + 1][k2 - 1] = 0.f;
            if (k2 < i - 1) H[k2 + 2][k2 - 1] = 0.f;
          } else if (m > l) {
            H[k2][k2 - 1] = __fmul_rn(H[k2][k2 - 1], __fsub_rn(1.f, t1));
          }
          const float v2 = v[1], t2 = __fmul_rn(t1, v2);
          if (nr == 3) {
            const float v3 = v[2], t3 = __fmul_rn(t1, v3);
            for (int j = k2; j <= i2; ++j) {
              const float sm = __fadd_rn(__fadd_rn(H[k2][j], __fmul_rn(v2, H[k2 + 1][j])), __fmul_rn(v3, H[k2 + 2][j]));
              H[k2][j] = __fsub_rn(H[k2][j], __fmul_rn(sm, t1));
              H[k2 + 1][j] = __fsub_rn(H[k2 + 1][j], __fmul_rn(sm, t2));
              H[k2 + 2][j] = __fsub_rn(H[k2 + 2][j], __fmul_rn(sm, t3));
            }
            const int jend = (k2 + 3 < i) ? k2 + 3 : i;
            for (int j = i1; j <= jend; ++j) {
              const float sm = __fadd_rn(__fadd_rn(H[j][k2], __fmul_rn(v2, H[j][k2 + 1])), __fmul_rn(v3, H[j][k2 + 2]));
              H[j][k2] = __fsub_rn(H[j][k2], __fmul_rn(sm, t1));
              H[j][k2 + 1] = __fsub_rn(H[j][k2 + 1], __fmul_rn(sm, t2));
              H[j][k2 + 2] = __fsub_rn(H[j][k2 + 2], __fmul_rn(sm, t3));
            }
          } else if (nr == 2) {
            for (int j = k2; j <= i2; ++j) {
              const float sm = __fadd_rn(H[k2][j], __fmul_rn(v2, H[k2 + 1][j]));
              H[k2][j] = __fsub_rn(H[k2][j], __fmul_rn(sm, t1));
              H[k2 + 1][j] = __fsub_rn(H[k2 + 1][j], __fmul_rn(sm, t2));
            }
            for (int j = i1; j <= i; ++j) {
              const float sm = __fadd_rn(H[j][k2], __fmul_rn(v2, H[j][k2 + 1]));
              H[j][k2] = __fsub_rn(H[j][k2], __fmul_rn(sm, t1));
              H[j][k2 + 1] = __fsub_rn(H[j][k2 + 1], __fmul_rn(sm, t2));
            }
          }
        }
      }
      if (!conv) return false;
      if (l == i) {
        wr[i] = H[i][i];
        wi[i] = 0.f;
      } else {
        float w2r[2], w2i[2];
        slanv2(H[i - 1][i - 1], H[i - 1][i], H[i][i - 1], H[i][i], w2r, w2i);
        wr[i - 1] = w2r[0]; wr[i] = w2r[1]; wi[i - 1] = w2i[0]; wi[i] = w2i[1];
      }
      kdefl = 0;
      i = l - 1;
    }
    return true;
  }

  // eigenvalues of H in LAPACK order; false: no convergence
  __device__ bool solve() {
    int k, l;
    balance(k, l);
    hessenberg(k, l);
    return qr(k, l);
  }
};

// the reference's choice for a companion of degree N (3 or 4): the last
// eigenvalue in LAPACK order that is real and in [0, 1]; -1 if none
template <int N>
__device__ float last_root01(const float* c, int lead) {
  SmallEig<N> e;
  for (int r = 0; r < N; ++r)
    for (int q = 0; q < N; ++q) e.H[r][q] = (q == r + 1) ? 1.f : 0.f;
  // C[:, -1] = -coeffs[:-1] / coeffs[lead] on the flipped (ascending) row:
  // last row entry q is -c_asc[q] / c_lead, c_asc[q] = c[lead + N - q]
  for (int q = 0; q < N; ++q) e.H[N - 1][q] = __fdiv_rn(-c[lead + N - q], c[lead]);
  if (!e.solve()) return -1.f;
  float r = -1.f;
  for (int q = 0; q < N; ++q)
    if (fabsf(e.wi[q]) <= ROOT_EPS && e.wr[q] >= 0.f && e.wr[q] <= 1.f) r = e.wr[q];
  return r;
}

// batched_polynomial_roots (geometry.py:259-299) for one row of 5 fp32
// coefficients (leading first): tiny coefficients zeroed, degree from the
// first non-zero one, companion row r_k = -c_k / c_lead in fp32 (what LAPACK
// sees), the last real eigenvalue in [0, 1] in LAPACK order, -1 if none.
__device__ float largest_root01(float c[5]) {
#pragma unroll
  for (int k = 0; k < 5; ++k)
    if (fabsf(c[k]) < ROOT_EPS) c[k] = 0.f;
  int i = 0;
  while (i < 4 && c[i] == 0.f) ++i;
  if (i == 4) return -1.f;
  const int N = 4 - i;
  float s = 0.f;
  for (int k = 4; k >= i; --k) s = __fadd_rn(s, fabsf(c[k]));
  if (!(__fdiv_rn(s, (float)(N + 1)) > ROOT_EPS)) return -1.f;
  if (N == 1) {
    float r = __fdiv_rn(-c[4], c[3]);
    return (r >= 0.f && r <= 1.f) ? r : -1.f;
  }
  if (N == 2) {
    // companion [[0, 1], [-c4/c2, -c3/c2]]; the LAST eigenvalue (LAPACK's
    // order) that is real and in [0, 1]
    float A[2][2] = {{0.f, 1.f}, {__fdiv_rn(-c[4], c[2]), __fdiv_rn(-c[3], c[2])}};
    float wr[2], wi[2];
    eig2x2(A, wr, wi);
    float r = -1.f;
    for (int k = 0; k < 2; ++k)
      if (fabsf(wi[k]) <= ROOT_EPS && wr[k] >= 0.f && wr[k] <= 1.f) r = wr[k];
    return r;
  }
  return N == 3 ? last_root01<3>(c, i) : last_root01<4>(c, i);
}

// intersection_of_two_planes (geometry.py:24-138), "xz" assumption
__device__ void plane_intersection(const float p[8], const float q[8], float t[3]) {
  const int LO[4] = {0, 1, 4, 5}, HI[4] = {2, 3, 6, 7};
  float zq_lo[3] = {q[LO[0]], __fadd_rn(q[LO[1]], q[LO[2]]), q[LO[3]]};
  float zq_hi[3] = {q[HI[0]], __fadd_rn(q[HI[1]], q[HI[2]]), q[HI[3]]};
  float zp_lo[3] = {p[LO[0]], __fadd_rn(p[LO[1]], p[LO[2]]), p[LO[3]]};
  float zp_hi[3] = {p[HI[0]], __fadd_rn(p[HI[1]], p[HI[2]]), p[HI[3]]};
  float A[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      A[i][j] = __fsub_rn(__fmul_rn(zq_lo[i], zp_hi[j]), __fmul_rn(zq_hi[i], zp_lo[j]));
  const float T[3][3] = {{1.f, -2.f, 1.f}, {-1.f, 1.f, 0.f}, {1.f, 0.f, 0.f}};
  float M[3][3], Bm[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) acc = __fmaf_rn(T[k][i], A[k][j], acc);
      M[i][j] = acc;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) acc = __fmaf_rn(M[i][k], T[k][j], acc);
      Bm[i][j] = acc;
    }
  float c[5] = {Bm[0][0], __fadd_rn(Bm[1][0], Bm[0][1]),
                __fadd_rn(__fadd_rn(Bm[2][0], Bm[1][1]), Bm[0][2]),
                __fadd_rn(Bm[1][2], Bm[2][1]), Bm[2][2]};
  float x = largest_root01(c);
  float om = __fsub_rn(1.f, x);
  float X[4] = {__fmul_rn(om, om), __fmul_rn(x, om), __fmul_rn(x, om), __fmul_rn(x, x)};
  float ax = 0.f, bx = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ax = __fadd_rn(ax, __fmul_rn(q[LO[k]], X[k]));
    bx = __fadd_rn(bx, __fmul_rn(q[HI[k]], X[k]));
  }
  float y = __fdiv_rn(ax, __fsub_rn(ax, bx));
  // bilinear boxes (both planes constant along one axis): the reference's
  // failover=False branch marks them -1 (geometry.py:106-136)
  const int FT[3][4] = {{0, 1, 4, 5}, {0, 1, 2, 3}, {0, 4, 2, 6}};
  const int FU[3][4] = {{2, 3, 6, 7}, {4, 5, 6, 7}, {1, 5, 3, 7}};
  bool flat = false;
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    bool all = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) all &= (p[FT[f][k]] == p[FU[f][k]]) && (q[FT[f][k]] == q[FU[f][k]]);
    flat |= all;
  }
  if (flat) x = y = -1.f;
  t[0] = x;
  t[1] = y;
  t[2] = x;
}

__global__ void k_curve_solve(int64_t B, const float* __restrict__ stage_c, int64_t ldc,
                              const int32_t* __restrict__ plane, int idx,
                              const int32_t* __restrict__ crow, const int32_t* __restrict__ sa,
                              const int32_t* __restrict__ sb, const float* __restrict__ xyz,
                              float* __restrict__ ints, float* __restrict__ pts) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float p[8], q[8];
  const float* P = stage_c + (int64_t)plane[b] * ldc + 8 * b;
  const float* Q = stage_c + (int64_t)idx * ldc + 8 * b;
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    p[n] = P[n];
    q[n] = Q[n];
  }
  float t[3];
  plane_intersection(p, q, t);
  int r = crow[b];
  int64_t a = sa[r], e = sb[r];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    ints[3 * b + d] = t[d];
    pts[3 * b + d] = __fadd_rn(__fmul_rn(xyz[3 * a + d], __fsub_rn(1.f, t[d])),
                               __fmul_rn(xyz[3 * e + d], t[d]));
  }
}

// residuals at the solved points; gg (no root in the box), gd (needs descent)
__global__ void k_curve_dnew(int64_t B, const float* __restrict__ stage_p, int64_t ldp,
                             const int32_t* __restrict__ plane, int idx,
                             const float* __restrict__ ints, float eps, float* __restrict__ d0s,
                             float* __restrict__ d1s, int32_t* __restrict__ gg,
                             int32_t* __restrict__ gd) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float d0 = stage_p[(int64_t)plane[b] * ldp + b];
  float d1 = stage_p[(int64_t)idx * ldp + b];
  bool out = false;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float t = ints[3 * b + d];
    out |= (t < 0.f) || (t > 1.f);
  }
  d0s[b] = d0;
  d1s[b] = d1;
  gg[b] = out;
  gd[b] = !out && (fabsf(d0) > eps || fabsf(d1) > eps);
}

__global__ void k_gd_rows(const int32_t* __restrict__ gd, const int64_t* __restrict__ goff, int64_t B,
                          int32_t* __restrict__ glist) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B && gd[b]) glist[goff[b]] = (int32_t)b;
}

// v = e0 + t (e1 - e0) for c rows (subpoly.py:204-207) and the per-split
// strict-filter inputs: cinfo bit0 c row, bit1 gg, bit2 |d0| < eps; the
// global "some kept c row has |d0| > eps" flag (subpoly_debug.py:253-257).
__global__ void k_curve_apply(int64_t B, const int32_t* __restrict__ crow,
                              const int32_t* __restrict__ sa, const int32_t* __restrict__ sb,
                              float* __restrict__ xyz, int64_t V, const float* __restrict__ ints,
                              const float* __restrict__ d0s, const int32_t* __restrict__ gg,
                              float eps, int32_t* __restrict__ cinfo, int64_t* __restrict__ ctr) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool tight = false;
  if (b < B) {
    int r = crow[b];
    int64_t a = sa[r], e = sb[r];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float e0 = xyz[3 * a + d];
      float dd = __fsub_rn(xyz[3 * e + d], e0);
      xyz[3 * (V + r) + d] = __fadd_rn(e0, __fmul_rn(ints[3 * b + d], dd));
    }
    bool out = gg[b] != 0;
    float d0 = out ? 0.f : d0s[b];
    cinfo[r] = 1 | (out ? 2 : 0) | (fabsf(d0) < eps ? 4 : 0);
    tight = fabsf(d0) > eps;
  }
  if (__ballot(tight) && tnp::lane() == 0) tnp::or_sticky(&ctr[CTR_TIGHT], 1ull);
}

// strict_check (subpoly_debug.py:234-271) after the override
template <int KW>
__global__ void k_strict_keep(int64_t S, const int32_t* __restrict__ cinfo,
                              const float* __restrict__ stage, int idx, int override_,
                              const uint64_t* __restrict__ shared, float eps, int tight, int strict,
                              int32_t* __restrict__ keep) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= S) return;
  float chk = stage[(int64_t)idx * S + r];
  if (override_ && tnp::key_test(tnp::key_load<KW>(shared, r), idx)) chk = 0.f;
  bool k = fabsf(chk) < eps;
  int ci = cinfo[r];
  if (ci & 1) k = k && !(ci & 2) && (!tight || (ci & 4));
  keep[r] = strict ? k : 1;  // strict=False: every split stays (subpoly.py:198-202)
}

// surviving splits -> consecutive new ids in edge order; the split edge's
// second endpoint becomes the new vertex (masked_scatter_, subpoly.py:211)
template <int KW>
__global__ void k_compact_splits(int64_t S, int K, const int32_t* __restrict__ keep,
                                 const int64_t* __restrict__ nid, const int32_t* __restrict__ eidx,
                                 int64_t V, const int32_t* __restrict__ sa,
                                 const int32_t* __restrict__ sb, const uint64_t* __restrict__ shared,
                                 const float* __restrict__ stage, const float* __restrict__ xyz,
                                 const uint64_t* __restrict__ grid, int64_t S2,
                                 int32_t* __restrict__ sa2, int32_t* __restrict__ sb2,
                                 uint64_t* __restrict__ shared2, float* __restrict__ stage2,
                                 float* __restrict__ xyz2, uint64_t* __restrict__ grid2,
                                 int32_t* __restrict__ edges) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= S || !keep[r]) return;
  int64_t n = nid[r];
  sa2[n] = sa[r];
  sb2[n] = sb[r];
  tnp::key_store(shared2, n, tnp::key_load<KW>(shared, r));
  for (int p = 0; p < K; ++p) stage2[(int64_t)p * S2 + n] = stage[(int64_t)p * S + r];
#pragma unroll
  for (int d = 0; d < 3; ++d) xyz2[3 * n + d] = xyz[3 * (V + r) + d];
  grid2[n] = grid[V + r];
  edges[2 * (int64_t)eidx[r] + 1] = (int32_t)(V + n);
}

}  // namespace

int launch_curve_flags(const int32_t* sa, const int32_t* sb, int64_t S, const float* xyz, float eps,
                       int32_t* cflag, hipStream_t s) {
  if (S <= 0) return 0;
  hipLaunchKernelGGL(k_curve_flags, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, sa, sb, S, xyz, eps,
                     cflag);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_curve_rows(const int32_t* cflag, const int64_t* coff, int64_t S, int32_t* crow,
                      hipStream_t s) {
  if (S <= 0) return 0;
  hipLaunchKernelGGL(k_curve_rows, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, cflag, coff, S, crow);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_curve_corners(const int32_t* crow, int64_t B, const int32_t* sa, const int32_t* sb,
                         const float* xyz, const uint64_t* zero, const uint64_t* grid, int idx, float* corners,
                         int32_t* plane, int64_t* ctr, int kw, hipStream_t s) {
  if (B <= 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_curve_corners<2>, dim3(tnp_grid(8 * B)), dim3(TNP_BLOCK), 0, s, crow, B, sa, sb,
                       xyz, zero, grid, idx, corners, plane, ctr);
  else
    hipLaunchKernelGGL(k_curve_corners<1>, dim3(tnp_grid(8 * B)), dim3(TNP_BLOCK), 0, s, crow, B, sa, sb,
                       xyz, zero, grid, idx, corners, plane, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_curve_solve(int64_t B, const float* stage_c, int64_t ldc, const int32_t* plane, int idx,
                       const int32_t* crow, const int32_t* sa, const int32_t* sb, const float* xyz,
                       float* ints, float* pts, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_curve_solve, dim3(tnp_grid(B)), dim3(TNP_BLOCK), 0, s, B, stage_c, ldc, plane,
                     idx, crow, sa, sb, xyz, ints, pts);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_curve_dnew(int64_t B, const float* stage_p, int64_t ldp, const int32_t* plane, int idx,
                      const float* ints, float eps, float* d0s, float* d1s, int32_t* gg, int32_t* gd,
                      hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_curve_dnew, dim3(tnp_grid(B)), dim3(TNP_BLOCK), 0, s, B, stage_p, ldp, plane,
                     idx, ints, eps, d0s, d1s, gg, gd);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_gd_rows(const int32_t* gd, const int64_t* goff, int64_t B, int32_t* glist, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_gd_rows, dim3(tnp_grid(B)), dim3(TNP_BLOCK), 0, s, gd, goff, B, glist);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_descend(const NetDev& net, int64_t G, const int32_t* glist, const int32_t* crow,
                   const int32_t* sa, const int32_t* sb, const float* xyz, const int32_t* plane,
                   int idx, float eps, int iters, int record, float* ints, float* d0s, float* d1s,
                   unsigned long long* conv, hipStream_t s) {
  if (G <= 0) return 0;
  if (!net_supported(net)) { tnp_set_error("the curve descent: net shape not instantiated"); return -1; }
  if (iters > 512) { tnp_set_error("descend: at most 512 iterations"); return -1; }
  // TNP_DESCEND_THREAD=1: the one-thread-per-row kernel (tests compare both)
  const char* pt = getenv("TNP_DESCEND_THREAD");
  const bool per_thread = pt && pt[0] == '1';
  TNP_LV_SWITCH(net.n_levels, return lv_descend<L_>(net, G, glist, crow, sa, sb, xyz, plane, idx, eps, iters, record,
                                                     ints, d0s, d1s, conv, per_thread, s));
  return 0;
}
int launch_curve_apply(int64_t B, const int32_t* crow, const int32_t* sa, const int32_t* sb,
                       float* xyz, int64_t V, const float* ints, const float* d0s, const int32_t* gg,
                       float eps, int32_t* cinfo, int64_t* ctr, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_curve_apply, dim3(tnp_grid(B)), dim3(TNP_BLOCK), 0, s, B, crow, sa, sb, xyz, V,
                     ints, d0s, gg, eps, cinfo, ctr);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_strict_keep(int64_t S, const int32_t* cinfo, const float* stage, int idx, int override_,
                       const uint64_t* shared, float eps, int tight, int strict, int32_t* keep, int kw,
                       hipStream_t s) {
  if (S <= 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_strict_keep<2>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, S, cinfo, stage, idx,
                       override_, shared, eps, tight, strict, keep);
  else
    hipLaunchKernelGGL(k_strict_keep<1>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, S, cinfo, stage, idx,
                       override_, shared, eps, tight, strict, keep);
  TNP_CHECK(hipGetLastError());
  return 0;
}
int launch_compact_splits(int64_t S, int K, const int32_t* keep, const int64_t* nid,
                          const int32_t* eidx, int64_t V, const int32_t* sa, const int32_t* sb,
                          const uint64_t* shared, const float* stage, const float* xyz,
                          const uint64_t* grid, int64_t S2, int32_t* sa2, int32_t* sb2,
                          uint64_t* shared2, float* stage2, float* xyz2, uint64_t* grid2,
                          int32_t* edges, int kw, hipStream_t s) {
  if (S <= 0) return 0;
  if (kw == 2)
    hipLaunchKernelGGL(k_compact_splits<2>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, S, K, keep, nid,
                       eidx, V, sa, sb, shared, stage, xyz, grid, S2, sa2, sb2, shared2, stage2, xyz2,
                       grid2, edges);
  else
    hipLaunchKernelGGL(k_compact_splits<1>, dim3(tnp_grid(S)), dim3(TNP_BLOCK), 0, s, S, K, keep, nid,
                       eidx, V, sa, sb, shared, stage, xyz, grid, S2, sa2, sb2, shared2, stage2, xyz2,
                       grid2, edges);
  TNP_CHECK(hipGetLastError());
  return 0;
}
