// Shared device utilities for the gfx950 (CDNA4) extraction kernels.
// Wave size is 64 on CDNA; every wave idiom below is written for 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Rounding: every square root is sqrtf (hipcc's default lowering is the
// correctly rounded v_sqrt_f32 + fma-check sequence); HIP's __fsqrt_rn is
// the bare v_sqrt_f32 (up to 1 ulp off) unless OCML_BASIC_ROUNDED_OPERATIONS
// is defined, so it never appears in a kernel that must match torch bitwise.
// __fdiv_rn and plain '/' are the correctly rounded division sequence.
#define TNP_BLOCK 256
#define TNP_WAVES (TNP_BLOCK / 64)

#define TNP_CHECK(expr)                                                        \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      tnp_set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr,                 \
                    hipGetErrorString(_e));                                    \
      return -1;                                                               \
    }                                                                          \
  } while (0)

// Host-side error slot (engine.cpp); printf-style.
void tnp_set_error(const char* fmt, ...);

static inline unsigned tnp_grid(int64_t n, int per_block = TNP_BLOCK) {
  int64_t g = (n + per_block - 1) / per_block;
  return (unsigned)(g < 1 ? 1 : g);
}

namespace tnp {

__device__ __forceinline__ int lane() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave() { return threadIdx.x >> 6; }

// XCD-aware block remap (bijective for any grid): blocks the dispatcher
// places on one XCD (blockIdx % 8 share an L2) take one CONTIGUOUS chunk of
// the work, so spatially coherent work items share that XCD's L2
__device__ __forceinline__ int64_t xcd_block(int64_t bid, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// rank of this lane among the lanes of its wave whose bit is set in `mask`
__device__ __forceinline__ int mbcnt(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// inclusive wave scan
template <typename T>
__device__ __forceinline__ T wave_scan_incl(T v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T n = __shfl_up(v, o, 64);
    if (lane() >= o) v += n;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}

// Sticky flag / bit-mask OR into a device counter word shared by the whole
// grid.  Same-address atomics serialise in the memory-side atomic unit, so
// the word is read first (agent scope: sees other XCDs' updates) and the
// atomic only issued while it would still add a bit -- a mask saturates
// after a few waves instead of costing one atomic per wave.
__device__ __forceinline__ void or_sticky(int64_t* p, uint64_t bits) {
  if (!bits) return;
  uint64_t cur = __hip_atomic_load(reinterpret_cast<uint64_t*>(p), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  if (bits & ~cur) atomicOr(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
}

// Block-wide exclusive rank of a 0/1 flag (order = thread order). Returns
// the rank; `total` receives the block count. `lds` needs TNP_WAVES ints.
// Contains two barriers: every thread of the block must call it.
__device__ __forceinline__ int block_rank(bool f, int* lds, int& total) {
  uint64_t b = __ballot(f);
  int r = mbcnt(b);
  if (lane() == 0) lds[wave()] = __popcll(b);
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < TNP_WAVES; ++i) {
    int c = lds[i];
    off += (i < wave()) ? c : 0;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return off + r;
}

// Block-wide exclusive scan of an int64 value (thread order).
__device__ __forceinline__ int64_t block_scan_excl(int64_t v, int64_t* lds, int64_t& total) {
  int64_t inc = wave_scan_incl(v);
  if (lane() == 63) lds[wave()] = inc;
  __syncthreads();
  int64_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < TNP_WAVES; ++i) {
    int64_t c = lds[i];
    off += (i < wave()) ? c : 0;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return off + inc - v;
}

// ---------------------------------------------------------------------------
// Single-pass ordered compaction / scan: decoupled look-back over tiles.
// Tiles are numbered by a ticket taken at block start (so every tile a block
// waits on belongs to a block that is already running: no co-residency
// assumption).  One 64-bit status word per tile holds
//   bits 63..62 flag (1 = tile aggregate, 2 = inclusive prefix)
//   bits 61..40 launch epoch (22 bits: stale words of earlier launches never match)
//   bits 39..0  value
// so a single relaxed agent-scope atomic load observes a consistent record.
// The ticket counter is never reset: the host passes the count already issued.
// ---------------------------------------------------------------------------
struct TnpLB {
  unsigned long long* ticket;
  uint64_t* st;
  uint64_t tbase;
  uint32_t epoch;
  int32_t spin;  // lb_prefix_rc polls before recomputing; < 0: the kernel's default
  unsigned long long* rc;  // nullable: lb_prefix_rc counts its recomputes here (diagnostics)
};

__device__ __forceinline__ int64_t lb_tile(const TnpLB& lb, int64_t* slot) {
  if (threadIdx.x == 0) *slot = (int64_t)(atomicAdd(lb.ticket, 1ull) - lb.tbase);
  __syncthreads();
  int64_t t = *slot;
  __syncthreads();
  return t;
}

// exclusive prefix of tile `tile` whose aggregate is `agg` (block-uniform);
// publishes the tile's inclusive prefix.  All threads call it.
__device__ __forceinline__ int64_t lb_prefix(const TnpLB& lb, int64_t tile, int64_t agg,
                                             int64_t* slot) {
  constexpr uint64_t VMASK = (1ull << 40) - 1ull;
  const uint64_t tag = (uint64_t)(lb.epoch & 0x3FFFFFu) << 40;
  if (threadIdx.x < 64) {
    int64_t prefix = 0;
    if (tile == 0) {
      if (lane() == 0)
        __hip_atomic_store(&lb.st[0], (2ull << 62) | tag | (uint64_t)agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane() == 0)
        __hip_atomic_store(&lb.st[tile], (1ull << 62) | tag | (uint64_t)agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      int64_t w = tile - 1;
      while (true) {
        const int64_t t = w - lane();
        uint64_t word = 0;
        int flag = 2;  // before tile 0: an inclusive zero
        if (t >= 0) {
          while (true) {
            word = __hip_atomic_load(&lb.st[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            flag = ((word & (0x3FFFFFull << 40)) == tag) ? (int)(word >> 62) : 0;
            if (flag) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        const uint64_t incl = __ballot(flag == 2);
        const int first = incl ? __builtin_ctzll(incl) : 64;
        int64_t v = (lane() <= first && t >= 0) ? (int64_t)(word & VMASK) : 0;
        prefix += wave_sum(v);
        if (incl) break;
        w -= 64;
      }
      if (lane() == 0)
        __hip_atomic_store(&lb.st[tile], (2ull << 62) | tag | (uint64_t)(prefix + agg),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) *slot = prefix;
  }
  __syncthreads();
  int64_t r = *slot;
  __syncthreads();
  return r;
}

// Ticket-free variant: the tile is blockIdx.x, so no block takes a ticket
// (one returning atomic per block on ONE word: they serialise, ~11 ns each,
// a floor of tiles * 11 ns per launch).  Without tickets a predecessor tile
// may belong to a block that is not running yet, so the look-back never
// waits unboundedly: a predecessor still unpublished after `spin` polls has
// its aggregate recomputed by the waiting wave through `tile_agg(t)` (called
// by all 64 lanes of wave 0 with a wave-uniform t; returns the tile's
// aggregate in every lane).  Deadlock-free for any dispatch order; with the
// in-order dispatch the hardware actually does, the recompute is rare.
template <class F>
__device__ __forceinline__ int64_t lb_prefix_rc(const TnpLB& lb, int64_t tile, int64_t agg,
                                                int64_t* slot, F&& tile_agg, int spin = 64) {
  constexpr uint64_t VMASK = (1ull << 40) - 1ull;
  const uint64_t tag = (uint64_t)(lb.epoch & 0x3FFFFFu) << 40;
  if (lb.spin >= 0) spin = lb.spin;
  if (threadIdx.x < 64) {
    int64_t prefix = 0;
    if (tile == 0) {
      if (lane() == 0)
        __hip_atomic_store(&lb.st[0], (2ull << 62) | tag | (uint64_t)agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane() == 0)
        __hip_atomic_store(&lb.st[tile], (1ull << 62) | tag | (uint64_t)agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      int64_t w = tile - 1;
      while (true) {
        const int64_t t = w - lane();
        int64_t val = 0;
        uint64_t word = 0;
        int flag = 2;  // before tile 0: an inclusive zero
        if (t >= 0) {
          for (int k = 0;; ++k) {
            word = __hip_atomic_load(&lb.st[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            flag = ((word & (0x3FFFFFull << 40)) == tag) ? (int)(word >> 62) : 0;
            val = (int64_t)(word & VMASK);
            if (flag || k >= spin) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        const uint64_t incl = __ballot(flag == 2);
        const int first = incl ? __builtin_ctzll(incl) : 64;
        const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
        uint64_t miss = __ballot(flag == 0) & upto;
        while (miss) {  // unpublished predecessors: recompute their aggregates
          const int l = __builtin_ctzll(miss);
          miss &= miss - 1ull;
          const int64_t v = tile_agg(w - l);
          if (lane() == l) {
            val = v;
            if (lb.rc) atomicAdd(lb.rc, 1ull);
            // publish it as that tile's aggregate unless its owner has since
            // published (so later waiters need not recompute it again)
            atomicCAS((unsigned long long*)&lb.st[w - l], (unsigned long long)word,
                      (unsigned long long)((1ull << 62) | tag | (uint64_t)v));
          }
        }
        prefix += wave_sum((lane() <= first && t >= 0) ? val : (int64_t)0);
        if (incl) break;
        w -= 64;
      }
      if (lane() == 0)
        __hip_atomic_store(&lb.st[tile], (2ull << 62) | tag | (uint64_t)(prefix + agg),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) *slot = prefix;
  }
  __syncthreads();
  int64_t r = *slot;
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// Packed per-vertex grid word (cell offsets + on-grid-plane flags).
//   bits  0..15  offset x + 2      bits 48..50 zero flag per dim (on a mark)
//   bits 16..31  offset y + 2
//   bits 32..47  offset z + 2
// offset = searchsorted(marks, x + eps) - 1 in [-1, M-1] (tropical.py:230-231)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int grid_off(uint64_t g, int d) {
  return (int)((g >> (16 * d)) & 0xFFFF) - 2;
}
__device__ __forceinline__ bool grid_zero(uint64_t g, int d) {
  return (g >> (48 + d)) & 1;
}

// A shard's owned box of the mark grid: along axis d, the cells lo[d] <= c <
// hi[d] and the mark planes lo[d] < p <= hi[d] (plane 0 by the shard with
// lo[d] == 0); lo[d] > hi[d]: the axis is not cut.  x-slabs cut x only.
struct OwnBox {
  int lo[3], hi[3];
};
__host__ __device__ __forceinline__ bool own_any(const OwnBox& o) {
  return o.lo[0] <= o.hi[0] || o.lo[1] <= o.hi[1] || o.lo[2] <= o.hi[2];
}
// a vertex (grid word g) lies in the box in the grid-region sense
__device__ __forceinline__ bool owned_by(const OwnBox& o, uint64_t g) {
  bool in = true;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int lo = o.lo[d], hi = o.hi[d], c = grid_off(g, d);
    const bool ok = grid_zero(g, d) ? ((c > lo || (lo == 0 && c == 0)) && c <= hi) : (c >= lo && c < hi);
    in &= lo > hi || ok;
  }
  return in;
}

// True in every thread of the workgroup that finishes a launch last, so it
// can finish the launch's reduction without another launch.  Hand-off
// (MI355X_MICROARCH.md, inter-workgroup visibility, first row): the values
// handed over are written with agent-scope (sc1) stores or device atomics,
// every storing wave waits for its stores, then one lane per workgroup adds
// to a zeroed ticket; the last workgroup reads them with sc1 loads
// (ld_agent).  Every thread of every workgroup must call it.
__device__ __forceinline__ bool last_block(int64_t* ticket, int* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = atomicAdd((unsigned long long*)ticket, 1ull);
    *lds_flag = t == (unsigned long long)gridDim.x * gridDim.y - 1ull;
  }
  __syncthreads();
  return *lds_flag != 0;
}
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// Sign keys of KW 64-bit words (bit p of word p / 64: plane p).  Nets of
// K <= 63 planes use one word (every kernel's original form), K in 64..127
// two (the wide shapes, net_device.h TNP_WIDE_SHAPES).  Arrays of keys are
// word arrays with KW words per entry (key_load / key_store); the vertex
// keys are ONE interleaved array pz, pos words then zero words, 2 KW per
// vertex (vkey_load, pz_load, pz_store).
// ---------------------------------------------------------------------------
template <int KW>
struct Key {
  uint64_t w[KW];
};
template <int KW>
__host__ __device__ __forceinline__ Key<KW> key_zero() {
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) k.w[q] = 0;
  return k;
}
// bits [0, n) (n <= 64 KW)
template <int KW>
__host__ __device__ __forceinline__ Key<KW> key_below(int n) {
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) {
    const int b = n - 64 * q;
    k.w[q] = b >= 64 ? ~0ull : (b <= 0 ? 0ull : ((1ull << b) - 1ull));
  }
  return k;
}
template <int KW>
__host__ __device__ __forceinline__ Key<KW> key_bit(int p) {
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) k.w[q] = (p >> 6) == q ? (1ull << (p & 63)) : 0ull;
  return k;
}
// bits [lo, hi] (0 <= lo, hi < 64 KW; empty if lo > hi)
template <int KW>
__host__ __device__ __forceinline__ Key<KW> key_range(int lo, int hi) {
  const Key<KW> a = key_below<KW>(hi + 1), b = key_below<KW>(lo);
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) k.w[q] = a.w[q] & ~b.w[q];
  return k;
}
template <int KW>
__host__ __device__ __forceinline__ Key<KW> operator&(const Key<KW>& a, const Key<KW>& b) {
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) k.w[q] = a.w[q] & b.w[q];
  return k;
}
template <int KW>
__host__ __device__ __forceinline__ Key<KW> operator|(const Key<KW>& a, const Key<KW>& b) {
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) k.w[q] = a.w[q] | b.w[q];
  return k;
}
template <int KW>
__host__ __device__ __forceinline__ Key<KW> operator^(const Key<KW>& a, const Key<KW>& b) {
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) k.w[q] = a.w[q] ^ b.w[q];
  return k;
}
template <int KW>
__host__ __device__ __forceinline__ Key<KW> operator~(const Key<KW>& a) {
  Key<KW> k;
#pragma unroll
  for (int q = 0; q < KW; ++q) k.w[q] = ~a.w[q];
  return k;
}
template <int KW>
__host__ __device__ __forceinline__ bool key_any(const Key<KW>& a) {
  uint64_t o = 0;
#pragma unroll
  for (int q = 0; q < KW; ++q) o |= a.w[q];
  return o != 0;
}
template <int KW>
__device__ __forceinline__ int key_pop(const Key<KW>& a) {
  int c = 0;
#pragma unroll
  for (int q = 0; q < KW; ++q) c += __popcll(a.w[q]);
  return c;
}
template <int KW>
__host__ __device__ __forceinline__ bool key_test(const Key<KW>& a, int p) {
  return (a.w[p >> 6] >> (p & 63)) & 1;
}
// set bit p to b (bit p clear on entry)
template <int KW>
__host__ __device__ __forceinline__ void key_put(Key<KW>& a, int p, bool b) {
  a.w[p >> 6] |= (uint64_t)b << (p & 63);
}
// 1 + the highest set bit (0: none)
template <int KW>
__device__ __forceinline__ int key_high(const Key<KW>& a) {
  int h = 0;
#pragma unroll
  for (int q = 0; q < KW; ++q)
    if (a.w[q]) h = 64 * q + 64 - __clzll(a.w[q]);
  return h;
}
// lowest set bit (-1: none)
template <int KW>
__device__ __forceinline__ int key_first(const Key<KW>& a) {
#pragma unroll
  for (int q = 0; q < KW; ++q)
    if (a.w[q]) return 64 * q + __builtin_ctzll(a.w[q]);
  return -1;
}
// key of vertex v of a word array (KW words per vertex)
template <int KW>
__device__ __forceinline__ Key<KW> key_load(const uint64_t* a, int64_t v) {
  Key<KW> k;
  if constexpr (KW == 2) {
    const ulonglong2 t = reinterpret_cast<const ulonglong2*>(a)[v];
    k.w[0] = t.x;
    k.w[1] = t.y;
  } else {
#pragma unroll
    for (int q = 0; q < KW; ++q) k.w[q] = a[KW * v + q];
  }
  return k;
}
template <int KW>
__device__ __forceinline__ void key_store(uint64_t* a, int64_t v, const Key<KW>& k) {
  if constexpr (KW == 2) {
    reinterpret_cast<ulonglong2*>(a)[v] = make_ulonglong2(k.w[0], k.w[1]);
  } else {
#pragma unroll
    for (int q = 0; q < KW; ++q) a[KW * v + q] = k.w[q];
  }
}
// Vertex keys live ONLY in the interleaved array pz (2 KW words per vertex:
// pos words, then zero words).  A kernel's `pos` / `zero` vertex-key
// pointers are views of it -- pos = pz, zero = pz + KW (engine.cpp VP / VZ)
// -- read with vkey_load; writers store the pair with pz_store.  (Round 5
// kept separate pos and zero arrays besides pz: 16 B more per new vertex.)
template <int KW>
__device__ __forceinline__ Key<KW> vkey_load(const uint64_t* a, int64_t v) {
  Key<KW> k;
  if constexpr (KW == 2) {
    const ulonglong2 t = *reinterpret_cast<const ulonglong2*>(a + 4 * v);
    k.w[0] = t.x;
    k.w[1] = t.y;
  } else {
    k.w[0] = a[2 * v];
  }
  return k;
}
// the (pos, zero) pair of vertex v from the interleaved copy
template <int KW>
__device__ __forceinline__ void pz_load(const uint64_t* pz, int64_t v, Key<KW>& p, Key<KW>& z) {
  const ulonglong2* t = reinterpret_cast<const ulonglong2*>(pz) + KW * v;
  if constexpr (KW == 1) {
    const ulonglong2 a = t[0];
    p.w[0] = a.x;
    z.w[0] = a.y;
  } else {
    const ulonglong2 a = t[0], b = t[1];
    p.w[0] = a.x;
    p.w[1] = a.y;
    z.w[0] = b.x;
    z.w[1] = b.y;
  }
}
template <int KW>
__device__ __forceinline__ void pz_store(uint64_t* pz, int64_t v, const Key<KW>& p, const Key<KW>& z) {
  ulonglong2* t = reinterpret_cast<ulonglong2*>(pz) + KW * v;
  if constexpr (KW == 1) {
    t[0] = make_ulonglong2(p.w[0], z.w[0]);
  } else {
    t[0] = make_ulonglong2(p.w[0], p.w[1]);
    t[1] = make_ulonglong2(z.w[0], z.w[1]);
  }
}
// an active-plane word: bit p for plane p < 63, bit 63 for every plane >= 63
__host__ __device__ __forceinline__ uint64_t act_bit(int p) { return 1ull << (p < 63 ? p : 63); }
__host__ __device__ __forceinline__ bool act_test(uint64_t m, int p) { return (m >> (p < 63 ? p : 63)) & 1; }

}  // namespace tnp

using tnp::TnpLB;
using tnp::Key;
using tnp::OwnBox;
