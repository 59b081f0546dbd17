// Radix sorts: (1) cell bucketing of (cell, member) entries; (2) packed u64 keys (connecting edges lo << nb | hi)
// on their 2*nb significant bits: the lexicographic order of
// c_new.sort(-1).unique(dim=0) (subpoly.py:243-244) -- the keys are already
// unique, one per canonical cell.  rocPRIM's onesweep radix sort is the
// primitive; only the significant bits are visited.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"
#include "step.h"

// rocPRIM sorts up to 1 M keys by block sort + merge passes (a dozen launches
// for 2 M keys); the connecting-edge keys go to onesweep above this size
#ifndef TNP_SORT_MERGE_LIMIT
#define TNP_SORT_MERGE_LIMIT (256 * 1024)
#endif
// onesweep in 1024-thread blocks of 8 keys per thread: 0.43 -> 0.40 ms per
// 128^3 pass against rocPRIM's gfx950 default (512 x 12); 1024 x 6 measured
// the same, 1024 x 12 and 768 x 8 slower (tools/sort_cfg_bench.hip, A/B in
// the engine)
using KeySortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 8,
                                        rocprim::block_radix_rank_algorithm::match>,
    TNP_SORT_MERGE_LIMIT>;

size_t sort_scratch_bytes(int64_t n, int bits) {
  size_t bytes = 0;
  rocprim::double_buffer<uint64_t> db(nullptr, nullptr);
  if (rocprim::radix_sort_keys<KeySortCfg>(nullptr, bytes, db, (size_t)std::max<int64_t>(n, 1), 0u,
                                           (unsigned)bits) != hipSuccess)
    return 0;
  return bytes;
}

int sort_keys_u64(uint64_t* a, uint64_t* b, int64_t n, int bits, void* scratch, size_t scratch_bytes,
                  uint64_t** out, hipStream_t s) {
  *out = a;
  if (n <= 1) return 0;
  rocprim::double_buffer<uint64_t> db(a, b);
  size_t bytes = scratch_bytes;
  TNP_CHECK(rocprim::radix_sort_keys<KeySortCfg>(scratch, bytes, db, (size_t)n, 0u, (unsigned)bits, s));
  *out = db.current();
  return 0;
}

size_t sort_pairs_scratch_bytes(int64_t n, int bits) {
  size_t bytes = 0;
  rocprim::double_buffer<uint32_t> k(nullptr, nullptr);
  rocprim::double_buffer<int32_t> v(nullptr, nullptr);
  if (rocprim::radix_sort_pairs(nullptr, bytes, k, v, (size_t)std::max<int64_t>(n, 1), 0u,
                                (unsigned)bits) != hipSuccess)
    return 0;
  return bytes;
}

int sort_pairs_u32(uint32_t* ka, uint32_t* kb, int32_t* va, int32_t* vb, int64_t n, int bits,
                   void* scratch, size_t scratch_bytes, uint32_t** ko, int32_t** vo, hipStream_t s) {
  *ko = ka;
  *vo = va;
  if (n <= 1) return 0;
  rocprim::double_buffer<uint32_t> k(ka, kb);
  rocprim::double_buffer<int32_t> v(va, vb);
  size_t bytes = scratch_bytes;
  TNP_CHECK(rocprim::radix_sort_pairs(scratch, bytes, k, v, (size_t)n, 0u, (unsigned)bits, s));
  *ko = k.current();
  *vo = v.current();
  return 0;
}
