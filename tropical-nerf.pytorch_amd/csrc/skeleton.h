// Internal: skeleton launchers (skeleton.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

int launch_skel_eval(const NetDev& net, int i0, int j0, int k0, int n0, int n1, int n2,
                     float* dist, unsigned int* gmax_bits, hipStream_t s);
int64_t skel_candidates(int n0, int n1, int n2);
int64_t skel_tiles(int64_t n);
// the tile's lattice points as vertices (sign mode's forward input)
int launch_skel_points(int i0, int j0, int k0, int n0, int n1, int n2, const float* marks, float* xyz,
                       hipStream_t s);
// keys != null (2 kw x u64 per tile point, (pos, zero) as pz): sign mode, else distance
int launch_skel_edges(bool emit, int i0, int j0, int k0, int n0, int n1, int n2, int L,
                      const float* dist, const uint64_t* keys, float dmax, const unsigned int* gmax_bits,
                      int32_t* blk, const int64_t* blkoff, int64_t out_base, int32_t* out, int32_t* used,
                      hipStream_t s, int kw = 1);
// per-axis, per-mark-plane counts of the tile's points under its edge
// threshold (the sharded skeleton's load balance), added into load[3][L]
int launch_skel_load(int i0, int j0, int k0, int n0, int n1, int n2, int L, const float* dist, float dmax,
                     const unsigned int* gmax_bits, int64_t* load, hipStream_t s);
int launch_skel_vertices(const int32_t* used, const int64_t* nid, int64_t n, int L,
                         const float* marks, float* xyz, hipStream_t s);
int launch_remap_i32(int32_t* e, int64_t n, const int64_t* nid, hipStream_t s);
