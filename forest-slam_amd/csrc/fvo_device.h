// Device-side helpers shared by the HIP translation units (the host-only declarations are in
// fvo_internal.h, which capi.cpp includes alone: it compiles as plain host C++ too, e.g. for
// the sanitizer build of the argument validation, tools/sanitize.sh).
#pragma once

#include "fvo_internal.h"

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ int wave_lane() { return (int)(threadIdx.x & 63); }

// XCD-aware block order.  Dispatch sends linear block L to XCD L mod 8, so neighbouring
// blocks (which read overlapping image rows / patches) would land in 8 different L2s; the
// logical index returned here hands each XCD one contiguous eighth of the grid instead.
struct XcdBlock {
  int x, y, z;
};
__device__ __forceinline__ XcdBlock xcd_block() {
  const int gx = gridDim.x, gy = gridDim.y;
  const int N = gx * gy * gridDim.z;
  const int L = (blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x;
  const int per = N >> 3;
  const int lg = L < (per << 3) ? (L & 7) * per + (L >> 3) : L;
  const int t = lg / gx;
  return XcdBlock{lg - t * gx, t % gy, t / gy};
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
