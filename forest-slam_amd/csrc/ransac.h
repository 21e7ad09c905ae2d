// RANSACPointSetRegistrator pieces shared by the PnP (pose.hip) and essential-matrix
// (essential.hip) estimators: OpenCV's RNG(-1) multiply-with-carry generator, getSubset()'s
// draws of distinct indices and RANSACUpdateNumIters (calib3d/src/ptsetreg.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

namespace fvo_rs {

struct RNG {
  uint64_t state;
  __device__ unsigned next() {
    state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
    return (unsigned)state;
  }
  __device__ int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

__device__ inline int update_num_iters(double p, double ep, int m, int maxIters) {
  p = fmax(p, 0.);
  p = fmin(p, 1.);
  ep = fmax(ep, 0.);
  ep = fmin(ep, 1.);
  double num = fmax(1. - p, DBL_MIN);
  double denom = 1. - pow(1. - ep, (double)m);
  if (denom < DBL_MIN) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)rint(num / denom);
}

// Subsets of every potential RANSAC iteration as getSubset() draws them with RNG(-1):
// 5 distinct indices from rng.uniform(0, n), repeats rejected.  The draws depend only on
// n, so all maxIters subsets can be generated before any hypothesis is scored.
__device__ inline void draw_subsets(int n, int maxIters, int16_t* out) {
  RNG rng{~0ull};
  for (int it = 0; it < maxIters; ++it) {
    int idx[5];
    for (int i = 0; i < 5; ++i) {
      int j;
      for (;;) {
        j = rng.uniform(0, n);
        bool dup = false;
        for (int q = 0; q < i; ++q) dup |= idx[q] == j;
        if (!dup) break;
      }
      idx[i] = j;
      out[it * 5 + i] = (int16_t)j;
    }
  }
}

}  // namespace fvo_rs
