// ORACLE — test infrastructure only. Never linked into the product.
//
// Restates cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True).match(d0, d1) as called at
// ros_ws/src/stereo_slam.py:85,234,242 (OpenCV 4.x batchDistance(..., K=1, crosscheck)):
//   * Hamming distance = popcount(d0[q] xor d1[t]) over the 32-byte rows;
//   * per-row argmin with strict '<' (first index wins ties), both directions;
//   * query q is kept iff sidx[q] = t and tidx[t] = q (mutual nearest neighbour);
//   * output in ascending queryIdx order (DescriptorMatcher::match, compactResult).
// Parity vs OpenCV: UNPINNED.
#include <climits>
#include <cstdint>

static inline int hamming32(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

extern "C" int ref_bf_match(const uint8_t* d0, int n0, const uint8_t* d1, int n1, int32_t* q_out, int32_t* t_out,
                            int32_t* dist_out) {
  if (n0 <= 0 || n1 <= 0) return 0;
  int* sidx = new int[n0];
  int* tidx = new int[n1];
  int* sdist = new int[n0];
  for (int q = 0; q < n0; ++q) {
    int best = INT_MAX, bi = -1;
    for (int t = 0; t < n1; ++t) {
      int d = hamming32(d0 + 32 * q, d1 + 32 * t);
      if (d < best) { best = d; bi = t; }
    }
    sidx[q] = bi;
    sdist[q] = best;
  }
  for (int t = 0; t < n1; ++t) {
    int best = INT_MAX, bi = -1;
    for (int q = 0; q < n0; ++q) {
      int d = hamming32(d1 + 32 * t, d0 + 32 * q);
      if (d < best) { best = d; bi = q; }
    }
    tidx[t] = bi;
  }
  int m = 0;
  for (int q = 0; q < n0; ++q) {
    int t = sidx[q];
    if (t >= 0 && tidx[t] == q) {
      q_out[m] = q;
      t_out[m] = t;
      dist_out[m] = sdist[q];
      ++m;
    }
  }
  delete[] sidx;
  delete[] tidx;
  delete[] sdist;
  return m;
}
