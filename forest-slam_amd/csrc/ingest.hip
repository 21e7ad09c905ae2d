// Image ingest for gfx950 — replaces ros_ws/src/stereo_slam.py:184-186 / :196-198 and
// mono_slam.py:92-93:
//   img = cv2.cvtColor(cv2.undistort(img_bgr8, K, dist), cv2.COLOR_BGR2GRAY)
// as one streaming kernel: every thread produces 4 consecutive gray pixels of a row — the
// undistortion map entry of each (initUndistortRectifyMap, CV_16SC2, evaluated in fp64 on
// the fly: no map is stored or read), the fixed-point bilinear remap of the three channels
// (INTER_LINEAR, BORDER_CONSTANT 0) and the 14-bit BGR2GRAY, one 32-bit store.
// HBM traffic per pixel: the 3 source bytes (the 2x2 gathers of neighbouring outputs hit
// the same lines in L1/L2) + 1 output byte.  Specification: oracle/ingest_ref.cpp.
#include "fvo_internal.h"

namespace {

struct Lens {
  double K[9];
  double k1, k2, p1, p2, k3;
};

// invert() 3x3 closed form (oracle inv3)
__device__ __forceinline__ void inv3(const double* S, double* t) {
  double d = S[0] * (S[4] * S[8] - S[5] * S[7]) - S[1] * (S[3] * S[8] - S[5] * S[6]) + S[2] * (S[3] * S[7] - S[4] * S[6]);
  if (d == 0.) {
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = 0.0;
    return;
  }
  d = 1. / d;
  t[0] = (S[4] * S[8] - S[5] * S[7]) * d;
  t[1] = (S[2] * S[7] - S[1] * S[8]) * d;
  t[2] = (S[1] * S[5] - S[2] * S[4]) * d;
  t[3] = (S[5] * S[6] - S[3] * S[8]) * d;
  t[4] = (S[0] * S[8] - S[2] * S[6]) * d;
  t[5] = (S[2] * S[3] - S[0] * S[5]) * d;
  t[6] = (S[3] * S[7] - S[4] * S[6]) * d;
  t[7] = (S[1] * S[6] - S[0] * S[7]) * d;
  t[8] = (S[0] * S[4] - S[1] * S[3]) * d;
}

__device__ __forceinline__ int round_sat(double v) {
  return v >= 2147483647.0 ? 2147483647 : (v <= -2147483648.0 ? (-2147483647 - 1) : (int)rint(v));
}

// PIX output pixels per thread, 4 rows x 64 threads per block.  kPinhole: K has the camera-matrix zero pattern
// (K[1] = K[3] = K[6] = K[7] = 0, K[8] = 1), so ir[6] = ir[7] = 0 (exact zeros of the closed
// form) and _w, hence w = 1/_w, is constant along a row: hoisted (bit-identical to the
// per-pixel evaluation).  The k4..k6 denominator is exactly 1 and x/1.0 == x, so it is dropped.
template <int PIX, bool kPinhole>
__global__ __launch_bounds__(256) void k_ing_undistort_gray(const uint8_t* __restrict__ src, int64_t sstride,
                                                            int spitch, uint8_t* __restrict__ dst, int64_t dstride,
                                                            int dpitch, int W, int H, int stripe0, Lens L) {
  // block = 4 rows x 64 threads, each thread PIX consecutive pixels of its row
  const int row = blockIdx.y * 4 + (threadIdx.x >> 6), b = blockIdx.z;
  const int c0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * PIX;
  if (c0 >= W || row >= H) return;
  const uint8_t* S = src + b * sstride;
  const int y0 = (row / stripe0) * stripe0, i = row - y0;
  double Ar[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) Ar[k] = L.K[k];
  Ar[5] = L.K[5] - y0;
  double ir[9];
  inv3(Ar, ir);
  const double fx = L.K[0], fy = L.K[4], u0 = L.K[2], v0 = L.K[5];
  const double bx = i * ir[1] + ir[2], by = i * ir[4] + ir[5], bw = i * ir[7] + ir[8];
  const double w_row = kPinhole ? 1. / (bw + 0 * ir[6]) : 0.0;
  uint32_t packed[PIX / 4];
#pragma unroll
  for (int k = 0; k < PIX / 4; ++k) packed[k] = 0;
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    const int col = c0 + q;
    if (col >= W) break;
    double _x = bx + col * ir[0], _y = by + col * ir[3];
    double w = kPinhole ? w_row : 1. / (bw + col * ir[6]);
    double x = _x * w, y = _y * w;
    double x2 = x * x, y2 = y * y;
    double r2 = x2 + y2, _2xy = 2 * x * y;
    double kr = (1 + ((L.k3 * r2 + L.k2) * r2 + L.k1) * r2);
    double xd = (x * kr + L.p1 * _2xy + L.p2 * (r2 + 2 * x2) + 0.0 * r2 + 0.0 * r2 * r2);
    double yd = (y * kr + L.p1 * (r2 + 2 * y2) + L.p2 * _2xy + 0.0 * r2 + 0.0 * r2 * r2);
    const int iu = round_sat((fx * xd + u0) * 32.0), iv = round_sat((fy * yd + v0) * 32.0);
    const int sx = (int16_t)(iu >> 5), sy = (int16_t)(iv >> 5);
    const int tx = iu & 31, ty = iv & 31;
    const int w0 = (32 - ty) * (32 - tx) * 32, w1 = (32 - ty) * tx * 32, w2 = ty * (32 - tx) * 32, w3 = ty * tx * 32;
    int ch[3] = {0, 0, 0};
    if (!(sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0)) {
      const bool xin0 = sx >= 0, xin1 = sx + 1 < W, yin0 = sy >= 0, yin1 = sy + 1 < H;
      const uint8_t* r0 = S + (int64_t)sy * spitch + sx * 3;
      const uint8_t* r1 = r0 + spitch;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int v00 = (yin0 && xin0) ? r0[k] : 0, v01 = (yin0 && xin1) ? r0[3 + k] : 0;
        const int v10 = (yin1 && xin0) ? r1[k] : 0, v11 = (yin1 && xin1) ? r1[3 + k] : 0;
        int s = v00 * w0 + v01 * w1 + v10 * w2 + v11 * w3;
        s = (s + (1 << 14)) >> 15;
        ch[k] = s < 0 ? 0 : (s > 255 ? 255 : s);
      }
    }
    const uint32_t g = (uint32_t)((ch[0] * 1868 + ch[1] * 9617 + ch[2] * 4899 + (1 << 13)) >> 14);
    packed[q / 4] |= g << (8 * (q % 4));
  }
  uint8_t* D = dst + b * dstride + (int64_t)row * dpitch + c0;
  if (c0 + PIX <= W && (((uintptr_t)D) & 3) == 0) {
#pragma unroll
    for (int k = 0; k < PIX / 4; ++k) reinterpret_cast<uint32_t*>(D)[k] = packed[k];
  } else {
    for (int q = 0; q < PIX && c0 + q < W; ++q) D[q] = (uint8_t)(packed[q / 4] >> (8 * (q % 4)));
  }
}

}  // namespace

int ingest_run(fvo_ctx* ctx, const uint8_t* bgr, int batch, int64_t sstride, int spitch, const double* K,
               const double* dist, uint8_t* gray, int64_t dstride, int dpitch, hipStream_t s) {
  const int W = ctx->cfg.width, H = ctx->cfg.height;
  Lens L;
  for (int i = 0; i < 9; ++i) L.K[i] = K[i];
  L.k1 = dist[0]; L.k2 = dist[1]; L.p1 = dist[2]; L.p2 = dist[3]; L.k3 = dist[4];
  int stripe0 = 4096 / (W > 1 ? W : 1);
  stripe0 = stripe0 < 1 ? 1 : (stripe0 > H ? H : stripe0);
  constexpr int PIX = 4;
  dim3 grid((W + 64 * PIX - 1) / (64 * PIX), (H + 3) / 4, batch);
  const bool pinhole = K[1] == 0.0 && K[3] == 0.0 && K[6] == 0.0 && K[7] == 0.0 && K[8] == 1.0;
  FVO_TIMED(ctx, KN_INGEST, s, {
    if (pinhole)
      hipLaunchKernelGGL((k_ing_undistort_gray<PIX, true>), grid, dim3(256), 0, s, bgr, sstride, spitch, gray, dstride,
                         dpitch, W, H, stripe0, L);
    else
      hipLaunchKernelGGL((k_ing_undistort_gray<PIX, false>), grid, dim3(256), 0, s, bgr, sstride, spitch, gray,
                         dstride, dpitch, W, H, stripe0, L);
  });
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
