// ORACLE — test infrastructure only. Never linked into the product.
//
// Restates the image ingest of ros_ws/src/stereo_slam.py:184-186 / :196-198 and
// mono_slam.py:92-93:
//   img = cv2.undistort(img_bgr8, K, dist)      # default newCameraMatrix = K
//   img = cv2.cvtColor(img, cv2.COLOR_BGR2GRAY)
// following OpenCV 4.x (imgproc undistort.dispatch.cpp, undistort.simd.hpp,
// imgwarp.cpp remapBilinear, color_rgb.simd.hpp RGB2Gray<uchar>):
//   * undistort works in horizontal stripes of stripe0 = min(max(1, 4096 / cols), rows)
//     rows; for the stripe starting at row y the new camera matrix is K with cy' = cy - y,
//     inverted by invert()'s 3x3 closed form (Cramer, det3, d = 1/det);
//   * initUndistortRectifyMap (R = I, CV_16SC2 map): row i of the stripe, column j:
//     _x = i*ir[1] + ir[2] + j*ir[0] (likewise _y, _w), w = 1/_w, x = _x*w, y = _y*w,
//     radial-tangential model (k1 k2 p1 p2 k3; k4..k6, s1..s4 = 0, no tilt),
//     u = fx*xd + cx, v = fy*yd + cy (the ORIGINAL K), iu = cvRound(u*32), iv = cvRound(v*32),
//     integer map (iu >> 5, iv >> 5), fractional index (iv & 31)*32 + (iu & 31);
//   * remap INTER_LINEAR, BORDER_CONSTANT 0: weights ((32-fy)(32-fx), (32-fy)fx, fy(32-fx),
//     fy fx) * 32 (INTER_REMAP_COEF_BITS 15, exact for INTER_TAB_SIZE 32), per channel
//     (sum + 2^14) >> 15 saturated to u8, out-of-image neighbours read as 0, a sample whose
//     2x2 support lies wholly outside is 0;
//   * BGR2GRAY: (B*1868 + G*9617 + R*4899 + 2^13) >> 14.
// The column term is evaluated directly (_x + j*ir[0]) instead of OpenCV's running sum;
// the two differ by ulps, which moves a map entry by 1/32 px only when u*32 lies within
// ~1e-9 of a rounding boundary.  Parity vs OpenCV: UNPINNED (no cv2 here).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <vector>

namespace ing {

// OpenCV invert() 3x3 closed form (DECOMP_LU branch for n == 3, double).
static bool inv3(const double* S, double* t) {
  auto m = [&](int r, int c) { return S[r * 3 + c]; };
  double d = m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) - m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
             m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
  if (d == 0.) return false;
  d = 1. / d;
  t[0] = (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) * d;
  t[1] = (m(0, 2) * m(2, 1) - m(0, 1) * m(2, 2)) * d;
  t[2] = (m(0, 1) * m(1, 2) - m(0, 2) * m(1, 1)) * d;
  t[3] = (m(1, 2) * m(2, 0) - m(1, 0) * m(2, 2)) * d;
  t[4] = (m(0, 0) * m(2, 2) - m(0, 2) * m(2, 0)) * d;
  t[5] = (m(0, 2) * m(1, 0) - m(0, 0) * m(1, 2)) * d;
  t[6] = (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0)) * d;
  t[7] = (m(0, 1) * m(2, 0) - m(0, 0) * m(2, 1)) * d;
  t[8] = (m(0, 0) * m(1, 1) - m(0, 1) * m(1, 0)) * d;
  return true;
}

// Map entry of output pixel (row, col): integer source (sx, sy) and fractional index.
static void map_entry(const double* K, const double* dist, int W, int H, int row, int col, int* sx, int* sy,
                      int* frac) {
  int stripe0 = 4096 / (W > 1 ? W : 1);
  if (stripe0 < 1) stripe0 = 1;
  if (stripe0 > H) stripe0 = H;
  const int y0 = (row / stripe0) * stripe0, i = row - y0;
  double Ar[9];
  std::memcpy(Ar, K, sizeof(Ar));
  Ar[5] = K[5] - y0;
  double ir[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  inv3(Ar, ir);
  const double fx = K[0], fy = K[4], u0 = K[2], v0 = K[5];
  const double k1 = dist[0], k2 = dist[1], p1 = dist[2], p2 = dist[3], k3 = dist[4];
  double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
  _x = _x + col * ir[0];
  _y = _y + col * ir[3];
  _w = _w + col * ir[6];
  double w = 1. / _w, x = _x * w, y = _y * w;
  double x2 = x * x, y2 = y * y;
  double r2 = x2 + y2, _2xy = 2 * x * y;
  double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((0.0 * r2 + 0.0) * r2 + 0.0) * r2);
  double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + 0.0 * r2 + 0.0 * r2 * r2);
  double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + 0.0 * r2 + 0.0 * r2 * r2);
  double u = fx * xd + u0;
  double v = fy * yd + v0;
  double su = u * 32.0, sv = v * 32.0;
  int iu = su >= 2147483647.0 ? 2147483647 : (su <= -2147483648.0 ? (-2147483647 - 1) : (int)std::lrint(su));
  int iv = sv >= 2147483647.0 ? 2147483647 : (sv <= -2147483648.0 ? (-2147483647 - 1) : (int)std::lrint(sv));
  *sx = (int16_t)(iu >> 5);  // map storage is CV_16SC2: a plain (short) cast
  *sy = (int16_t)(iv >> 5);
  *frac = (iv & 31) * 32 + (iu & 31);
}

}  // namespace ing

extern "C" {

// cv2.undistort(src, K, dist) then cv2.cvtColor(., COLOR_BGR2GRAY) on one H x W BGR8 image
// (rows `pitch` bytes apart).  K row-major 3x3, dist (k1, k2, p1, p2, k3).
void ref_undistort_gray(const uint8_t* bgr, int H, int W, int pitch, const double* K, const double* dist,
                        uint8_t* gray) {
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c) {
      int sx, sy, f;
      ing::map_entry(K, dist, W, H, r, c, &sx, &sy, &f);
      const int fx = f & 31, fy = f >> 5;
      const int w[4] = {(32 - fy) * (32 - fx) * 32, (32 - fy) * fx * 32, fy * (32 - fx) * 32, fy * fx * 32};
      int ch[3] = {0, 0, 0};
      if (!(sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0)) {
        for (int k = 0; k < 3; ++k) {
          int v[4];
          for (int q = 0; q < 4; ++q) {
            int xx = sx + (q & 1), yy = sy + (q >> 1);
            v[q] = (xx >= 0 && xx < W && yy >= 0 && yy < H) ? bgr[(size_t)yy * pitch + xx * 3 + k] : 0;
          }
          int s = v[0] * w[0] + v[1] * w[1] + v[2] * w[2] + v[3] * w[3];
          s = (s + (1 << 14)) >> 15;
          ch[k] = s < 0 ? 0 : (s > 255 ? 255 : s);
        }
      }
      gray[(size_t)r * W + c] = (uint8_t)((ch[0] * 1868 + ch[1] * 9617 + ch[2] * 4899 + (1 << 13)) >> 14);
    }
}

// The undistortion map alone (debug / tests): sx, sy, frac per output pixel.
void ref_undistort_map(int H, int W, const double* K, const double* dist, int16_t* mxy, uint16_t* frac) {
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c) {
      int sx, sy, f;
      ing::map_entry(K, dist, W, H, r, c, &sx, &sy, &f);
      mxy[((size_t)r * W + c) * 2] = (int16_t)sx;
      mxy[((size_t)r * W + c) * 2 + 1] = (int16_t)sy;
      frac[(size_t)r * W + c] = (uint16_t)f;
    }
}


// Motion-blur ablation, forest_slam_ros/src/stereo_slam.py:142-178:
//   kernel = warpAffine(np.diag(np.ones(k)), getRotationMatrix2D((k//2, k//2), 0, 1), (k, k)) / k
//     (angle 0: M = [[1, 0, 0], [0, 1, 0]], the warp is the identity -> diag(1/k), float64)
//   blurred = cv2.filter2D(img, -1, kernel)  (anchor (k//2, k//2), BORDER_REFLECT_101)
//     OpenCV 4.x filter.dispatch.cpp: kernels with k*k >= 130 (8U -> 8U, SSE3 host) go to
//     dftFilter2D (crossCorr in float32, cvRound on convert): its value is S/k within DFT
//     rounding; restated as the exact S/k, ties (even k, S = q*k + k/2) half to even (unpinned);
//     smaller kernels go to Filter2D<uchar, Cast<float, uchar>, FilterVec_8u>: nonzero taps
//     (preprocess2DKernel, row-major) with float coefficients, s = fma(x, kf, s) from delta 0
//     (v_muladd on the AVX2+FMA3 dispatch), v_round (half to even), saturate.
//   mask[max(0, y-k//2):min(H, y+k//2+1), max(0, x-k//2):min(W, x+k//2+1)] = 1 per sampled pixel
//   out = np.where(mask, blurred, img)
static int refl101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

void ref_motion_blur(const uint8_t* img, int H, int W, int k, const int32_t* centers, int n_centers, uint8_t* mask,
                     uint8_t* out) {
  // the kernel matrix (angle 0) and its nonzero taps in row-major order
  std::vector<double> kern((size_t)k * k, 0.0);
  for (int i = 0; i < k; ++i) kern[(size_t)i * k + i] = 1.0 / k;
  std::vector<int> ty, tx;
  std::vector<float> tw;
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c)
      if (kern[(size_t)r * k + c] != 0.0) { ty.push_back(r); tx.push_back(c); tw.push_back((float)kern[(size_t)r * k + c]); }
  const int ax = k / 2, ay = k / 2;
  const bool dft = k * k >= 130;
  std::vector<uint8_t> blurred((size_t)H * W);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      int v;
      if (dft) {
        long S = 0;
        for (size_t t = 0; t < ty.size(); ++t) S += img[(size_t)refl101(y + ty[t] - ay, H) * W + refl101(x + tx[t] - ax, W)];
        long q = S / k, r = S % k;
        if (2 * r > k || (2 * r == k && (q & 1))) ++q;
        v = (int)q;
      } else {
        float s = 0.f;
        for (size_t t = 0; t < ty.size(); ++t)
          s = std::fma((float)img[(size_t)refl101(y + ty[t] - ay, H) * W + refl101(x + tx[t] - ax, W)], tw[t], s);
        v = (int)std::nearbyint(s);
      }
      blurred[(size_t)y * W + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
  std::memset(mask, 0, (size_t)H * W);
  const int h = k / 2;
  for (int i = 0; i < n_centers; ++i) {
    const int y = centers[i] / W, x = centers[i] % W;
    for (int yy = std::max(0, y - h); yy < std::min(H, y + h + 1); ++yy)
      for (int xx = std::max(0, x - h); xx < std::min(W, x + h + 1); ++xx) mask[(size_t)yy * W + xx] = 1;
  }
  for (size_t p = 0; p < (size_t)H * W; ++p) out[p] = mask[p] ? blurred[p] : img[p];
}

}  // extern "C"
