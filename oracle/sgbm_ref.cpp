// ORACLE — test infrastructure only. Never linked into the product.
//
// Restates the disparity the reference computes at ros_ws/src/stereo_slam.py:108-117:
//   cv2.StereoSGBM_create(numDisparities=96, minDisparity=0, blockSize=7, P1=392, P2=1568,
//                         mode=cv2.STEREO_SGBM_MODE_SGBM_3WAY).compute(prevL, prevR)
// i.e. OpenCV 4.x StereoSGBMImpl::compute -> computeDisparity3WaySGBM(nstripes = 4)
// -> medianBlur(disp, 3).  Defaults: disp12MaxDiff 0 -> 1, preFilterCap 0 -> ftzero 15,
// uniquenessRatio 0 (check off), speckleWindowSize 0 (no speckle filter).
// Per stripe s (stripe_sz = ceil(H/4), overlap = blockSize/2 + 1 + ceil(0.1*stripe_sz)):
//   * Birchfield-Tomasi pixel cost on (a) the x-Sobel response clipped to [-15,15]
//     (+15) and (b) raw intensity >> 2; the two outer columns of both planes read 15;
//   * 7x7 box sum with clamped (replicated) rows/columns; rows clamp at the stripe's
//     first processed row, not at image row 0;
//   * three aggregation paths: left->right, right->left, top->down (reset per stripe);
//   * WTA (first minimum), parabolic sub-pixel step in integers, pseudo L/R check
//     against a right-view disparity accumulated from the same cost sums.
// Parity vs OpenCV: UNPINNED.  int16 output, disparity*16,
// invalid = (minDisparity-1)*16.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>

namespace {

typedef short Cost;

struct SgbmParams {
  int minD = 0, numD = 96, block = 7, P1 = 392, P2 = 1568, nstripes = 4;
  int disp12MaxDiff = 1, ftzero = 15;
};

// calcPixelCostBT for one row, cost[x1*D + d], x1 in [0,width1).
static void pixel_cost_bt(const uint8_t* L, const uint8_t* R, int H, int W, int stride, int y,
                          const SgbmParams& p, std::vector<Cost>& cost) {
  const int minD = p.minD, maxD = p.minD + p.numD, D = p.numD;
  const int minX1 = std::max(maxD, 0), maxX1 = W + std::min(minD, 0), width1 = maxX1 - minX1;
  cost.assign((size_t)width1 * D, 0);
  auto clip = [&](int v) { return std::min(std::max(v, -p.ftzero), p.ftzero) + p.ftzero; };
  std::vector<int> a[2], b[2];  // a: left planes, b: right planes (natural x order)
  for (int c = 0; c < 2; ++c) { a[c].assign(W, clip(0)); b[c].assign(W, clip(0)); }
  const uint8_t* r1 = L + (size_t)y * stride;
  const uint8_t* r2 = R + (size_t)y * stride;
  const uint8_t* n1 = L + (size_t)(y > 0 ? y - 1 : y) * stride;
  const uint8_t* s1 = L + (size_t)(y < H - 1 ? y + 1 : y) * stride;
  const uint8_t* n2 = R + (size_t)(y > 0 ? y - 1 : y) * stride;
  const uint8_t* s2 = R + (size_t)(y < H - 1 ? y + 1 : y) * stride;
  for (int x = 1; x < W - 1; ++x) {
    a[0][x] = clip((r1[x + 1] - r1[x - 1]) * 2 + n1[x + 1] - n1[x - 1] + s1[x + 1] - s1[x - 1]);
    b[0][x] = clip((r2[x + 1] - r2[x - 1]) * 2 + n2[x + 1] - n2[x - 1] + s2[x + 1] - s2[x - 1]);
    a[1][x] = r1[x];
    b[1][x] = r2[x];
  }
  for (int c = 0; c < 2; ++c) {
    const int diff_scale = c == 0 ? 0 : 2;
    std::vector<int> v0(W), v1(W);
    for (int x = 0; x < W; ++x) {
      int v = b[c][x];
      int vl = x > 0 ? (v + b[c][x - 1]) / 2 : v;
      int vr = x < W - 1 ? (v + b[c][x + 1]) / 2 : v;
      v0[x] = std::min(std::min(vl, vr), v);
      v1[x] = std::max(std::max(vl, vr), v);
    }
    for (int x = minX1; x < maxX1; ++x) {
      int u = a[c][x];
      int ul = x > 0 ? (u + a[c][x - 1]) / 2 : u;
      int ur = x < W - 1 ? (u + a[c][x + 1]) / 2 : u;
      int u0 = std::min(std::min(ul, ur), u), u1 = std::max(std::max(ul, ur), u);
      for (int d = minD; d < maxD; ++d) {
        int xr = x - d;
        int v = b[c][xr], vv0 = v0[xr], vv1 = v1[xr];
        int c0 = std::max(0, u - vv1); c0 = std::max(c0, vv0 - u);
        int c1 = std::max(0, v - u1); c1 = std::max(c1, u0 - v);
        Cost& o = cost[(size_t)(x - minX1) * D + (d - minD)];
        o = (Cost)(o + (std::min(c0, c1) >> diff_scale));
      }
    }
  }
}

static inline Cost sat(int v) { return (Cost)std::min(std::max(v, (int)SHRT_MIN), (int)SHRT_MAX); }

static void sgbm_3way(const uint8_t* L, const uint8_t* R, int H, int W, int stride, const SgbmParams& p,
                      int16_t* disp) {
  const int DISP_SHIFT = 4, DISP_SCALE = 1 << DISP_SHIFT;
  const int minD = p.minD, maxD = p.minD + p.numD, D = p.numD;
  const int minX1 = std::max(maxD, 0), maxX1 = W + std::min(minD, 0), width1 = maxX1 - minX1;
  const int SW2 = p.block / 2, SH2 = p.block / 2;
  const int INVALID = (minD - 1) * DISP_SCALE;
  const int P1 = p.P1, P2 = std::max(p.P2, p.P1 + 1);
  const int ss = (int)std::ceil(H / (double)p.nstripes);
  const int ov = (p.block / 2 + 1) + (int)std::ceil(0.1 * ss);

  // hsum per image row (x-window clamped): independent of the stripe.
  std::vector<std::vector<Cost>> hsum(H);
  {
    std::vector<Cost> pd;
    for (int y = 0; y < H; ++y) {
      pixel_cost_bt(L, R, H, W, stride, y, p, pd);
      hsum[y].assign((size_t)width1 * D, 0);
      for (int x1 = 0; x1 < width1; ++x1)
        for (int d = 0; d < D; ++d) {
          int s = 0;
          for (int c = x1 - SW2; c <= x1 + SW2; ++c) s += pd[(size_t)std::min(std::max(c, 0), width1 - 1) * D + d];
          hsum[y][(size_t)x1 * D + d] = (Cost)s;
        }
    }
  }
  for (int i = 0; i < H * W; ++i) disp[i] = (int16_t)INVALID;

  std::vector<Cost> C((size_t)width1 * D), Lh((size_t)width1 * D), V((size_t)width1 * D), Rb(D), Rn(D), Lprev(D);
  std::vector<int> vmin(width1);
  std::vector<int16_t> drow(W), disp2(W);
  std::vector<int> disp2cost(W);
  for (int s = 0; s < p.nstripes; ++s) {
    int start = std::max(std::min(s * ss - ov, H), 0);
    int end = std::min((s + 1) * ss, H);
    int first_out = std::min(s * ss, H);
    std::fill(V.begin(), V.end(), 0);
    std::fill(vmin.begin(), vmin.end(), 0);
    for (int y = start; y < end; ++y) {
      for (size_t i = 0; i < C.size(); ++i) {
        int acc = 0;
        for (int r = y - SH2; r <= y + SH2; ++r) acc += hsum[std::min(std::max(r, start), H - 1)][i];
        C[i] = (Cost)acc;
      }
      for (int x = 0; x < W; ++x) { disp2[x] = (int16_t)INVALID; disp2cost[x] = SHRT_MAX; drow[x] = (int16_t)INVALID; }
      // forward: left->right and top->down
      int leftMin = 0;
      for (int x1 = 0; x1 < width1; ++x1) {
        const Cost* c = &C[(size_t)x1 * D];
        Cost* lb = &Lh[(size_t)x1 * D];
        if (x1 == 0) std::fill(Lprev.begin(), Lprev.end(), 0);
        else std::copy(&Lh[(size_t)(x1 - 1) * D], &Lh[(size_t)x1 * D], Lprev.begin());
        int newMin = SHRT_MAX;
        for (int d = 0; d < D; ++d) {
          int m = Lprev[d];
          m = std::min(m, leftMin + P2);
          if (d > 0) m = std::min(m, Lprev[d - 1] + P1);
          if (d < D - 1) m = std::min(m, Lprev[d + 1] + P1);
          lb[d] = sat(c[d] + m - leftMin);
          newMin = std::min(newMin, (int)lb[d]);
        }
        leftMin = newMin;
        Cost* vb = &V[(size_t)x1 * D];
        std::copy(vb, vb + D, Rn.begin());  // old V(y-1)
        int topMin = vmin[x1], newTop = SHRT_MAX;
        for (int d = 0; d < D; ++d) {
          int m = Rn[d];
          m = std::min(m, topMin + P2);
          if (d > 0) m = std::min(m, Rn[d - 1] + P1);
          if (d < D - 1) m = std::min(m, Rn[d + 1] + P1);
          vb[d] = sat(c[d] + m - topMin);
          newTop = std::min(newTop, (int)vb[d]);
        }
        vmin[x1] = newTop;
      }
      // backward: right->left, sum, WTA, sub-pixel, disp2
      std::fill(Rb.begin(), Rb.end(), 0);
      int rightMin = 0;
      for (int x1 = width1 - 1; x1 >= 0; --x1) {
        const Cost* c = &C[(size_t)x1 * D];
        Cost* S = &Lh[(size_t)x1 * D];
        const Cost* vb = &V[(size_t)x1 * D];
        int newMin = SHRT_MAX, minCost = SHRT_MAX, best = 0;
        for (int d = 0; d < D; ++d) {
          int m = Rb[d];
          m = std::min(m, rightMin + P2);
          if (d > 0) m = std::min(m, Rb[d - 1] + P1);
          if (d < D - 1) m = std::min(m, Rb[d + 1] + P1);
          Rn[d] = sat(c[d] + m - rightMin);
          newMin = std::min(newMin, (int)Rn[d]);
        }
        for (int d = 0; d < D; ++d) {
          Rb[d] = Rn[d];
          S[d] = sat((int)S[d] + Rb[d] + vb[d]);
          if (S[d] < minCost) { minCost = S[d]; best = d; }
        }
        rightMin = newMin;
        int d = best;
        int x2 = x1 + minX1 - d - minD;
        if (x2 >= 0 && x2 < W && disp2cost[x2] > minCost) { disp2cost[x2] = minCost; disp2[x2] = (int16_t)(d + minD); }
        int dd;
        if (0 < d && d < D - 1) {
          int denom2 = std::max(S[d - 1] + S[d + 1] - 2 * S[d], 1);
          dd = d * DISP_SCALE + ((S[d - 1] - S[d + 1]) * DISP_SCALE + denom2) / (denom2 * 2);
        } else {
          dd = d * DISP_SCALE;
        }
        drow[x1 + minX1] = (int16_t)(dd + minD * DISP_SCALE);
      }
      for (int x = minX1; x < maxX1; ++x) {
        int d1 = drow[x];
        if (d1 == INVALID) continue;
        int _d = d1 >> DISP_SHIFT, d_ = (d1 + DISP_SCALE - 1) >> DISP_SHIFT;
        int _x = x - _d, x_ = x - d_;
        if (0 <= x_ && x_ < W && disp2[x_] >= minD && std::abs(disp2[x_] - d_) > p.disp12MaxDiff && 0 <= _x &&
            _x < W && disp2[_x] >= minD && std::abs(disp2[_x] - _d) > p.disp12MaxDiff)
          drow[x] = (int16_t)INVALID;
      }
      if (y >= first_out)
        for (int x = 0; x < W; ++x) disp[(size_t)y * W + x] = drow[x];
    }
  }
}

static void median3_s16(const int16_t* src, int16_t* dst, int H, int W) {
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      int16_t v[9];
      int k = 0;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          int yy = std::min(std::max(y + dy, 0), H - 1), xx = std::min(std::max(x + dx, 0), W - 1);
          v[k++] = src[(size_t)yy * W + xx];
        }
      std::nth_element(v, v + 4, v + 9);
      dst[(size_t)y * W + x] = v[4];
    }
}

}  // namespace

extern "C" {

// StereoSGBM(3-way).compute(L, R) incl. the final 3x3 median.  disp_out: int16 [H*W].
// raw_out (optional): the disparity before the median filter.
void ref_sgbm(const uint8_t* L, const uint8_t* R, int H, int W, int stride, int minD, int numD, int block, int P1,
              int P2, int16_t* disp_out, int16_t* raw_out) {
  SgbmParams p;
  p.minD = minD; p.numD = numD; p.block = block; p.P1 = P1; p.P2 = P2;
  std::vector<int16_t> raw((size_t)H * W);
  sgbm_3way(L, R, H, W, stride, p, raw.data());
  if (raw_out) std::copy(raw.begin(), raw.end(), raw_out);
  median3_s16(raw.data(), disp_out, H, W);
}

// pixel cost + hsum for one row (debug / parity of the first kernel stage).
void ref_sgbm_row_cost(const uint8_t* L, const uint8_t* R, int H, int W, int stride, int y, int numD,
                       int16_t* pixdiff_out) {
  SgbmParams p;
  p.numD = numD;
  std::vector<Cost> c;
  pixel_cost_bt(L, R, H, W, stride, y, p, c);
  std::copy(c.begin(), c.end(), pixdiff_out);
}

}  // extern "C"
