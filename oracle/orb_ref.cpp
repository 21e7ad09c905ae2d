// ORACLE — test infrastructure only. Never linked into the product (forest-slam_amd/).
//
// Scalar C++ restatement of the ORB path the reference calls at
//   ros_ws/src/stereo_slam.py:84       orb = cv2.ORB_create()            (all defaults)
//   ros_ws/src/stereo_slam.py:232-233  orb.detectAndCompute(img, None)
// The arithmetic lives in OpenCV 4.x (features2d/src/orb.cpp, fast.cpp, keypoint.cpp,
// imgproc resize/filter), which is NOT present in this container; this file restates
// the semantics recalled in SURVEY.md Appendix A plus the corrections listed in
// DESIGN.md §Oracle.  Parity status vs OpenCV: UNPINNED (no golden vectors for this
// stage exist in the reference).  What IS pinned: the GPU product is
// compared bit-for-bit against this file.
//
// Compile with -ffp-contract=off (OpenCV's baseline x86-64 build has no FMA in these
// translation units), so every float expression below rounds exactly as written.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orb_pattern_ref.inc"

namespace ref {

struct KP {
  float x, y, size, angle, response;
  int octave;
};

static inline int cv_round(double v) { return (int)std::lrint(v); }  // half-to-even
static inline int cv_roundf(float v) { return (int)std::lrintf(v); }
static inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil(double v) { int i = (int)v; return i + (i < v); }

struct Plane {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
  uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
  uint8_t& at(int x, int y) { return px[(size_t)y * w + x]; }
};

// ---------------------------------------------------------------- pyramid
// OpenCV: getScale() = (float)pow(scaleFactor, level) with scaleFactor = (double)1.2f,
// level size = cvRound(cols * (1.f/scale)) (orb.cpp detectAndCompute).
static float level_scale(int level, double scale_factor) {
  return (float)std::pow(scale_factor, (double)level);
}

// resize(..., INTER_LINEAR_EXACT): ufixedpoint16 (8-bit) coefficients,
// horizontal pass -> 8 frac bits, vertical pass -> 16 frac bits, round-half-up.
// Source coordinate fval = (1/inv_scale)*(d+0.5)-0.5 in double; fval<0 clamps to
// the first sample, ival>=src-1 clamps to the last sample.
struct LinCoef {
  std::vector<int> ofs;   // -1: left clamp, -2: right clamp
  std::vector<int> c0, c1;
};
static LinCoef linear_coeffs(int src, int dst) {
  LinCoef r;
  r.ofs.resize(dst); r.c0.resize(dst); r.c1.resize(dst);
  double inv_scale = (double)dst / (double)src;
  double scale = 1.0 / inv_scale;
  for (int d = 0; d < dst; ++d) {
    double fval = scale * ((double)d + 0.5) - 0.5;
    int ival = cv_floor(fval);
    if (ival >= 0 && src > 1) {
      if (ival < src - 1) {
        double frac = fval - (double)ival;
        int c1 = frac < 0 ? 0 : (int)std::llrint(frac * 256.0);
        r.ofs[d] = ival; r.c1[d] = c1; r.c0[d] = 256 - c1;
      } else {
        r.ofs[d] = -2; r.c0[d] = 256; r.c1[d] = 0;
      }
    } else {
      r.ofs[d] = -1; r.c0[d] = 256; r.c1[d] = 0;
    }
  }
  return r;
}

static void resize_linear_exact(const Plane& s, Plane& d) {
  LinCoef cx = linear_coeffs(s.w, d.w), cy = linear_coeffs(s.h, d.h);
  auto hrow = [&](int r, std::vector<uint32_t>& out) {
    out.resize(d.w);
    for (int x = 0; x < d.w; ++x) {
      int o = cx.ofs[x];
      if (o == -1) out[x] = (uint32_t)s.at(0, r) << 8;
      else if (o == -2) out[x] = (uint32_t)s.at(s.w - 1, r) << 8;
      else out[x] = (uint32_t)cx.c0[x] * s.at(o, r) + (uint32_t)cx.c1[x] * s.at(o + 1, r);
    }
  };
  std::vector<uint32_t> h0, h1;
  for (int y = 0; y < d.h; ++y) {
    int o = cy.ofs[y];
    if (o == -1 || o == -2) {
      hrow(o == -1 ? 0 : s.h - 1, h0);
      for (int x = 0; x < d.w; ++x) d.at(x, y) = (uint8_t)std::min<uint32_t>(255, (h0[x] + 128) >> 8);
    } else {
      hrow(o, h0); hrow(o + 1, h1);
      for (int x = 0; x < d.w; ++x) {
        uint32_t v = h0[x] * (uint32_t)cy.c0[y] + h1[x] * (uint32_t)cy.c1[y];
        d.at(x, y) = (uint8_t)std::min<uint32_t>(255, (v + 32768u) >> 16);
      }
    }
  }
}

// ---------------------------------------------------------------- FAST-9/16
static const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                   {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// cornerScore<16> (fast_score.cpp), scalar form.
static int corner_score(const Plane& im, int x, int y, int threshold) {
  int v = im.at(x, y);
  short d[25];
  for (int k = 0; k < 25; ++k) d[k] = (short)(v - im.at(x + kCircle[k % 16][0], y + kCircle[k % 16][1]));
  int a0 = threshold;
  for (int k = 0; k < 16; k += 2) {
    int a = std::min((int)d[k + 1], (int)d[k + 2]);
    a = std::min(a, (int)d[k + 3]);
    if (a <= a0) continue;
    for (int j = 4; j <= 8; ++j) a = std::min(a, (int)d[k + j]);
    a0 = std::max(a0, std::min(a, (int)d[k]));
    a0 = std::max(a0, std::min(a, (int)d[k + 9]));
  }
  int b0 = -a0;
  for (int k = 0; k < 16; k += 2) {
    int b = std::max((int)d[k + 1], (int)d[k + 2]);
    b = std::max(b, (int)d[k + 3]);
    b = std::max(b, (int)d[k + 4]);
    b = std::max(b, (int)d[k + 5]);
    if (b >= b0) continue;
    b = std::max(b, (int)d[k + 6]);
    b = std::max(b, (int)d[k + 7]);
    b = std::max(b, (int)d[k + 8]);
    b0 = std::min(b0, std::max(b, (int)d[k]));
    b0 = std::min(b0, std::max(b, (int)d[k + 9]));
  }
  return -b0 - 1;
}

// FAST_t<16> (fast.cpp): corner if >=9 contiguous circle pixels are all > v+t or
// all < v-t; score map is 0 off-corner and outside [3,w-4]x[3,h-4]; 3x3 NMS with
// strict '>' against all 8 neighbours; emission row-major.
static void fast_score_map(const Plane& im, int threshold, std::vector<uint8_t>& score) {
  score.assign((size_t)im.w * im.h, 0);
  for (int y = 3; y < im.h - 3; ++y)
    for (int x = 3; x < im.w - 3; ++x) {
      int v = im.at(x, y);
      int p[25];
      for (int k = 0; k < 25; ++k) p[k] = im.at(x + kCircle[k % 16][0], y + kCircle[k % 16][1]);
      bool corner = false;
      int cnt = 0;
      for (int k = 0; k < 25 && !corner; ++k) {
        if (p[k] < v - threshold) { if (++cnt > 8) corner = true; } else cnt = 0;
      }
      cnt = 0;
      for (int k = 0; k < 25 && !corner; ++k) {
        if (p[k] > v + threshold) { if (++cnt > 8) corner = true; } else cnt = 0;
      }
      if (corner) score[(size_t)y * im.w + x] = (uint8_t)corner_score(im, x, y, threshold);
    }
}

static void fast_detect(const Plane& im, int threshold, std::vector<KP>& kps) {
  std::vector<uint8_t> s;
  fast_score_map(im, threshold, s);
  kps.clear();
  for (int y = 3; y < im.h - 3; ++y)
    for (int x = 3; x < im.w - 3; ++x) {
      int sc = s[(size_t)y * im.w + x];
      if (!sc) continue;
      bool keep = true;
      for (int dy = -1; dy <= 1 && keep; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dx && !dy) continue;
          if (!(sc > s[(size_t)(y + dy) * im.w + x + dx])) { keep = false; break; }
        }
      if (keep) kps.push_back(KP{(float)x, (float)y, 7.f, -1.f, (float)sc, 0});
    }
}

// KeyPointsFilter::runByImageBorder: keep border <= x < w-border (same for y); order kept.
static void run_by_image_border(std::vector<KP>& k, int w, int h, int border) {
  if (h <= 2 * border || w <= 2 * border) { k.clear(); return; }
  std::vector<KP> o;
  for (auto& p : k)
    if (p.x >= border && p.x < w - border && p.y >= border && p.y < h - border) o.push_back(p);
  k.swap(o);
}

// KeyPointsFilter::retainBest: nth_element(greater-by-response) at n-1, then
// partition the tail keeping responses >= the boundary response.  Uses the host
// libstdc++ algorithms on purpose: their element order is what OpenCV emits.
static void retain_best(std::vector<KP>& k, int n) {
  if (n >= 0 && k.size() > (size_t)n) {
    if (n == 0) { k.clear(); return; }
    std::nth_element(k.begin(), k.begin() + n - 1, k.end(),
                     [](const KP& a, const KP& b) { return a.response > b.response; });
    float amb = k[n - 1].response;
    auto e = std::partition(k.begin() + n, k.end(), [amb](const KP& a) { return a.response >= amb; });
    k.resize(e - k.begin());
  }
}

// HarrisResponses (orb.cpp), blockSize 7, k = 0.04f, float expression order kept.
static void harris_responses(const std::vector<Plane>& lv, std::vector<KP>& pts) {
  const int bs = 7, r = bs / 2;
  const float harris_k = 0.04f;
  float scale = 1.f / ((1 << 2) * bs * 255.f);
  float scale_sq_sq = scale * scale * scale * scale;
  for (auto& p : pts) {
    const Plane& im = lv[p.octave];
    int x0 = cv_roundf(p.x), y0 = cv_roundf(p.y);
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < bs; ++i)
      for (int j = 0; j < bs; ++j) {
        int x = x0 - r + j, y = y0 - r + i;
        int Ix = (im.at(x + 1, y) - im.at(x - 1, y)) * 2 + (im.at(x + 1, y - 1) - im.at(x - 1, y - 1)) +
                 (im.at(x + 1, y + 1) - im.at(x - 1, y + 1));
        int Iy = (im.at(x, y + 1) - im.at(x, y - 1)) * 2 + (im.at(x - 1, y + 1) - im.at(x - 1, y - 1)) +
                 (im.at(x + 1, y + 1) - im.at(x + 1, y - 1));
        a += Ix * Ix; b += Iy * Iy; c += Ix * Iy;
      }
    p.response = ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
  }
}

// cv::fastAtan2 (float polynomial, degrees).
static float fast_atan2(float y, float x) {
  const float k = (float)(180 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k, p5 = 0.1555786518463281f * k,
              p7 = -0.04432655554792128f * k;
  const float eps = (float)2.220446049250313080847e-16;
  float ax = std::fabs(x), ay = std::fabs(y), a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps); c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps); c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

static std::vector<int> make_umax(int half) {
  std::vector<int> umax(half + 2);
  int vmax = cv_floor(half * std::sqrt(2.f) / 2 + 1);
  int vmin = cv_ceil(half * std::sqrt(2.f) / 2);
  for (int v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt((double)half * half - v * v));
  for (int v = half, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
  return umax;
}

static void ic_angles(const std::vector<Plane>& lv, std::vector<KP>& pts, const std::vector<int>& umax, int half) {
  for (auto& p : pts) {
    const Plane& im = lv[p.octave];
    int cx = cv_roundf(p.x), cy = cv_roundf(p.y);
    int m01 = 0, m10 = 0;
    for (int u = -half; u <= half; ++u) m10 += u * im.at(cx + u, cy);
    for (int v = 1; v <= half; ++v) {
      int vs = 0, d = umax[v];
      for (int u = -d; u <= d; ++u) {
        int vp = im.at(cx + u, cy + v), vm = im.at(cx + u, cy - v);
        vs += vp - vm;
        m10 += u * (vp + vm);
      }
      m01 += v * vs;
    }
    p.angle = fast_atan2((float)m01, (float)m10);
  }
}

// GaussianBlur(level ROI, 7x7, sigma 2, REFLECT_101) on an 8U submatrix goes through
// sepFilter2D's 8-bit fixed-point path: kernel round(k*256) = [18 34 49 55 49 34 18],
// int row sums, column sum of int products, result (s + 2^15) >> 16 saturated.
// NOTE: OpenCV's SIMD column filter (SymmColumnVec_32s8u) rounds ties to even; ties
// (s mod 2^16 == 2^15) are resolved half-to-even here, see DESIGN.md §Oracle.
static const int kGauss7[7] = {18, 34, 49, 55, 49, 34, 18};
static inline int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) { if (i < 0) i = -i; if (i >= n) i = 2 * n - 2 - i; }
  return i;
}
static void gaussian_blur7(Plane& im) {
  std::vector<int> rows((size_t)im.w * im.h);
  for (int y = 0; y < im.h; ++y)
    for (int x = 0; x < im.w; ++x) {
      int s = 0;
      for (int k = -3; k <= 3; ++k) s += kGauss7[k + 3] * im.at(reflect101(x + k, im.w), y);
      rows[(size_t)y * im.w + x] = s;
    }
  for (int y = 0; y < im.h; ++y)
    for (int x = 0; x < im.w; ++x) {
      int s = 0;
      for (int k = -3; k <= 3; ++k) s += kGauss7[k + 3] * rows[(size_t)reflect101(y + k, im.h) * im.w + x];
      int q = (s + 32767 + ((s >> 16) & 1)) >> 16;  // round half to even
      im.at(x, y) = (uint8_t)std::min(255, std::max(0, q));
    }
}

static void compute_descriptors(const std::vector<Plane>& blurred, const std::vector<float>& lscale,
                                const std::vector<KP>& kps, uint8_t* desc) {
  for (size_t j = 0; j < kps.size(); ++j) {
    const KP& k = kps[j];
    const Plane& im = blurred[k.octave];
    float scale = 1.f / lscale[k.octave];
    float angle = k.angle;
    angle *= (float)(3.14159265358979323846 / 180.f);
    float a = (float)std::cos((double)angle), b = (float)std::sin((double)angle);
    int cy = cv_roundf(k.y * scale), cx = cv_roundf(k.x * scale);
    auto val = [&](int idx) -> int {
      int px = FVO_ORB_PATTERN[(idx >> 1) * 4 + (idx & 1) * 2 + 0];
      int py = FVO_ORB_PATTERN[(idx >> 1) * 4 + (idx & 1) * 2 + 1];
      float x = px * a - py * b;
      float y = px * b + py * a;
      int ix = cv_roundf(x), iy = cv_roundf(y);
      return im.at(cx + ix, cy + iy);
    };
    for (int i = 0; i < 32; ++i) {
      int v = 0;
      for (int bit = 0; bit < 8; ++bit) {
        int p = i * 16 + bit * 2;
        v |= (val(p) < val(p + 1)) << bit;
      }
      desc[j * 32 + i] = (uint8_t)v;
    }
  }
}

struct OrbParams {
  int nfeatures = 500;
  double scale_factor = (double)1.2f;
  int nlevels = 8;
  int edge_threshold = 31;
  int patch_size = 31;
  int fast_threshold = 20;
};

static void build_pyramid(const uint8_t* img, int H, int W, int stride, const OrbParams& P,
                          std::vector<Plane>& lv, std::vector<float>& lscale) {
  lv.assign(P.nlevels, Plane());
  lscale.assign(P.nlevels, 1.f);
  for (int l = 0; l < P.nlevels; ++l) {
    float s = level_scale(l, P.scale_factor);
    lscale[l] = s;
    float inv = 1.0f / s;
    lv[l].w = cv_roundf(W * inv);
    lv[l].h = cv_roundf(H * inv);
    lv[l].px.resize((size_t)lv[l].w * lv[l].h);
    if (l == 0) {
      for (int y = 0; y < H; ++y) std::memcpy(&lv[0].px[(size_t)y * W], img + (size_t)y * stride, W);
    } else {
      resize_linear_exact(lv[l - 1], lv[l]);
    }
  }
}

static std::vector<int> features_per_level(const OrbParams& P) {
  std::vector<int> n(P.nlevels);
  float factor = (float)(1.0 / P.scale_factor);
  float nd = P.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)P.nlevels));
  int sum = 0;
  for (int l = 0; l < P.nlevels - 1; ++l) {
    n[l] = cv_roundf(nd);
    sum += n[l];
    nd *= factor;
  }
  n[P.nlevels - 1] = std::max(P.nfeatures - sum, 0);
  return n;
}

static void compute_keypoints(const std::vector<Plane>& lv, const std::vector<float>& lscale, const OrbParams& P,
                              std::vector<KP>& all) {
  std::vector<int> nper = features_per_level(P);
  const int half = P.patch_size / 2;
  std::vector<int> umax = make_umax(half);
  all.clear();
  std::vector<int> counters(P.nlevels);
  for (int l = 0; l < P.nlevels; ++l) {
    std::vector<KP> k;
    fast_detect(lv[l], P.fast_threshold, k);
    run_by_image_border(k, lv[l].w, lv[l].h, P.edge_threshold);
    retain_best(k, 2 * nper[l]);
    counters[l] = (int)k.size();
    for (auto& p : k) { p.octave = l; p.size = P.patch_size * lscale[l]; }
    all.insert(all.end(), k.begin(), k.end());
  }
  if (all.empty()) return;
  harris_responses(lv, all);
  std::vector<KP> out;
  size_t off = 0;
  for (int l = 0; l < P.nlevels; ++l) {
    std::vector<KP> k(all.begin() + off, all.begin() + off + counters[l]);
    off += counters[l];
    retain_best(k, nper[l]);
    out.insert(out.end(), k.begin(), k.end());
  }
  all.swap(out);
  ic_angles(lv, all, umax, half);
  for (auto& p : all) {
    float s = lscale[p.octave];
    p.x *= s;
    p.y *= s;
  }
}

}  // namespace ref

extern "C" {

// Full ORB detectAndCompute.  kp_out rows: x, y, size, angle, response, octave.
// Returns the keypoint count, or -(count) if it exceeds cap (nothing written).
int ref_orb_detect_compute(const uint8_t* img, int H, int W, int stride, int nfeatures, int fast_threshold,
                           float* kp_out, uint8_t* desc_out, int cap) {
  ref::OrbParams P;
  P.nfeatures = nfeatures;
  P.fast_threshold = std::min(std::max(fast_threshold, 0), 255);
  std::vector<ref::Plane> lv;
  std::vector<float> ls;
  ref::build_pyramid(img, H, W, stride, P, lv, ls);
  std::vector<ref::KP> kps;
  ref::compute_keypoints(lv, ls, P, kps);
  int n = (int)kps.size();
  if (n > cap) return -n;
  for (auto& p : lv) ref::gaussian_blur7(p);
  ref::compute_descriptors(lv, ls, kps, desc_out);
  for (int i = 0; i < n; ++i) {
    float* o = kp_out + 6 * i;
    o[0] = kps[i].x; o[1] = kps[i].y; o[2] = kps[i].size; o[3] = kps[i].angle; o[4] = kps[i].response;
    o[5] = (float)kps[i].octave;
  }
  return n;
}

// Pyramid levels packed back to back (level l at offset sum_{k<l} w_k*h_k).
// sizes_out gets (w,h) per level.  Returns total bytes.
int ref_orb_pyramid(const uint8_t* img, int H, int W, int stride, int nlevels, uint8_t* out, int32_t* sizes_out,
                    int blurred) {
  ref::OrbParams P;
  P.nlevels = nlevels;
  std::vector<ref::Plane> lv;
  std::vector<float> ls;
  ref::build_pyramid(img, H, W, stride, P, lv, ls);
  size_t off = 0;
  for (int l = 0; l < nlevels; ++l) {
    if (blurred) ref::gaussian_blur7(lv[l]);
    sizes_out[2 * l] = lv[l].w;
    sizes_out[2 * l + 1] = lv[l].h;
    if (out) std::memcpy(out + off, lv[l].px.data(), lv[l].px.size());
    off += lv[l].px.size();
  }
  return (int)off;
}

// FAST score map (0 off-corner) for one plane.
void ref_fast_score_map(const uint8_t* img, int H, int W, int stride, int threshold, uint8_t* score_out) {
  ref::Plane p;
  p.w = W; p.h = H; p.px.resize((size_t)W * H);
  for (int y = 0; y < H; ++y) std::memcpy(&p.px[(size_t)y * W], img + (size_t)y * stride, W);
  std::vector<uint8_t> s;
  ref::fast_score_map(p, threshold, s);
  std::memcpy(score_out, s.data(), s.size());
}

// FAST + NMS keypoints (x, y, score) in emission order.  Returns count or -count.
int ref_fast_detect(const uint8_t* img, int H, int W, int stride, int threshold, int32_t* out, int cap) {
  ref::Plane p;
  p.w = W; p.h = H; p.px.resize((size_t)W * H);
  for (int y = 0; y < H; ++y) std::memcpy(&p.px[(size_t)y * W], img + (size_t)y * stride, W);
  std::vector<ref::KP> k;
  ref::fast_detect(p, threshold, k);
  if ((int)k.size() > cap) return -(int)k.size();
  for (size_t i = 0; i < k.size(); ++i) {
    out[3 * i] = (int)k[i].x; out[3 * i + 1] = (int)k[i].y; out[3 * i + 2] = (int)k[i].response;
  }
  return (int)k.size();
}

// retainBest on an arbitrary float response list: writes the surviving original
// indices, in output order.  Returns the survivor count.
int ref_retain_best(const float* resp, int n, int keep, int32_t* idx_out) {
  std::vector<ref::KP> k(n);
  for (int i = 0; i < n; ++i) { k[i] = ref::KP{(float)i, 0.f, 0.f, 0.f, resp[i], 0}; }
  ref::retain_best(k, keep);
  for (size_t i = 0; i < k.size(); ++i) idx_out[i] = (int)k[i].x;
  return (int)k.size();
}

float ref_fast_atan2(float y, float x) { return ref::fast_atan2(y, x); }

void ref_features_per_level(int nfeatures, int nlevels, int32_t* out) {
  ref::OrbParams P;
  P.nfeatures = nfeatures;
  P.nlevels = nlevels;
  auto v = ref::features_per_level(P);
  for (int i = 0; i < nlevels; ++i) out[i] = v[i];
}

}  // extern "C"
