// ORACLE — test infrastructure only. Never linked into the product.
//
// Restates the pose step of ros_ws/src/stereo_slam.py:292-306:
//   cv2.solvePnPRansac(points3D, mkpts1_l, K0, dist_coeffs_l, reprojectionError=1.0,
//                      confidence=0.99, iterationsCount=1000, flags=cv2.SOLVEPNP_ITERATIVE)
//   cv2.Rodrigues(rvec) -> T -> cumulative = cumulative @ T
// following OpenCV 4.x (calib3d/src/solvepnp.cpp, ptsetreg.cpp, epnp.cpp, calibration.cpp,
// undistort.dispatch.cpp) as restated in SURVEY.md Appendix A and DESIGN.md §Oracle:
//   * object points are cast to float32 before RANSAC (opoints.depth()==CV_64F -> CV_32F);
//   * RNG(-1) multiply-with-carry, 5-point subsets of distinct indices;
//   * hypothesis = EPnP on undistortPoints()-normalised (float32) image points;
//   * score = float squared reprojection error (projectPoints with k1,k2,p1,p2,k3),
//     inlier iff err <= 1.0f; accept iff goodCount > max(best, 4); adaptive niters;
//   * refinement = solvePnP(inliers, useExtrinsicGuess=false, ITERATIVE): DLT init
//     (homography init for planar sets), then CvLevMarq, 20 iterations, eps FLT_EPSILON;
//     if exactly 5 inliers the DLT would throw and the RANSAC model is returned.
// Any accurate SVD is used in place of OpenCV's JacobiSVD: the quantities consumed are
// sign/rotation invariant, so results agree to ~1e-12 relative, well inside the 1e-4
// pose tolerance of BASELINE.json.  Parity vs OpenCV: UNPINNED.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace pnp {

// ------------------------------------------------------------------ linear algebra
// A (m x n, row-major, m >= n) = U diag(W) V^T; W descending; U m x n, V n x n.
static void svd(const double* A, int m, int n, double* W, double* U, double* V) {
  std::vector<double> u(A, A + (size_t)m * n), v((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i) v[(size_t)i * n + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        double a = 0, b = 0, g = 0;
        for (int i = 0; i < m; ++i) {
          double up = u[(size_t)i * n + p], uq = u[(size_t)i * n + q];
          a += up * up; b += uq * uq; g += up * uq;
        }
        if (g == 0.0 || std::fabs(g) <= 1e-300) continue;
        double rel = std::fabs(g) / std::sqrt(a * b);
        off = std::max(off, rel);
        if (rel < 1e-15) continue;
        double zeta = (b - a) / (2.0 * g);
        double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
        double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
        for (int i = 0; i < m; ++i) {
          double up = u[(size_t)i * n + p], uq = u[(size_t)i * n + q];
          u[(size_t)i * n + p] = c * up - s * uq;
          u[(size_t)i * n + q] = s * up + c * uq;
        }
        for (int i = 0; i < n; ++i) {
          double vp = v[(size_t)i * n + p], vq = v[(size_t)i * n + q];
          v[(size_t)i * n + p] = c * vp - s * vq;
          v[(size_t)i * n + q] = s * vp + c * vq;
        }
      }
    if (off < 1e-15) break;
  }
  std::vector<double> w(n);
  for (int j = 0; j < n; ++j) {
    double s = 0;
    for (int i = 0; i < m; ++i) s += u[(size_t)i * n + j] * u[(size_t)i * n + j];
    w[j] = std::sqrt(s);
  }
  std::vector<int> ord(n);
  for (int j = 0; j < n; ++j) ord[j] = j;
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return w[a] > w[b]; });
  for (int jj = 0; jj < n; ++jj) {
    int j = ord[jj];
    W[jj] = w[j];
    double inv = w[j] > 0 ? 1.0 / w[j] : 0.0;
    for (int i = 0; i < m; ++i) U[(size_t)i * n + jj] = u[(size_t)i * n + j] * inv;
    for (int i = 0; i < n; ++i) V[(size_t)i * n + jj] = v[(size_t)i * n + j];
  }
}

// least squares / pseudo-inverse solve of A x = b (A m x n, m >= n), SVD based.
static void solve_svd(const double* A, int m, int n, const double* b, double* x) {
  std::vector<double> W(n), U((size_t)m * n), V((size_t)n * n);
  svd(A, m, n, W.data(), U.data(), V.data());
  double thr = DBL_EPSILON * std::max(m, n) * W[0];
  std::vector<double> tmp(n, 0.0);
  for (int j = 0; j < n; ++j) {
    if (W[j] <= thr) continue;
    double s = 0;
    for (int i = 0; i < m; ++i) s += U[(size_t)i * n + j] * b[i];
    tmp[j] = s / W[j];
  }
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int j = 0; j < n; ++j) s += V[(size_t)i * n + j] * tmp[j];
    x[i] = s;
  }
}

static double det3(const double* R) {
  return R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) + R[2] * (R[3] * R[7] - R[4] * R[6]);
}

// ------------------------------------------------------------------ Rodrigues
static void rodrigues_r2R(const double* r, double* R, double* J /*3x9 or null*/) {
  double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < DBL_EPSILON) {
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (J) {
      static const double J0[27] = {0, 0, 0, 0, 0, 1, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 1, 0, -1, 0, 0, 0, 0, 0};
      std::memcpy(J, J0, sizeof(J0));
    }
    return;
  }
  double c = std::cos(th), s = std::sin(th), c1 = 1.0 - c, it = th ? 1.0 / th : 0.0;
  double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int k = 0; k < 9; ++k) R[k] = c * I[k] + c1 * rrt[k] + s * rx[k];
  if (J) {
    double drrt[27] = {x + x, y, z, y, 0, 0, z, 0, 0, 0, x, 0, x, y + y, z, 0, z, 0, 0, 0, x, 0, 0, y, x, y, z + z};
    static const double drx[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 1, 0, 0, 0, 0, 0};
    for (int i = 0; i < 3; ++i) {
      double ri = i == 0 ? x : i == 1 ? y : z;
      double a0 = -s * ri, a1 = (s - 2 * c1 * it) * ri, a2 = c1 * it, a3 = (c - s * it) * ri, a4 = s * it;
      for (int k = 0; k < 9; ++k)
        J[i * 9 + k] = a0 * I[k] + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * rx[k] + a4 * drx[i * 9 + k];
    }
  }
}

static void rodrigues_R2r(const double* Rin, double* r) {
  double W[3], U[9], V[9], R[9];
  svd(Rin, 3, 3, W, U, V);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i * 3 + j] = U[i * 3 + 0] * V[j * 3 + 0] + U[i * 3 + 1] * V[j * 3 + 1] + U[i * 3 + 2] * V[j * 3 + 2];
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  double th = std::acos(c);
  if (s < 1e-5) {
    if (c > 0) { rx = ry = rz = 0; }
    else {
      double t = (R[0] + 1) * 0.5;
      rx = std::sqrt(std::max(t, 0.));
      t = (R[4] + 1) * 0.5;
      ry = std::sqrt(std::max(t, 0.)) * (R[1] < 0 ? -1. : 1.);
      t = (R[8] + 1) * 0.5;
      rz = std::sqrt(std::max(t, 0.)) * (R[2] < 0 ? -1. : 1.);
      if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
      double nn = std::sqrt(rx * rx + ry * ry + rz * rz);
      th /= nn;
      rx *= th; ry *= th; rz *= th;
    }
  } else {
    double vth = 1 / (2 * s);
    vth *= th;
    rx *= vth; ry *= vth; rz *= vth;
  }
  r[0] = rx; r[1] = ry; r[2] = rz;
}

// ------------------------------------------------------------------ camera model
struct Cam {
  double fx, fy, cx, cy;
  double k[5];  // k1 k2 p1 p2 k3
};

// cvProjectPoints2Internal for one point; optional d(u,v)/d(r,t) (2x6, row-major).
static void project(const Cam& K, const double* R, const double* dRdr, const double* t, const double* M, double* uv,
                    double* J) {
  double X = M[0], Y = M[1], Z = M[2];
  double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
  double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
  double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
  z = z ? 1. / z : 1;
  x *= z; y *= z;
  const double* k = K.k;
  double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
  double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
  double cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
  double icdist2 = 1.;
  double xd = x * cdist * icdist2 + k[2] * a1 + k[3] * a2;
  double yd = y * cdist * icdist2 + k[2] * a3 + k[3] * a1;
  uv[0] = xd * K.fx + K.cx;
  uv[1] = yd * K.fy + K.cy;
  if (!J) return;
  auto fill = [&](double dxd, double dyd, int col) {
    double dr2 = 2 * x * dxd + 2 * y * dyd;
    double dcdist = k[0] * dr2 + 2 * k[1] * r2 * dr2 + 3 * k[4] * r4 * dr2;
    double da1 = 2 * (x * dyd + y * dxd);
    double dmx = dxd * cdist * icdist2 + x * dcdist * icdist2 + k[2] * da1 + k[3] * (dr2 + 4 * x * dxd);
    double dmy = dyd * cdist * icdist2 + y * dcdist * icdist2 + k[2] * (dr2 + 4 * y * dyd) + k[3] * da1;
    J[col] = K.fx * dmx;
    J[6 + col] = K.fy * dmy;
  };
  for (int j = 0; j < 3; ++j) {
    double dx0 = X * dRdr[j * 9 + 0] + Y * dRdr[j * 9 + 1] + Z * dRdr[j * 9 + 2];
    double dy0 = X * dRdr[j * 9 + 3] + Y * dRdr[j * 9 + 4] + Z * dRdr[j * 9 + 5];
    double dz0 = X * dRdr[j * 9 + 6] + Y * dRdr[j * 9 + 7] + Z * dRdr[j * 9 + 8];
    fill(z * (dx0 - x * dz0), z * (dy0 - y * dz0), j);
  }
  double dxdt[3] = {z, 0, -x * z}, dydt[3] = {0, z, -y * z};
  for (int j = 0; j < 3; ++j) fill(dxdt[j], dydt[j], 3 + j);
}

// undistortPoints(..., P empty): 5 fixed-point iterations, normalised output.
static void undistort_point(const Cam& K, double u, double v, double* xy) {
  const double ifx = 1. / K.fx, ify = 1. / K.fy;
  double x = (u - K.cx) * ifx, y = (v - K.cy) * ify;
  double x0 = x, y0 = y;
  const double* k = K.k;
  for (int j = 0; j < 5; ++j) {
    double r2 = x * x + y * y;
    double icdist = 1. / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
    if (icdist < 0) { x = (u - K.cx) * ifx; y = (v - K.cy) * ify; break; }
    double dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
    double dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
    x = (x0 - dx) * icdist;
    y = (y0 - dy) * icdist;
  }
  xy[0] = x; xy[1] = y;
}

// ------------------------------------------------------------------ EPnP
struct EPnP {
  int n;
  double fu, fv, uc, vc;
  std::vector<double> pws, us, alphas, pcs;
  double cws[4][3], ccs[4][3];

  void choose_control_points() {
    for (int j = 0; j < 3; ++j) cws[0][j] = 0;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < 3; ++j) cws[0][j] += pws[3 * i + j];
    for (int j = 0; j < 3; ++j) cws[0][j] /= n;
    double A[9] = {0};
    for (int i = 0; i < n; ++i) {
      double d[3] = {pws[3 * i] - cws[0][0], pws[3 * i + 1] - cws[0][1], pws[3 * i + 2] - cws[0][2]};
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) A[a * 3 + b] += d[a] * d[b];
    }
    double W[3], U[9], V[9];
    svd(A, 3, 3, W, U, V);
    for (int i = 1; i < 4; ++i) {
      double k = std::sqrt(W[i - 1] / n);
      for (int j = 0; j < 3; ++j) cws[i][j] = cws[0][j] + k * U[j * 3 + (i - 1)];
    }
  }
  void barycentric() {
    double cc[9], ci[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
    double W[3], U[9], V[9];
    svd(cc, 3, 3, W, U, V);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double s = 0;
        for (int k = 0; k < 3; ++k) s += (W[k] > 0 ? V[i * 3 + k] / W[k] : 0.0) * U[j * 3 + k];
        ci[i * 3 + j] = s;
      }
    alphas.resize(4 * n);
    for (int i = 0; i < n; ++i) {
      const double* p = &pws[3 * i];
      double* a = &alphas[4 * i];
      for (int j = 0; j < 3; ++j)
        a[1 + j] = ci[3 * j] * (p[0] - cws[0][0]) + ci[3 * j + 1] * (p[1] - cws[0][1]) + ci[3 * j + 2] * (p[2] - cws[0][2]);
      a[0] = 1.0f - a[1] - a[2] - a[3];
    }
  }
  static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
  static double dist2(const double* a, const double* b) {
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
  }
  void compute_ccs(const double* betas, const double* ut) {
    for (int i = 0; i < 4; ++i) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
    for (int i = 0; i < 4; ++i) {
      const double* v = ut + 12 * (11 - i);
      for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[3 * j + k];
    }
  }
  void compute_pcs() {
    pcs.resize(3 * n);
    for (int i = 0; i < n; ++i) {
      const double* a = &alphas[4 * i];
      for (int j = 0; j < 3; ++j) pcs[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
    }
  }
  void solve_for_sign() {
    if (pcs[2] < 0.0) {
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j) ccs[i][j] = -ccs[i][j];
      for (auto& v : pcs) v = -v;
    }
  }
  void estimate_R_and_t(double R[3][3], double t[3]) {
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < 3; ++j) { pc0[j] += pcs[3 * i + j]; pw0[j] += pws[3 * i + j]; }
    for (int j = 0; j < 3; ++j) { pc0[j] /= n; pw0[j] /= n; }
    double abt[9] = {0};
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < 3; ++j) {
        double dc = pcs[3 * i + j] - pc0[j];
        abt[3 * j] += dc * (pws[3 * i] - pw0[0]);
        abt[3 * j + 1] += dc * (pws[3 * i + 1] - pw0[1]);
        abt[3 * j + 2] += dc * (pws[3 * i + 2] - pw0[2]);
      }
    double W[3], U[9], V[9];
    svd(abt, 3, 3, W, U, V);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) R[i][j] = U[i * 3] * V[j * 3] + U[i * 3 + 1] * V[j * 3 + 1] + U[i * 3 + 2] * V[j * 3 + 2];
    double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                 R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0) { R[2][0] = -R[2][0]; R[2][1] = -R[2][1]; R[2][2] = -R[2][2]; }
    for (int i = 0; i < 3; ++i) t[i] = pc0[i] - dot3(R[i], pw0);
  }
  double reprojection_error(const double R[3][3], const double t[3]) {
    double sum2 = 0.0;
    for (int i = 0; i < n; ++i) {
      const double* pw = &pws[3 * i];
      double Xc = dot3(R[0], pw) + t[0], Yc = dot3(R[1], pw) + t[1];
      double iz = 1.0 / (dot3(R[2], pw) + t[2]);
      double ue = uc + fu * Xc * iz, ve = vc + fv * Yc * iz;
      double u = us[2 * i], v = us[2 * i + 1];
      sum2 += std::sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / n;
  }
  double compute_R_and_t(const double* ut, const double* betas, double R[3][3], double t[3]) {
    compute_ccs(betas, ut);
    compute_pcs();
    solve_for_sign();
    estimate_R_and_t(R, t);
    return reprojection_error(R, t);
  }
  void compute_L_6x10(const double* ut, double* L) {
    const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
    double dv[4][6][3];
    for (int i = 0; i < 4; ++i) {
      int a = 0, b = 1;
      for (int j = 0; j < 6; ++j) {
        for (int k = 0; k < 3; ++k) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
        if (++b > 3) { ++a; b = a + 1; }
      }
    }
    for (int i = 0; i < 6; ++i) {
      double* r = L + 10 * i;
      r[0] = dot3(dv[0][i], dv[0][i]);
      r[1] = 2.0f * dot3(dv[0][i], dv[1][i]);
      r[2] = dot3(dv[1][i], dv[1][i]);
      r[3] = 2.0f * dot3(dv[0][i], dv[2][i]);
      r[4] = 2.0f * dot3(dv[1][i], dv[2][i]);
      r[5] = dot3(dv[2][i], dv[2][i]);
      r[6] = 2.0f * dot3(dv[0][i], dv[3][i]);
      r[7] = 2.0f * dot3(dv[1][i], dv[3][i]);
      r[8] = 2.0f * dot3(dv[2][i], dv[3][i]);
      r[9] = dot3(dv[3][i], dv[3][i]);
    }
  }
  void compute_rho(double* rho) {
    rho[0] = dist2(cws[0], cws[1]); rho[1] = dist2(cws[0], cws[2]); rho[2] = dist2(cws[0], cws[3]);
    rho[3] = dist2(cws[1], cws[2]); rho[4] = dist2(cws[1], cws[3]); rho[5] = dist2(cws[2], cws[3]);
  }
  static void betas_from(const double* L, const double* rho, const int* cols, int nc, double* b) {
    double A[60];
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < nc; ++j) A[i * nc + j] = L[i * 10 + cols[j]];
    solve_svd(A, 6, nc, rho, b);
  }
  void approx1(const double* L, const double* rho, double* betas) {
    int c[4] = {0, 1, 3, 6};
    double b4[4];
    betas_from(L, rho, c, 4, b4);
    if (b4[0] < 0) {
      betas[0] = std::sqrt(-b4[0]);
      betas[1] = -b4[1] / betas[0]; betas[2] = -b4[2] / betas[0]; betas[3] = -b4[3] / betas[0];
    } else {
      betas[0] = std::sqrt(b4[0]);
      betas[1] = b4[1] / betas[0]; betas[2] = b4[2] / betas[0]; betas[3] = b4[3] / betas[0];
    }
  }
  void approx2(const double* L, const double* rho, double* betas) {
    int c[3] = {0, 1, 2};
    double b3[3];
    betas_from(L, rho, c, 3, b3);
    if (b3[0] < 0) {
      betas[0] = std::sqrt(-b3[0]);
      betas[1] = (b3[2] < 0) ? std::sqrt(-b3[2]) : 0.0;
    } else {
      betas[0] = std::sqrt(b3[0]);
      betas[1] = (b3[2] > 0) ? std::sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0; betas[3] = 0.0;
  }
  void approx3(const double* L, const double* rho, double* betas) {
    int c[5] = {0, 1, 2, 3, 4};
    double b5[5];
    betas_from(L, rho, c, 5, b5);
    if (b5[0] < 0) {
      betas[0] = std::sqrt(-b5[0]);
      betas[1] = (b5[2] < 0) ? std::sqrt(-b5[2]) : 0.0;
    } else {
      betas[0] = std::sqrt(b5[0]);
      betas[1] = (b5[2] > 0) ? std::sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
  }
  // Householder QR least squares (epnp::qr_solve), A 6x4.
  static void qr_solve(double* A, double* b, double* X, int nr, int nc) {
    double A1[8], A2[8];
    for (int k = 0; k < nc; ++k) {
      double eta = std::fabs(A[k * nc + k]);
      for (int i = k + 1; i < nr; ++i) eta = std::max(eta, std::fabs(A[i * nc + k]));
      if (eta == 0) { return; }
      double sum2 = 0.0, inv = 1. / eta;
      for (int i = k; i < nr; ++i) { A[i * nc + k] *= inv; sum2 += A[i * nc + k] * A[i * nc + k]; }
      double sigma = std::sqrt(sum2);
      if (A[k * nc + k] < 0) sigma = -sigma;
      A[k * nc + k] += sigma;
      A1[k] = sigma * A[k * nc + k];
      A2[k] = -eta * sigma;
      for (int j = k + 1; j < nc; ++j) {
        double sum = 0;
        for (int i = k; i < nr; ++i) sum += A[i * nc + k] * A[i * nc + j];
        double tau = sum / A1[k];
        for (int i = k; i < nr; ++i) A[i * nc + j] -= tau * A[i * nc + k];
      }
    }
    for (int j = 0; j < nc; ++j) {
      double tau = 0;
      for (int i = j; i < nr; ++i) tau += A[i * nc + j] * b[i];
      tau /= A1[j];
      for (int i = j; i < nr; ++i) b[i] -= tau * A[i * nc + j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; --i) {
      double sum = 0;
      for (int j = i + 1; j < nc; ++j) sum += A[i * nc + j] * X[j];
      X[i] = (b[i] - sum) / A2[i];
    }
  }
  void gauss_newton(const double* L, const double* rho, double* betas) {
    for (int it = 0; it < 5; ++it) {
      double A[24], b[6], x[4] = {0, 0, 0, 0};
      for (int i = 0; i < 6; ++i) {
        const double* r = L + 10 * i;
        A[i * 4 + 0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
        A[i * 4 + 1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
        A[i * 4 + 2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
        A[i * 4 + 3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
        b[i] = rho[i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] + r[2] * betas[1] * betas[1] +
                         r[3] * betas[0] * betas[2] + r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                         r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] + r[8] * betas[2] * betas[3] +
                         r[9] * betas[3] * betas[3]);
      }
      qr_solve(A, b, x, 6, 4);
      for (int i = 0; i < 4; ++i) betas[i] += x[i];
    }
  }
  void compute_pose(double R[3][3], double t[3]) {
    choose_control_points();
    barycentric();
    std::vector<double> M((size_t)2 * n * 12);
    for (int i = 0; i < n; ++i) {
      const double* as = &alphas[4 * i];
      double u = us[2 * i], v = us[2 * i + 1];
      double* M1 = &M[(size_t)(2 * i) * 12];
      double* M2 = M1 + 12;
      for (int j = 0; j < 4; ++j) {
        M1[3 * j] = as[j] * fu; M1[3 * j + 1] = 0.0; M1[3 * j + 2] = as[j] * (uc - u);
        M2[3 * j] = 0.0; M2[3 * j + 1] = as[j] * fv; M2[3 * j + 2] = as[j] * (vc - v);
      }
    }
    double MtM[144] = {0};
    for (int i = 0; i < 2 * n; ++i)
      for (int a = 0; a < 12; ++a)
        for (int b = 0; b < 12; ++b) MtM[a * 12 + b] += M[(size_t)i * 12 + a] * M[(size_t)i * 12 + b];
    double W[12], U[144], V[144], ut[144];
    svd(MtM, 12, 12, W, U, V);
    for (int i = 0; i < 12; ++i)
      for (int j = 0; j < 12; ++j) ut[i * 12 + j] = U[j * 12 + i];  // rows = singular vectors
    double L[60], rho[6];
    compute_L_6x10(ut, L);
    compute_rho(rho);
    double Betas[4][4], err[4], Rs[4][3][3], ts[4][3];
    approx1(L, rho, Betas[1]); gauss_newton(L, rho, Betas[1]); err[1] = compute_R_and_t(ut, Betas[1], Rs[1], ts[1]);
    approx2(L, rho, Betas[2]); gauss_newton(L, rho, Betas[2]); err[2] = compute_R_and_t(ut, Betas[2], Rs[2], ts[2]);
    approx3(L, rho, Betas[3]); gauss_newton(L, rho, Betas[3]); err[3] = compute_R_and_t(ut, Betas[3], Rs[3], ts[3]);
    int N = 1;
    if (err[2] < err[1]) N = 2;
    if (err[3] < err[N]) N = 3;
    for (int i = 0; i < 3; ++i) {
      t[i] = ts[N][i];
      for (int j = 0; j < 3; ++j) R[i][j] = Rs[N][i][j];
    }
  }
};

// solvePnP(..., SOLVEPNP_EPNP) on float32 inputs: undistortPoints -> float32 -> EPnP.
static void solve_epnp(const Cam& K, const float* P3, const float* p2, int n, double* rvec, double* tvec) {
  EPnP e;
  e.n = n; e.fu = K.fx; e.fv = K.fy; e.uc = K.cx; e.vc = K.cy;
  e.pws.resize(3 * n); e.us.resize(2 * n);
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < 3; ++j) e.pws[3 * i + j] = P3[3 * i + j];
    double xy[2];
    undistort_point(K, p2[2 * i], p2[2 * i + 1], xy);
    float fx = (float)xy[0], fy = (float)xy[1];
    e.us[2 * i] = fx * K.fx + K.cx;
    e.us[2 * i + 1] = fy * K.fy + K.cy;
  }
  double R[3][3];
  e.compute_pose(R, tvec);
  double Rf[9];
  for (int i = 0; i < 9; ++i) Rf[i] = R[i / 3][i % 3];
  rodrigues_R2r(Rf, rvec);
}

struct RNG {
  uint64_t state;
  explicit RNG(uint64_t s) : state(s ? s : 0xffffffffu) {}
  unsigned next() {
    state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
    return (unsigned)state;
  }
  int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

static int update_num_iters(double p, double ep, int m, int maxIters) {
  p = std::max(p, 0.); p = std::min(p, 1.);
  ep = std::max(ep, 0.); ep = std::min(ep, 1.);
  double num = std::max(1. - p, DBL_MIN);
  double denom = 1. - std::pow(1. - ep, m);
  if (denom < DBL_MIN) return 0;
  num = std::log(num);
  denom = std::log(denom);
  return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)std::lrint(num / denom);
}

// PnPRansacCallback::computeError -> findInliers.
static int find_inliers(const Cam& K, const float* P3, const float* p2, int n, const double* rvec, const double* tvec,
                        float thr2, uint8_t* mask) {
  double R[9], dR[27];
  rodrigues_r2R(rvec, R, dR);
  int good = 0;
  for (int i = 0; i < n; ++i) {
    double M[3] = {P3[3 * i], P3[3 * i + 1], P3[3 * i + 2]}, uv[2];
    project(K, R, dR, tvec, M, uv, nullptr);
    float pu = (float)uv[0], pv = (float)uv[1];
    float dx = p2[2 * i] - pu, dy = p2[2 * i + 1] - pv;
    float err = dx * dx + dy * dy;
    int f = err <= thr2;
    mask[i] = (uint8_t)f;
    good += f;
  }
  return good;
}

// Homography (planar init branch only; rare).  Normalised DLT, no refinement.
static bool homography_dlt(const double* src, const double* dst, int n, double* H) {
  std::vector<double> A((size_t)2 * n * 9);
  for (int i = 0; i < n; ++i) {
    double X = src[2 * i], Y = src[2 * i + 1], u = dst[2 * i], v = dst[2 * i + 1];
    double* a = &A[(size_t)18 * i];
    double r0[9] = {X, Y, 1, 0, 0, 0, -u * X, -u * Y, -u};
    double r1[9] = {0, 0, 0, X, Y, 1, -v * X, -v * Y, -v};
    std::memcpy(a, r0, sizeof(r0));
    std::memcpy(a + 9, r1, sizeof(r1));
  }
  double AtA[81] = {0};
  for (int i = 0; i < 2 * n; ++i)
    for (int a = 0; a < 9; ++a)
      for (int b = 0; b < 9; ++b) AtA[a * 9 + b] += A[(size_t)i * 9 + a] * A[(size_t)i * 9 + b];
  double W[9], U[81], V[81];
  svd(AtA, 9, 9, W, U, V);
  for (int i = 0; i < 9; ++i) H[i] = V[i * 9 + 8];
  if (std::fabs(H[8]) < 1e-300) return false;
  for (int i = 0; i < 9; ++i) H[i] /= H[8];
  return true;
}

// cvFindExtrinsicCameraParams2(useExtrinsicGuess=false): init + LM.  Returns false if
// the DLT would throw (non-planar and < 6 points).
static bool find_extrinsic(const Cam& K, const double* M, const double* m, int n, double* rvec, double* tvec) {
  std::vector<double> mn(2 * n);
  for (int i = 0; i < n; ++i) undistort_point(K, m[2 * i], m[2 * i + 1], &mn[2 * i]);
  double param[6] = {0, 0, 0, 0, 0, 0};
  double Mc[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 3; ++j) Mc[j] += M[3 * i + j];
  for (int j = 0; j < 3; ++j) Mc[j] /= n;
  double MM[9] = {0};
  for (int i = 0; i < n; ++i) {
    double d[3] = {M[3 * i] - Mc[0], M[3 * i + 1] - Mc[1], M[3 * i + 2] - Mc[2]};
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) MM[a * 3 + b] += d[a] * d[b];
  }
  double W[3], U3[9], V3[9];
  svd(MM, 3, 3, W, U3, V3);
  double R[9];
  if (W[2] / W[1] < 1e-3) {
    // planar: R_transform = V^T (rows = principal axes)
    double Rt[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rt[i * 3 + j] = V3[j * 3 + i];
    if (Rt[2] * Rt[2] + Rt[5] * Rt[5] < 1e-10) { for (int i = 0; i < 9; ++i) Rt[i] = (i % 4 == 0); }
    if (det3(Rt) < 0) for (int i = 0; i < 9; ++i) Rt[i] = -Rt[i];
    double T[3];
    for (int i = 0; i < 3; ++i) T[i] = -(Rt[i * 3] * Mc[0] + Rt[i * 3 + 1] * Mc[1] + Rt[i * 3 + 2] * Mc[2]);
    std::vector<double> Mxy(2 * n);
    for (int i = 0; i < n; ++i) {
      const double* s = &M[3 * i];
      Mxy[2 * i] = Rt[0] * s[0] + Rt[1] * s[1] + Rt[2] * s[2] + T[0];
      Mxy[2 * i + 1] = Rt[3] * s[0] + Rt[4] * s[1] + Rt[5] * s[2] + T[1];
    }
    double H[9], t[3];
    if (homography_dlt(Mxy.data(), mn.data(), n, H)) {
      double h1 = std::sqrt(H[0] * H[0] + H[3] * H[3] + H[6] * H[6]);
      double h2 = std::sqrt(H[1] * H[1] + H[4] * H[4] + H[7] * H[7]);
      for (int i = 0; i < 3; ++i) {
        H[i * 3] /= std::max(h1, DBL_EPSILON);
        H[i * 3 + 1] /= std::max(h2, DBL_EPSILON);
        t[i] = H[i * 3 + 2] * 2. / std::max(h1 + h2, DBL_EPSILON);
      }
      H[2] = H[3] * H[7] - H[6] * H[4];
      H[5] = H[6] * H[1] - H[0] * H[7];
      H[8] = H[0] * H[4] - H[3] * H[1];
      double r[3];
      rodrigues_R2r(H, r);
      rodrigues_r2R(r, H, nullptr);
      for (int i = 0; i < 3; ++i) t[i] += H[i * 3] * T[0] + H[i * 3 + 1] * T[1] + H[i * 3 + 2] * T[2];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = H[i * 3] * Rt[j] + H[i * 3 + 1] * Rt[3 + j] + H[i * 3 + 2] * Rt[6 + j];
      param[3] = t[0]; param[4] = t[1]; param[5] = t[2];
    } else {
      for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0);
    }
    rodrigues_R2r(R, param);
  } else {
    if (n < 6) return false;
    double LL[144] = {0};
    for (int i = 0; i < n; ++i) {
      double x = -mn[2 * i], y = -mn[2 * i + 1];
      const double* P = &M[3 * i];
      double r0[12] = {P[0], P[1], P[2], 1., 0, 0, 0, 0, x * P[0], x * P[1], x * P[2], x};
      double r1[12] = {0, 0, 0, 0, P[0], P[1], P[2], 1., y * P[0], y * P[1], y * P[2], y};
      for (int a = 0; a < 12; ++a)
        for (int b = 0; b < 12; ++b) LL[a * 12 + b] += r0[a] * r0[b] + r1[a] * r1[b];
    }
    double LW[12], LU[144], LV[144];
    svd(LL, 12, 12, LW, LU, LV);
    double RRt[12];
    for (int i = 0; i < 12; ++i) RRt[i] = LV[i * 12 + 11];
    double RR[9] = {RRt[0], RRt[1], RRt[2], RRt[4], RRt[5], RRt[6], RRt[8], RRt[9], RRt[10]};
    double tt[3] = {RRt[3], RRt[7], RRt[11]};
    if (det3(RR) < 0) {
      for (int i = 0; i < 9; ++i) RR[i] = -RR[i];
      for (int i = 0; i < 3; ++i) tt[i] = -tt[i];
    }
    double sc = 0;
    for (int i = 0; i < 9; ++i) sc += RR[i] * RR[i];
    sc = std::sqrt(sc);
    double Wr[3], Ur[9], Vr[9];
    svd(RR, 3, 3, Wr, Ur, Vr);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) R[i * 3 + j] = Ur[i * 3] * Vr[j * 3] + Ur[i * 3 + 1] * Vr[j * 3 + 1] + Ur[i * 3 + 2] * Vr[j * 3 + 2];
    double nR = 0;
    for (int i = 0; i < 9; ++i) nR += R[i] * R[i];
    nR = std::sqrt(nR);
    for (int i = 0; i < 3; ++i) param[3 + i] = tt[i] * nR / sc;
    rodrigues_R2r(R, param);
  }
  // CvLevMarq: lambda 10^-3, max 20 iterations, eps FLT_EPSILON, DECOMP_SVD solve.
  double prev[6], JtJ[36], JtErr[6];
  double lambdaLg10 = -3;
  double prevErrNorm = DBL_MAX;
  std::vector<double> J((size_t)2 * n * 6), err(2 * n);
  auto eval = [&](const double* p, bool withJ) {
    double Rm[9], dR[27];
    rodrigues_r2R(p, Rm, dR);
    double ssq = 0;
    for (int i = 0; i < n; ++i) {
      double uv[2], Ji[12];
      project(K, Rm, dR, p + 3, &M[3 * i], uv, withJ ? Ji : nullptr);
      err[2 * i] = uv[0] - m[2 * i];
      err[2 * i + 1] = uv[1] - m[2 * i + 1];
      ssq += err[2 * i] * err[2 * i] + err[2 * i + 1] * err[2 * i + 1];
      if (withJ) { std::memcpy(&J[(size_t)(2 * i) * 6], Ji, 6 * sizeof(double)); std::memcpy(&J[(size_t)(2 * i + 1) * 6], Ji + 6, 6 * sizeof(double)); }
    }
    return std::sqrt(ssq);
  };
  auto step = [&]() {
    double lambda = std::exp(lambdaLg10 * std::log(10.));
    double A[36], x[6];
    std::memcpy(A, JtJ, sizeof(A));
    for (int i = 0; i < 6; ++i) A[i * 6 + i] *= 1. + lambda;
    solve_svd(A, 6, 6, JtErr, x);
    for (int i = 0; i < 6; ++i) param[i] = prev[i] - x[i];
  };
  int iters = 0;
  for (;;) {
    // CALC_J
    double e0 = eval(param, true);
    for (int a = 0; a < 6; ++a) {
      for (int b = 0; b < 6; ++b) {
        double s = 0;
        for (int i = 0; i < 2 * n; ++i) s += J[(size_t)i * 6 + a] * J[(size_t)i * 6 + b];
        JtJ[a * 6 + b] = s;
      }
      double s = 0;
      for (int i = 0; i < 2 * n; ++i) s += J[(size_t)i * 6 + a] * err[i];
      JtErr[a] = s;
    }
    std::memcpy(prev, param, sizeof(prev));
    step();
    if (iters == 0) prevErrNorm = e0;
    // CHECK_ERR (possibly repeated with larger lambda)
    double errNorm;
    for (;;) {
      errNorm = eval(param, false);
      if (errNorm > prevErrNorm && ++lambdaLg10 <= 16) { step(); continue; }
      break;
    }
    lambdaLg10 = std::max(lambdaLg10 - 1, -16.0);
    double dn = 0, pn = 0;
    for (int i = 0; i < 6; ++i) { dn += (param[i] - prev[i]) * (param[i] - prev[i]); pn += prev[i] * prev[i]; }
    double rel = std::sqrt(dn) / (std::sqrt(pn) + DBL_EPSILON);
    if (++iters >= 20 || rel < FLT_EPSILON) break;
    prevErrNorm = errNorm;
  }
  for (int i = 0; i < 3; ++i) { rvec[i] = param[i]; tvec[i] = param[3 + i]; }
  return true;
}

}  // namespace pnp

extern "C" {

// solvePnPRansac(P3 f64[n,3], p2 f32[n,2], K, dist(5), 1.0, 0.99, 1000, ITERATIVE).
// Returns 1 on success (rvec/tvec/inlier mask written), 0 on failure.
// n_iters_out: RANSAC iterations actually run (debug), best_good_out: RANSAC inliers.
int ref_solve_pnp_ransac(const double* P3d, const float* p2, int n, const double* Kmat, const double* dist,
                         int max_iters, float reproj, double confidence, double* rvec, double* tvec,
                         uint8_t* inlier_mask, int32_t* n_iters_out, int32_t* best_good_out) {
  pnp::Cam K{Kmat[0], Kmat[4], Kmat[2], Kmat[5], {dist[0], dist[1], dist[2], dist[3], dist[4]}};
  std::vector<float> P3(3 * n);
  for (int i = 0; i < 3 * n; ++i) P3[i] = (float)P3d[i];
  const int mp = 5;
  if (n < mp) return 0;
  std::vector<uint8_t> mask(n), best(n, 0);
  double bestModel[6] = {0};
  int maxGood = 0, niters = std::max(max_iters, 1), iter;
  pnp::RNG rng(~0ull);
  float ms1[15], ms2[10];
  if (n == mp) {
    // count == modelPoints: solve directly, all inliers (RANSACPointSetRegistrator::run)
    pnp::solve_epnp(K, P3.data(), p2, n, rvec, tvec);
    for (int i = 0; i < n; ++i) inlier_mask[i] = 1;
    if (n_iters_out) *n_iters_out = 0;
    if (best_good_out) *best_good_out = n;
    return 1;
  }
  for (iter = 0; iter < niters; ++iter) {
    int idx[mp];
    for (int i = 0; i < mp; ++i) {
      int j;
      for (;;) {
        j = rng.uniform(0, n);
        bool dup = false;
        for (int k = 0; k < i; ++k) dup |= idx[k] == j;
        if (!dup) break;
      }
      idx[i] = j;
      for (int k = 0; k < 3; ++k) ms1[3 * i + k] = P3[3 * j + k];
      for (int k = 0; k < 2; ++k) ms2[2 * i + k] = p2[2 * j + k];
    }
    double rv[3], tv[3];
    pnp::solve_epnp(K, ms1, ms2, mp, rv, tv);
    int good = pnp::find_inliers(K, P3.data(), p2, n, rv, tv, (float)((double)reproj * reproj), mask.data());
    if (good > std::max(maxGood, mp - 1)) {
      best.swap(mask);
      mask.assign(n, 0);
      for (int i = 0; i < 3; ++i) { bestModel[i] = rv[i]; bestModel[3 + i] = tv[i]; }
      maxGood = good;
      niters = pnp::update_num_iters(confidence, (double)(n - good) / n, mp, niters);
    }
  }
  if (n_iters_out) *n_iters_out = iter;
  if (best_good_out) *best_good_out = maxGood;
  if (maxGood <= 0) return 0;
  std::vector<double> Mi, mi;
  for (int i = 0; i < n; ++i)
    if (best[i]) {
      for (int k = 0; k < 3; ++k) Mi.push_back((double)P3[3 * i + k]);
      for (int k = 0; k < 2; ++k) mi.push_back((double)p2[2 * i + k]);
    }
  int ni = (int)Mi.size() / 3;
  double rv[3], tv[3];
  bool ok = pnp::find_extrinsic(K, Mi.data(), mi.data(), ni, rv, tv);
  if (!ok) {
    for (int i = 0; i < 3; ++i) { rv[i] = bestModel[i]; tv[i] = bestModel[3 + i]; }
  }
  for (int i = 0; i < 3; ++i) { rvec[i] = rv[i]; tvec[i] = tv[i]; }
  std::memcpy(inlier_mask, best.data(), n);
  return 1;
}

// Debug: the RANSAC hypotheses of the first `iters` iterations (EPnP model per subset and its
// inlier count), without the acceptance rule -- for stage-by-stage comparison with the GPU.
int ref_pnp_hypotheses(const double* P3d, const float* p2, int n, const double* Kmat, const double* dist, int iters,
                       float reproj, double* models, int32_t* good) {
  pnp::Cam K{Kmat[0], Kmat[4], Kmat[2], Kmat[5], {dist[0], dist[1], dist[2], dist[3], dist[4]}};
  std::vector<float> P3(3 * n);
  for (int i = 0; i < 3 * n; ++i) P3[i] = (float)P3d[i];
  if (n < 6) return 0;
  std::vector<uint8_t> mask(n);
  pnp::RNG rng(~0ull);
  float ms1[15], ms2[10];
  for (int it = 0; it < iters; ++it) {
    int idx[5];
    for (int i = 0; i < 5; ++i) {
      int j;
      for (;;) {
        j = rng.uniform(0, n);
        bool dup = false;
        for (int k = 0; k < i; ++k) dup |= idx[k] == j;
        if (!dup) break;
      }
      idx[i] = j;
      for (int k = 0; k < 3; ++k) ms1[3 * i + k] = P3[3 * j + k];
      for (int k = 0; k < 2; ++k) ms2[2 * i + k] = p2[2 * j + k];
    }
    double rv[3], tv[3];
    pnp::solve_epnp(K, ms1, ms2, 5, rv, tv);
    good[it] = pnp::find_inliers(K, P3.data(), p2, n, rv, tv, (float)((double)reproj * reproj), mask.data());
    for (int i = 0; i < 3; ++i) { models[it * 6 + i] = rv[i]; models[it * 6 + 3 + i] = tv[i]; }
  }
  return iters;
}

void ref_rodrigues(const double* rvec, double* R) { pnp::rodrigues_r2R(rvec, R, nullptr); }
void ref_rodrigues_jac(const double* rvec, double* R, double* J) { pnp::rodrigues_r2R(rvec, R, J); }
void ref_rodrigues_inv(const double* R, double* rvec) { pnp::rodrigues_R2r(R, rvec); }

void ref_project_points(const double* P3, int n, const double* rvec, const double* tvec, const double* Kmat,
                        const double* dist, double* uv) {
  pnp::Cam K{Kmat[0], Kmat[4], Kmat[2], Kmat[5], {dist[0], dist[1], dist[2], dist[3], dist[4]}};
  double R[9], dR[27];
  pnp::rodrigues_r2R(rvec, R, dR);
  for (int i = 0; i < n; ++i) pnp::project(K, R, dR, tvec, P3 + 3 * i, uv + 2 * i, nullptr);
}

}  // extern "C"
