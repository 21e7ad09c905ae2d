// Mono pose stage for gfx950 — replaces ros_ws/src/mono_slam.py:111-118:
//   E, mask = cv2.findEssentialMat(mkpts0, mkpts1, focal=fx, pp=(cx, cy), RANSAC, 0.999, 1.0)
//   _, R, t, _ = cv2.recoverPose(E, mkpts0, mkpts1, focal=fx, pp=(cx, cy))
//
// k_gather_matches  one block per frame pair: mkpts0 = kp0[queryIdx].xy, mkpts1 = kp1[trainIdx].xy.
// k_em_prep         one thread per frame: RANSAC subsets with OpenCV's RNG(-1) (ransac.h) and
//                   the RANSAC state; normalised fp64 points written once per frame.
// k_em_coef / k_em_elim / k_em_roots / k_em_hyp  the 5-point solver per RANSAC iteration (null
//                   space of the 5x9 epipolar system as OpenCV's JacobiSVD builds it, 10x20 cubic
//                   constraints, Gauss-Jordan, degree-10 det B(z), Durand-Kerner roots as
//                   solvePoly, up to 10 models), then the float32 Sampson-type error of every
//                   model over all points from LDS.
// k_em_replay       the serial acceptance rule of RANSACPointSetRegistrator::run over
//                   (iteration, model) in order: goodCount > max(best, 4), adaptive niters.
// k_em_final        one wave per frame: E and the inlier mask of the winning model.
// k_em_recover      one 256-thread block per frame: decomposeEssentialMat, DLT triangulation of
//                   every point against the four (R, t) candidates (one-sided Jacobi 4x4 SVD per
//                   point), cheirality counts reduced across the block, first maximum wins.
// Specification, operation by operation: oracle/essential_ref.cpp.  fp64, -ffp-contract=off.
#include <cfloat>

#include "fvo_device.h"
#include "ransac.h"

namespace {

struct EmState {
  int maxGood, niters, best, n;  // best = it * 10 + model
};

// ------------------------------------------------------------------ cubic polynomials
// OpenCV getCoeffMat monomial order: x^3 y^3 x^2y xy^2 x^2z x^2 y^2z y^2 xyz xy | xz^2 xz x
// yz^2 yz y z^3 z^2 z 1.  Products of the linear entries E_ij = [x y z 1] are formed with
// compile-time index tables (every loop below is fully unrolled).
__host__ __device__ constexpr int mono_index(int a, int b, int c) {
  // (a, b, c) exponents of x, y, z
  return a == 3 ? 0 : a == 2 ? (b == 1 ? 2 : c == 1 ? 4 : 5)
       : a == 1 ? (b == 2 ? 3 : b == 1 ? (c == 1 ? 8 : 9) : c == 2 ? 10 : c == 1 ? 11 : 12)
       : b == 3 ? 1 : b == 2 ? (c == 1 ? 6 : 7) : b == 1 ? (c == 2 ? 13 : c == 1 ? 14 : 15)
       : c == 3 ? 16 : c == 2 ? 17 : c == 1 ? 18 : 19;
}
// exponents of the linear terms [x, y, z, 1] and of the degree <= 2 monomials in the fixed
// order {x^2, y^2, xy, xz, yz, z^2, x, y, z, 1} (oracle kQuad).
__device__ constexpr int kLinE[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
__device__ constexpr int kQuadE[10][3] = {{2, 0, 0}, {0, 2, 0}, {1, 1, 0}, {1, 0, 1}, {0, 1, 1},
                                          {0, 0, 2}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};

// quadratic as 10 coefficients in kQuadE order
__device__ __forceinline__ int quad_slot(int a, int b, int c) {
  return a == 2 ? 0 : b == 2 ? 1 : (a == 1 && b == 1) ? 2 : (a == 1 && c == 1) ? 3 : (b == 1 && c == 1) ? 4
       : c == 2 ? 5 : a == 1 ? 6 : b == 1 ? 7 : c == 1 ? 8 : 9;
}

// q = a * b (linear x linear), accumulation order i-major, j-minor (oracle mul_ll).
__device__ __forceinline__ void mul_ll(const double* a, const double* b, double* q) {
#pragma unroll
  for (int k = 0; k < 10; ++k) q[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      q[quad_slot(kLinE[i][0] + kLinE[j][0], kLinE[i][1] + kLinE[j][1], kLinE[i][2] + kLinE[j][2])] += a[i] * b[j];
}
// c += s * (q * l) (oracle madd_ql)
__device__ __forceinline__ void madd_ql(const double* q, const double* l, double s, double* c) {
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      c[mono_index(kQuadE[i][0] + kLinE[j][0], kQuadE[i][1] + kLinE[j][1], kQuadE[i][2] + kLinE[j][2])] +=
          s * (q[i] * l[j]);
}

// ------------------------------------------------------------------ 5-point kernel
// Null space of the 5x9 epipolar matrix as OpenCV's SVD::compute(Q, ..., FULL_UV) produces
// it (oracle/essential_ref.cpp null_space_5x9, operation for operation): cyclic one-sided
// Jacobi on the 5 rows (every pair index static, the sweep loop dynamic), rows sorted by
// norm, then rows 5..8 built from RNG(0x12345678) sign vectors by two Gram-Schmidt passes
// with L1 rescales and normalised.  All indices are compile-time, so A stays in VGPRs.
// hypot(2p, beta) is sqrt(4p^2 + beta^2) on both sides (the device libm's hypot differs from
// glibc's by an ulp, which the root solve amplifies to ~2e-9 in E).
__device__ void null_space_5x9(const double* Q, double* basis) {
  constexpr int m = 9, n = 5;
  const double eps = DBL_EPSILON * 10, minval = DBL_MIN;
  double A[9][9];
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int k = 0; k < m; ++k) A[i][k] = Q[i * 9 + k];
  double W[n];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double sd = 0;
#pragma unroll
    for (int k = 0; k < m; ++k) sd += A[i][k] * A[i][k];
    W[i] = sd;
  }
  for (int iter = 0; iter < 30; ++iter) {
    bool changed = false;
#pragma unroll
    for (int i = 0; i < n - 1; ++i)
#pragma unroll
      for (int j = i + 1; j < n; ++j) {
        double a = W[i], p = 0, b = W[j];
#pragma unroll
        for (int k = 0; k < m; ++k) p += A[i][k] * A[j][k];
        if (!(fabs(p) <= eps * sqrt(a * b))) {
          p *= 2;
          const double beta = a - b, gamma = sqrt(p * p + beta * beta);  // hypot: see above
          double c, s;
          if (beta < 0) {
            const double delta = (gamma - beta) * 0.5;
            s = sqrt(delta / gamma);
            c = p / (gamma * s * 2);
          } else {
            c = sqrt((gamma + beta) / (gamma * 2));
            s = p / (gamma * c * 2);
          }
          a = b = 0;
#pragma unroll
          for (int k = 0; k < m; ++k) {
            const double t0 = c * A[i][k] + s * A[j][k];
            const double t1 = -s * A[i][k] + c * A[j][k];
            A[i][k] = t0;
            A[j][k] = t1;
            a += t0 * t0;
            b += t1 * t1;
          }
          W[i] = a;
          W[j] = b;
          changed = true;
        }
      }
    if (!changed) break;
  }
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double sd = 0;
#pragma unroll
    for (int k = 0; k < m; ++k) sd += A[i][k] * A[i][k];
    W[i] = sqrt(sd);
  }
  // selection sort, descending; the swaps are predicated register selects
#pragma unroll
  for (int i = 0; i < n - 1; ++i) {
    int j = i;
#pragma unroll
    for (int k = i + 1; k < n; ++k)
      if (W[j] < W[k]) j = k;
#pragma unroll
    for (int k = i + 1; k < n; ++k) {
      if (j == k) {
        const double tw = W[i]; W[i] = W[k]; W[k] = tw;
#pragma unroll
        for (int e = 0; e < m; ++e) { const double t = A[i][e]; A[i][e] = A[k][e]; A[k][e] = t; }
      }
    }
  }
  uint64_t rs = 0x12345678u;  // cv::RNG(0x12345678)
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    double sd = i < n ? W[i] : 0;
    for (int ii = 0; ii < 100 && sd <= minval; ++ii) {
      const double val0 = 1.0 / m;
#pragma unroll
      for (int k = 0; k < m; ++k) {
        rs = (uint64_t)(unsigned)rs * 4164903690u + (unsigned)(rs >> 32);
        A[i][k] = ((unsigned)rs & 256) != 0 ? val0 : -val0;
      }
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int j = 0; j < i; ++j) {
          sd = 0;
#pragma unroll
          for (int k = 0; k < m; ++k) sd += A[i][k] * A[j][k];
          double asum = 0;
#pragma unroll
          for (int k = 0; k < m; ++k) {
            const double t = A[i][k] - sd * A[j][k];
            A[i][k] = t;
            asum += fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
#pragma unroll
          for (int k = 0; k < m; ++k) A[i][k] *= asum;
        }
      sd = 0;
#pragma unroll
      for (int k = 0; k < m; ++k) sd += A[i][k] * A[i][k];
      sd = sqrt(sd);
    }
    const double sc = sd > minval ? 1 / sd : 0.;
#pragma unroll
    for (int k = 0; k < m; ++k) A[i][k] *= sc;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < 9; ++i) basis[c * 9 + i] = A[5 + c][i];
}

template <int NA, int NB>
__device__ __forceinline__ void pmul(const double* a, const double* b, double* c) {
#pragma unroll
  for (int k = 0; k < NA + NB - 1; ++k) c[k] = 0.0;
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) c[i + j] += a[i] * b[j];
}

// det B(z), ascending coefficients (oracle det_poly).
__device__ void det_poly(const double* b, double* c) {
  double p[3][3][5];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double* br = b + j * 13;
#pragma unroll
    for (int k = 0; k < 4; ++k) p[j][0][k] = br[3 - k];
#pragma unroll
    for (int k = 0; k < 4; ++k) p[j][1][k] = br[7 - k];
#pragma unroll
    for (int k = 0; k < 5; ++k) p[j][2][k] = br[12 - k];
  }
  double m0[8], m1[8], m2[8], u[8], v[8], t[12];
  // m0 = p11 p22 - p12 p21 (deg 7)
  pmul<4, 5>(p[1][1], p[2][2], u);
  pmul<5, 4>(p[1][2], p[2][1], v);
#pragma unroll
  for (int k = 0; k < 8; ++k) m0[k] = u[k] - v[k];
  // m1 = p10 p22 - p12 p20 (deg 7)
  pmul<4, 5>(p[1][0], p[2][2], u);
  pmul<5, 4>(p[1][2], p[2][0], v);
#pragma unroll
  for (int k = 0; k < 8; ++k) m1[k] = u[k] - v[k];
  // m2 = p10 p21 - p11 p20 (deg 6)
  pmul<4, 4>(p[1][0], p[2][1], u);
  pmul<4, 4>(p[1][1], p[2][0], v);
#pragma unroll
  for (int k = 0; k < 7; ++k) m2[k] = u[k] - v[k];
  m2[7] = 0.0;
#pragma unroll
  for (int k = 0; k < 11; ++k) c[k] = 0.0;
  pmul<4, 8>(p[0][0], m0, t);
#pragma unroll
  for (int k = 0; k < 11; ++k) c[k] += t[k];
  pmul<4, 8>(p[0][1], m1, t);
#pragma unroll
  for (int k = 0; k < 11; ++k) c[k] -= t[k];
  pmul<5, 7>(p[0][2], m2, t);
#pragma unroll
  for (int k = 0; k < 11; ++k) c[k] += t[k];
}

struct Cx {
  double re, im;
};
__device__ __forceinline__ Cx cmul(Cx a, Cx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ Cx cdiv(Cx a, Cx b) {
  double t = 1. / (b.re * b.re + b.im * b.im);
  return {(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
}

__device__ __forceinline__ void null3(const double* B, double* v) {
  constexpr int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
  v[0] = 0.0; v[1] = 0.0; v[2] = 0.0;
  double best = -1.0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double* a = B + pr[q][0] * 3;
    const double* b = B + pr[q][1] * 3;
    double c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    double n2 = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    if (n2 > best) {
      best = n2;
      v[0] = c[0]; v[1] = c[1]; v[2] = c[2];
    }
  }
  double nrm = sqrt(best);
  if (nrm > 0.0)
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] /= nrm;
}

// computeError of one point (float, as EMEstimatorCallback writes it).
__device__ __forceinline__ float em_error(const double* E, double a1, double b1, double a2, double b2) {
  double Ex0 = E[0] * a1 + E[1] * b1 + E[2];
  double Ex1 = E[3] * a1 + E[4] * b1 + E[5];
  double Ex2 = E[6] * a1 + E[7] * b1 + E[8];
  double Et0 = E[0] * a2 + E[3] * b2 + E[6];
  double Et1 = E[1] * a2 + E[4] * b2 + E[7];
  double x2tEx1 = a2 * Ex0 + b2 * Ex1 + Ex2;
  double den = Ex0 * Ex0 + Ex1 * Ex1 + Et0 * Et0 + Et1 * Et1;
  return (float)(x2tEx1 * x2tEx1 / den);
}

// ------------------------------------------------------------------ recoverPose helpers
__device__ void eig3(const double* Sin, double* w, double* V) {
  double S[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) S[i] = Sin[i];
#pragma unroll
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = S[1] * S[1] + S[2] * S[2] + S[5] * S[5];
    if (off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = p + 1; q < 3; ++q) {
        double apq = S[p * 3 + q];
        if (apq == 0.0) continue;
        double theta = (S[q * 3 + q] - S[p * 3 + p]) / (2.0 * apq);
        double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double skp = S[k * 3 + p], skq = S[k * 3 + q];
          S[k * 3 + p] = c * skp - s * skq;
          S[k * 3 + q] = s * skp + c * skq;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double spk = S[p * 3 + k], sqk = S[q * 3 + k];
          S[p * 3 + k] = c * spk - s * sqk;
          S[q * 3 + k] = s * spk + c * sqk;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double vkp = V[k * 3 + p], vkq = V[k * 3 + q];
          V[k * 3 + p] = c * vkp - s * vkq;
          V[k * 3 + q] = s * vkp + c * vkq;
        }
      }
  }
  double d[3] = {S[0], S[4], S[8]};
  int o[3] = {0, 1, 2};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i + 1; j < 3; ++j)
      if (d[o[j]] > d[o[i]]) { int t = o[i]; o[i] = o[j]; o[j] = t; }
  double Vs[9];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    w[j] = d[o[j]];
#pragma unroll
    for (int k = 0; k < 3; ++k) Vs[k * 3 + j] = V[k * 3 + o[j]];
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) V[i] = Vs[i];
}

__device__ __forceinline__ void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ void decompose_essential(const double* E, double* R1, double* R2, double* t) {
  double S[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += E[k * 3 + i] * E[k * 3 + j];
      S[i * 3 + j] = s;
    }
  double w[3], V[9];
  eig3(S, w, V);
  double v0[3] = {V[0], V[3], V[6]}, v1[3] = {V[1], V[4], V[7]}, v2[3];
  cross3(v0, v1, v2);
  double u0[3], u1[3], u2[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    u0[i] = E[i * 3] * v0[0] + E[i * 3 + 1] * v0[1] + E[i * 3 + 2] * v0[2];
    u1[i] = E[i * 3] * v1[0] + E[i * 3 + 1] * v1[1] + E[i * 3 + 2] * v1[2];
  }
  double n0 = sqrt(u0[0] * u0[0] + u0[1] * u0[1] + u0[2] * u0[2]);
#pragma unroll
  for (int i = 0; i < 3; ++i) u0[i] /= n0;
  double d = u0[0] * u1[0] + u0[1] * u1[1] + u0[2] * u1[2];
#pragma unroll
  for (int i = 0; i < 3; ++i) u1[i] -= d * u0[i];
  double n1 = sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
#pragma unroll
  for (int i = 0; i < 3; ++i) u1[i] /= n1;
  cross3(u0, u1, u2);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double vj[3] = {v0[j], v1[j], v2[j]};
      R1[i * 3 + j] = -u1[i] * vj[0] + u0[i] * vj[1] + u2[i] * vj[2];
      R2[i * 3 + j] = u1[i] * vj[0] - u0[i] * vj[1] + u2[i] * vj[2];
    }
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = u2[i];
}

__device__ void null4(const double* Ain, double* x) {
  double A[16], V[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { A[i] = Ain[i]; V[i] = (i % 5 == 0) ? 1.0 : 0.0; }
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double a = 0, b = 0, g = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a += A[i * 4 + p] * A[i * 4 + p];
          b += A[i * 4 + q] * A[i * 4 + q];
          g += A[i * 4 + p] * A[i * 4 + q];
        }
        if (!(fabs(g) > 1e-15 * sqrt(a * b))) continue;
        rotated = true;
        double zeta = (b - a) / (2.0 * g);
        double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double ap = A[i * 4 + p], aq = A[i * 4 + q];
          A[i * 4 + p] = c * ap - s * aq;
          A[i * 4 + q] = s * ap + c * aq;
          double vp = V[i * 4 + p], vq = V[i * 4 + q];
          V[i * 4 + p] = c * vp - s * vq;
          V[i * 4 + q] = s * vp + c * vq;
        }
      }
    if (!rotated) break;
  }
  int best = 0;
  double bn = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double n2 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) n2 += A[i * 4 + j] * A[i * 4 + j];
    if (j == 0 || n2 < bn) { bn = n2; best = j; }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = V[i * 4 + best];
}

__device__ int cheiral(const double* R, const double* t, double a1, double b1, double a2, double b2, double dist) {
  double A[16] = {-1.0, 0.0, a1, 0.0, 0.0, -1.0, b1, 0.0};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double p0 = k < 3 ? R[k] : t[0], p1 = k < 3 ? R[3 + k] : t[1], p2 = k < 3 ? R[6 + k] : t[2];
    A[8 + k] = a2 * p2 - p0;
    A[12 + k] = b2 * p2 - p1;
  }
  double Q[4];
  null4(A, Q);
  bool m = Q[2] * Q[3] > 0;
  double X = Q[0] / Q[3], Y = Q[1] / Q[3], Z = Q[2] / Q[3];
  m = m && Z < dist;
  double z2 = R[6] * X + R[7] * Y + R[8] * Z + t[2];
  m = m && z2 > 0 && z2 < dist;
  return m ? 1 : 0;
}

struct Pinhole {
  double f, cx, cy;
};

// ------------------------------------------------------------------ kernels
__global__ void k_gather_matches(const float* __restrict__ kp0, const float* __restrict__ kp1,
                                 const int32_t* __restrict__ matches, const int32_t* __restrict__ nmatch, int cap,
                                 float* __restrict__ p0, float* __restrict__ p1, int32_t* __restrict__ npts) {
  const int b = blockIdx.x;
  int n = nmatch[b];
  n = n < 0 ? 0 : (n > cap ? cap : n);
  const int32_t* m = matches + (int64_t)b * cap * 3;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    int q = m[3 * i], t = m[3 * i + 1];
    const float* a = kp0 + ((int64_t)b * cap + q) * FVO_KP_STRIDE;
    const float* c = kp1 + ((int64_t)b * cap + t) * FVO_KP_STRIDE;
    p0[((int64_t)b * cap + i) * 2] = a[0];
    p0[((int64_t)b * cap + i) * 2 + 1] = a[1];
    p1[((int64_t)b * cap + i) * 2] = c[0];
    p1[((int64_t)b * cap + i) * 2 + 1] = c[1];
  }
  if (threadIdx.x == 0) npts[b] = n;
}

// Normalised points (x1, y1, x2, y2) fp64 per point and the RANSAC state per frame (the
// subsets come from the context's RNG(-1) table, drawn once: ransac_table_init).
// recoverPose normalises exactly as findEssentialMat does (five-point.cpp), so it reuses this.
__global__ void k_em_prep(const float* __restrict__ p0all, const float* __restrict__ p1all,
                          const int32_t* __restrict__ npts, int cap, Pinhole K, int maxIters,
                          double* __restrict__ xn, EmState* __restrict__ state) {
  const int b = blockIdx.x;
  int n = npts[b];
  n = n < 0 ? 0 : (n > cap ? cap : n);
  const float* p0 = p0all + (int64_t)b * cap * 2;
  const float* p1 = p1all + (int64_t)b * cap * 2;
  double* x = xn + (int64_t)b * cap * 4;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    x[4 * i] = ((double)p0[2 * i] - K.cx) / K.f;
    x[4 * i + 1] = ((double)p0[2 * i + 1] - K.cy) / K.f;
    x[4 * i + 2] = ((double)p1[2 * i] - K.cx) / K.f;
    x[4 * i + 3] = ((double)p1[2 * i + 1] - K.cy) / K.f;
  }
  if (threadIdx.x != 0 || maxIters == 0) return;  // maxIters 0: points only (recoverPose)
  EmState st;
  st.maxGood = 0;
  st.niters = n == 5 ? 1 : maxIters;
  st.best = -1;
  st.n = n;
  state[b] = st;
}

// ---- the 5-point solver in three launches over the RANSAC subsets of one iteration range
// (each a different mapping of the same arithmetic as five_point(), operation for operation):
//   k_em_coef   lane per subset: 5x9 epipolar rows, null-space basis (JacobiSVD), the 10x20
//               cubic-constraint matrix, row by row -> workspace.
//   k_em_elim   16-lane group per subset: Gauss-Jordan on the 10x20 matrix with a row per lane
//               (pivot = first maximum found by a group butterfly, rows swapped by relabelling,
//               pivot row broadcast by shuffles), then B(z) and det B(z) -> workspace.
//   k_em_roots  16-lane row per subset, lane i = root i: Durand-Kerner on det B(z) (300
//               sweeps unless the roots stop moving -- OpenCV's rule, so almost always 300) with
//               the Gauss-Seidel sweep's products split over the lanes, then the models.
//   k_em_hyp    every model of 64 subsets scored over the points in LDS: the (subset, model)
//               pairs spread over a 256-thread block, 4 lanes per pair splitting the points.
// Before: one lane ran five_point() whole (1.9 KB of scratch per lane for the 10x20 matrix and
// the root array, 1 wave per SIMD) -- 13 ms per 64 frames; then a lane per subset ran the whole
// Durand-Kerner sweep (one wave's 300-sweep chain per launch) -- 4.1 ms.
constexpr int EM_WS = 288;  // doubles per subset: basis 36 | A 200 | b 39 | det 11 | ok
constexpr int EMW_BASIS = 0, EMW_A = 36, EMW_B = 236, EMW_C = 275, EMW_OK = 286;

__device__ __forceinline__ bool em_active(const EmState& st, int it, int maxIters) {
  return st.n >= 5 && it < maxIters && it < st.niters;
}

// coeff_matrix, one row at a time (each row's accumulation order unchanged).
__device__ void coeff_rows(const double* basis, double* __restrict__ A) {
  double L[9][4];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) L[i][k] = basis[k * 9 + i];
  {
    constexpr int cof[3][5] = {{0, 4, 8, 5, 7}, {1, 3, 8, 5, 6}, {2, 3, 7, 4, 6}};
    constexpr double sgn[3] = {1.0, -1.0, 1.0};
    double row[20];
#pragma unroll
    for (int k = 0; k < 20; ++k) row[k] = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double q[10], t[10];
      mul_ll(L[cof[c][1]], L[cof[c][2]], q);
      mul_ll(L[cof[c][3]], L[cof[c][4]], t);
#pragma unroll
      for (int k = 0; k < 10; ++k) q[k] -= t[k];
      madd_ql(q, L[cof[c][0]], sgn[c], row);
    }
#pragma unroll
    for (int k = 0; k < 20; ++k) A[k] = row[k];
  }
  // EEt[ij] = sum_k L[i*3+k] L[j*3+k] (k ascending from zero); only the three diagonal
  // entries feed the trace, and row block i needs EEt[i*3+0..2]
  auto eet = [&](int i, int j, double* e) {
#pragma unroll
    for (int m = 0; m < 10; ++m) e[m] = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double q[10];
      mul_ll(L[i * 3 + k], L[j * 3 + k], q);
#pragma unroll
      for (int m = 0; m < 10; ++m) e[m] += q[m];
    }
  };
  double tr[10];
  {
    double e0[10], e4[10], e8[10];
    eet(0, 0, e0);
    eet(1, 1, e4);
    eet(2, 2, e8);
#pragma unroll
    for (int k = 0; k < 10; ++k) tr[k] = e0[k] + e4[k] + e8[k];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double Mq[3][10];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double e[10];
      eet(i, k, e);
      const int ii = i * 3 + k;
#pragma unroll
      for (int m = 0; m < 10; ++m) Mq[k][m] = 2.0 * e[m] - ((ii % 4 == 0) ? tr[m] : 0.0);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double row[20];
#pragma unroll
      for (int k = 0; k < 20; ++k) row[k] = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) madd_ql(Mq[k], L[k * 3 + j], 1.0, row);
#pragma unroll
      for (int k = 0; k < 20; ++k) A[(1 + i * 3 + j) * 20 + k] = row[k];
    }
  }
}

__global__ __launch_bounds__(64) void k_em_coef(const double* __restrict__ xn, int cap, int maxIters, int it_lo,
                                                const int16_t* __restrict__ table, int table_iters,
                                                const EmState* __restrict__ state, double* __restrict__ ws) {
  const int b = blockIdx.y;
  const int it = it_lo + blockIdx.x * 64 + threadIdx.x;
  const EmState st = state[b];
  if (!em_active(st, it, maxIters)) return;
  const double* x = xn + (int64_t)b * cap * 4;
  // count == modelPoints (5): runKernel on all points; else the subset of row n of the table
  const int16_t* sb = table + ((int64_t)st.n * table_iters + it) * 5;
  double Q[45];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int j = st.n == 5 ? i : sb[i];
    const double a = x[4 * j], bb = x[4 * j + 1], c = x[4 * j + 2], d = x[4 * j + 3];
    double* q = Q + i * 9;
    q[0] = a * c; q[1] = bb * c; q[2] = c;
    q[3] = a * d; q[4] = bb * d; q[5] = d;
    q[6] = a; q[7] = bb; q[8] = 1.0;
  }
  double* w = ws + ((int64_t)b * maxIters + it) * EM_WS;
  double basis[36];
  null_space_5x9(Q, basis);
#pragma unroll
  for (int k = 0; k < 36; ++k) w[EMW_BASIS + k] = basis[k];
  coeff_rows(basis, w + EMW_A);
}

// reduce_10x20 with logical row r held by the group lane whose `pos` is r.
__global__ __launch_bounds__(64) void k_em_elim(int maxIters, int it_lo, const EmState* __restrict__ state,
                                                double* __restrict__ ws) {
  __shared__ double sR[4][6][10];  // rows 4..9 of the reduced right half, per group
  const int b = blockIdx.y, g = threadIdx.x >> 4, l = threadIdx.x & 15;
  const int it = it_lo + blockIdx.x * 4 + g;
  const EmState st = state[b];
  const bool active = em_active(st, it, maxIters);  // uniform over the group
  double* w = ws + ((int64_t)b * maxIters + (active ? it : 0)) * EM_WS;
  const bool has = active && l < 10;
  double row[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) row[k] = has ? w[EMW_A + l * 20 + k] : 0.0;
  int pos = l;
  bool ok = active;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    if (ok) {
      // pivot: the first (lowest logical row) maximum of |A[r][c]| over r >= c; a NaN on the
      // diagonal fails (reduce_10x20's !(best > 0)), NaNs below it never win
      const bool elig = has && pos >= c;
      double v = elig && !isnan(row[c]) ? fabs(row[c]) : -1.0;
      int kp = elig ? pos : 64, kl = l;
      int nanfail = (has && pos == c && isnan(row[c])) ? 1 : 0;
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        const double ov = __shfl_xor(v, off, 16);
        const int op = __shfl_xor(kp, off, 16), ol = __shfl_xor(kl, off, 16);
        nanfail |= __shfl_xor(nanfail, off, 16);
        if (ov > v || (ov == v && op < kp)) { v = ov; kp = op; kl = ol; }
      }
      if (nanfail || !(v > 0.0)) {
        ok = false;
      } else {
        const int p = kp, plane = kl;
        if (pos == c) pos = p;
        else if (pos == p) pos = c;
        if (l == plane) {
          const double inv = 1.0 / row[c];
#pragma unroll
          for (int k = c; k < 20; ++k) row[k] *= inv;
        }
        double pr[20];
#pragma unroll
        for (int k = c; k < 20; ++k) pr[k] = __shfl(row[k], plane, 16);
        if (has && l != plane) {
          const double f = row[c];
          if (f != 0.0)
#pragma unroll
            for (int k = c; k < 20; ++k) row[k] -= f * pr[k];
        }
      }
    }
  }
  if (ok && has && pos >= 4)
#pragma unroll
    for (int k = 0; k < 10; ++k) sR[g][pos - 4][k] = row[10 + k];
  __syncthreads();
  if (!active || l != 0) return;
  if (!ok) {
    w[EMW_OK] = 0.0;
    return;
  }
  double bv[39];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double* a1 = sR[g][2 * i];
    const double* a2 = sR[g][2 * i + 1];
    double r1[13], r2[13];
#pragma unroll
    for (int k = 0; k < 13; ++k) { r1[k] = 0.0; r2[k] = 0.0; }
#pragma unroll
    for (int k = 0; k < 3; ++k) { r1[1 + k] = a1[k]; r1[5 + k] = a1[3 + k]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) r1[9 + k] = a1[6 + k];
#pragma unroll
    for (int k = 0; k < 3; ++k) { r2[k] = a2[k]; r2[4 + k] = a2[3 + k]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) r2[8 + k] = a2[6 + k];
#pragma unroll
    for (int k = 0; k < 13; ++k) bv[i * 13 + k] = r1[k] - r2[k];
  }
  double cz[11];
  det_poly(bv, cz);
#pragma unroll
  for (int k = 0; k < 39; ++k) w[EMW_B + k] = bv[k];
#pragma unroll
  for (int k = 0; k < 11; ++k) w[EMW_C + k] = cz[k];
  w[EMW_OK] = 1.0;
}

// solvePoly's Durand-Kerner sweep by a 16-lane row per subset, lane i owning root i.  The
// sweep is Gauss-Seidel: root i's update reads roots 0..i-1 already updated in this sweep and
// roots i+1.. from the previous one, and its denominator multiplies the factors (p_i - root_j)
// in ascending j.  So: every lane evaluates its numerator (Horner at its own root, which no
// other update changes) at the start of the sweep; at step i lane i multiplies its remaining
// factors j > i (previous-sweep roots), divides and publishes its new root (DPP row broadcast),
// and every lane k > i multiplies factor j = i (the new root) into its denominator -- the same
// products in the same order as the serial loop, the sweep's dependent chain cut from ten full
// evaluations to ~n^2/2 products.  Lanes >= n (degree trimmed) and 10..15 idle; rows whose
// polynomials all have degree 10 (the usual case) run a copy without the degree tests.
constexpr int EM_G = 16, EM_GPW = 4;  // lanes per subset (one DPP row), subsets per wave

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// lane i of the row (i a compile-time constant after unrolling)
__device__ __forceinline__ Cx row_bcast(Cx v, int i) {
  switch (i) {
#define FVO_BC(k) case k: return {dpp_d<0x150 + k>(v.re), dpp_d<0x150 + k>(v.im)};
    FVO_BC(0) FVO_BC(1) FVO_BC(2) FVO_BC(3) FVO_BC(4) FVO_BC(5) FVO_BC(6) FVO_BC(7) FVO_BC(8) FVO_BC(9)
#undef FVO_BC
    default: return v;
  }
}
// max over the 16-lane row: quad xor 1, xor 2, half-row mirror, row mirror
__device__ __forceinline__ double row_max(double m) {
  m = fmax(m, dpp_d<0xB1>(m));
  m = fmax(m, dpp_d<0x4E>(m));
  m = fmax(m, dpp_d<0x141>(m));
  return fmax(m, dpp_d<0x140>(m));
}

// den * (p - r), skipped when p - r is exactly 0 (solvePoly's test), without a branch
__device__ __forceinline__ Cx dk_factor(Cx den, Cx p, Cx r) {
  const Cx d{p.re - r.re, p.im - r.im};
  const Cx m = cmul(den, d);
  const bool nz = d.re != 0 || d.im != 0;
  return {nz ? m.re : den.re, nz ? m.im : den.im};
}

template <bool FULL>
__device__ __forceinline__ void dk_sweeps(Cx (&R)[10], Cx& own, const double (&cc)[11], int n, int l, bool mine) {
  for (int iter = 0; iter < 300; ++iter) {
    const Cx p = own;
    Cx num{cc[0], 0}, den{cc[0], 0};
#pragma unroll
    for (int j = 0; j < 10; ++j)
      if (FULL || j < n) {
        num = cmul(num, p);
        num.re += cc[j + 1];
      }
    double mx = 0.0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (FULL || i < n) {
        if (mine && l == i) {
#pragma unroll
          for (int j = i + 1; j < 10; ++j)
            if (FULL || j < n) den = dk_factor(den, p, R[j]);
          const Cx q = cdiv(num, den);
          own = {p.re - q.re, p.im - q.im};
          mx = q.re * q.re + q.im * q.im;
        }
        R[i] = row_bcast(own, i);
        if (mine && l > i) den = dk_factor(den, p, R[i]);
      }
    }
    // the sweep's max |step|^2 (fmax: order-free and NaN-ignoring like the serial fold)
    if (row_max(mx) <= 0) break;  // row-uniform
  }
}

__global__ __launch_bounds__(64) void k_em_roots(int maxIters, int it_lo, const EmState* __restrict__ state,
                                                 const double* __restrict__ ws, double* __restrict__ models,
                                                 int8_t* __restrict__ nmod) {
  const int b = blockIdx.y, lane = threadIdx.x, g = lane >> 4, l = lane & 15, base = g * EM_G;
  const int it = it_lo + blockIdx.x * EM_GPW + g;
  const EmState st = state[b];
  if (st.n < 5 || it_lo + (int)blockIdx.x * EM_GPW >= min(st.niters, maxIters)) return;  // block-uniform
  const bool active = em_active(st, it, maxIters);                                      // row-uniform
  const int64_t slot = (int64_t)b * maxIters + (active ? it : 0);
  const double* w = ws + slot * EM_WS;
  const bool solve = active && w[EMW_OK] != 0.0;
  double c[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) c[k] = solve ? w[EMW_C + k] : 0.0;
  int n = 10;
#pragma unroll
  for (int k = 10; k >= 2; --k)
    if (n == k && fabs(c[k]) <= DBL_EPSILON) n = k - 1;
  double cc[11];  // cc[m] = c[n - m]
#pragma unroll
  for (int m = 0; m <= 10; ++m) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k <= 10; ++k) v = (n - m == k) ? c[k] : v;
    cc[m] = v;
  }
  Cx R[10];  // every root, kept current on every lane of the row
  {
    Cx p{1, 0}, r{1, 1};
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      R[i] = p;
      p = cmul(p, r);
    }
  }
  Cx own{0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i)
    if (l == i) own = R[i];
  const bool mine = solve && l < n;
  if (__ballot(solve && n != 10) == 0ull) dk_sweeps<true>(R, own, cc, n, l, mine);
  else dk_sweeps<false>(R, own, cc, n, l, mine);
  // models: root i (real, |im| <= 1e-10) -> B(z) null vector -> E; lane i, compacted in root order
  bool valid = false;
  double e[9];
  if (mine && !(fabs(own.im) > 1e-10)) {
    const double* bb = w + EMW_B;
    const double* basis = w + EMW_BASIS;
    const double z1 = own.re, z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
    double bz[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double* br = bb + j * 13;
      bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
      bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
      bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
    }
    double v[3];
    null3(bz, v);
    if (!(fabs(v[2]) < 1e-10)) {
      const double xx = v[0] / v[2], yy = v[1] / v[2];
      double n2 = 0.0;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        e[k] = basis[k] * xx + basis[9 + k] * yy + basis[18 + k] * z1 + basis[27 + k];
        n2 += e[k] * e[k];
      }
      const double nrm = sqrt(n2);
#pragma unroll
      for (int k = 0; k < 9; ++k) e[k] = e[k] / nrm;
      valid = true;
    }
  }
  const uint64_t vm = __ballot(valid), gm = 0xFFFFull << base;
  const int rank = __popcll(vm & gm & ((1ull << lane) - 1ull));
  if (valid) {
    double* eo = models + slot * 90 + rank * 9;
#pragma unroll
    for (int k = 0; k < 9; ++k) eo[k] = e[k];
  }
  if (active && l == 0) nmod[slot] = (int8_t)__popcll(vm & gm);
}

// Scoring: every (subset, model) pair of the block's 64 subsets spread evenly over the lanes,
// the points staged in LDS.
constexpr int EM_SC_THREADS = 256, EM_SC_PARTS = 4;  // scoring block; lanes per (subset, model) pair
__global__ __launch_bounds__(EM_SC_THREADS) void k_em_hyp(const double* __restrict__ xn, int cap, float thr2,
                                                          int maxIters, int it_lo, const EmState* __restrict__ state,
                                                          const double* __restrict__ models,
                                                          int32_t* __restrict__ good, const int8_t* __restrict__ nmod) {
  extern __shared__ __attribute__((aligned(16))) double sx[];  // [n][4]
  __shared__ int mlist[640];                                   // (subset << 4 | model) of the block's models
  __shared__ int s_total;
  const int b = blockIdx.y, tid = threadIdx.x;
  const EmState st = state[b];
  const int n = st.n;
  if (n < 5 || it_lo + (int)blockIdx.x * 64 >= min(st.niters, maxIters)) return;  // block-uniform
  const double* x = xn + (int64_t)b * cap * 4;
  for (int i = tid; i < 4 * n; i += EM_SC_THREADS) sx[i] = x[i];
  if (tid < 64) {  // the block's 64 subsets: exclusive scan of their model counts
    const int it = it_lo + blockIdx.x * 64 + tid;
    const int count = em_active(st, it, maxIters) ? (int)nmod[(int64_t)b * maxIters + it] : 0;
    int off = count;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(off, d, 64);
      if (tid >= d) off += t;
    }
    if (tid == 63) s_total = off;
    off -= count;
    for (int k = 0; k < count; ++k) mlist[off + k] = (tid << 4) | k;
  }
  __syncthreads();
  // EM_SC_PARTS consecutive lanes per pair, each counting every EM_SC_PARTS-th point (integer
  // counts: the sum is order-free)
  const int total = s_total, part = tid % EM_SC_PARTS;
  for (int m0 = tid / EM_SC_PARTS; m0 < total; m0 += EM_SC_THREADS / EM_SC_PARTS) {  // uniform per pair's lanes
    const int ml = mlist[m0];
    const int who = ml >> 4, k = ml & 15;
    const int64_t s2 = (int64_t)b * maxIters + it_lo + blockIdx.x * 64 + who;
    const double* mE = models + s2 * 90 + k * 9;
    double E[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) E[q] = mE[q];
    int g = 0;
    for (int i = part; i < n; i += EM_SC_PARTS)
      g += em_error(E, sx[4 * i], sx[4 * i + 1], sx[4 * i + 2], sx[4 * i + 3]) <= thr2;
#pragma unroll
    for (int o = 1; o < EM_SC_PARTS; o <<= 1) g += __shfl_xor(g, o, EM_SC_PARTS);
    if (part == 0) good[s2 * 10 + k] = g;
  }
}

// RANSACPointSetRegistrator::run's acceptance rule over (iteration, model) in order: one
// wave per frame loads 64 iterations' counts at a time, then walks them in order with
// wave-uniform reads (the loop bound niters shrinks as models are accepted).
__global__ __launch_bounds__(64) void k_em_replay(int maxIters, int it_lo, int it_hi, double conf,
                                                  const int32_t* __restrict__ good, const int8_t* __restrict__ nmod,
                                                  EmState* __restrict__ state) {
  const int b = blockIdx.x, lane = threadIdx.x;
  EmState st = state[b];
  if (st.n < 6) return;
  for (int base = it_lo; base < it_hi && base < st.niters; base += 64) {
    const int it = base + lane;
    int nm = 0, g[10], gmax = -1;
#pragma unroll
    for (int k = 0; k < 10; ++k) g[k] = 0;
    if (it < it_hi && it < st.niters) {
      const int64_t slot = (int64_t)b * maxIters + it;
      nm = nmod[slot];
#pragma unroll
      for (int k = 0; k < 10; ++k)
        if (k < nm) {
          g[k] = good[slot * 10 + k];
          gmax = max(gmax, g[k]);
        }
    }
    for (int j = 0; j < 64; ++j) {
      if (base + j >= it_hi || base + j >= st.niters) break;
      // an iteration whose best model does not beat the current record changes nothing: only
      // the (rare) record-setting iterations walk their models one by one
      if (__builtin_amdgcn_readlane(gmax, j) <= max(st.maxGood, 4)) continue;
      const int nmj = __builtin_amdgcn_readlane(nm, j);
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        if (k < nmj) {
          const int gj = __builtin_amdgcn_readlane(g[k], j);
          if (gj > max(st.maxGood, 4)) {
            st.best = (base + j) * 10 + k;
            st.maxGood = gj;
            st.niters = fvo_rs::update_num_iters(conf, (double)(st.n - gj) / st.n, 5, st.niters);
          }
        }
      }
    }
  }
  if (lane == 0) state[b] = st;
}

// E + inlier mask of the accepted model; status 1 ok, 0 no model, -1 n < 5,
// -2 five points with several solutions (findEssentialMat would return a 3k x 3 E).
__global__ __launch_bounds__(64) void k_em_final(const double* __restrict__ xn, int cap, float thr2, int maxIters,
                                                 const EmState* __restrict__ state,
                                                 const double* __restrict__ models, const int8_t* __restrict__ nmod,
                                                 double* __restrict__ Eout, uint8_t* __restrict__ mask,
                                                 int32_t* __restrict__ status) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const EmState st = state[b];
  const int n = st.n;
  int sel = -1, stat;
  if (n < 5) {
    stat = -1;
  } else if (n == 5) {
    int nm = nmod[(int64_t)b * maxIters];
    stat = nm <= 0 ? 0 : (nm > 1 ? -2 : 1);
    if (nm == 1) sel = 0;
  } else {
    stat = st.maxGood > 0 ? 1 : 0;
    if (stat == 1) sel = st.best;
  }
  if (lane < 9) {
    double e = 0.0;
    if (sel >= 0) e = models[((int64_t)b * maxIters + sel / 10) * 90 + (sel % 10) * 9 + lane];
    Eout[b * 9 + lane] = e;
  }
  if (lane == 0) status[b] = stat;
  if (!mask) return;
  uint8_t* mk = mask + (int64_t)b * cap;
  double E[9];
  if (sel >= 0)
#pragma unroll
    for (int q = 0; q < 9; ++q) E[q] = models[((int64_t)b * maxIters + sel / 10) * 90 + (sel % 10) * 9 + q];
  const double* x = xn + (int64_t)b * cap * 4;
  for (int i = lane; i < cap; i += 64) {
    uint8_t f = 0;
    if (sel >= 0 && i < n) f = n == 5 ? 1 : (em_error(E, x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]) <= thr2);
    mk[i] = f;
  }
}

// recoverPose: one 256-thread block per frame.
__global__ __launch_bounds__(256) void k_em_recover(const double* __restrict__ Ein, const int32_t* __restrict__ est,
                                                    const double* __restrict__ xn, const int32_t* __restrict__ npts,
                                                    int cap, double dist, double* __restrict__ Rout,
                                                    double* __restrict__ tout, double* __restrict__ Tout,
                                                    int32_t* __restrict__ ngood) {
  __shared__ int cnt[4][4];
  const int b = blockIdx.x, tid = threadIdx.x;
  int n = npts[b];
  n = n < 0 ? 0 : (n > cap ? cap : n);
  double* T = Tout + (int64_t)b * 16;
  if (est && est[b] != 1) {  // no essential matrix: cv2.recoverPose would raise
    if (tid < 16) T[tid] = (tid % 5 == 0) ? 1.0 : 0.0;
    if (tid < 9) Rout[b * 9 + tid] = (tid % 4 == 0) ? 1.0 : 0.0;
    if (tid < 3) tout[b * 3 + tid] = 0.0;
    if (tid == 0) ngood[b] = -1;
    return;
  }
  double E[9], R1[9], R2[9], tt[3], tn[3];
#pragma unroll
  for (int q = 0; q < 9; ++q) E[q] = Ein[b * 9 + q];
  decompose_essential(E, R1, R2, tt);
#pragma unroll
  for (int i = 0; i < 3; ++i) tn[i] = -tt[i];
  int g[4] = {0, 0, 0, 0};
  const double* x = xn + (int64_t)b * cap * 4;
  for (int i = tid; i < n; i += 256) {
    double a1 = x[4 * i], b1 = x[4 * i + 1], a2 = x[4 * i + 2], b2 = x[4 * i + 3];
    g[0] += cheiral(R1, tt, a1, b1, a2, b2, dist);
    g[1] += cheiral(R2, tt, a1, b1, a2, b2, dist);
    g[2] += cheiral(R1, tn, a1, b1, a2, b2, dist);
    g[3] += cheiral(R2, tn, a1, b1, a2, b2, dist);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) g[k] = wave_sum(g[k]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) cnt[tid >> 6][k] = g[k];
  __syncthreads();
  if (tid != 0) return;
  int G[4];
  for (int k = 0; k < 4; ++k) G[k] = cnt[0][k] + cnt[1][k] + cnt[2][k] + cnt[3][k];
  int sel;
  if (G[0] >= G[1] && G[0] >= G[2] && G[0] >= G[3]) sel = 0;
  else if (G[1] >= G[0] && G[1] >= G[2] && G[1] >= G[3]) sel = 1;
  else if (G[2] >= G[0] && G[2] >= G[1] && G[2] >= G[3]) sel = 2;
  else sel = 3;
  const double* R = (sel & 1) ? R2 : R1;
  const double* t = sel < 2 ? tt : tn;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) {
      Rout[b * 9 + i * 3 + j] = R[i * 3 + j];
      T[i * 4 + j] = R[i * 3 + j];
    }
    tout[b * 3 + i] = t[i];
    T[i * 4 + 3] = t[i];
  }
  T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
  ngood[b] = G[sel];
}

}  // namespace

int mono_init(fvo_ctx* ctx) {
  ctx->em_max_iters = 1000;
  const int64_t B = ctx->cfg.max_batch, it = B * ctx->em_max_iters;
  int rc;
  if ((rc = fvo_alloc(ctx, &ctx->em_x, B * ctx->kp_cap * 4)) || (rc = ransac_table_init(ctx)) ||
      (rc = fvo_alloc(ctx, &ctx->em_models, it * 90)) || (rc = fvo_alloc(ctx, &ctx->em_good, it * 10)) ||
      (rc = fvo_alloc(ctx, &ctx->em_nmod, it)) || (rc = fvo_alloc(ctx, (EmState**)&ctx->em_state, B)) ||
      (rc = fvo_alloc(ctx, &ctx->em_ws, it * EM_WS)))
    return rc;
  return 0;
}

int gather_run(fvo_ctx* ctx, const float* kp0, const float* kp1, const int32_t* matches, const int32_t* nmatch,
               int batch, int cap, float* p0, float* p1, int32_t* npts, hipStream_t s) {
  FVO_TIMED(ctx, KN_GATHER, s, hipLaunchKernelGGL(k_gather_matches, dim3(batch), dim3(256), 0, s, kp0, kp1, matches,
                                                  nmatch, cap, p0, p1, npts));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

int essential_run(fvo_ctx* ctx, const float* p0, const float* p1, const int32_t* npts, int batch, int cap,
                  double focal, double cx, double cy, double prob, double threshold, int maxIters, double* E,
                  uint8_t* mask, int32_t* status, hipStream_t s) {
  if (cap > ctx->kp_cap) return fvo_fail(ctx, "essential: cap exceeds the context keypoint capacity");
  if (maxIters < 1 || maxIters > ctx->em_max_iters || maxIters > ctx->rs_table_iters)
    return fvo_fail(ctx, "essential: max_iters out of range");
  Pinhole K{focal, cx, cy};
  const double thr = threshold / ((focal + focal) / 2);
  const float thr2 = (float)(thr * thr);
  EmState* st = (EmState*)ctx->em_state;
  const size_t shm = (size_t)cap * 4 * sizeof(double);
  if (shm + 640 * sizeof(int) > 160 * 1024) return fvo_fail(ctx, "essential: point capacity exceeds LDS (cap <= 5040)");
  if (shm > 64 * 1024)
    FVO_HIP(ctx, hipFuncSetAttribute((const void*)k_em_hyp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  // round 1: the first 128 subsets of every frame (the adaptive bound usually ends below)
  const int first = std::min(maxIters, 128);
  auto solve = [&](int lo, int hi) {
    const int nit = hi - lo;
    hipLaunchKernelGGL(k_em_coef, dim3((nit + 63) / 64, batch), dim3(64), 0, s, ctx->em_x, cap, maxIters, lo,
                       ctx->rs_table, ctx->rs_table_iters, st, ctx->em_ws);
    hipLaunchKernelGGL(k_em_elim, dim3((nit + 3) / 4, batch), dim3(64), 0, s, maxIters, lo, st, ctx->em_ws);
    hipLaunchKernelGGL(k_em_roots, dim3((nit + EM_GPW - 1) / EM_GPW, batch), dim3(64), 0, s, maxIters, lo, st,
                       ctx->em_ws, ctx->em_models, ctx->em_nmod);
    hipLaunchKernelGGL(k_em_hyp, dim3((nit + 63) / 64, batch), dim3(EM_SC_THREADS), shm, s, ctx->em_x, cap, thr2, maxIters, lo,
                       st, ctx->em_models, ctx->em_good, ctx->em_nmod);
    hipLaunchKernelGGL(k_em_replay, dim3(batch), dim3(64), 0, s, maxIters, lo, hi, prob, ctx->em_good, ctx->em_nmod,
                       st);
  };
  FVO_TIMED(ctx, KN_ESSENTIAL, s, {
    hipLaunchKernelGGL(k_em_prep, dim3(batch), dim3(256), 0, s, p0, p1, npts, cap, K, maxIters, ctx->em_x, st);
    solve(0, first);
    if (maxIters > first) solve(first, maxIters);
    hipLaunchKernelGGL(k_em_final, dim3(batch), dim3(64), 0, s, ctx->em_x, cap, thr2, maxIters, st, ctx->em_models,
                       ctx->em_nmod, E, mask, status);
  });
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

int recover_run(fvo_ctx* ctx, const double* E, const int32_t* est, const float* p0, const float* p1,
                const int32_t* npts, int batch, int cap, double focal, double cx, double cy, double dist, double* R,
                double* t, double* T, int32_t* ngood, hipStream_t s) {
  if (cap > ctx->kp_cap) return fvo_fail(ctx, "recover_pose: cap exceeds the context keypoint capacity");
  Pinhole K{focal, cx, cy};
  // normalised points (the recoverPose normalisation equals findEssentialMat's)
  FVO_TIMED(ctx, KN_RECOVER, s, {
    hipLaunchKernelGGL(k_em_prep, dim3(batch), dim3(256), 0, s, p0, p1, npts, cap, K, 0, ctx->em_x,
                       (EmState*)ctx->em_state);
    hipLaunchKernelGGL(k_em_recover, dim3(batch), dim3(256), 0, s, E, est, ctx->em_x, npts, cap, dist, R, t, T,
                       ngood);
  });
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
