// ORACLE — test infrastructure only. Never linked into the product.
//
// Restates the mono pose step of ros_ws/src/mono_slam.py:111-118:
//   E, mask = cv2.findEssentialMat(mkpts0, mkpts1, focal=K0[0,0], pp=(K0[0,2], K0[1,2]),
//                                  method=cv2.RANSAC, prob=0.999, threshold=1.0)
//   _, R, t, _ = cv2.recoverPose(E, mkpts0, mkpts1, focal=K0[0,0], pp=(K0[0,2], K0[1,2]))
//   T = [R | t]; cumulative = cumulative @ T
// following OpenCV 4.x calib3d (five-point.cpp, ptsetreg.cpp, triangulate.cpp,
// mathfuncs.cpp solvePoly):
//   * points converted to float64 and normalised: x = (u - cx)/f, y = (v - cy)/f;
//     threshold /= f (f = (fx+fy)/2), inlier iff (float)err <= (float)(thr*thr);
//   * RANSACPointSetRegistrator: RNG(-1), 5-point subsets drawn as getSubset()
//     (the same draws as solvePnPRansac's), every model of a subset scored in turn,
//     accept iff goodCount > max(maxGoodCount, 4), niters = RANSACUpdateNumIters(prob, ...);
//   * EMEstimatorCallback::runKernel (Nister / Stewenius 5-point): 4-d null space of the
//     5x9 epipolar system, 10x20 cubic constraint matrix (det E = 0, 2EE^tE - tr(EE^t)E = 0)
//     over the monomials [x^3 y^3 x^2y xy^2 x^2z x^2 y^2z y^2 xyz xy | xz^2 xz x yz^2 yz y
//     z^3 z^2 z 1], Gauss-Jordan elimination, 3x13 B(z), degree-10 det B(z), roots by
//     solvePoly's Durand-Kerner iteration (initial guesses (1+i)^k, at most 300 sweeps,
//     stop on a zero update), real roots |im| <= 1e-10, (x, y) from the null vector of
//     B(z), E = xX + yY + zZ + W normalised to unit Frobenius norm;
//   * computeError: (x2^T E x1)^2 / ((Ex1)_0^2 + (Ex1)_1^2 + (E^Tx2)_0^2 + (E^Tx2)_1^2), as float;
//   * recoverPose (distanceThresh 50, no mask): decomposeEssentialMat (R1 = U W V^T,
//     R2 = U W^T V^T, t = U[:,2], U and V proper rotations), DLT triangulation of every
//     point against [I|0] and each of (R1,t) (R2,t) (R1,-t) (R2,-t), cheirality counts,
//     first maximum in that order wins.
// The 5-point null space follows OpenCV's SVD::compute -> JacobiSVDImpl_ step by step
// (null_space_5x9 below: the basis is the RNG-seeded Gram-Schmidt complement of the row
// space, so the models of a subset come out in OpenCV's order).  Numerical building blocks
// that are this restatement's own (documented in DESIGN.md §2): the polynomial det B(z) by
// cofactor expansion, cross-product null vector of B(z), Jacobi eigen-decomposition for the
// 3x3 SVD of E and one-sided Jacobi for the 4x4 triangulation SVD.  The HIP kernels (csrc/essential.hip) follow this file operation by
// operation.  Parity vs OpenCV: UNPINNED (no cv2, no reference fixtures).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace em {

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

// ------------------------------------------------------------------ cubic polynomials
// Monomial order of OpenCV's getCoeffMat; index of x^a y^b z^c (a+b+c <= 3).
static int mono_index(int a, int b, int c) {
  static const int tbl[4][4][4] = {
      // a = 0: b = 0..3, c = 0..3
      {{19, 18, 17, 16}, {15, 14, 13, -1}, {7, 6, -1, -1}, {1, -1, -1, -1}},
      // a = 1
      {{12, 11, 10, -1}, {9, 8, -1, -1}, {3, -1, -1, -1}, {-1, -1, -1, -1}},
      // a = 2
      {{5, 4, -1, -1}, {2, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}},
      // a = 3
      {{0, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}}};
  return tbl[a][b][c];
}
// exponents of the 20 monomials
static const int kExp[20][3] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                                {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                                {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
// linear terms [x, y, z, 1] -> monomial index
static const int kLin[4] = {12, 15, 18, 19};
// degree <= 2 monomials, in this fixed order
static const int kQuad[10] = {5, 7, 9, 11, 14, 17, 12, 15, 18, 19};

// q = a * b for linear a, b (4 coefficients each); q as 20-vector (only quad entries set).
static void mul_ll(const double* a, const double* b, double* q) {
  for (int k = 0; k < 20; ++k) q[k] = 0.0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      const int* ei = kExp[kLin[i]];
      const int* ej = kExp[kLin[j]];
      q[mono_index(ei[0] + ej[0], ei[1] + ej[1], ei[2] + ej[2])] += a[i] * b[j];
    }
}
// c += s * q * l for quadratic q (20-vector) and linear l.
static void madd_ql(const double* q, const double* l, double s, double* c) {
  for (int i = 0; i < 10; ++i) {
    const int* ei = kExp[kQuad[i]];
    for (int j = 0; j < 4; ++j) {
      const int* ej = kExp[kLin[j]];
      c[mono_index(ei[0] + ej[0], ei[1] + ej[1], ei[2] + ej[2])] += s * (q[kQuad[i]] * l[j]);
    }
  }
}

// ------------------------------------------------------------------ 5-point kernel
// Null space of the 5x9 epipolar matrix Q as EMEstimatorCallback::runKernel obtains it:
//   SVD::compute(Q, W, U, Vt, MODIFY_A | FULL_UV);  EE = Vt.t().colRange(5, 9)
// [OCV, recalled; lapack.cpp _SVDcompute + JacobiSVDImpl_<double>]: Q is wider than tall, so
// the SVD runs on At = Q (5 rows of length m = 9) inside a 9 x 9 buffer whose rows 5..8 are
// zero, n = 5, n1 = 9 (FULL_UV), minval = DBL_MIN, eps = 10 DBL_EPSILON:
//  1. W[i] = |At_i|^2; cyclic one-sided Jacobi over the row pairs (i < j), at most
//     max(m, 30) = 30 sweeps, a pair skipped when |At_i . At_j| <= eps sqrt(W_i W_j), rotation
//     (c, s) from beta = W_i - W_j, gamma = hypot(2p, beta) in the two-branch form, W_i / W_j
//     re-accumulated from the rotated rows; stop after a sweep without a rotation.
//  2. W[i] = sqrt(|At_i|^2); selection sort descending (rows swapped with their W).
//  3. rows i = 0..8 normalised; a row whose singular value is <= minval (rows 5..8: the
//     null space) is replaced by a vector of +-1/m with the signs from RNG(0x12345678)
//     (bit 8 of each draw, one RNG per call), orthogonalised twice against every previous row
//     (Gram-Schmidt, each projection followed by an L1 rescale) and normalised.
// Vt = those 9 rows, so the basis is rows 5..8: the Gram-Schmidt complement of the row space
// seeded by the fixed RNG.  The reduction orders are the scalar source's (OpenCV's SIMD
// builds may accumulate the dot products in two lanes: ulp-level, unpinned).  hypot(2p, beta)
// is evaluated as sqrt(4p^2 + beta^2) -- within an ulp of libm's hypot (no overflow at these
// magnitudes) and, unlike hypot, the same correctly rounded operations on the host and the
// device: an ulp of difference in one rotation grows to ~2e-9 in E through the degree-10
// root solve (measured against the device libm's hypot), above the tests' 1e-9.
static void null_space_5x9(const double* Q, double* basis) {
  const int m = 9, n = 5;
  const double eps = DBL_EPSILON * 10, minval = DBL_MIN;
  double A[9][9];
  for (int i = 0; i < 9; ++i)
    for (int k = 0; k < 9; ++k) A[i][k] = i < n ? Q[i * 9 + k] : 0.0;
  double W[9];
  for (int i = 0; i < n; ++i) {
    double sd = 0;
    for (int k = 0; k < m; ++k) sd += A[i][k] * A[i][k];
    W[i] = sd;
  }
  for (int iter = 0; iter < 30; ++iter) {
    bool changed = false;
    for (int i = 0; i < n - 1; ++i)
      for (int j = i + 1; j < n; ++j) {
        double a = W[i], p = 0, b = W[j];
        for (int k = 0; k < m; ++k) p += A[i][k] * A[j][k];
        if (std::fabs(p) <= eps * std::sqrt(a * b)) continue;
        p *= 2;
        const double beta = a - b, gamma = std::sqrt(p * p + beta * beta);  // hypot: see above
        double c, s;
        if (beta < 0) {
          const double delta = (gamma - beta) * 0.5;
          s = std::sqrt(delta / gamma);
          c = p / (gamma * s * 2);
        } else {
          c = std::sqrt((gamma + beta) / (gamma * 2));
          s = p / (gamma * c * 2);
        }
        a = b = 0;
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
    if (!changed) break;
  }
  for (int i = 0; i < n; ++i) {
    double sd = 0;
    for (int k = 0; k < m; ++k) sd += A[i][k] * A[i][k];
    W[i] = std::sqrt(sd);
  }
  for (int i = 0; i < n - 1; ++i) {
    int j = i;
    for (int k = i + 1; k < n; ++k)
      if (W[j] < W[k]) j = k;
    if (i != j) {
      std::swap(W[i], W[j]);
      for (int k = 0; k < m; ++k) std::swap(A[i][k], A[j][k]);
    }
  }
  RNG rng(0x12345678u);
  for (int i = 0; i < 9; ++i) {
    double sd = i < n ? W[i] : 0;
    for (int ii = 0; ii < 100 && sd <= minval; ++ii) {
      const double val0 = 1.0 / m;
      for (int k = 0; k < m; ++k) A[i][k] = (rng.next() & 256) != 0 ? val0 : -val0;
      for (int it = 0; it < 2; ++it)
        for (int j = 0; j < i; ++j) {
          sd = 0;
          for (int k = 0; k < m; ++k) sd += A[i][k] * A[j][k];
          double asum = 0;
          for (int k = 0; k < m; ++k) {
            const double t = A[i][k] - sd * A[j][k];
            A[i][k] = t;
            asum += std::fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
          for (int k = 0; k < m; ++k) A[i][k] *= asum;
        }
      sd = 0;
      for (int k = 0; k < m; ++k) sd += A[i][k] * A[i][k];
      sd = std::sqrt(sd);
    }
    const double sc = sd > minval ? 1 / sd : 0.;
    for (int k = 0; k < m; ++k) A[i][k] *= sc;
  }
  for (int c = 0; c < 4; ++c)
    for (int i = 0; i < 9; ++i) basis[c * 9 + i] = A[5 + c][i];
}

// 10x20 constraint matrix from the basis X, Y, Z, W (E = xX + yY + zZ + W).
static void coeff_matrix(const double* basis, double* A) {
  double L[9][4];  // E_ij as linear polynomial [x, y, z, 1]
  for (int i = 0; i < 9; ++i)
    for (int k = 0; k < 4; ++k) L[i][k] = basis[k * 9 + i];
  for (int r = 0; r < 200; ++r) A[r] = 0.0;
  // det(E) = E00 (E11 E22 - E12 E21) - E01 (E10 E22 - E12 E20) + E02 (E10 E21 - E11 E20)
  {
    double q[20], t[20];
    const int cof[3][5] = {{0, 4, 8, 5, 7}, {1, 3, 8, 5, 6}, {2, 3, 7, 4, 6}};
    const double sgn[3] = {1.0, -1.0, 1.0};
    for (int c = 0; c < 3; ++c) {
      mul_ll(L[cof[c][1]], L[cof[c][2]], q);
      mul_ll(L[cof[c][3]], L[cof[c][4]], t);
      for (int k = 0; k < 20; ++k) q[k] -= t[k];
      madd_ql(q, L[cof[c][0]], sgn[c], A);
    }
  }
  // EEt_ij = sum_k E_ik E_jk (quadratic)
  double EEt[9][20];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double q[20];
      for (int k = 0; k < 20; ++k) EEt[i * 3 + j][k] = 0.0;
      for (int k = 0; k < 3; ++k) {
        mul_ll(L[i * 3 + k], L[j * 3 + k], q);
        for (int m = 0; m < 20; ++m) EEt[i * 3 + j][m] += q[m];
      }
    }
  // M = 2 EEt - tr(EEt) I;  rows 1..9: (M E)_ij = sum_k M_ik E_kj
  double Mq[9][20];
  for (int i = 0; i < 9; ++i)
    for (int k = 0; k < 20; ++k) {
      double tr = EEt[0][k] + EEt[4][k] + EEt[8][k];
      Mq[i][k] = 2.0 * EEt[i][k] - ((i % 4 == 0) ? tr : 0.0);
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k) madd_ql(Mq[i * 3 + k], L[k * 3 + j], 1.0, A + (1 + i * 3 + j) * 20);
}

// Gauss-Jordan with partial pivoting: A (10x20) -> R (10x10) = A[:, :10]^-1 A[:, 10:].
static bool reduce_10x20(double* A, double* R) {
  for (int c = 0; c < 10; ++c) {
    int p = c;
    double best = std::fabs(A[c * 20 + c]);
    for (int r = c + 1; r < 10; ++r)
      if (std::fabs(A[r * 20 + c]) > best) { best = std::fabs(A[r * 20 + c]); p = r; }
    if (!(best > 0.0)) return false;
    if (p != c)
      for (int k = 0; k < 20; ++k) std::swap(A[c * 20 + k], A[p * 20 + k]);
    double inv = 1.0 / A[c * 20 + c];
    for (int k = c; k < 20; ++k) A[c * 20 + k] *= inv;
    for (int r = 0; r < 10; ++r) {
      if (r == c) continue;
      double f = A[r * 20 + c];
      if (f == 0.0) continue;
      for (int k = c; k < 20; ++k) A[r * 20 + k] -= f * A[c * 20 + k];
    }
  }
  for (int r = 0; r < 10; ++r)
    for (int k = 0; k < 10; ++k) R[r * 10 + k] = A[r * 20 + 10 + k];
  return true;
}

// ascending-order polynomial product
static void pmul(const double* a, int na, const double* b, int nb, double* c) {
  for (int k = 0; k < na + nb - 1; ++k) c[k] = 0.0;
  for (int i = 0; i < na; ++i)
    for (int j = 0; j < nb; ++j) c[i + j] += a[i] * b[j];
}

// degree-10 polynomial det B(z), c[k] = coefficient of z^k.
static void det_poly(const double* b, double* c) {
  double p[3][3][5];  // ascending coefficients, degree 3 / 3 / 4
  int deg[3] = {3, 3, 4};
  for (int j = 0; j < 3; ++j) {
    const double* br = b + j * 13;
    for (int k = 0; k < 4; ++k) p[j][0][k] = br[3 - k];
    for (int k = 0; k < 4; ++k) p[j][1][k] = br[7 - k];
    for (int k = 0; k < 5; ++k) p[j][2][k] = br[12 - k];
  }
  auto minor = [&](int r1, int c1, int r2, int c2, double* out) {  // p[1][c1] p[2][c2] - p[1][c2] p[2][c1]
    double u[8], v[8];
    pmul(p[r1][c1], deg[c1] + 1, p[r2][c2], deg[c2] + 1, u);
    pmul(p[r1][c2], deg[c2] + 1, p[r2][c1], deg[c1] + 1, v);
    int n = deg[c1] + deg[c2] + 1;
    for (int k = 0; k < n; ++k) out[k] = u[k] - v[k];
    for (int k = n; k < 8; ++k) out[k] = 0.0;
  };
  double m0[8], m1[8], m2[8], t[12];
  minor(1, 1, 2, 2, m0);  // deg 7
  minor(1, 0, 2, 2, m1);  // deg 7
  minor(1, 0, 2, 1, m2);  // deg 6
  for (int k = 0; k < 11; ++k) c[k] = 0.0;
  pmul(p[0][0], 4, m0, 8, t);
  for (int k = 0; k < 11; ++k) c[k] += t[k];
  pmul(p[0][1], 4, m1, 8, t);
  for (int k = 0; k < 11; ++k) c[k] -= t[k];
  pmul(p[0][2], 5, m2, 7, t);
  for (int k = 0; k < 11; ++k) c[k] += t[k];
}

struct Cx {
  double re, im;
};
static inline Cx cmul(Cx a, Cx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
static inline Cx cdiv(Cx a, Cx b) {
  double t = 1. / (b.re * b.re + b.im * b.im);
  return {(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
}

// solvePoly: Durand-Kerner; returns the degree actually solved (leading |c| <= DBL_EPSILON trimmed).
static int solve_poly(const double* c, Cx* roots) {
  int n = 10;
  while (n > 1 && std::fabs(c[n]) <= DBL_EPSILON) --n;
  Cx p{1, 0}, r{1, 1};
  for (int i = 0; i < n; ++i) {
    roots[i] = p;
    p = cmul(p, r);
  }
  for (int iter = 0; iter < 300; ++iter) {
    double maxDiff = 0;
    for (int i = 0; i < n; ++i) {
      p = roots[i];
      Cx num{c[n], 0}, den{c[n], 0};
      for (int j = 0; j < n; ++j) {
        num = cmul(num, p);
        num.re += c[n - j - 1];
        if (j != i) {
          Cx d{p.re - roots[j].re, p.im - roots[j].im};
          if (d.re != 0 || d.im != 0) den = cmul(den, d);
        }
      }
      num = cdiv(num, den);
      roots[i] = {p.re - num.re, p.im - num.im};
      maxDiff = std::max(maxDiff, std::sqrt(num.re * num.re + num.im * num.im));
    }
    if (maxDiff <= 0) break;
  }
  return n;
}

// unit null vector of a rank-2 3x3 matrix: the longest cross product of two rows.
static void null3(const double* B, double* v) {
  const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
  v[0] = 0.0; v[1] = 0.0; v[2] = 0.0;
  double best = -1.0;
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
  double nrm = std::sqrt(best);
  if (nrm > 0.0)
    for (int i = 0; i < 3; ++i) v[i] /= nrm;
}

// EMEstimatorCallback::runKernel on 5 normalised correspondences (x1[2i], x1[2i+1]) etc.
// Writes up to 10 models (9 doubles each, row-major E) and returns their count.
static int five_point(const double* x1, const double* x2, double* models) {
  double Q[45];
  for (int i = 0; i < 5; ++i) {
    double a = x1[2 * i], b = x1[2 * i + 1], c = x2[2 * i], d = x2[2 * i + 1];
    double* q = Q + i * 9;
    q[0] = a * c; q[1] = b * c; q[2] = c;
    q[3] = a * d; q[4] = b * d; q[5] = d;
    q[6] = a; q[7] = b; q[8] = 1.0;
  }
  double basis[36], A[200], R[100];
  null_space_5x9(Q, basis);
  coeff_matrix(basis, A);
  if (!reduce_10x20(A, R)) return 0;
  double b[39];
  for (int i = 0; i < 3; ++i) {
    const double* a1 = R + (2 * i + 4) * 10;
    const double* a2 = R + (2 * i + 5) * 10;
    double r1[13] = {0}, r2[13] = {0};
    for (int k = 0; k < 3; ++k) { r1[1 + k] = a1[k]; r1[5 + k] = a1[3 + k]; }
    for (int k = 0; k < 4; ++k) r1[9 + k] = a1[6 + k];
    for (int k = 0; k < 3; ++k) { r2[k] = a2[k]; r2[4 + k] = a2[3 + k]; }
    for (int k = 0; k < 4; ++k) r2[8 + k] = a2[6 + k];
    for (int k = 0; k < 13; ++k) b[i * 13 + k] = r1[k] - r2[k];
  }
  double c[11];
  det_poly(b, c);
  Cx roots[10];
  int nr = solve_poly(c, roots);
  int count = 0;
  for (int i = 0; i < nr; ++i) {
    if (std::fabs(roots[i].im) > 1e-10) continue;
    double z1 = roots[i].re, z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
    double bz[9];
    for (int j = 0; j < 3; ++j) {
      const double* br = b + j * 13;
      bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
      bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
      bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
    }
    double v[3];
    null3(bz, v);
    if (std::fabs(v[2]) < 1e-10) continue;
    double x = v[0] / v[2], y = v[1] / v[2];
    double* e = models + count * 9;
    double n2 = 0.0;
    for (int k = 0; k < 9; ++k) {
      e[k] = basis[k] * x + basis[9 + k] * y + basis[18 + k] * z1 + basis[27 + k];
      n2 += e[k] * e[k];
    }
    double nrm = std::sqrt(n2);
    for (int k = 0; k < 9; ++k) e[k] /= nrm;
    ++count;
  }
  return count;
}

// EMEstimatorCallback::computeError + findInliers
static int find_inliers(const double* E, const double* x1, const double* x2, int n, float thr2, uint8_t* mask) {
  int good = 0;
  for (int i = 0; i < n; ++i) {
    double a1 = x1[2 * i], b1 = x1[2 * i + 1], a2 = x2[2 * i], b2 = x2[2 * i + 1];
    double Ex0 = E[0] * a1 + E[1] * b1 + E[2];
    double Ex1 = E[3] * a1 + E[4] * b1 + E[5];
    double Ex2 = E[6] * a1 + E[7] * b1 + E[8];
    double Et0 = E[0] * a2 + E[3] * b2 + E[6];
    double Et1 = E[1] * a2 + E[4] * b2 + E[7];
    double x2tEx1 = a2 * Ex0 + b2 * Ex1 + Ex2;
    double den = Ex0 * Ex0 + Ex1 * Ex1 + Et0 * Et0 + Et1 * Et1;
    float err = (float)(x2tEx1 * x2tEx1 / den);
    int f = err <= thr2;
    if (mask) mask[i] = (uint8_t)f;
    good += f;
  }
  return good;
}

// ------------------------------------------------------------------ recoverPose
// Symmetric 3x3 Jacobi eigen-decomposition: S = V diag(w) V^T, w descending.
static void eig3(const double* Sin, double* w, double* V) {
  double S[9];
  std::memcpy(S, Sin, sizeof(S));
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = S[1] * S[1] + S[2] * S[2] + S[5] * S[5];
    if (off == 0.0) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double apq = S[p * 3 + q];
        if (apq == 0.0) continue;
        double theta = (S[q * 3 + q] - S[p * 3 + p]) / (2.0 * apq);
        double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; ++k) {  // S <- S J (columns p, q)
          double skp = S[k * 3 + p], skq = S[k * 3 + q];
          S[k * 3 + p] = c * skp - s * skq;
          S[k * 3 + q] = s * skp + c * skq;
        }
        for (int k = 0; k < 3; ++k) {  // S <- J^T S (rows p, q)
          double spk = S[p * 3 + k], sqk = S[q * 3 + k];
          S[p * 3 + k] = c * spk - s * sqk;
          S[q * 3 + k] = s * spk + c * sqk;
        }
        for (int k = 0; k < 3; ++k) {
          double vkp = V[k * 3 + p], vkq = V[k * 3 + q];
          V[k * 3 + p] = c * vkp - s * vkq;
          V[k * 3 + q] = s * vkp + c * vkq;
        }
      }
  }
  double d[3] = {S[0], S[4], S[8]};
  int o[3] = {0, 1, 2};
  for (int i = 0; i < 3; ++i)  // stable selection sort, descending
    for (int j = i + 1; j < 3; ++j)
      if (d[o[j]] > d[o[i]]) std::swap(o[i], o[j]);
  double Vs[9];
  for (int j = 0; j < 3; ++j) {
    w[j] = d[o[j]];
    for (int k = 0; k < 3; ++k) Vs[k * 3 + j] = V[k * 3 + o[j]];
  }
  std::memcpy(V, Vs, sizeof(Vs));
}

static inline void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// decomposeEssentialMat: E = U diag(s,s,0) V^T with U, V proper rotations.
static void decompose_essential(const double* E, double* R1, double* R2, double* t) {
  double S[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += E[k * 3 + i] * E[k * 3 + j];
      S[i * 3 + j] = s;
    }
  double w[3], V[9];
  eig3(S, w, V);
  double v0[3] = {V[0], V[3], V[6]}, v1[3] = {V[1], V[4], V[7]}, v2[3];
  cross3(v0, v1, v2);
  double u0[3], u1[3], u2[3];
  for (int i = 0; i < 3; ++i) {
    u0[i] = E[i * 3] * v0[0] + E[i * 3 + 1] * v0[1] + E[i * 3 + 2] * v0[2];
    u1[i] = E[i * 3] * v1[0] + E[i * 3 + 1] * v1[1] + E[i * 3 + 2] * v1[2];
  }
  double n0 = std::sqrt(u0[0] * u0[0] + u0[1] * u0[1] + u0[2] * u0[2]);
  for (int i = 0; i < 3; ++i) u0[i] /= n0;
  double d = u0[0] * u1[0] + u0[1] * u1[1] + u0[2] * u1[2];
  for (int i = 0; i < 3; ++i) u1[i] -= d * u0[i];
  double n1 = std::sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
  for (int i = 0; i < 3; ++i) u1[i] /= n1;
  cross3(u0, u1, u2);
  // W = [[0,1,0],[-1,0,0],[0,0,1]]: U W = [-u1, u0, u2], U W^T = [u1, -u0, u2]
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double vj[3] = {v0[j], v1[j], v2[j]};
      R1[i * 3 + j] = -u1[i] * vj[0] + u0[i] * vj[1] + u2[i] * vj[2];
      R2[i * 3 + j] = u1[i] * vj[0] - u0[i] * vj[1] + u2[i] * vj[2];
    }
  for (int i = 0; i < 3; ++i) t[i] = u2[i];
}

// One-sided Jacobi: unit right singular vector of the smallest singular value of A (4x4).
static void null4(const double* Ain, double* x) {
  double A[16], V[16];
  std::memcpy(A, Ain, sizeof(A));
  for (int i = 0; i < 16; ++i) V[i] = (i % 5 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool rotated = false;
    for (int p = 0; p < 3; ++p)
      for (int q = p + 1; q < 4; ++q) {
        double a = 0, b = 0, g = 0;
        for (int i = 0; i < 4; ++i) {
          a += A[i * 4 + p] * A[i * 4 + p];
          b += A[i * 4 + q] * A[i * 4 + q];
          g += A[i * 4 + p] * A[i * 4 + q];
        }
        if (!(std::fabs(g) > 1e-15 * std::sqrt(a * b))) continue;
        rotated = true;
        double zeta = (b - a) / (2.0 * g);
        double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
        double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
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
  for (int j = 0; j < 4; ++j) {
    double n2 = 0;
    for (int i = 0; i < 4; ++i) n2 += A[i * 4 + j] * A[i * 4 + j];
    if (j == 0 || n2 < bn) { bn = n2; best = j; }
  }
  for (int i = 0; i < 4; ++i) x[i] = V[i * 4 + best];
}

// cheirality test of one point against P = [R | t] (recoverPose's mask for one P).
static int cheiral(const double* R, const double* t, double a1, double b1, double a2, double b2, double dist) {
  double A[16] = {-1.0, 0.0, a1, 0.0, 0.0, -1.0, b1, 0.0};
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

static int recover_pose(const double* E, const double* x1, const double* x2, int n, double dist, double* R,
                        double* t) {
  double R1[9], R2[9], tt[3], tn[3];
  decompose_essential(E, R1, R2, tt);
  for (int i = 0; i < 3; ++i) tn[i] = -tt[i];
  int g[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    double a1 = x1[2 * i], b1 = x1[2 * i + 1], a2 = x2[2 * i], b2 = x2[2 * i + 1];
    g[0] += cheiral(R1, tt, a1, b1, a2, b2, dist);
    g[1] += cheiral(R2, tt, a1, b1, a2, b2, dist);
    g[2] += cheiral(R1, tn, a1, b1, a2, b2, dist);
    g[3] += cheiral(R2, tn, a1, b1, a2, b2, dist);
  }
  int sel;
  if (g[0] >= g[1] && g[0] >= g[2] && g[0] >= g[3]) sel = 0;
  else if (g[1] >= g[0] && g[1] >= g[2] && g[1] >= g[3]) sel = 1;
  else if (g[2] >= g[0] && g[2] >= g[1] && g[2] >= g[3]) sel = 2;
  else sel = 3;
  std::memcpy(R, (sel & 1) ? R2 : R1, 9 * sizeof(double));
  std::memcpy(t, sel < 2 ? tt : tn, 3 * sizeof(double));
  return g[sel];
}

static void normalise(const float* p, int n, double f, double cx, double cy, std::vector<double>& x) {
  x.resize(2 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    x[2 * i] = ((double)p[2 * i] - cx) / f;
    x[2 * i + 1] = ((double)p[2 * i + 1] - cy) / f;
  }
}

}  // namespace em

extern "C" {

// 5-point kernel on 5 normalised correspondences; returns the model count.
int ref_five_point(const double* x1, const double* x2, double* models) { return em::five_point(x1, x2, models); }

// findEssentialMat(p1, p2, focal, pp, RANSAC, prob, threshold, maxIters).
// Returns 1 (E, mask written), 0 RANSAC found nothing, -1 fewer than 5 points,
// -2 exactly 5 points with several solutions (E would be 3k x 3; recoverPose raises).
int ref_find_essential(const float* p1, const float* p2, int n, double focal, double cx, double cy, double prob,
                       double threshold, int max_iters, double* E, uint8_t* mask, int32_t* n_iters_out,
                       int32_t* best_good_out) {
  if (n_iters_out) *n_iters_out = 0;
  if (best_good_out) *best_good_out = 0;
  if (n < 5) return -1;
  std::vector<double> x1, x2;
  em::normalise(p1, n, focal, cx, cy, x1);
  em::normalise(p2, n, focal, cx, cy, x2);
  double thr = threshold / ((focal + focal) / 2);
  float thr2 = (float)(thr * thr);
  double models[90];
  if (n == 5) {
    int nm = em::five_point(x1.data(), x2.data(), models);
    if (nm <= 0) return 0;
    if (nm > 1) return -2;
    std::memcpy(E, models, 9 * sizeof(double));
    for (int i = 0; i < n; ++i) mask[i] = 1;
    if (best_good_out) *best_good_out = 5;
    return 1;
  }
  std::vector<uint8_t> m(n), best(n, 0);
  int maxGood = 0, niters = std::max(max_iters, 1), iter;
  em::RNG rng(~0ull);
  for (iter = 0; iter < niters; ++iter) {
    int idx[5];
    double s1[10], s2[10];
    for (int i = 0; i < 5; ++i) {
      int j;
      for (;;) {
        j = rng.uniform(0, n);
        bool dup = false;
        for (int k = 0; k < i; ++k) dup |= idx[k] == j;
        if (!dup) break;
      }
      idx[i] = j;
      s1[2 * i] = x1[2 * j]; s1[2 * i + 1] = x1[2 * j + 1];
      s2[2 * i] = x2[2 * j]; s2[2 * i + 1] = x2[2 * j + 1];
    }
    int nm = em::five_point(s1, s2, models);
    for (int k = 0; k < nm; ++k) {
      int good = em::find_inliers(models + 9 * k, x1.data(), x2.data(), n, thr2, m.data());
      if (good > std::max(maxGood, 4)) {
        best.swap(m);
        std::memcpy(E, models + 9 * k, 9 * sizeof(double));
        maxGood = good;
        niters = em::update_num_iters(prob, (double)(n - good) / n, 5, niters);
      }
    }
  }
  if (n_iters_out) *n_iters_out = iter;
  if (best_good_out) *best_good_out = maxGood;
  if (maxGood <= 0) return 0;
  std::memcpy(mask, best.data(), n);
  return 1;
}

// recoverPose(E, p1, p2, focal, pp) with distanceThresh; returns the cheirality count.
int ref_recover_pose(const double* E, const float* p1, const float* p2, int n, double focal, double cx, double cy,
                     double dist, double* R, double* t) {
  std::vector<double> x1, x2;
  em::normalise(p1, n, focal, cx, cy, x1);
  em::normalise(p2, n, focal, cx, cy, x2);
  return em::recover_pose(E, x1.data(), x2.data(), n, dist, R, t);
}

void ref_decompose_essential(const double* E, double* R1, double* R2, double* t) {
  em::decompose_essential(E, R1, R2, t);
}

}  // extern "C"
