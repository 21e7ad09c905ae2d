// Pose stage for gfx950 — replaces ros_ws/src/stereo_slam.py:262-303:
//   depth / back-projection of the matched previous-frame keypoints (:262-289), then
//   cv2.solvePnPRansac(points3D, mkpts1_l, K0, dist_l, 1.0, 0.99, 1000, ITERATIVE) and
//   cv2.Rodrigues -> T (:294-303).
//
// k_backproject  one thread per match, float32 arithmetic in NumPy 1.x order
//                (the reference environment's value-based casting),
//                ordered compaction of 0.1 < Z < 1000 (block scan), one block per frame.
// k_pnp          one wavefront per frame.  RANSAC iterations are evaluated 64 at a time:
//                lane 0 draws the subsets with OpenCV's RNG(-1) (the draws depend only on
//                the point count), every lane solves EPnP for its subset and scores it over
//                all points; lane 0 then replays OpenCV's sequential acceptance rule
//                (goodCount > max(best, 4), adaptive niters) over the chunk, so the
//                winning hypothesis and the iteration count are those of the serial loop.
//                Refinement: DLT (or homography for planar sets) + Levenberg-Marquardt
//                (CvLevMarq: lambda 1e-3, 20 iterations, eps FLT_EPSILON) with the
//                per-point Jacobian rows accumulated across lanes.
// All pose math is fp64 (as in OpenCV); compiled with -ffp-contract=off.
#include <cfloat>
#include <cstdlib>
#include <type_traits>

#include "fvo_device.h"
#include "ransac.h"

namespace {

constexpr int kChunk = 64;

// ------------------------------------------------------------------ back-projection
struct CamF {
  double fx, fy, cx, cy, fxB;
};

__global__ void k_backproject(const int16_t* __restrict__ disp, const float* __restrict__ kp0,
                              const float* __restrict__ kp1, const int32_t* __restrict__ matches,
                              const int32_t* __restrict__ nmatch, int W, int H, int cap, CamF K,
                              float* __restrict__ P3, float* __restrict__ p2, int32_t* __restrict__ npts) {
  const int b = blockIdx.x;
  int n = nmatch[b];
  n = n < 0 ? 0 : (n > cap ? cap : n);
  __shared__ int s_w[16];
  __shared__ int s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  const float fxB = (float)K.fxB, fcx = (float)K.cx, fcy = (float)K.cy, ffx = (float)K.fx, ffy = (float)K.fy;
  const float lo = (float)0.1, hi = 1000.f;
  for (int base = 0; base < n; base += blockDim.x) {
    int i = base + threadIdx.x;
    bool keep = false;
    float X = 0, Y = 0, Z = 0, u = 0, v = 0;
    if (i < n) {
      const int32_t* m = matches + ((int64_t)b * cap + i) * 3;
      const float* a = kp0 + ((int64_t)b * cap + m[0]) * FVO_KP_STRIDE;
      const float* c = kp1 + ((int64_t)b * cap + m[1]) * FVO_KP_STRIDE;
      float x = a[0], y = a[1];
      int xi = (int)x, yi = (int)y;
      xi = min(max(xi, 0), W - 1);
      yi = min(max(yi, 0), H - 1);
      float d = (float)disp[((int64_t)b * H + yi) * W + xi] / 16.f;
      if (d == 0.0f) d = lo;
      if (d == -1.0f) d = lo;
      Z = fxB / d;
      X = ((x - fcx) / ffx) * Z;
      Y = ((y - fcy) / ffy) * Z;
      keep = (Z > lo) && (Z < hi);
      u = c[0];
      v = c[1];
    }
    unsigned long long mk = __ballot(keep);
    int pre = __popcll(mk & ((1ull << wave_lane()) - 1ull));
    if (wave_lane() == 0) s_w[threadIdx.x >> 6] = __popcll(mk);
    __syncthreads();
    int wpre = 0, tot = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
      if (k < (int)(threadIdx.x >> 6)) wpre += s_w[k];
      tot += s_w[k];
    }
    if (keep) {
      int o = s_carry + wpre + pre;
      float* P = P3 + ((int64_t)b * cap + o) * 3;
      P[0] = X;
      P[1] = Y;
      P[2] = Z;
      p2[((int64_t)b * cap + o) * 2] = u;
      p2[((int64_t)b * cap + o) * 2 + 1] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) s_carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) npts[b] = s_carry;
}

// ------------------------------------------------------------------ small fp64 linear algebra
// Stable insertion sort of w descending (ord[] as dsvd's loop builds it) with every index
// static: position j holds (sw[j], so[j]); the while loop becomes a predicated shift.
template <int N>
__device__ __forceinline__ void sort_desc(const double* w, double* sw, int* so) {
#pragma unroll
  for (int j = 0; j < N; ++j) { sw[j] = w[j]; so[j] = j; }
#pragma unroll
  for (int i = 1; i < N; ++i) {
    const double wk = sw[i];
    const int k = so[i];
    bool mv = true;
#pragma unroll
    for (int j = i; j > 0; --j) {
      const bool sh = mv && sw[j - 1] < wk;
      const double nw = sh ? sw[j - 1] : (mv ? wk : sw[j]);
      const int no = sh ? so[j - 1] : (mv ? k : so[j]);
      sw[j] = nw;
      so[j] = no;
      mv = sh;
    }
    if (mv) { sw[0] = wk; so[0] = k; }
  }
}

// One-sided Jacobi on u (m x n row-major, starts as A) accumulating v (n x n, starts as I);
// the columns of u end up as U diag(W) in unsorted order.
template <int M, int N>
__device__ __forceinline__ void dsvd_jacobi(double (&u)[M * N], double (&v)[N * N]) {
  #pragma unroll
  for (int i = 0; i < N * N; ++i) v[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    #pragma unroll
    for (int p = 0; p < N - 1; ++p)
      #pragma unroll
      for (int q = p + 1; q < N; ++q) {
        double a = 0, bb = 0, g = 0;
        #pragma unroll
        for (int i = 0; i < M; ++i) {
          double up = u[i * N + p], uq = u[i * N + q];
          a += up * up;
          bb += uq * uq;
          g += up * uq;
        }
        if (g == 0.0 || fabs(g) <= 1e-300) continue;
        double rel = fabs(g) / sqrt(a * bb);
        off = fmax(off, rel);
        if (rel < 1e-15) continue;
        double zeta = (bb - a) / (2.0 * g);
        double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
        #pragma unroll
        for (int i = 0; i < M; ++i) {
          double up = u[i * N + p], uq = u[i * N + q];
          u[i * N + p] = c * up - s * uq;
          u[i * N + q] = s * up + c * uq;
        }
        #pragma unroll
        for (int i = 0; i < N; ++i) {
          double vp = v[i * N + p], vq = v[i * N + q];
          v[i * N + p] = c * vp - s * vq;
          v[i * N + q] = s * vp + c * vq;
        }
      }
    if (off < 1e-15) break;
  }
}

// Column norms of u sorted descending (stable): sw = W, ord = source column of each.
template <int M, int N>
__device__ __forceinline__ void dsvd_order(const double (&u)[M * N], double* sw, int* ord) {
  double w[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) s += u[i * N + j] * u[i * N + j];
    w[j] = sqrt(s);
  }
  sort_desc<N>(w, sw, ord);
}

// column j (runtime) of a register matrix by compile-time selects (a runtime column index
// would put the matrix in scratch for the whole decomposition)
template <int R, int N>
__device__ __forceinline__ double dsel(const double (&m)[R * N], int i, int j) {
  double x = 0.0;
#pragma unroll
  for (int c = 0; c < N; ++c) x = (c == j) ? m[i * N + c] : x;
  return x;
}

// A (m x n row-major, m >= n) = U diag(W) V^T, W descending (one-sided Jacobi).
template <int M, int N>
__device__ void dsvd(const double* A, double* W, double* U, double* V) {
  double u[M * N], v[N * N];
  #pragma unroll
  for (int i = 0; i < M * N; ++i) u[i] = A[i];
  dsvd_jacobi<M, N>(u, v);
  double sw[N];
  int ord[N];
  dsvd_order<M, N>(u, sw, ord);
#pragma unroll
  for (int jj = 0; jj < N; ++jj) {
    const int j = ord[jj];
    const double wj = sw[jj];
    W[jj] = wj;
    const double inv = wj > 0 ? 1.0 / wj : 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) U[i * N + jj] = dsel<M, N>(u, i, j) * inv;
#pragma unroll
    for (int i = 0; i < N; ++i) V[i * N + jj] = dsel<N, N>(v, i, j);
  }
}

// dsvd with caller-provided work arrays (e.g. LDS for the single-lane 12x12 DLT SVD of the
// refinement: no scratch).  Same operations as dsvd.
template <int M, int N>
__device__ void dsvd_ws(const double* A, double* W, double* U, double* V, double* u, double* v) {
  double w[N];
  for (int i = 0; i < M * N; ++i) u[i] = A[i];
  for (int i = 0; i < N * N; ++i) v[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < N - 1; ++p)
      for (int q = p + 1; q < N; ++q) {
        double a = 0, bb = 0, g = 0;
        for (int i = 0; i < M; ++i) {
          double up = u[i * N + p], uq = u[i * N + q];
          a += up * up;
          bb += uq * uq;
          g += up * uq;
        }
        if (g == 0.0 || fabs(g) <= 1e-300) continue;
        double rel = fabs(g) / sqrt(a * bb);
        off = fmax(off, rel);
        if (rel < 1e-15) continue;
        double zeta = (bb - a) / (2.0 * g);
        double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
        for (int i = 0; i < M; ++i) {
          double up = u[i * N + p], uq = u[i * N + q];
          u[i * N + p] = c * up - s * uq;
          u[i * N + q] = s * up + c * uq;
        }
        for (int i = 0; i < N; ++i) {
          double vp = v[i * N + p], vq = v[i * N + q];
          v[i * N + p] = c * vp - s * vq;
          v[i * N + q] = s * vp + c * vq;
        }
      }
    if (off < 1e-15) break;
  }
  int ord[N];
  for (int j = 0; j < N; ++j) {
    double s = 0;
    for (int i = 0; i < M; ++i) s += u[i * N + j] * u[i * N + j];
    w[j] = sqrt(s);
    ord[j] = j;
  }
  for (int i = 1; i < N; ++i) {
    int k = ord[i], j = i;
    while (j > 0 && w[ord[j - 1]] < w[k]) { ord[j] = ord[j - 1]; --j; }
    ord[j] = k;
  }
  for (int jj = 0; jj < N; ++jj) {
    int j = ord[jj];
    W[jj] = w[j];
    double inv = w[j] > 0 ? 1.0 / w[j] : 0.0;
    for (int i = 0; i < M; ++i) U[i * N + jj] = u[i * N + j] * inv;
    for (int i = 0; i < N; ++i) V[i * N + jj] = v[i * N + j];
  }
}

// SPD 6x6 solve by Cholesky for the LM step (JtJ with the (1 + lambda) diagonal).  Returns
// false when a pivot is not clearly positive (pivot^2 below 1e-12 of the largest diagonal
// entry): the caller then takes OpenCV's DECOMP_SVD path (dsolve), which also handles the
// rank-deficient case.  On well-conditioned systems both give the same step to rounding.
__device__ bool chol_solve6(const double* A, const double* b, double* x) {
  double L[6][6], y[6], dmax = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) dmax = fmax(dmax, A[i * 6 + i]);
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      double s = A[i * 6 + j];
#pragma unroll
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (!(s > 1e-12 * dmax)) return false;
        L[i][i] = sqrt(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return true;
}

// x = V diag(1/W) U^T b over the singular values above DBL_EPSILON * max(m, n) * W[0]
// (cv::solve DECOMP_SVD); U and V are read from the Jacobi's u and v in place -- the same
// products and sums as forming them first, without holding both copies.
template <int M, int N>
__device__ void dsolve(const double* A, const double* b, double* x) {
  double u[M * N], v[N * N], tmp[N];
#pragma unroll
  for (int i = 0; i < M * N; ++i) u[i] = A[i];
  dsvd_jacobi<M, N>(u, v);
  double sw[N];
  int ord[N];
  dsvd_order<M, N>(u, sw, ord);
  const double thr = DBL_EPSILON * (M > N ? M : N) * sw[0];
#pragma unroll
  for (int jj = 0; jj < N; ++jj) {
    const int j = ord[jj];
    const double wj = sw[jj];
    tmp[jj] = 0.0;
    if (wj <= thr) continue;
    const double inv = wj > 0 ? 1.0 / wj : 0.0;
    double s = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) s += (dsel<M, N>(u, i, j) * inv) * b[i];
    tmp[jj] = s / wj;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double s = 0;
#pragma unroll
    for (int jj = 0; jj < N; ++jj) s += dsel<N, N>(v, i, ord[jj]) * tmp[jj];
    x[i] = s;
  }
}

__device__ double ddet3(const double* R) {
  return R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) + R[2] * (R[3] * R[7] - R[4] * R[6]);
}

// ------------------------------------------------------------------ camera / Rodrigues
struct Cam {
  double fx, fy, cx, cy, k[5];
};

__device__ void rod_r2R(const double* r, double* R, double* J) {
  double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < DBL_EPSILON) {
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (J) {
      const double J0[27] = {0, 0, 0, 0, 0, 1, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 1, 0, -1, 0, 0, 0, 0, 0};
      for (int i = 0; i < 27; ++i) J[i] = J0[i];
    }
    return;
  }
  double c = cos(th), s = sin(th), c1 = 1.0 - c, it = 1.0 / th;
  double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int k = 0; k < 9; ++k) R[k] = c * I[k] + c1 * rrt[k] + s * rx[k];
  if (J) {
    double drrt[27] = {x + x, y, z, y, 0, 0, z, 0, 0, 0, x, 0, x, y + y, z, 0, z, 0, 0, 0, x, 0, 0, y, x, y, z + z};
    const double drx[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 1, 0, 0, 0, 0, 0};
    for (int i = 0; i < 3; ++i) {
      double ri = i == 0 ? x : i == 1 ? y : z;
      double a0 = -s * ri, a1 = (s - 2 * c1 * it) * ri, a2 = c1 * it, a3 = (c - s * it) * ri, a4 = s * it;
      for (int k = 0; k < 9; ++k)
        J[i * 9 + k] = a0 * I[k] + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * rx[k] + a4 * drx[i * 9 + k];
    }
  }
}

__device__ void rod_R2r(const double* Rin, double* r) {
  double W[3], U[9], V[9], R[9];
  dsvd<3, 3>(Rin, W, U, V);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i * 3 + j] = U[i * 3] * V[j * 3] + U[i * 3 + 1] * V[j * 3 + 1] + U[i * 3 + 2] * V[j * 3 + 2];
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  double th = acos(c);
  if (s < 1e-5) {
    if (c > 0) {
      rx = ry = rz = 0;
    } else {
      double t = (R[0] + 1) * 0.5;
      rx = sqrt(fmax(t, 0.));
      t = (R[4] + 1) * 0.5;
      ry = sqrt(fmax(t, 0.)) * (R[1] < 0 ? -1. : 1.);
      t = (R[8] + 1) * 0.5;
      rz = sqrt(fmax(t, 0.)) * (R[2] < 0 ? -1. : 1.);
      if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
      th /= sqrt(rx * rx + ry * ry + rz * rz);
      rx *= th; ry *= th; rz *= th;
    }
  } else {
    double vth = 1 / (2 * s);
    vth *= th;
    rx *= vth; ry *= vth; rz *= vth;
  }
  r[0] = rx; r[1] = ry; r[2] = rz;
}

// projectPoints (k1 k2 p1 p2 k3) for one point; J (2x6) optional.
__device__ void dproject(const Cam& K, const double* R, const double* dRdr, const double* t, const double* M,
                         double* uv, double* J) {
  double X = M[0], Y = M[1], Z = M[2];
  double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
  double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
  double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
  z = z ? 1. / z : 1;
  x *= z;
  y *= z;
  const double* k = K.k;
  double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
  double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
  double cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
  double xd = x * cdist + k[2] * a1 + k[3] * a2;
  double yd = y * cdist + k[2] * a3 + k[3] * a1;
  uv[0] = xd * K.fx + K.cx;
  uv[1] = yd * K.fy + K.cy;
  if (!J) return;
  for (int j = 0; j < 6; ++j) {
    double dxd, dyd;
    if (j < 3) {
      double dx0 = X * dRdr[j * 9 + 0] + Y * dRdr[j * 9 + 1] + Z * dRdr[j * 9 + 2];
      double dy0 = X * dRdr[j * 9 + 3] + Y * dRdr[j * 9 + 4] + Z * dRdr[j * 9 + 5];
      double dz0 = X * dRdr[j * 9 + 6] + Y * dRdr[j * 9 + 7] + Z * dRdr[j * 9 + 8];
      dxd = z * (dx0 - x * dz0);
      dyd = z * (dy0 - y * dz0);
    } else {
      dxd = j == 3 ? z : j == 4 ? 0.0 : -x * z;
      dyd = j == 3 ? 0.0 : j == 4 ? z : -y * z;
    }
    double dr2 = 2 * x * dxd + 2 * y * dyd;
    double dcd = k[0] * dr2 + 2 * k[1] * r2 * dr2 + 3 * k[4] * r4 * dr2;
    double da1 = 2 * (x * dyd + y * dxd);
    J[j] = K.fx * (dxd * cdist + x * dcd + k[2] * da1 + k[3] * (dr2 + 4 * x * dxd));
    J[6 + j] = K.fy * (dyd * cdist + y * dcd + k[2] * (dr2 + 4 * y * dyd) + k[3] * da1);
  }
}

__device__ void dundistort(const Cam& K, double u, double v, double* xy) {
  const double ifx = 1. / K.fx, ify = 1. / K.fy;
  double x = (u - K.cx) * ifx, y = (v - K.cy) * ify;
  double x0 = x, y0 = y;
  const double* k = K.k;
  for (int j = 0; j < 5; ++j) {
    double r2 = x * x + y * y;
    double icdist = 1. / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
    if (icdist < 0) {
      x = (u - K.cx) * ifx;
      y = (v - K.cy) * ify;
      break;
    }
    double dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
    double dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
    x = (x0 - dx) * icdist;
    y = (y0 - dy) * icdist;
  }
  xy[0] = x;
  xy[1] = y;
}

// dsvd<12,12> specialised for EPnP: only U is consumed (the rows ut[8..11] of U^T, i.e. the
// singular vectors of the four smallest singular values), so V is not accumulated; the
// operations on u, the norms, the stable descending order and the scaling are exactly those
// of dsvd (and of the oracle's svd()).  Run by an 8-lane group, u[144] (row-major) in LDS
// shared by the group.  The
// cyclic pair order (0,1), (0,2), ..., (10,11) is replaced by its anti-diagonals p + q = 2..21:
// a pair's columns are touched, before and after it, by exactly the same pairs in the same
// order in both orders (pair (p,q) follows (p,q-1) and (p-1,q) and nothing else on p or q
// sits between), and the pairs of one anti-diagonal share no column, so the group rotates
// them at once -- bit-identical to the serial sweep, with 21 dependent steps instead of 66.
// The column norms, the sort and the output (out[r * 12 + i], r = 0..3) are lane 0's.
// The sweeps of dsvd<12,12> (cyclic one-sided Jacobi on u, and on v when V is wanted) by an
// 8-lane group on row-major [144] arrays in LDS.
template <bool WITH_V>
__device__ __forceinline__ void jacobi12_sweeps_group(double* __restrict__ u, double* __restrict__ v, int l) {
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
#pragma nounroll
    for (int d = 1; d <= 21; ++d) {
      const int p0 = d > 11 ? d - 11 : 0;
      const int cnt = (d - 1) / 2 - p0 + 1;
      if (l < cnt) {
        const int p = p0 + l, q = d - p;
        double a = 0, bb = 0, g = 0;
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          const double up = u[i * 12 + p], uq = u[i * 12 + q];
          a += up * up;
          bb += uq * uq;
          g += up * uq;
        }
        // the rotation is formed before the tests that gate it, so its sqrt / div chain
        // overlaps the one of rel (same expressions: the values used are unchanged)
        const double zeta = (bb - a) / (2.0 * g);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
        if (!(g == 0.0 || fabs(g) <= 1e-300)) {
          const double rel = fabs(g) / sqrt(a * bb);
          off = fmax(off, rel);
          if (!(rel < 1e-15)) {
#pragma unroll
            for (int i = 0; i < 12; ++i) {
              const double up = u[i * 12 + p], uq = u[i * 12 + q];
              u[i * 12 + p] = c * up - sn * uq;
              u[i * 12 + q] = sn * up + c * uq;
            }
            if (WITH_V)
#pragma unroll
              for (int i = 0; i < 12; ++i) {
                const double vp = v[i * 12 + p], vq = v[i * 12 + q];
                v[i * 12 + p] = c * vp - sn * vq;
                v[i * 12 + q] = sn * vp + c * vq;
              }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) off = fmax(off, __shfl_xor(off, o, 8));
    if (off < 1e-15) break;
  }
}

// The same sweeps with V by a whole wave (the refinement's single DLT per frame, where the
// 8-lane group's sweeps were the kernel's critical path: 60 sweeps x 21 dependent steps).
// 8 lanes per pair of an anti-diagonal: the pair's 8 lanes form its three dot products
// redundantly (the same sequential sums, hence the same rotation), then each rotates rows
// sl and sl + 8 of u and v -- every element gets the group version's arithmetic.
__device__ void jacobi12_sweeps_wave(double* __restrict__ u, double* __restrict__ v) {
  const int lane = threadIdx.x & 63, pr = lane >> 3, sl = lane & 7;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
#pragma nounroll
    for (int d = 1; d <= 21; ++d) {
      const int p0 = d > 11 ? d - 11 : 0;
      const int cnt = (d - 1) / 2 - p0 + 1;
      if (pr < cnt) {
        const int p = p0 + pr, q = d - p;
        double a = 0, bb = 0, g = 0;
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          const double up = u[i * 12 + p], uq = u[i * 12 + q];
          a += up * up;
          bb += uq * uq;
          g += up * uq;
        }
        // the rotation is formed before the tests that gate it, so its sqrt / div chain
        // overlaps the one of rel (same expressions: the values used are unchanged)
        const double zeta = (bb - a) / (2.0 * g);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
        if (!(g == 0.0 || fabs(g) <= 1e-300)) {
          const double rel = fabs(g) / sqrt(a * bb);
          off = fmax(off, rel);
          if (!(rel < 1e-15)) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const int i = sl + 8 * k;
              if (i < 12) {
                const double up = u[i * 12 + p], uq = u[i * 12 + q];
                u[i * 12 + p] = c * up - sn * uq;
                u[i * 12 + q] = sn * up + c * uq;
                const double vp = v[i * 12 + p], vq = v[i * 12 + q];
                v[i * 12 + p] = c * vp - sn * vq;
                v[i * 12 + q] = sn * vp + c * vq;
              }
            }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) off = fmax(off, __shfl_xor(off, o, 64));
    if (off < 1e-15) break;
  }
}

__device__ __forceinline__ void jacobi12_null4_group(double* __restrict__ u, int l, double* __restrict__ out) {
  jacobi12_sweeps_group<false>(u, nullptr, l);
  if (l != 0) return;
  double w[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) s += u[i * 12 + j] * u[i * 12 + j];
    w[j] = sqrt(s);
  }
  double sw[12];
  int ord[12];
  sort_desc<12>(w, sw, ord);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = ord[8 + r];
    const double wj = sw[8 + r];
    const double inv = wj > 0 ? 1.0 / wj : 0.0;
#pragma unroll
    for (int i = 0; i < 12; ++i) out[r * 12 + i] = u[i * 12 + j] * inv;  // u is in LDS: index it directly
  }
}

// Right singular vector of the smallest singular value of the symmetric 12x12 DLT matrix
// (packed upper triangle LLp, identical on every lane) -- column 11 of dsvd_ws<12,12>'s V,
// with dsvd_ws's exact arithmetic -- by the whole wave on LDS work arrays u, v [144].
// Returns the vector on every lane.
__device__ void dlt12_null(const double* LLp, double* __restrict__ u, double* __restrict__ v, double* out) {
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < 144; k += 64) v[k] = (k % 13 == 0) ? 1.0 : 0.0;
  if (lane < 12) {
#pragma unroll
    for (int a = 0, k = 0; a < 12; ++a)
#pragma unroll
      for (int b = a; b < 12; ++b, ++k) {
        if (lane == a) u[a * 12 + b] = LLp[k];
        if (lane == b) u[b * 12 + a] = LLp[k];  // each lane writes its row of the symmetric matrix
      }
  }
  __syncthreads();
  jacobi12_sweeps_wave(u, v);
  __syncthreads();
  // the smallest column norm, the last one in dsvd_ws's stable descending order
  double w[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) s += u[i * 12 + j] * u[i * 12 + j];
    w[j] = sqrt(s);
  }
  double sw[12];
  int ord[12];
  sort_desc<12>(w, sw, ord);
  const int j = ord[11];
#pragma unroll
  for (int i = 0; i < 12; ++i) out[i] = v[i * 12 + j];
  __syncthreads();
}

// ------------------------------------------------------------------ EPnP (5 points)
__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ double dist2(const double* a, const double* b) {
  return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

// VIEW: the subset's points, barycentric coordinates and control points are read in place
// (workspace pointers) instead of held in registers -- the β stage only reads them.
template <int NP, bool VIEW = false>
struct EPnPd {
  template <int N>
  using Arr = typename std::conditional<VIEW, const double*, double[N]>::type;
  using Cws = typename std::conditional<VIEW, const double (*)[3], double[4][3]>::type;
  double fu, fv, uc, vc;
  Arr<3 * NP> pws;
  Arr<2 * NP> us;
  Arr<4 * NP> alphas;
  Cws cws;
  double pcs[3 * NP], ccs[4][3];

  __device__ void choose_control_points() {
    #pragma unroll
    for (int j = 0; j < 3; ++j) cws[0][j] = 0;
    #pragma unroll
    for (int i = 0; i < NP; ++i)
      #pragma unroll
      for (int j = 0; j < 3; ++j) cws[0][j] += pws[3 * i + j];
    #pragma unroll
    for (int j = 0; j < 3; ++j) cws[0][j] /= NP;
    double A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    #pragma unroll
    for (int i = 0; i < NP; ++i) {
      double d[3] = {pws[3 * i] - cws[0][0], pws[3 * i + 1] - cws[0][1], pws[3 * i + 2] - cws[0][2]};
      #pragma unroll
      for (int a = 0; a < 3; ++a)
        #pragma unroll
        for (int bb = 0; bb < 3; ++bb) A[a * 3 + bb] += d[a] * d[bb];
    }
    double W[3], U[9], V[9];
    dsvd<3, 3>(A, W, U, V);
    #pragma unroll
    for (int i = 1; i < 4; ++i) {
      double k = sqrt(W[i - 1] / NP);
      #pragma unroll
      for (int j = 0; j < 3; ++j) cws[i][j] = cws[0][j] + k * U[j * 3 + (i - 1)];
    }
  }
  __device__ void barycentric() {
    double cc[9], ci[9], W[3], U[9], V[9];
    #pragma unroll
    for (int i = 0; i < 3; ++i)
      #pragma unroll
      for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
    dsvd<3, 3>(cc, W, U, V);
    #pragma unroll
    for (int i = 0; i < 3; ++i)
      #pragma unroll
      for (int j = 0; j < 3; ++j) {
        double s = 0;
        #pragma unroll
        for (int k = 0; k < 3; ++k) s += (W[k] > 0 ? V[i * 3 + k] / W[k] : 0.0) * U[j * 3 + k];
        ci[i * 3 + j] = s;
      }
    #pragma unroll
    for (int i = 0; i < NP; ++i) {
      const double* p = &pws[3 * i];
      double* a = &alphas[4 * i];
      #pragma unroll
      for (int j = 0; j < 3; ++j)
        a[1 + j] = ci[3 * j] * (p[0] - cws[0][0]) + ci[3 * j + 1] * (p[1] - cws[0][1]) + ci[3 * j + 2] * (p[2] - cws[0][2]);
      a[0] = 1.0f - a[1] - a[2] - a[3];
    }
  }
  // nv[r] = ut row 8 + r (EPnP's v_{3-r}); rows 11..8 are the four null-space directions
  __device__ void compute_ccs(const double* betas, const double (*nv)[12]) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double* v = nv[3 - i];
      #pragma unroll
      for (int j = 0; j < 4; ++j)
        #pragma unroll
        for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[3 * j + k];
    }
  }
  __device__ void compute_pcs() {
    #pragma unroll
    for (int i = 0; i < NP; ++i) {
      const double* a = &alphas[4 * i];
      #pragma unroll
      for (int j = 0; j < 3; ++j) pcs[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
    }
  }
  __device__ double compute_R_and_t(const double (*nv)[12], const double* betas, double* R, double* t) {
    compute_ccs(betas, nv);
    compute_pcs();
    if (pcs[2] < 0.0) {
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 3; ++j) ccs[i][j] = -ccs[i][j];
      #pragma unroll
      for (int i = 0; i < 3 * NP; ++i) pcs[i] = -pcs[i];
    }
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    #pragma unroll
    for (int i = 0; i < NP; ++i)
      #pragma unroll
      for (int j = 0; j < 3; ++j) {
        pc0[j] += pcs[3 * i + j];
        pw0[j] += pws[3 * i + j];
      }
    #pragma unroll
    for (int j = 0; j < 3; ++j) {
      pc0[j] /= NP;
      pw0[j] /= NP;
    }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    #pragma unroll
    for (int i = 0; i < NP; ++i)
      #pragma unroll
      for (int j = 0; j < 3; ++j) {
        double dc = pcs[3 * i + j] - pc0[j];
        abt[3 * j] += dc * (pws[3 * i] - pw0[0]);
        abt[3 * j + 1] += dc * (pws[3 * i + 1] - pw0[1]);
        abt[3 * j + 2] += dc * (pws[3 * i + 2] - pw0[2]);
      }
    double W[3], U[9], V[9];
    dsvd<3, 3>(abt, W, U, V);
    #pragma unroll
    for (int i = 0; i < 3; ++i)
      #pragma unroll
      for (int j = 0; j < 3; ++j) R[i * 3 + j] = U[i * 3] * V[j * 3] + U[i * 3 + 1] * V[j * 3 + 1] + U[i * 3 + 2] * V[j * 3 + 2];
    double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] - R[1] * R[3] * R[8] -
                 R[0] * R[5] * R[7];
    if (det < 0) {
      R[6] = -R[6];
      R[7] = -R[7];
      R[8] = -R[8];
    }
    #pragma unroll
    for (int i = 0; i < 3; ++i) t[i] = pc0[i] - dot3(&R[3 * i], pw0);
    double sum2 = 0.0;
    #pragma unroll
    for (int i = 0; i < NP; ++i) {
      const double* pw = &pws[3 * i];
      double Xc = dot3(&R[0], pw) + t[0], Yc = dot3(&R[3], pw) + t[1];
      double iz = 1.0 / (dot3(&R[6], pw) + t[2]);
      double ue = uc + fu * Xc * iz, ve = vc + fv * Yc * iz;
      double u = us[2 * i], v = us[2 * i + 1];
      sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / NP;
  }
  __device__ static void qr_solve(double* A, double* b, double* X) {
    const int nr = 6, nc = 4;
    double A1[4], A2[4];
    #pragma unroll
    for (int k = 0; k < nc; ++k) {
      double eta = fabs(A[k * nc + k]);
      #pragma unroll
      for (int i = k + 1; i < nr; ++i) eta = fmax(eta, fabs(A[i * nc + k]));
      if (eta == 0) return;
      double sum2 = 0.0, inv = 1. / eta;
      #pragma unroll
      for (int i = k; i < nr; ++i) {
        A[i * nc + k] *= inv;
        sum2 += A[i * nc + k] * A[i * nc + k];
      }
      double sigma = sqrt(sum2);
      if (A[k * nc + k] < 0) sigma = -sigma;
      A[k * nc + k] += sigma;
      A1[k] = sigma * A[k * nc + k];
      A2[k] = -eta * sigma;
      #pragma unroll
      for (int j = k + 1; j < nc; ++j) {
        double sum = 0;
        #pragma unroll
        for (int i = k; i < nr; ++i) sum += A[i * nc + k] * A[i * nc + j];
        double tau = sum / A1[k];
        #pragma unroll
        for (int i = k; i < nr; ++i) A[i * nc + j] -= tau * A[i * nc + k];
      }
    }
    #pragma unroll
    for (int j = 0; j < nc; ++j) {
      double tau = 0;
      #pragma unroll
      for (int i = j; i < nr; ++i) tau += A[i * nc + j] * b[i];
      tau /= A1[j];
      #pragma unroll
      for (int i = j; i < nr; ++i) b[i] -= tau * A[i * nc + j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    #pragma unroll
    for (int i = nc - 2; i >= 0; --i) {
      double sum = 0;
      #pragma unroll
      for (int j = i + 1; j < nc; ++j) sum += A[i * nc + j] * X[j];
      X[i] = (b[i] - sum) / A2[i];
    }
  }
  __device__ static void gauss_newton(const double* L, const double* rho, double* betas) {
#pragma nounroll
    for (int it = 0; it < 5; ++it) {
      double A[24], b[6], x[4] = {0, 0, 0, 0};
      // L and rho are re-read every iteration: hoisted out of the loop they held 66 doubles
      // in registers (hyp_b at 256 VGPRs + AGPRs, one wave per SIMD)
      int o = 0;
      asm volatile("" : "+v"(o));
      #pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double* r = L + o + 10 * i;
        A[i * 4 + 0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
        A[i * 4 + 1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
        A[i * 4 + 2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
        A[i * 4 + 3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
        b[i] = rho[o + i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] + r[2] * betas[1] * betas[1] +
                         r[3] * betas[0] * betas[2] + r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                         r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] + r[8] * betas[2] * betas[3] +
                         r[9] * betas[3] * betas[3]);
      }
      qr_solve(A, b, x);
      #pragma unroll
      for (int i = 0; i < 4; ++i) betas[i] += x[i];
    }
  }
  // First half of compute_pose: control points, barycentric coordinates and M^T M (element k
  // at MtM[k * S]); its four null-space directions come from jacobi12_null4.
  template <int S>
  __device__ void build_mtm(double* __restrict__ MtM) {
    choose_control_points();
    barycentric();
#pragma unroll
    for (int i = 0; i < 144; ++i) MtM[i * S] = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const double* as = &alphas[4 * i];
      double u = us[2 * i], v = us[2 * i + 1];
      double M1[12], M2[12];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        M1[3 * j] = as[j] * fu; M1[3 * j + 1] = 0.0; M1[3 * j + 2] = as[j] * (uc - u);
        M2[3 * j] = 0.0; M2[3 * j + 1] = as[j] * fv; M2[3 * j + 2] = as[j] * (vc - v);
      }
      // rows of M in order (M1 then M2), each accumulated on its own: the oracle's summation order
#pragma unroll
      for (int a = 0; a < 12; ++a)
#pragma unroll
        for (int bb = 0; bb < 12; ++bb) MtM[(a * 12 + bb) * S] += M1[a] * M1[bb];
#pragma unroll
      for (int a = 0; a < 12; ++a)
#pragma unroll
        for (int bb = 0; bb < 12; ++bb) MtM[(a * 12 + bb) * S] += M2[a] * M2[bb];
    }
  }
  // Second half: L (6x10) and rho from the null space and the control points ...
  __device__ void prep(const double (*nv)[12], double* L, double* rho) const {
    const double* vv[4] = {nv[3], nv[2], nv[1], nv[0]};
    constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
    // one control-point pair at a time (all 6 pairs' differences held at once were 72 doubles)
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      double dv[4][3];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int k = 0; k < 3; ++k) dv[a][k] = vv[a][3 * pa[i] + k] - vv[a][3 * pb[i] + k];
      double* r = L + 10 * i;
      r[0] = dot3(dv[0], dv[0]);
      r[1] = 2.0f * dot3(dv[0], dv[1]);
      r[2] = dot3(dv[1], dv[1]);
      r[3] = 2.0f * dot3(dv[0], dv[2]);
      r[4] = 2.0f * dot3(dv[1], dv[2]);
      r[5] = dot3(dv[2], dv[2]);
      r[6] = 2.0f * dot3(dv[0], dv[3]);
      r[7] = 2.0f * dot3(dv[1], dv[3]);
      r[8] = 2.0f * dot3(dv[2], dv[3]);
      r[9] = dot3(dv[3], dv[3]);
    }
    rho[0] = dist2(cws[0], cws[1]); rho[1] = dist2(cws[0], cws[2]); rho[2] = dist2(cws[0], cws[3]);
    rho[3] = dist2(cws[1], cws[2]); rho[4] = dist2(cws[1], cws[3]); rho[5] = dist2(cws[2], cws[3]);
  }
  // ... and beta approximation N (1..3) + Gauss-Newton -> (R, t) and its reprojection error.
  // compute_pose keeps approximation 1 and replaces it by a later one with a strictly smaller
  // error (the caller does that selection).
  __device__ double approx(int N, const double* L, const double* rho, const double (*nv)[12], double* R, double* t) {
    double betas[4];
    if (N == 1) {
      double A[24], b4[4];
      constexpr int c[4] = {0, 1, 3, 6};
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) A[i * 4 + j] = L[i * 10 + c[j]];
      dsolve<6, 4>(A, rho, b4);
      double s = b4[0] < 0 ? -1.0 : 1.0;
      betas[0] = sqrt(s * b4[0]);
      betas[1] = s * b4[1] / betas[0];
      betas[2] = s * b4[2] / betas[0];
      betas[3] = s * b4[3] / betas[0];
    } else if (N == 2) {
      double A[18], b3[3];
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A[i * 3 + j] = L[i * 10 + j];
      dsolve<6, 3>(A, rho, b3);
      if (b3[0] < 0) {
        betas[0] = sqrt(-b3[0]);
        betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
      } else {
        betas[0] = sqrt(b3[0]);
        betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
      }
      if (b3[1] < 0) betas[0] = -betas[0];
      betas[2] = 0.0;
      betas[3] = 0.0;
    } else {
      double A[30], b5[5];
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) A[i * 5 + j] = L[i * 10 + j];
      dsolve<6, 5>(A, rho, b5);
      if (b5[0] < 0) {
        betas[0] = sqrt(-b5[0]);
        betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
      } else {
        betas[0] = sqrt(b5[0]);
        betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
      }
      if (b5[1] < 0) betas[0] = -betas[0];
      betas[2] = b5[3] / betas[0];
      betas[3] = 0.0;
    }
    gauss_newton(L, rho, betas);
    return compute_R_and_t(nv, betas, R, t);
  }
};

using fvo_rs::RNG;
using fvo_rs::update_num_iters;

__device__ __forceinline__ double wsum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------ RANSAC + refine
constexpr int kRefineLds = 1024;  // inliers staged in k_pnp_refine's LDS (20 KB)

struct PnpShared {
  double dlt[5][144];  // DLT 12x12 SVD: input, work u / v, outputs U / V (lane 0 only)
  int sub[kChunk][5];
  int good[kChunk];
  double model[kChunk][6];
  double best[6];
  double param[6];
  double jtj[21], jte[6];  // the LM normal equations (J^T J packed upper triangle, J^T e)
  double llp[78];          // the DLT's packed A^T A, wave-summed
  double rrt[12];          // the DLT null vector (non-planar)
  double rt[9], t3[3];     // the planar case's frame (Rt, T)
  double prev[6];          // the LM step's base point
  int maxGood, niters, done, next_iter;
  uint64_t rng;
  int ninl;
  int flag;
};

// The DLT's pose (lane 0): R, t from the null vector, or the planar homography's
// decomposition, into sh.param.  noinline, as lm_eval / lm_step below: the refinement runs as
// one wave per frame, so its code is fetched cold -- one copy of each phase instead of the
// inlined copies (a 219 KB kernel) keeps the LM loop in the instruction cache.
__device__ __attribute__((noinline)) void dlt_pose(PnpShared& sh, bool planar) {
  double param[6] = {0, 0, 0, 0, 0, 0};
  double R[9];
  if (!planar) {
    double RR[9] = {sh.rrt[0], sh.rrt[1], sh.rrt[2], sh.rrt[4], sh.rrt[5], sh.rrt[6], sh.rrt[8], sh.rrt[9], sh.rrt[10]};
    double tt[3] = {sh.rrt[3], sh.rrt[7], sh.rrt[11]};
    if (ddet3(RR) < 0) {
#pragma unroll
      for (int i = 0; i < 9; ++i) RR[i] = -RR[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) tt[i] = -tt[i];
    }
    double sc = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) sc += RR[i] * RR[i];
    sc = sqrt(sc);
    double Wr[3], Ur[9], Vr[9];
    dsvd<3, 3>(RR, Wr, Ur, Vr);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) R[i * 3 + j] = Ur[i * 3] * Vr[j * 3] + Ur[i * 3 + 1] * Vr[j * 3 + 1] + Ur[i * 3 + 2] * Vr[j * 3 + 2];
    double nR = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) nR += R[i] * R[i];
    nR = sqrt(nR);
#pragma unroll
    for (int i = 0; i < 3; ++i) param[3 + i] = tt[i] * nR / sc;
    rod_R2r(R, param);
  } else {
    double* AtA = sh.dlt[0];
    double* U9 = sh.dlt[3];
    double* V9 = sh.dlt[4];
    double W9[9], H[9], t[3];
    int k = 0;
#pragma unroll
    for (int a = 0; a < 9; ++a)
#pragma unroll
      for (int b = a; b < 9; ++b) { AtA[a * 9 + b] = sh.llp[k]; AtA[b * 9 + a] = sh.llp[k]; ++k; }
    dsvd_ws<9, 9>(AtA, W9, U9, V9, sh.dlt[1], sh.dlt[2]);
#pragma unroll
    for (int i = 0; i < 9; ++i) H[i] = V9[i * 9 + 8];
    if (fabs(H[8]) >= 1e-300) {
#pragma unroll
      for (int i = 0; i < 9; ++i) H[i] /= H[8];
      double h1 = sqrt(H[0] * H[0] + H[3] * H[3] + H[6] * H[6]);
      double h2 = sqrt(H[1] * H[1] + H[4] * H[4] + H[7] * H[7]);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        H[i * 3] /= fmax(h1, DBL_EPSILON);
        H[i * 3 + 1] /= fmax(h2, DBL_EPSILON);
        t[i] = H[i * 3 + 2] * 2. / fmax(h1 + h2, DBL_EPSILON);
      }
      H[2] = H[3] * H[7] - H[6] * H[4];
      H[5] = H[6] * H[1] - H[0] * H[7];
      H[8] = H[0] * H[4] - H[3] * H[1];
      double r[3];
      rod_R2r(H, r);
      rod_r2R(r, H, nullptr);
#pragma unroll
      for (int i = 0; i < 3; ++i) t[i] += H[i * 3] * sh.t3[0] + H[i * 3 + 1] * sh.t3[1] + H[i * 3 + 2] * sh.t3[2];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = H[i * 3] * sh.rt[j] + H[i * 3 + 1] * sh.rt[3 + j] + H[i * 3 + 2] * sh.rt[6 + j];
      param[3] = t[0]; param[4] = t[1]; param[5] = t[2];
    } else {
#pragma unroll
      for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0);
    }
    rod_R2r(R, param);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) sh.param[i] = param[i];
}

// One LM evaluation over the inliers: the reprojection error norm, and with withJ the normal
// equations J^T J / J^T e into sh.jtj / sh.jte (lane 0 writes).  Every lane returns the norm.
__device__ __attribute__((noinline)) double lm_eval(PnpShared& sh, const Cam K, const float* P3, const float* p2,
                                                    int n, bool withJ) {
  const int lane = wave_lane();
  double p[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) p[i] = sh.param[i];
  double R[9], dR[27];
  rod_r2R(p, R, dR);
  double a[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) a[k] = 0;
  for (int i = lane; i < n; i += 64) {
    const int j = i;
    double M[3] = {(double)P3[3 * j], (double)P3[3 * j + 1], (double)P3[3 * j + 2]}, uv[2], J[12];
    dproject(K, R, dR, p + 3, M, uv, withJ ? J : nullptr);
    double e0 = uv[0] - (double)p2[2 * j], e1 = uv[1] - (double)p2[2 * j + 1];
    a[27] += e0 * e0 + e1 * e1;
    if (withJ) {
      int k = 0;
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) a[k++] += J[r] * J[c] + J[6 + r] * J[6 + c];
#pragma unroll
      for (int r = 0; r < 6; ++r) a[21 + r] += J[r] * e0 + J[6 + r] * e1;
    }
  }
  if (withJ) {
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      const double t = wsum_d(a[k]);
      if (lane == 0) {
        if (k < 21) sh.jtj[k] = t;
        else sh.jte[k - 21] = t;
      }
    }
  }
  return sqrt(wsum_d(a[27]));
}

// The LM step (lane 0): (J^T J with the (1 + lambda) diagonal) x = J^T e from the packed
// sh.jtj / sh.jte, sh.param = sh.prev - x.
__device__ __attribute__((noinline)) void lm_step(PnpShared& sh, double lambdaLg10) {
  const double lambda = exp(lambdaLg10 * log(10.));
  double A[36], x[6], g[6];
  int k = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = r; c < 6; ++c) { A[r * 6 + c] = sh.jtj[k]; A[c * 6 + r] = sh.jtj[k]; ++k; }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    A[i * 6 + i] *= 1. + lambda;
    g[i] = sh.jte[i];
  }
  if (!chol_solve6(A, g, x)) dsolve<6, 6>(A, g, x);
#pragma unroll
  for (int i = 0; i < 6; ++i) sh.param[i] = sh.prev[i] - x[i];
}

// P3 / p2: the inliers' points, compacted (k_pnp_refine stages them in LDS)
__device__ void lm_refine(PnpShared& sh, const Cam& K, const float* P3, const float* p2, int n, double* mn) {
  // ---- init (cvFindExtrinsicCameraParams2, useExtrinsicGuess = false)
  const int lane = wave_lane();
  double acc[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) acc[k] = 0;
  for (int i = lane; i < n; i += 64) {
    const int j = i;
    dundistort(K, (double)p2[2 * j], (double)p2[2 * j + 1], &mn[2 * i]);
    acc[0] += (double)P3[3 * j];
    acc[1] += (double)P3[3 * j + 1];
    acc[2] += (double)P3[3 * j + 2];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) acc[k] = wsum_d(acc[k]);
  double Mc[3] = {acc[0] / n, acc[1] / n, acc[2] / n};
  double MM[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = lane; i < n; i += 64) {
    const int j = i;
    double d[3] = {(double)P3[3 * j] - Mc[0], (double)P3[3 * j + 1] - Mc[1], (double)P3[3 * j + 2] - Mc[2]};
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) MM[a * 3 + b] += d[a] * d[b];
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) MM[k] = wsum_d(MM[k]);
  double W3[3], U3[9], V3[9];
  dsvd<3, 3>(MM, W3, U3, V3);
  const bool planar = W3[2] / W3[1] < 1e-3;
  if (!planar && n < 6) {
    if (lane == 0) sh.flag = 0;  // DLT would throw: keep the RANSAC model
    __syncthreads();
    return;
  }
  double LLp[78];
#pragma unroll
  for (int k = 0; k < 78; ++k) LLp[k] = 0;
  double Rt[9], T[3];
  if (!planar) {
    for (int i = lane; i < n; i += 64) {
      const int j = i;
      double x = -mn[2 * i], y = -mn[2 * i + 1];
      double P[3] = {(double)P3[3 * j], (double)P3[3 * j + 1], (double)P3[3 * j + 2]};
      double r0[12] = {P[0], P[1], P[2], 1., 0, 0, 0, 0, x * P[0], x * P[1], x * P[2], x};
      double r1[12] = {0, 0, 0, 0, P[0], P[1], P[2], 1., y * P[0], y * P[1], y * P[2], y};
      int k = 0;
#pragma unroll
      for (int a = 0; a < 12; ++a)
#pragma unroll
        for (int b = a; b < 12; ++b) LLp[k++] += r0[a] * r0[b] + r1[a] * r1[b];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Rt[i * 3 + j] = V3[j * 3 + i];
    if (Rt[2] * Rt[2] + Rt[5] * Rt[5] < 1e-10)
#pragma unroll
      for (int i = 0; i < 9; ++i) Rt[i] = (i % 4 == 0);
    if (ddet3(Rt) < 0)
#pragma unroll
      for (int i = 0; i < 9; ++i) Rt[i] = -Rt[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) T[i] = -(Rt[i * 3] * Mc[0] + Rt[i * 3 + 1] * Mc[1] + Rt[i * 3 + 2] * Mc[2]);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 9; ++i) sh.rt[i] = Rt[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) sh.t3[i] = T[i];
    }
    // homography DLT (A^T A, 9x9 upper triangle = 45 entries)
    for (int i = lane; i < n; i += 64) {
      const int j = i;
      double s0 = P3[3 * j], s1 = P3[3 * j + 1], s2 = P3[3 * j + 2];
      double X = Rt[0] * s0 + Rt[1] * s1 + Rt[2] * s2 + T[0];
      double Y = Rt[3] * s0 + Rt[4] * s1 + Rt[5] * s2 + T[1];
      double u = mn[2 * i], v = mn[2 * i + 1];
      double r0[9] = {X, Y, 1, 0, 0, 0, -u * X, -u * Y, -u};
      double r1[9] = {0, 0, 0, X, Y, 1, -v * X, -v * Y, -v};
      int k = 0;
#pragma unroll
      for (int a = 0; a < 9; ++a)
#pragma unroll
        for (int b = a; b < 9; ++b) LLp[k++] += r0[a] * r0[b] + r1[a] * r1[b];
    }
  }
#pragma unroll
  for (int k = 0; k < 78; ++k) {
    const double t = wsum_d(LLp[k]);
    if (lane == 0) sh.llp[k] = t;  // in LDS: the SVD below runs beside no register copy of it
  }
  __syncthreads();
  if (!planar) dlt12_null(sh.llp, sh.dlt[1], sh.dlt[2], sh.rrt);  // the whole wave (same sh.rrt on every lane)
  if (lane == 0) dlt_pose(sh, planar);
  __syncthreads();
  // ---- Levenberg-Marquardt (CvLevMarq semantics)
  double prev[6];
  double lambdaLg10 = -3, prevErrNorm = DBL_MAX;
  int iters = 0;
  for (;;) {
    double e0 = lm_eval(sh, K, P3, p2, n, true);
#pragma unroll
    for (int i = 0; i < 6; ++i) prev[i] = sh.param[i];
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 6; ++i) sh.prev[i] = prev[i];
    }
    __syncthreads();
    if (lane == 0) lm_step(sh, lambdaLg10);
    __syncthreads();
    if (iters == 0) prevErrNorm = e0;
    double errNorm;
    for (;;) {
      errNorm = lm_eval(sh, K, P3, p2, n, false);
      if (errNorm > prevErrNorm && ++lambdaLg10 <= 16) {
        if (lane == 0) lm_step(sh, lambdaLg10);
        __syncthreads();
        continue;
      }
      break;
    }
    lambdaLg10 = fmax(lambdaLg10 - 1, -16.0);
    double dn = 0, pn = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      dn += (sh.param[i] - prev[i]) * (sh.param[i] - prev[i]);
      pn += prev[i] * prev[i];
    }
    double rel = sqrt(dn) / (sqrt(pn) + DBL_EPSILON);
    if (++iters >= 20 || rel < FLT_EPSILON) break;
    prevErrNorm = errNorm;
  }
  if (lane == 0) sh.flag = 1;
  __syncthreads();
}

struct PnpState {
  int maxGood, niters, best_it, n;
};

// Subsets of every potential RANSAC iteration, drawn exactly as getSubset() with
// RNG(-1): 5 distinct indices from rng.uniform(0, n) with rejection of repeats.  The draws
// depend only on the point count n (solvePnPRansac seeds a fresh RNG(-1) per call), so the
// table of every n in [6, cap] is drawn once when the context is created (one thread per n)
// and a frame's hypotheses read row n of it.
__global__ void k_pnp_table(int cap, int maxIters, int16_t* __restrict__ table) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < 6 || n > cap) return;
  fvo_rs::draw_subsets(n, maxIters, table + (int64_t)n * maxIters * 5);
}

__global__ void k_pnp_subsets(const int32_t* __restrict__ npts, int batch, int cap, int maxIters,
                              PnpState* __restrict__ state) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  int n = npts[b];
  n = n < 0 ? 0 : (n > cap ? cap : n);
  PnpState st;
  st.maxGood = 0;
  st.niters = maxIters;
  st.best_it = -1;
  st.n = n;
  state[b] = st;
}

// One lane per RANSAC iteration, EPnP in two launches (one kernel held the whole EPnP state
// plus the scoring loop at 256 VGPRs with 1.6 KB of scratch per lane):
//   k_pnp_hyp_a  the subset's points (undistorted, float32-rounded normalised image points, as
//                solvePnP(SOLVEPNP_EPNP) sees them), control points, barycentric coordinates,
//                M^T M in LDS and its null space -> workspace;
//   k_pnp_hyp_b  the beta approximations + Gauss-Newton + (R, t), the model, and its inlier
//                count over all points (projectPoints in fp64, error in float32).
// Blocks whose first iteration is past the frame's current iteration bound exit immediately.
constexpr int PNP_WS = 256;  // doubles per subset: nv 48 | cws 12 | alphas 20 | pws 15 | us 10 | pad | MtM 144
constexpr int PW_NV = 0, PW_CWS = 48, PW_AL = 60, PW_PWS = 80, PW_US = 95, PW_MTM = 112;

// Round 1 runs every frame's first PNP_FIRST iterations on a (chunks, frames) grid. Round 2
// runs only where round 1's adaptive bound left iterations over -- usually none, sometimes one
// hard frame (a large motion, few inliers) needing up to maxIters: k_pnp_plan turns the frames'
// remaining iterations into prefix sums of work units, and a fixed grid strides over the flat
// unit space with round 1's grid size, so the hard frames share the whole grid and the easy
// case dispatches one round-1 grid of blocks that exit at once. (A (chunks, frames) grid there was thousands of blocks that only
// read the bound, each waiting for a register slot while the next step's disparity kernels
// hold the CUs; a few blocks per frame serialised the hard frame.)
constexpr int PNP_FIRST = 128;
constexpr int PNP_CS = 64, PNP_CA = 8, PNP_CB = 16;  // iterations per setup / hyp_a / hyp_b unit

__global__ __launch_bounds__(64) void k_pnp_plan(int batch, int maxIters, const PnpState* __restrict__ state,
                                                 int32_t* __restrict__ plan) {
  const int lane = threadIdx.x;
  int carry[3] = {0, 0, 0};
  const int C[3] = {PNP_CS, PNP_CA, PNP_CB};
  for (int b0 = 0; b0 < batch; b0 += 64) {
    const int b = b0 + lane;
    int rem = 0;
    if (b < batch) {
      const PnpState st = state[b];
      if (st.n >= 6) rem = max(0, min(st.niters, maxIters) - PNP_FIRST);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      int v = (rem + C[k] - 1) / C[k];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
      }
      const int incl = v, excl = incl - (rem + C[k] - 1) / C[k];
      if (b < batch) plan[k * (batch + 1) + b] = carry[k] + excl;
      carry[k] += __shfl(incl, 63, 64);
    }
  }
  if (lane < 3) plan[lane * (batch + 1) + batch] = carry[lane];
}

// Work unit u of round 2 (granularity k) -> frame and its first iteration; wave-uniform.
__device__ __forceinline__ void pnp_unit(const int32_t* __restrict__ pre, int batch, int u, int C, int& b, int& base) {
  int lo = 0, hi = batch - 1;  // the largest b with pre[b] <= u
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= u) lo = mid; else hi = mid - 1;
  }
  b = lo;
  base = PNP_FIRST + (u - pre[lo]) * C;
}

// Drives a kernel body over its units: round 1 (plan == nullptr) one unit per block at
// (blockIdx.x, blockIdx.y); round 2 the flat unit space, grid-strided. (One call site for the
// body: two inlined copies cost hyp_a 64 VGPRs.)
template <int C, typename Body>
__device__ __forceinline__ void pnp_units(const int32_t* __restrict__ plan, int k, int batch, int maxIters,
                                          const PnpState* __restrict__ state, Body body) {
  const int32_t* pre = plan ? plan + k * (batch + 1) : nullptr;
  const int total = plan ? pre[batch] : (int)blockIdx.x + 1;
  for (int u = blockIdx.x; u < total; u += gridDim.x) {
    int b, base, lim;
    if (plan) {
      pnp_unit(pre, batch, u, C, b, base);
      lim = maxIters;
    } else {
      b = blockIdx.y;
      base = u * C;
      lim = PNP_FIRST;
    }
    const PnpState st = state[b];
    const int hi = min(min(st.niters, maxIters), lim);
    if (st.n < 6 || base >= hi) continue;
    body(b, base, hi, st.n);
  }
}

// lane per subset: points, control points, barycentric coordinates, M^T M -> workspace (the
// register-heavy part, kept out of the long Jacobi kernel so that one stays small)
__global__ __launch_bounds__(64, 4) void k_pnp_setup(const float* __restrict__ P3all, const float* __restrict__ p2all,
                                                  int cap, Cam K, int maxIters, int batch,
                                                  const int32_t* __restrict__ plan,
                                                  const int16_t* __restrict__ table, int table_iters,
                                                  const PnpState* __restrict__ state, double* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) double smt[];  // [144][64]: one M^T M column per lane
  double* mt = smt + threadIdx.x;
  pnp_units<PNP_CS>(plan, 0, batch, maxIters, state, [&](int b, int base, int hi, int n) {
    const int it = base + threadIdx.x;
    if (it >= hi) return;
    const float* __restrict__ P3 = P3all + (int64_t)b * cap * 3;
    const float* __restrict__ p2 = p2all + (int64_t)b * cap * 2;
    double* w = ws + ((int64_t)b * maxIters + it) * PNP_WS;
    const int16_t* sb = table + ((int64_t)n * table_iters + it) * 5;
    EPnPd<5> e;
    e.fu = K.fx; e.fv = K.fy; e.uc = K.cx; e.vc = K.cy;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      int j = sb[i];
#pragma unroll
      for (int c = 0; c < 3; ++c) e.pws[3 * i + c] = (double)P3[j * 3 + c];
      double xy[2];
      dundistort(K, (double)p2[j * 2], (double)p2[j * 2 + 1], xy);
      float fx = (float)xy[0], fy = (float)xy[1];
      e.us[2 * i] = fx * K.fx + K.cx;
      e.us[2 * i + 1] = fy * K.fy + K.cy;
    }
    e.build_mtm<64>(mt);
#pragma unroll 8
    for (int k = 0; k < 144; ++k) w[PW_MTM + k] = mt[k * 64];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) w[PW_CWS + r * 3 + k] = e.cws[r][k];
#pragma unroll
    for (int k = 0; k < 20; ++k) w[PW_AL + k] = e.alphas[k];
#pragma unroll
    for (int k = 0; k < 15; ++k) w[PW_PWS + k] = e.pws[k];
#pragma unroll
    for (int k = 0; k < 10; ++k) w[PW_US + k] = e.us[k];
  });
}

// 8-lane group per subset: the null space of its M^T M (staged in LDS)
__global__ __launch_bounds__(64) void k_pnp_hyp_a(int maxIters, int batch, const int32_t* __restrict__ plan,
                                                  const PnpState* __restrict__ state, double* __restrict__ ws) {
  __shared__ double su[8][144];  // M^T M of the block's 8 subsets (one 8-lane group each)
  const int g = threadIdx.x >> 3, l = threadIdx.x & 7;
  double* u = su[g];
  pnp_units<PNP_CA>(plan, 1, batch, maxIters, state, [&](int b, int base, int hi, int) {
    const int it = base + g;
    if (it >= hi) return;  // the whole group
    double* w = ws + ((int64_t)b * maxIters + it) * PNP_WS;
    for (int k = l; k < 144; k += 8) u[k] = w[PW_MTM + k];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    jacobi12_null4_group(u, l, w + PW_NV);
  });
}

// Register budgets (hyp_b <= 168 VGPRs, 416 B of scratch; refine <= 256, 1040 B): in the
// overlapped pipeline this stage runs beside the disparity kernels, whose waves hold 128 VGPRs
// each, and a wave needing more than a few of their slots on one SIMD waits for them to drain
// (hyp_b at 276 registers: 2.6-3.4 ms per launch beside k_sg_rows).  Measured (bench.py, 20
// steps, 2 runs each): unbounded 5110 frames/s; hyp_b at 256 / 168 / 128 VGPRs 5130 / 5177 /
// 5173; then refine at 256 / 168 VGPRs 5237 / 5222 (in-order PnP 1.57 -> 1.73 ms).  Forcing
// k_ba_build (512 threads) to 128 VGPRs instead collapsed the overlapped step (21 ms).
__global__ __launch_bounds__(64, 3) void k_pnp_hyp_b(const float* __restrict__ P3all, const float* __restrict__ p2all,
                                                  int cap, Cam K, float thr2, int maxIters, int batch,
                                                  const int32_t* __restrict__ plan,
                                                  const PnpState* __restrict__ state, const double* __restrict__ ws,
                                                  double* __restrict__ model, int32_t* __restrict__ good) {
  // a 4-lane group per subset: lanes 0..2 run the three beta approximations side by side (the
  // serial loop's selection -- approximation 1, replaced by a later one only on a strictly
  // smaller error -- is applied to their results in order), then all four lanes score the
  // model over a quarter of the points each
  __shared__ double sL[16][66];  // per group: L (6x10) then rho (6)
  const int g = threadIdx.x >> 2, l = threadIdx.x & 3;
  double* L = sL[g];
  pnp_units<PNP_CB>(plan, 2, batch, maxIters, state, [&](int b, int base, int hi, int n) {
    const int it = base + g;
    if (it >= hi) return;  // the whole group
    const float* __restrict__ P3 = P3all + (int64_t)b * cap * 3;
    const float* __restrict__ p2 = p2all + (int64_t)b * cap * 2;
    const double* w = ws + ((int64_t)b * maxIters + it) * PNP_WS;
    EPnPd<5, true> e;
    e.fu = K.fx; e.fv = K.fy; e.uc = K.cx; e.vc = K.cy;
    e.pws = w + PW_PWS;
    e.us = w + PW_US;
    e.alphas = w + PW_AL;
    e.cws = reinterpret_cast<const double (*)[3]>(w + PW_CWS);
    const double (*nv)[12] = reinterpret_cast<const double (*)[12]>(w + PW_NV);
    // L (6x10) and rho are the same for the group's three approximations: lane 0 forms them
    if (l == 0) e.prep(nv, L, L + 60);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    double R[9], t[3];
    const double err = e.approx(l < 3 ? l + 1 : 3, L, L + 60, nv, R, t);
    const int gb = threadIdx.x & ~3;
    const double e1 = __shfl(err, gb + 1, 64), e2 = __shfl(err, gb + 2, 64);
    int sel = 0;
    double best = __shfl(err, gb, 64);
    if (e1 < best) { best = e1; sel = 1; }
    if (e2 < best) sel = 2;
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = __shfl(R[k], gb + sel, 64);
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = __shfl(t[k], gb + sel, 64);
    double r[3], dR[27];
    rod_R2r(R, r);
    if (l == 0) {
      double* mo = model + ((int64_t)b * maxIters + it) * 6;
      for (int i = 0; i < 3; ++i) { mo[i] = r[i]; mo[3 + i] = t[i]; }
    }
    rod_r2R(r, R, dR);
    int gcount = 0;
#pragma nounroll
    for (int i = l; i < n; i += 4) {
      double M[3] = {(double)P3[3 * i], (double)P3[3 * i + 1], (double)P3[3 * i + 2]}, uv[2];
      dproject(K, R, dR, t, M, uv, nullptr);
      float du = p2[2 * i] - (float)uv[0], dv = p2[2 * i + 1] - (float)uv[1];
      gcount += (du * du + dv * dv) <= thr2;
    }
    gcount += __shfl_xor(gcount, 1, 4);
    gcount += __shfl_xor(gcount, 2, 4);
    if (l == 0) good[(int64_t)b * maxIters + it] = gcount;
  });
}

// One wave per frame: 64 iterations' counts loaded at once, then walked in order with
// wave-uniform reads (a lane per frame walking global memory was 73 us per launch).
__global__ __launch_bounds__(64) void k_pnp_replay(int maxIters, int it_lo, int it_hi, double conf,
                                                   const int32_t* __restrict__ good, PnpState* __restrict__ state) {
  const int b = blockIdx.x, lane = threadIdx.x;
  PnpState st = state[b];
  if (st.n < 6) return;
  for (int base = it_lo; base < it_hi && base < st.niters; base += 64) {
    const int it = base + lane;
    const int g = (it < it_hi && it < st.niters) ? good[(int64_t)b * maxIters + it] : 0;
    for (int j = 0; j < 64; ++j) {
      if (base + j >= it_hi || base + j >= st.niters) break;
      const int gj = __builtin_amdgcn_readlane(g, j);
      if (gj > max(st.maxGood, 4)) {
        st.best_it = base + j;
        st.maxGood = gj;
        st.niters = update_num_iters(conf, (double)(st.n - gj) / st.n, 5, st.niters);
      }
    }
  }
  if (lane == 0) state[b] = st;
}

__global__ __launch_bounds__(64, 2) void k_pnp_refine(const float* __restrict__ P3all, const float* __restrict__ p2all,
                                                   int cap, Cam K, float thr2, int maxIters,
                                                   const PnpState* __restrict__ state,
                                                   const double* __restrict__ model, double* __restrict__ rvec,
                                                   double* __restrict__ tvec, double* __restrict__ T,
                                                   int32_t* __restrict__ status, uint8_t* __restrict__ inliers,
                                                   int32_t* __restrict__ inl_idx, double* __restrict__ mn_buf,
                                                   float* __restrict__ pts) {
  __shared__ PnpShared sh;
  __shared__ float s_pts[5 * kRefineLds];  // the inliers' P3 then p2, compacted, when they fit
  const int b = blockIdx.x, lane = threadIdx.x;
  const PnpState st = state[b];
  const int n = st.n;
  const float* P3 = P3all + (int64_t)b * cap * 3;
  const float* p2 = p2all + (int64_t)b * cap * 2;
  double* Tout = T + (int64_t)b * 16;
  if (n < 6 || st.maxGood <= 0) {
    if (lane < 16) Tout[lane] = (lane % 5 == 0) ? 1.0 : 0.0;
    if (lane < 3) { rvec[b * 3 + lane] = 0; tvec[b * 3 + lane] = 0; }
    if (inliers)
      for (int i = lane; i < cap; i += 64) inliers[(int64_t)b * cap + i] = 0;
    if (lane == 0) status[b] = n < 6 ? -1 : 0;
    return;
  }
  const double* mo = model + ((int64_t)b * maxIters + st.best_it) * 6;
  if (lane < 6) sh.best[lane] = mo[lane];
  __syncthreads();
  int* inl = inl_idx + (int64_t)b * cap;
  {
    double r[3] = {sh.best[0], sh.best[1], sh.best[2]}, t[3] = {sh.best[3], sh.best[4], sh.best[5]};
    double R[9], dR[27];
    rod_r2R(r, R, dR);
    int carry = 0;
    for (int base = 0; base < n; base += 64) {
      int i = base + lane;
      bool f = false;
      if (i < n) {
        double M[3] = {(double)P3[3 * i], (double)P3[3 * i + 1], (double)P3[3 * i + 2]}, uv[2];
        dproject(K, R, dR, t, M, uv, nullptr);
        float du = p2[2 * i] - (float)uv[0], dv = p2[2 * i + 1] - (float)uv[1];
        f = du * du + dv * dv <= thr2;
        if (inliers) inliers[(int64_t)b * cap + i] = (uint8_t)f;
      }
      unsigned long long m = __ballot(f);
      if (f) {
        const int k = carry + __popcll(m & ((1ull << lane) - 1ull));
        inl[k] = i;
        if (k < kRefineLds) {
          s_pts[3 * k] = P3[3 * i];
          s_pts[3 * k + 1] = P3[3 * i + 1];
          s_pts[3 * k + 2] = P3[3 * i + 2];
          s_pts[3 * kRefineLds + 2 * k] = p2[2 * i];
          s_pts[3 * kRefineLds + 2 * k + 1] = p2[2 * i + 1];
        }
      }
      carry += __popcll(m);
    }
    if (inliers)
      for (int i = n + lane; i < cap; i += 64) inliers[(int64_t)b * cap + i] = 0;
    if (lane == 0) sh.ninl = carry;
  }
  __syncthreads();
  // the LM's evaluations read every inlier several times: from LDS (~100 cycles) instead of a
  // dependent global gather per point (~1 us) -- or, past kRefineLds inliers, compacted in the
  // global buffer pts (same values: the results do not depend on where they are read from)
  const int ninl = sh.ninl;
  const float* Pc = s_pts;
  const float* Qc = s_pts + 3 * kRefineLds;
  if (ninl > kRefineLds) {
    float* gP = pts + (int64_t)b * cap * 5;
    float* gQ = gP + 3 * cap;
    for (int k = lane; k < ninl; k += 64) {
      const int i = inl[k];
      gP[3 * k] = P3[3 * i];
      gP[3 * k + 1] = P3[3 * i + 1];
      gP[3 * k + 2] = P3[3 * i + 2];
      gQ[2 * k] = p2[2 * i];
      gQ[2 * k + 1] = p2[2 * i + 1];
    }
    __syncthreads();
    Pc = gP;
    Qc = gQ;
  }
  lm_refine(sh, K, Pc, Qc, ninl, mn_buf + (int64_t)b * cap * 2);
  double out[6];
  for (int i = 0; i < 6; ++i) out[i] = sh.flag ? sh.param[i] : sh.best[i];
  if (lane == 0) {
    double R[9];
    rod_r2R(out, R, nullptr);
    for (int i = 0; i < 3; ++i) {
      rvec[b * 3 + i] = out[i];
      tvec[b * 3 + i] = out[3 + i];
      Tout[i * 4 + 0] = R[i * 3];
      Tout[i * 4 + 1] = R[i * 3 + 1];
      Tout[i * 4 + 2] = R[i * 3 + 2];
      Tout[i * 4 + 3] = out[3 + i];
    }
    Tout[12] = 0; Tout[13] = 0; Tout[14] = 0; Tout[15] = 1;
    status[b] = 1;
  }
}

}  // namespace

int pose_init(fvo_ctx* ctx) {
  ctx->pnp_max_iters = 1000;
  const int64_t B = ctx->cfg.max_batch, n = B * ctx->kp_cap, it = B * ctx->pnp_max_iters;
  int rc;
  if ((rc = fvo_alloc(ctx, &ctx->pnp_sub, n)) || (rc = fvo_alloc(ctx, &ctx->pnp_hyp, 2 * n)) ||
      (rc = ransac_table_init(ctx)) || (rc = fvo_alloc(ctx, &ctx->pnp_models, it * 6)) ||
      (rc = fvo_alloc(ctx, &ctx->pnp_ws, it * PNP_WS)) ||
      (rc = hipFuncSetAttribute((const void*)k_pnp_setup, hipFuncAttributeMaxDynamicSharedMemorySize,
                                144 * 64 * (int)sizeof(double)) == hipSuccess ? 0 : fvo_fail(ctx, "pnp: LDS attribute")) ||
      (rc = fvo_alloc(ctx, &ctx->pnp_good, it)) || (rc = fvo_alloc(ctx, (PnpState**)&ctx->pnp_state, B)) ||
      (rc = fvo_alloc(ctx, &ctx->pnp_plan, 3 * (B + 1))) || (rc = fvo_alloc(ctx, &ctx->pnp_pts, 5 * n)))
    return rc;
  return 0;
}

// The RNG(-1) subset table shared by PnP and the essential-matrix RANSAC (both draw 5-point
// subsets with getSubset() from a fresh RNG(-1) per call): built once per context.
int ransac_table_init(fvo_ctx* ctx) {
  if (ctx->rs_table) return 0;
  ctx->rs_table_iters = 1000;
  int rc;
  if ((rc = fvo_alloc(ctx, &ctx->rs_table, (int64_t)(ctx->kp_cap + 1) * ctx->rs_table_iters * 5))) return rc;
  hipLaunchKernelGGL(k_pnp_table, dim3((ctx->kp_cap + 1 + 63) / 64), dim3(64), 0, 0, ctx->kp_cap,
                     ctx->rs_table_iters, ctx->rs_table);
  FVO_LAUNCH_CHECK(ctx);
  FVO_HIP(ctx, hipDeviceSynchronize());
  return 0;
}

int backproject_run(fvo_ctx* ctx, const int16_t* disp, const float* kp0, const float* kp1, const int32_t* matches,
                    const int32_t* nmatch, int batch, int cap, const double* K, double baseline, float* P3, float* p2,
                    int32_t* npts, hipStream_t s) {
  CamF c{K[0], K[4], K[2], K[5], K[0] * baseline};
  FVO_TIMED(ctx, KN_BACKPROJECT, s, hipLaunchKernelGGL(k_backproject, dim3(batch), dim3(256), 0, s, disp, kp0, kp1,
                                                       matches, nmatch, ctx->cfg.width, ctx->cfg.height, cap, c, P3,
                                                       p2, npts));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

int pnp_run(fvo_ctx* ctx, const float* P3, const float* p2, const int32_t* npts, int batch, int cap, const double* K,
            const double* dist, float reproj, double conf, int iters, double* rvec, double* tvec, double* T,
            int32_t* status, uint8_t* inliers, hipStream_t s) {
  if (cap > ctx->kp_cap) return fvo_fail(ctx, "pnp: cap exceeds the context keypoint capacity");
  Cam c{K[0], K[4], K[2], K[5], {dist[0], dist[1], dist[2], dist[3], dist[4]}};
  const float thr2 = (float)((double)reproj * reproj);
  const int maxIters = iters;
  PnpState* st = (PnpState*)ctx->pnp_state;
  const int first = std::min(maxIters, PNP_FIRST);
  auto hyp = [&](const int32_t* plan, dim3 gs, dim3 ga, dim3 gb, int lo, int hi) {
    hipLaunchKernelGGL(k_pnp_setup, gs, dim3(64), 144 * 64 * sizeof(double), s, P3, p2, cap, c, maxIters, batch, plan,
                       ctx->rs_table, ctx->rs_table_iters, st, ctx->pnp_ws);
    hipLaunchKernelGGL(k_pnp_hyp_a, ga, dim3(64), 0, s, maxIters, batch, plan, st, ctx->pnp_ws);
    hipLaunchKernelGGL(k_pnp_hyp_b, gb, dim3(64), 0, s, P3, p2, cap, c, thr2, maxIters, batch, plan, st, ctx->pnp_ws,
                       ctx->pnp_models, ctx->pnp_good);
    hipLaunchKernelGGL(k_pnp_replay, dim3(batch), dim3(64), 0, s, maxIters, lo, hi, conf, ctx->pnp_good, st);
  };
  FVO_TIMED(ctx, KN_PNP, s, {
    hipLaunchKernelGGL(k_pnp_subsets, dim3((batch + 63) / 64), dim3(64), 0, s, npts, batch, cap, maxIters, st);
    hyp(nullptr, dim3((first + PNP_CS - 1) / PNP_CS, batch), dim3((first + PNP_CA - 1) / PNP_CA, batch),
        dim3((first + PNP_CB - 1) / PNP_CB, batch), 0, first);
    if (maxIters > first) {
      hipLaunchKernelGGL(k_pnp_plan, dim3(1), dim3(64), 0, s, batch, maxIters, st, ctx->pnp_plan);
      const int gs = batch * ((PNP_FIRST + PNP_CS - 1) / PNP_CS), ga = batch * ((PNP_FIRST + PNP_CA - 1) / PNP_CA),
                gb = batch * ((PNP_FIRST + PNP_CB - 1) / PNP_CB);
      hyp(ctx->pnp_plan, dim3(gs), dim3(ga), dim3(gb), first, maxIters);
    }
    hipLaunchKernelGGL(k_pnp_refine, dim3(batch), dim3(64), 0, s, P3, p2, cap, c, thr2, maxIters, st,
                       ctx->pnp_models, rvec, tvec, T, status, inliers, ctx->pnp_sub, ctx->pnp_hyp, ctx->pnp_pts);
  });
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
