// Windowed local bundle adjustment for gfx950 (BASELINE.json north_star
// "extract+match+local-BA").  The reference chains PnP poses only (stereo_slam.py:306);
// this stage refines each frame's relative pose over the window of the last K frames.
// The specification — landmark construction, residuals, robust weights, LM schedule —
// is oracle/ba_ref.py; this file implements it in fp64.
//
// Problem construction, one block per window:
//   k_ba_stereo  per keypoint, the reference's float32 back-projection through the
//                disparity map (the fvo_backproject arithmetic) -> (X, Y, Z, d)
//   k_ba_build   match-chain landmarks (ordered births via block scans), landmark-major
//                observations, per-frame observation lists, initial poses / LM state
// One LM iteration = five launches whose grids span every window x chunk, so the whole
// GPU works on the batch of windows (one block per window would leave most CUs idle and
// every phase latency-bound):
//   k_ba_pp      (window, frame): H_pp, g_p of the frame's observations (deterministic
//                block reduction) and W = J_p^T w J_l per observation
//   k_ba_lin     (window, landmark chunk): H_ll, g_l, damped 3x3 Cholesky L_l; the chunk's
//                Y = W L_l^-T rows and z = L_l^-1 g_l are laid out in LDS as Yt [3 LPC][NR]
//                and contracted on MFMA (v_mfma_f64_16x16x4_f64, upper 16x16 tiles):
//                G_chunk = Yt^T Yt = sum_l W H_ll^-1 W^T (the Schur complement term) with
//                its last column W H_ll^-1 g — the dense J^T J block contraction
//   k_ba_solve   (window): S = H_pp + lam diag + 1e-6 I - sum_chunks G, Cholesky (fp64, LDS),
//                pose step, tentative poses
//   k_ba_upd     (window, 8-16 landmarks): back-substitution X' = X + H_ll^-1 (-g - W^T dp),
//                cost partials at the tentative point
//   k_ba_accept  (window): LM accept / reject, lambda update
// fp64 everywhere (the GEMM too): S = H_pp - G cancels, and with fp32 operands the refined
// poses moved by 1.3e-4 against the fp64 oracle (measured), outside north_star's 1e-4.
// All reductions have a fixed order, so results are run-to-run deterministic.
#include <cfloat>
#include <type_traits>

#include "fvo_device.h"

namespace {

struct BaObs {
  int lm;
  short frame, oct;  // window-relative frame; ORB octave (weight 1 / scale^(2 oct)), -1 = rejected
  float u, v, ur;    // ur NaN: mono observation
};

struct BaCam {
  double fx, fy, cx, cy, b;
};

constexpr int kKMax = 21;
// parallel problem construction scratch per window (ints): births per birth frame [kKMax],
// their observations [kKMax], created landmarks / observations [2], observations per frame [kKMax]
constexpr int kBldL = 0, kBldO = kKMax, kBldTot = 2 * kKMax, kBldF = 2 * kKMax + 2, kBldInts = 3 * kKMax + 2;
constexpr int kBlock = 256;
// k_ba_lin: blocks per window NPART = (chunk capacity) / kLinChunksPerPart, clamped to [1,
// kLinParts]; block p reduces the landmark chunks p, p + NPART, ...
// into one partial Schur product (MFMA accumulators kept across its chunks), so k_ba_solve
// sums NPART partials instead of one per chunk.  Fixed chunk order: deterministic.  The
// count matters in the overlapped pipeline: each k_ba_lin block holds a whole CU (its LDS
// slice), so more, shorter blocks evict the concurrent front stage from more CUs per LM
// iteration, fewer leave the BA latency-bound.  Measured (bench.py, overlapped): 600p / 64
// windows / 64 chunks: 16 parts 4770 frames/s, 8: 4787, 4: 4848, 2: 4556, 1: 4054; 1080p /
// 32 windows / 256 chunks: 16 parts 1219, 8: 1120, 4: 1125.
// r6: at most 12 parts -- at 1080p (16 windows per stream, 16 parts) one stream's k_ba_lin took
// every CU and the other stream's k_ba_solve waited for it; with 12, 64 CUs stay free for it:
// BA 1080p 3.99-4.05 -> 3.74 ms in order (16 / 15 / 14 / 12 / 10 / 8 / 6 parts: 4.03 / 3.82 / 3.77
// / 3.74 / 3.87 / 3.93 / 4.43 ms), overlapped 1080p bench 1542-1544 -> 1545-1555 frames/s; 600p
// (4 parts) unchanged, 3 / 2 parts slower there (1.82 / 2.29 vs 1.63 ms)
// r6, after the producer/consumer split: 8 chunks per part (600p: 8 parts instead of 4; 1080p
// still clamped at 12): 600p BA 1.52 -> 1.48-1.49 ms, overlapped 5757-5759 -> 5766-5772 frames/s
// (11 / 6 / 4 chunks per part: 1.48-1.50 / 1.66 / 1.59-1.60 ms)
constexpr int kLinParts = 12, kLinChunksPerPart = 8;
// landmarks per k_ba_lin chunk at NR = 64 (half at NR = 128); measured: 32 / 16 per chunk
// (4610 / 4404 frames/s) and two 8-wave blocks per CU (4796) lose to one 16-wave block with 64
constexpr int kLinLPC64 = 64, kLinWavesDefault = 16;
// k_ba_lin runs a group of kLinBlock / LPC lanes per landmark inside one wave: LPC >= 16
static_assert(64 * kLinWavesDefault / (kLinLPC64 / 2) <= 64 && 64 * kLinWavesDefault / kLinLPC64 >= 16,
              "a landmark's lane group fits one wave and holds K observations");
// k_ba_lin runs 16 waves per block: its LDS slice (up to 150 KB) allows one block per CU, so
// the block's own waves are all the latency hiding the CU gets
constexpr int kLinWaves = kLinWavesDefault, kLinBlock = 64 * kLinWaves;
// r6: the block's waves split into producers (the landmark blocks and Y rows of half a chunk,
// VALU) and consumers (the MFMA contraction of the previous half) over a double-buffered Y
constexpr int kLinProd = kLinWaves / 2, kLinCons = kLinWaves - kLinProd;
constexpr int kLinMaxTiles = (36 + kLinCons - 1) / kLinCons;  // 16x16 tiles per consumer wave: 36 upper tiles at NR = 128
constexpr int kLinTiles64 = (10 + kLinCons - 1) / kLinCons;   // 10 upper tiles at NR = 64
// a half chunk (LPC / 2 landmarks, 3 Y rows each) fits s_tm's 32 slots, its 4-row MFMA steps one
// lane each, and its lane groups the producer waves
static_assert(kLinLPC64 / 2 <= 32 && (3 * (kLinLPC64 / 4)) % 4 == 0 && 3 * (kLinLPC64 / 2) / 4 <= 64,
              "half-chunk shape");
static_assert((64 * kLinProd) % (kLinLPC64 / 2) == 0, "producer lanes split evenly over a half chunk");
constexpr double kD2Mono = 5.991, kD2Stereo = 7.815, kMinZ = 0.01, kLam0 = 1e-3;

struct BaState {
  double T[kKMax][12], Tt[kKMax][12];  // poses [R row-major | t], current / tentative
  double dp[6 * kKMax];
  double Hpp[kKMax][27];  // per frame: 21 upper entries of H_pp, then g_p
  double lam, cost, cost0;
  int parity, fail, acc, active, L, O, n, s;
};

struct BaDims {
  int Lmax, Omax, K, cap, NR, LPC, NCH, NCU, NPART, LPU, NCUP;
  int64_t oSt, oX0, oX1, oL, oG, oLs, oObs, oFl, oGp, oCp, oNext, oHdr, oBld, win;
};

struct BaWin {
  BaState* st;
  double *X0, *X1, *Lf, *gl, *Gp, *cp;
  int *lstart, *flist, *next, *hdr, *bld;
  BaObs* obs;
};

__device__ __forceinline__ BaWin view(void* base, const BaDims& d, int w) {
  char* p = (char*)base + d.win * w;
  BaWin v;
  v.st = (BaState*)(p + d.oSt);
  v.X0 = (double*)(p + d.oX0);
  v.X1 = (double*)(p + d.oX1);
  v.Lf = (double*)(p + d.oL);
  v.gl = (double*)(p + d.oG);
  v.lstart = (int*)(p + d.oLs);
  v.obs = (BaObs*)(p + d.oObs);
  v.flist = (int*)(p + d.oFl);
  v.Gp = (double*)(p + d.oGp);
  v.cp = (double*)(p + d.oCp);
  v.next = (int*)(p + d.oNext);
  v.hdr = (int*)(p + d.oHdr);
  v.bld = (int*)(p + d.oBld);
  return v;
}
// hdr: [8 + f] per-frame observation list offsets

// exclusive block scan of v (blockDim = kBlock); returns prefix, *total = block sum
__device__ int block_scan(int v, int* s_tmp, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[wid] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kBlock / 64; ++k) {
    if (k < wid) pre += s_tmp[k];
    tot += s_tmp[k];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// the same for a block of NT threads
template <int NT>
__device__ int block_scan_n(int v, int* s_tmp, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[wid] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) {
    if (k < wid) pre += s_tmp[k];
    tot += s_tmp[k];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// deterministic block sum of doubles (fixed tree); result valid in every thread
__device__ double block_sum(double v, double* s_red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0;
#pragma unroll
  for (int k = 0; k < kBlock / 64; ++k) t += s_red[k];
  __syncthreads();
  return t;
}

// ------------------------------------------------------------------ stereo points
__global__ void k_ba_stereo(const int16_t* __restrict__ disp, const float* __restrict__ kp,
                            const int32_t* __restrict__ nkp, int W, int H, int cap, double fx, double fy, double cx,
                            double cy, double fxB, float4* __restrict__ out) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  int n = nkp[b];
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n) {
    const float* a = kp + ((int64_t)b * cap + i) * FVO_KP_STRIDE;
    const float x = a[0], y = a[1];
    int xi = min(max((int)x, 0), W - 1), yi = min(max((int)y, 0), H - 1);
    const float lo = (float)0.1, hi = 1000.f;
    float d = (float)disp[((int64_t)b * H + yi) * W + xi] / 16.f;
    if (d == 0.0f) d = lo;
    if (d == -1.0f) d = lo;
    const float Z = (float)fxB / d;
    const float X = ((x - (float)cx) / (float)fx) * Z;
    const float Y = ((y - (float)cy) / (float)fy) * Z;
    if (Z > lo && Z < hi) r = make_float4(X, Y, Z, d);
  }
  out[(int64_t)b * cap + i] = r;
}

// ------------------------------------------------------------------ geometry helpers
struct BaIn {
  const float* kp;
  const int32_t* nkp;
  const int32_t* matches;
  const int32_t* nmatch;
  const float4* stereo;
  const double* Trel;
  double isig2[FVO_MAX_LEVELS];  // per-octave weights, by value
  int nlev;
};

// T = [R (9, row-major) | t (3)];  C = A * B (rigid)
__device__ __forceinline__ void mat_mul_T(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    C[9 + i] = A[3 * i] * B[9] + A[3 * i + 1] * B[10] + A[3 * i + 2] * B[11] + A[9 + i];
  }
}

__device__ __forceinline__ void exp_so3(const double* w, double* R) {
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  if (th < 1e-12) {
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double kx = w[0] / th, ky = w[1] / th, kz = w[2] / th;
  const double K[9] = {0, -kz, ky, kz, 0, -kx, -ky, kx, 0};
  double K2[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) K2[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
  const double s = sin(th), c1 = 1.0 - cos(th);
  for (int i = 0; i < 9; ++i) R[i] = ((i % 4 == 0) ? 1.0 : 0.0) + s * K[i] + c1 * K2[i];
}

// 1 / sqrt(d): the hardware estimate refined by one Newton step (relative error ~1e-15)
// a lane's double, read by the whole wave (two v_readlane_b32)
__device__ __forceinline__ double rl_f64(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double rsq_r(double d) {
  const double r = __builtin_amdgcn_rsq(d);
  return r * fma(-0.5 * d * r, r, 1.5);
}

// observation weight 1 / sigma2[octave]; 0 once the observation was rejected (oct = -1)
__device__ __forceinline__ double obs_is2(const BaIn& in, const BaObs& o) {
  return o.oct < 0 ? 0.0 : in.isig2[o.oct];
}

// residual, robust weight (x information) and cost of one observation; Jacobians if J (the
// pose Jacobian Jp only if JP)
template <bool J, bool JP = true, bool JL = true>
__device__ __forceinline__ void ba_eval(const double* T, const double* X, const BaObs& o, const BaCam& c,
                                        double is2, double* r, double& w, double& rho, double (*Jp)[6],
                                        double (*Jl)[3]) {
  const double x = T[0] * X[0] + T[1] * X[1] + T[2] * X[2] + T[9];
  const double y = T[3] * X[0] + T[4] * X[1] + T[5] * X[2] + T[10];
  const double z = T[6] * X[0] + T[7] * X[1] + T[8] * X[2] + T[11];
  const bool ok = z > kMinZ;
  const double iz = 1.0 / (ok ? z : 1.0);
  const bool st = !isnan(o.ur);
  r[0] = c.fx * x * iz + c.cx - (double)o.u;
  r[1] = c.fy * y * iz + c.cy - (double)o.v;
  r[2] = st ? c.fx * (x - c.b) * iz + c.cx - (double)o.ur : 0.0;
  const double s = (r[0] * r[0] + r[1] * r[1] + r[2] * r[2]) * is2;
  const double d2 = st ? kD2Stereo : kD2Mono;
  const bool inl = s <= d2;
  rho = ok ? (inl ? s : 2.0 * sqrt(d2 * s) - d2) : 0.0;
  w = ok ? (inl ? 1.0 : sqrt(d2 / fmax(s, 1e-300))) * is2 : 0.0;
  if (!J) return;
  const double Jc[3][3] = {{c.fx * iz, 0.0, -c.fx * x * iz * iz},
                           {0.0, c.fy * iz, -c.fy * y * iz * iz},
                           {st ? c.fx * iz : 0.0, 0.0, st ? -c.fx * (x - c.b) * iz * iz : 0.0}};
  // d(Xc)/d(w, v) = [-[Xc]x | I]
  const double sk[3][6] = {{0.0, z, -y, 1.0, 0.0, 0.0}, {-z, 0.0, x, 0.0, 1.0, 0.0}, {y, -x, 0.0, 0.0, 0.0, 1.0}};
  for (int k = 0; k < 3; ++k) {
    if (JP)
      for (int j = 0; j < 6; ++j) Jp[k][j] = Jc[k][0] * sk[0][j] + Jc[k][1] * sk[1][j] + Jc[k][2] * sk[2][j];
    if (JL)
      for (int j = 0; j < 3; ++j) Jl[k][j] = Jc[k][0] * T[j] + Jc[k][1] * T[3 + j] + Jc[k][2] * T[6 + j];
  }
}

// Residual, weight, cost, J_l and what the pose / landmark coupling block W = J_p^T w J_l
// (6 x 3) of one observation is made of, without forming J_p: with J_c the projection
// Jacobian and J_p = J_c [-[X_c]x | I], W = w [-[X_c]x | I]^T M with M = J_c^T J_l, so a row
// of W (ba_wrow) is w times a row of M (translation) or a skew combination of M's rows
// (rotation).  M and X_c take fewer live registers than J_p or W; k_ba_lin and k_ba_upd form
// W's rows with the same arithmetic.
struct BaCoupling {
  double M[3][3];  // J_c^T J_l
  double xc[3];    // the point in the camera frame
  double w;
};
__device__ __forceinline__ void ba_eval_lw(const double* T, const double* X, const BaObs& o, const BaCam& c,
                                           double is2, double* r, double& rho, double (*Jl)[3], BaCoupling& cp) {
  const double x = T[0] * X[0] + T[1] * X[1] + T[2] * X[2] + T[9];
  const double y = T[3] * X[0] + T[4] * X[1] + T[5] * X[2] + T[10];
  const double z = T[6] * X[0] + T[7] * X[1] + T[8] * X[2] + T[11];
  const bool ok = z > kMinZ;
  const double iz = 1.0 / (ok ? z : 1.0);
  const bool st = !isnan(o.ur);
  r[0] = c.fx * x * iz + c.cx - (double)o.u;
  r[1] = c.fy * y * iz + c.cy - (double)o.v;
  r[2] = st ? c.fx * (x - c.b) * iz + c.cx - (double)o.ur : 0.0;
  const double s = (r[0] * r[0] + r[1] * r[1] + r[2] * r[2]) * is2;
  const double d2 = st ? kD2Stereo : kD2Mono;
  const bool inl = s <= d2;
  rho = ok ? (inl ? s : 2.0 * sqrt(d2 * s) - d2) : 0.0;
  cp.w = ok ? (inl ? 1.0 : sqrt(d2 / fmax(s, 1e-300))) * is2 : 0.0;
  const double Jc[3][3] = {{c.fx * iz, 0.0, -c.fx * x * iz * iz},
                           {0.0, c.fy * iz, -c.fy * y * iz * iz},
                           {st ? c.fx * iz : 0.0, 0.0, st ? -c.fx * (x - c.b) * iz * iz : 0.0}};
  for (int k = 0; k < 3; ++k)
    for (int j = 0; j < 3; ++j) Jl[k][j] = Jc[k][0] * T[j] + Jc[k][1] * T[3 + j] + Jc[k][2] * T[6 + j];
  for (int q = 0; q < 3; ++q)
    for (int k = 0; k < 3; ++k) cp.M[q][k] = Jc[0][q] * Jl[0][k] + Jc[1][q] * Jl[1][k] + Jc[2][q] * Jl[2][k];
  cp.xc[0] = x;
  cp.xc[1] = y;
  cp.xc[2] = z;
}

// row a of W: rows of [-[X_c]x]^T are a = 0: (0, -z, y), 1: (z, 0, -x), 2: (-y, x, 0)
__device__ __forceinline__ void ba_wrow(const BaCoupling& cp, int a, double* wr) {
  const double x = cp.xc[0], y = cp.xc[1], z = cp.xc[2];
  for (int k = 0; k < 3; ++k) {
    const double m = a == 0 ? y * cp.M[2][k] - z * cp.M[1][k]
                   : a == 1 ? z * cp.M[0][k] - x * cp.M[2][k]
                   : a == 2 ? x * cp.M[1][k] - y * cp.M[0][k]
                            : cp.M[a - 3][k];
    wr[k] = cp.w * m;
  }
}

// outlier test of oracle/ba_ref.py _reject (current estimate)
__device__ __forceinline__ bool ba_outlier(const double* T, const double* X, const BaObs& o, const BaCam& c,
                                           double is2) {
  const double x = T[0] * X[0] + T[1] * X[1] + T[2] * X[2] + T[9];
  const double y = T[3] * X[0] + T[4] * X[1] + T[5] * X[2] + T[10];
  const double z = T[6] * X[0] + T[7] * X[1] + T[8] * X[2] + T[11];
  const bool ok = z > kMinZ;
  const double iz = 1.0 / (ok ? z : 1.0);
  const bool st = !isnan(o.ur);
  const double r0 = c.fx * x * iz + c.cx - (double)o.u;
  const double r1 = c.fy * y * iz + c.cy - (double)o.v;
  const double r2 = st ? c.fx * (x - c.b) * iz + c.cx - (double)o.ur : 0.0;
  const double s = (r0 * r0 + r1 * r1 + r2 * r2) * is2;
  return !(ok && s <= (st ? kD2Stereo : kD2Mono));
}

// ------------------------------------------------------------------ problem construction
// k_ba_build: one 512-thread block per window, birth frames in order.  Since r4 it runs only
// when the window's u16 match maps do not fit in LDS (LMAP = false: the maps in the global
// v.next copy); otherwise k_ba_births / k_ba_emit / k_ba_lists build the same problem on a
// (window, frame) grid (below; 1080p 0.55 ms -> BA 5.0 -> 4.63 ms, 600p 1.86 -> 1.81 ms,
// bit-identical results).  Following a track -- a chain of dependent lookups up to K-1 long --
// costs LDS latency with the maps in LDS; each candidate records its chain in registers on
// the first walk, and the keypoints along it are then loaded all at once.
constexpr int kBuildBlock = 512;
template <bool LMAP>
__global__ __launch_bounds__(kBuildBlock) void k_ba_build(BaIn in, void* ws, BaDims dm, int first_end, int first_valid) {
  extern __shared__ uint8_t s_dyn[];  // LMAP: [K-1][cap] u16 maps, then [cap] tracked flags
  __shared__ double sT[kKMax][12];
  __shared__ int s_tmp[kBuildBlock / 64];
  __shared__ int s_L, s_O, s_stop;
  const int w = blockIdx.x, tid = threadIdx.x;
  const int e = first_end + w;
  const int s = max(first_valid, e - dm.K + 1);
  const int n = e - s + 1;
  BaWin v = view(ws, dm, w);
  BaState* S = v.st;
  const int cap = dm.cap;
  uint16_t* s_next = reinterpret_cast<uint16_t*>(s_dyn);
  uint8_t* s_tracked = LMAP ? s_dyn + 2 * (dm.K - 1) * cap : s_dyn;
  auto nxt = [&](int k, int b) -> int {
    if (LMAP) {
      const int r = s_next[k * cap + b];
      return r == 0xFFFF ? -1 : r;
    }
    return v.next[k * cap + b];
  };
  if (tid == 0) {
    S->L = 0;
    S->O = 0;
    S->n = n;
    S->s = s;
    S->active = 0;
    s_L = 0;
    s_O = 0;
    s_stop = 0;
  }
  if (n < 3) return;
  if (tid == 0) {  // initial poses: T_0 = I, T_{k+1} = rel_{s+k} T_k
    for (int i = 0; i < 12; ++i) sT[0][i] = (i < 9 && i % 4 == 0) ? 1.0 : 0.0;
    for (int k = 0; k + 1 < n; ++k) {
      const double* M = in.Trel + (int64_t)(s + k) * 16;
      const double A[12] = {M[0], M[1], M[2], M[4], M[5], M[6], M[8], M[9], M[10], M[3], M[7], M[11]};
      mat_mul_T(A, sT[k], sT[k + 1]);
    }
  }
  // forward match maps of frames s..e-1
  for (int k = 0; k + 1 < n; ++k)
    for (int i = tid; i < cap; i += kBuildBlock) {
      if (LMAP) s_next[k * cap + i] = 0xFFFF;
      else v.next[k * cap + i] = -1;
    }
  __syncthreads();
  for (int k = 0; k + 1 < n; ++k) {
    const int f = s + k, M = min(max(in.nmatch[f], 0), cap);
    const int32_t* m = in.matches + (int64_t)f * cap * 3;
    for (int r = tid; r < M; r += kBuildBlock) {
      if (LMAP) s_next[k * cap + m[3 * r]] = (uint16_t)m[3 * r + 1];
      else v.next[k * cap + m[3 * r]] = m[3 * r + 1];
    }
  }
  __syncthreads();
  for (int j = 0; j + 1 < n; ++j) {
    const int f = s + j;
    for (int i = tid; i < cap; i += kBuildBlock) s_tracked[i] = 0;
    __syncthreads();
    if (j > 0) {
      const int Mp = min(max(in.nmatch[f - 1], 0), cap);
      const int32_t* mp = in.matches + (int64_t)(f - 1) * cap * 3;
      for (int r = tid; r < Mp; r += kBuildBlock) s_tracked[mp[3 * r + 1]] = 1;
    }
    __syncthreads();
    const int M = min(max(in.nmatch[f], 0), cap);
    const int32_t* m = in.matches + (int64_t)f * cap * 3;
    const double* Tj = sT[j];
    for (int base = 0; base < M; base += kBuildBlock) {
      if (s_stop) break;  // uniform: written before the last barrier
      const int r = base + tid;
      bool cand = false;
      int len = 0, q = 0;
      int bs[kKMax - 1];  // the track's keypoint in frames j+1, j+2, ... (static indices only)
      float4 sp = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < M) {
        q = m[3 * r];
        bs[0] = m[3 * r + 1];
        sp = in.stereo[(int64_t)f * cap + q];
        cand = !s_tracked[q] && sp.z > 0.f;
      }
      if (cand) {
        len = 2;
        bool go = true;
#pragma unroll
        for (int kk = 1; kk < kKMax - 1; ++kk) {  // frame j + kk + 1 from frame j + kk
          const int k = j + kk;
          if (go && k + 1 < n) {
            const int nb = nxt(k, bs[kk - 1]);
            if (nb < 0) go = false;
            else { bs[kk] = nb; ++len; }
          } else {
            go = false;
          }
        }
      }
      // one scan of (observations << 10 | candidate): len <= 21, so both sums fit
      int tp;
      const int packed = block_scan_n<kBuildBlock>((len << 10) | (cand ? 1 : 0), s_tmp, &tp);
      const int lid = packed & 1023, oof = packed >> 10, tl = tp & 1023, to = tp >> 10;
      const int L0 = s_L, O0 = s_O;
      // creation stops at the first landmark that does not fit (the failing rows are a
      // suffix of this chunk's candidates: both prefix sums are monotone); when the whole
      // chunk fits (the block totals say so, uniformly) no per-thread test is needed
      const bool allfit = L0 + tl <= dm.Lmax && O0 + to <= dm.Omax;
      const bool ok = cand && (allfit || ((L0 + lid < dm.Lmax) && (O0 + oof + len <= dm.Omax)));
      const int nok = allfit ? tl : __syncthreads_count(ok);
      const int nfail = allfit ? 0 : __syncthreads_count(cand && !ok);
      if (ok) {
        const int id = L0 + lid;
        int o = O0 + oof;
        // X_world = R^T (Xc - t)
        const double Xc[3] = {(double)sp.x - Tj[9], (double)sp.y - Tj[10], (double)sp.z - Tj[11]};
        for (int i = 0; i < 3; ++i) v.X0[3 * id + i] = Tj[i] * Xc[0] + Tj[3 + i] * Xc[1] + Tj[6 + i] * Xc[2];
        v.lstart[id] = o;
        const float* kq = in.kp + ((int64_t)f * cap + q) * FVO_KP_STRIDE;
        const int oq = min(max((int)kq[5], 0), in.nlev - 1);
        v.obs[o++] = BaObs{id, (short)j, (short)oq, kq[0], kq[1], kq[0] - sp.w};
        // the track's keypoints: every load issued before the first observation is written
        float ku[kKMax - 1], kvv[kKMax - 1], ko[kKMax - 1];
#pragma unroll
        for (int kk = 0; kk < kKMax - 1; ++kk)
          if (kk < len - 1) {
            const float* kb = in.kp + ((int64_t)(s + j + 1 + kk) * cap + bs[kk]) * FVO_KP_STRIDE;
            ku[kk] = kb[0];
            kvv[kk] = kb[1];
            ko[kk] = kb[5];
          }
#pragma unroll
        for (int kk = 0; kk < kKMax - 1; ++kk)
          if (kk < len - 1) {
            const int ob = min(max((int)ko[kk], 0), in.nlev - 1);
            v.obs[o++] = BaObs{id, (short)(j + 1 + kk), (short)ob, ku[kk], kvv[kk], __builtin_nanf("")};
          }
      }
      int tot_ok = to;
      if (!allfit) (void)block_scan_n<kBuildBlock>(ok ? len : 0, s_tmp, &tot_ok);
      if (tid == 0) {
        s_L = L0 + nok;
        s_O = O0 + tot_ok;
        if (nfail) s_stop = 1;
      }
      __syncthreads();
    }
    __syncthreads();
    if (s_stop) break;
  }
  __syncthreads();
  const int L = s_L, O = s_O;
  // per-frame observation lists (stable, landmark-major order inside a frame): a counting
  // sort -- frame sizes by LDS atomics, then per 512-observation chunk every wave ranks its
  // lanes within each frame by ballots, the waves' counts give the chunk's offsets (three
  // barriers per chunk instead of two per frame per chunk)
  __shared__ int s_fcnt[kKMax], s_foff[kKMax], s_wcnt[kBuildBlock / 64][kKMax];
  if (tid < kKMax) s_fcnt[tid] = 0;
  __syncthreads();
  for (int i = tid; i < O; i += kBuildBlock) atomicAdd(&s_fcnt[v.obs[i].frame], 1);
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int f = 0; f < n; ++f) {
      v.hdr[8 + f] = acc;
      s_foff[f] = acc;
      acc += s_fcnt[f];
    }
    v.hdr[8 + n] = acc;
  }
  __syncthreads();
  const int lane = tid & 63, wid = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int base = 0; base < O; base += kBuildBlock) {
    const int i = base + tid;
    const int f = i < O ? (int)v.obs[i].frame : -1;
    int rank = 0;
    for (int ff = 0; ff < n; ++ff) {
      const unsigned long long mk = __ballot(f == ff);
      if (f == ff) rank = __popcll(mk & lt);
      if (lane == 0) s_wcnt[wid][ff] = __popcll(mk);
    }
    __syncthreads();
    if (f >= 0) {
      int pos = s_foff[f] + rank;
      for (int w2 = 0; w2 < wid; ++w2) pos += s_wcnt[w2][f];
      v.flist[pos] = i;
    }
    __syncthreads();
    if (tid < n) {
      int c = 0;
      for (int w2 = 0; w2 < kBuildBlock / 64; ++w2) c += s_wcnt[w2][tid];
      s_foff[tid] += c;
    }
    __syncthreads();
  }
  if (tid == 0) {
    v.lstart[L] = O;
    S->L = L;
    S->O = O;
    S->active = L > 0;
    S->lam = kLam0;
    S->parity = 0;
    S->fail = 0;
    S->acc = 0;
    S->cost = 0.0;
    S->cost0 = 0.0;
  }
  for (int i = tid; i < n * 12; i += kBuildBlock) S->T[i / 12][i % 12] = sT[i / 12][i % 12];
}

// ---- parallel construction (r4): the same landmarks, ids, observations and per-frame lists
// as k_ba_build<true>, from a (window, frame) grid instead of one block per window.  A
// landmark is born at frame j from j's match rows alone (the tracked test reads frame j-1's
// matches, the track follows the maps of frames j+1..), so every birth frame is counted and
// emitted by its own block; the ids come from prefix sums over the birth frames, and the
// lists per observed frame from a scan over the landmarks.  Creation stops at the first
// candidate in (frame, row) order that does not fit: both prefix sums are monotone, so a
// candidate is created iff its all-candidate prefixes fit -- the same set as the serial stop.
// r6: 512 threads (half the row passes over a birth frame's matches in k_ba_emit; bit-identical):
// 1080p BA 3.24 -> 3.17-3.19 ms; 600p BA and overlapped bench within noise (two A/Bs: +0.8 %, -0.3 %)
constexpr int kBirthBlock = 512;

struct BirthFrame {
  int e, s, n, f, M;
  const int32_t* m;
};
__device__ __forceinline__ BirthFrame birth_frame(const BaIn& in, const BaDims& dm, int w, int j, int first_end,
                                                  int first_valid) {
  BirthFrame b;
  b.e = first_end + w;
  b.s = max(first_valid, b.e - dm.K + 1);
  b.n = b.e - b.s + 1;
  b.f = b.s + j;
  b.M = (b.n >= 3 && j + 1 < b.n) ? min(max(in.nmatch[b.f], 0), dm.cap) : 0;
  b.m = in.matches + (int64_t)b.f * dm.cap * 3;
  return b;
}

// the u16 forward maps of frames j+1 .. n-2 and frame j's tracked flags (from frame j-1's rows)
__device__ void birth_maps(const BaIn& in, const BaDims& dm, const BirthFrame& b, int j, uint16_t* s_next,
                           uint8_t* s_tr) {
  const int cap = dm.cap, tid = threadIdx.x;
  for (int k = j + 1; k + 1 < b.n; ++k)
    for (int i = tid; i < cap; i += kBirthBlock) s_next[k * cap + i] = 0xFFFF;
  for (int i = tid; i < cap; i += kBirthBlock) s_tr[i] = 0;
  __syncthreads();
  for (int k = j + 1; k + 1 < b.n; ++k) {
    const int f = b.s + k, M = min(max(in.nmatch[f], 0), cap);
    const int32_t* m = in.matches + (int64_t)f * cap * 3;
    for (int r = tid; r < M; r += kBirthBlock) s_next[k * cap + m[3 * r]] = (uint16_t)m[3 * r + 1];
  }
  if (j > 0) {
    const int Mp = min(max(in.nmatch[b.f - 1], 0), cap);
    const int32_t* mp = in.matches + (int64_t)(b.f - 1) * cap * 3;
    for (int r = tid; r < Mp; r += kBirthBlock) s_tr[mp[3 * r + 1]] = 1;
  }
  __syncthreads();
}

// row r of frame j: candidate test and track (len observations, keypoints bs[] in j+1, ...)
__device__ __forceinline__ bool birth_track(const BaIn& in, const BaDims& dm, const BirthFrame& b, int j, int r,
                                            const uint16_t* s_next, const uint8_t* s_tr, int& len, int& q,
                                            int (&bs)[kKMax - 1], float4& sp) {
  len = 0;
  q = 0;
  sp = make_float4(0.f, 0.f, 0.f, 0.f);
  if (r >= b.M) return false;
  q = b.m[3 * r];
  bs[0] = b.m[3 * r + 1];
  sp = in.stereo[(int64_t)b.f * dm.cap + q];
  if (s_tr[q] || !(sp.z > 0.f)) return false;
  len = 2;
  bool go = true;
#pragma unroll
  for (int kk = 1; kk < kKMax - 1; ++kk) {
    const int k = j + kk;
    if (go && k + 1 < b.n) {
      const int nb = s_next[k * dm.cap + bs[kk - 1]];
      if (nb == 0xFFFF) go = false;
      else { bs[kk] = nb; ++len; }
    } else {
      go = false;
    }
  }
  return true;
}

__device__ __forceinline__ int block_isum(int v, int* s_tmp) {  // all threads get the sum
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_tmp[threadIdx.x >> 6] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int k = 0; k < kBirthBlock / 64; ++k) t += s_tmp[k];
  __syncthreads();
  return t;
}

// (window, birth frame): candidate and observation counts of the frame's rows
__global__ __launch_bounds__(kBirthBlock) void k_ba_births(BaIn in, void* ws, BaDims dm, int first_end,
                                                           int first_valid) {
  extern __shared__ uint8_t s_dyn[];  // [K-1][cap] u16 maps, then [cap] tracked flags
  __shared__ int s_tmp[kBirthBlock / 64];
  const int w = blockIdx.x, j = blockIdx.y;
  BaWin v = view(ws, dm, w);
  const BirthFrame b = birth_frame(in, dm, w, j, first_end, first_valid);
  if (j == 0 && threadIdx.x < kBldInts - kBldTot) v.bld[kBldTot + threadIdx.x] = 0;  // emit's totals
  if (b.n < 3 || j + 1 >= b.n) {
    if (threadIdx.x == 0) { v.bld[kBldL + j] = 0; v.bld[kBldO + j] = 0; }
    return;
  }
  uint16_t* s_next = reinterpret_cast<uint16_t*>(s_dyn);
  uint8_t* s_tr = s_dyn + 2 * (dm.K - 1) * dm.cap;
  birth_maps(in, dm, b, j, s_next, s_tr);
  int nl = 0, no = 0;
  for (int r = threadIdx.x; r < b.M; r += kBirthBlock) {
    int len, q, bs[kKMax - 1];
    float4 sp;
    if (birth_track(in, dm, b, j, r, s_next, s_tr, len, q, bs, sp)) { ++nl; no += len; }
  }
  nl = block_isum(nl, s_tmp);
  no = block_isum(no, s_tmp);
  if (threadIdx.x == 0) { v.bld[kBldL + j] = nl; v.bld[kBldO + j] = no; }
}

// (window, birth frame): ids from the prefix over earlier birth frames, then the landmarks and
// their observations exactly as k_ba_build writes them
__global__ __launch_bounds__(kBirthBlock) void k_ba_emit(BaIn in, void* ws, BaDims dm, int first_end,
                                                         int first_valid) {
  extern __shared__ uint8_t s_dyn[];
  __shared__ double sTj[12];
  __shared__ int s_tmp[kBirthBlock / 64];
  __shared__ int s_fc[kKMax];
  const int w = blockIdx.x, j = blockIdx.y, tid = threadIdx.x;
  BaWin v = view(ws, dm, w);
  const BirthFrame b = birth_frame(in, dm, w, j, first_end, first_valid);
  if (b.M == 0) return;
  int L0 = 0, O0 = 0;
  for (int jj = 0; jj < j; ++jj) {
    L0 += v.bld[kBldL + jj];
    O0 += v.bld[kBldO + jj];
  }
  if (L0 >= dm.Lmax || O0 >= dm.Omax) return;  // every candidate of this frame fails
  if (tid < kKMax) s_fc[tid] = 0;
  if (tid == 0) {  // the pose of frame j: T_0 = I, T_{k+1} = rel_{s+k} T_k (k_ba_build's chain)
    double T[12], U[12];
    for (int i = 0; i < 12; ++i) T[i] = (i < 9 && i % 4 == 0) ? 1.0 : 0.0;
    for (int k = 0; k < j; ++k) {
      const double* M = in.Trel + (int64_t)(b.s + k) * 16;
      const double A[12] = {M[0], M[1], M[2], M[4], M[5], M[6], M[8], M[9], M[10], M[3], M[7], M[11]};
      mat_mul_T(A, T, U);
      for (int i = 0; i < 12; ++i) T[i] = U[i];
    }
    for (int i = 0; i < 12; ++i) sTj[i] = T[i];
  }
  uint16_t* s_next = reinterpret_cast<uint16_t*>(s_dyn);
  uint8_t* s_tr = s_dyn + 2 * (dm.K - 1) * dm.cap;
  birth_maps(in, dm, b, j, s_next, s_tr);  // (barriers: sTj / s_fc visible after it)
  int okl = 0, oko = 0;
  for (int base = 0; base < b.M; base += kBirthBlock) {
    const int r = base + tid;
    int len, q, bs[kKMax - 1];
    float4 sp;
    const bool cand = birth_track(in, dm, b, j, r, s_next, s_tr, len, q, bs, sp);
    int tp;
    const int packed = block_scan_n<kBirthBlock>((len << 10) | (cand ? 1 : 0), s_tmp, &tp);
    const int lid = packed & 1023, oof = packed >> 10;
    const bool ok = cand && L0 + lid < dm.Lmax && O0 + oof + len <= dm.Omax;
    if (ok) {
      const int id = L0 + lid;
      int o = O0 + oof;
      const double Xc[3] = {(double)sp.x - sTj[9], (double)sp.y - sTj[10], (double)sp.z - sTj[11]};
      for (int i = 0; i < 3; ++i) v.X0[3 * id + i] = sTj[i] * Xc[0] + sTj[3 + i] * Xc[1] + sTj[6 + i] * Xc[2];
      v.lstart[id] = o;
      const float* kq = in.kp + ((int64_t)b.f * dm.cap + q) * FVO_KP_STRIDE;
      const int oq = min(max((int)kq[5], 0), in.nlev - 1);
      v.obs[o++] = BaObs{id, (short)j, (short)oq, kq[0], kq[1], kq[0] - sp.w};
      float ku[kKMax - 1], kvv[kKMax - 1], ko[kKMax - 1];
#pragma unroll
      for (int kk = 0; kk < kKMax - 1; ++kk)
        if (kk < len - 1) {
          const float* kb = in.kp + ((int64_t)(b.f + 1 + kk) * dm.cap + bs[kk]) * FVO_KP_STRIDE;
          ku[kk] = kb[0];
          kvv[kk] = kb[1];
          ko[kk] = kb[5];
        }
#pragma unroll
      for (int kk = 0; kk < kKMax - 1; ++kk)
        if (kk < len - 1) {
          const int ob = min(max((int)ko[kk], 0), in.nlev - 1);
          v.obs[o++] = BaObs{id, (short)(j + 1 + kk), (short)ob, ku[kk], kvv[kk], __builtin_nanf("")};
        }
      for (int k = 0; k < len; ++k) atomicAdd(&s_fc[j + k], 1);
      ++okl;
      oko += len;
    }
    L0 += tp & 1023;
    O0 += tp >> 10;
    if (L0 >= dm.Lmax || O0 >= dm.Omax) break;  // uniform: the rest fails
  }
  okl = block_isum(okl, s_tmp);
  oko = block_isum(oko, s_tmp);
  if (tid == 0) {
    atomicAdd(&v.bld[kBldTot], okl);
    atomicAdd(&v.bld[kBldTot + 1], oko);
  }
  if (tid < kKMax && s_fc[tid]) atomicAdd(&v.bld[kBldF + tid], s_fc[tid]);
}

// (window, frame k): frame k's observation list in landmark order (a scan over the landmarks);
// block (w, 0) also writes the window's header, poses and LM state
__global__ __launch_bounds__(kBirthBlock) void k_ba_lists(BaIn in, void* ws, BaDims dm, int first_end,
                                                          int first_valid) {
  __shared__ int s_tmp[kBirthBlock / 64];
  const int w = blockIdx.x, k = blockIdx.y, tid = threadIdx.x;
  BaWin v = view(ws, dm, w);
  BaState* S = v.st;
  const int e = first_end + w, s = max(first_valid, e - dm.K + 1), n = e - s + 1;
  const bool live = n >= 3;
  const int L = live ? v.bld[kBldTot] : 0, O = live ? v.bld[kBldTot + 1] : 0;
  if (k == 0 && tid == 0) {
    S->L = L;
    S->O = O;
    S->n = n;
    S->s = s;
    S->active = L > 0;
    if (live) {
      v.lstart[L] = O;
      S->lam = kLam0;
      S->parity = 0;
      S->fail = 0;
      S->acc = 0;
      S->cost = 0.0;
      S->cost0 = 0.0;
      int acc = 0;
      for (int f = 0; f < n; ++f) {
        v.hdr[8 + f] = acc;
        acc += v.bld[kBldF + f];
      }
      v.hdr[8 + n] = acc;
      double T[12], U[12];
      for (int i = 0; i < 12; ++i) T[i] = (i < 9 && i % 4 == 0) ? 1.0 : 0.0;
      for (int f = 0; f < n; ++f) {
        for (int i = 0; i < 12; ++i) S->T[f][i] = T[i];
        if (f + 1 < n) {
          const double* M = in.Trel + (int64_t)(s + f) * 16;
          const double A[12] = {M[0], M[1], M[2], M[4], M[5], M[6], M[8], M[9], M[10], M[3], M[7], M[11]};
          mat_mul_T(A, T, U);
          for (int i = 0; i < 12; ++i) T[i] = U[i];
        }
      }
    }
  }
  if (!live || k >= n || L == 0) return;
  int pos = 0;
  for (int f = 0; f < k; ++f) pos += v.bld[kBldF + f];
  for (int base = 0; base < L; base += kBirthBlock) {
    const int l = base + tid;
    int o0 = 0, jl = 0, len = 0;
    if (l < L) {
      o0 = v.lstart[l];
      len = (l + 1 < L ? v.lstart[l + 1] : O) - o0;
      jl = v.obs[o0].frame;
    }
    const bool sees = l < L && jl <= k && k < jl + len;
    int tot;
    const int rank = block_scan_n<kBirthBlock>(sees ? 1 : 0, s_tmp, &tot);
    if (sees) v.flist[pos + rank] = o0 + (k - jl);
    pos += tot;
  }
}

// ------------------------------------------------------------------ LM iteration kernels
__device__ __forceinline__ const double* cur_X(const BaWin& v, const BaState* S) { return S->parity ? v.X1 : v.X0; }
__device__ __forceinline__ double* new_X(const BaWin& v, const BaState* S) { return S->parity ? v.X0 : v.X1; }

// cost partials at the current estimate, optionally rejecting outliers first
__global__ __launch_bounds__(kBlock) void k_ba_cost(BaIn in, void* ws, BaDims dm, BaCam cam, int reject) {
  __shared__ double s_red[kBlock / 64];
  const BaWin v = view(ws, dm, blockIdx.x);
  const BaState* S = v.st;
  if (!S->active) return;
  const int L = S->L, c = blockIdx.y;
  if (c * kBlock >= L) return;
  const double* X = cur_X(v, S);
  const int l = c * kBlock + threadIdx.x;
  double acc = 0;
  if (l < L) {
    for (int oi = v.lstart[l]; oi < v.lstart[l + 1]; ++oi) {
      BaObs o = v.obs[oi];
      if (reject && o.oct >= 0 && ba_outlier(S->T[o.frame], X + 3 * l, o, cam, in.isig2[o.oct])) {
        o.oct = -1;
        v.obs[oi].oct = -1;
      }
      double r[3], w, rho;
      ba_eval<false>(S->T[o.frame], X + 3 * l, o, cam, obs_is2(in, o), r, w, rho, nullptr, nullptr);
      acc += rho;
    }
  }
  const double t = block_sum(acc, s_red);
  if (threadIdx.x == 0) v.cp[c] = t;
}

__global__ void k_ba_setcost(void* ws, BaDims dm, int first) {
  const BaWin v = view(ws, dm, blockIdx.x);
  BaState* S = v.st;
  if (threadIdx.x != 0 || !S->active) return;
  const int nc = (S->L + kBlock - 1) / kBlock;
  double c = 0;
  for (int i = 0; i < nc; ++i) c += v.cp[i];
  S->cost = 0.5 * c;
  if (first) S->cost0 = 0.5 * c;
}

// pose blocks of one frame (H_pp, g_p); the coupling blocks W are recomputed where they are
// used (k_ba_lin, k_ba_upd) instead of crossing HBM
__global__ __launch_bounds__(kBlock) void k_ba_pp(BaIn in, void* ws, BaDims dm, BaCam cam) {
  const BaWin v = view(ws, dm, blockIdx.x);
  BaState* S = v.st;
  const int f = blockIdx.y + 1;
  if (!S->active || f >= S->n) return;
  const double* X = cur_X(v, S);
  const double* T = S->T[f];
  double h[27];
  for (int i = 0; i < 27; ++i) h[i] = 0;
  const int b0 = v.hdr[8 + f], b1 = v.hdr[8 + f + 1];
  for (int ii = b0 + threadIdx.x; ii < b1; ii += kBlock) {
    const int oi = v.flist[ii];
    const BaObs o = v.obs[oi];
    double r[3], w, rho, Jp[3][6];
    ba_eval<true, true, false>(T, X + 3 * o.lm, o, cam, obs_is2(in, o), r, w, rho, Jp, nullptr);
    int q = 0;
    for (int a = 0; a < 6; ++a) {
      for (int bb = a; bb < 6; ++bb) h[q++] += w * (Jp[0][a] * Jp[0][bb] + Jp[1][a] * Jp[1][bb] + Jp[2][a] * Jp[2][bb]);
      h[21 + a] += w * (Jp[0][a] * r[0] + Jp[1][a] * r[1] + Jp[2][a] * r[2]);
    }
  }
  // the 27 block sums at once (same order as block_sum: wave sums, then the waves in order)
  __shared__ double s_part[kBlock / 64][27];
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const double wv = wave_sum(h[i]);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6][i] = wv;
  }
  __syncthreads();
  if (threadIdx.x < 27) {
    double t = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) t += s_part[k][threadIdx.x];
    S->Hpp[f][threadIdx.x] = t;
  }
}

// landmark blocks of a window's chunks + their share of the reduced camera system on MFMA
// (tile k of the enumeration I <= J over the pose rows and the z column goes to wave k mod kLinWaves)
__device__ __forceinline__ void lin_tile(int k, int ntu, int NT, int& I, int& J) {
  int idx = 0;
  for (int i = 0; i < ntu; ++i)
    for (int j = i; j < NT; ++j) {
      if (j >= ntu && j != NT - 1) continue;
      if (idx++ == k) { I = i; J = j; return; }
    }
  I = J = -1;
}

// Per chunk of LPC landmarks: (1) a group of GL = kLinBlock / LPC lanes per landmark, lane j =
// the landmark's j-th observation (at most one per frame): residual, weight, J_p and J_l from
// the poses staged in LDS, W = J_p^T w J_l in registers (never stored), w J_l^T J_l and
// w J_l^T r summed over the group (xor butterfly), the damped 3x3 Cholesky (redundantly per
// lane), z = L^-1 g and the rows Y = W L^-T; the group writes its landmark's three rows of Yt
// whole (zeros in the columns of frames it is not seen in), so the buffer needs no clearing
// pass, and one word of which 16-column tiles those rows touch.  (2) G += Yt^T Yt on MFMA.
// The next chunk's landmark starts / observation / position are loaded during this chunk
// (starts before its arithmetic, the observation record before its MFMA phase), so its
// arithmetic starts from registers.
// r6: each chunk in two halves of LPC / 2 landmarks, (1) by the producer waves into one half of a
// double-buffered Y while the consumer waves run (2) over the previous half -- the VALU phase and
// the MFMA phase overlap instead of alternating between barriers, and each tile still accumulates
// the chunk's rows in order (bit-identical to the alternating schedule).
// MAXT: 16x16 tiles per consumer wave (2 at NR = 64: 10 tiles over 8 waves; 5 at NR = 128: 36)
// Sum / OR of a value over an aligned group of GL lanes (2 <= GL <= 32, a power of two), every
// lane receiving the same result: within a DPP row by quad permutes (xor 1, xor 2), the half-row
// mirror and the row mirror (each pairs lanes whose partial sums are equal, so both ends of a
// pair add the same two values: bit-identical results in every lane), across the two rows of
// 32 lanes by one ds_swizzle (xor 16) -- no LDS round trips for the first four steps.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}
__device__ __forceinline__ double swz16_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)u, 0x401F);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(u >> 32), 0x401F);
  return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}
template <int GL>
__device__ __forceinline__ double group_sum(double v) {
  static_assert(GL >= 2 && GL <= 32 && (GL & (GL - 1)) == 0, "group of 2..32 lanes");
  v += dpp_f64<0xB1>(v);                         // quad_perm [1,0,3,2]
  if constexpr (GL >= 4) v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (GL >= 8) v += dpp_f64<0x141>(v);  // row_half_mirror
  if constexpr (GL >= 16) v += dpp_f64<0x140>(v); // row_mirror
  if constexpr (GL >= 32) v += swz16_f64(v);      // xor 16
  return v;
}
template <int GL, int N>
__device__ __forceinline__ void group_sum_or(double (&v)[N], uint32_t& fm) {
  // one value at a time through all its steps (few live temporaries: the kernel is at its
  // register budget)
#pragma unroll
  for (int q = 0; q < N; ++q) v[q] = group_sum<GL>(v[q]);
  fm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fm, 0xB1, 0xF, 0xF, false);
  if constexpr (GL >= 4) fm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fm, 0x4E, 0xF, 0xF, false);
  if constexpr (GL >= 8) fm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fm, 0x141, 0xF, 0xF, false);
  if constexpr (GL >= 16) fm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fm, 0x140, 0xF, 0xF, false);
  if constexpr (GL >= 32) fm |= (uint32_t)__builtin_amdgcn_ds_swizzle((int)fm, 0x401F);
}

template <int MAXT>
__global__ __launch_bounds__(kLinBlock) void k_ba_lin(BaIn in, void* ws, BaDims dm, BaCam cam) {
  extern __shared__ double sY[];    // [2][3 LPC / 2][NR + 2]: the two half-chunk buffers
  __shared__ double sT[kKMax][12];  // the window's current poses
  __shared__ uint32_t s_tm[2][32];  // per landmark of a half chunk: bit I = its rows reach tile I's columns
  const BaWin v = view(ws, dm, blockIdx.x);
  const BaState* S = v.st;
  if (!S->active) return;
  const int L = S->L, part = blockIdx.y, LPC = dm.LPC, LPH = LPC / 2;
  if (part * LPC >= L) return;  // no chunk for this partial (k_ba_solve sums only the used ones)
  const int n = S->n;
  const int np = 6 * (n - 1);
  const int NR = dm.NR, NRP = NR + 2, rows = 3 * LPH;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int NT = NR / 16, ntu = (np + 15) / 16;  // tiles covering the pose rows
  for (int i = threadIdx.x; i < n * 12; i += kLinBlock) sT[i / 12][i % 12] = S->T[i / 12][i % 12];
  // the block's chunks c = part, part + NPART, ... (c LPC < L), each as two halves of LPH landmarks
  const int nch = ((L + LPC - 1) / LPC - part + dm.NPART - 1) / dm.NPART, nh = 2 * nch;
  auto half_l0 = [&](int h) { return (part + (h >> 1) * dm.NPART) * LPC + (h & 1) * LPH; };
  __syncthreads();  // sT
  if (wid < kLinProd) {
    // ---- producers: half chunk h into buffer h & 1 while the consumers multiply half h - 1
    const double lam = S->lam;
    const double* X = cur_X(v, S);
    const int GL = kLinBlock / LPC, t = threadIdx.x / GL, j = threadIdx.x % GL;
    // one half ahead: the landmark's observation range, its observation j, its position
    int ns0 = 0, ns1 = 0;
    BaObs onext{};
    double xn[3] = {0.0, 0.0, 0.0};
    auto fetch_start = [&](int h) {
      const int l = half_l0(h) + t;
      ns0 = ns1 = 0;
      if (h < nh && l < L) {
        ns0 = v.lstart[l];
        ns1 = v.lstart[l + 1];
        xn[0] = X[3 * l];
        xn[1] = X[3 * l + 1];
        xn[2] = X[3 * l + 2];
      }
    };
    auto fetch_obs = [&]() {
      if (j < ns1 - ns0) onext = v.obs[ns0 + j];
    };
    fetch_start(0);
    fetch_obs();
    for (int h = 0; h <= nh; ++h) {
      if (h < nh) {
        const BaObs o = onext;
        const int cnt = ns1 - ns0;
        const double xl[3] = {xn[0], xn[1], xn[2]};
        const int l = half_l0(h) + t;
        const bool live = l < L, has = live && j < cnt;
        fetch_start(h + 1);  // the next half's landmark starts / position
        // (a) lane j: observation j's landmark-block terms w Jl^T Jl (upper 6) and w Jl^T r (3), and
        // its coupling block W; (b) their sum over the group (every lane ends with the same sums),
        // the damped 3x3 Cholesky and z = L^-1 g; (c) lane j: rows 6 (f-1) .. 6 (f-1) + 5 of W L^-T
        double hg[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        BaCoupling cpl{};
        const int f = has ? (int)o.frame : 0;
        if (has) {
          double r[3], rho, Jl[3][3];
          ba_eval_lw(sT[f], xl, o, cam, obs_is2(in, o), r, rho, Jl, cpl);
          const double w = cpl.w;
          int q = 0;
          for (int a2 = 0; a2 < 3; ++a2) {
            for (int b2 = a2; b2 < 3; ++b2) hg[q++] = w * (Jl[0][a2] * Jl[0][b2] + Jl[1][a2] * Jl[1][b2] + Jl[2][a2] * Jl[2][b2]);
            hg[6 + a2] = w * (Jl[0][a2] * r[0] + Jl[1][a2] * r[1] + Jl[2][a2] * r[2]);
          }
        }
        fetch_obs();  // the next half's observation record
        uint32_t fm = has && f > 0 ? 1u << f : 0u;  // frames with pose columns that see the landmark
        if (GL == 32) group_sum_or<32>(hg, fm);
        else if (GL == 16) group_sum_or<16>(hg, fm);
        else
          for (int m = GL >> 1; m >= 1; m >>= 1) {
#pragma unroll
            for (int q = 0; q < 9; ++q) hg[q] += __shfl_xor(hg[q], m, 64);
            fm |= (uint32_t)__shfl_xor((int)fm, m, 64);
          }
        const double* H = hg;
        const double a00 = H[0] + lam * H[0] + 1e-6, a11 = H[3] + lam * H[3] + 1e-6, a22 = H[5] + lam * H[5] + 1e-6;
        const double i00 = rsq_r(a00), l00 = a00 * i00;
        const double l10 = H[1] * i00, l20 = H[2] * i00;
        const double d11 = a11 - l10 * l10, i11 = rsq_r(d11), l11 = d11 * i11;
        const double l21 = (H[4] - l20 * l10) * i11;
        const double d22 = a22 - l20 * l20 - l21 * l21, i22 = rsq_r(d22), l22 = d22 * i22;
        double* Y0 = sY + (h & 1) * rows * NRP + 3 * t * NRP;
        if (j == 0) {
          double z0 = 0.0, z1 = 0.0, z2 = 0.0;
          if (live) {
            double* Lf = v.Lf + 6 * l;
            Lf[0] = l00; Lf[1] = l10; Lf[2] = l11; Lf[3] = l20; Lf[4] = l21; Lf[5] = l22;
            v.gl[3 * l] = H[6]; v.gl[3 * l + 1] = H[7]; v.gl[3 * l + 2] = H[8];
            z0 = H[6] * i00;
            z1 = (H[7] - l10 * z0) * i11;
            z2 = (H[8] - l20 * z0 - l21 * z1) * i22;
          }
          Y0[NR - 1] = z0;
          Y0[NRP + NR - 1] = z1;
          Y0[2 * NRP + NR - 1] = z2;
          uint32_t tm = 0;
          for (uint32_t mm = fm; mm; mm &= mm - 1) {
            const int ff = __builtin_ctz(mm);
            tm |= (1u << (6 * (ff - 1) / 16)) | (1u << ((6 * (ff - 1) + 5) / 16));
          }
          s_tm[h & 1][t] = tm;
        }
        if (f > 0) {
          for (int pp = 0; pp < 6; ++pp) {
            double wr[3];
            ba_wrow(cpl, pp, wr);
            const double y0 = wr[0] * i00;
            const double y1 = (wr[1] - l10 * y0) * i11;
            const double y2 = (wr[2] - l20 * y0 - l21 * y1) * i22;
            const int col = 6 * (f - 1) + pp;
            Y0[col] = y0;
            Y0[NRP + col] = y1;
            Y0[2 * NRP + col] = y2;
          }
        }
        // zeros: the pose column blocks of frames that do not see the landmark, and the padding
        // columns np .. NR-2 (column NR-1 is z)
        for (int fb = 1 + j; fb < n; fb += GL)
          if (!((fm >> fb) & 1u))
            for (int pp = 0; pp < 6; ++pp) {
              const int col = 6 * (fb - 1) + pp;
              Y0[col] = 0.0;
              Y0[NRP + col] = 0.0;
              Y0[2 * NRP + col] = 0.0;
            }
        for (int col = np + j; col < NR - 1; col += GL) {
          Y0[col] = 0.0;
          Y0[NRP + col] = 0.0;
          Y0[2 * NRP + col] = 0.0;
        }
      }
      __syncthreads();  // half h complete / half h - 1 consumed
    }
    return;
  }
  // ---- consumers: G += Yt^T Yt of half h - 1 on MFMA while the producers fill half h.
  // Tile k of the enumeration goes to consumer wave k mod kLinCons.  A[i][k] = Yt[k][16I + i],
  // B[k][j] = Yt[k][16J + j], lane holds k = lane >> 4.  A 4-row step g (rows 4g .. 4g+3:
  // landmarks 4g/3 and (4g+3)/3) of tile (I, J) is skipped when those rows are zero in tile I's
  // or J's columns (the z column tile NT-1 always counts); each tile's steps ascend into its own
  // accumulator -- half 0's steps then half 1's, i.e. the chunk's rows in order -- and the
  // operands are loaded two active steps ahead of the MFMA that uses them.  (Walking the union of
  // the wave's tiles' steps with every active tile issued back to back -- independent
  // accumulators in flight -- measured slower: 1080p BA 5.0 -> 6.8 ms, 600p 1.87 -> 2.21 ms, the
  // operand arrays spilling at 128 VGPRs.)
  const int wc = wid - kLinProd;
  int ntiles = 0;
  for (int i = 0; i < ntu; ++i) ntiles += (ntu - i) + (ntu < NT ? 1 : 0);
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 acc[MAXT];
  int tI[MAXT], tJ[MAXT];
#pragma unroll
  for (int lt = 0; lt < MAXT; ++lt) {
    acc[lt] = d4{0.0, 0.0, 0.0, 0.0};
    const int k = kLinCons * lt + wc;
    tI[lt] = tJ[lt] = -1;
    if (k < ntiles) lin_tile(k, ntu, NT, tI[lt], tJ[lt]);
  }
  for (int h = 0; h <= nh; ++h) {
    if (h > 0) {
      const int hb = (h - 1) & 1;
      const double* Yb = sY + hb * rows * NRP;
      const uint32_t actl = lane < rows / 4 ? (s_tm[hb][(4 * lane) / 3] | s_tm[hb][(4 * lane + 3) / 3]) : 0u;
#pragma unroll
      for (int lt = 0; lt < MAXT; ++lt) {
        const int I = tI[lt], J = tJ[lt];
        if (I < 0) continue;
        const double* ya = Yb + (lane >> 4) * NRP + 16 * I + (lane & 15);
        const double* yb = Yb + (lane >> 4) * NRP + 16 * J + (lane & 15);
        uint64_t m = __ballot(((actl >> I) & 1u) && (((actl >> J) & 1u) || J == NT - 1));
        if (!m) continue;
        int g = __builtin_ctzll(m);
        m &= m - 1;
        double a0 = ya[4 * g * NRP], b0 = yb[4 * g * NRP];
        bool h1 = m != 0;
        if (h1) {
          g = __builtin_ctzll(m);
          m &= m - 1;
        }
        double a1 = ya[4 * g * NRP], b1 = yb[4 * g * NRP];
        while (h1) {
          const bool h2 = m != 0;
          if (h2) {
            g = __builtin_ctzll(m);
            m &= m - 1;
          }
          const double a2 = ya[4 * g * NRP], b2 = yb[4 * g * NRP];
          acc[lt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[lt], 0, 0, 0);
          a0 = a1, b0 = b1, a1 = a2, b1 = b2, h1 = h2;
        }
        acc[lt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[lt], 0, 0, 0);
      }
    }
    __syncthreads();  // half h complete / half h - 1 consumed
  }
  // f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
  double* Gc = v.Gp + (int64_t)part * NR * NR;
#pragma unroll
  for (int lt = 0; lt < MAXT; ++lt) {
    const int I = tI[lt], J = tJ[lt];
    if (I >= 0)
      for (int i = 0; i < 4; ++i) Gc[(16 * I + (lane >> 4) + 4 * i) * NR + 16 * J + (lane & 15)] = acc[lt][i];
  }
}

// With more than one k_ba_lin partial their sum is formed by the whole GPU first (k_ba_gsum,
// into partial 0, the order k_ba_solve's own sum had), so the one block per window that
// assembles S reads one partial instead of NPART.  r6: for every NPART >= 2 (r4/r5: >= 8, the
// 1080p case; at 600p the solve summed 4 partials itself -- its assembly took ~0.4 of the 1.65 ms
// BA, measured by a no-assembly ablation)
constexpr int kGsumParts = 2;
__global__ __launch_bounds__(256) void k_ba_gsum(void* ws, BaDims dm) {
  const BaWin v = view(ws, dm, blockIdx.x);
  const BaState* S = v.st;
  if (!S->active) return;
  const int nch0 = (S->L + dm.LPC - 1) / dm.LPC, nch = nch0 < dm.NPART ? nch0 : dm.NPART;
  const int64_t NN = (int64_t)dm.NR * dm.NR;
  const int64_t i2 = (int64_t)blockIdx.y * 256 + threadIdx.x;  // 2 consecutive doubles
  if (2 * i2 >= NN) return;
  typedef double d2 __attribute__((ext_vector_type(2)));
  d2* g = reinterpret_cast<d2*>(v.Gp) + i2;
  d2 part[kLinParts];
#pragma unroll
  for (int c = 0; c < kLinParts; ++c)
    if (c < nch) part[c] = g[c * (NN / 2)];
  d2 gs = {0.0, 0.0};
#pragma unroll
  for (int c = 0; c < kLinParts; ++c)
    if (c < nch) gs += part[c];
  g[0] = gs;
}

// reduced camera system, Cholesky, pose step and tentative poses; 512 threads per window.
// The system S (np x np, np = 6 (n-1) <= 120) lives in LDS padded to NP = 16 ceil(np / 16)
// (identity in the padding) with row stride NP + 2 (== 2 mod 32 doubles: the 16 rows x 2
// columns of a wave half's 16x16x4 MFMA operand fetch hit 32 distinct bank pairs).  Factor:
// right-looking Cholesky by 16-column panels, three phases per panel —
//   (A) the diagonal 16x16 tile by wave 0 in registers (lane = row i; pivots as rsq + one
//       Newton step; r6: the pivot and the column entries by v_readlane, no LDS round trip),
//   (B) the panel below it, one thread per row (16-step substitution against the tile),
//   (C) the trailing update S_IJ -= L_Ip L_Jp^T of every lower tile on
//       v_mfma_f64_16x16x4_f64 (4 K-steps per panel), tiles spread over the waves; r6: with
//       look-ahead -- wave 0 updates the next diagonal tile and factors it (A of the next
//       panel) while waves 1..7 update the rest —
// two barriers per panel (r5: three; r3: two per 4 columns); the update, the bulk of the
// arithmetic, leaves the LDS-bound scalar loop for the matrix pipe.
constexpr int kSolveBlock = 512, kSolveWaves = kSolveBlock / 64;
__host__ __device__ constexpr int ba_np16(int np) { return (np + 15) & ~15; }
__host__ __device__ constexpr int ba_sstride(int np16) { return np16 + 2; }
__global__ __launch_bounds__(kSolveBlock) void k_ba_solve(void* ws, BaDims dm) {
  extern __shared__ double sS[];  // [NP][NP + 2] S then L (lower), rhs[NP], rinv[NP], linvT[NP / 16][16][16]
  __shared__ int s_fail;
  const BaWin v = view(ws, dm, blockIdx.x);
  BaState* S = v.st;
  if (!S->active) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = S->n, L = S->L, NR = dm.NR;
  const int np = 6 * (n - 1), NP = ba_np16(np), STR = ba_sstride(NP), NTl = NP / 16;
  const int nch0 = (L + dm.LPC - 1) / dm.LPC;
  const int nch = dm.NPART >= kGsumParts ? 1 : (nch0 < dm.NPART ? nch0 : dm.NPART);  // partials to sum (k_ba_gsum)
  const double lam = S->lam;
  double* rhs = sS + NP * STR;
  double* rinv = rhs + NP;  // reciprocal pivots of the factor
  constexpr int LS = 17;      // row stride of linvT (16 + 1: a column of stores hits 16 bank pairs)
  double* linvT = rinv + NP;  // per panel p: row j = column j of L_pp^-1 (the blocked solves below)
  double* dcol = linvT + 17 * NP;  // [16]: the diagonal tile's current column of L (factor_diag)
  if (tid == 0) s_fail = 0;
  // the right-hand side's global reads first (issued beside the assembly's below; r6: they
  // were a second round trip after its LDS stores)
  double rhs_v = 0.0;
  if (tid < np) {
    double gs = 0.0;
    const double* gp = v.Gp + tid * NR + NR - 1;
    for (int c = 0; c < nch; ++c) gs += gp[(int64_t)c * NR * NR];
    rhs_v = -S->Hpp[tid / 6 + 1][21 + tid % 6] + gs;
  }
  // padding: identity rows / columns past np (r6: only those entries, not a pass over NP x NP)
  const int pad = NP - np;
  for (int t = tid; t < pad * NP; t += kSolveBlock) {
    const int a = np + t / NP, b = t % NP;
    sS[a * STR + b] = a == b ? 1.0 : 0.0;
  }
  for (int t = tid; t < np * pad; t += kSolveBlock) sS[(t / pad) * STR + np + t % pad] = 0.0;
  // S = H_pp + lam diag + 1e-6 I - sum_c G_c (upper triangle, mirrored), G summed by
  // k_ba_gsum (nch == 1 whenever NPART > 1).  A thread takes 4 consecutive columns b0..b0+3 of
  // a row a (b0 from the row's diagonal 16 x 16 tile, which k_ba_lin writes in full).  r6: all of
  // a thread's global reads (its <= kAsmIt slices of G and the H_pp entries they need) are
  // issued before any LDS write -- the reads go through generic pointers, so the compiler kept
  // each iteration's read behind the previous iteration's LDS stores (one global latency per
  // iteration, ~0.8 ms of the 1080p BA by a no-assembly ablation)
  typedef double d4 __attribute__((ext_vector_type(4)));
  const int nq = (np + 3) / 4;  // column quads per row
  constexpr int kAsmIt = 8;     // ceil(np nq / kSolveBlock) <= 7 for np <= 120
  d4 gq[kAsmIt];
  double hq[kAsmIt][4];
#pragma unroll
  for (int k = 0; k < kAsmIt; ++k) {
    const int t = tid + k * kSolveBlock;
    const int a = t / nq, b0 = 4 * (t - a * nq);
    gq[k] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < 4; ++u) hq[k][u] = 0.0;
    if (t >= np * nq || b0 + 3 < a) continue;
    const d4* gp = reinterpret_cast<const d4*>(v.Gp + a * NR + b0);
    d4 gs = {0.0, 0.0, 0.0, 0.0};
    for (int c = 0; c < nch; ++c) gs += gp[(int64_t)c * NR * NR / 4];  // nch == 1 but for NPART == 1
    gq[k] = gs;
    const int fa = a / 6 + 1, ia = a - 6 * (fa - 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int bb = b0 + u;
      if (bb < a || bb >= np || bb / 6 + 1 != fa) continue;
      const int j = bb - 6 * (fa - 1);
      hq[k][u] = S->Hpp[fa][ia * 6 - ia * (ia - 1) / 2 + (j - ia)];
    }
  }
#pragma unroll
  for (int k = 0; k < kAsmIt; ++k) {
    const int t = tid + k * kSolveBlock;
    const int a = t / nq, b0 = 4 * (t - a * nq);
    if (t >= np * nq || b0 + 3 < a) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int bb = b0 + u;
      if (bb < a || bb >= np) continue;
      double hv = hq[k][u];
      if (bb == a) hv += lam * hv + 1e-6;
      sS[a * STR + bb] = hv - gq[k][u];
      sS[bb * STR + a] = hv - gq[k][u];
    }
  }
  static_assert(kSolveBlock >= 128, "one thread per row of the reduced system (np <= 120)");
  if (tid < NP) rhs[tid] = rhs_v;
  __syncthreads();
  typedef double d4 __attribute__((ext_vector_type(4)));
  // (A) the diagonal tile of panel p on wave 0: lane i (< 16; lanes 16..63 mirror row i & 15)
  // holds row i of the tile in registers; the pivot and every L[j][c] an update needs are
  // wave-uniform reads (v_readlane) of the lane that owns them, so the column chain has no LDS
  // round trip (r5: three ds_bpermute per column).  Pivots as rsq + one Newton step.
  auto factor_diag = [&](int p) {
    const int c0 = 16 * p, i = lane & 15;
    double r[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) r[q] = sS[(c0 + i) * STR + c0 + q];
    bool bad = false;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const double piv = rl_f64(r[c], c);
      bad |= !(piv > 0.0);
      const double rp = rsq_r(piv);
      const double lic = r[c] * rp;  // L[i][c] (the diagonal piv rp on row c)
      // r6: every entry updated (one FMA, no select): a lane's entries right of its diagonal
      // become garbage that nothing reads (pivots and multipliers come from lanes at or below
      // their column) and are zeroed as each column completes.  The next column's multiplier
      // (the chain to the next pivot) by v_readlane; the rest of the column through LDS (one
      // store, broadcast reads: ~8 instead of ~28 readlanes), needed a column or more later.
      if (lane < 16) dcol[lane] = lic;
      if (c + 1 < 16) r[c + 1] = fma(-lic, rl_f64(lic, c + 1), r[c + 1]);
#pragma unroll
      for (int j = c + 2; j < 16; ++j) r[j] = fma(-lic, dcol[j], r[j]);
      r[c] = i >= c ? lic : 0.0;
      if (lane == 0) rinv[c0 + c] = rp;
    }
    if (lane < 16) {
#pragma unroll
      for (int q = 0; q < 16; ++q) sS[(c0 + i) * STR + c0 + q] = r[q];
    }
    if (bad && lane == 0) s_fail = 1;
  };
  // S_IJ -= L_Ip L_Jp^T of one lower tile on MFMA (A[i][k] = L[16I + i][c0 + k], B[k][j] =
  // L[16J + j][c0 + k]), 4 K-steps
  auto tile_upd = [&](int c0, int I, int J) {
    const double* pa = sS + (16 * I + (lane & 15)) * STR + c0 + (lane >> 4);
    const double* pb = sS + (16 * J + (lane & 15)) * STR + c0 + (lane >> 4);
    const double a0 = pa[0], a1 = pa[4], a2 = pa[8], a3 = pa[12];
    const double b0 = pb[0], b1 = pb[4], b2 = pb[8], b3 = pb[12];
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, b2, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a3, b3, acc, 0, 0, 0);
    double* pc = sS + (16 * I + (lane >> 4)) * STR + 16 * J + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) pc[4 * r * STR] -= acc[r];
  };
  auto panel_subst = [&](double (&x)[16], int c0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      x[c] *= rinv[c0 + c];
#pragma unroll
      for (int c2 = c + 1; c2 < 16; ++c2) x[c2] = fma(-x[c], sS[(c0 + c2) * STR + c0 + c], x[c2]);
    }
  };
  if (wid == 0) factor_diag(0);
  __syncthreads();
  for (int p = 0; p < NTl; ++p) {
    if (s_fail) break;  // uniform: read after the barrier that follows the tile's factorisation
    const int c0 = 16 * p;
    // (B) the panel's rows below the tile: L_Ip = S_Ip L_pp^-T, one thread per row
    const int nb = NP - c0 - 16;
    // r6: right-looking substitution (x[c] final, then its term leaves every later entry at
    // once: a chain of 16 multiply + FMA steps instead of the 136-deep dot products of the
    // row-by-row substitution); the tile's column c is a uniform (broadcast) read.  The same
    // substitution on the unit vectors e_j gives the columns of L_pp^-1 for the blocked solves
    // below -- run by the last wave during (C) (it has the fewest tiles), for the last panel here.
    const bool unit = p == NTl - 1 && tid < 16;
    if (tid < nb || unit) {
      double* row = unit ? linvT + (p * 16 + tid) * LS : sS + (c0 + 16 + tid) * STR + c0;
      double x[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) x[c] = unit ? (c == tid ? 1.0 : 0.0) : row[c];
      panel_subst(x, c0);
#pragma unroll
      for (int c = 0; c < 16; ++c) row[c] = x[c];
    }
    __syncthreads();
    // (C) trailing update of the lower tiles (I, J), p < J <= I < NTl, with look-ahead: wave 0
    // updates the next diagonal tile (p + 1, p + 1) and factors it at once (A of panel p + 1)
    // while waves 1..7 update every other tile -- two barriers per panel instead of three, and
    // the next tile's serial factorisation overlaps this panel's update (r6; each element still
    // gets the same updates in the same panel order: bit-identical)
    const int m = NTl - p - 1;
    if (m > 0) {
      if (wid == 0) {
        tile_upd(c0, p + 1, p + 1);
        factor_diag(p + 1);
      } else {
        for (int t = wid; t < m * (m + 1) / 2; t += kSolveWaves - 1) {
          int I = p + 1, rem = t;
          while (rem >= I - p) {
            rem -= I - p;
            ++I;
          }
          tile_upd(c0, I, p + 1 + rem);
        }
        if (wid == kSolveWaves - 1 && lane < 16) {  // the columns of L_pp^-1 (above)
          double x[16];
#pragma unroll
          for (int c = 0; c < 16; ++c) x[c] = c == lane ? 1.0 : 0.0;
          panel_subst(x, c0);
          double* row = linvT + (p * 16 + lane) * LS;
#pragma unroll
          for (int c = 0; c < 16; ++c) row[c] = x[c];
        }
      }
    }
    __syncthreads();
  }
  if (s_fail) {
    if (tid == 0) S->fail = 1;
    return;
  }
  if (wid == 0) {
    // L y = rhs, then L^T x = y, blocked by the 16-row panels on wave 0 (r6; r5 walked the rows
    // one dependent step each, 2 x 114 steps of readlane + multiply + FMA at 1080p, ~18 us): a
    // quad of lanes per row of the panel, lane q of the quad summing every 4th term.
    //   forward, panel p:  r = b_p - L_p,<p y_<p (left-looking), y_p = L_pp^-1 r
    //   backward, panel p: t = y_p - L_>p,p^T x_>p,              x_p = L_pp^-T t
    // the panel's intermediate vector crosses the quads through rhs (one wave: its LDS accesses
    // complete in order once waited for).
    const int i = lane >> 2, q = lane & 3;
    auto quad_sum = [](double v) {
      v += dpp_f64<0xB1>(v);  // quad_perm [1,0,3,2]
      v += dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
      return v;
    };
    auto lds_done = []() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    // (four partial sums per lane, so the loads of a panel's terms are issued together)
    for (int p = 0; p < NTl; ++p) {
      const int c0 = 16 * p;
      const double* Lr = sS + (c0 + i) * STR;
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int k0 = q; k0 < c0; k0 += 16)
#pragma unroll
        for (int u = 0; u < 4; ++u) a4[u] = fma(Lr[k0 + 4 * u], rhs[k0 + 4 * u], a4[u]);
      const double acc = quad_sum((a4[0] + a4[1]) + (a4[2] + a4[3]));
      const double r = rhs[c0 + i] - acc;
      lds_done();
      if (q == 0) rhs[c0 + i] = r;
      lds_done();
      const double* Li = linvT + p * 16 * LS;
      double y = 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u) y = fma(Li[(4 * q + u) * LS + i], rhs[c0 + 4 * q + u], y);
      y = quad_sum(y);
      lds_done();
      if (q == 0) rhs[c0 + i] = y;
      lds_done();
    }
    for (int p = NTl - 1; p >= 0; --p) {
      const int c0 = 16 * p;
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int k0 = c0 + 16 + q; k0 < NP; k0 += 16)
#pragma unroll
        for (int u = 0; u < 4; ++u) a4[u] = fma(sS[(k0 + 4 * u) * STR + c0 + i], rhs[k0 + 4 * u], a4[u]);
      const double acc = quad_sum((a4[0] + a4[1]) + (a4[2] + a4[3]));
      const double t = rhs[c0 + i] - acc;
      lds_done();
      if (q == 0) rhs[c0 + i] = t;
      lds_done();
      const double* Li = linvT + (p * 16 + i) * LS;
      double x = 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u) x = fma(Li[4 * q + u], rhs[c0 + 4 * q + u], x);
      x = quad_sum(x);
      lds_done();
      if (q == 0) rhs[c0 + i] = x;
      lds_done();
    }
  }
  __syncthreads();
  for (int a = tid; a < 6 * n; a += kSolveBlock) S->dp[a] = a < 6 ? 0.0 : rhs[a - 6];
  if (tid < n) {
    const int f = tid;
    double* Tt = S->Tt[f];
    const double* T = S->T[f];
    if (f == 0) {
      for (int i = 0; i < 12; ++i) Tt[i] = T[i];
    } else {
      double Rw[9];
      const double* d = rhs + 6 * (f - 1);
      exp_so3(d, Rw);
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Tt[3 * i + j] = Rw[3 * i] * T[j] + Rw[3 * i + 1] * T[3 + j] + Rw[3 * i + 2] * T[6 + j];
        Tt[9 + i] = Rw[3 * i] * T[9] + Rw[3 * i + 1] * T[10] + Rw[3 * i + 2] * T[11] + d[3 + i];
      }
    }
  }
}

// landmark back-substitution + cost partials at the tentative point.  A group of GLU lanes per
// landmark, LPU = kBlock / GLU landmarks per block: lane j takes the landmark's observations
// j, j + GLU, ... (all of them at GLU = 1, one each at GLU >= K) and forms their W^T dp (W from
// ba_eval_lw at the linearisation point, as k_ba_lin) and, after the step, their cost at the
// tentative poses; the group sums both over its lanes (xor butterfly), the block sums the cost
// (fixed order) into one partial per block.  kUpdGluShort = 2 lanes at K <= 16 (BA 600p / K = 10
// 1.80 -> 1.75 ms against 1 lane, 4: 1.76 ms), kUpdGluLong = 8 at K > 16 (up to 3 observations
// each of a 20-frame track; BA 1080p / K = 20 4.53 -> 4.27 ms against 32 lanes, which sat mostly
// idle on tracks of a few observations; 16: 4.43, 4: 4.26 ms).
// r6 (after the solve / k_ba_lin changes): 4 lanes at K > 16, 1080p BA 3.32-3.33 -> 3.23 ms (2 / 4
// lanes at K <= 16: 1.50-1.52 vs 1.51-1.52 ms, unchanged)
constexpr int kUpdGluShort = 2, kUpdGluLong = 4;
template <int GLU>
__global__ __launch_bounds__(kBlock) void k_ba_upd(BaIn in, void* ws, BaDims dm, BaCam cam) {
  constexpr int LPU = kBlock / GLU;
  __shared__ double s_red[kBlock / 64];
  __shared__ double sT[kKMax][12], sTt[kKMax][12], sdp[kKMax][6];
  const BaWin v = view(ws, dm, blockIdx.x);
  const BaState* S = v.st;
  if (!S->active || S->fail) return;
  const int L = S->L, c = blockIdx.y;
  if (c * LPU >= L) return;
  const int n = S->n;
  for (int i = threadIdx.x; i < n * 12; i += kBlock) {
    sT[i / 12][i % 12] = S->T[i / 12][i % 12];
    sTt[i / 12][i % 12] = S->Tt[i / 12][i % 12];
  }
  for (int i = threadIdx.x; i < n * 6; i += kBlock) sdp[i / 6][i % 6] = S->dp[i];
  const double* X = cur_X(v, S);
  double* Xn = new_X(v, S);
  const int t = threadIdx.x / GLU, j = threadIdx.x % GLU, l = c * LPU + t;
  const bool live = l < L;
  int o0 = 0, o1 = 0;
  double Xc[3] = {0.0, 0.0, 0.0};
  if (live) {
    o0 = v.lstart[l];
    o1 = v.lstart[l + 1];
    Xc[0] = X[3 * l];
    Xc[1] = X[3 * l + 1];
    Xc[2] = X[3 * l + 2];
  }
  __syncthreads();  // staged poses
  double wd[3] = {0.0, 0.0, 0.0};  // sum of W^T dp over this lane's observations
  for (int oi = o0 + j; oi < o1; oi += GLU) {
    const BaObs o = v.obs[oi];
    if (o.frame == 0) continue;
    double r[3], rho, Jl[3][3];
    BaCoupling cpl;
    ba_eval_lw(sT[o.frame], Xc, o, cam, obs_is2(in, o), r, rho, Jl, cpl);
    const double* dp = sdp[o.frame];
    double ow[3] = {0.0, 0.0, 0.0};
    for (int a = 0; a < 6; ++a) {
      double wr[3];
      ba_wrow(cpl, a, wr);
      for (int k = 0; k < 3; ++k) ow[k] += wr[k] * dp[a];
    }
    for (int k = 0; k < 3; ++k) wd[k] += ow[k];
  }
  for (int m = GLU >> 1; m >= 1; m >>= 1)
    for (int k = 0; k < 3; ++k) wd[k] += __shfl_xor(wd[k], m, 64);
  double rho = 0.0;
  if (live) {
    const double b0 = -v.gl[3 * l] - wd[0], b1 = -v.gl[3 * l + 1] - wd[1], b2 = -v.gl[3 * l + 2] - wd[2];
    const double* Lf = v.Lf + 6 * l;
    const double y0 = b0 / Lf[0], y1 = (b1 - Lf[1] * y0) / Lf[2], y2 = (b2 - Lf[3] * y0 - Lf[4] * y1) / Lf[5];
    const double x2 = y2 / Lf[5], x1 = (y1 - Lf[4] * x2) / Lf[2], x0 = (y0 - Lf[1] * x1 - Lf[3] * x2) / Lf[0];
    const double Xl[3] = {Xc[0] + x0, Xc[1] + x1, Xc[2] + x2};
    if (j == 0) {
      Xn[3 * l] = Xl[0];
      Xn[3 * l + 1] = Xl[1];
      Xn[3 * l + 2] = Xl[2];
    }
    for (int oi = o0 + j; oi < o1; oi += GLU) {
      const BaObs o = v.obs[oi];
      double r[3], w, ro;
      ba_eval<false>(sTt[o.frame], Xl, o, cam, obs_is2(in, o), r, w, ro, nullptr, nullptr);
      rho += ro;
    }
  }
  for (int m = GLU >> 1; m >= 1; m >>= 1) rho += __shfl_xor(rho, m, 64);
  const double tot = block_sum(j == 0 ? rho : 0.0, s_red);
  if (threadIdx.x == 0) v.cp[c] = tot;
}

// LM accept / reject from k_ba_upd's cost partials (LPU landmarks each): one wave sums them,
// lane i the partials i, i + 64, ... in order, then a fixed xor tree
__global__ __launch_bounds__(64) void k_ba_accept(void* ws, BaDims dm) {
  const BaWin v = view(ws, dm, blockIdx.x);
  BaState* S = v.st;
  if (!S->active) return;
  const int n = S->n;
  __shared__ int s_acc;
  __shared__ double s_sum;
  {
    const int nc = (S->L + dm.LPU - 1) / dm.LPU;
    double part = 0.0;
    if (!S->fail)
      for (int i = threadIdx.x; i < nc; i += 64) part += v.cp[i];
    part = wave_sum(part);
    if (threadIdx.x == 0) s_sum = 0.5 * part;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s_acc = 0;
    if (S->fail) {
      S->lam = fmin(S->lam * 10.0, 1e7);
      S->fail = 0;
    } else {
      double c = s_sum;
      if (c < S->cost) {
        S->cost = c;
        S->lam = fmax(S->lam / 10.0, 1e-7);
        S->parity ^= 1;
        S->acc += 1;
        s_acc = 1;
      } else {
        S->lam = fmin(S->lam * 10.0, 1e7);
      }
    }
  }
  __syncthreads();
  if (s_acc)
    for (int i = threadIdx.x; i < n * 12; i += blockDim.x) S->T[i / 12][i % 12] = S->Tt[i / 12][i % 12];
}

// refined relative transform of the last pair: T_{n-1} T_{n-2}^-1, and statistics
__global__ void k_ba_final(const double* __restrict__ Trel, void* ws, BaDims dm, int first_end,
                           double* __restrict__ Tout_all, double* __restrict__ stats) {
  const int wi = blockIdx.x;
  const BaWin v = view(ws, dm, wi);
  const BaState* S = v.st;
  double* Tout = Tout_all + (int64_t)wi * 16;
  double* st = stats + (int64_t)wi * 6;
  if (threadIdx.x != 0) return;
  const int e = first_end + wi, n = S->n;
  if (!S->active) {
    for (int i = 0; i < 16; ++i) Tout[i] = Trel[(int64_t)(e - 1) * 16 + i];
    for (int i = 0; i < 6; ++i) st[i] = 0.0;
    st[4] = (double)n;
    return;
  }
  const double* A = S->T[n - 1];
  const double* B = S->T[n - 2];
  double Bi[12];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Bi[3 * i + j] = B[3 * j + i];
  for (int i = 0; i < 3; ++i) Bi[9 + i] = -(Bi[3 * i] * B[9] + Bi[3 * i + 1] * B[10] + Bi[3 * i + 2] * B[11]);
  double C[12];
  mat_mul_T(A, Bi, C);
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Tout[4 * i + j] = C[3 * i + j];
    Tout[4 * i + 3] = C[9 + i];
  }
  Tout[12] = Tout[13] = Tout[14] = 0.0;
  Tout[15] = 1.0;
  st[0] = S->cost0;
  st[1] = S->cost;
  st[2] = (double)S->L;
  st[3] = (double)S->O;
  st[4] = (double)n;
  st[5] = (double)S->acc;
}

// copy of one window's current landmark estimate (keyframe map export)
__global__ void k_ba_export(void* ws, BaDims dm, int wi, double* __restrict__ xyz, int32_t* __restrict__ count) {
  const BaWin v = view(ws, dm, wi);
  const BaState* S = v.st;
  const int L = S->active ? S->L : 0;
  const double* X = cur_X(v, S);
  if (blockIdx.x == 0 && threadIdx.x == 0) *count = L;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 3 * L; i += gridDim.x * blockDim.x) xyz[i] = X[i];
}

BaDims make_dims(const fvo_ctx* ctx) {
  const fvo_config& c = ctx->cfg;
  BaDims d{};
  d.Lmax = c.ba_max_landmarks;
  d.Omax = c.ba_max_obs;
  d.K = c.ba_window;
  d.cap = ctx->kp_cap;
  d.NR = 6 * (d.K - 1) < 63 ? 64 : 128;
  // landmarks per k_ba_lin chunk: LDS slice 3 LPC x (NR + 2) doubles <= 99 KB (+ the chunk's
  // observation terms); measured: halving LPC (two blocks per CU) is slower at both shapes
  d.LPC = d.NR == 64 ? kLinLPC64 : kLinLPC64 / 2;
  d.NCH = (d.Lmax + d.LPC - 1) / d.LPC;
  d.NPART = d.NCH / kLinChunksPerPart;
  d.NPART = d.NPART < 1 ? 1 : d.NPART > kLinParts ? kLinParts : d.NPART;
  if (d.NPART > d.NCH) d.NPART = d.NCH;
  d.NCU = (d.Lmax + kBlock - 1) / kBlock;
  d.LPU = kBlock / (d.K <= 16 ? kUpdGluShort : kUpdGluLong);  // k_ba_upd: landmarks per block
  d.NCUP = (d.Lmax + d.LPU - 1) / d.LPU;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    int64_t r = o;
    o += (bytes + 255) / 256 * 256;
    return r;
  };
  d.oSt = take((int64_t)sizeof(BaState));
  d.oX0 = take(8ll * 3 * d.Lmax);
  d.oX1 = take(8ll * 3 * d.Lmax);
  d.oL = take(8ll * 6 * d.Lmax);
  d.oG = take(8ll * 3 * d.Lmax);
  d.oLs = take(4ll * (d.Lmax + 1));
  d.oObs = take((int64_t)sizeof(BaObs) * d.Omax);
  d.oFl = take(4ll * d.Omax);
  d.oGp = take(8ll * d.NPART * d.NR * d.NR);
  d.oCp = take(8ll * (d.NCU > d.NCUP ? d.NCU : d.NCUP));  // cost partials (k_ba_cost / k_ba_upd)
  d.oNext = take(4ll * kKMax * d.cap);
  d.oHdr = take(4ll * (8 + kKMax + 1));
  d.oBld = take(4ll * kBldInts);
  d.win = o;
  return d;
}

// k_ba_build's dynamic LDS: the u16 match maps + tracked flags when they fit (and cap < 65535),
// else the flags alone (maps in the global workspace)
size_t build_shm(const BaDims& d) {
  const size_t maps = (size_t)2 * (d.K - 1) * d.cap + d.cap;
  return (d.cap < 0xFFFF && maps <= 156 * 1024) ? maps : (size_t)d.cap;  // + ~4 KB static <= 160 KiB
}
size_t lin_shm(const BaDims& d) { return (size_t)8 * 3 * d.LPC * (d.NR + 2); }
size_t solve_shm(int K) {
  const int np = 6 * (K - 1), NP = ba_np16(np);
  return (size_t)8 * (NP * ba_sstride(NP) + 2 * NP + 17 * NP + 16);  // S / L (padded), rhs, reciprocal pivots, L_pp^-1, a column
}

}  // namespace

int ba_init(fvo_ctx* ctx) {
  const fvo_config& c = ctx->cfg;
  if (c.ba_window < 3 || c.ba_window > kKMax) return fvo_fail(ctx, "ba_window must be in [3, 21]");
  if (c.ba_max_landmarks < 1 || c.ba_max_obs < 2) return fvo_fail(ctx, "bad BA landmark / observation caps");
  BaDims d = make_dims(ctx);
  ctx->ba_win_bytes = d.win;
  char* p = nullptr;
  int rc = fvo_alloc(ctx, &p, (size_t)d.win * c.max_batch);
  if (rc) return rc;
  ctx->ba_ws = p;
  FVO_HIP(ctx, hipStreamCreateWithFlags(&ctx->ba_s2, hipStreamNonBlocking));
  FVO_HIP(ctx, hipEventCreateWithFlags(&ctx->ba_fork, hipEventDisableTiming));
  FVO_HIP(ctx, hipEventCreateWithFlags(&ctx->ba_join, hipEventDisableTiming));
  // dynamic LDS above 64 KiB: the MFMA slice always, the reduced system for K > 11, the match maps
  if (build_shm(d) > 65536) {
    FVO_HIP(ctx, hipFuncSetAttribute((const void*)k_ba_births, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)build_shm(d)));
    FVO_HIP(ctx, hipFuncSetAttribute((const void*)k_ba_emit, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)build_shm(d)));
  }
  FVO_HIP(ctx, hipFuncSetAttribute((const void*)k_ba_lin<kLinTiles64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lin_shm(d)));
  FVO_HIP(ctx, hipFuncSetAttribute((const void*)k_ba_lin<kLinMaxTiles>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lin_shm(d)));
  if (solve_shm(c.ba_window) > 65536)
    FVO_HIP(ctx, hipFuncSetAttribute((const void*)k_ba_solve, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)solve_shm(c.ba_window)));
  return 0;
}

int ba_stereo_run(fvo_ctx* ctx, const int16_t* disp, const float* kp, const int32_t* nkp, int batch, int cap,
                  const double* K, double baseline, float* stereo, hipStream_t s) {
  const double fxB = K[0] * baseline;
  FVO_TIMED(ctx, KN_BA_STEREO, s,
            hipLaunchKernelGGL(k_ba_stereo, dim3((cap + 255) / 256, batch), dim3(256), 0, s, disp, kp, nkp,
                               ctx->cfg.width, ctx->cfg.height, cap, K[0], K[4], K[2], K[5], fxB,
                               reinterpret_cast<float4*>(stereo)));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

namespace {
// build + LM iterations + final transform of windows [w0, w0 + nw) on stream s
void ba_windows_launch(fvo_ctx* ctx, const BaIn& in, const BaCam& cam, const BaDims& d, int w0, int nw, int first_end,
                       int first_valid, int iters, double* Tout, double* stats, hipStream_t s, bool births_done) {
  void* ws = static_cast<char*>(ctx->ba_ws) + (int64_t)d.win * w0;
  const int fe = first_end + w0;
  const size_t shb = build_shm(d);
  if (shb > (size_t)d.cap) {  // the match maps fit in LDS: the parallel construction
    if (!births_done)  // (fvo_ba_count_births ran it ahead for this window range)
      hipLaunchKernelGGL(k_ba_births, dim3(nw, d.K - 1), dim3(kBirthBlock), shb, s, in, ws, d, fe, first_valid);
    hipLaunchKernelGGL(k_ba_emit, dim3(nw, d.K - 1), dim3(kBirthBlock), shb, s, in, ws, d, fe, first_valid);
    hipLaunchKernelGGL(k_ba_lists, dim3(nw, d.K), dim3(kBirthBlock), 0, s, in, ws, d, fe, first_valid);
  } else {
    hipLaunchKernelGGL(k_ba_build<false>, dim3(nw), dim3(kBuildBlock), shb, s, in, ws, d, fe, first_valid);
  }
  const dim3 gcu(nw, d.NCU), gch(nw, d.NPART), gfr(nw, d.K - 1);
  const size_t shl = lin_shm(d), shs = solve_shm(d.K);
  hipLaunchKernelGGL(k_ba_cost, gcu, dim3(kBlock), 0, s, in, ws, d, cam, 0);
  hipLaunchKernelGGL(k_ba_setcost, dim3(nw), dim3(64), 0, s, ws, d, 1);
  for (int it = 0; it < iters; ++it) {
    if (it == iters / 2 && iters >= 2) {  // outlier rejection, then the cost of the kept set
      hipLaunchKernelGGL(k_ba_cost, gcu, dim3(kBlock), 0, s, in, ws, d, cam, 1);
      hipLaunchKernelGGL(k_ba_setcost, dim3(nw), dim3(64), 0, s, ws, d, 0);
    }
    hipLaunchKernelGGL(k_ba_pp, gfr, dim3(kBlock), 0, s, in, ws, d, cam);
    if (d.NR == 64) hipLaunchKernelGGL(k_ba_lin<kLinTiles64>, gch, dim3(kLinBlock), shl, s, in, ws, d, cam);
    else hipLaunchKernelGGL(k_ba_lin<kLinMaxTiles>, gch, dim3(kLinBlock), shl, s, in, ws, d, cam);
    if (d.NPART >= kGsumParts)
      hipLaunchKernelGGL(k_ba_gsum, dim3(nw, (d.NR * d.NR / 2 + 255) / 256), dim3(256), 0, s, ws, d);
    hipLaunchKernelGGL(k_ba_solve, dim3(nw), dim3(kSolveBlock), shs, s, ws, d);
    if (d.K <= 16) hipLaunchKernelGGL(k_ba_upd<kUpdGluShort>, dim3(nw, d.NCUP), dim3(kBlock), 0, s, in, ws, d, cam);
    else hipLaunchKernelGGL(k_ba_upd<kUpdGluLong>, dim3(nw, d.NCUP), dim3(kBlock), 0, s, in, ws, d, cam);
    hipLaunchKernelGGL(k_ba_accept, dim3(nw), dim3(64), 0, s, ws, d);
  }
  hipLaunchKernelGGL(k_ba_final, dim3(nw), dim3(64), 0, s, in.Trel, ws, d, fe, Tout + 16 * (int64_t)w0,
                     stats + 6 * (int64_t)w0);
}
}  // namespace

int ba_run(fvo_ctx* ctx, const float* kp, const int32_t* nkp, const int32_t* matches, const int32_t* nmatch,
           const float* stereo, const double* Trel, int nframes, int cap, int first_end, int nwin, int first_valid,
           const double* K, double baseline, const double* inv_sigma2, int nlev, int iters, double* Tout,
           double* stats, hipStream_t s) {
  if (cap != ctx->kp_cap) return fvo_fail(ctx, "ba: cap must equal the context keypoint capacity");
  if (nwin > ctx->cfg.max_batch) return fvo_fail(ctx, "ba: n_windows exceeds max_batch");
  if (first_end < 1 || first_end + nwin > nframes) return fvo_fail(ctx, "ba: windows exceed the frame range");
  if (first_valid < 0 || first_valid >= first_end) return fvo_fail(ctx, "ba: first_valid out of range");
  if (nlev < 1 || nlev > FVO_MAX_LEVELS) return fvo_fail(ctx, "ba: bad level count");
  if (iters < 0 || iters > 100) return fvo_fail(ctx, "ba: iterations out of range");
  const BaDims d = make_dims(ctx);
  BaIn in{kp, nkp, matches, nmatch, reinterpret_cast<const float4*>(stereo), Trel, {}, nlev};
  for (int i = 0; i < nlev; ++i) in.isig2[i] = inv_sigma2[i];
  const BaCam cam{K[0], K[4], K[2], K[5], baseline};
  // the birth counts of exactly this call's window range already computed (fvo_ba_count_births)?
  const auto& pb = ctx->ba_births;
  const bool births_done = pb.valid && pb.matches == matches && pb.stereo == stereo && pb.nframes == nframes &&
                           pb.first_end == first_end && pb.nwin == nwin && pb.first_valid == first_valid;
  ctx->ba_births.valid = false;
  // The windows are independent: the batch is split in two halves whose LM sequences run on
  // two streams, so one half's latency-bound kernels (build, the per-window solve on one
  // block each) overlap the other half's whole-GPU kernels instead of leaving most CUs idle.
  const int nh = nwin >= 8 ? (nwin + 1) / 2 : nwin;
  const bool two = nh < nwin;
  if (two) {
    FVO_HIP(ctx, hipEventRecord(ctx->ba_fork, s));
    FVO_HIP(ctx, hipStreamWaitEvent(ctx->ba_s2, ctx->ba_fork, 0));
  }
  FVO_TIMED(ctx, KN_BA_SOLVE, s, {
    ba_windows_launch(ctx, in, cam, d, 0, nh, first_end, first_valid, iters, Tout, stats, s, births_done);
    if (two)
      ba_windows_launch(ctx, in, cam, d, nh, nwin - nh, first_end, first_valid, iters, Tout, stats, ctx->ba_s2,
                        births_done);
    if (two) {
      (void)hipEventRecord(ctx->ba_join, ctx->ba_s2);
      (void)hipStreamWaitEvent(s, ctx->ba_join, 0);
    }
  });
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

// k_ba_births of every window of a coming fvo_ba_windows call, ahead of it (it reads the match rows
// and the stereo points only); recorded so that call skips it
int ba_births_run(fvo_ctx* ctx, const int32_t* matches, const int32_t* nmatch, const float* stereo, int nframes,
                  int cap, int first_end, int nwin, int first_valid, hipStream_t s) {
  if (cap != ctx->kp_cap) return fvo_fail(ctx, "ba: cap must equal the context keypoint capacity");
  if (nwin > ctx->cfg.max_batch) return fvo_fail(ctx, "ba: n_windows exceeds max_batch");
  if (first_end < 1 || first_end + nwin > nframes) return fvo_fail(ctx, "ba: windows exceed the frame range");
  if (first_valid < 0 || first_valid >= first_end) return fvo_fail(ctx, "ba: first_valid out of range");
  const BaDims d = make_dims(ctx);
  const size_t shb = build_shm(d);
  if (!(shb > (size_t)d.cap)) return 0;  // serial construction: fvo_ba_windows counts in k_ba_build
  BaIn in{nullptr, nullptr, matches, nmatch, reinterpret_cast<const float4*>(stereo), nullptr, {}, 1};
  hipLaunchKernelGGL(k_ba_births, dim3(nwin, d.K - 1), dim3(kBirthBlock), shb, s, in, ctx->ba_ws, d, first_end,
                     first_valid);
  FVO_LAUNCH_CHECK(ctx);
  auto& pb = ctx->ba_births;
  pb.valid = true;
  pb.matches = matches;
  pb.stereo = stereo;
  pb.nframes = nframes;
  pb.first_end = first_end;
  pb.nwin = nwin;
  pb.first_valid = first_valid;
  return 0;
}

int ba_export_run(fvo_ctx* ctx, int window, double* xyz, int32_t* count, hipStream_t s) {
  if (window < 0 || window >= ctx->cfg.max_batch) return fvo_fail(ctx, "ba: window index out of range");
  const BaDims d = make_dims(ctx);
  hipLaunchKernelGGL(k_ba_export, dim3(32), dim3(256), 0, s, ctx->ba_ws, d, window, xyz, count);
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
