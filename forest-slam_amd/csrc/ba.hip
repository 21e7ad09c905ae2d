// Windowed local bundle adjustment for gfx950 (BASELINE.json north_star
// "extract+match+local-BA").  The reference chains PnP poses only (stereo_slam.py:306);
// this stage refines each frame's relative pose over the window of the last K frames.
// The specification — landmark construction, residuals, robust weights, LM schedule —
// is oracle/ba_ref.py; this file implements it (fp64 except the reduced-camera GEMM).
//
// k_ba_stereo  per keypoint (thread), the reference's float32 back-projection through the
//              disparity map (the fvo_backproject arithmetic) -> (X, Y, Z, d)
// k_ba_build   one block per window: match-chain landmarks (ordered births via block
//              scans), landmark-major observations, per-frame observation lists
// k_ba_solve   one block (4 waves) per window, the whole LM loop in one launch:
//   P1 per-frame pose blocks H_pp, g_p (a wave per frame, lanes over the frame's obs,
//      deterministic wave reductions) and per-observation W = J_p^T w J_l
//   P2 per-landmark H_ll, g_l, damped 3x3 Cholesky L_l; Y = W L_l^-T and z = L_l^-1 g_l
//      written as the columns 3l..3l+2 of Yt [3L][NR] (row NR-1 carries z)
//   P3 MFMA: G = Yt^T Yt (v_mfma_f64_16x16x4_f64, upper tiles, 2 accumulators), which is
//      sum_l W H_ll^-1 W^T (the Schur complement term) and its last column W H_ll^-1 g.
//      fp64, not the fp32 SURVEY.md a15 suggests: S = H_pp - G cancels, and with fp32
//      operands the refined poses moved by 1.3e-4 against the fp64 oracle (measured),
//      outside north_star's 1e-4; the f64 MFMA keeps them at ~1e-12.
//   P4 reduced camera system S = H_pp + lam diag - G, Cholesky in LDS (fp64), solve
//   P5 landmark back-substitution, pose update R <- Exp(w) R, t <- Exp(w) t + v
//   P6 cost at the tentative point (deterministic block reduction), P7 accept / reject
#include <cfloat>

#include "fvo_internal.h"

namespace {

struct BaObs {
  int lm;
  short frame, oct;   // window-relative frame, ORB octave (weight 1 / scale^(2 oct))
  float u, v, ur;     // ur NaN: mono observation
};

struct BaCam {
  double fx, fy, cx, cy, b;
};

constexpr int kKMax = 21;
constexpr int kBlock = 256;
constexpr double kD2Mono = 5.991, kD2Stereo = 7.815, kMinZ = 0.01, kLam0 = 1e-3;

struct BaDims {
  int Lmax, Omax, K, cap, NR, KP;
  int64_t oX, oXt, oL, oG, oLs, oObs, oFl, oW, oYt, oNext, oSg, oHdr, oCm, win;
};

struct BaWin {
  double *X, *Xt, *Lf, *gl, *W;
  int *lstart, *flist, *next, *hdr;
  uint32_t* cmask;  // per 4-row chunk of Yt: frames its landmarks touch (bit 31: z row)
  BaObs* obs;
  double *Yt, *Sg;
};

__device__ __forceinline__ BaWin view(void* base, const BaDims& d, int w) {
  char* p = (char*)base + d.win * w;
  BaWin v;
  v.X = (double*)(p + d.oX);
  v.Xt = (double*)(p + d.oXt);
  v.Lf = (double*)(p + d.oL);
  v.gl = (double*)(p + d.oG);
  v.lstart = (int*)(p + d.oLs);
  v.obs = (BaObs*)(p + d.oObs);
  v.flist = (int*)(p + d.oFl);
  v.W = (double*)(p + d.oW);
  v.Yt = (double*)(p + d.oYt);
  v.next = (int*)(p + d.oNext);
  v.Sg = (double*)(p + d.oSg);
  v.hdr = (int*)(p + d.oHdr);
  v.cmask = (uint32_t*)(p + d.oCm);
  return v;
}
// hdr: [0] landmarks [1] observations [2] frames n [3] first frame s [8 + f] frame list offsets

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

// deterministic block sum of doubles (fixed tree)
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

// T = [R (9, row-major) | t (3)]
__device__ __forceinline__ void mat_mul_T(const double* A, const double* B, double* C) {  // C = A * B (rigid)
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

// observation weight 1 / sigma2[octave]; 0 once the observation was rejected (oct = -1)
__device__ __forceinline__ double obs_is2(const BaIn& in, const BaObs& o) {
  return o.oct < 0 ? 0.0 : in.isig2[o.oct];
}

// residual, robust weight (x information) and cost of one observation; Jacobians if J
template <bool J>
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
  double Jc[3][3] = {{c.fx * iz, 0.0, -c.fx * x * iz * iz},
                     {0.0, c.fy * iz, -c.fy * y * iz * iz},
                     {st ? c.fx * iz : 0.0, 0.0, st ? -c.fx * (x - c.b) * iz * iz : 0.0}};
  // d(Xc)/d(w, v) = [-[Xc]x | I]
  const double sk[3][6] = {{0.0, z, -y, 1.0, 0.0, 0.0}, {-z, 0.0, x, 0.0, 1.0, 0.0}, {y, -x, 0.0, 0.0, 0.0, 1.0}};
  for (int k = 0; k < 3; ++k) {
    for (int j = 0; j < 6; ++j) Jp[k][j] = Jc[k][0] * sk[0][j] + Jc[k][1] * sk[1][j] + Jc[k][2] * sk[2][j];
    for (int j = 0; j < 3; ++j) Jl[k][j] = Jc[k][0] * T[j] + Jc[k][1] * T[3 + j] + Jc[k][2] * T[6 + j];
  }
}

// ------------------------------------------------------------------ problem construction
__global__ __launch_bounds__(kBlock) void k_ba_build(BaIn in, void* ws, BaDims dm, BaCam cam, int first_end,
                                                    int first_valid) {
  extern __shared__ uint8_t s_tracked[];  // [cap]
  __shared__ double sT[kKMax][12];
  __shared__ int s_tmp[kBlock / 64];
  __shared__ int s_L, s_O, s_stop;
  const int w = blockIdx.x, tid = threadIdx.x;
  const int e = first_end + w;
  const int s = max(first_valid, e - dm.K + 1);
  const int n = e - s + 1;
  BaWin v = view(ws, dm, w);
  const int cap = dm.cap;
  if (tid == 0) {
    v.hdr[0] = 0;
    v.hdr[1] = 0;
    v.hdr[2] = n;
    v.hdr[3] = s;
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
    for (int i = tid; i < cap; i += kBlock) v.next[k * cap + i] = -1;
  __syncthreads();
  for (int k = 0; k + 1 < n; ++k) {
    const int f = s + k, M = min(max(in.nmatch[f], 0), cap);
    const int32_t* m = in.matches + (int64_t)f * cap * 3;
    for (int r = tid; r < M; r += kBlock) v.next[k * cap + m[3 * r]] = m[3 * r + 1];
  }
  __syncthreads();
  for (int j = 0; j + 1 < n; ++j) {
    const int f = s + j;
    for (int i = tid; i < cap; i += kBlock) s_tracked[i] = 0;
    __syncthreads();
    if (j > 0) {
      const int Mp = min(max(in.nmatch[f - 1], 0), cap);
      const int32_t* mp = in.matches + (int64_t)(f - 1) * cap * 3;
      for (int r = tid; r < Mp; r += kBlock) s_tracked[mp[3 * r + 1]] = 1;
    }
    __syncthreads();
    const int M = min(max(in.nmatch[f], 0), cap);
    const int32_t* m = in.matches + (int64_t)f * cap * 3;
    // inverse of the initial pose j (world <- camera j)
    const double* Tj = sT[j];
    for (int base = 0; base < M; base += kBlock) {
      if (s_stop) break;  // uniform: written before the last barrier
      const int r = base + tid;
      bool cand = false;
      int len = 0, q = 0, t = 0;
      float4 sp = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < M) {
        q = m[3 * r];
        t = m[3 * r + 1];
        sp = in.stereo[(int64_t)f * cap + q];
        cand = !s_tracked[q] && sp.z > 0.f;
      }
      if (cand) {
        len = 2;
        int b = t;
        for (int k = j + 1; k + 1 < n; ++k) {
          const int nb = v.next[k * cap + b];
          if (nb < 0) break;
          b = nb;
          ++len;
        }
      }
      int tl, to;
      const int lid = block_scan(cand ? 1 : 0, s_tmp, &tl);
      const int oof = block_scan(len, s_tmp, &to);
      const int L0 = s_L, O0 = s_O;
      const bool ok = cand && (L0 + lid < dm.Lmax) && (O0 + oof + len <= dm.Omax);
      const int nok = __syncthreads_count(ok);
      const int nfail = __syncthreads_count(cand && !ok);
      if (ok) {
        const int id = L0 + lid;
        int o = O0 + oof;
        // X_world = R^T (Xc - t)
        const double Xc[3] = {(double)sp.x - Tj[9], (double)sp.y - Tj[10], (double)sp.z - Tj[11]};
        for (int i = 0; i < 3; ++i) v.X[3 * id + i] = Tj[i] * Xc[0] + Tj[3 + i] * Xc[1] + Tj[6 + i] * Xc[2];
        v.lstart[id] = o;
        const float* kq = in.kp + ((int64_t)f * cap + q) * FVO_KP_STRIDE;
        const int oq = min(max((int)kq[5], 0), in.nlev - 1);
        v.obs[o++] = BaObs{id, (short)j, (short)oq, kq[0], kq[1], kq[0] - sp.w};
        int b = t;
        for (int k = j + 1;; ++k) {
          const float* kb = in.kp + ((int64_t)(s + k) * cap + b) * FVO_KP_STRIDE;
          const int ob = min(max((int)kb[5], 0), in.nlev - 1);
          v.obs[o++] = BaObs{id, (short)k, (short)ob, kb[0], kb[1], __builtin_nanf("")};
          if (k + 1 >= n) break;
          const int nb = v.next[k * cap + b];
          if (nb < 0) break;
          b = nb;
        }
      }
      // totals of the ok rows (failing rows are a suffix of the candidates)
      int okl = ok ? len : 0, tot_ok;
      (void)block_scan(okl, s_tmp, &tot_ok);
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
  if (tid == 0) {
    v.hdr[0] = L;
    v.hdr[1] = O;
    v.lstart[L] = O;
  }
  // per-frame observation lists (stable, landmark-major order inside a frame)
  int fbase = 0;
  for (int f = 0; f < n; ++f) {
    if (tid == 0) v.hdr[8 + f] = fbase;
    for (int base = 0; base < O; base += kBlock) {
      const int i = base + tid;
      const bool hit = i < O && v.obs[i].frame == f;
      int tot;
      const int pos = block_scan(hit ? 1 : 0, s_tmp, &tot);
      if (hit) v.flist[fbase + pos] = i;
      fbase += tot;
    }
  }
  if (tid == 0) v.hdr[8 + n] = fbase;
}

// ------------------------------------------------------------------ LM solve
struct BaOut {
  double* Tout;
  double* stats;
};

__device__ double ba_cost(const BaWin& v, int O, const double (*T)[12], const double* X, const BaCam& cam,
                          const BaIn& in, double* s_red) {
  double acc = 0;
  for (int i = threadIdx.x; i < O; i += kBlock) {
    const BaObs o = v.obs[i];
    double r[3], w, rho;
    ba_eval<false>(T[o.frame], X + 3 * o.lm, o, cam, obs_is2(in, o), r, w, rho, nullptr, nullptr);
    acc += rho;
  }
  return 0.5 * block_sum(acc, s_red);
}

__global__ __launch_bounds__(kBlock) void k_ba_solve(BaIn in, void* ws, BaDims dm, BaCam cam, int first_end,
                                                    int iters, BaOut out) {
  extern __shared__ double sS[];  // [np*np] + rhs[np]
  __shared__ double sT[kKMax][12], sTt[kKMax][12];
  __shared__ double sH[kKMax][21], sg[kKMax][6];
  __shared__ double sdp[6 * kKMax];
  __shared__ double s_red[kBlock / 64];
  __shared__ double s_lam, s_cost, s_costn;
  __shared__ int s_fail, s_acc;
  const int wi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  BaWin v = view(ws, dm, wi);
  const int L = v.hdr[0], O = v.hdr[1], n = v.hdr[2], s = v.hdr[3];
  const int e = first_end + wi;
  double* Tout = out.Tout + (int64_t)wi * 16;
  double* st = out.stats + (int64_t)wi * 6;
  if (n < 3 || L == 0) {
    for (int i = tid; i < 16; i += kBlock) Tout[i] = in.Trel[(int64_t)(e - 1) * 16 + i];
    if (tid < 6) st[tid] = tid == 4 ? (double)n : 0.0;
    return;
  }
  const int np = 6 * (n - 1);
  const int NR = np < 63 ? 64 : 128;
  const int KP = ((3 * L + 7) / 8) * 8;
  double* rhs = sS + np * np;
  if (tid == 0) {
    for (int i = 0; i < 12; ++i) sT[0][i] = (i < 9 && i % 4 == 0) ? 1.0 : 0.0;
    for (int k = 0; k + 1 < n; ++k) {
      const double* M = in.Trel + (int64_t)(s + k) * 16;
      const double A[12] = {M[0], M[1], M[2], M[4], M[5], M[6], M[8], M[9], M[10], M[3], M[7], M[11]};
      mat_mul_T(A, sT[k], sT[k + 1]);
    }
    s_lam = kLam0;
    s_acc = 0;
  }
  // Yt is zeroed once (coalesced); every iteration rewrites only the structurally nonzero
  // entries (the 6x3 block of each observation and the z row), whose positions are fixed.
  for (int64_t i = tid; i < (int64_t)KP * NR; i += kBlock) v.Yt[i] = 0.0;
  // frame mask of every 4-row chunk of Yt, so P3 skips chunks that cannot touch a tile
  for (int c = tid; c < KP / 4; c += kBlock) {
    uint32_t m = 0;
    for (int k = 4 * c; k < 4 * c + 4 && k < 3 * L; ++k) {
      const int l = k / 3;
      m |= 1u << 31;
      for (int oi = v.lstart[l]; oi < v.lstart[l + 1]; ++oi) m |= 1u << v.obs[oi].frame;
    }
    v.cmask[c] = m;
  }
  __syncthreads();
  double* X = v.X;
  double* Xt = v.Xt;
  {
    const double c = ba_cost(v, O, sT, X, cam, in, s_red);
    if (tid == 0) {
      s_cost = c;
      st[0] = c;
    }
  }
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    if (it == iters / 2 && iters >= 2) {
      // outlier rejection at the current estimate (oracle/ba_ref.py _reject)
      for (int i = tid; i < O; i += kBlock) {
        const BaObs o = v.obs[i];
        if (o.oct < 0) continue;
        const double* T = sT[o.frame];
        const double* Xl = X + 3 * o.lm;
        const double x = T[0] * Xl[0] + T[1] * Xl[1] + T[2] * Xl[2] + T[9];
        const double y = T[3] * Xl[0] + T[4] * Xl[1] + T[5] * Xl[2] + T[10];
        const double z = T[6] * Xl[0] + T[7] * Xl[1] + T[8] * Xl[2] + T[11];
        const bool ok = z > kMinZ;
        const double iz = 1.0 / (ok ? z : 1.0);
        const bool st = !isnan(o.ur);
        const double r0 = cam.fx * x * iz + cam.cx - (double)o.u;
        const double r1 = cam.fy * y * iz + cam.cy - (double)o.v;
        const double r2 = st ? cam.fx * (x - cam.b) * iz + cam.cx - (double)o.ur : 0.0;
        const double s = (r0 * r0 + r1 * r1 + r2 * r2) * in.isig2[o.oct];
        if (!(ok && s <= (st ? kD2Stereo : kD2Mono))) v.obs[i].oct = -1;
      }
      __syncthreads();
      const double c = ba_cost(v, O, sT, X, cam, in, s_red);
      if (tid == 0) s_cost = c;
      __syncthreads();
    }
    const double lam = s_lam;
    // ---- P1: pose blocks (wave per frame)
    for (int f = 1 + wid; f < n; f += kBlock / 64) {
      double h[21], g[6];
      for (int i = 0; i < 21; ++i) h[i] = 0;
      for (int i = 0; i < 6; ++i) g[i] = 0;
      const int b0 = v.hdr[8 + f], b1 = v.hdr[8 + f + 1];
      for (int ii = b0 + lane; ii < b1; ii += 64) {
        const int oi = v.flist[ii];
        const BaObs o = v.obs[oi];
        double r[3], w, rho, Jp[3][6], Jl[3][3];
        ba_eval<true>(sT[f], X + 3 * o.lm, o, cam, obs_is2(in, o), r, w, rho, Jp, Jl);
        int q = 0;
        for (int a = 0; a < 6; ++a) {
          for (int b = a; b < 6; ++b) h[q++] += w * (Jp[0][a] * Jp[0][b] + Jp[1][a] * Jp[1][b] + Jp[2][a] * Jp[2][b]);
          g[a] += w * (Jp[0][a] * r[0] + Jp[1][a] * r[1] + Jp[2][a] * r[2]);
        }
        double* Wo = v.W + (int64_t)oi * 18;
        for (int a = 0; a < 6; ++a)
          for (int b = 0; b < 3; ++b) Wo[3 * a + b] = w * (Jp[0][a] * Jl[0][b] + Jp[1][a] * Jl[1][b] + Jp[2][a] * Jl[2][b]);
      }
      for (int i = 0; i < 21; ++i) h[i] = wave_sum(h[i]);
      for (int i = 0; i < 6; ++i) g[i] = wave_sum(g[i]);
      if (lane == 0) {
        for (int i = 0; i < 21; ++i) sH[f][i] = h[i];
        for (int i = 0; i < 6; ++i) sg[f][i] = g[i];
      }
    }
    __syncthreads();  // W of every observation is complete before P2 reads it
    // ---- P2: landmarks -> L_l, g_l, Yt columns
    for (int l = tid; l < L; l += kBlock) {
      const int o0 = v.lstart[l], o1 = v.lstart[l + 1];
      double H[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
      for (int oi = o0; oi < o1; ++oi) {
        const BaObs o = v.obs[oi];
        double r[3], w, rho, Jp[3][6], Jl[3][3];
        ba_eval<true>(sT[o.frame], X + 3 * l, o, cam, obs_is2(in, o), r, w, rho, Jp, Jl);
        int q = 0;
        for (int a = 0; a < 3; ++a) {
          for (int b = a; b < 3; ++b) H[q++] += w * (Jl[0][a] * Jl[0][b] + Jl[1][a] * Jl[1][b] + Jl[2][a] * Jl[2][b]);
          g[a] += w * (Jl[0][a] * r[0] + Jl[1][a] * r[1] + Jl[2][a] * r[2]);
        }
      }
      // damped Cholesky of [H0 H1 H2; . H3 H4; . . H5]
      const double a00 = H[0] + lam * H[0] + 1e-6, a11 = H[3] + lam * H[3] + 1e-6, a22 = H[5] + lam * H[5] + 1e-6;
      const double l00 = sqrt(a00);
      const double l10 = H[1] / l00, l20 = H[2] / l00;
      const double l11 = sqrt(a11 - l10 * l10);
      const double l21 = (H[4] - l20 * l10) / l11;
      const double l22 = sqrt(a22 - l20 * l20 - l21 * l21);
      double* Lf = v.Lf + 6 * l;
      Lf[0] = l00; Lf[1] = l10; Lf[2] = l11; Lf[3] = l20; Lf[4] = l21; Lf[5] = l22;
      v.gl[3 * l] = g[0]; v.gl[3 * l + 1] = g[1]; v.gl[3 * l + 2] = g[2];
      double* Y0 = v.Yt + (int64_t)(3 * l) * NR;
      for (int oi = o0; oi < o1; ++oi) {
        const int f = v.obs[oi].frame;
        if (f == 0) continue;
        const double* Wo = v.W + (int64_t)oi * 18;
        for (int p = 0; p < 6; ++p) {  // row p of W L^-T: solve L y = W_p
          const double y0 = Wo[3 * p] / l00;
          const double y1 = (Wo[3 * p + 1] - l10 * y0) / l11;
          const double y2 = (Wo[3 * p + 2] - l20 * y0 - l21 * y1) / l22;
          const int row = 6 * (f - 1) + p;
          Y0[row] = y0;
          Y0[NR + row] = y1;
          Y0[2 * NR + row] = y2;
        }
      }
      const double z0 = g[0] / l00, z1 = (g[1] - l10 * z0) / l11, z2 = (g[2] - l20 * z0 - l21 * z1) / l22;
      Y0[NR - 1] = z0;
      Y0[2 * NR - 1] = z1;
      Y0[3 * NR - 1] = z2;
    }
    __syncthreads();
    // ---- P3: G = Yt^T Yt on MFMA (upper 16x16 tiles)
    {
      const int NT = NR / 16;
      const int npairs = NT * (NT + 1) / 2;
      for (int pidx = wid; pidx < npairs; pidx += kBlock / 64) {
        int I = 0, rem = pidx;
        while (rem >= NT - I) {
          rem -= NT - I;
          ++I;
        }
        const int J = I + rem;
        typedef double d4 __attribute__((ext_vector_type(4)));
        d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
        // A[i][k] = Yt[k][16I + i], B[k][j] = Yt[k][16J + j]; lane holds k = lane >> 4
        const double* ya = v.Yt + (lane >> 4) * NR + 16 * I + (lane & 15);
        const double* yb = v.Yt + (lane >> 4) * NR + 16 * J + (lane & 15);
        // frames whose pose rows fall in tile I / J (bit 31: the z column NR-1); a 4-row
        // chunk contributes only if its landmarks touch both (skipped chunks add exact 0)
        uint32_t mI = 0, mJ = 0;
        for (int r = 0; r < 16; ++r) {
          const int ra = 16 * I + r, rb = 16 * J + r;
          mI |= ra < np ? 1u << (ra / 6 + 1) : (ra == NR - 1 ? 1u << 31 : 0u);
          mJ |= rb < np ? 1u << (rb / 6 + 1) : (rb == NR - 1 ? 1u << 31 : 0u);
        }
        int par = 0;
        for (int c = 0; c < KP / 4; ++c) {
          const uint32_t cm = v.cmask[c];
          if (!(cm & mI) || !(cm & mJ)) continue;
          const int64_t o = (int64_t)(4 * c) * NR;
          if (par)
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[o], yb[o], acc1, 0, 0, 0);
          else
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[o], yb[o], acc0, 0, 0, 0);
          par ^= 1;
        }
        // f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
        for (int i = 0; i < 4; ++i)
          v.Sg[(16 * I + (lane >> 4) + 4 * i) * NR + 16 * J + (lane & 15)] = acc0[i] + acc1[i];
      }
    }
    __syncthreads();
    // ---- P4: reduced camera system, Cholesky
    for (int idx = tid; idx < np * np; idx += kBlock) {
      const int a = idx / np, b = idx % np;
      const int fa = a / 6 + 1, fb = b / 6 + 1;
      double hv = 0.0;
      if (fa == fb) {
        const int i = min(a % 6, b % 6), j = max(a % 6, b % 6);
        const int q = i * 6 - i * (i - 1) / 2 + (j - i);
        hv = sH[fa][q];
        if (i == j) hv += lam * hv + 1e-6;
      }
      const double gv = a <= b ? v.Sg[a * NR + b] : v.Sg[b * NR + a];
      sS[idx] = hv - gv;
    }
    for (int a = tid; a < np; a += kBlock) rhs[a] = -sg[a / 6 + 1][a % 6] + v.Sg[a * NR + NR - 1];
    if (tid == 0) s_fail = 0;
    __syncthreads();
    for (int k = 0; k < np; ++k) {
      if (tid == 0) {
        const double d = sS[k * np + k];
        if (!(d > 0.0)) s_fail = 1;
        else sS[k * np + k] = sqrt(d);
      }
      __syncthreads();
      if (s_fail) break;
      const double dk = sS[k * np + k];
      for (int i = k + 1 + tid; i < np; i += kBlock) sS[i * np + k] /= dk;
      __syncthreads();
      const int m = np - k - 1;
      for (int idx = tid; idx < m * m; idx += kBlock) {
        const int i = k + 1 + idx / m, j = k + 1 + idx % m;
        if (j <= i) sS[i * np + j] -= sS[i * np + k] * sS[j * np + k];
      }
      __syncthreads();
    }
    if (s_fail) {
      if (tid == 0) s_lam = fmin(s_lam * 10.0, 1e7);
      __syncthreads();
      continue;
    }
    if (wid == 0) {  // L y = rhs, L^T x = y (wave 0)
      for (int i = 0; i < np; ++i) {
        double p = 0;
        for (int j = lane; j < i; j += 64) p += sS[i * np + j] * rhs[j];
        p = wave_sum(p);
        if (lane == 0) rhs[i] = (rhs[i] - p) / sS[i * np + i];
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
      }
      for (int i = np - 1; i >= 0; --i) {
        double p = 0;
        for (int j = i + 1 + lane; j < np; j += 64) p += sS[j * np + i] * rhs[j];
        p = wave_sum(p);
        if (lane == 0) rhs[i] = (rhs[i] - p) / sS[i * np + i];
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    for (int a = tid; a < 6 * n; a += kBlock) sdp[a] = a < 6 ? 0.0 : rhs[a - 6];
    __syncthreads();
    // ---- P5: landmark back-substitution and pose update
    for (int l = tid; l < L; l += kBlock) {
      const int o0 = v.lstart[l], o1 = v.lstart[l + 1];
      double b[3] = {-v.gl[3 * l], -v.gl[3 * l + 1], -v.gl[3 * l + 2]};
      for (int oi = o0; oi < o1; ++oi) {
        const int f = v.obs[oi].frame;
        if (f == 0) continue;
        const double* Wo = v.W + (int64_t)oi * 18;
        const double* dp = sdp + 6 * f;
        for (int c = 0; c < 3; ++c)
          b[c] -= Wo[c] * dp[0] + Wo[3 + c] * dp[1] + Wo[6 + c] * dp[2] + Wo[9 + c] * dp[3] + Wo[12 + c] * dp[4] +
                  Wo[15 + c] * dp[5];
      }
      const double* Lf = v.Lf + 6 * l;
      const double y0 = b[0] / Lf[0], y1 = (b[1] - Lf[1] * y0) / Lf[2], y2 = (b[2] - Lf[3] * y0 - Lf[4] * y1) / Lf[5];
      const double x2 = y2 / Lf[5], x1 = (y1 - Lf[4] * x2) / Lf[2], x0 = (y0 - Lf[1] * x1 - Lf[3] * x2) / Lf[0];
      Xt[3 * l] = X[3 * l] + x0;
      Xt[3 * l + 1] = X[3 * l + 1] + x1;
      Xt[3 * l + 2] = X[3 * l + 2] + x2;
    }
    if (tid < n) {
      const int f = tid;
      if (f == 0) {
        for (int i = 0; i < 12; ++i) sTt[0][i] = sT[0][i];
      } else {
        double Rw[9];
        exp_so3(sdp + 6 * f, Rw);
        const double* T = sT[f];
        for (int i = 0; i < 3; ++i) {
          for (int j = 0; j < 3; ++j) sTt[f][3 * i + j] = Rw[3 * i] * T[j] + Rw[3 * i + 1] * T[3 + j] + Rw[3 * i + 2] * T[6 + j];
          sTt[f][9 + i] = Rw[3 * i] * T[9] + Rw[3 * i + 1] * T[10] + Rw[3 * i + 2] * T[11] + sdp[6 * f + 3 + i];
        }
      }
    }
    __syncthreads();
    // ---- P6/P7: cost at the tentative point, accept / reject
    const double cn = ba_cost(v, O, sTt, Xt, cam, in, s_red);
    if (tid == 0) {
      if (cn < s_cost) {
        s_cost = cn;
        s_lam = fmax(s_lam / 10.0, 1e-7);
        s_fail = 0;
        ++s_acc;
      } else {
        s_lam = fmin(s_lam * 10.0, 1e7);
        s_fail = 1;
      }
    }
    __syncthreads();
    if (!s_fail) {
      if (tid < n)
        for (int i = 0; i < 12; ++i) sT[tid][i] = sTt[tid][i];
      double* tmp = X;
      X = Xt;
      Xt = tmp;
    }
    __syncthreads();
  }
  // refined relative transform of the last pair: T_{n-1} T_{n-2}^-1
  if (tid == 0) {
    const double* A = sT[n - 1];
    const double* B = sT[n - 2];
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
    st[1] = s_cost;
    st[2] = (double)L;
    st[3] = (double)O;
    st[4] = (double)n;
    st[5] = (double)s_acc;
  }
  // the final landmark estimate lives in X (either buffer); keep v.X current for debugging
  if (X != v.X)
    for (int i = tid; i < 3 * L; i += kBlock) v.X[i] = X[i];
}

BaDims make_dims(const fvo_ctx* ctx) {
  const fvo_config& c = ctx->cfg;
  BaDims d{};
  d.Lmax = c.ba_max_landmarks;
  d.Omax = c.ba_max_obs;
  d.K = c.ba_window;
  d.cap = ctx->kp_cap;
  d.NR = 6 * (d.K - 1) < 63 ? 64 : 128;
  d.KP = ((3 * d.Lmax + 7) / 8) * 8;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    int64_t r = o;
    o += (bytes + 255) / 256 * 256;
    return r;
  };
  d.oX = take(8ll * 3 * d.Lmax);
  d.oXt = take(8ll * 3 * d.Lmax);
  d.oL = take(8ll * 6 * d.Lmax);
  d.oG = take(8ll * 3 * d.Lmax);
  d.oLs = take(4ll * (d.Lmax + 1));
  d.oObs = take((int64_t)sizeof(BaObs) * d.Omax);
  d.oFl = take(4ll * d.Omax);
  d.oW = take(8ll * 18 * d.Omax);
  d.oYt = take(8ll * d.KP * d.NR);
  d.oNext = take(4ll * kKMax * d.cap);
  d.oSg = take(8ll * d.NR * d.NR);
  d.oHdr = take(4ll * (8 + kKMax + 1));
  d.oCm = take(4ll * (d.KP / 4));
  d.win = o;
  return d;
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
  // the solver's dynamic LDS (reduced camera system) can exceed 64 KiB for K > 11
  const int np = 6 * (c.ba_window - 1);
  const size_t shm = (size_t)8 * (np * np + np);
  if (shm > 65536) FVO_HIP(ctx, hipFuncSetAttribute((const void*)k_ba_solve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
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
  BaDims d = make_dims(ctx);
  BaIn in{kp, nkp, matches, nmatch, reinterpret_cast<const float4*>(stereo), Trel, {}, nlev};
  for (int i = 0; i < nlev; ++i) in.isig2[i] = inv_sigma2[i];
  BaCam cam{K[0], K[4], K[2], K[5], baseline};
  FVO_TIMED(ctx, KN_BA_BUILD, s,
            hipLaunchKernelGGL(k_ba_build, dim3(nwin), dim3(kBlock), (size_t)cap, s, in, ctx->ba_ws, d, cam,
                               first_end, first_valid));
  const int np = 6 * (ctx->cfg.ba_window - 1);
  const size_t shm = (size_t)8 * (np * np + np);
  FVO_TIMED(ctx, KN_BA_SOLVE, s,
            hipLaunchKernelGGL(k_ba_solve, dim3(nwin), dim3(kBlock), shm, s, in, ctx->ba_ws, d, cam, first_end, iters,
                               BaOut{Tout, stats}));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
