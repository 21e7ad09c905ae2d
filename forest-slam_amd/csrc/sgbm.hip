// StereoSGBM (MODE_SGBM_3WAY) for gfx950 — replaces the disparity the reference computes in
// get_disparity_map (ros_ws/src/stereo_slam.py:108-117): numDisparities 96, minDisparity 0,
// blockSize 7, P1 392, P2 1568, 3-way aggregation, 4 fixed stripes, then medianBlur(3).
//
// Layout in HBM (per pair b): every volume is [row][x1][d] u16 with x1 = x - max(maxD,0)
// in [0, width1) and d in [0, D): a row slice is width1*D*2 bytes (166 KB at 600p).
//   k_sg_hsum    BT pixel cost (x-Sobel clipped + intensity>>2) staged per row chunk in
//                LDS, 7-tap horizontal box sum (clamped) -> hsum volume
//   k_sg_vsum    7-tap vertical running sum (rows clamped to [0,H-1]) -> cost volume C,
//                plus the 3 stripe-start rows whose window clamps at the stripe's first row
//   k_sg_vert    top->down SGM path, one lane per column x1, all D in packed u16x2 VGPRs,
//                restarted at each stripe's first processed row (OpenCV's overlap rule)
//   k_sg_horiz   left->right path (stored), right->left path fused with S = L+R+V, WTA,
//                parabolic sub-pixel step and the pseudo left-right check; one lane per row
//   k_sg_median  3x3 median (replicated border) -> int16 disparity*16
// Integer arithmetic only; results are bit-identical to oracle/sgbm_ref.cpp.
#include "fvo_internal.h"

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_v(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 vmin(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 splat(uint32_t s) { return as_v((s & 0xFFFFu) | (s << 16)); }

struct SgParams {
  int W, H, D, minD, minX1, width1, P1, P2, ftzero, disp12, ss, ov, nstripes;
};

// ------------------------------------------------------------------ pixel cost + hsum
constexpr int kChunk = 256;  // x1 outputs per block

__global__ __launch_bounds__(256) void k_sg_hsum(const uint8_t* __restrict__ Limg, const uint8_t* __restrict__ Rimg,
                                                 int64_t stride, int pitch, SgParams p,
                                                 uint16_t* __restrict__ hsum) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int W = p.W, D = p.D;
  // per-pixel planes for the whole row: a0,a1 (left), b0,b1 (right) + BT min/max of each
  uint8_t* la = smem;               // [2][W]
  uint8_t* lmn = la + 2 * W;        // [2][W]
  uint8_t* lmx = lmn + 2 * W;       // [2][W]
  uint8_t* rb = lmx + 2 * W;        // [2][W]
  uint8_t* rmn = rb + 2 * W;        // [2][W]
  uint8_t* rmx = rmn + 2 * W;       // [2][W]
  uint8_t* pd = rmx + 2 * W;        // [kChunk + 6][D]
  const int y = blockIdx.y, b = blockIdx.z;
  const int x1s = blockIdx.x * kChunk;
  const int x1e = min(x1s + kChunk, p.width1);
  const uint8_t* L = Limg + b * stride;
  const uint8_t* R = Rimg + b * stride;
  const uint8_t* r1 = L + (int64_t)y * pitch;
  const uint8_t* r2 = R + (int64_t)y * pitch;
  const uint8_t* n1 = L + (int64_t)(y > 0 ? y - 1 : y) * pitch;
  const uint8_t* s1 = L + (int64_t)(y < p.H - 1 ? y + 1 : y) * pitch;
  const uint8_t* n2 = R + (int64_t)(y > 0 ? y - 1 : y) * pitch;
  const uint8_t* s2 = R + (int64_t)(y < p.H - 1 ? y + 1 : y) * pitch;
  const int ft = p.ftzero;
  auto clip = [ft](int v) { return min(max(v, -ft), ft) + ft; };
  for (int x = threadIdx.x; x < W; x += blockDim.x) {
    int a0 = clip(0), a1v = clip(0), b0 = clip(0), b1v = clip(0);
    if (x >= 1 && x < W - 1) {
      a0 = clip((r1[x + 1] - r1[x - 1]) * 2 + n1[x + 1] - n1[x - 1] + s1[x + 1] - s1[x - 1]);
      b0 = clip((r2[x + 1] - r2[x - 1]) * 2 + n2[x + 1] - n2[x - 1] + s2[x + 1] - s2[x - 1]);
      a1v = r1[x];
      b1v = r2[x];
    }
    la[x] = (uint8_t)a0;
    la[W + x] = (uint8_t)a1v;
    rb[x] = (uint8_t)b0;
    rb[W + x] = (uint8_t)b1v;
  }
  __syncthreads();
  for (int x = threadIdx.x; x < W; x += blockDim.x) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint8_t* A = la + c * W;
      const uint8_t* Bv = rb + c * W;
      int u = A[x], ul = x > 0 ? (u + A[x - 1]) / 2 : u, ur = x < W - 1 ? (u + A[x + 1]) / 2 : u;
      lmn[c * W + x] = (uint8_t)min(min(ul, ur), u);
      lmx[c * W + x] = (uint8_t)max(max(ul, ur), u);
      int v = Bv[x], vl = x > 0 ? (v + Bv[x - 1]) / 2 : v, vr = x < W - 1 ? (v + Bv[x + 1]) / 2 : v;
      rmn[c * W + x] = (uint8_t)min(min(vl, vr), v);
      rmx[c * W + x] = (uint8_t)max(max(vl, vr), v);
    }
  }
  __syncthreads();
  // pixel cost for x1 in [x1s-3, x1e+3) (clamped to [0,width1-1]) into pd
  const int nloc = (x1e - x1s) + 6;
  for (int i = threadIdx.x; i < nloc * D; i += blockDim.x) {
    int xl = i / D, d = i - xl * D;
    int x1 = min(max(x1s - 3 + xl, 0), p.width1 - 1);
    int x = x1 + p.minX1;
    int xr = x - (d + p.minD);
    int cost = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      int u = la[c * W + x], u0 = lmn[c * W + x], u1 = lmx[c * W + x];
      int v = rb[c * W + xr], v0 = rmn[c * W + xr], v1 = rmx[c * W + xr];
      int c0 = max(0, u - v1);
      c0 = max(c0, v0 - u);
      int c1 = max(0, v - u1);
      c1 = max(c1, u0 - v);
      cost += min(c0, c1) >> (c == 0 ? 0 : 2);
    }
    pd[i] = (uint8_t)cost;
  }
  __syncthreads();
  uint16_t* out = hsum + ((int64_t)b * p.H + y) * p.width1 * D;
  for (int i = threadIdx.x; i < (x1e - x1s) * D; i += blockDim.x) {
    int xl = i / D, d = i - xl * D;
    int s = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) s += pd[(xl + k) * D + d];
    out[(int64_t)(x1s + xl) * D + d] = (uint16_t)s;
  }
}

// ------------------------------------------------------------------ vertical box sum
__global__ void k_sg_vsum(const uint16_t* __restrict__ hsum, uint16_t* __restrict__ cost,
                          uint16_t* __restrict__ cost_extra, SgParams p) {
  const int64_t plane = (int64_t)p.width1 * p.D;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= plane) return;
  const uint16_t* hs = hsum + (int64_t)b * p.H * plane + i;
  uint16_t* co = cost + (int64_t)b * p.H * plane + i;
  const int H = p.H;
  auto hrow = [&](int r) -> int { return hs[(int64_t)min(max(r, 0), H - 1) * plane]; };
  int acc = 0;
  for (int r = -3; r <= 3; ++r) acc += hrow(r);
  co[0] = (uint16_t)acc;
  for (int y = 1; y < H; ++y) {
    acc += hrow(y + 3) - hrow(y - 4);
    co[(int64_t)y * plane] = (uint16_t)acc;
  }
  // stripe-start rows: window rows clamp at the stripe's first processed row
  uint16_t* ce = cost_extra + (int64_t)b * (p.nstripes - 1) * 3 * plane + i;
  for (int s = 1; s < p.nstripes; ++s) {
    int start = max(min(s * p.ss - p.ov, H), 0);
    for (int k = 0; k < 3; ++k) {
      int y = start + k;
      int a = 0;
      for (int r = y - 3; r <= y + 3; ++r) a += hs[(int64_t)min(max(r, start), H - 1) * plane];
      ce[(int64_t)((s - 1) * 3 + k) * plane] = (uint16_t)a;
    }
  }
}

// ------------------------------------------------------------------ top->down path
template <int D>
__global__ __launch_bounds__(64) void k_sg_vert(const uint16_t* __restrict__ cost, const uint16_t* __restrict__ cost_extra,
                                                uint16_t* __restrict__ V, SgParams p) {
  constexpr int NP = D / 2;
  const int x1 = blockIdx.x * 64 + threadIdx.x;
  const int s = blockIdx.y, b = blockIdx.z;
  if (x1 >= p.width1) return;
  const int64_t plane = (int64_t)p.width1 * D;
  const int H = p.H;
  const int start = max(min(s * p.ss - p.ov, H), 0);
  const int end = min((s + 1) * p.ss, H);
  const int first_out = min(s * p.ss, H);
  uint32_t st[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) st[k] = 0;
  uint32_t minPrev = 0;
  const u16x2 P1 = splat(p.P1);
  const uint32_t SENT = 0x7FFFu;
  for (int y = start; y < end; ++y) {
    const uint16_t* crow;
    if (s > 0 && y < start + 3)
      crow = cost_extra + ((int64_t)b * (p.nstripes - 1) * 3 + (s - 1) * 3 + (y - start)) * plane;
    else
      crow = cost + ((int64_t)b * H + y) * plane;
    const uint4* cp = reinterpret_cast<const uint4*>(crow + (int64_t)x1 * D);
    uint32_t c[NP];
#pragma unroll
    for (int k = 0; k < NP / 4; ++k) {
      uint4 q = cp[k];
      c[4 * k] = q.x; c[4 * k + 1] = q.y; c[4 * k + 2] = q.z; c[4 * k + 3] = q.w;
    }
    const u16x2 mp2 = splat(minPrev + p.P2);
    const u16x2 mpv = splat(minPrev);
    uint32_t nst[NP];
    u16x2 mn = splat(0xFFFF);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      uint32_t lo = k > 0 ? st[k - 1] : (SENT << 16);
      uint32_t hi = k < NP - 1 ? st[k + 1] : SENT;
      u16x2 cur = as_v(st[k]);
      u16x2 dm = as_v(__builtin_amdgcn_alignbit(st[k], lo, 16));  // (prev[2k-1], prev[2k])
      u16x2 dp = as_v(__builtin_amdgcn_alignbit(hi, st[k], 16));  // (prev[2k+1], prev[2k+2])
      u16x2 m = vmin(vmin(dm + P1, dp + P1), vmin(cur, mp2));
      u16x2 nv = as_v(c[k]) + m - mpv;
      nst[k] = as_u(nv);
      mn = vmin(mn, nv);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) st[k] = nst[k];
    uint32_t mu = as_u(mn);
    minPrev = min(mu & 0xFFFFu, mu >> 16);
    if (y >= first_out) {
      uint4* vp = reinterpret_cast<uint4*>(V + ((int64_t)b * H + y) * plane + (int64_t)x1 * D);
#pragma unroll
      for (int k = 0; k < NP / 4; ++k) vp[k] = make_uint4(st[4 * k], st[4 * k + 1], st[4 * k + 2], st[4 * k + 3]);
    }
  }
}

// ------------------------------------------------------------------ horizontal paths + WTA
template <int D>
__global__ __launch_bounds__(64) void k_sg_horiz(const uint16_t* __restrict__ cost, const uint16_t* __restrict__ V,
                                                 uint16_t* __restrict__ Lv, int16_t* __restrict__ raw,
                                                 int16_t* __restrict__ d2, int32_t* __restrict__ d2c, SgParams p) {
  constexpr int NP = D / 2;
  __shared__ uint32_t sS[64][NP + 1];
  const int lane = threadIdx.x;
  const int y = blockIdx.x * 64 + lane;
  const int b = blockIdx.y;
  const int H = p.H, W = p.W;
  if (y >= H) return;
  const int64_t plane = (int64_t)p.width1 * D;
  const uint16_t* crow = cost + ((int64_t)b * H + y) * plane;
  uint16_t* lrow = Lv + ((int64_t)b * H + y) * plane;
  const uint16_t* vrow = V + ((int64_t)b * H + y) * plane;
  const u16x2 P1 = splat(p.P1);
  const uint32_t SENT = 0x7FFFu;
  // ---- left -> right
  uint32_t st[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) st[k] = 0;
  uint32_t minPrev = 0;
  for (int x1 = 0; x1 < p.width1; ++x1) {
    const uint4* cp = reinterpret_cast<const uint4*>(crow + (int64_t)x1 * D);
    uint32_t c[NP];
#pragma unroll
    for (int k = 0; k < NP / 4; ++k) {
      uint4 q = cp[k];
      c[4 * k] = q.x; c[4 * k + 1] = q.y; c[4 * k + 2] = q.z; c[4 * k + 3] = q.w;
    }
    const u16x2 mp2 = splat(minPrev + p.P2), mpv = splat(minPrev);
    uint32_t nst[NP];
    u16x2 mn = splat(0xFFFF);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      uint32_t lo = k > 0 ? st[k - 1] : (SENT << 16);
      uint32_t hi = k < NP - 1 ? st[k + 1] : SENT;
      u16x2 dm = as_v(__builtin_amdgcn_alignbit(st[k], lo, 16));
      u16x2 dp = as_v(__builtin_amdgcn_alignbit(hi, st[k], 16));
      u16x2 m = vmin(vmin(dm + P1, dp + P1), vmin(as_v(st[k]), mp2));
      u16x2 nv = as_v(c[k]) + m - mpv;
      nst[k] = as_u(nv);
      mn = vmin(mn, nv);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) st[k] = nst[k];
    uint32_t mu = as_u(mn);
    minPrev = min(mu & 0xFFFFu, mu >> 16);
    uint4* lp = reinterpret_cast<uint4*>(lrow + (int64_t)x1 * D);
#pragma unroll
    for (int k = 0; k < NP / 4; ++k) lp[k] = make_uint4(st[4 * k], st[4 * k + 1], st[4 * k + 2], st[4 * k + 3]);
  }
  // ---- right -> left, sum, WTA, sub-pixel, right-view disparity
  const int INVALID = (p.minD - 1) * 16;
  int16_t* drow = raw + ((int64_t)b * H + y) * W;
  int16_t* d2row = d2 + ((int64_t)b * H + y) * W;
  int32_t* d2crow = d2c + ((int64_t)b * H + y) * W;
  for (int x = 0; x < W; ++x) {
    drow[x] = (int16_t)INVALID;
    d2row[x] = (int16_t)INVALID;
    d2crow[x] = 0x7FFF;
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) st[k] = 0;
  minPrev = 0;
  for (int x1 = p.width1 - 1; x1 >= 0; --x1) {
    const uint4* cp = reinterpret_cast<const uint4*>(crow + (int64_t)x1 * D);
    const uint4* lp = reinterpret_cast<const uint4*>(lrow + (int64_t)x1 * D);
    const uint4* vp = reinterpret_cast<const uint4*>(vrow + (int64_t)x1 * D);
    uint32_t c[NP], lv[NP], vv[NP];
#pragma unroll
    for (int k = 0; k < NP / 4; ++k) {
      uint4 q = cp[k], l4 = lp[k], v4 = vp[k];
      c[4 * k] = q.x; c[4 * k + 1] = q.y; c[4 * k + 2] = q.z; c[4 * k + 3] = q.w;
      lv[4 * k] = l4.x; lv[4 * k + 1] = l4.y; lv[4 * k + 2] = l4.z; lv[4 * k + 3] = l4.w;
      vv[4 * k] = v4.x; vv[4 * k + 1] = v4.y; vv[4 * k + 2] = v4.z; vv[4 * k + 3] = v4.w;
    }
    const u16x2 mp2 = splat(minPrev + p.P2), mpv = splat(minPrev);
    uint32_t nst[NP];
    u16x2 mn = splat(0xFFFF), smn = splat(0xFFFF);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      uint32_t lo = k > 0 ? st[k - 1] : (SENT << 16);
      uint32_t hi = k < NP - 1 ? st[k + 1] : SENT;
      u16x2 dm = as_v(__builtin_amdgcn_alignbit(st[k], lo, 16));
      u16x2 dp = as_v(__builtin_amdgcn_alignbit(hi, st[k], 16));
      u16x2 m = vmin(vmin(dm + P1, dp + P1), vmin(as_v(st[k]), mp2));
      u16x2 nv = as_v(c[k]) + m - mpv;
      nst[k] = as_u(nv);
      mn = vmin(mn, nv);
      u16x2 S = as_v(lv[k]) + nv + as_v(vv[k]);
      sS[lane][k] = as_u(S);
      smn = vmin(smn, S);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) st[k] = nst[k];
    uint32_t mu = as_u(mn);
    minPrev = min(mu & 0xFFFFu, mu >> 16);
    uint32_t su = as_u(smn);
    const int minCost = (int)min(su & 0xFFFFu, su >> 16);
    int best = D - 1;
    for (int k = NP - 1; k >= 0; --k) {
      uint32_t w = sS[lane][k];
      if ((int)(w >> 16) == minCost) best = 2 * k + 1;
      if ((int)(w & 0xFFFFu) == minCost) best = 2 * k;
    }
    auto Sd = [&](int d) -> int {
      uint32_t w = sS[lane][d >> 1];
      return (int)((d & 1) ? (w >> 16) : (w & 0xFFFFu));
    };
    const int d = best;
    const int x2 = x1 + p.minX1 - d - p.minD;
    if (x2 >= 0 && x2 < W && d2crow[x2] > minCost) {
      d2crow[x2] = minCost;
      d2row[x2] = (int16_t)(d + p.minD);
    }
    int dd;
    if (0 < d && d < D - 1) {
      int sm = Sd(d - 1), sp = Sd(d + 1), s0 = Sd(d);
      int denom2 = max(sm + sp - 2 * s0, 1);
      dd = d * 16 + ((sm - sp) * 16 + denom2) / (denom2 * 2);
    } else {
      dd = d * 16;
    }
    drow[x1 + p.minX1] = (int16_t)(dd + p.minD * 16);
  }
  // ---- pseudo left-right consistency check
  for (int x = p.minX1; x < p.minX1 + p.width1; ++x) {
    int d1 = drow[x];
    if (d1 == INVALID) continue;
    int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
    int _x = x - _d, x_ = x - d_;
    if (0 <= x_ && x_ < W && d2row[x_] >= p.minD && abs(d2row[x_] - d_) > p.disp12 && 0 <= _x && _x < W &&
        d2row[_x] >= p.minD && abs(d2row[_x] - _d) > p.disp12)
      drow[x] = (int16_t)INVALID;
  }
}

// ------------------------------------------------------------------ median 3x3
__global__ void k_sg_median(const int16_t* __restrict__ raw, int16_t* __restrict__ out, int W, int H) {
  int x = blockIdx.x * blockDim.x + threadIdx.x;
  int y = blockIdx.y, b = blockIdx.z;
  if (x >= W) return;
  const int16_t* s = raw + (int64_t)b * H * W;
  int v[9];
  int k = 0;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      int yy = min(max(y + dy, 0), H - 1), xx = min(max(x + dx, 0), W - 1);
      v[k++] = s[(int64_t)yy * W + xx];
    }
  // Paeth's 19-compare median-of-9 network
#define SG_S(a, b) { int t_ = min(v[a], v[b]); v[b] = max(v[a], v[b]); v[a] = t_; }
  SG_S(1, 2) SG_S(4, 5) SG_S(7, 8) SG_S(0, 1) SG_S(3, 4) SG_S(6, 7) SG_S(1, 2) SG_S(4, 5) SG_S(7, 8)
  SG_S(0, 3) SG_S(5, 8) SG_S(4, 7) SG_S(3, 6) SG_S(1, 4) SG_S(2, 5) SG_S(4, 7) SG_S(4, 2) SG_S(6, 4)
  SG_S(4, 2)
#undef SG_S
  out[((int64_t)b * H + y) * W + x] = (int16_t)v[4];
}

SgParams make_params(const fvo_config& c) {
  SgParams p;
  p.W = c.width;
  p.H = c.height;
  p.D = c.num_disparities;
  p.minD = c.min_disparity;
  int maxD = p.minD + p.D;
  p.minX1 = maxD > 0 ? maxD : 0;
  int maxX1 = c.width + (p.minD < 0 ? p.minD : 0);
  p.width1 = maxX1 - p.minX1;
  p.P1 = c.P1 > 0 ? c.P1 : 2;
  p.P2 = std::max(c.P2 > 0 ? c.P2 : 5, p.P1 + 1);
  p.ftzero = std::max(c.pre_filter_cap, 15) | 1;
  p.disp12 = c.disp12_max_diff > 0 ? c.disp12_max_diff : 1;
  p.nstripes = c.sgbm_stripes;
  p.ss = (int)std::ceil(c.height / (double)p.nstripes);
  p.ov = (c.block_size / 2 + 1) + (int)std::ceil(0.1 * p.ss);
  return p;
}

}  // namespace

int sgbm_init(fvo_ctx* ctx) {
  const fvo_config& c = ctx->cfg;
  if (c.block_size != 7) return fvo_fail(ctx, "SGBM: only blockSize=7 is supported");
  if (c.num_disparities != 64 && c.num_disparities != 96 && c.num_disparities != 128)
    return fvo_fail(ctx, "SGBM: numDisparities must be 64, 96 or 128");
  if (c.uniqueness_ratio != 0) return fvo_fail(ctx, "SGBM: only uniquenessRatio=0 is supported");
  if (c.sgbm_stripes < 1) return fvo_fail(ctx, "SGBM: stripes must be >= 1");
  SgParams p = make_params(c);
  if (p.width1 <= 0) return fvo_fail(ctx, "SGBM: image narrower than numDisparities");
  const int64_t B = c.max_batch, plane = (int64_t)p.width1 * p.D;
  ctx->sg_extra_rows = (p.nstripes - 1) * 3;
  int rc;
  if ((rc = fvo_alloc(ctx, &ctx->sg_cost, B * (p.H + ctx->sg_extra_rows) * plane)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_L, B * p.H * plane)) || (rc = fvo_alloc(ctx, &ctx->sg_V, B * p.H * plane)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_raw, B * p.H * p.W)) || (rc = fvo_alloc(ctx, &ctx->sg_d2, B * p.H * p.W)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_d2c, B * p.H * p.W)))
    return rc;
  return 0;
}

int sgbm_run(fvo_ctx* ctx, const uint8_t* L, const uint8_t* R, int batch, int64_t image_stride, int pitch,
             int16_t* disp, hipStream_t s) {
  const fvo_config& c = ctx->cfg;
  SgParams p = make_params(c);
  const int64_t plane = (int64_t)p.width1 * p.D;
  uint16_t* hsum = ctx->sg_L;  // the L volume doubles as hsum scratch (consumed before L is written)
  uint16_t* cost = ctx->sg_cost;
  uint16_t* cost_extra = ctx->sg_cost + (int64_t)batch * p.H * plane;
  size_t shm = (size_t)12 * p.W + (size_t)(kChunk + 6) * p.D;
  FVO_TIMED(ctx, KN_SG_HSUM, s, hipLaunchKernelGGL(k_sg_hsum, dim3((p.width1 + kChunk - 1) / kChunk, p.H, batch), dim3(256), shm, s, L, R,
                     image_stride, pitch, p, hsum));
  FVO_TIMED(ctx, KN_SG_VSUM, s, hipLaunchKernelGGL(k_sg_vsum, dim3((unsigned)((plane + 255) / 256), batch), dim3(256), 0, s, hsum, cost, cost_extra,
                     p));
  dim3 gv((p.width1 + 63) / 64, p.nstripes, batch), gh((p.H + 63) / 64, batch);
  switch (p.D) {
    case 64:
      FVO_TIMED(ctx, KN_SG_VERT, s, hipLaunchKernelGGL(k_sg_vert<64>, gv, dim3(64), 0, s, cost, cost_extra, ctx->sg_V, p));
      FVO_TIMED(ctx, KN_SG_HORIZ, s, hipLaunchKernelGGL(k_sg_horiz<64>, gh, dim3(64), 0, s, cost, ctx->sg_V, ctx->sg_L, ctx->sg_raw, ctx->sg_d2,
                         ctx->sg_d2c, p));
      break;
    case 96:
      FVO_TIMED(ctx, KN_SG_VERT, s, hipLaunchKernelGGL(k_sg_vert<96>, gv, dim3(64), 0, s, cost, cost_extra, ctx->sg_V, p));
      FVO_TIMED(ctx, KN_SG_HORIZ, s, hipLaunchKernelGGL(k_sg_horiz<96>, gh, dim3(64), 0, s, cost, ctx->sg_V, ctx->sg_L, ctx->sg_raw, ctx->sg_d2,
                         ctx->sg_d2c, p));
      break;
    default:
      FVO_TIMED(ctx, KN_SG_VERT, s, hipLaunchKernelGGL(k_sg_vert<128>, gv, dim3(64), 0, s, cost, cost_extra, ctx->sg_V, p));
      FVO_TIMED(ctx, KN_SG_HORIZ, s, hipLaunchKernelGGL(k_sg_horiz<128>, gh, dim3(64), 0, s, cost, ctx->sg_V, ctx->sg_L, ctx->sg_raw, ctx->sg_d2,
                         ctx->sg_d2c, p));
      break;
  }
  FVO_TIMED(ctx, KN_SG_MEDIAN, s, hipLaunchKernelGGL(k_sg_median, dim3((p.W + 255) / 256, p.H, batch), dim3(256), 0, s, ctx->sg_raw, disp, p.W, p.H));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
