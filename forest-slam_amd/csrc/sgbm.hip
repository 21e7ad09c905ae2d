// StereoSGBM (MODE_SGBM_3WAY) for gfx950 — replaces the disparity the reference computes in
// get_disparity_map (ros_ws/src/stereo_slam.py:108-117): numDisparities 96, minDisparity 0,
// blockSize 7, P1 392, P2 1568, 3-way aggregation, 4 fixed stripes, then medianBlur(3).
//
// Volumes per pair, u16 [HG][x1][16][d] (row groups of 16 rows interleaved per column, so
// the 16 rows a wave of k_sg_horiz scans read 3 KB contiguous per column step; x1 = x -
// max(maxD,0) in [0,width1), d in [0,D)): C and V (k_sg_costvert -> k_sg_horiz), LV = L + V
// (the left->right pass).  raw is [x][row] int16, the right-view keys [x][row] u32.
// Kernels
//   k_sg_costvert<D,CB>  block of CB column quads (D/4 disparities per lane) marching down a
//                  stripe: BT pixel cost of both channels in one u16x2 word from LDS-staged
//                  rows, 7x7 box sum (7-column sum from LDS, 7-row running sum over a VGPR
//                  shift register, rows clamped to the stripe's first row and to H-1 -- the
//                  overlap rule of OpenCV's 4 stripes), fused with the top->down path
//   k_sg_horiz<D,PF> quad of lanes per row: left->right path (stores LV), right->left path
//                  fused with S = LV + R, first-minimum WTA, integer parabolic sub-pixel,
//                  right-view disparity (atomicMin keys) and the pseudo left-right check
//   k_sg_median    3x3 median (replicated border) -> int16 disparity*16
// Path states are packed u16x2 VGPRs (v_pk_add/sub/min_u16, v_alignbit for d-1 / d+1);
// neighbours across the quad come from DPP quad permutes.  Integer arithmetic only;
// bit-identical to oracle/sgbm_ref.cpp.
#include <algorithm>
#include <cstdlib>

#include "fvo_internal.h"

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_v(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 vmin(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 splat(uint32_t s) { return as_v((s & 0xFFFFu) | (s << 16)); }

struct SgParams {
  int W, H, D, minD, minX1, width1, P1, P2, ftzero, disp12, ss, ov, nstripes;
  int HG;  // row groups of 16 (volume layout)
};

// SGM recurrence for one packed pair k of a lane's disparity run, in place.  `old_km1`
// carries the previous value of pair k-1 (already overwritten); lo0 / hiN are the words
// that border the run (sentinels, or the neighbour lane's old values).
template <int NPL>
__device__ __forceinline__ uint32_t sgm_pair(uint32_t* st, int k, uint32_t& old_km1, uint32_t c, u16x2 P1,
                                             u16x2 mp2, u16x2 mpv, uint32_t lo0, uint32_t hiN) {
  uint32_t cur = st[k];
  uint32_t lo = k > 0 ? old_km1 : lo0;
  uint32_t hi = k < NPL - 1 ? st[k + 1] : hiN;
  u16x2 dm = as_v(__builtin_amdgcn_alignbit(cur, lo, 16));  // (prev[2k-1], prev[2k])
  u16x2 dp = as_v(__builtin_amdgcn_alignbit(hi, cur, 16));  // (prev[2k+1], prev[2k+2])
  u16x2 m = vmin(vmin(dm + P1, dp + P1), vmin(as_v(cur), mp2));
  uint32_t nv = as_u(as_v(c) + m - mpv);
  old_km1 = cur;
  st[k] = nv;
  return nv;
}

constexpr uint32_t kSent = 0x7FFFu;  // "no neighbour" entry: P1 + 0x7FFF never wins the min

// ------------------------------------------------------------------ quad helpers
// A quad of lanes owns one row; lane q of the quad holds disparities [q*D/4, (q+1)*D/4).
// Neighbour entries across the quad come from DPP quad permutes; minima by two xor steps.
constexpr int kQPrev = 0x90;  // quad_perm [0,0,1,2]: value of lane q-1
constexpr int kQNext = 0xF9;  // quad_perm [1,2,3,3]: value of lane q+1
constexpr int kQX1 = 0xB1;    // quad_perm [1,0,3,2]
constexpr int kQX2 = 0x4E;    // quad_perm [2,3,0,1]

template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

template <int NV4>
__device__ __forceinline__ void load_run(const uint16_t* base, uint32_t* out) {
  const uint4* p4 = reinterpret_cast<const uint4*>(base);
#pragma unroll
  for (int i = 0; i < NV4; ++i) {
    uint4 q = p4[i];
    out[4 * i] = q.x; out[4 * i + 1] = q.y; out[4 * i + 2] = q.z; out[4 * i + 3] = q.w;
  }
}

// One step of a path over a lane's run with G lanes per column (G = 4: quad; G = 8: half
// row, neighbours by DPP row shifts, minimum by two quad steps + row_half_mirror); returns
// the group-wide minimum.
template <int PQ, int G>
__device__ __forceinline__ uint32_t hstepG(uint32_t* st, const uint32_t* c, int q, u16x2 P1, uint32_t minPrev,
                                           uint32_t P2) {
  uint32_t prevLast, nextFirst;
  if (G == 4) {
    prevLast = qperm<kQPrev>(st[PQ - 1]);
    nextFirst = qperm<kQNext>(st[0]);
  } else {
    prevLast = (uint32_t)__builtin_amdgcn_mov_dpp((int)st[PQ - 1], 0x111, 0xF, 0xF, false);  // row_shr:1
    nextFirst = (uint32_t)__builtin_amdgcn_mov_dpp((int)st[0], 0x101, 0xF, 0xF, false);      // row_shl:1
  }
  const uint32_t lo0 = q == 0 ? (kSent << 16) : prevLast;
  const uint32_t hiN = q == G - 1 ? kSent : nextFirst;
  const u16x2 mp2 = splat(minPrev + P2), mpv = splat(minPrev);
  u16x2 mn = splat(0xFFFF);
  uint32_t oldk = 0;
#pragma unroll
  for (int k = 0; k < PQ; ++k) mn = vmin(mn, as_v(sgm_pair<PQ>(st, k, oldk, c[k], P1, mp2, mpv, lo0, hiN)));
  uint32_t m = as_u(mn);
  m = min(m & 0xFFFFu, m >> 16);
  m = min(m, qperm<kQX1>(m));
  m = min(m, qperm<kQX2>(m));
  if (G == 8) m = min(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x141, 0xF, 0xF, false));  // row_half_mirror
  return m;
}

template <int NV2>
__device__ __forceinline__ void load_run2(const uint16_t* base, uint32_t* out) {
  const uint2* p2 = reinterpret_cast<const uint2*>(base);
#pragma unroll
  for (int i = 0; i < NV2; ++i) {
    uint2 q = p2[i];
    out[2 * i] = q.x; out[2 * i + 1] = q.y;
  }
}

// One step of a horizontal path over a lane's run; returns the quad-wide minimum.
template <int PQ>
__device__ __forceinline__ uint32_t hstep(uint32_t* st, const uint32_t* c, int q, u16x2 P1, uint32_t minPrev,
                                          uint32_t P2) {
  const uint32_t prevLast = qperm<kQPrev>(st[PQ - 1]);
  const uint32_t nextFirst = qperm<kQNext>(st[0]);
  const uint32_t lo0 = q == 0 ? (kSent << 16) : prevLast;
  const uint32_t hiN = q == 3 ? kSent : nextFirst;
  const u16x2 mp2 = splat(minPrev + P2), mpv = splat(minPrev);
  u16x2 mn = splat(0xFFFF);
  uint32_t oldk = 0;
#pragma unroll
  for (int k = 0; k < PQ; ++k) mn = vmin(mn, as_v(sgm_pair<PQ>(st, k, oldk, c[k], P1, mp2, mpv, lo0, hiN)));
  uint32_t m = as_u(mn);
  m = min(m & 0xFFFFu, m >> 16);
  m = min(m, qperm<kQX1>(m));
  m = min(m, qperm<kQX2>(m));
  return m;
}


// ------------------------------------------------------------------ fused cost + vertical pass
// One block (4 waves) per (64 columns, stripe, pair); quad of lanes per column as in
// k_sg_vert.  Per new hsum row (the row entering the 7-row window) the block stages the 3
// image rows of its column range in LDS (left: 70 px, right: 70 + D - 1 px, +2 apron),
// derives the (x-Sobel, intensity) channel words and their BT min/max, evaluates the packed
// BT pixel cost of its 70 x D cells into LDS and box-sums 7 columns per lane.  The window's
// 8 hsum rows are a shift register in VGPRs, so the hsum volume never goes to HBM.  The next
// row's image bytes are fetched before the current row is processed.  Same integer
// arithmetic as k_sg_hsum + k_sg_vert (order-independent sums).
template <int D, int CB, int G>
__global__ __launch_bounds__(G * CB) void k_sg_costvert(const uint8_t* __restrict__ Limg, const uint8_t* __restrict__ Rimg,
                                                    int64_t stride, int pitch, SgParams p, uint16_t* __restrict__ Cvol,
                                                    uint16_t* __restrict__ Vvol) {
  constexpr int DQ = D / G, PQ = DQ / 2, NV2 = DQ / 4;
  constexpr int NT = G * CB;                // threads: G lanes per column
  constexpr int kCX = CB + 6;               // pixel-cost columns (7-wide box apron)
  constexpr int NRC = kCX + D - 1;          // right-image core pixels
  constexpr int NLI = kCX + 4, NRI = NRC + 4;  // staged pixels per image row (core + 2 each side)
  constexpr int NIMG = 3 * (NLI + NRI);     // staged bytes per hsum row
  constexpr int PER = (NIMG + NT - 1) / NT;  // staged bytes per thread
  __shared__ uint8_t sImg[3][NLI + NRI];
  __shared__ uint32_t sCh[kCX + 2 + NRC + 2];                       // (Sobel, intensity), L then R
  __shared__ uint32_t sW[3][kCX + NRC];                            // u, BT min, BT max, L then R
  __shared__ __attribute__((aligned(16))) uint16_t sPC[kCX][D];    // pixel cost
  const int tid = threadIdx.x, lane = tid & 63, q = lane % G;
  const int col = (tid >> 6) * (64 / G) + lane / G;  // 0..CB-1
  const int c0 = blockIdx.x * CB;
  const int s = blockIdx.y, b = blockIdx.z;
  const int H = p.H, W = p.W;
  const int start = max(min(s * p.ss - p.ov, H), 0);
  const int end = min((s + 1) * p.ss, H);
  const int first_out = min(s * p.ss, H);
  if (start >= end) return;
  const uint8_t* Lb = Limg + b * stride;
  const uint8_t* Rb = Rimg + b * stride;
  const int xl0 = max(c0 - 3, 0) + p.minX1;                    // first left core pixel
  const int xl1 = min(c0 + CB + 2, p.width1 - 1) + p.minX1;   // last left core pixel
  const int nl = xl1 - xl0 + 1;                                // <= kCX
  const int xr0 = xl0 - (D - 1) - p.minD;                      // first right core pixel (>= 1)
  const int nr = nl + D - 1;                                   // <= NRC
  const int ft = p.ftzero;
  auto clip = [ft](int v) { return min(max(v, -ft), ft) + ft; };

  // image bytes of hsum row r (rows r-1, r, r+1, clamped): thread-private prefetch slots
  uint8_t pre[PER];
  auto fetch = [&](int r) {
    const int rows[3] = {r > 0 ? r - 1 : r, r, r < H - 1 ? r + 1 : r};
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + NT * k;
      uint8_t v = 0;
      if (i < NIMG) {
        const int rr = i / (NLI + NRI), j = i % (NLI + NRI);
        if (j < NLI) v = Lb[(int64_t)rows[rr] * pitch + min(max(xl0 - 2 + j, 0), W - 1)];
        else v = Rb[(int64_t)rows[rr] * pitch + min(max(xr0 - 2 + (j - NLI), 0), W - 1)];
      }
      pre[k] = v;
    }
  };
  // hsum row from the staged bytes -> acc (this lane's column and disparity run)
  auto hs_row = [&](uint32_t* acc) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + NT * k;
      if (i < NIMG) (&sImg[0][0])[i] = pre[k];
    }
    __syncthreads();
    // channel words at core-1 .. core+1 of both images; borders (x < 1, x >= W-1) read ftzero
    for (int j = tid; j < (nl + 2) + (nr + 2); j += NT) {
      const bool left = j < nl + 2;
      const int k = left ? j : j - (nl + 2);
      const int x = (left ? xl0 : xr0) - 1 + k;
      const uint8_t* r0 = &sImg[0][left ? 0 : NLI];
      const uint8_t* r1 = &sImg[1][left ? 0 : NLI];
      const uint8_t* r2 = &sImg[2][left ? 0 : NLI];
      const int jj = k + 1;
      uint32_t wv = (uint32_t)clip(0) * 0x10001u;
      if (x >= 1 && x < W - 1) {
        const int sb = (r1[jj + 1] - r1[jj - 1]) * 2 + r0[jj + 1] - r0[jj - 1] + r2[jj + 1] - r2[jj - 1];
        wv = (uint32_t)clip(sb) | ((uint32_t)r1[jj] << 16);
      }
      sCh[left ? k : (kCX + 2) + k] = wv;
    }
    __syncthreads();
    // BT words: u, min(u, (u+ul)/2, (u+ur)/2), max(...); at x = 0 / W-1 the half is u itself
    for (int j = tid; j < nl + nr; j += NT) {
      const bool left = j < nl;
      const int k = left ? j : j - nl;
      const int x = left ? xl0 + k : xr0 + k;
      const uint32_t* ch = left ? sCh : sCh + (kCX + 2);
      const u16x2 u = as_v(ch[k + 1]);
      u16x2 hl = (u + as_v(ch[k])) >> 1, hr = (u + as_v(ch[k + 2])) >> 1;
      if (x == 0) hl = u;
      if (x == W - 1) hr = u;
      const int o = left ? k : kCX + k;
      sW[0][o] = as_u(u);
      sW[1][o] = as_u(vmin(vmin(hl, hr), u));
      sW[2][o] = as_u(__builtin_elementwise_max(__builtin_elementwise_max(hl, hr), u));
    }
    __syncthreads();
    // pixel costs of the kCX (clamped) columns x D disparities, 8 disparities per task
    for (int task = tid; task < kCX * (D / 8); task += NT) {
      const int i = task / (D / 8), d0 = (task % (D / 8)) * 8;
      const int x1c = min(max(c0 - 3 + i, 0), p.width1 - 1);
      const int kl = x1c + p.minX1 - xl0;
      const u16x2 u = as_v(sW[0][kl]), u0 = as_v(sW[1][kl]), u1 = as_v(sW[2][kl]);
      uint32_t out[4];
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        const int kr = kCX + kl + (D - 1) - (d0 + h);
        const u16x2 v = as_v(sW[0][kr]), v0 = as_v(sW[1][kr]), v1 = as_v(sW[2][kr]);
        const u16x2 cA = __builtin_elementwise_max(__builtin_elementwise_sub_sat(u, v1), __builtin_elementwise_sub_sat(v0, u));
        const u16x2 cB = __builtin_elementwise_max(__builtin_elementwise_sub_sat(v, u1), __builtin_elementwise_sub_sat(u0, v));
        const uint32_t m = as_u(vmin(cA, cB));
        const uint32_t cst = (m & 0xFFFFu) + (m >> 18);
        if (h & 1) out[h >> 1] |= cst << 16; else out[h >> 1] = cst;
      }
      *reinterpret_cast<uint4*>(&sPC[i][d0]) = make_uint4(out[0], out[1], out[2], out[3]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PQ; ++k) acc[k] = 0;
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const uint2* src = reinterpret_cast<const uint2*>(&sPC[col + t][q * DQ]);
#pragma unroll
      for (int k = 0; k < NV2; ++k) {
        const uint2 w2 = src[k];
        acc[2 * k] = as_u(as_v(acc[2 * k]) + as_v(w2.x));
        acc[2 * k + 1] = as_u(as_v(acc[2 * k + 1]) + as_v(w2.y));
      }
    }
    // no trailing barrier: the next row's first LDS write (sImg) comes after every thread
    // has passed this row's later barriers, i.e. finished reading sImg / sCh / sW / sPC
  };

  // window shift register: win[k] = hsum(clamp(y - 3 + k)), k = 0..6, for the output row y
  uint32_t win[7][PQ], crun[PQ], st[PQ];
  fetch(start);
  hs_row(win[6]);
  for (int r = start + 1; r <= start + 3; ++r) {
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int j = 0; j < PQ; ++j) win[k][j] = win[k + 1][j];
    if (r <= H - 1) {  // rows past H-1 clamp to H-1 (win[6] keeps it)
      fetch(r);
      hs_row(win[6]);
    }
  }
  // win[3..6] = hs(start..start+3 clamped); rows above start clamp to start
  if (start + 4 <= H - 1) fetch(start + 4);
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int j = 0; j < PQ; ++j) win[k][j] = win[3][j];
#pragma unroll
  for (int j = 0; j < PQ; ++j) {
    u16x2 a = as_v(win[0][j]) + as_v(win[1][j]) + as_v(win[2][j]) + as_v(win[3][j]);
    a = a + as_v(win[4][j]) + as_v(win[5][j]) + as_v(win[6][j]);
    crun[j] = as_u(a);
  }
#pragma unroll
  for (int k = 0; k < PQ; ++k) st[k] = 0;
  uint32_t minPrev = 0;
  const u16x2 P1 = splat(p.P1);
  const int x1 = c0 + col;
  const int64_t plane = (int64_t)p.width1 * D;
  const int64_t colofs = (int64_t)b * p.HG * 16 * plane + (int64_t)x1 * 16 * D + q * DQ;
  for (int y = start; y < end; ++y) {
    if (y > start) {  // window [y-3, y+3] clamped to [start, H-1]: out clamp(y-4), in clamp(y+3)
      uint32_t nw[PQ];
      if (y + 3 <= H - 1) {
        hs_row(nw);
        if (y + 4 <= H - 1) fetch(y + 4);
      } else {
#pragma unroll
        for (int j = 0; j < PQ; ++j) nw[j] = win[6][j];
      }
#pragma unroll
      for (int j = 0; j < PQ; ++j) crun[j] = as_u(as_v(crun[j]) - as_v(win[0][j]) + as_v(nw[j]));
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int j = 0; j < PQ; ++j) win[k][j] = win[k + 1][j];
#pragma unroll
      for (int j = 0; j < PQ; ++j) win[6][j] = nw[j];
    }
    minPrev = hstepG<PQ, G>(st, crun, q, P1, minPrev, p.P2);
    if (y >= first_out && x1 < p.width1) {
      const int64_t yo = (int64_t)(y >> 4) * 16 * plane + (y & 15) * D;
      uint2* cp = reinterpret_cast<uint2*>(Cvol + colofs + yo);
      uint2* vp = reinterpret_cast<uint2*>(Vvol + colofs + yo);
#pragma unroll
      for (int i = 0; i < NV2; ++i) {
        cp[i] = make_uint2(crun[2 * i], crun[2 * i + 1]);
        vp[i] = make_uint2(st[2 * i], st[2 * i + 1]);
      }
    }
  }
}

// ------------------------------------------------------------------ horizontal paths + WTA
// Quad of lanes per row (16 rows per wave).  raw is stored transposed, [x][row], so the rows
// of a wave are contiguous.  The right-view disparity of the pseudo left-right check is one
// 32-bit key per right-image column, (cost << 16) | (0xFFFF - x1), lowered by a
// fire-and-forget atomicMin: the smallest cost wins and, among equal costs, the largest x1 --
// the first one the right->left scan visits -- which is the serial rule "replace iff
// disp2cost > cost" of sgbm_ref.cpp; d + minD = x1 + minX1 - x2 is recovered from x1.  The
// scan therefore never waits on a load of its own (the old read-modify-write of the right-view
// cost drained every outstanding load once per column), and the volume loads of both passes
// run PF columns ahead.
template <int D, int PF, int G>
__global__ __launch_bounds__(64) void k_sg_horiz(const uint16_t* __restrict__ Cvol, const uint16_t* __restrict__ Vvol,
                                                 uint16_t* __restrict__ LVvol, int16_t* __restrict__ rawT,
                                                 uint32_t* __restrict__ keyT, SgParams p) {
  constexpr int DQ = D / G, PQ = DQ / 2, NV2 = DQ / 4;
  const int q = threadIdx.x % G;
  const int y = blockIdx.x * (64 / G) + threadIdx.x / G;
  const int b = blockIdx.y;
  const int H = p.H, W = p.W, n1 = p.width1;
  if (y >= H) return;  // whole quads leave together
  constexpr int64_t XS = 16 * D;  // x1 stride: the 16 rows of a group are interleaved per column
  const int64_t rowofs = ((int64_t)b * p.HG + (y >> 4)) * n1 * XS + (y & 15) * D + q * DQ;
  const uint16_t* Crow = Cvol + rowofs;
  const uint16_t* Vrow = Vvol + rowofs;
  uint16_t* LVrow = LVvol + rowofs;
  const u16x2 P1 = splat(p.P1);
  const int INVALID = (p.minD - 1) * 16;
  const int64_t colT = (int64_t)b * W * H + y;  // + x*H
  for (int x = q; x < W; x += G) {
    rawT[colT + (int64_t)x * H] = (int16_t)INVALID;
    keyT[colT + (int64_t)x * H] = 0xFFFFFFFFu;
  }
  uint32_t st[PQ], cb[PF][PQ], vb[PF][PQ];
  // ---- left -> right: LV = L + V
#pragma unroll
  for (int k = 0; k < PQ; ++k) st[k] = 0;
  uint32_t minPrev = 0;
#pragma unroll
  for (int j = 0; j < PF; ++j)
    if (j < n1) {
      load_run2<NV2>(Crow + (int64_t)j * XS, cb[j]);
      load_run2<NV2>(Vrow + (int64_t)j * XS, vb[j]);
    }
  for (int x0 = 0; x0 < n1; x0 += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int x1 = x0 + j;
      if (x1 < n1) {
        uint32_t c[PQ], v[PQ];
#pragma unroll
        for (int k = 0; k < PQ; ++k) { c[k] = cb[j][k]; v[k] = vb[j][k]; }
        if (x1 + PF < n1) {
          load_run2<NV2>(Crow + (int64_t)(x1 + PF) * XS, cb[j]);
          load_run2<NV2>(Vrow + (int64_t)(x1 + PF) * XS, vb[j]);
        }
        minPrev = hstepG<PQ, G>(st, c, q, P1, minPrev, p.P2);
        uint2* lp = reinterpret_cast<uint2*>(LVrow + (int64_t)x1 * XS);
#pragma unroll
        for (int i = 0; i < NV2; ++i)
          lp[i] = make_uint2(as_u(as_v(st[2 * i]) + as_v(v[2 * i])), as_u(as_v(st[2 * i + 1]) + as_v(v[2 * i + 1])));
      }
    }
  }
  // the initialisation stores above have completed before the quad leaders' atomics / stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // ---- right -> left, S = LV + R, first-minimum WTA, sub-pixel, right-view key
#pragma unroll
  for (int k = 0; k < PQ; ++k) st[k] = 0;
  minPrev = 0;
#pragma unroll
  for (int j = 0; j < PF; ++j)
    if (j < n1) {
      load_run2<NV2>(Crow + (int64_t)(n1 - 1 - j) * XS, cb[j]);
      load_run2<NV2>(LVrow + (int64_t)(n1 - 1 - j) * XS, vb[j]);
    }
  for (int i0 = 0; i0 < n1; i0 += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int i = i0 + j, x1 = n1 - 1 - i;
      if (i < n1) {
        uint32_t c[PQ], v[PQ];
#pragma unroll
        for (int k = 0; k < PQ; ++k) { c[k] = cb[j][k]; v[k] = vb[j][k]; }
        if (i + PF < n1) {
          load_run2<NV2>(Crow + (int64_t)(x1 - PF) * XS, cb[j]);
          load_run2<NV2>(LVrow + (int64_t)(x1 - PF) * XS, vb[j]);
        }
        minPrev = hstepG<PQ, G>(st, c, q, P1, minPrev, p.P2);
        // local first-minimum over this lane's run, with its S neighbours
        int best = 0x7FFFFFFF, bd = 0, sm1 = 0, sp1 = 0, prevv = 0;
        bool cap = false;
        uint32_t sFirst = 0, sLast = 0;
#pragma unroll
        for (int k = 0; k < PQ; ++k) {
          uint32_t S = as_u(as_v(v[k]) + as_v(st[k]));
          if (k == 0) sFirst = S & 0xFFFFu;
          if (k == PQ - 1) sLast = S >> 16;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            int sv = h ? (int)(S >> 16) : (int)(S & 0xFFFFu);
            if (cap) { sp1 = sv; cap = false; }
            if (sv < best) { best = sv; bd = 2 * k + h; sm1 = prevv; cap = true; }
            prevv = sv;
          }
        }
        const int fromPrev = G == 4 ? (int)qperm<kQPrev>(sLast) : __builtin_amdgcn_mov_dpp((int)sLast, 0x111, 0xF, 0xF, false);
        const int fromNext = G == 4 ? (int)qperm<kQNext>(sFirst) : __builtin_amdgcn_mov_dpp((int)sFirst, 0x101, 0xF, 0xF, false);
        if (bd == 0) sm1 = fromPrev;
        if (bd == DQ - 1) sp1 = fromNext;
        bd += q * DQ;
        // group reduction: smaller cost wins, ties go to the smaller disparity
#pragma unroll
        for (int r = 0; r < (G == 8 ? 3 : 2); ++r) {
          int ob, od, om, op;
          if (r == 0) {
            ob = (int)qperm<kQX1>(best); od = (int)qperm<kQX1>(bd); om = (int)qperm<kQX1>(sm1); op = (int)qperm<kQX1>(sp1);
          } else if (r == 1) {
            ob = (int)qperm<kQX2>(best); od = (int)qperm<kQX2>(bd); om = (int)qperm<kQX2>(sm1); op = (int)qperm<kQX2>(sp1);
          } else {  // row_half_mirror: the other quad of the 8 lanes
            ob = __builtin_amdgcn_mov_dpp(best, 0x141, 0xF, 0xF, false); od = __builtin_amdgcn_mov_dpp(bd, 0x141, 0xF, 0xF, false);
            om = __builtin_amdgcn_mov_dpp(sm1, 0x141, 0xF, 0xF, false); op = __builtin_amdgcn_mov_dpp(sp1, 0x141, 0xF, 0xF, false);
          }
          if (ob < best || (ob == best && od < bd)) { best = ob; bd = od; sm1 = om; sp1 = op; }
        }
        if (q == 0) {
          const int d = bd;
          const int x2 = x1 + p.minX1 - d - p.minD;
          if (x2 >= 0 && x2 < W && best < 0x7FFF)  // disp2cost starts at SHRT_MAX
            atomicMin(&keyT[colT + (int64_t)x2 * H], ((uint32_t)best << 16) | (uint32_t)(0xFFFF - x1));
          int dd;
          if (0 < d && d < D - 1) {
            int denom2 = max(sm1 + sp1 - 2 * best, 1);
            dd = d * 16 + ((sm1 - sp1) * 16 + denom2) / (denom2 * 2);
          } else {
            dd = d * 16;
          }
          rawT[colT + (int64_t)(x1 + p.minX1) * H] = (int16_t)(dd + p.minD * 16);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // ---- pseudo left-right consistency check, columns split over the quad; the keys are read
  // from L2 (the atomics were performed there)
  auto disp2 = [&](int x2) -> int {
    const uint32_t k = __hip_atomic_load(keyT + colT + (int64_t)x2 * H, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return k == 0xFFFFFFFFu ? INVALID : (int)(0xFFFFu - (k & 0xFFFFu)) + p.minX1 - x2;
  };
  for (int x = p.minX1 + q; x < p.minX1 + n1; x += G) {
    const int64_t ix = colT + (int64_t)x * H;
    const int d1 = rawT[ix];
    if (d1 == INVALID) continue;
    const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
    const int _x = x - _d, x_ = x - d_;
    if (0 <= x_ && x_ < W && 0 <= _x && _x < W) {
      const int a = disp2(x_), cc = disp2(_x);
      if (a >= p.minD && abs(a - d_) > p.disp12 && cc >= p.minD && abs(cc - _d) > p.disp12) rawT[ix] = (int16_t)INVALID;
    }
  }
}

// ------------------------------------------------------------------ median 3x3
__global__ void k_sg_median(const int16_t* __restrict__ rawT, int16_t* __restrict__ out, int W, int H) {
  int y = blockIdx.x * blockDim.x + threadIdx.x;  // rows contiguous in the transposed input
  int x = blockIdx.y, b = blockIdx.z;
  if (y >= H) return;
  const int16_t* s = rawT + (int64_t)b * W * H;
  int v[9];
  int k = 0;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      int yy = min(max(y + dy, 0), H - 1), xx = min(max(x + dx, 0), W - 1);
      v[k++] = s[(int64_t)xx * H + yy];
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
  p.HG = (c.height + 15) / 16;
  return p;
}

// Experiment / tuning knobs (read per launch): FVO_SG_G lanes per column in the cost pass
// (4 or 8), FVO_SG_CB columns per cost block (G=4: 32/64; G=8: 16/32), FVO_SG_HG lanes per
// row in the horizontal pass (4 or 8),
// FVO_SG_PF horizontal-pass prefetch depth (1/2/4), FVO_SG_CHUNKS batch chunks alternated
// over the caller's stream and a second stream (cost pass of one chunk overlaps the
// HBM-bound horizontal pass of the other).  All variants are bit-identical.
int env_int(const char* name, int def) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : def;
}

template <int D>
void launch_chunk(fvo_ctx* ctx, const SgParams& p, const uint8_t* L, const uint8_t* R, int nb, int64_t stride,
                  int pitch, uint16_t* C, uint16_t* V, uint16_t* LV, int16_t* raw, uint32_t* key, int16_t* disp,
                  int cb, int g, int pf, hipStream_t s) {
  const dim3 gcv((p.width1 + cb - 1) / cb, p.nstripes, nb);
  FVO_TIMED(ctx, KN_SG_VERT, s, {
    if (g == 8 && cb == 32) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_costvert<D, 32, 8>), gcv, dim3(256), 0, s, L, R, stride, pitch, p, C, V);
    else if (g == 8) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_costvert<D, 16, 8>), gcv, dim3(128), 0, s, L, R, stride, pitch, p, C, V);
    else if (cb == 32) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_costvert<D, 32, 4>), gcv, dim3(128), 0, s, L, R, stride, pitch, p, C, V);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_costvert<D, 64, 4>), gcv, dim3(256), 0, s, L, R, stride, pitch, p, C, V);
  });
  const int hg = env_int("FVO_SG_HG", 4);
  const dim3 ghz(hg == 8 ? (p.H + 7) / 8 : (p.H + 15) / 16, nb);
  FVO_TIMED(ctx, KN_SG_HORIZ, s, {
    if (hg == 8 && pf == 2) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_horiz<D, 2, 8>), ghz, dim3(64), 0, s, C, V, LV, raw, key, p);
    else if (hg == 8) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_horiz<D, 1, 8>), ghz, dim3(64), 0, s, C, V, LV, raw, key, p);
    else if (pf == 2) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_horiz<D, 2, 4>), ghz, dim3(64), 0, s, C, V, LV, raw, key, p);
    else if (pf == 4) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_horiz<D, 4, 4>), ghz, dim3(64), 0, s, C, V, LV, raw, key, p);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_horiz<D, 1, 4>), ghz, dim3(64), 0, s, C, V, LV, raw, key, p);
  });
  FVO_TIMED(ctx, KN_SG_MEDIAN, s, hipLaunchKernelGGL(k_sg_median, dim3((p.H + 255) / 256, p.W, nb), dim3(256), 0, s,
                                                     raw, disp, p.W, p.H));
}

template <int D>
void launch_sgbm(fvo_ctx* ctx, const SgParams& p, const uint8_t* L, const uint8_t* R, int batch, int64_t stride,
                 int pitch, int16_t* disp, hipStream_t s) {
  const int g = env_int("FVO_SG_G", 8), cb = env_int("FVO_SG_CB", g == 8 ? 32 : 64), pf = env_int("FVO_SG_PF", 1);
  const int nch = std::max(1, std::min(env_int("FVO_SG_CHUNKS", 1), batch));
  const int64_t vol = (int64_t)p.HG * 16 * p.width1 * D, img = (int64_t)p.H * p.W;
  if (nch > 1) {
    (void)hipEventRecord(ctx->sg_fork, s);
    (void)hipStreamWaitEvent(ctx->sg_s2, ctx->sg_fork, 0);
  }
  for (int k = 0; k < nch; ++k) {
    const int b0 = (int)((int64_t)batch * k / nch), b1 = (int)((int64_t)batch * (k + 1) / nch);
    if (b1 <= b0) continue;
    hipStream_t sk = (k & 1) ? ctx->sg_s2 : s;
    launch_chunk<D>(ctx, p, L + b0 * stride, R + b0 * stride, b1 - b0, stride, pitch, ctx->sg_L + b0 * vol,
                    ctx->sg_V + b0 * vol, ctx->sg_cost + b0 * vol, ctx->sg_raw + b0 * img, ctx->sg_d2 + b0 * img,
                    disp + b0 * img, cb, g, pf, sk);
  }
  if (nch > 1) {
    (void)hipEventRecord(ctx->sg_join, ctx->sg_s2);
    (void)hipStreamWaitEvent(s, ctx->sg_join, 0);
  }
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
  const int64_t B = c.sgbm_max_batch > 0 ? std::min(c.sgbm_max_batch, c.max_batch) : c.max_batch;
  const int64_t plane = (int64_t)p.width1 * p.D;
  int rc;
  // sg_L: C, sg_V: V, sg_cost: LV = L + V; each [B][HG][width1][16][D] u16
  const int64_t vol = (int64_t)p.HG * 16 * plane;
  if ((rc = fvo_alloc(ctx, &ctx->sg_cost, B * vol)) || (rc = fvo_alloc(ctx, &ctx->sg_L, B * vol)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_V, B * vol)) || (rc = fvo_alloc(ctx, &ctx->sg_raw, B * p.H * p.W)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_d2, B * p.H * p.W)))
    return rc;
  FVO_HIP(ctx, hipStreamCreateWithFlags(&ctx->sg_s2, hipStreamNonBlocking));
  FVO_HIP(ctx, hipEventCreateWithFlags(&ctx->sg_fork, hipEventDisableTiming));
  FVO_HIP(ctx, hipEventCreateWithFlags(&ctx->sg_join, hipEventDisableTiming));
  return 0;
}

int sgbm_run(fvo_ctx* ctx, const uint8_t* L, const uint8_t* R, int batch, int64_t image_stride, int pitch,
             int16_t* disp, hipStream_t s) {
  SgParams p = make_params(ctx->cfg);
  switch (p.D) {
    case 64: launch_sgbm<64>(ctx, p, L, R, batch, image_stride, pitch, disp, s); break;
    case 96: launch_sgbm<96>(ctx, p, L, R, batch, image_stride, pitch, disp, s); break;
    default: launch_sgbm<128>(ctx, p, L, R, batch, image_stride, pitch, disp, s); break;
  }
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
