// StereoSGBM (MODE_SGBM_3WAY) for gfx950 — replaces the disparity the reference computes in
// get_disparity_map (ros_ws/src/stereo_slam.py:108-117): numDisparities 96, minDisparity 0,
// blockSize 7, P1 392, P2 1568, 3-way aggregation, 4 fixed stripes, then medianBlur(3).
//
// One cost-volume-sized buffer crosses HBM per pair: the top-down path V, u16
// [HG4 + nstripes][x1][4][d] (4-row groups interleaved per column, so the 4 rows of a group at
// one column are 4*D*2 contiguous bytes and a wave of the row pass streams contiguous memory;
// x1 = x - max(maxD,0) in [0,width1), d in [0,D)); the extra nstripes groups hold, per stripe
// s > 0, the path's row first_out(s) - 1 (an overlap row the previous stripe outputs).  The
// 7x7 cost C is not stored: the recurrence V(y) = C(y) + min(V(y-1)[d], V(y-1)[d+-1] + P1,
// minV(y-1) + P2) - minV(y-1) is inverted exactly (u16 modular arithmetic) from V(y) and
// V(y-1), which the row pass reads anyway -- one volume write and two reads per pair instead
// of two writes and three reads.
// Kernels
//   k_sg_costvert<D,CB,G> block of CB columns (G lanes per column, D/G disparities per lane)
//                  marching down a stripe: BT pixel cost of both channels in one u16x2 word
//                  from LDS-staged rows, 7x7 box sum (7-column sum from LDS, 7-row running
//                  sum over a VGPR shift register, rows clamped to the stripe's first row and to
//                  H-1 -- the overlap rule of OpenCV's 4 stripes), fused with the top->down
//                  path; stores V
//   k_sg_rows<D>   wave per 4 rows (16 lanes per row, D/16 disparities per lane): C derived
//                  from V and the previous V row, left->right path over C storing its state
//                  every 8 columns (checkpoints), then segments of 8 columns right->left: the
//                  left->right path recomputed over the segment from its checkpoint, the
//                  right->left path, S = L + R + V, first-minimum WTA, integer sub-pixel,
//                  right-view keys by LDS atomicMin, the pseudo left-right check -- the L + V
//                  volume the forward pass would otherwise store and re-read never exists
//   k_sg_median    3x3 median (replicated border) -> int16 disparity*16
// Path states are packed u16x2 VGPRs (v_pk_add/sub/min_u16, v_alignbit for d-1 / d+1);
// neighbours across lanes come from DPP.  Integer arithmetic only; bit-identical to
// oracle/sgbm_ref.cpp.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "fvo_device.h"

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_v(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 vmin(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 splat(uint32_t s) { return as_v((s & 0xFFFFu) | (s << 16)); }
// (m + P2) in both halves for a path minimum m: one v_mad_u32_u24 (m * 0x10001 + P2 * 0x10001)
// instead of add + shift + and_or.  Exact: m <= 49 x the largest pixel cost + P2, so m + P2 <
// 3 (49 (2 ftzero + 63) + P2) <= 0xFFFF (sgbm_init) and no carry crosses the halves.
__device__ __forceinline__ u16x2 splat_p2(uint32_t m, uint32_t P2) { return as_v(__umul24(m, 0x10001u) + P2 * 0x10001u); }

struct SgParams {
  int W, H, D, minD, minX1, width1, P1, P2, ftzero, disp12, ss, ov, nstripes;
  int HG;   // row groups of 16
  int HG4;  // row groups of 4 (volume layout)
};

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

// min / or with a DPP-permuted copy of v: the permute's old value is the operation's identity,
// so the compiler folds the move into the VALU op (v_min_u32_dpp / v_or_b32_dpp)
template <int CTRL>
__device__ __forceinline__ uint32_t dmin(uint32_t v) {
  return min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dor(uint32_t v) {
  return v | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
// the value of a DPP-shifted lane, `old` where the shift has no source lane (row edges)
template <int CTRL>
__device__ __forceinline__ uint32_t dshift(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, 0xF, 0xF, false);
}

// the same with `edge` = the wanted value on the row's edge lane and 0 on the others: the shift
// reads 0 where it has no source (the old value), OR-ed with `edge` -- one v_or_b32_dpp instead
// of a move of the sentinel plus a DPP move
template <int CTRL>
__device__ __forceinline__ uint32_t dshift_or(uint32_t v, uint32_t edge) {
  return edge | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
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

template <int PQ>
__device__ __forceinline__ uint32_t step16(uint32_t* st, const uint32_t* c, int q, u16x2 P1, uint32_t minPrev,
                                           uint32_t P2);

// One step of a path over a lane's run with G lanes per column (G = 4: quad; G = 8: half
// row, neighbours by DPP row shifts, minimum by two quad steps + row_half_mirror; G = 16: a
// DPP row, step16); the path minimum in both u16 halves in and out, the step regrouped as
// step16's (below).
template <int PQ, int G>
__device__ __forceinline__ uint32_t hstepG(uint32_t* st, const uint32_t* c, int q, u16x2 P1, uint32_t mps,
                                           uint32_t P2) {
  if constexpr (G == 16) return step16<PQ>(st, c, q, P1, mps, P2);
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
  const u16x2 mpv = as_v(mps), p2 = splat(P2);
  u16x2 mn = splat(0xFFFF);
  uint32_t oldk = 0;
#pragma unroll
  for (int k = 0; k < PQ; ++k) {
    const uint32_t cur = st[k];
    const uint32_t lo = k > 0 ? oldk : lo0;
    const uint32_t hi = k < PQ - 1 ? st[k + 1] : hiN;
    const u16x2 dm = as_v(__builtin_amdgcn_alignbit(cur, lo, 16));
    const u16x2 dp = as_v(__builtin_amdgcn_alignbit(hi, cur, 16));
    const u16x2 A = vmin(vmin(dm, dp) + P1, as_v(cur));
    const u16x2 nv = vmin(A + as_v(c[k]) - mpv, as_v(c[k]) + p2);
    oldk = cur;
    st[k] = as_u(nv);
    mn = vmin(mn, nv);
  }
  uint32_t m = as_u(vmin(mn, __builtin_shufflevector(mn, mn, 1, 0)));
  m = dmin<kQX1>(m);
  m = dmin<kQX2>(m);
  if (G == 8) m = dmin<0x141>(m);  // row_half_mirror
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

// PQ packed words (4*PQ bytes) through a buffer descriptor: per-lane byte offset + a
// wave-uniform (SGPR) byte offset; out-of-range offsets read zeros.
template <int PQ>
__device__ __forceinline__ void bload(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint32_t* out) {
  if constexpr (PQ == 2) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
    out[0] = v[0]; out[1] = v[1];
  } else if constexpr (PQ == 3) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, voff, soff, 0);
    out[0] = v[0]; out[1] = v[1]; out[2] = v[2];
  } else {
    static_assert(PQ == 4, "D = 64, 96 or 128");
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
    out[0] = v[0]; out[1] = v[1]; out[2] = v[2]; out[3] = v[3];
  }
}

// ------------------------------------------------------------------ row bands: C + left/right paths + WTA
// A row of 16 lanes is one DPP row: neighbours by row_shr/row_shl:1, minima by quad xor 1/2,
// row_half_mirror and row_mirror.
constexpr int kRShr1 = 0x111;        // row_shr:1 -- value of lane i-1
constexpr int kRShl1 = 0x101;        // row_shl:1 -- value of lane i+1
constexpr int kRHalfMirror = 0x141;  // lane i <-> 7-i within each half row
constexpr int kRMirror = 0x140;      // lane i <-> 15-i

template <int CTRL>
__device__ __forceinline__ uint32_t rdpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

// Ring sizes of the row pass's LDS windows (powers of two): keys cover x2 over 2D + 4 SEG
// columns, raw disparities wait D + 2 SEG columns for their check.
__host__ __device__ constexpr int sg_pow2(int n) { return n <= 1 ? 1 : 2 * sg_pow2((n + 1) / 2); }
__host__ __device__ constexpr int sg_ring_keys(int D) { return sg_pow2(2 * D + 32); }
__host__ __device__ constexpr int sg_ring_raw(int D) { return sg_pow2(D + 16); }

// One path step of a 16-lane row (PQ packed words per lane).  The path minimum travels in both
// u16 halves (mps, and the returned row minimum), and the step is regrouped so that it sits
// two operations from the next state instead of five:
//   c + min(A, mp + P2) - mp  ==  min((A + c) - mp, c + P2),  A = min(min(dm, dp) + P1, cur)
// exact, not only modulo 2^16: A >= mp (every term is a state entry of the previous column or
// a sentinel, and mp is their minimum), and A + c <= Lmax + Cmax <= 2 Cmax + P2 < 0xFFFF by
// sgbm_init's bound (Cmax = 49 (2 ftzero + 63)), so neither side wraps and the min compares
// true values; min(dm + P1, dp + P1) = min(dm, dp) + P1 (no path value + P1 wraps, by the same
// bound).  A + c and c + P2 do not depend on mp.  The row minimum: the packed minimum of
// the words, its halves swapped and min-ed (both halves then hold it), four DPP steps as u32
// minima (a value splatted into both halves orders as u32 exactly as its u16) -- no split, and
// no splat before the next step.
template <int PQ>
__device__ __forceinline__ uint32_t step16(uint32_t* st, const uint32_t* c, int q, u16x2 P1, uint32_t mps,
                                           uint32_t P2) {
  // a row's lanes 0 / 15 have no left / right neighbour: the sentinel there
  const uint32_t lo0 = dshift_or<kRShr1>(st[PQ - 1], q == 0 ? kSent << 16 : 0u);
  const uint32_t hiN = dshift_or<kRShl1>(st[0], q == 15 ? kSent : 0u);
  const u16x2 mpv = as_v(mps), p2 = splat(P2);
  u16x2 mn = splat(0xFFFF);
  uint32_t oldk = 0;
#pragma unroll
  for (int k = 0; k < PQ; ++k) {
    const uint32_t cur = st[k];
    const uint32_t lo = k > 0 ? oldk : lo0;
    const uint32_t hi = k < PQ - 1 ? st[k + 1] : hiN;
    const u16x2 dm = as_v(__builtin_amdgcn_alignbit(cur, lo, 16));  // (prev[2k-1], prev[2k])
    const u16x2 dp = as_v(__builtin_amdgcn_alignbit(hi, cur, 16));  // (prev[2k+1], prev[2k+2])
    const u16x2 A = vmin(vmin(dm, dp) + P1, as_v(cur));
    const u16x2 nv = vmin(A + as_v(c[k]) - mpv, as_v(c[k]) + p2);
    oldk = cur;
    st[k] = as_u(nv);
    mn = vmin(mn, nv);
  }
  uint32_t m = as_u(vmin(mn, __builtin_shufflevector(mn, mn, 1, 0)));
  m = dmin<kQX1>(m);
  m = dmin<kQX2>(m);
  m = dmin<kRHalfMirror>(m);
  m = dmin<kRMirror>(m);
  return m;
}

template <int PQ>
__device__ __forceinline__ void vadd(uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int k = 0; k < PQ; ++k) a[k] = as_u(as_v(a[k]) + as_v(b[k]));
}

// C of one column from the top-down path: V(y) = C + min(Vp[d], Vp[d-1] + P1, Vp[d+1] + P1,
// min Vp + P2) - min Vp with Vp = V(y-1) of the same stripe's path (zero above its first
// row), so C = V(y) - (that minimum) + min Vp -- the cost pass's u16 arithmetic undone
// exactly (modular).  16 lanes per row as step16; m = min Vp (stored by the cost pass).
template <int PQ>
__device__ __forceinline__ void derive16(const uint32_t* vp, const uint32_t* v, uint32_t* c, uint32_t m, u16x2 P1,
                                         uint32_t P2, int q) {
  // a row's lanes 0 / 15 have no left / right neighbour: the sentinel there
  const uint32_t lo0 = dshift_or<kRShr1>(vp[PQ - 1], q == 0 ? kSent << 16 : 0u);
  const uint32_t hiN = dshift_or<kRShl1>(vp[0], q == 15 ? kSent : 0u);
  const u16x2 mp2 = splat_p2(m, P2), mpv = splat(m);
#pragma unroll
  for (int k = 0; k < PQ; ++k) {
    const uint32_t cur = vp[k];
    const uint32_t lo = k > 0 ? vp[k - 1] : lo0;
    const uint32_t hi = k < PQ - 1 ? vp[k + 1] : hiN;
    const u16x2 dm = as_v(__builtin_amdgcn_alignbit(cur, lo, 16));
    const u16x2 dp = as_v(__builtin_amdgcn_alignbit(hi, cur, 16));
    const u16x2 mm = vmin(vmin(dm, dp) + P1, vmin(as_v(cur), mp2));
    c[k] = as_u(as_v(v[k]) - mm + mpv);
  }
}

// ------------------------------------------------------------------ fused cost + vertical pass
// One block (G*CB threads) per (CB columns, stripe, pair), G lanes per column.  Per new hsum
// row (the row entering the 7-row window) the block stages the 3 image rows of its column
// range in LDS (left: CB+6 px, right: CB+6+D-1 px, +2 apron each side), derives the
// (x-Sobel, intensity) channel words and their BT min/max, evaluates the packed BT pixel
// cost of its (CB+6) x D cells into LDS (task slots laid out so neither the BT word reads nor
// the cost stores conflict on LDS banks) and box-sums 7 columns per lane.  The window's 7
// hsum rows are a shift register in VGPRs, so the hsum volume never goes to HBM.  The next
// row's image bytes are loaded right after the current row is staged and taken before the
// row's C / V stores (vmcnt retires in order: a wait for them behind the stores would also
// wait for the stores).  Integer arithmetic as oracle/sgbm_ref.cpp (order-independent sums).
// The left->right path (LP = true, fvo_config.sgbm_mode = FVO_SGBM_LPATH; classic is the default): the block also runs the L path of
// its CB columns -- per group of 4 output rows, one wave (16 lanes per row, D/16 disparities
// per lane) steps the 4 rows across the columns over C read back from a 4-row LDS ring, starting
// from the state the block of the previous column range handed over for those rows, stores the
// row pass's checkpoints and hands its own last state on (SgLink below).  The row pass then
// needs only its right->left sweep: one V read per pair fewer.
struct SgLink {
  uint32_t* ckpt;           // [B][H][nck][16][CKW] L checkpoints (the row pass's, per row)
  int nck, nk;              // checkpoint slots per row; column blocks per stripe
  uint64_t* hand;           // [B][H][2][PQ16][16] hand-off granules {tag, word}, by column-block parity
  uint32_t* ctl;            // [0] ticket, [1] generation, [2] timeouts, [4 + b] pair failed
  uint64_t deadline;        // bound on one hand-off wait, s_memrealtime ticks (100 MHz)
  int force_timeout;        // test hook (sgbm_handoff_us = -1): every hand-off times out
};

typedef __attribute__((address_space(1))) unsigned long long sg_gu64;
typedef __attribute__((address_space(1))) unsigned int sg_gu32;

// The L path of a group of nrows (<= 4) output rows y0.. of one column block (LP schedule), run
// by one wave while the block's other waves wait at a barrier (so at raised priority): lane = row
// r (4) x disparity run q (16 lanes, D/32 words each); C from the block's LDS ring (row y0 + r in
// slot s0 + r mod 4), the entering state from the previous column block's hand-off granules, the row pass's
// checkpoints, the leaving state handed on.  Not inlined:
// inlined into the cost pass's 7-way unrolled row loop its address arithmetic was hoisted and
// kept the whole kernel above 128 VGPRs (156 VGPRs / 3 waves per SIMD, or 33 spills at 128).
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;

// the granules of rows ya.. (nr rows) of column block kb - 1 from memory: one pass, no waiting
template <int PQ16>
__device__ __forceinline__ void sg_load_granules(const SgLink& lk, int b, int H, int kb, int ya, int nr, uint64_t* g) {
  const int lane = (int)(threadIdx.x & 63), rr = lane >> 4, qq = lane & 15;
  const int64_t hrow = ((int64_t)b * H + ya + min(rr, nr - 1)) * 2;
  sg_gu64* hp = (sg_gu64*)lk.hand + ((hrow + ((kb - 1) & 1)) * PQ16) * 16 + qq;
#pragma unroll
  for (int k = 0; k < PQ16; ++k) g[k] = __hip_atomic_load(hp + k * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int D, int CB>
__device__ __attribute__((noinline)) void sg_run_L(SgLink lk, lds_cu32* ring, int s0, int b, int H, int kb, int c0,
                                                   int width1, uint32_t gen, int y0, int nrows, uint32_t P1s, int P2) {
  // the arguments are wave-uniform: keep them (and the loop control) in SGPRs
  auto uni = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
  s0 = uni(s0), b = uni(b), H = uni(H), kb = uni(kb), c0 = uni(c0), width1 = uni(width1);
  gen = (uint32_t)uni((int)gen), y0 = uni(y0), nrows = uni(nrows), P1s = (uint32_t)uni((int)P1s), P2 = uni(P2);
  constexpr int PQ16 = D / 32;
  constexpr int CKW = PQ16 + 1 <= 4 ? 4 : 8;
  constexpr int RW = CB * D / 2 + 16;
  __builtin_amdgcn_s_setprio(3);
  const u16x2 P1 = splat(P1s);
  const int lane = (int)(threadIdx.x & 63);
  const int rr = lane >> 4, qq = lane & 15;
  const int yr = y0 + min(rr, nrows - 1);  // lanes of missing rows repeat the last row (no stores)
  const bool live = rr < nrows;
  uint32_t lst[PQ16];
  uint32_t lmin = 0;
  const int64_t hrow = ((int64_t)b * H + yr) * 2;
  if (kb == 0) {
#pragma unroll
    for (int g = 0; g < PQ16; ++g) lst[g] = 0;  // the path starts at x1 = 0 from the zero state
  } else {
    // granules {tag, word} of the previous column block (the data is its own flag: no fence,
    // no ordering): re-read until every tag is (generation, kb - 1)
    const uint32_t tag = (gen << 7) | (uint32_t)(kb - 1);
    uint64_t gv[PQ16];
    sg_load_granules<PQ16>(lk, b, H, kb, y0, nrows, gv);
    uint64_t t0 = 0;
    const bool force = __builtin_amdgcn_readfirstlane(lk.force_timeout) != 0;
    for (int it = 0;; ++it) {
      bool ok = !force;
#pragma unroll
      for (int g = 0; g < PQ16; ++g) {
        lst[g] = (uint32_t)gv[g];
        ok &= (uint32_t)(gv[g] >> 32) == tag;
      }
      if (__all(ok)) break;
      // bounded wait: past the deadline (and at least 64 polls, so one long preemption of the
      // queue -- the clock runs while the waves are suspended -- cannot end a wait on its first
      // re-check), or once the pair is marked failed upstream, give up: mark the pair failed (its
      // disparities come out invalid, fvo_sgbm's status says so) and count the timeout
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (it == 0) t0 = now;
      const bool failed = __hip_atomic_load((sg_gu32*)lk.ctl + 4 + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      if (failed || force || (it >= 64 && now - t0 > lk.deadline)) {
        if (lane == 0 && !failed) {
          __hip_atomic_fetch_or((sg_gu32*)lk.ctl + 4 + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add((sg_gu32*)lk.ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int g = 0; g < PQ16; ++g) lst[g] = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      sg_load_granules<PQ16>(lk, b, H, kb, y0, nrows, gv);
    }
    // the state's minimum over d (the next step's minPrev)
    uint32_t m = 0xFFFFFFFFu;
#pragma unroll
    for (int g = 0; g < PQ16; ++g) m = min(m, min(lst[g] & 0xFFFFu, lst[g] >> 16));
    m = dmin<kQX1>(m);
    m = dmin<kQX2>(m);
    m = dmin<kRHalfMirror>(m);
    m = dmin<kRMirror>(m);
    lmin = m | (m << 16);  // step16's minimum travels in both halves
  }
  const int nx = min(CB, width1 - c0);
  // checkpoints after the columns x1 = W1 - 9 - 8 m (m >= 0): the row pass's segment m starts there
  const int i0 = (((width1 - 9 - c0) % 8) + 8) % 8;
  uint32_t* ckrow = lk.ckpt + (((int64_t)b * H + yr) * lk.nck * 16 + qq) * CKW;
  lds_cu32* rbase = ring + ((s0 + rr) & 3) * RW + qq * PQ16;  // row y0 + r sits in ring slot s0 + r
  uint32_t c[PQ16];
#pragma unroll
  for (int g = 0; g < PQ16; ++g) c[g] = rbase[g];
#pragma unroll 1
  for (int i = 0; i < nx; ++i) {
    uint32_t cn[PQ16];  // the next column's C, read one step ahead
    const int in = min(i + 1, CB - 1);
#pragma unroll
    for (int g = 0; g < PQ16; ++g) cn[g] = rbase[in * (D / 2) + g];
    lmin = step16<PQ16>(lst, c, qq, P1, lmin, P2);
    if (((i - i0) & 7) == 0 && c0 + i <= width1 - 9 && live) {
      const int slot = (width1 - 9 - (c0 + i)) >> 3;
      uint32_t v[CKW];
#pragma unroll
      for (int g = 0; g < CKW; ++g) v[g] = g < PQ16 ? lst[g] : g == PQ16 ? lmin : 0u;
      sg_gu32* cp = (sg_gu32*)(ckrow + (int64_t)slot * 16 * CKW);  // global, not flat, stores
#pragma unroll
      for (int g = 0; g < CKW; ++g) cp[g] = v[g];
    }
#pragma unroll
    for (int g = 0; g < PQ16; ++g) c[g] = cn[g];
  }
  if (kb < lk.nk - 1 && live) {
    const uint64_t tag = (uint64_t)((gen << 7) | (uint32_t)kb) << 32;
    sg_gu64* hp = (sg_gu64*)lk.hand + ((hrow + (kb & 1)) * PQ16) * 16 + qq;
#pragma unroll
    for (int g = 0; g < PQ16; ++g) __hip_atomic_store(hp + g * 16, tag | lst[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __builtin_amdgcn_s_setprio(0);
}

template <int D, int CB, int G, bool LP>
__global__ __launch_bounds__(G * CB, LP ? 4 : (G == 16 && D <= 96 ? 6 : (G == 8 ? (D <= 96 ? 4 : 3) : 1))) void k_sg_costvert(const uint8_t* __restrict__ Limg, const uint8_t* __restrict__ Rimg,
                                                    int64_t stride, int pitch, SgParams p, uint16_t* __restrict__ Vvol,
                                                    uint16_t* __restrict__ Mvol, SgLink lk) {
  constexpr int DQ = D / G, PQ = DQ / 2, NV2 = DQ / 4;  // NV2 = 0: a run of 6 (G = 16) moves as words
  constexpr int NT = G * CB;                // threads: G lanes per column
  constexpr int kCX = CB + 6;               // pixel-cost columns (7-wide box apron)
  constexpr int NRC = kCX + D - 1;          // right-image core pixels
  constexpr int NLI = kCX + 4, NRI = NRC + 4;  // staged pixels per image row (core + 2 each side)
  constexpr int NIMG = NLI + NRI;           // staged bytes per image row
  constexpr int PER = (NIMG + NT - 1) / NT;  // staged bytes per thread
  constexpr int PQ16 = D / 32;              // L path: packed words per lane (16 lanes per row)
  constexpr int CKW = PQ16 + 1 <= 4 ? 4 : 8;
  // C ring of the L path: 4 rows x CB columns x D/2 words, the row stride = 16 mod 32 words so
  // the 4 rows' lanes (3 words apart within a row) hit disjoint banks
  constexpr int RW = LP ? CB * D / 2 + 16 : 1;
  __shared__ uint8_t sImg[4][NLI + NRI];                            // image rows (ring by row & 3), L then R
  // per hsum row of a call (two per call in the classic schedule, one under LP)
  constexpr int NRS = LP ? 1 : 2;
  __shared__ uint32_t sCh[NRS][kCX + 2 + NRC + 2];                  // (Sobel, intensity), L then R
  __shared__ uint32_t sU[NRS][6][kCX];                             // left BT words per channel (splat)
  __shared__ uint32_t sV[NRS][6][NRC];                             // right BT words per channel (pixel pairs)
  __shared__ __attribute__((aligned(16))) uint16_t sPC[NRS][kCX][D];  // pixel cost
  __shared__ uint32_t sRing[LP ? 4 : 1][RW];
  __shared__ int sUnit;
  const int tid = threadIdx.x, lane = tid & 63, q = lane % G;
  const int col = (tid >> 6) * (64 / G) + lane / G;  // 0..CB-1
  int c0, s, b, kb;
  if constexpr (LP) {
    // units (column block k, pair b, stripe s) in ticket order, k major: the block that hands
    // this one its L states took its ticket nchains tickets earlier, so it is running or done
    // whatever the dispatch order (no deadlock), and usually far enough ahead that nobody waits
    if (tid == 0) sUnit = (int)atomicAdd(lk.ctl, 1u);
    __syncthreads();
    const int nch = (int)gridDim.x / lk.nk;
    const int t = sUnit;
    kb = t / nch;
    const int ch = t - kb * nch;
    b = ch / p.nstripes;
    s = ch - b * p.nstripes;
    c0 = kb * CB;
  } else {
    const XcdBlock xb = xcd_block();  // neighbouring column blocks (shared image rows) on one XCD
    c0 = xb.x * CB;
    s = xb.y, b = xb.z, kb = xb.x;
  }
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

  // ---- image rows: a 4-slot LDS ring (slot = image row & 3) of the block's core columns (+2 each
  // side) of both images; hsum row r reads rows r-1, r, r+1 (clamped), so each new hsum row stages
  // one new image row, loaded one call ahead into registers (one byte per thread and row; up to
  // two rows wait, A and B, for a two-row call)
  const uint8_t* colsrc[PER];  // this thread's bytes of a staged row (clamped columns)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int jb = min(tid + NT * k, NIMG - 1);
    colsrc[k] = jb < NLI ? Lb + min(max(xl0 - 2 + jb, 0), W - 1) : Rb + min(max(xr0 - 2 + (jb - NLI), 0), W - 1);
  }
  uint32_t preA[PER], preB[PER];
  int pendA = -1, pendB = -1;  // image rows waiting in preA / preB (-1: none)
  int hi = -1;                 // the highest image row in the ring or waiting
  auto put_row = [&](const uint32_t* pr, int row) {
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (tid + NT * k < NIMG) sImg[row & 3][tid + NT * k] = (uint8_t)pr[k];
  };
  auto load_row = [&](uint32_t* pr, int row) {
#pragma unroll
    for (int k = 0; k < PER; ++k) pr[k] = colsrc[k][(int64_t)row * pitch];
  };
  // a call's staging: the waiting rows into the ring, then the rows up to `upto` (<= 2 of them)
  // loaded for the next call.  A call for hsum rows e.. (NR of them) needs image rows up to e + NR
  // and loads up to e + NR + 2, so the next call -- one or two rows -- finds its rows waiting, and
  // the ring (the 4 most recent rows) still holds row e + NR - 2, the first one it reads
  auto stage = [&](int upto) {
    if (pendA >= 0) put_row(preA, pendA);
    if (pendB >= 0) put_row(preB, pendB);
    pendA = pendB = -1;
    upto = min(upto, H - 1);
    if (hi + 1 <= upto) { load_row(preA, hi + 1); pendA = ++hi; }
    if (hi + 1 <= upto) { load_row(preB, hi + 1); pendB = ++hi; }
  };
  // ---- per-thread pixel-cost tasks (8 disparities of one column each), fixed for the block:
  // left word index kl, right pair index of the first disparity pair, output offset
  constexpr int NDB = D / 32;
  constexpr int NSLOT = ((kCX + 7) / 8) * NDB * 32;
  constexpr int NTASK = (NSLOT + NT - 1) / NT;
  int tk_kl[NTASK], tk_jr[NTASK], tk_out[NTASK];
#pragma unroll
  for (int m = 0; m < NTASK; ++m) {
    const int t = tid + NT * m;
    const int g = t >> 5, w = t & 31;
    const int i = (g / NDB) * 8 + (w >> 2), d0 = ((g % NDB) * 4 + (w & 3)) * 8;
    const int x1c = min(max(c0 - 3 + i, 0), p.width1 - 1);
    tk_kl[m] = x1c + p.minX1 - xl0;
    tk_jr[m] = tk_kl[m] + (D - 1) - d0;  // right pixel of disparity d0 (pairs: d0 + 2j at tk_jr - 2j)
    tk_out[m] = (t < NSLOT && i < kCX) ? i * D + d0 : -1;
  }
  // hsum rows e .. e + NR - 1 (rows past H - 1 clamp to it) from the ring -> acc0 (, acc1): this
  // lane's column and disparity run.  NR = 2 (classic schedule): two rows per phase, one barrier
  // per phase for both (r6: 4 barriers per two rows instead of per row)
  auto hs_rows = [&](auto nr_t, uint32_t* acc0, uint32_t* acc1, int e) {
    constexpr int NR = decltype(nr_t)::value;
    stage(e + NR + 2);
    __syncthreads();
    // channel words at core-1 .. core+1 of both images; borders (x < 1, x >= W-1) read ftzero
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int r = min(e + rr, H - 1);
      const uint8_t* r0 = sImg[(r > 0 ? r - 1 : r) & 3];
      const uint8_t* r1 = sImg[r & 3];
      const uint8_t* r2 = sImg[(r < H - 1 ? r + 1 : r) & 3];
      for (int j = tid; j < (nl + 2) + (nr + 2); j += NT) {
        const bool left = j < nl + 2;
        const int k = left ? j : j - (nl + 2);
        const int x = (left ? xl0 : xr0) - 1 + k;
        const int jj = k + 1 + (left ? 0 : NLI);
        uint32_t wv = (uint32_t)clip(0) * 0x10001u;
        if (x >= 1 && x < W - 1) {
          const int sb = (r1[jj + 1] - r1[jj - 1]) * 2 + r0[jj + 1] - r0[jj - 1] + r2[jj + 1] - r2[jj - 1];
          wv = (uint32_t)clip(sb) | ((uint32_t)r1[jj] << 16);
        }
        sCh[rr][left ? k : (kCX + 2) + k] = wv;
      }
    }
    __syncthreads();
    // BT words per channel c (lo half: x-Sobel, hi: intensity): value, min(u, (u+ul)/2, (u+ur)/2),
    // max(...) (at x = 0 / W-1 the half is u itself).  Left pixels as splat words (both halves
    // the pixel's), right pixels as pairs (pixel k, pixel k-1): a pixel-cost word then holds
    // disparities (d, d+1) of one column, both from one packed operation
    auto btw = [&](const uint32_t* ch, int k, int x, u16x2& u, u16x2& mn, u16x2& mx) {
      u = as_v(ch[k + 1]);
      u16x2 hl = (u + as_v(ch[k])) >> 1, hr = (u + as_v(ch[k + 2])) >> 1;
      if (x == 0) hl = u;
      if (x == W - 1) hr = u;
      mn = vmin(vmin(hl, hr), u);
      mx = __builtin_elementwise_max(__builtin_elementwise_max(hl, hr), u);
    };
#pragma unroll
    for (int rr = 0; rr < NR; ++rr)
    for (int j = tid; j < nl + nr; j += NT) {
      const bool left = j < nl;
      const int k = left ? j : j - nl;
      const int x = left ? xl0 + k : xr0 + k;
      const uint32_t* ch = left ? sCh[rr] : sCh[rr] + (kCX + 2);
      u16x2 u, mn, mx;
      btw(ch, k, x, u, mn, mx);
      if (left) {
        const u16x2 w3[3] = {u, mn, mx};
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 3; ++e) sU[rr][3 * c + e][k] = as_u(splat(c ? as_u(w3[e]) >> 16 : as_u(w3[e])));
      } else if (k > 0) {
        u16x2 up, mnp, mxp;  // the right pixel k - 1
        btw(ch, k - 1, x - 1, up, mnp, mxp);
        const uint32_t a3[3] = {as_u(u), as_u(mn), as_u(mx)}, b3[3] = {as_u(up), as_u(mnp), as_u(mxp)};
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          sV[rr][e][k] = (a3[e] & 0xFFFFu) | (b3[e] << 16);             // x-Sobel (k, k-1)
          sV[rr][3 + e][k] = (a3[e] >> 16) | (b3[e] & 0xFFFF0000u);     // intensity (k, k-1)
        }
      }
    }
    __syncthreads();
    // pixel costs of the kCX (clamped) columns x D disparities, 8 disparities per task, two per
    // packed operation: cost = BT(x-Sobel) + (BT(intensity) >> 2)
#pragma unroll
    for (int rr = 0; rr < NR; ++rr)
#pragma unroll
    for (int m = 0; m < NTASK; ++m) {
      if (tk_out[m] < 0) continue;
      const int kl = tk_kl[m];
      u16x2 uu[6];
#pragma unroll
      for (int e = 0; e < 6; ++e) uu[e] = as_v(sU[rr][e][kl]);
      uint32_t out[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int jr = tk_jr[m] - 2 * h;
        u16x2 mc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const u16x2 v = as_v(sV[rr][3 * c][jr]), v0 = as_v(sV[rr][3 * c + 1][jr]), v1 = as_v(sV[rr][3 * c + 2][jr]);
          const u16x2 u = uu[3 * c], u0 = uu[3 * c + 1], u1 = uu[3 * c + 2];
          const u16x2 cA = __builtin_elementwise_max(__builtin_elementwise_sub_sat(u, v1), __builtin_elementwise_sub_sat(v0, u));
          const u16x2 cB = __builtin_elementwise_max(__builtin_elementwise_sub_sat(v, u1), __builtin_elementwise_sub_sat(u0, v));
          mc[c] = vmin(cA, cB);
        }
        out[h] = as_u(mc[0] + (mc[1] >> 2));
      }
      *reinterpret_cast<uint4*>(&sPC[rr][0][0] + tk_out[m]) = make_uint4(out[0], out[1], out[2], out[3]);
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      uint32_t* acc = rr == 0 ? acc0 : acc1;
#pragma unroll
      for (int k = 0; k < PQ; ++k) acc[k] = 0;
#pragma unroll
      for (int t = 0; t < 7; ++t) {
        if constexpr (DQ % 4 == 0) {
          const uint2* src = reinterpret_cast<const uint2*>(&sPC[rr][col + t][q * DQ]);
#pragma unroll
          for (int k = 0; k < NV2; ++k) {
            const uint2 w2 = src[k];
            acc[2 * k] = as_u(as_v(acc[2 * k]) + as_v(w2.x));
            acc[2 * k + 1] = as_u(as_v(acc[2 * k + 1]) + as_v(w2.y));
          }
        } else {
          const uint32_t* src = reinterpret_cast<const uint32_t*>(&sPC[rr][col + t][q * DQ]);
#pragma unroll
          for (int k = 0; k < PQ; ++k) acc[k] = as_u(as_v(acc[k]) + as_v(src[k]));
        }
      }
    }
    // no trailing barrier: the next call's first LDS writes (its image rows, into ring slots no
    // phase still running reads -- those finished before this call's third barrier) come before
    // its first barrier, and every later write after it
  };
  const std::integral_constant<int, 1> one{};
  const std::integral_constant<int, 2> two{};

  // window: win[k] = hsum(clamp(start - 3 + k)), k = 0..6, for the output row start
  uint32_t win[7][PQ], crun[PQ], st[PQ];
  // the first hsum row's image rows (start - 1, start, start + 1, clamped) straight into the ring
  hi = min(start + 1, H - 1);
  for (int row = max(start - 1, 0); row <= hi; ++row) {
    load_row(preA, row);
    put_row(preA, row);
  }
  hs_rows(one, win[6], nullptr, start);
  for (int r = start + 1; r <= start + 3; ++r) {
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int j = 0; j < PQ; ++j) win[k][j] = win[k + 1][j];
    if (r <= H - 1) hs_rows(one, win[6], nullptr, r);
  }
  // win[3..6] = hs(start..start+3 clamped); rows above start clamp to start
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
  const int64_t colofs = (int64_t)b * (p.HG4 + p.nstripes) * 4 * plane + (int64_t)x1 * 4 * D + q * DQ;
  const uint32_t gen = LP ? lk.ctl[1] : 0u;
  // V step + stores of output row y
  auto vrow = [&](int y) {
    minPrev = hstepG<PQ, G>(st, crun, q, P1, minPrev, p.P2);
#pragma unroll
    for (int k = 0; k < PER; ++k) asm volatile("" : "+v"(preA[k]), "+v"(preB[k]) :: "memory");
    // output rows, and for s > 0 the row above the stripe's first output row (the row pass
    // inverts the recurrence at first_out from it): group HG4 + s, sub-row 0
    const bool out_row = y >= first_out, top_row = s > 0 && y == first_out - 1;
    if ((out_row || top_row) && x1 < p.width1) {
      const int64_t yo = out_row ? (int64_t)(y >> 2) * 4 * plane + (y & 3) * D : (int64_t)(p.HG4 + s) * 4 * plane;
      if constexpr (DQ % 4 == 0) {
        uint2* vp = reinterpret_cast<uint2*>(Vvol + colofs + yo);
#pragma unroll
        for (int i = 0; i < NV2; ++i) {
          typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
          __builtin_nontemporal_store(u32x2{st[2 * i], st[2 * i + 1]}, reinterpret_cast<u32x2*>(vp + i));
        }
      } else {
        uint32_t* vp = reinterpret_cast<uint32_t*>(Vvol + colofs + yo);
#pragma unroll
        for (int i = 0; i < PQ; ++i) __builtin_nontemporal_store(st[i], vp + i);
      }
      // min over d of this V row (the next row's minPrev): the row pass's inversion needs it
      if (q == 0) Mvol[(colofs - q * DQ + yo) / D] = (uint16_t)minPrev;
    }
    if constexpr (LP) {
      if (out_row) {
        // groups of 4 rows at a phase of their own per column block (kb & 3), so the blocks
        // sharing a CU -- which otherwise run in lockstep -- do not all wait for their L waves at once
        const int yi = y - first_out + (kb & 3);
        uint32_t* rp = &sRing[yi & 3][col * (D / 2) + q * PQ];
#pragma unroll
        for (int k = 0; k < PQ; ++k) rp[k] = crun[k];
        if ((yi & 3) == 3 || y == end - 1) {  // a complete group (or the stripe's last rows)
          __syncthreads();
          const int y0 = max(first_out, y - (yi & 3));
          if ((tid >> 6) == ((yi >> 2) & 3))
            sg_run_L<D, CB>(lk, (lds_cu32*)&sRing[0][0], (y0 - first_out + (kb & 3)) & 3, b, H, kb, c0, p.width1, gen, y0,
                            y - y0 + 1, (uint32_t)p.P1, p.P2);
          __syncthreads();  // the ring is rewritten from the next row on
        }
      }
    }
  };
  vrow(start);
  // rows start+1, ...: the 7-row window is a ring -- row y = start + t replaces slot (t-1) mod 7
  // (the row leaving, y-4) by the row entering (y+3); the loop is unrolled by 7 (pairs of rows:
  // 14) so every slot index is static (no register shuffling).  Below H-1 the entering row is
  // clamped, i.e. the last one entered (slot (t-2) mod 7).
  auto enter = [&](int ph, const uint32_t* nw) {
#pragma unroll
    for (int j = 0; j < PQ; ++j) {
      crun[j] = as_u(as_v(crun[j]) - as_v(win[ph][j]) + as_v(nw[j]));
      win[ph][j] = nw[j];
    }
  };
  if constexpr (!LP) {
    // two output rows per step: their entering hsum rows y + 3, y + 4 from one two-row call (the
    // second clamps to H - 1 when past it; a call at or past H - 1 is not needed)
#pragma unroll 1
    for (int y0 = start + 1; y0 < end; y0 += 14) {
#pragma unroll
      for (int pp = 0; pp < 7; ++pp) {
        const int y = y0 + 2 * pp;
        if (y >= end) break;
        const int ph0 = (2 * pp) % 7, ph1 = (2 * pp + 1) % 7;
        uint32_t nw0[PQ], nw1[PQ];
        if (y + 3 <= H - 1) {
          hs_rows(two, nw0, nw1, y + 3);
        } else {
#pragma unroll
          for (int j = 0; j < PQ; ++j) nw0[j] = nw1[j] = win[(ph0 + 6) % 7][j];
        }
        enter(ph0, nw0);
        vrow(y);
        if (y + 1 >= end) break;
        enter(ph1, nw1);
        vrow(y + 1);
      }
    }
  } else {
#pragma unroll 1
    for (int y0 = start + 1; y0 < end; y0 += 7) {
#pragma unroll
      for (int ph = 0; ph < 7; ++ph) {
        const int y = y0 + ph;
        if (y >= end) break;
        uint32_t nw[PQ];
        if (y + 3 <= H - 1) {
          hs_rows(one, nw, nullptr, y + 3);
        } else {
#pragma unroll
          for (int j = 0; j < PQ; ++j) nw[j] = win[(ph + 6) % 7][j];
        }
        enter(ph, nw);
        vrow(y);
      }
    }
  }
}

// Wave per 4 rows (one block), 16 lanes per row, D/16 disparities per lane.  Sweep 1 walks
// the row left->right over C (prefetched PF columns ahead) running the L path and storing
// its state (+ minimum) every SEG columns -- at x = W1-1-SEG*(s+1), the left neighbour of sweep
// 2's segment s.  Sweep 2 walks segments of SEG columns right->left (double-buffered C and V
// loads one segment ahead): L recomputed forward over the segment from its checkpoint, then
// the R path, S = L + R + V, first-minimum WTA as one u32 min of (S << 8 | d) across the
// row's lanes, integer sub-pixel, and the right-view key (cost << 16 | 0xFFFF - x1) lowered
// by an LDS atomicMin -- the serial rule "replace iff disp2cost > cost" of sgbm_ref.cpp (the
// smallest cost wins, among equal costs the largest x1, the first one the scan visits).  The
// pseudo left-right check then runs on the LDS row and writes the row-major raw disparity.
// SW: kSwBoth = both sweeps (checkpoints per 4-row block: [B][row blocks][nck][64 lanes][CKW]);
// kSwRight = sweep 2 only, over the per-row checkpoints ([B][H][nck][16 lanes][CKW]) the L-path
// cost pass stored.  (r5, measured and not kept: sweep 1 as a launch of its own, kSwLeft, per chunk
// of pairs on a second stream beside the next chunk's cost pass -- bit-exact, 8.1-8.4 vs 8.1-8.2 ms:
// the cost pass slowed by what sweep 1 cost.)
constexpr int kSwBoth = 0, kSwRight = 1, kSwLeft = 2;
template <int D, int SW>
__global__ __launch_bounds__(64, D <= 96 ? 4 : 2) void k_sg_rows(const uint16_t* __restrict__ Vvol,
                                                                 const uint16_t* __restrict__ Mvol, SgParams p,
                                                                 uint32_t* __restrict__ ckpt, int nck,
                                                                 int16_t* __restrict__ raw) {
  constexpr int DQ = D / 16, PQ = DQ / 2, SEG = 8, PF = 8, PD = 4;  // PD: prefetch distance (measured 2/4/8)
  constexpr int CKW = PQ + 1 <= 4 ? 4 : 8;
  constexpr int XS = 2 * D;  // u32 words per column of a 4-row group
  constexpr int RK = sg_ring_keys(D), RS = sg_ring_raw(D);
  constexpr bool S1 = SW != kSwRight, S2 = SW != kSwLeft;
  __shared__ uint32_t s_key[4][S2 ? RK : 1];  // right-view keys of the live x2 window (ring, by x2)
  __shared__ __attribute__((aligned(16))) uint16_t s_S[4][S2 ? D : 2];  // one column's S of each row (WTA neighbours)
  __shared__ int16_t s_raw[4][S2 ? RS : 2];   // raw disparities awaiting their check (ring, by x1)
  const int lane = threadIdx.x, q = lane & 15, r = lane >> 4;
  // consecutive row groups on one XCD: a group's first row reads the previous group's last
  // V row, which that group's wave streams at about the same time (an L2 hit)
  const XcdBlock xb = xcd_block();
  const int blk = xb.x, b = xb.y;
  const int y = blk * 4 + r;
  const int H = p.H, W = p.W, W1 = p.width1;
  const bool rowok = y < H;
  const int yy = min(y, H - 1);  // rows past H walk the last row's volumes (never output)
  uint32_t* key = s_key[r];
  int16_t* sraw = s_raw[r];
  const int INVALID = (p.minD - 1) * 16;
  int16_t* out = raw + ((int64_t)b * H + yy) * W;
  if constexpr (S2) {
    for (int k = q; k < RK; k += 16) key[k] = 0xFFFFFFFFu;
    if (rowok)  // columns left of the first x1 (and right of the last) never get a disparity
      for (int x = q; x < W; x += 16)
        if (x < p.minX1 || x >= p.minX1 + W1) out[x] = (int16_t)INVALID;
  }
  // pseudo left-right check of pixel x1 (its right-view keys are final once the sweep has
  // passed x1 - D: every x2 it reads lies within D of x1 + minX1 - minD)
  auto disp2 = [&](int x2) -> int {
    const uint32_t kv = key[x2 & (RK - 1)];
    return kv == 0xFFFFFFFFu ? INVALID : (int)(0xFFFFu - (kv & 0xFFFFu)) + p.minX1 - x2;
  };
  auto checked = [&](int x1) -> int {
    const int x = x1 + p.minX1;
    int d1 = sraw[x1 & (RS - 1)];
    if (d1 != INVALID) {
      const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
      const int _x = x - _d, x_ = x - d_;
      if (0 <= x_ && x_ < W && 0 <= _x && _x < W) {
        const int a = disp2(x_), cc = disp2(_x);
        if (a >= p.minD && abs(a - d_) > p.disp12 && cc >= p.minD && abs(cc - _d) > p.disp12) d1 = INVALID;
      }
    }
    return d1;
  };
  auto check = [&](int x1) {
    const int d1 = checked(x1);
    if (rowok) out[x1 + p.minX1] = (int16_t)d1;
  };
  // lanes with no pixel to check store into this lane's words of the dummy checkpoint slot, so
  // every segment issues the same global stores: with a conditional store the compiler's vmcnt
  // bookkeeping falls back to draining every load in flight at the next segment
  // (S1 layout: [B][row blocks][nck][64 lanes][CKW]; per-row layout: [B][H][nck][16 lanes][CKW])
  auto ckptr = [&](int slot) -> uint32_t* {
    return SW == kSwBoth ? ckpt + ((((int64_t)b * gridDim.x + blk) * nck + slot) * 64 + lane) * CKW
              : ckpt + ((((int64_t)b * H + yy) * nck + slot) * 16 + q) * CKW;
  };
  int16_t* const sink = reinterpret_cast<int16_t*>(ckptr(nck - 1));
  int next_chk = W1 - 1;  // highest pixel not yet checked
  // V of this row and of the previous row of the same stripe's path: inside the stripe the
  // row above, at its first output row (s > 0) the overlap row the cost pass kept in group
  // HG4 + s, above row 0 nothing (a zero state: C = V there)
  const int64_t plane4 = (int64_t)W1 * (4 * D);  // u16 per 4-row group
  const int stripe = yy / p.ss;
  const bool ptop = yy == stripe * p.ss, pzero = yy == 0;
  const int yp = ptop ? 0 : yy - 1;
  const int64_t prow = ptop ? (int64_t)(p.HG4 + stripe) * plane4 : (int64_t)(yp >> 2) * plane4 + (yp & 3) * D;
  // the pair's volume through one buffer descriptor (built from wave-uniform values): a lane's
  // row / disparity offset in a VGPR, the column offset x * 4D * 2 bytes in an SGPR; above
  // row 0 the offset points past the buffer, so the previous row reads as zeros
  const uint16_t* vpair = Vvol + (int64_t)b * (p.HG4 + p.nstripes) * plane4;
  const uint32_t vbytes = (uint32_t)((p.HG4 + p.nstripes) * plane4 * 2);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)vpair)) |
              ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)vpair >> 32)) << 32)),
      (short)0, (int)__builtin_amdgcn_readfirstlane((int)vbytes), 0x00020000);
  const uint32_t voffV = (uint32_t)(((int64_t)(yy >> 2) * plane4 + (yy & 3) * D + q * DQ) * 2);
  // rows 1..3 of a group read V(y-1) from memory although the same wave loads those bytes as
  // the row above's own V: taking them from those lanes by a cross-lane permute instead (only
  // row 0 / stripe-top lanes loading) was measured slower (r4: 3.90 -> 4.06 ms; the duplicate
  // loads are L1 hits, the 3 ds_bpermute + select per column are not free)
  const uint32_t voffP = pzero ? 0x80000000u : (uint32_t)((prow + q * DQ) * 2);
  // the previous row's minimum over d, [group][x1][4] u16 (zero above row 0)
  const uint16_t* mpair = Mvol + (int64_t)b * (p.HG4 + p.nstripes) * W1 * 4;
  const uint32_t mbytes = (uint32_t)((p.HG4 + p.nstripes) * W1 * 8);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)mpair)) |
              ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)mpair >> 32)) << 32)),
      (short)0, (int)__builtin_amdgcn_readfirstlane((int)mbytes), 0x00020000);
  const int pgrp = ptop ? p.HG4 + stripe : yp >> 2, psub = ptop ? 0 : yp & 3;
  const uint32_t voffM = pzero ? 0x80000000u : (uint32_t)(((int64_t)pgrp * W1 * 4 + psub) * 2);
  const u16x2 P1 = splat(p.P1);
  // column offsets are wave-uniform (readfirstlane keeps them in SGPRs: a VGPR soffset would
  // make the compiler wrap each load in a waterfall loop)
  auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
  auto ld = [&](int x, uint32_t* out) { bload<PQ>(vrs, voffV, uni((uint32_t)x * (XS * 4)), out); };
  auto ldp = [&](int x, uint32_t* out) { bload<PQ>(vrs, voffP, uni((uint32_t)x * (XS * 4)), out); };
  auto ldm = [&](int x) -> uint32_t {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(mrs, voffM, uni((uint32_t)x * 8), 0);
  };

  // ---- sweep 1: left -> right, checkpoints, in blocks of SEG columns that end at the
  // checkpoint columns x = W1-1-SEG*m, so every block is full and its checkpoint is its last
  // state (stored once per block; slot nck-1 is a dummy for the last block, which holds none).
  // The first block starts at xs <= 0: its columns left of 0 step with C = 0, which keeps the
  // zero start state exactly (C + min(0, P1, P2) - 0 = 0).  Loads are unconditional (clamped
  // columns) so the compiler's vmcnt waits stay precise, and the block body has no branches,
  // so the scheduler overlaps one column's serial min-reduction with the next column's work.
  // V and the previous row PD columns ahead (a ring of PD column buffers)
  static_assert(PF == SEG && SEG % PD == 0, "ring slots line up across blocks");
  if constexpr (S1) {
  uint32_t st[PQ], vb[PD][PQ], pb[PD][PQ], mb[PD];
  uint32_t minPrev = 0;
  const int xs = ((W1 - 1) & (SEG - 1)) - (SEG - 1);
#pragma unroll
  for (int k = 0; k < PQ; ++k) st[k] = 0;
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    const int xx = min(max(xs + j, 0), W1 - 1);
    ld(xx, vb[j]);
    ldp(xx, pb[j]);
    mb[j] = ldm(xx);
  }
  auto block1 = [&](int x0, auto first_t) {
    constexpr bool FIRST = decltype(first_t)::value;
#pragma unroll
    for (int j = 0; j < SEG; ++j) {
      const int x = x0 + j;
      uint32_t c[PQ];
      derive16<PQ>(pb[j % PD], vb[j % PD], c, mb[j % PD], P1, p.P2, q);
      if (FIRST) {
#pragma unroll
        for (int k = 0; k < PQ; ++k) c[k] = x < 0 ? 0u : c[k];
      }
      const int xn = FIRST ? min(max(x + PD, 0), W1 - 1) : min(x + PD, W1 - 1);
      ld(xn, vb[j % PD]);
      ldp(xn, pb[j % PD]);
      mb[j % PD] = ldm(xn);
      minPrev = step16<PQ>(st, c, q, P1, minPrev, p.P2);
    }
    const int rem = W1 - 1 - SEG - (x0 + SEG - 1);
    const int slot = rem >= 0 ? rem / SEG : nck - 1;
    uint32_t* cp = ckptr(slot);
    uint32_t v[CKW];
#pragma unroll
    for (int kk = 0; kk < CKW; ++kk) v[kk] = kk < PQ ? st[kk] : kk == PQ ? minPrev : 0u;
#pragma unroll
    for (int kk = 0; kk < CKW; kk += 4) *reinterpret_cast<uint4*>(cp + kk) = make_uint4(v[kk], v[kk + 1], v[kk + 2], v[kk + 3]);
  };
  block1(xs, std::true_type{});
#pragma unroll 1
  for (int x0 = xs + SEG; x0 < W1; x0 += SEG) block1(x0, std::false_type{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the checkpoints, re-read below by the lanes that stored them
  }
  if constexpr (!S2) return;

  // ---- sweep 2: segments s of reflected columns x' = SEG*s + i (x1 = W1-1-x'), right to left
  const int nseg = (W1 + SEG - 1) / SEG;
  uint32_t Rst[PQ];
  uint32_t minR = 0;
#pragma unroll
  for (int k = 0; k < PQ; ++k) Rst[k] = 0;
  // V and the previous V row of segment sg + 1 are loaded column by column inside segment
  // sg's R path, each into the registers of a column that path has just finished (the next L
  // recompute consumes the columns in the reverse order, so the first one it needs is loaded
  // first); its checkpoint is loaded as the R path starts
  uint32_t Vn[SEG][PQ], Pn[SEG][PQ], Mn[SEG], ckn[CKW];
  auto ldck = [&](int sg) {
    const int slot = SEG * (sg + 1) > W1 - 1 ? nck - 1 : sg;
    const uint32_t* cp = ckptr(slot);
#pragma unroll
    for (int kk = 0; kk < CKW; kk += 4) {
      const uint4 w4 = *reinterpret_cast<const uint4*>(cp + kk);
      ckn[kk] = w4.x; ckn[kk + 1] = w4.y; ckn[kk + 2] = w4.z; ckn[kk + 3] = w4.w;
    }
  };
  auto ldcol = [&](int sg, int i) {
    const int xx = max(W1 - 1 - (SEG * sg + i), 0);
    ld(xx, Vn[i]);
    ldp(xx, Pn[i]);
    Mn[i] = ldm(xx);
  };
  auto ldseg = [&](int sg) {
    ldck(sg);
#pragma unroll
    for (int i = SEG - 1; i >= 0; --i) ldcol(sg, i);
  };
  ldseg(0);
  // one segment; FULL (every segment but the last): 8 valid columns and a checkpoint, so the
  // body has no per-column conditions
  // WTA of column i of a segment from its S words: first minimum over d as one u32 min of
  // (S << 8 | d) across the row's lanes, then S[d-1] << 16 | S[d+1] from the lanes that hold
  // them (OR across the row); every lane of the row ends with both, lane q keeps column q's
  auto ihi_of = [&](int sg) { return min(SEG - 1, W1 - 1 - SEG * sg); };  // valid i: x' < W1
  uint32_t wk = 0, wn = 0;
  auto wta = [&](int i, const uint32_t* Sw) {
    // keys (S << 8 | j) with j the disparity's index in this lane's run, built by byte permutes
    // (S's two bytes above a byte of the constant (j, j + 1) pair word), min3-folded, then the
    // lane's first disparity q * DQ added to the index byte (j + q * DQ < D <= 128: no carry)
    uint32_t kmin = 0;
#pragma unroll
    for (int kk = 0; kk < PQ; ++kk) {
      const uint32_t jj = (uint32_t)(2 * kk) | ((uint32_t)(2 * kk + 1) << 8);
      const uint32_t klo = __builtin_amdgcn_perm(Sw[kk], jj, 0x0c050400u);  // S[2kk] << 8 | 2kk
      const uint32_t khi = __builtin_amdgcn_perm(Sw[kk], jj, 0x0c070601u);  // S[2kk+1] << 8 | 2kk+1
      kmin = kk == 0 ? min(klo, khi) : min(kmin, min(klo, khi));
    }
    kmin += (uint32_t)(q * DQ);
    kmin = dmin<kQX1>(kmin);
    kmin = dmin<kQX2>(kmin);
    kmin = dmin<kRHalfMirror>(kmin);
    kmin = dmin<kRMirror>(kmin);
    const int d = (int)(kmin & 0xFFu);
    // S[d-1] << 16 | S[d+1] (only read when 0 < d < D-1): the row's S words through a one-column
    // LDS slot (a wave's LDS accesses execute in order: no barrier, and the next column's store
    // comes after these loads)
    uint32_t* sw = reinterpret_cast<uint32_t*>(&s_S[r][q * DQ]);
#pragma unroll
    for (int kk = 0; kk < PQ; ++kk) sw[kk] = Sw[kk];
    asm volatile("" ::: "memory");  // u32 stores, u16 loads: keep the compiler from reordering them
    const uint32_t nb = ((uint32_t)s_S[r][max(d - 1, 0)] << 16) | s_S[r][min(d + 1, D - 1)];
    asm volatile("" ::: "memory");
    wk = q == i ? kmin : wk;
    wn = q == i ? nb : wn;
  };
  // one segment.  FULL (every segment but the last: 8 valid columns and a checkpoint): the L
  // recompute (columns 7 -> 0 = real x ascending) and the R path (0 -> 7) run interleaved --
  // step t advances L on column 7-t and R on column t, two independent dependency chains --
  // and each column's S is formed when its second path reaches it (the first one's state is
  // kept as path + V).  The next segment's inputs are loaded into the registers of the
  // columns finished at steps 4..7, its first-needed columns (7 and 0) first.  The last
  // segment (partial) runs L, then R, column by column.
  auto segment = [&](int sg, auto full_t) {
    constexpr bool FULL = decltype(full_t)::value;
    if constexpr (FULL) {
      uint32_t lst[PQ], Cs[SEG][PQ], part[SEG][PQ];
#pragma unroll
      for (int kk = 0; kk < PQ; ++kk) lst[kk] = ckn[kk];
      uint32_t lmin = ckn[PQ];
      ldck(sg + 1);
#pragma unroll
      for (int t = 0; t < SEG; ++t) {
        const int a = SEG - 1 - t, c = t;  // L column, R column
        if (t < SEG / 2) {
          derive16<PQ>(Pn[a], Vn[a], Cs[a], Mn[a], P1, p.P2, q);
          derive16<PQ>(Pn[c], Vn[c], Cs[c], Mn[c], P1, p.P2, q);
        }
        lmin = step16<PQ>(lst, Cs[a], q, P1, lmin, p.P2);
        minR = step16<PQ>(Rst, Cs[c], q, P1, minR, p.P2);
        if (t < SEG / 2) {  // first path at both columns: keep path + V
#pragma unroll
          for (int kk = 0; kk < PQ; ++kk) {
            part[a][kk] = as_u(as_v(lst[kk]) + as_v(Vn[a][kk]));
            part[c][kk] = as_u(as_v(Rst[kk]) + as_v(Vn[c][kk]));
          }
        } else {  // second path: S = L + R + V
          uint32_t Sa[PQ], Sc[PQ];
#pragma unroll
          for (int kk = 0; kk < PQ; ++kk) {
            Sa[kk] = as_u(as_v(part[a][kk]) + as_v(lst[kk]));
            Sc[kk] = as_u(as_v(part[c][kk]) + as_v(Rst[kk]));
          }
          wta(a, Sa);
          wta(c, Sc);
          const int u = t - SEG / 2;  // next segment: columns 7-u and u
          ldcol(sg + 1, SEG - 1 - u);
          ldcol(sg + 1, u);
        }
      }
    } else {
      uint32_t lst[PQ], Ls[SEG][PQ], Cs[SEG][PQ];
      const bool zero = SEG * (sg + 1) > W1 - 1;
      // L over the segment (i descending = real x ascending) from the checkpoint at the real
      // column left of it, x' = SEG*(sg+1); zero state when the segment starts at x = 0.
#pragma unroll
      for (int kk = 0; kk < PQ; ++kk) lst[kk] = zero ? 0u : ckn[kk];
      uint32_t lmin = zero ? 0u : ckn[PQ];
#pragma unroll
      for (int i = SEG - 1; i >= 0; --i) {
        derive16<PQ>(Pn[i], Vn[i], Cs[i], Mn[i], P1, p.P2, q);
        if (i <= ihi_of(sg)) lmin = step16<PQ>(lst, Cs[i], q, P1, lmin, p.P2);
#pragma unroll
        for (int kk = 0; kk < PQ; ++kk) Ls[i][kk] = as_u(as_v(lst[kk]) + as_v(Vn[i][kk]));
      }
#pragma unroll
      for (int i = 0; i < SEG; ++i) {
        if (i > ihi_of(sg)) break;
        minR = step16<PQ>(Rst, Cs[i], q, P1, minR, p.P2);
        uint32_t Sw[PQ];
#pragma unroll
        for (int kk = 0; kk < PQ; ++kk) Sw[kk] = as_u(as_v(Ls[i][kk]) + as_v(Rst[kk]));
        wta(i, Sw);
      }
    }
    {
      const int ihi = FULL ? SEG - 1 : ihi_of(sg);
      // the segment's columns, one lane each (lane q of a row = column q of the segment), so
      // the sub-pixel division and the key updates run once per segment, not once per column.
      // Every ring slot reset comes before any key update: the slot column i resets (the
      // lowest x2 it can reach) is reachable only from columns i, i+1, ... (further left), so
      // the final keys equal the serial order's.
      {
        const bool colv = q < SEG && q <= ihi;
        const int x1 = W1 - 1 - (SEG * sg + q);
        if (colv) key[(x1 + p.minX1 - p.minD - (D - 1)) & (RK - 1)] = 0xFFFFFFFFu;
        if (colv) {
          const int best = (int)(wk >> 8), d = (int)(wk & 0xFFu);
          const int sm1 = (int)(wn >> 16), sp1 = (int)(wn & 0xFFFFu);
          const int x2 = x1 + p.minX1 - d - p.minD;
          if (x2 >= 0 && x2 < W && best < 0x7FFF)  // disp2cost starts at SHRT_MAX
            atomicMin(&key[x2 & (RK - 1)], ((uint32_t)best << 16) | (uint32_t)(0xFFFF - x1));
          int dd;
          if (0 < d && d < D - 1) {
            const int denom2 = max(sm1 + sp1 - 2 * best, 1);
            dd = d * 16 + ((sm1 - sp1) * 16 + denom2) / (denom2 * 2);
          } else {
            dd = d * 16;
          }
          sraw[x1 & (RS - 1)] = (int16_t)(dd + p.minD * 16);
        }
      }
      // pixels whose keys became final with this segment (at most SEG): one lane each
      const int x1_lo = W1 - 1 - (SEG * sg + ihi);
      {
        const int cnt = ihi >= 0 ? min(next_chk - (x1_lo + D) + 1, SEG) : 0;
        const bool act = q < cnt && rowok;
        const int d1 = checked(next_chk - q);
        *(act ? out + (next_chk - q + p.minX1) : sink) = (int16_t)d1;
        if (cnt > 0) next_chk -= cnt;
      }
    }
  };
#pragma unroll 1
  for (int sg = 0; sg < nseg - 1; ++sg) segment(sg, std::true_type{});
  segment(nseg - 1, std::false_type{});
  for (int x1 = next_chk - q; x1 >= 0; x1 -= 16) check(x1);  // the last D (+ < SEG) pixels
}

// ------------------------------------------------------------------ median 3x3
// fail (may be null): pairs whose L-path hand-off timed out come out invalid everywhere;
// status (may be null): per pair FVO_SGBM_OK / FVO_SGBM_HANDOFF_TIMEOUT, for the caller
__global__ void k_sg_median(const int16_t* __restrict__ raw, int16_t* __restrict__ out, int W, int H,
                            const uint32_t* __restrict__ fail, int16_t invalid, int32_t* __restrict__ status) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, b = blockIdx.z;
  if (status && x == 0 && y == 0) status[b] = (fail && fail[b]) ? FVO_SGBM_HANDOFF_TIMEOUT : FVO_SGBM_OK;
  if (x >= W) return;
  const int16_t* s = raw + (int64_t)b * W * H;
  int v[9];
  int k = 0;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = min(max(y + dy, 0), H - 1), xx = min(max(x + dx, 0), W - 1);
      v[k++] = s[(int64_t)yy * W + xx];
    }
  // Paeth's 19-compare median-of-9 network
#define SG_S(a, b) { int t_ = min(v[a], v[b]); v[b] = max(v[a], v[b]); v[a] = t_; }
  SG_S(1, 2) SG_S(4, 5) SG_S(7, 8) SG_S(0, 1) SG_S(3, 4) SG_S(6, 7) SG_S(1, 2) SG_S(4, 5) SG_S(7, 8)
  SG_S(0, 3) SG_S(5, 8) SG_S(4, 7) SG_S(3, 6) SG_S(1, 4) SG_S(2, 5) SG_S(4, 7) SG_S(4, 2) SG_S(6, 4)
  SG_S(4, 2)
#undef SG_S
  out[((int64_t)b * H + y) * W + x] = (fail && fail[b]) ? invalid : (int16_t)v[4];
}

// Per call of the L-path schedule: ticket counter reset, generation advanced (never 0, < 2^25:
// tags are generation << 7 | column block), failure flags of the batch's pairs cleared.
__global__ void k_sg_prep(uint32_t* ctl, int nb) {
  const int t = threadIdx.x;
  if (t == 0) {
    ctl[0] = 0;
    const uint32_t g = ctl[1] + 1;
    ctl[1] = g >= (1u << 25) ? 1u : g;
  }
  for (int b = t; b < nb; b += blockDim.x) ctl[4 + b] = 0;
}

// Schedules and launch shapes (fvo_config, validated by sgbm_init; every variant is
// bit-identical and parity-tested), sgbm_mode:
//   FVO_SGBM_CLASSIC  one cost pass, one row pass running both sweeps, with sgbm_lanes lanes per
//                     column (4, 8 or 16) and sgbm_cols columns per block (4: 32/64; 8: 16/32; 16: 32)
//   FVO_SGBM_LPATH    the L path in the cost pass, handed from column block to column block: one V
//                     read per pair fewer (<= 300 MB/pair) but slower -- DESIGN.md §4.2 r5
int sg_lanes(const fvo_config& c) { return c.sgbm_lanes > 0 ? c.sgbm_lanes : 8; }
int sg_cols(const fvo_config& c) { return c.sgbm_cols > 0 ? c.sgbm_cols : (sg_lanes(c) == 4 ? 64 : 32); }

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
  p.HG4 = (c.height + 3) / 4;
  return p;
}

// Checkpoints of the left->right path (per 4-row block or per row): at x = W1-9-8s, s < nck.
int sg_nck(const SgParams& p) { return p.width1 / 8 + 2; }  // + a dummy slot
int sg_ckw(int D) { return D / 32 + 1 <= 4 ? 4 : 8; }
int sg_nblk(const SgParams& p) { return (p.H + 3) / 4; }
constexpr int kSgCB = 32;  // columns per cost block of the L-path schedule
int sg_nk(const SgParams& p) { return (p.width1 + kSgCB - 1) / kSgCB; }

template <int D>
void launch_sgbm(fvo_ctx* ctx, const SgParams& p, const uint8_t* L, const uint8_t* R, int nb, int64_t stride,
                 int pitch, int16_t* disp, int32_t* status, hipStream_t s) {
  uint16_t* V = ctx->sg_V;
  uint16_t* M = ctx->sg_M;
  const int nck = sg_nck(p);
  const int16_t invalid = (int16_t)((p.minD - 1) * 16);
  const fvo_config& cfg = ctx->cfg;
  if (cfg.sgbm_mode == FVO_SGBM_CLASSIC) {
    // (G, CB) of the cost pass, validated by sgbm_init; the grid follows the kernel launched
    const int g = sg_lanes(cfg), cbr = sg_cols(cfg);
    typedef void (*CostKernel)(const uint8_t*, const uint8_t*, int64_t, int, SgParams, uint16_t*, uint16_t*, SgLink);
    CostKernel kern;
    int gg, cb;
    if (g == 16) kern = k_sg_costvert<D, 32, 16, false>, gg = 16, cb = 32;
    else if (g == 4 && cbr == 32) kern = k_sg_costvert<D, 32, 4, false>, gg = 4, cb = 32;
    else if (g == 4) kern = k_sg_costvert<D, 64, 4, false>, gg = 4, cb = 64;
    else if (cbr == 16) kern = k_sg_costvert<D, 16, 8, false>, gg = 8, cb = 16;
    else kern = k_sg_costvert<D, 32, 8, false>, gg = 8, cb = 32;
    const dim3 gcv((p.width1 + cb - 1) / cb, p.nstripes, nb);
    const SgLink lk{};
    FVO_TIMED(ctx, KN_SG_VERT, s, hipLaunchKernelGGL(kern, gcv, dim3(gg * cb), 0, s, L, R, stride, pitch, p, V, M, lk));
    FVO_TIMED(ctx, KN_SG_ROWS, s, hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_rows<D, kSwBoth>), dim3(sg_nblk(p), nb), dim3(64), 0, s,
                                                     V, M, p, ctx->sg_ckpt, nck, ctx->sg_raw));
    FVO_TIMED(ctx, KN_SG_MEDIAN, s, hipLaunchKernelGGL(k_sg_median, dim3((p.W + 255) / 256, p.H, nb), dim3(256), 0, s,
                                                       ctx->sg_raw, disp, p.W, p.H, nullptr, invalid, status));
    return;
  }
  const int nk = sg_nk(p);
  const int64_t us = cfg.sgbm_handoff_us > 0 ? cfg.sgbm_handoff_us : 250000;
  const SgLink lk{ctx->sg_ckpt, nck, nk, ctx->sg_hand, ctx->sg_ctl, (uint64_t)us * 100u, cfg.sgbm_handoff_us < 0 ? 1 : 0};
  hipLaunchKernelGGL(k_sg_prep, dim3(1), dim3(256), 0, s, ctx->sg_ctl, nb);
  FVO_TIMED(ctx, KN_SG_VERT, s, hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_costvert<D, kSgCB, 8, true>),
                                                   dim3(nk * p.nstripes * nb), dim3(8 * kSgCB), 0, s, L, R, stride, pitch,
                                                   p, V, M, lk));
  FVO_TIMED(ctx, KN_SG_ROWS, s, hipLaunchKernelGGL(HIP_KERNEL_NAME(k_sg_rows<D, kSwRight>), dim3(sg_nblk(p), nb), dim3(64), 0, s,
                                                   V, M, p, ctx->sg_ckpt, nck, ctx->sg_raw));
  FVO_TIMED(ctx, KN_SG_MEDIAN, s, hipLaunchKernelGGL(k_sg_median, dim3((p.W + 255) / 256, p.H, nb), dim3(256), 0, s,
                                                     ctx->sg_raw, disp, p.W, p.H, ctx->sg_ctl + 4, invalid, status));
}

}  // namespace

int sgbm_init(fvo_ctx* ctx) {
  const fvo_config& c = ctx->cfg;
  if (c.block_size != 7) return fvo_fail(ctx, "SGBM: only blockSize=7 is supported");
  if (c.num_disparities != 64 && c.num_disparities != 96 && c.num_disparities != 128)
    return fvo_fail(ctx, "SGBM: numDisparities must be 64, 96 or 128");
  if (c.uniqueness_ratio != 0) return fvo_fail(ctx, "SGBM: only uniquenessRatio=0 is supported");
  if (c.sgbm_stripes < 1) return fvo_fail(ctx, "SGBM: stripes must be >= 1");
  if (c.sgbm_mode != FVO_SGBM_CLASSIC && c.sgbm_mode != FVO_SGBM_LPATH)
    return fvo_fail(ctx, "SGBM: sgbm_mode must be FVO_SGBM_CLASSIC or FVO_SGBM_LPATH");
  if (c.sgbm_mode == FVO_SGBM_CLASSIC) {
    const int g = sg_lanes(c), cb = sg_cols(c);
    if (!((g == 4 && (cb == 32 || cb == 64)) || (g == 8 && (cb == 16 || cb == 32)) || (g == 16 && cb == 32)))
      return fvo_fail(ctx, "SGBM: (sgbm_lanes, sgbm_cols) must be (4, 32|64), (8, 16|32) or (16, 32)");
  } else if (c.sgbm_lanes != 0 || c.sgbm_cols != 0) {
    return fvo_fail(ctx, "SGBM: sgbm_lanes / sgbm_cols apply to the classic schedule only (leave them 0)");
  }
  if (c.sgbm_handoff_us < -1) return fvo_fail(ctx, "SGBM: sgbm_handoff_us must be >= -1");
  SgParams p = make_params(c);
  if (p.width1 <= 0) return fvo_fail(ctx, "SGBM: image narrower than numDisparities");
  // path values are at most C + P2 with C <= 49 x the largest BT pixel cost (2 ftzero + 255/4);
  // the kernels add P1 to them in u16 (min(a, b) + P1 for min(a + P1, b + P1)), so that sum
  // must not wrap -- OpenCV's 16-bit CostType carries the same assumption
  if (49 * (2 * p.ftzero + 63) + p.P2 + p.P1 > 0xFFFF)
    return fvo_fail(ctx, "SGBM: P1/P2/preFilterCap too large for 16-bit path costs");
  // the row pass sums S = L + R + V in u16 lanes and its WTA keys on S: each path is at most
  // C + P2, so 3 (C + P2) must not wrap either
  if (3 * (49 * (2 * p.ftzero + 63) + p.P2) > 0xFFFF)
    return fvo_fail(ctx, "SGBM: P2/preFilterCap too large for the 16-bit aggregated cost");
  const int64_t B = c.sgbm_max_batch > 0 ? std::min(c.sgbm_max_batch, c.max_batch) : c.max_batch;
  const int64_t plane = (int64_t)p.width1 * p.D;
  int rc;
  // sg_V: top-down path V [B][HG4 + nstripes][width1][4][D] u16 (the extra groups: the
  // stripes' overlap rows); sg_ckpt: the left->right path checkpoints; sg_raw: pre-median
  // disparity [B][H][W]
  const int64_t vol = (int64_t)(p.HG4 + p.nstripes) * 4 * plane;
  // (the per-block layout of the classic schedule is the larger one: 64 lanes per 4 rows)
  const int64_t ckp = (int64_t)sg_nblk(p) * sg_nck(p) * 64 * sg_ckw(p.D);
  // sg_hand: the L path's hand-off granules [B][H][2][D/32][16] u64; sg_ctl: ticket, generation,
  // timeout count, per-pair failure flags.  Both zeroed once (tags of a zeroed granule never match)
  const int64_t hand = (int64_t)p.H * 2 * (p.D / 32) * 16;
  // the L path's hand-off tags carry the column block in 7 bits
  if (c.sgbm_mode == FVO_SGBM_LPATH && sg_nk(p) >= 128)
    return fvo_fail(ctx, "SGBM: FVO_SGBM_LPATH needs width - numDisparities <= 4064 (use the classic schedule)");
  // sg_M: min over d of every stored V row, [B][HG4 + nstripes][width1][4] u16
  if ((rc = fvo_alloc(ctx, &ctx->sg_V, B * vol)) || (rc = fvo_alloc(ctx, &ctx->sg_M, B * vol / p.D)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_ckpt, B * ckp)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_raw, B * p.H * p.W)) || (rc = fvo_alloc(ctx, &ctx->sg_hand, B * hand)) ||
      (rc = fvo_alloc(ctx, &ctx->sg_ctl, 4 + B)))
    return rc;
  FVO_HIP(ctx, hipMemset(ctx->sg_hand, 0, B * hand * sizeof(uint64_t)));
  FVO_HIP(ctx, hipMemset(ctx->sg_ctl, 0, (4 + B) * sizeof(uint32_t)));
  return 0;
}

int sgbm_run(fvo_ctx* ctx, const uint8_t* L, const uint8_t* R, int batch, int64_t image_stride, int pitch,
             int16_t* disp, int32_t* status, hipStream_t s) {
  SgParams p = make_params(ctx->cfg);
  switch (p.D) {
    case 64: launch_sgbm<64>(ctx, p, L, R, batch, image_stride, pitch, disp, status, s); break;
    case 96: launch_sgbm<96>(ctx, p, L, R, batch, image_stride, pitch, disp, status, s); break;
    default: launch_sgbm<128>(ctx, p, L, R, batch, image_stride, pitch, disp, status, s); break;
  }
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
