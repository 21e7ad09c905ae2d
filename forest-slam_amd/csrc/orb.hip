// ORB detectAndCompute for gfx950 — replaces cv2.ORB_create() + orb.detectAndCompute
// (ros_ws/src/stereo_slam.py:84, :232-233, :240-241).  Batched over images.
//
// Stages (one launch each, all images of the batch at once):
//   pyramid      level 0 copy + 7 INTER_LINEAR_EXACT downscales (ufixedpoint16 weights)
//   fast_score   FAST-9/16 corner test + cornerScore<16> -> u8 score map (all levels)
//   nms_count    3x3 strict-max NMS + 31-px border filter, per-row counts
//   row_scan     per-level exclusive scan of row counts
//   nms_compact  ordered (row-major) compaction -> packed candidates (score<<24|y<<12|x)
//   select       KeyPointsFilter::retainBest(2n_l) — block-parallel, bit-identical to
//                libstdc++'s nth_element + partition element order (see select_block)
//   harris       7x7 Harris response per candidate (wave per keypoint)
//   select       retainBest(n_l) on the Harris responses
//   finalize     per-image level offsets / counts
//   angle        intensity-centroid angle (fastAtan2) + keypoint records
//   blur         GaussianBlur 7x7 sigma 2 (8-bit fixed-point separable, REFLECT_101)
//   brief        steered rBRIEF, one wave per keypoint, 4 ballots = 32 bytes
// All float expressions are evaluated in the order OpenCV writes them; the library is
// compiled with -ffp-contract=off so no FMA contraction changes a rounding.
#include <cmath>
#include <cstring>

#include "fvo_device.h"
#include "orb_pattern.inc"

namespace {

// Pyramid geometry, passed BY VALUE to every kernel (kernarg segment, scalar loads): each
// context has its own image size, so module-global __constant__ tables would be clobbered
// by the next fvo_create of a different size.
struct OrbDev {
  int nlevels, total_rows;
  int row0[FVO_MAX_LEVELS + 1];
  int w[FVO_MAX_LEVELS], h[FVO_MAX_LEVELS];
  long long off[FVO_MAX_LEVELS + 1];
  long long cand_off[FVO_MAX_LEVELS + 1];
  float scale[FVO_MAX_LEVELS];
  int nfeat[FVO_MAX_LEVELS];
  int tile0[FVO_MAX_LEVELS + 1];  // first 64x32 FAST tile of each level (per image)
  int ntx[FVO_MAX_LEVELS];        // tiles per row of each level
  int btile0[FVO_MAX_LEVELS + 1]; // first 256x32 blur tile of each level (per image)
  int bntx[FVO_MAX_LEVELS];       // blur tiles per row of each level
};
__constant__ int c_umax[20];
__constant__ signed char c_pattern[256 * 4];

constexpr int kSelThreads = 512;
// LDS capacity of the selection kernels (candidates per (image, level)); larger levels select
// in global memory.  select 1: u32 candidates, select 2: u64 Harris records.
constexpr int kSelCap1 = 10000, kSelCap2 = 4096;

__device__ __forceinline__ int level_of_row(const OrbDev& G, int r) {
  int l = 0;
#pragma unroll
  for (int k = 1; k < FVO_MAX_LEVELS; ++k)
    if (k < G.nlevels && r >= G.row0[k]) l = k;
  return l;
}

// ------------------------------------------------------------------ pyramid
__global__ void k_copy_level0(const uint8_t* __restrict__ img, int64_t stride, int pitch, uint8_t* __restrict__ pyr,
                              int64_t total, int W, int H) {
  int x = blockIdx.x * blockDim.x + threadIdx.x;
  int y = blockIdx.y;
  int b = blockIdx.z;
  if (x >= W) return;
  pyr[b * total + (int64_t)y * W + x] = img[b * stride + (int64_t)y * pitch + x];
}

// 16 pixels per thread when rows, strides and both bases are 16-byte aligned (the usual
// contiguous [B][H][W] batch with W % 16 == 0; the pyramid's per-image size is padded to 256)
__global__ void k_copy_level0_v(const uint4* __restrict__ img, int64_t stride16, int pitch16,
                                uint4* __restrict__ pyr, int64_t total16, int W16, int H, int batch) {
  const int64_t n = (int64_t)batch * H * W16;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / W16;
    const int x = (int)(i - row * W16);
    const int b = (int)(row / H), y = (int)(row - (int64_t)b * H);
    pyr[b * total16 + (int64_t)y * W16 + x] = img[b * stride16 + (int64_t)y * pitch16 + x];
  }
}

// INTER_LINEAR_EXACT level l from level l-1; a thread covers kResCols consecutive columns x
// kResRows rows (the column tables are read once per thread).  The border cases are folded
// into the weights (a clamped source index with weights 256 / 0 gives exactly the border
// formulas: s << 8 for a column, (h + 128) >> 8 = (256 h + 32768) >> 16 for a row), so every
// load is unconditional and the rows' loads are all in flight at once.  Interior threads read
// the source bytes of their 4 columns as one 8-byte window per source row (three aligned
// dwords, v_alignbyte) instead of 16 byte loads; a window never reaches past level l-1's
// successor in the same image, so the aligned over-read stays inside the pyramid buffer.
constexpr int kResRows = 4, kResCols = 4;
__global__ void k_resize(const OrbDev G, uint8_t* __restrict__ pyr, int64_t total, int l, const int32_t* __restrict__ xofs,
                         const int32_t* __restrict__ xc1, const int32_t* __restrict__ yofs,
                         const int32_t* __restrict__ yc1) {
  const XcdBlock xb = xcd_block();  // blocks sharing source rows on one XCD
  const int x0 = (xb.x * blockDim.x + threadIdx.x) * kResCols;
  const int b = xb.z;
  const int w = G.w[l], h = G.h[l];
  if (x0 >= w) return;
  const int sw = G.w[l - 1], sh = G.h[l - 1];
  const uint8_t* src = pyr + b * total + G.off[l - 1];
  uint8_t* dst = pyr + b * total + G.off[l];
  int oxa[kResCols], oxb[kResCols];
  uint32_t cx0[kResCols], cx1[kResCols];
#pragma unroll
  for (int i = 0; i < kResCols; ++i) {
    const int ox = xofs[min(x0 + i, w - 1)];
    oxa[i] = ox >= 0 ? ox : (ox == -1 ? 0 : sw - 1);
    oxb[i] = ox >= 0 ? ox + 1 : oxa[i];
    cx1[i] = ox >= 0 ? (uint32_t)xc1[min(x0 + i, w - 1)] : 0u;
    cx0[i] = 256u - cx1[i];
  }
  // interior: every column regular (ox >= 0) and the 4 columns' sources within 8 bytes
  const bool win8 = x0 + kResCols <= w && xofs[x0] >= 0 && xofs[x0 + kResCols - 1] >= 0 &&
                    oxb[kResCols - 1] - oxa[0] <= 7;
  auto window = [&](const uint8_t* row) -> uint64_t {
    const uintptr_t pa = reinterpret_cast<uintptr_t>(row + oxa[0]);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(pa & ~(uintptr_t)3);
    const uint32_t sft = (uint32_t)(pa & 3);
    const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
    return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sft) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sft);
  };
  uint32_t v[kResRows][kResCols];
#pragma unroll
  for (int k = 0; k < kResRows; ++k) {
    const int y = min(xb.y * kResRows + k, h - 1);
    const int oy = yofs[y];
    const int ra = oy >= 0 ? oy : (oy == -1 ? 0 : sh - 1), rb = oy >= 0 ? oy + 1 : ra;
    const uint32_t cy1 = oy >= 0 ? (uint32_t)yc1[y] : 0u, cy0 = 256u - cy1;
    const uint8_t* sa = src + (int64_t)ra * sw;
    const uint8_t* sb = src + (int64_t)rb * sw;
    if (win8) {
      const uint64_t wa = window(sa), wb = window(sb);
#pragma unroll
      for (int i = 0; i < kResCols; ++i) {
        const int da = 8 * (oxa[i] - oxa[0]), db = 8 * (oxb[i] - oxa[0]);
        const uint32_t ha = cx0[i] * (uint32_t)((wa >> da) & 255u) + cx1[i] * (uint32_t)((wa >> db) & 255u);
        const uint32_t hb = cx0[i] * (uint32_t)((wb >> da) & 255u) + cx1[i] * (uint32_t)((wb >> db) & 255u);
        v[k][i] = (ha * cy0 + hb * cy1 + 32768u) >> 16;
      }
    } else {
#pragma unroll
      for (int i = 0; i < kResCols; ++i) {
        const uint32_t ha = cx0[i] * sa[oxa[i]] + cx1[i] * sa[oxb[i]], hb = cx0[i] * sb[oxa[i]] + cx1[i] * sb[oxb[i]];
        v[k][i] = (ha * cy0 + hb * cy1 + 32768u) >> 16;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kResRows; ++k) {
    const int y = xb.y * kResRows + k;
#pragma unroll
    for (int i = 0; i < kResCols; ++i)
      if (y < h && x0 + i < w) dst[(int64_t)y * w + x0 + i] = (uint8_t)(v[k][i] > 255u ? 255u : v[k][i]);
  }
}

// ------------------------------------------------------------------ FAST
__constant__ int c_cdx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int c_cdy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

// ------------------------------------------------------------------ FAST + NMS (tiled)
// One block per 64 x 32 tile of a level: the image patch (tile + 4-px apron) is staged in
// LDS; the FAST test runs on the tile + 1-px halo, the positions that pass are packed into
// an LDS list so cornerScore<16> runs on dense lanes (textured frames make ~80 % of waves
// contain a corner, so per-pixel scoring ran the score code on nearly every wave); then the
// strict 3x3 NMS + border filter of the tile is evaluated from the LDS score tile.  Output:
// per tile one record, written as contiguous runs: the rows' keep bits (a 64-bit word per tile
// row), the rows' keep prefixes (32 u16) and the kept pixels' scores in row-major order -- no
// full-level score map and no scattered per-row keep words or counters cross HBM (the row
// counts are popcounts of the records' words, taken by k_row_scan; the score map itself is
// produced only on request, by the SCOREMAP instance, for the debug hook).
constexpr int kTW = 64, kTH = 32, kFT = 256;  // tile, threads per tile block
static_assert(kTH <= 64 && kFT >= 2 * kTH && kFT % 64 == 0, "FAST tile shape");
constexpr int kRecKeep = 0, kRecPre = 8 * kTH, kRecSc = kRecPre + 2 * kTH;  // byte offsets in a record
constexpr int kTRec = kRecSc + kTH * kTW / 2;  // + <= 1024 kept scores

constexpr int kFW = kTW + 2, kFH = kTH + 2;  // FAST region (NMS halo)
constexpr int kPG = (kFW + 3) / 4;           // 4-pixel groups of a FAST region row
// image patch: staged column j holds x0 - 5 + j, so FAST position c (x = x0 - 1 + c) sits at
// column c + kIC and a group of 4 positions (c = 4g..4g+3) is the aligned dword g + 1
constexpr int kIC = 4, kIW = kTW + 12, kIH = kTH + 8;

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// bytes 0, 2 / 1, 3 of a dword as two u16 lanes
__device__ __forceinline__ u16x2 bytes02(uint32_t v) { return as_u16x2(__builtin_amdgcn_perm(0u, v, 0x0c020c00u)); }
__device__ __forceinline__ u16x2 bytes13(uint32_t v) { return as_u16x2(__builtin_amdgcn_perm(0u, v, 0x0c030c01u)); }

// FAST prefilter on two pixels (u16 lanes): at least two of the four cardinal circle pixels
// brighter than v + t, or at least two darker than v - t.  With s_k = sat(p_k - (v + t))
// (nonzero = brighter), "two of a, b, c, d nonzero" = max(min(a,b), min(c,d),
// min(max(a,b), max(c,d))) != 0: saturating subtracts and min/max only, all packed.
__device__ __forceinline__ u16x2 two_of_four(u16x2 a, u16x2 b, u16x2 c, u16x2 d) {
  const u16x2 lab = __builtin_elementwise_min(a, b), hab = __builtin_elementwise_max(a, b);
  const u16x2 lcd = __builtin_elementwise_min(c, d), hcd = __builtin_elementwise_max(c, d);
  return __builtin_elementwise_max(__builtin_elementwise_max(lab, lcd), __builtin_elementwise_min(hab, hcd));
}
__device__ __forceinline__ uint32_t fast_pre2(u16x2 v, u16x2 p0, u16x2 p4, u16x2 p8, u16x2 p12, u16x2 t) {
  const u16x2 vt = v + t, vm = __builtin_elementwise_sub_sat(v, t);
  auto br = [&](u16x2 p) { return __builtin_elementwise_sub_sat(p, vt); };
  auto dk = [&](u16x2 p) { return __builtin_elementwise_sub_sat(vm, p); };
  return as_u32(__builtin_elementwise_max(two_of_four(br(p0), br(p4), br(p8), br(p12)),
                                          two_of_four(dk(p0), dk(p4), dk(p8), dk(p12))));
}

// a run of >= 9 set bits on the 16-circle (bit k = circle pixel k): doubling windows
__device__ __forceinline__ bool has9(unsigned m) {
  const unsigned mm = m | (m << 16);
  const unsigned c2 = mm & (mm >> 1), c4 = c2 & (c2 >> 2), c8 = c4 & (c4 >> 4), c9 = c8 & (c8 >> 1);
  return (c9 & 0xFFFFu) != 0;
}

__device__ __forceinline__ int tile_level(const OrbDev& G, int t) {
  int l = 0;
#pragma unroll
  for (int k = 1; k < FVO_MAX_LEVELS; ++k)
    if (k < G.nlevels && t >= G.tile0[k]) l = k;
  return l;
}

template <bool SCOREMAP>
__global__ __launch_bounds__(kFT) void k_fast_nms(const OrbDev G, const uint8_t* __restrict__ pyr,
                                                  uint8_t* __restrict__ score, uint8_t* __restrict__ trec,
                                                  int64_t total, int thr, int edge, int ntiles) {
  __shared__ __attribute__((aligned(16))) uint8_t s_img[kIH][kIW];
  __shared__ __attribute__((aligned(16))) uint8_t s_sc[kFH][kFW];
  __shared__ uint16_t s_list[kFH * kFW];
  __shared__ uint16_t s_pre[kFH * kPG * 4];
  __shared__ uint32_t s_m[kTH][2];  // keep bits of a tile row (64 px), as two dwords
  __shared__ int s_rp[kTH];
  __shared__ int s_n, s_npre;
  // XCD-aware tile order (xcd_block): tiles whose staged aprons share cache lines meet in
  // one L2 instead of being fetched by two XCDs
  const XcdBlock xb = xcd_block();
  const int b = xb.y, t = xb.x;
  const int l = tile_level(G, t);
  const int lt = t - G.tile0[l];
  const int tx = lt % G.ntx[l], ty = lt / G.ntx[l];
  const int x0 = tx * kTW, y0 = ty * kTH;
  const int w = G.w[l], h = G.h[l];
  const uint8_t* im = pyr + b * total + G.off[l];
  if (x0 >= 8 && x0 + kTW + 12 <= w && y0 >= 4 && y0 + kTH + 4 <= h) {
    // interior tile: the staged rows and the aligned dwords around them lie inside the level
    // row, so a row's 76 bytes come from 20 aligned dwords, byte-aligned by v_alignbyte
    for (int i = threadIdx.x; i < kIH * (kIW / 4); i += kFT) {
      const int r = i / (kIW / 4), k = i % (kIW / 4);
      const uint8_t* p = im + (int64_t)(y0 - 4 + r) * w + x0 - 1 - kIC + 4 * k;
      const uint32_t* a = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
      *reinterpret_cast<uint32_t*>(&s_img[r][4 * k]) = __builtin_amdgcn_alignbyte(a[1], a[0], sh);
    }
  } else {
    for (int i = threadIdx.x; i < kIH * kIW; i += kFT) {
      const int r = i / kIW, c = i % kIW;
      const int y = min(max(y0 - 4 + r, 0), h - 1), x = min(max(x0 - 1 - kIC + c, 0), w - 1);
      s_img[r][c] = im[(int64_t)y * w + x];
    }
  }
  for (int i = threadIdx.x; i < kFH * kFW / 4; i += kFT) reinterpret_cast<uint32_t*>(&s_sc[0][0])[i] = 0;
  if (threadIdx.x < 2 * kTH) (&s_m[0][0])[threadIdx.x] = 0u;
  if (threadIdx.x == 0) { s_n = 0; s_npre = 0; }
  __syncthreads();
  // FAST-9 on the tile + halo in two compacted stages.  (1) A 9-arc of the 16-circle always
  // holds at least two of the four cardinal pixels (0, 4, 8, 12), so a position with fewer
  // than two cardinals brighter than v+t and fewer than two darker than v-t cannot be a
  // corner; the rest go to a pre-list.  This stage runs on 4 positions per lane: the centre
  // and cardinal bytes of the group are 5 dword reads, tested as u16 pairs (saturating
  // subtracts).  (2) The full 16-pixel test on the pre-list; corners go to the list.  Same
  // corners as testing every position.
  const u16x2 tt = {(unsigned short)thr, (unsigned short)thr};
  for (int i0 = 0; i0 < kFH * kPG; i0 += kFT) {  // uniform trip count: ballots see whole waves
    const int i = i0 + threadIdx.x;
    const int r = i / kPG, g = i % kPG;
    const int y = y0 - 1 + r, xg = x0 - 1 + 4 * g;
    unsigned f = 0;
    if (i < kFH * kPG && y >= 3 && y < h - 3) {
      const uint32_t* rc = reinterpret_cast<const uint32_t*>(&s_img[r + 3][0]);
      const uint32_t dv = rc[g + 1];
      const uint32_t d0 = reinterpret_cast<const uint32_t*>(&s_img[r + 6][0])[g + 1];  // circle 0: dy +3
      const uint32_t d8 = reinterpret_cast<const uint32_t*>(&s_img[r][0])[g + 1];      // circle 8: dy -3
      const uint32_t d4 = __builtin_amdgcn_alignbyte(rc[g + 2], dv, 3);                 // circle 4: dx +3
      const uint32_t d12 = __builtin_amdgcn_alignbyte(dv, rc[g], 1);                    // circle 12: dx -3
      const uint32_t e = fast_pre2(bytes02(dv), bytes02(d0), bytes02(d4), bytes02(d8), bytes02(d12), tt);
      const uint32_t o = fast_pre2(bytes13(dv), bytes13(d0), bytes13(d4), bytes13(d8), bytes13(d12), tt);
      f = (unsigned)((e & 0xFFFFu) != 0) | (unsigned)((o & 0xFFFFu) != 0) << 1 | (unsigned)((e >> 16) != 0) << 2 |
          (unsigned)((o >> 16) != 0) << 3;
      // positions inside the region and 3 px from the level's sides
      const int lo = max(3 - xg, 0), hi = min(min(w - 3 - xg, kFW - 4 * g), 4);
      f &= hi > lo ? ((1u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
    }
    const unsigned long long m0 = __ballot(f & 1u), m1 = __ballot(f & 2u), m2 = __ballot(f & 4u),
                             m3 = __ballot(f & 8u);
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    int pos = __popcll(m0 & below) + __popcll(m1 & below) + __popcll(m2 & below) + __popcll(m3 & below);
    int base = 0;
    const int tot = __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
    if (lane == 0 && tot) base = atomicAdd(&s_npre, tot);
    pos += __shfl(base, 0, 64);
    const int ib = r * kFW + 4 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((f >> j) & 1u) s_pre[pos++] = (uint16_t)(ib + j);
  }
  __syncthreads();
  const int npre = s_npre;
  for (int j0 = 0; j0 < npre; j0 += kFT) {  // uniform trip count
    const int j = j0 + threadIdx.x;
    bool corner = false;
    int i = 0;
    if (j < npre) {
      i = s_pre[j];
      const int r = i / kFW, c = i % kFW;
      const int v = s_img[r + 3][c + kIC];
      // circle pixels k and k + 8 share a dword (u16 lanes); the sign bit of (v + t) - p
      // (bright) / p - (v - t) (dark) is shifted to bit k of its lane and merged into the mask
      const u16x2 vt = {(unsigned short)(v + thr), (unsigned short)(v + thr)};
      const u16x2 vm = {(unsigned short)(v - thr), (unsigned short)(v - thr)};
      uint32_t ab = 0, ad = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t pk = (uint32_t)s_img[r + 3 + c_cdy[k]][c + kIC + c_cdx[k]] |
                            (uint32_t)s_img[r + 3 + c_cdy[k + 8]][c + kIC + c_cdx[k + 8]] << 16;
        const u16x2 sh = {(unsigned short)(15 - k), (unsigned short)(15 - k)};
        const uint32_t K = 0x10001u << k;
        ab |= as_u32((vt - as_u16x2(pk)) >> sh) & K;
        ad |= as_u32((as_u16x2(pk) - vm) >> sh) & K;
      }
      // lanes -> 16-bit masks: bits 0..7 from the low lane, 8..15 from the high lane
      const unsigned bright = __builtin_amdgcn_perm(0u, ab, 0x0c0c0200u);
      const unsigned dark = __builtin_amdgcn_perm(0u, ad, 0x0c0c0200u);
      corner = has9(bright) || has9(dark);
    }
    const unsigned long long m = __ballot(corner);
    int base = 0;
    if ((threadIdx.x & 63) == 0 && m) base = atomicAdd(&s_n, __popcll(m));
    base = __shfl(base, 0, 64);
    if (corner) s_list[base + __popcll(m & ((1ull << (threadIdx.x & 63)) - 1ull))] = (uint16_t)i;
  }
  __syncthreads();
  // cornerScore<16>: max(t, max over 9-arcs of min(v-p), max over 9-arcs of min(p-v)) - 1
  const int nc = s_n;
  for (int j = threadIdx.x; j < nc; j += kFT) {
    const int i = s_list[j];
    const int r = i / kFW, c = i % kFW;
    const int v = s_img[r + 3][c + kIC];
    // the minimum / maximum of d = v - p over every 9-arc of the circle by doubling windows
    // (2, 4, 8, then + 1): 128 min/max instead of 2 x 16 x 9 -- exact, order-free
    int d[16], n2[16], x2[16], n4[16], x4[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = v - (int)s_img[r + 3 + c_cdy[k]][c + kIC + c_cdx[k]];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      n2[k] = min(d[k], d[(k + 1) & 15]);
      x2[k] = max(d[k], d[(k + 1) & 15]);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      n4[k] = min(n2[k], n2[(k + 2) & 15]);
      x4[k] = max(x2[k], x2[(k + 2) & 15]);
    }
    int a0 = thr, b0 = thr;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int n9 = min(min(n4[k], n4[(k + 4) & 15]), d[(k + 8) & 15]);
      const int x9 = max(max(x4[k], x4[(k + 4) & 15]), d[(k + 8) & 15]);
      a0 = max(a0, n9);   // max over arcs of min(v - p)
      b0 = max(b0, -x9);  // max over arcs of min(p - v)
    }
    s_sc[r][c] = (uint8_t)(max(a0, b0) - 1);
  }
  __syncthreads();
  if (SCOREMAP) {  // debug hook: the score of every tile pixel (0 = no corner)
    const int c = threadIdx.x & 63, x = x0 + c;
    for (int rr = threadIdx.x >> 6; rr < kTH; rr += kFT / 64) {
      const int y = y0 + rr;
      if (y < h && x < w) score[b * total + G.off[l] + (int64_t)y * w + x] = s_sc[rr + 1][c + 1];
    }
    return;
  }
  // strict 3x3 NMS + border filter, on the corners only (every other pixel scores 0): a kept
  // corner sets its bit in its row's keep word and is marked in the list
  for (int j = threadIdx.x; j < nc; j += kFT) {
    const int i = s_list[j];
    const int r = i / kFW, c = i % kFW;
    const int x = x0 - 1 + c, y = y0 - 1 + r;
    if (r < 1 || r > kTH || c < 1 || c > kTW || x >= w - edge || y >= h - edge || x < edge || y < edge) continue;
    const int sv = s_sc[r][c];
    const bool k = sv && sv > s_sc[r - 1][c - 1] && sv > s_sc[r - 1][c] && sv > s_sc[r - 1][c + 1] && sv > s_sc[r][c - 1] &&
                   sv > s_sc[r][c + 1] && sv > s_sc[r + 1][c - 1] && sv > s_sc[r + 1][c] && sv > s_sc[r + 1][c + 1];
    if (k) {
      atomicOr(&s_m[r - 1][(c - 1) >> 5], 1u << ((c - 1) & 31));
      s_list[j] = (uint16_t)(i | 0x8000);
    }
  }
  __syncthreads();
  // tile-local prefix of the rows' keep counts (rows past the level's end hold none)
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    const int v = c < kTH ? __popc(s_m[c][0]) + __popc(s_m[c][1]) : 0;
    int inc = v;
#pragma unroll
    for (int o = 1; o < kTH; o <<= 1) {
      const int u = __shfl_up(inc, o, 64);
      if (c >= o) inc += u;
    }
    if (c < kTH) s_rp[c] = inc - v;
  }
  __syncthreads();
  uint8_t* rec = trec + ((int64_t)b * ntiles + t) * kTRec;
  if (threadIdx.x < kTH)
    reinterpret_cast<unsigned long long*>(rec + kRecKeep)[threadIdx.x] =
        (unsigned long long)s_m[threadIdx.x][0] | (unsigned long long)s_m[threadIdx.x][1] << 32;
  else if (threadIdx.x < 2 * kTH)
    reinterpret_cast<uint16_t*>(rec + kRecPre)[threadIdx.x - kTH] = (uint16_t)s_rp[threadIdx.x - kTH];
  for (int j = threadIdx.x; j < nc; j += kFT) {
    const int e = s_list[j];
    if (!(e & 0x8000)) continue;
    const int i = e & 0x7FFF;
    const int r = i / kFW, c = i % kFW;
    const unsigned long long m = (unsigned long long)s_m[r - 1][0] | (unsigned long long)s_m[r - 1][1] << 32;
    rec[kRecSc + s_rp[r - 1] + __popcll(m & ((1ull << (c - 1)) - 1ull))] = s_sc[r][c];
  }
}

// ------------------------------------------------------------------ retainBest
// Element views: key() is the KeyPoint.response the comparator looks at.
struct ElemFast {
  typedef uint32_t T;
  __device__ static float key(uint32_t e) { return (float)(e >> 24); }
};
struct ElemHarris {
  typedef uint64_t T;
  __device__ static float key(uint64_t e) { return __uint_as_float((uint32_t)(e >> 32)); }
};

struct SelShared {
  int wsum[2][kSelThreads / 64];
  int carry[2];
  int cnt;
  int lo, hi, cut;
};

// Block-wide exclusive scan of two per-thread counts (< 2^NB); returns the prefixes (including the
// running carries) and advances the carries (uniform afterwards).
template <int NB = 6>
__device__ __forceinline__ void scan2(SelShared& sh, int v0, int v1, int& p0, int& p1) {
  const int lane = wave_lane(), wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // wave exclusive prefixes and totals of counts in [0, 2^NB), bit-sliced: one ballot per bit
  const unsigned long long below = (1ull << lane) - 1ull;
  int e0 = 0, e1 = 0, s0 = 0, s1 = 0;
#pragma unroll
  for (int bt = 0; bt < NB; ++bt) {
    const unsigned long long m0 = __ballot((v0 >> bt) & 1), m1 = __ballot((v1 >> bt) & 1);
    e0 += __popcll(m0 & below) << bt;
    e1 += __popcll(m1 & below) << bt;
    s0 += __popcll(m0) << bt;
    s1 += __popcll(m1) << bt;
  }
  if (lane == 0) { sh.wsum[0][wid] = s0; sh.wsum[1][wid] = s1; }
  __syncthreads();
  int a0 = 0, a1 = 0, t0 = 0, t1 = 0;
  for (int i = 0; i < nw; ++i) {
    const int w0 = sh.wsum[0][i], w1 = sh.wsum[1][i];
    if (i < wid) { a0 += w0; a1 += w1; }
    t0 += w0; t1 += w1;
  }
  p0 = sh.carry[0] + a0 + e0;
  p1 = sh.carry[1] + a1 + e1;
  __syncthreads();
  if (threadIdx.x == 0) { sh.carry[0] += t0; sh.carry[1] += t1; }
  __syncthreads();
}

// block sum of per-thread counts in [0, 2^NB)
template <int NB>
__device__ __forceinline__ int block_sum(SelShared& sh, int v) {
  int x = 0;
#pragma unroll
  for (int bt = 0; bt < NB; ++bt) x += __popcll(__ballot((v >> bt) & 1)) << bt;
  if (wave_lane() == 0) sh.wsum[0][threadIdx.x >> 6] = x;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh.wsum[0][i];
  __syncthreads();
  return t;
}

// Elements per thread of one scan pass (bits of a u32 flag word): a range of up to
// kSelThreads * kSelPer positions costs one block scan, not one per kSelThreads.
constexpr int kSelPer = 32;

// Compact positions i in [first,last) with predicate A (ascending into SA) and B
// (ascending into SB).  Returns counts.  Each thread takes a run of consecutive positions,
// so thread order = position order and one exclusive scan of the per-thread counts places
// every position.
template <class E, class I, class PA, class PB>
__device__ void compact2(SelShared& sh, const typename E::T* a, int first, int last, I* SA, I* SB, PA pa, PB pb,
                         int& nA, int& nB) {
  if (threadIdx.x == 0) { sh.carry[0] = 0; sh.carry[1] = 0; }
  __syncthreads();
  for (int base = first; base < last; base += (int)blockDim.x * kSelPer) {
    const int len = min(last - base, (int)blockDim.x * kSelPer);
    const int per = (len + (int)blockDim.x - 1) / (int)blockDim.x;
    const int i0 = base + (int)threadIdx.x * per, i1 = min(i0 + per, base + len);
    uint32_t ma = 0, mb = 0;
    for (int i = i0; i < i1; ++i) {
      const float k = E::key(a[i]);
      ma |= (uint32_t)pa(k) << (i - i0);
      mb |= (uint32_t)pb(k) << (i - i0);
    }
    int p0, p1;
    if (per == 1) scan2<1>(sh, (int)ma, (int)mb, p0, p1);  // uniform: flags, one ballot each
    else scan2<6>(sh, __popc(ma), __popc(mb), p0, p1);
    while (ma) {
      const int j = __builtin_ctz(ma);
      ma &= ma - 1u;
      SA[p0++] = (I)(i0 + j);
    }
    while (mb) {
      const int j = __builtin_ctz(mb);
      mb &= mb - 1u;
      SB[p1++] = (I)(i0 + j);
    }
  }
  nA = sh.carry[0];
  nB = sh.carry[1];
  __syncthreads();
}

// Pair the k-th A position (ascending) with the k-th B position from the right while
// A_k < B_k; swap each pair.  This is exactly the set of swaps a sequential Hoare scan
// (libstdc++ __unguarded_partition / bidirectional __partition) performs.  Returns k*
// (the predicate is monotone in k -- A_k rises, B_{nB-1-k} falls -- so k* is its count).
template <class E, class I>
__device__ int pair_swap(SelShared& sh, typename E::T* a, const I* SA, int nA, const I* SB, int nB) {
  const int m = min(nA, nB);
  int c = 0;
  for (int base = 0; base < m; base += (int)blockDim.x * kSelPer) {
    const int len = min(m - base, (int)blockDim.x * kSelPer);
    const int per = (len + (int)blockDim.x - 1) / (int)blockDim.x;
    const int k0 = base + (int)threadIdx.x * per, k1 = min(k0 + per, base + len);
    int f = 0;
    for (int k = k0; k < k1; ++k) f += (int)SA[k] < (int)SB[nB - 1 - k];
    c += per == 1 ? block_sum<1>(sh, f) : block_sum<6>(sh, f);
  }
  for (int k = threadIdx.x; k < c; k += blockDim.x) {
    int i = SA[k], j = SB[nB - 1 - k];
    typename E::T t = a[i];
    a[i] = a[j];
    a[j] = t;
  }
  __syncthreads();
  return c;
}

// ---- serial pieces (lane 0), libstdc++ semantics with comp(x,y) = key(x) > key(y)
template <class E>
__device__ void move_median_to_first(typename E::T* a, int result, int ia, int ib, int ic) {
  auto cmp = [&](int x, int y) { return E::key(a[x]) > E::key(a[y]); };
  auto sw = [&](int x, int y) { typename E::T t = a[x]; a[x] = a[y]; a[y] = t; };
  if (cmp(ia, ib)) {
    if (cmp(ib, ic)) sw(result, ib);
    else if (cmp(ia, ic)) sw(result, ic);
    else sw(result, ia);
  } else if (cmp(ia, ic)) sw(result, ia);
  else if (cmp(ib, ic)) sw(result, ic);
  else sw(result, ib);
}

template <class E>
__device__ void insertion_sort(typename E::T* a, int first, int last) {
  if (first == last) return;
  for (int i = first + 1; i != last; ++i) {
    typename E::T v = a[i];
    float kv = E::key(v);
    if (kv > E::key(a[first])) {
      for (int j = i; j > first; --j) a[j] = a[j - 1];
      a[first] = v;
    } else {
      int j = i, nx = i - 1;
      while (kv > E::key(a[nx])) { a[j] = a[nx]; j = nx; --nx; }
      a[j] = v;
    }
  }
}

template <class E>
__device__ void adjust_heap(typename E::T* f, int hole, int len, typename E::T value) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (E::key(f[second]) > E::key(f[second - 1])) second--;
    f[hole] = f[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    f[hole] = f[second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  float kv = E::key(value);
  while (hole > top && E::key(f[parent]) > kv) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = value;
}

template <class E>
__device__ void heap_select(typename E::T* a, int first, int middle, int last) {
  typename E::T* f = a + first;
  int len = middle - first;
  if (len >= 2) {
    for (int parent = (len - 2) / 2;; --parent) {
      adjust_heap<E>(f, parent, len, f[parent]);
      if (parent == 0) break;
    }
  }
  for (int i = middle; i < last; ++i) {
    if (E::key(a[i]) > E::key(f[0])) {
      typename E::T v = a[i];
      a[i] = f[0];
      adjust_heap<E>(f, 0, len, v);
    }
  }
}

__device__ __forceinline__ int ilog2(int n) { return 31 - __clz(n); }

// KeyPointsFilter::retainBest(a[0..n), keep) executed by one workgroup.  Returns the
// surviving count; a[] is left in OpenCV's element order.
template <class E, class I>
__device__ int select_block(SelShared& sh, typename E::T* a, int n, int keep, I* SA, I* SB) {
  if (keep < 0 || n <= keep) return n;
  if (keep == 0) return 0;
  const int nth = keep - 1;
  int lo = 0, hi = n, depth = 2 * ilog2(n);
  bool heaped = false;
  while (hi - lo > 3) {
    if (depth == 0) {
      if (threadIdx.x == 0) {
        heap_select<E>(a, lo, nth + 1, hi);
        typename E::T t = a[lo]; a[lo] = a[nth]; a[nth] = t;
      }
      __syncthreads();
      heaped = true;
      break;
    }
    --depth;
    if (threadIdx.x == 0) move_median_to_first<E>(a, lo, lo + 1, lo + (hi - lo) / 2, hi - 1);
    __syncthreads();
    const float P = E::key(a[lo]);
    int nL, nR;
    compact2<E, I>(sh, a, lo + 1, hi, SA, SB, [P](float k) { return k <= P; }, [P](float k) { return k >= P; }, nL, nR);
    int ks = pair_swap<E, I>(sh, a, SA, nL, SB, nR);
    int Lk = ks < nL ? SA[ks] : hi;
    int Rk = ks > 0 ? SB[nR - ks] : hi;
    int cut = min(Lk, Rk);
    if (cut <= nth) lo = cut; else hi = cut;
  }
  if (!heaped) {
    if (threadIdx.x == 0) insertion_sort<E>(a, lo, hi);
    __syncthreads();
  }
  const float amb = E::key(a[nth]);
  int nF, nG;
  compact2<E, I>(sh, a, keep, n, SA, SB, [amb](float k) { return !(k >= amb); }, [amb](float k) { return k >= amb; },
                 nF, nG);
  pair_swap<E, I>(sh, a, SA, nF, SB, nG);
  return keep + nG;
}

// Ordered (row-major) compaction of level l's kept pixels from the tile records k_fast_nms
// wrote: (row, tile) keep words in row-major order, a thread per run of up to kCmpPer
// consecutive words (all loads in flight at once), one block scan of the runs' counts, each
// word's pixels written at its offset -- (score << 24 | y << 12 | x), the order cv::FAST lists
// keypoints in.  Candidates go to the global array and, while they fit, to the LDS copy.
// Returns the count.
constexpr int kCmpPer = 16;
template <int CAP>
__device__ int compact_level(SelShared& sh, const OrbDev& G, const uint8_t* __restrict__ trec, int ntiles, int edge,
                             int l, int b, uint32_t* __restrict__ out, uint32_t* s_out) {
  const int h = G.h[l], ntx = G.ntx[l];
  const int ya = edge, yb = h - edge;  // the NMS border filter keeps nothing outside
  const int npairs = yb > ya ? (yb - ya) * ntx : 0;
  const uint8_t* lrec = trec + ((int64_t)b * ntiles + G.tile0[l]) * kTRec;
  if (threadIdx.x == 0) { sh.carry[0] = 0; sh.carry[1] = 0; }
  __syncthreads();
  for (int base = 0; base < npairs; base += (int)blockDim.x * kCmpPer) {
    const int len = min(npairs - base, (int)blockDim.x * kCmpPer);
    const int per = (len + (int)blockDim.x - 1) / (int)blockDim.x;
    const int q0 = base + (int)threadIdx.x * per, q1 = min(q0 + per, base + len);
    const int y0 = ya + q0 / ntx, tx0 = q0 - (y0 - ya) * ntx;
    unsigned long long w[kCmpPer];
    int cnt = 0;
#pragma unroll
    for (int j = 0, y = y0, tx = tx0; j < kCmpPer; ++j) {
      w[j] = 0;
      if (q0 + j < q1)
        w[j] = reinterpret_cast<const unsigned long long*>(lrec + (int64_t)((y / kTH) * ntx + tx) * kTRec +
                                                           kRecKeep)[y % kTH];
      cnt += __popcll(w[j]);
      if (++tx == ntx) { tx = 0; ++y; }
    }
    int o, o1;
    scan2<11>(sh, cnt, 0, o, o1);  // <= kCmpPer * 64
#pragma unroll
    for (int j = 0, y = y0, tx = tx0; j < kCmpPer; ++j) {
      unsigned long long word = w[j];
      if (word) {
        const uint8_t* rec = lrec + (int64_t)((y / kTH) * ntx + tx) * kTRec;
        const uint8_t* sc = rec + kRecSc + reinterpret_cast<const uint16_t*>(rec + kRecPre)[y % kTH];
        for (int k = 0; word; ++k) {
          const int bit = __builtin_ctzll(word);
          word &= word - 1ull;
          const uint32_t e = ((uint32_t)sc[k] << 24) | ((uint32_t)y << 12) | (uint32_t)(64 * tx + bit);
          out[o] = e;
          if (o < CAP) s_out[o] = e;
          ++o;
        }
      }
      if (++tx == ntx) { tx = 0; ++y; }
    }
  }
  return sh.carry[0];
}

// KeyPointsFilter::retainBest on one (image, level) per block.  The array and the two
// position lists live in LDS while the level's count fits (CAP), else in global memory (the
// same code, on the global array and the scratch lists).  COMPACT: the candidates are first
// compacted from the FAST tile records (the first retainBest of ORB); otherwise they are
// read from arr (the Harris retainBest).  The first r elements of the result go back to arr.
template <class E, int CAP, bool COMPACT>
__global__ __launch_bounds__(kSelThreads, 4) void k_select(const OrbDev G, const uint8_t* __restrict__ trec, int ntiles,
                                                        int edge, typename E::T* __restrict__ arr,
                                                        int32_t* __restrict__ nin, int32_t* __restrict__ nout,
                                                        int32_t* __restrict__ scratch, int64_t scratch_per,
                                                        int64_t cand_total, int nlevels, int keep_mult) {
  using T = typename E::T;
  const int b = blockIdx.x, l = blockIdx.y;  // level-major dispatch: the large level-0 blocks start first
  __shared__ SelShared sh;
  __shared__ T s_a[CAP];
  __shared__ uint16_t s_pa[CAP], s_pb[CAP];
  T* a = arr + b * cand_total + G.cand_off[l];
  int n;
  if constexpr (COMPACT) {
    n = compact_level<CAP>(sh, G, trec, ntiles, edge, l, b, a, s_a);
    if (threadIdx.x == 0) nin[b * nlevels + l] = n;
  } else {
    n = nin[b * nlevels + l];
    if (n <= CAP)
      for (int i = threadIdx.x; i < n; i += blockDim.x) s_a[i] = a[i];
  }
  __syncthreads();
  const int keep = keep_mult * G.nfeat[l];
  int r;
  if (n <= CAP) {
    r = select_block<E, uint16_t>(sh, s_a, n, keep, s_pa, s_pb);
    // the selection permutes the array whenever it runs (n > keep), even when ties keep all
    // n; only an untouched compacted array is already in place
    if (n > keep || !COMPACT)
      for (int i = threadIdx.x; i < r; i += blockDim.x) a[i] = s_a[i];
  } else {
    int* SA = scratch + (int64_t)(b * nlevels + l) * scratch_per;
    r = select_block<E, int>(sh, a, n, keep, SA, SA + scratch_per / 2);
  }
  if (threadIdx.x == 0) nout[b * nlevels + l] = r;
}

// ------------------------------------------------------------------ Harris
__global__ void k_harris(const OrbDev G, const uint8_t* __restrict__ pyr, const uint32_t* __restrict__ cand,
                         const int32_t* __restrict__ nsel, uint64_t* __restrict__ hel, int64_t total,
                         int64_t cand_total, int nlevels) {
  const XcdBlock xb = xcd_block();  // one (image, level)'s blocks on one XCD: shared patches in one L2
  int l = xb.y, b = xb.z;
  int n = nsel[b * nlevels + l];
  int wpb = blockDim.x >> 6;
  int lane = wave_lane();
  const uint8_t* im = pyr + b * total + G.off[l];
  int w = G.w[l];
  const uint32_t* cin = cand + b * cand_total + G.cand_off[l];
  uint64_t* hout = hel + b * cand_total + G.cand_off[l];
  for (int i = xb.x * wpb + (threadIdx.x >> 6); i < n; i += gridDim.x * wpb) {
    uint32_t e = cin[i];
    int x0 = e & 0xFFF, y0 = (e >> 12) & 0xFFF;
    int A = 0, B = 0, C = 0;
    if (lane < 49) {
      int x = x0 - 3 + lane % 7, y = y0 - 3 + lane / 7;
      const uint8_t* p = im + (int64_t)y * w + x;
      int Ix = (p[1] - p[-1]) * 2 + (p[-w + 1] - p[-w - 1]) + (p[w + 1] - p[w - 1]);
      int Iy = (p[w] - p[-w]) * 2 + (p[w - 1] - p[-w - 1]) + (p[w + 1] - p[-w + 1]);
      A = Ix * Ix; B = Iy * Iy; C = Ix * Iy;
    }
    A = wave_sum(A); B = wave_sum(B); C = wave_sum(C);
    if (lane == 0) {
      const float harris_k = 0.04f;
      const float scale = 1.f / ((1 << 2) * 7 * 255.f);
      const float sss = scale * scale * scale * scale;
      float resp = ((float)A * B - (float)C * C - harris_k * ((float)A + B) * ((float)A + B)) * sss;
      hout[i] = ((uint64_t)__float_as_uint(resp) << 32) | e;
    }
  }
}

// ------------------------------------------------------------------ finalize + angle
__global__ void k_offsets(const int32_t* __restrict__ nsel2, int32_t* __restrict__ koff, int32_t* __restrict__ counts,
                          int batch, int nlevels, int cap) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  int s = 0;
  for (int l = 0; l < nlevels; ++l) {
    koff[b * (nlevels + 1) + l] = s;
    s += nsel2[b * nlevels + l];
  }
  koff[b * (nlevels + 1) + nlevels] = s;
  counts[b] = s <= cap ? s : -s;
}

__device__ __forceinline__ float fast_atan2_deg(float y, float x) {
  const float k = (float)(180 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k, p5 = 0.1555786518463281f * k,
              p7 = -0.04432655554792128f * k;
  const float eps = (float)2.220446049250313080847e-16;
  float ax = fabsf(x), ay = fabsf(y), a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

__global__ void k_angle(const OrbDev G, const uint8_t* __restrict__ pyr, const uint64_t* __restrict__ hel,
                        const int32_t* __restrict__ nsel2, const int32_t* __restrict__ koff, float* __restrict__ kp,
                        int64_t total, int64_t cand_total, int nlevels, int cap, int patch) {
  const XcdBlock xb = xcd_block();
  int l = xb.y, b = xb.z;
  int n = nsel2[b * nlevels + l];
  int base = koff[b * (nlevels + 1) + l];
  int wpb = blockDim.x >> 6, lane = wave_lane();
  const uint8_t* im = pyr + b * total + G.off[l];
  int w = G.w[l];
  const uint64_t* hin = hel + b * cand_total + G.cand_off[l];
  const int half = patch / 2;
  for (int i = xb.x * wpb + (threadIdx.x >> 6); i < n; i += gridDim.x * wpb) {
    if (base + i >= cap) break;
    uint64_t e = hin[i];
    int x0 = (int)(e & 0xFFF), y0 = (int)((e >> 12) & 0xFFF);
    float resp = __uint_as_float((uint32_t)(e >> 32));
    const uint8_t* c = im + (int64_t)y0 * w + x0;
    int m10 = 0, m01 = 0;
    int u = lane - half;
    if (lane <= 2 * half) {
      m10 += u * c[u];
      if (half == 15) {
        // the usual patch (31): every row's two bytes loaded unconditionally (keypoints lie at
        // least edgeThreshold >= 15 px inside the level) and masked by the circle afterwards,
        // so the 30 loads are in flight together instead of one round trip per row
        int vp[15], vm[15];
#pragma unroll
        for (int v = 1; v <= 15; ++v) {
          vp[v - 1] = c[u + v * w];
          vm[v - 1] = c[u - v * w];
        }
#pragma unroll
        for (int v = 1; v <= 15; ++v) {
          const int d = c_umax[v];
          if (u >= -d && u <= d) {
            m01 += v * (vp[v - 1] - vm[v - 1]);
            m10 += u * (vp[v - 1] + vm[v - 1]);
          }
        }
      } else {
        for (int v = 1; v <= half; ++v) {
          int d = c_umax[v];
          if (u >= -d && u <= d) {
            int vp = c[u + v * w], vm = c[u - v * w];
            m01 += v * (vp - vm);
            m10 += u * (vp + vm);
          }
        }
      }
    }
    m10 = wave_sum(m10);
    m01 = wave_sum(m01);
    if (lane == 0) {
      float s = G.scale[l];
      float* o = kp + ((int64_t)b * cap + base + i) * FVO_KP_STRIDE;
      o[0] = (float)x0 * s;
      o[1] = (float)y0 * s;
      o[2] = patch * s;
      o[3] = fast_atan2_deg((float)m01, (float)m10);
      o[4] = resp;
      o[5] = (float)l;
      o[6] = -1.f;
      o[7] = 0.f;
    }
  }
}

// ------------------------------------------------------------------ Gaussian blur
// 7x7 sigma-2 fixed-point kernel [18 34 49 55 49 34 18] (x) itself, REFLECT_101, on 64 x 16
// tiles: the patch + 3-px apron is staged in LDS, the horizontal pass keeps exact integer
// row sums in LDS, the vertical pass rounds once (the integer result is the separable
// 8-bit path's, any summation order).
__constant__ int c_gk[7] = {18, 34, 49, 55, 49, 34, 18};

__device__ __forceinline__ int reflect101(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// GaussianBlur 7x7 sigma 2 (8-bit fixed point, BORDER_REFLECT_101 per level).  Block = a
// 256 x 32 output tile: the (32+6) x (256+6) input patch is staged in LDS once, then each
// thread owns one column and streams down the 38 input rows, computing the horizontal 7-tap
// sum from LDS and the vertical 7-tap sum from a 7-entry register window (the row loop is
// unrolled, so the window is static registers).  Read amplification 1.2x, one byte store
// per pixel (64 B per wave instruction).
constexpr int kBW = 256, kBH = 32;

__device__ __forceinline__ int btile_level(const OrbDev& G, int t) {
  int l = 0;
#pragma unroll
  for (int k = 1; k < FVO_MAX_LEVELS; ++k)
    if (k < G.nlevels && t >= G.btile0[k]) l = k;
  return l;
}

__global__ __launch_bounds__(256) void k_blur(const OrbDev G, const uint8_t* __restrict__ pyr,
                                              uint8_t* __restrict__ blur, int64_t total) {
  constexpr int RW = kBW + 6, RH = kBH + 6;
  __shared__ uint8_t s_img[RH][RW + 2];
  const int b = blockIdx.y, t = blockIdx.x;
  const int l = btile_level(G, t);
  const int lt = t - G.btile0[l];
  const int tx = lt % G.bntx[l], ty = lt / G.bntx[l];
  const int x0 = tx * kBW, y0 = ty * kBH;
  const int w = G.w[l], h = G.h[l];
  const uint8_t* im = pyr + b * total + G.off[l];
  for (int r = 0; r < RH; ++r) {
    const int y = reflect101(min(y0 - 3 + r, 2 * (h - 1)), h);
    const uint8_t* row = im + (int64_t)y * w;
    for (int c = threadIdx.x; c < RW; c += 256) s_img[r][c] = row[reflect101(min(x0 - 3 + c, 2 * (w - 1)), w)];
  }
  __syncthreads();
  const int c = threadIdx.x, x = x0 + c;
  uint8_t* out = blur + b * total + G.off[l] + x;
  const bool xin = x < w;
  int win[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < RH; ++r) {
    int hs = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) hs += c_gk[k] * s_img[r][c + k];
#pragma unroll
    for (int j = 0; j < 6; ++j) win[j] = win[j + 1];
    win[6] = hs;
    if (r >= 6) {
      const int y = y0 + r - 6;
      int sv = 0;
#pragma unroll
      for (int j = 0; j < 7; ++j) sv += c_gk[j] * win[j];
      const int q = (sv + 32767 + ((sv >> 16) & 1)) >> 16;  // round half to even
      if (xin && y < h) out[(int64_t)y * w] = (uint8_t)min(q, 255);
    }
  }
}

// ------------------------------------------------------------------ rBRIEF
// The descriptor reads the blurred level only at its 512 rotated pattern samples, all within
// 19 px of the keypoint (|pattern| <= 13 * sqrt 2), so the blur is computed for that patch
// only instead of for the whole pyramid: one wave per keypoint stages the 45 x 45 source patch
// (REFLECT_101 resolved while staging, as k_blur does) in LDS, lanes 0..38 each stream one
// column down the 45 rows with the horizontal 7-tap sum from LDS and the vertical 7-tap sum
// from a register window -- exactly k_blur's integer arithmetic and rounding -- into a 39 x 39
// blurred patch in LDS, then the samples are compared from it (4 ballots = the 32 bytes).
constexpr int kBrR = 19, kBrP = 2 * kBrR + 1, kBrS = kBrP + 6;  // sample radius, blurred / source side
constexpr int kBrSW = kBrS + 3, kBrPW = kBrP + 1;                // LDS row pitches

__global__ __launch_bounds__(256, 4) void k_brief(const OrbDev G, const uint8_t* __restrict__ pyr,
                                               const float* __restrict__ kp, const int32_t* __restrict__ counts,
                                               uint8_t* __restrict__ desc, int64_t total, int cap) {
  __shared__ __attribute__((aligned(16))) uint8_t s_src[4][kBrS][kBrSW];
  __shared__ uint8_t s_blr[4][kBrP][kBrPW];
  const XcdBlock xb = xcd_block();  // one image's blocks on one XCD: overlapping patches in one L2
  const int b = xb.y;
  const int n = counts[b];
  if (n < 0) return;
  const int wpb = blockDim.x >> 6, lane = wave_lane(), wv = threadIdx.x >> 6;
  uint8_t(*src)[kBrSW] = s_src[wv];
  uint8_t(*blr)[kBrPW] = s_blr[wv];
  for (int j = xb.x * wpb + wv; j < n; j += gridDim.x * wpb) {
    const float* k = kp + ((int64_t)b * cap + j) * FVO_KP_STRIDE;
    const int l = (int)k[5];
    const float scale = 1.f / G.scale[l];
    float angle = k[3];
    angle *= (float)(3.14159265358979323846 / 180.f);
    const float a = (float)cos((double)angle), bb = (float)sin((double)angle);
    const int cy = (int)rintf(k[1] * scale), cx = (int)rintf(k[0] * scale);
    const int w = G.w[l], h = G.h[l];
    const uint8_t* im = pyr + b * total + G.off[l];
    const int sx0 = cx - kBrR - 3, sy0 = cy - kBrR - 3;
    if (sx0 >= 0 && sy0 >= 0 && sx0 + kBrS <= w && sy0 + kBrS <= h) {
      // the usual case (keypoints lie edgeThreshold >= 31 px inside their level, the patch
      // reaches 22): no border handling, each row's 48 bytes as 12 dwords from aligned loads
      // (v_alignbyte), all 9 of a lane's loads in flight together
      constexpr int kRW = kBrSW / 4, kN = kBrS * kRW, kIt = (kN + 63) / 64;
      const uint8_t* p0 = im + (int64_t)sy0 * w + sx0;
#pragma unroll
      for (int t = 0; t < kIt; ++t) {
        const int i = min(lane + 64 * t, kN - 1);
        const int r = i / kRW, q = i - r * kRW;
        const uintptr_t pa = reinterpret_cast<uintptr_t>(p0 + r * w + 4 * q);
        const uint32_t* a4 = reinterpret_cast<const uint32_t*>(pa & ~(uintptr_t)3);
        const uint32_t v = __builtin_amdgcn_alignbyte(a4[1], a4[0], (uint32_t)pa & 3u);
        if (lane + 64 * t < kN) reinterpret_cast<uint32_t*>(&src[r][0])[q] = v;
      }
    } else {
      // a patch crossing the level's border (REFLECT_101 per byte): not reached by keypoints
      // of the default edgeThreshold, kept small in registers
      constexpr int kBrN = kBrS * kBrS;
#pragma unroll 1
      for (int i = lane; i < kBrN; i += 64) {
        const int r = i / kBrS, c = i - r * kBrS;
        const int y = reflect101(min(sy0 + r, 2 * (h - 1)), h);
        const int x = reflect101(min(sx0 + c, 2 * (w - 1)), w);
        src[r][c] = im[(int64_t)y * w + x];
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (lane < kBrP) {
      const int c = lane;
      // vertical 7 taps from a 7-row ring: rows in groups of 7 (ring slot = row % 7, static
      // inside the unrolled group), the group loop itself not unrolled
      int win[7] = {0, 0, 0, 0, 0, 0, 0};
      const uint32_t sh = (uint32_t)c & 3u;
#pragma unroll 1
      for (int r0 = 0; r0 < kBrS; r0 += 7) {
#pragma unroll
        for (int t = 0; t < 7; ++t) {
          const int r = r0 + t;
          if (r < kBrS) {
            // horizontal 7 taps: bytes c..c+6 from three dwords, two v_dot4_u32_u8 with the
            // kernel's bytes (integer sums: exact, any order)
            const uint32_t* rw = reinterpret_cast<const uint32_t*>(&src[r][0]) + (c >> 2);
            const uint32_t d0 = rw[0], d1 = rw[1], d2 = rw[2];
            win[t] = (int)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, sh), 0x00122231u,
                                                 __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, sh),
                                                                        0x37312212u, 0u, false),
                                                 false);
            if (r >= 6) {
              int sv = 0;
#pragma unroll
              for (int q = 0; q < 7; ++q) sv += c_gk[q] * win[(t + 1 + q) % 7];  // rows r-6 .. r
              const int v = (sv + 32767 + ((sv >> 16) & 1)) >> 16;  // round half to even, as k_blur
              blr[r - 6][c] = (uint8_t)min(v, 255);
            }
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    unsigned long long words[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int pi = q * 64 + lane;
      int v[2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const float px = (float)c_pattern[pi * 4 + 2 * s2], py = (float)c_pattern[pi * 4 + 2 * s2 + 1];
        const float xx = px * a - py * bb;
        const float yy = px * bb + py * a;
        const int ix = (int)rintf(xx), iy = (int)rintf(yy);
        v[s2] = blr[iy + kBrR][ix + kBrR];
      }
      words[q] = __ballot(v[0] < v[1]);
    }
    if (lane < 4) {
      const unsigned long long wv4 = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
      reinterpret_cast<unsigned long long*>(desc + ((int64_t)b * cap + j) * FVO_DESC_BYTES)[lane] = wv4;
    }
    __builtin_amdgcn_wave_barrier();  // the next keypoint overwrites this wave's patches
  }
}

// ------------------------------------------------------------------ host geometry
static int cv_round_f(float v) { return (int)lrintf(v); }

}  // namespace

namespace {
OrbDev make_dev(const OrbGeom& g);
}

int orb_init(fvo_ctx* ctx) {
  const fvo_config& c = ctx->cfg;
  OrbGeom& g = ctx->g;
  if (c.nlevels < 1 || c.nlevels > FVO_MAX_LEVELS) return fvo_fail(ctx, "nlevels out of range");
  if (c.first_level != 0 || c.wta_k != 2 || c.score_type != 0 || c.patch_size != 31)
    return fvo_fail(ctx, "only firstLevel=0, WTA_K=2, HARRIS_SCORE, patchSize=31 are supported");
  if (c.width > 4095 || c.height > 4095) return fvo_fail(ctx, "image dimensions must be < 4096");
  // k_angle reads the whole 31x31 square around a keypoint unguarded; keypoints are kept
  // edgeThreshold px inside the level, so it must cover the half patch (k_brief stages its
  // rotated patch with REFLECT_101 and needs no such bound)
  if (c.edge_threshold < c.patch_size / 2)
    return fvo_fail(ctx, "edgeThreshold must be >= patchSize/2 (15)");
  g.nlevels = c.nlevels;
  const double sf = (double)c.scale_factor;
  int64_t off = 0, coff = 0;
  int row = 0;
  for (int l = 0; l < c.nlevels; ++l) {
    float s = (float)std::pow(sf, (double)l);
    float inv = 1.0f / s;
    g.scale[l] = s;
    g.w[l] = cv_round_f((float)c.width * inv);
    g.h[l] = cv_round_f((float)c.height * inv);
    g.off[l] = off;
    off += (int64_t)g.w[l] * g.h[l];
    g.row0[l] = row;
    row += g.h[l];
    int rw = std::max(g.w[l] - 2 * c.edge_threshold, 0), rh = std::max(g.h[l] - 2 * c.edge_threshold, 0);
    g.cand_off[l] = coff;
    coff += (int64_t)((rw + 1) / 2) * ((rh + 1) / 2) + 1;
  }
  g.off[c.nlevels] = off;
  g.row0[c.nlevels] = row;
  g.cand_off[c.nlevels] = coff;
  g.total_px = (off + 255) / 256 * 256;  // per-image stride: 256-byte aligned images
  g.total_rows = row;
  g.cand_total = coff;
  {
    float factor = (float)(1.0 / sf);
    float nd = c.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)c.nlevels));
    int sum = 0;
    for (int l = 0; l < c.nlevels - 1; ++l) {
      g.nfeat[l] = cv_round_f(nd);
      sum += g.nfeat[l];
      nd *= factor;
    }
    g.nfeat[c.nlevels - 1] = std::max(c.nfeatures - sum, 0);
  }

  // resize tables (levels 1..L-1), INTER_LINEAR_EXACT coefficient rule
  std::vector<int32_t> xo, xc, yo, yc;
  auto coeffs = [](int src, int dst, std::vector<int32_t>& ofs, std::vector<int32_t>& c1) {
    double inv_scale = (double)dst / (double)src;
    double scale = 1.0 / inv_scale;
    for (int d = 0; d < dst; ++d) {
      double fval = scale * ((double)d + 0.5) - 0.5;
      int ival = (int)std::floor(fval);
      if (ival >= 0 && src > 1) {
        if (ival < src - 1) {
          double frac = fval - (double)ival;
          ofs.push_back(ival);
          c1.push_back(frac < 0 ? 0 : (int)std::llrint(frac * 256.0));
        } else {
          ofs.push_back(-2);
          c1.push_back(0);
        }
      } else {
        ofs.push_back(-1);
        c1.push_back(0);
      }
    }
  };
  for (int l = 1; l < c.nlevels; ++l) {
    ctx->rt.xoff[l] = (int64_t)xo.size();
    coeffs(g.w[l - 1], g.w[l], xo, xc);
    ctx->rt.yoff[l] = (int64_t)yo.size();
    coeffs(g.h[l - 1], g.h[l], yo, yc);
  }
  if (xo.empty()) { xo.push_back(0); xc.push_back(0); yo.push_back(0); yc.push_back(0); }
  int rc = 0;
  if ((rc = fvo_alloc(ctx, &ctx->rt.xofs, xo.size())) || (rc = fvo_alloc(ctx, &ctx->rt.xc1, xc.size())) ||
      (rc = fvo_alloc(ctx, &ctx->rt.yofs, yo.size())) || (rc = fvo_alloc(ctx, &ctx->rt.yc1, yc.size())))
    return rc;
  FVO_HIP(ctx, hipMemcpy(ctx->rt.xofs, xo.data(), xo.size() * 4, hipMemcpyHostToDevice));
  FVO_HIP(ctx, hipMemcpy(ctx->rt.xc1, xc.data(), xc.size() * 4, hipMemcpyHostToDevice));
  FVO_HIP(ctx, hipMemcpy(ctx->rt.yofs, yo.data(), yo.size() * 4, hipMemcpyHostToDevice));
  FVO_HIP(ctx, hipMemcpy(ctx->rt.yc1, yc.data(), yc.size() * 4, hipMemcpyHostToDevice));

  // IC-angle row extents (orb.cpp computeKeyPoints: umax + symmetry fix-up)
  int half = c.patch_size / 2;
  std::vector<int> umax(half + 2 > 20 ? half + 2 : 20, 0);
  int vmax = (int)std::floor(half * std::sqrt(2.f) / 2 + 1);
  int vmin = (int)std::ceil(half * std::sqrt(2.f) / 2);
  for (int v = 0; v <= vmax; ++v) umax[v] = (int)std::lrint(std::sqrt((double)half * half - v * v));
  for (int v = half, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }

  // size-independent tables only: the geometry travels by value (OrbDev)
  FVO_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(c_umax), umax.data(), sizeof(int) * 20));
  FVO_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), FVO_ORB_PATTERN, sizeof(FVO_ORB_PATTERN)));

  const int64_t B = c.max_batch;
  int64_t maxcand = 0;
  for (int l = 0; l < c.nlevels; ++l) maxcand = std::max<int64_t>(maxcand, g.cand_off[l + 1] - g.cand_off[l]);
  ctx->scratch_per = 2 * maxcand;
  // (the full FAST score map, ctx->score, is allocated on first debug request)
  if ((rc = fvo_alloc(ctx, &ctx->pyr, B * g.total_px)) ||
      (rc = fvo_alloc(ctx, &ctx->cand, B * g.cand_total)) ||
      (rc = fvo_alloc(ctx, &ctx->hel, B * g.cand_total)) || (rc = fvo_alloc(ctx, &ctx->ncand, B * c.nlevels)) ||
      (rc = fvo_alloc(ctx, &ctx->nsel1, B * c.nlevels)) || (rc = fvo_alloc(ctx, &ctx->nsel2, B * c.nlevels)) ||
      (rc = fvo_alloc(ctx, &ctx->koff, B * (c.nlevels + 1))) ||
      (rc = fvo_alloc(ctx, &ctx->scratch, B * c.nlevels * ctx->scratch_per)))
    return rc;
  if ((g.w[0] + kTW - 1) / kTW > 64) return fvo_fail(ctx, "ORB: image wider than 4096 px");  // k_keep_compact: a lane per tile
  if ((rc = fvo_alloc(ctx, &ctx->fast_rec, B * make_dev(g).tile0[g.nlevels] * kTRec))) return rc;
  return 0;
}

namespace {
OrbDev make_dev(const OrbGeom& g) {
  OrbDev G{};
  G.nlevels = g.nlevels;
  G.total_rows = g.total_rows;
  int t = 0, bt = 0;
  for (int l = 0; l < g.nlevels; ++l) {
    G.row0[l] = g.row0[l];
    G.w[l] = g.w[l];
    G.h[l] = g.h[l];
    G.off[l] = g.off[l];
    G.cand_off[l] = g.cand_off[l];
    G.scale[l] = g.scale[l];
    G.nfeat[l] = g.nfeat[l];
    G.ntx[l] = (g.w[l] + kTW - 1) / kTW;
    G.tile0[l] = t;
    t += G.ntx[l] * ((g.h[l] + kTH - 1) / kTH);
    G.bntx[l] = (g.w[l] + kBW - 1) / kBW;
    G.btile0[l] = bt;
    bt += G.bntx[l] * ((g.h[l] + kBH - 1) / kBH);
  }
  G.btile0[g.nlevels] = bt;
  G.row0[g.nlevels] = g.row0[g.nlevels];
  G.off[g.nlevels] = g.off[g.nlevels];
  G.cand_off[g.nlevels] = g.cand_off[g.nlevels];
  G.tile0[g.nlevels] = t;
  return G;
}
}  // namespace

int orb_run(fvo_ctx* ctx, const uint8_t* images, int batch, int64_t image_stride, int pitch, float* kp, uint8_t* desc,
            int32_t* counts, int cap, hipStream_t s) {
  const fvo_config& c = ctx->cfg;
  const OrbGeom& g = ctx->g;
  const int L = g.nlevels;
  const int W = c.width, H = c.height;
  const int64_t total = g.total_px;
  const int thr = std::min(std::max(c.fast_threshold, 0), 255);
  const OrbDev G = make_dev(g);
  const int ntiles = G.tile0[L];
  const bool vec = ((uintptr_t)images & 15) == 0 && (image_stride & 15) == 0 && (pitch & 15) == 0 && (W & 15) == 0 &&
                   (total & 15) == 0;
  if (vec) {
    const int64_t n16 = (int64_t)batch * H * (W / 16);
    const int nblk = (int)std::min<int64_t>((n16 + 255) / 256, 4096);
    FVO_TIMED(ctx, KN_ORB_COPY, s, hipLaunchKernelGGL(k_copy_level0_v, dim3(nblk), dim3(256), 0, s,
                                                      reinterpret_cast<const uint4*>(images), image_stride / 16,
                                                      pitch / 16, reinterpret_cast<uint4*>(ctx->pyr), total / 16, W / 16,
                                                      H, batch));
  } else {
    FVO_TIMED(ctx, KN_ORB_COPY, s, hipLaunchKernelGGL(k_copy_level0, dim3((W + 255) / 256, H, batch), dim3(256), 0, s,
                                                      images, image_stride, pitch, ctx->pyr, total, W, H));
  }
  for (int l = 1; l < L; ++l)
    FVO_TIMED(ctx, KN_ORB_RESIZE, s, hipLaunchKernelGGL(k_resize, dim3((g.w[l] + 256 * kResCols - 1) / (256 * kResCols), (g.h[l] + kResRows - 1) / kResRows, batch), dim3(256), 0, s, G, ctx->pyr, total, l,
                       ctx->rt.xofs + ctx->rt.xoff[l], ctx->rt.xc1 + ctx->rt.xoff[l], ctx->rt.yofs + ctx->rt.yoff[l],
                       ctx->rt.yc1 + ctx->rt.yoff[l]));
  FVO_TIMED(ctx, KN_ORB_FAST, s, hipLaunchKernelGGL(k_fast_nms<false>, dim3(ntiles, batch), dim3(kFT), 0, s, G, ctx->pyr,
                     nullptr, ctx->fast_rec, total, thr, c.edge_threshold, ntiles));
  FVO_TIMED(ctx, KN_ORB_SELECT1, s, hipLaunchKernelGGL(HIP_KERNEL_NAME(k_select<ElemFast, kSelCap1, true>), dim3(batch, L),
                     dim3(kSelThreads), 0, s, G, ctx->fast_rec, ntiles, c.edge_threshold, ctx->cand, ctx->ncand,
                     ctx->nsel1, ctx->scratch, ctx->scratch_per, g.cand_total, L, 2));
  FVO_TIMED(ctx, KN_ORB_HARRIS, s, hipLaunchKernelGGL(k_harris, dim3(32, L, batch), dim3(256), 0, s, G, ctx->pyr, ctx->cand, ctx->nsel1, ctx->hel, total,
                     g.cand_total, L));
  FVO_TIMED(ctx, KN_ORB_SELECT2, s, hipLaunchKernelGGL(HIP_KERNEL_NAME(k_select<ElemHarris, kSelCap2, false>), dim3(batch, L),
                     dim3(kSelThreads), 0, s, G, nullptr, ntiles, c.edge_threshold, ctx->hel, ctx->nsel1,
                     ctx->nsel2, ctx->scratch, ctx->scratch_per, g.cand_total, L, 1));
  FVO_TIMED(ctx, KN_ORB_OFFSETS, s, hipLaunchKernelGGL(k_offsets, dim3((batch + 63) / 64), dim3(64), 0, s, ctx->nsel2, ctx->koff, counts, batch, L, cap));
  FVO_TIMED(ctx, KN_ORB_ANGLE, s, hipLaunchKernelGGL(k_angle, dim3(16, L, batch), dim3(256), 0, s, G, ctx->pyr, ctx->hel, ctx->nsel2, ctx->koff, kp,
                     total, g.cand_total, L, cap, c.patch_size));
  FVO_TIMED(ctx, KN_ORB_BRIEF, s, hipLaunchKernelGGL(k_brief, dim3(64, batch), dim3(256), 0, s, G, ctx->pyr, kp, counts, desc, total, cap));
  ctx->orb_last_batch = batch;
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

// Debug hook (fvo_debug_buffer 1): the blurred pyramid of the last fvo_orb_detect_compute
// call, which the hot path no longer materialises (k_brief blurs each keypoint's patch).
int orb_blur_debug(fvo_ctx* ctx) {
  if (!ctx->pyr) return fvo_fail(ctx, "orb stage not enabled");
  const OrbGeom& g = ctx->g;
  if (!ctx->blur) {
    int rc = fvo_alloc(ctx, &ctx->blur, (int64_t)ctx->cfg.max_batch * g.total_px);
    if (rc) return rc;
  }
  if (ctx->orb_last_batch > 0) {
    const OrbDev G = make_dev(g);
    hipLaunchKernelGGL(k_blur, dim3(G.btile0[g.nlevels], ctx->orb_last_batch), dim3(256), 0, 0, G, ctx->pyr, ctx->blur,
                       g.total_px);
    FVO_LAUNCH_CHECK(ctx);
  }
  FVO_HIP(ctx, hipDeviceSynchronize());
  return 0;
}

// Debug hook (fvo_debug_buffer 2): the FAST score map of the last call's pyramid, which the hot
// path does not write (k_fast_nms keeps only the kept pixels' scores).
int orb_score_debug(fvo_ctx* ctx) {
  if (!ctx->pyr) return fvo_fail(ctx, "orb stage not enabled");
  const OrbGeom& g = ctx->g;
  if (!ctx->score) {
    int rc = fvo_alloc(ctx, &ctx->score, (int64_t)ctx->cfg.max_batch * g.total_px);
    if (rc) return rc;
  }
  if (ctx->orb_last_batch > 0) {
    const OrbDev G = make_dev(g);
    const int ntiles = G.tile0[g.nlevels];
    hipLaunchKernelGGL(k_fast_nms<true>, dim3(ntiles, ctx->orb_last_batch), dim3(kFT), 0, 0, G, ctx->pyr, ctx->score,
                       nullptr, g.total_px, std::min(std::max(ctx->cfg.fast_threshold, 0), 255),
                       ctx->cfg.edge_threshold, ntiles);  // the threshold orb_run uses
    FVO_LAUNCH_CHECK(ctx);
  }
  FVO_HIP(ctx, hipDeviceSynchronize());
  return 0;
}

// ------------------------------------------------------------------ test hook
namespace {
__global__ void k_pack_keys(const float* __restrict__ k, uint64_t* __restrict__ a, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = ((uint64_t)__float_as_uint(k[i]) << 32) | (uint32_t)i;
}
__global__ void k_unpack_idx(const uint64_t* __restrict__ a, int32_t* __restrict__ idx, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) idx[i] = (int32_t)(uint32_t)a[i];
}
__global__ __launch_bounds__(kSelThreads) void k_select_test(uint64_t* __restrict__ a, int n, int keep,
                                                             int32_t* __restrict__ scratch, int32_t* __restrict__ out_n) {
  __shared__ SelShared sh;
  int r = select_block<ElemHarris>(sh, a, n, keep, scratch, scratch + n);
  if (threadIdx.x == 0) *out_n = r;
}
}  // namespace

// retainBest on n float keys (device memory); writes surviving original indices in
// output order to idx_out and the count to *n_out.  Test hook for the selection stage.
extern "C" int fvo_test_retain_best(fvo_ctx* ctx, const float* keys, int32_t n, int32_t keep, int32_t* idx_out,
                                    int32_t* n_out, fvo_stream stream) {
  hipStream_t s = (hipStream_t)stream;
  uint64_t* a = nullptr;
  int32_t* scr = nullptr;
  FVO_HIP(ctx, hipMallocAsync((void**)&a, sizeof(uint64_t) * (size_t)std::max(n, 1), s));
  FVO_HIP(ctx, hipMallocAsync((void**)&scr, sizeof(int32_t) * 2 * (size_t)std::max(n, 1), s));
  hipLaunchKernelGGL(k_pack_keys, dim3((n + 255) / 256 + 1), dim3(256), 0, s, keys, a, n);
  hipLaunchKernelGGL(k_select_test, dim3(1), dim3(kSelThreads), 0, s, a, n, keep, scr, n_out);
  hipLaunchKernelGGL(k_unpack_idx, dim3((n + 255) / 256 + 1), dim3(256), 0, s, a, idx_out, n);
  FVO_HIP(ctx, hipFreeAsync(a, s));
  FVO_HIP(ctx, hipFreeAsync(scr, s));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
