// Image ingest for gfx950 — replaces ros_ws/src/stereo_slam.py:184-186 / :196-198 and
// mono_slam.py:92-93:
//   img = cv2.cvtColor(cv2.undistort(img_bgr8, K, dist), cv2.COLOR_BGR2GRAY)
// as one streaming kernel: every thread produces 4 consecutive gray pixels of a row — the
// undistortion map entry of each (initUndistortRectifyMap, CV_16SC2, evaluated in fp64 on
// the fly: no map is stored or read), the fixed-point bilinear remap of the three channels
// (INTER_LINEAR, BORDER_CONSTANT 0) and the 14-bit BGR2GRAY, one 32-bit store.
// HBM traffic per pixel: the 3 source bytes (the 2x2 gathers of neighbouring outputs hit
// the same lines in L1/L2) + 1 output byte.  Specification: oracle/ingest_ref.cpp.
#include "fvo_device.h"

namespace {

struct Lens {
  double K[9];
  double k1, k2, p1, p2, k3;
};

// invert() 3x3 closed form (oracle inv3)
__device__ __forceinline__ void inv3(const double* S, double* t) {
  double d = S[0] * (S[4] * S[8] - S[5] * S[7]) - S[1] * (S[3] * S[8] - S[5] * S[6]) + S[2] * (S[3] * S[7] - S[4] * S[6]);
  if (d == 0.) {
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = 0.0;
    return;
  }
  d = 1. / d;
  t[0] = (S[4] * S[8] - S[5] * S[7]) * d;
  t[1] = (S[2] * S[7] - S[1] * S[8]) * d;
  t[2] = (S[1] * S[5] - S[2] * S[4]) * d;
  t[3] = (S[5] * S[6] - S[3] * S[8]) * d;
  t[4] = (S[0] * S[8] - S[2] * S[6]) * d;
  t[5] = (S[2] * S[3] - S[0] * S[5]) * d;
  t[6] = (S[3] * S[7] - S[4] * S[6]) * d;
  t[7] = (S[1] * S[6] - S[0] * S[7]) * d;
  t[8] = (S[0] * S[4] - S[1] * S[3]) * d;
}

__device__ __forceinline__ int round_sat(double v) {
  return v >= 2147483647.0 ? 2147483647 : (v <= -2147483648.0 ? (-2147483647 - 1) : (int)rint(v));
}

// PIX output pixels per thread, 4 rows x 64 threads per block.  kPinhole: K has the camera-matrix zero pattern
// (K[1] = K[3] = K[6] = K[7] = 0, K[8] = 1), so ir[6] = ir[7] = 0 (exact zeros of the closed
// form) and _w, hence w = 1/_w, is constant along a row: hoisted (bit-identical to the
// per-pixel evaluation).  The k4..k6 denominator is exactly 1 and x/1.0 == x, so it is dropped.
template <int PIX, bool kPinhole>
__global__ __launch_bounds__(256) void k_ing_undistort_gray(const uint8_t* __restrict__ src, int64_t sstride,
                                                            int spitch, uint8_t* __restrict__ dst, int64_t dstride,
                                                            int dpitch, int W, int H, int stripe0, Lens L) {
  // block = 4 rows x 64 threads, each thread PIX consecutive pixels of its row
  const int row = blockIdx.y * 4 + (threadIdx.x >> 6), b = blockIdx.z;
  const int c0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * PIX;
  if (c0 >= W || row >= H) return;
  const uint8_t* S = src + b * sstride;
  const int y0 = (row / stripe0) * stripe0, i = row - y0;
  double Ar[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) Ar[k] = L.K[k];
  Ar[5] = L.K[5] - y0;
  double ir[9];
  inv3(Ar, ir);
  const double fx = L.K[0], fy = L.K[4], u0 = L.K[2], v0 = L.K[5];
  const double bx = i * ir[1] + ir[2], by = i * ir[4] + ir[5], bw = i * ir[7] + ir[8];
  const double w_row = kPinhole ? 1. / (bw + 0 * ir[6]) : 0.0;
  uint32_t packed[PIX / 4];
#pragma unroll
  for (int k = 0; k < PIX / 4; ++k) packed[k] = 0;
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    const int col = c0 + q;
    if (col >= W) break;
    double _x = bx + col * ir[0], _y = by + col * ir[3];
    double w = kPinhole ? w_row : 1. / (bw + col * ir[6]);
    double x = _x * w, y = _y * w;
    double x2 = x * x, y2 = y * y;
    double r2 = x2 + y2, _2xy = 2 * x * y;
    double kr = (1 + ((L.k3 * r2 + L.k2) * r2 + L.k1) * r2);
    double xd = (x * kr + L.p1 * _2xy + L.p2 * (r2 + 2 * x2) + 0.0 * r2 + 0.0 * r2 * r2);
    double yd = (y * kr + L.p1 * (r2 + 2 * y2) + L.p2 * _2xy + 0.0 * r2 + 0.0 * r2 * r2);
    const int iu = round_sat((fx * xd + u0) * 32.0), iv = round_sat((fy * yd + v0) * 32.0);
    const int sx = (int16_t)(iu >> 5), sy = (int16_t)(iv >> 5);
    const int tx = iu & 31, ty = iv & 31;
    const int w0 = (32 - ty) * (32 - tx) * 32, w1 = (32 - ty) * tx * 32, w2 = ty * (32 - tx) * 32, w3 = ty * tx * 32;
    int ch[3] = {0, 0, 0};
    if (!(sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0)) {
      const bool xin0 = sx >= 0, xin1 = sx + 1 < W, yin0 = sy >= 0, yin1 = sy + 1 < H;
      const uint8_t* r0 = S + (int64_t)sy * spitch + sx * 3;
      const uint8_t* r1 = r0 + spitch;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int v00 = (yin0 && xin0) ? r0[k] : 0, v01 = (yin0 && xin1) ? r0[3 + k] : 0;
        const int v10 = (yin1 && xin0) ? r1[k] : 0, v11 = (yin1 && xin1) ? r1[3 + k] : 0;
        int s = v00 * w0 + v01 * w1 + v10 * w2 + v11 * w3;
        s = (s + (1 << 14)) >> 15;
        ch[k] = s < 0 ? 0 : (s > 255 ? 255 : s);
      }
    }
    const uint32_t g = (uint32_t)((ch[0] * 1868 + ch[1] * 9617 + ch[2] * 4899 + (1 << 13)) >> 14);
    packed[q / 4] |= g << (8 * (q % 4));
  }
  uint8_t* D = dst + b * dstride + (int64_t)row * dpitch + c0;
  if (c0 + PIX <= W && (((uintptr_t)D) & 3) == 0) {
#pragma unroll
    for (int k = 0; k < PIX / 4; ++k) reinterpret_cast<uint32_t*>(D)[k] = packed[k];
  } else {
    for (int q = 0; q < PIX && c0 + q < W; ++q) D[q] = (uint8_t)(packed[q / 4] >> (8 * (q % 4)));
  }
}

}  // namespace

int ingest_run(fvo_ctx* ctx, const uint8_t* bgr, int batch, int64_t sstride, int spitch, const double* K,
               const double* dist, uint8_t* gray, int64_t dstride, int dpitch, hipStream_t s) {
  const int W = ctx->cfg.width, H = ctx->cfg.height;
  Lens L;
  for (int i = 0; i < 9; ++i) L.K[i] = K[i];
  L.k1 = dist[0]; L.k2 = dist[1]; L.p1 = dist[2]; L.p2 = dist[3]; L.k3 = dist[4];
  int stripe0 = 4096 / (W > 1 ? W : 1);
  stripe0 = stripe0 < 1 ? 1 : (stripe0 > H ? H : stripe0);
  constexpr int PIX = 4;
  dim3 grid((W + 64 * PIX - 1) / (64 * PIX), (H + 3) / 4, batch);
  const bool pinhole = K[1] == 0.0 && K[3] == 0.0 && K[6] == 0.0 && K[7] == 0.0 && K[8] == 1.0;
  FVO_TIMED(ctx, KN_INGEST, s, {
    if (pinhole)
      hipLaunchKernelGGL((k_ing_undistort_gray<PIX, true>), grid, dim3(256), 0, s, bgr, sstride, spitch, gray, dstride,
                         dpitch, W, H, stripe0, L);
    else
      hipLaunchKernelGGL((k_ing_undistort_gray<PIX, false>), grid, dim3(256), 0, s, bgr, sstride, spitch, gray,
                         dstride, dpitch, W, H, stripe0, L);
  });
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Motion-blur ablation — stereo_slam.py:141-178 (forest_slam_ros/src/stereo_slam.py:142-178),
// SURVEY.md §8f rank 3:
//   apply_motion_blur:        kernel = warpAffine(diag(ones(k)), rot((k//2, k//2), angle=0)) / k
//                             blurred = cv2.filter2D(image, -1, kernel)   (BORDER_REFLECT_101)
//   apply_random_motion_blur: mask = union of (2*(k//2)+1)^2 squares around random.sample()d
//                             pixels (clipped), out = np.where(mask, blurred, image)
// At angle 0 the rotation is the identity and the kernel is the k-tap diagonal 1/k with
// anchor (k//2, k//2), so tap i reads src(y + i - a, x + i - a).  filter2D's arithmetic:
//   k*k <  130: direct Filter2D<uchar, float>: the nonzero taps in row-major (= diagonal)
//               order accumulated by FilterVec_8u, s = fma(x_i, (float)(1/k), s) from 0,
//               then cvRound (half to even) and saturate;
//   k*k >= 130: dftFilter2D (crossCorr in float32).  Its result is the exact S/k within DFT
//               rounding; S/k is never closer than 1/(2k) to a rounding boundary except at the
//               exact ties S = q*k + k/2 (even k), which are taken half to even (unpinned).
// k_mb_seed marks the sampled pixels; k_mb_blur (block = 256 columns x 32 rows, 64 threads x
// 4 px per row, 4 row groups) stages the (32+k-1) x (256+k-1) source tile (REFLECT_101
// resolved while staging) in LDS, dilates the seeds to the mask in LDS, blurs only masked
// pixels and writes out + mask with dword stores; k_mb_fix normalises the mask bytes.

namespace {

constexpr int kMbTileW = 256, kMbTileH = 32, kMbMaxK = 31;
constexpr int kMbTW = kMbTileW + kMbMaxK - 1 + 1, kMbTH = kMbTileH + kMbMaxK - 1;

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

// Seeds: bit 0 of the mask byte at every sampled pixel (one byte store per sample).
__global__ __launch_bounds__(256) void k_mb_seed(const int32_t* __restrict__ centers, const int32_t* __restrict__ ncent,
                                                 int cap, uint8_t* __restrict__ mask, int64_t mstride, int npix) {
  const int b = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= min(ncent[b], cap)) return;
  const int p = centers[(int64_t)b * cap + c];
  if (p < 0 || p >= npix) return;  // not a pixel index: ignored
  mask[b * mstride + p] = 1;
}

// mask byte = bit 1 (the dilated mask written by k_mb_blur) -> 0/1; 4 bytes per thread
__global__ __launch_bounds__(256) void k_mb_fix(uint8_t* __restrict__ m, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 4 <= n) {
    uint32_t* w = reinterpret_cast<uint32_t*>(m + i);
    *w = (*w >> 1) & 0x01010101u;
  } else {
    for (int64_t j = i; j < n; ++j) m[j] = (m[j] >> 1) & 1;
  }
}

// kSeeds: the mask is the (2h+1)^2 dilation of the seed bitmap (= the union of the reference's
// clipped squares), computed per block in LDS on bitmaps: seed rows (32+2h) x (256+2h) (zero
// outside the image) gathered by wave ballots, horizontal dilation as 2h+1 shift-ORs of a
// 64-bit funnel per 32 output columns, vertical as 2h+1 word ORs; each block writes its pixels' mask byte as
// seed | dilated << 1 (neighbours only read bit 0), k_mb_fix then leaves 0/1.
// Without seeds the mask is all zero and out = img.
template <bool kDirect, bool kSeeds>
__global__ __launch_bounds__(256) void k_mb_blur(const uint8_t* __restrict__ src, int64_t sstride, int spitch,
                                                 uint8_t* __restrict__ mask, int64_t mstride,
                                                 uint8_t* __restrict__ dst, int64_t dstride, int dpitch, int W, int H,
                                                 int k, int h, float kf) {
  __shared__ uint8_t tile[kMbTH][kMbTW];
  // seed rows as bitmaps (320 bits = 10 words per tile row), the horizontal dilation (8 words =
  // 256 output columns per row) and the full dilation of the block's 32 rows
  __shared__ uint32_t sbits[kSeeds ? kMbTH : 1][10];
  __shared__ uint32_t hbits[kSeeds ? kMbTH : 1][8];
  __shared__ uint32_t dbits[kSeeds ? kMbTileH : 1][8];
  const int b = blockIdx.z, a = k / 2;
  const int x0 = blockIdx.x * kMbTileW, y0 = blockIdx.y * kMbTileH;
  const uint8_t* S = src + b * sstride;
  const int rows = min(kMbTileH, H - y0);
  const int th = rows + k - 1, tw = kMbTileW + k - 1;
  for (int r = 0; r < th; ++r) {  // row-wise fill: REFLECT_101 row index once per row, coalesced columns
    const uint8_t* Srow = S + (int64_t)reflect101(y0 - a + r, H) * spitch;
    for (int c = threadIdx.x; c < tw; c += 256) {
      const int gx = x0 - a + c;  // columns past W-1+k feed no output
      tile[r][c] = gx < W + k ? Srow[reflect101(gx, W)] : 0;
    }
  }
  uint8_t* Mb = mask + b * mstride;
  if (kSeeds) {
    const int sh = rows + 2 * h, sw = kMbTileW + 2 * h;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int r = wave; r < sh; r += 4) {  // ballot per 64 columns: bit c of row r = seed at (y0-h+r, x0-h+c)
      const int gy = y0 - h + r;
      const bool rin = gy >= 0 && gy < H;
#pragma unroll
      for (int ch = 0; ch < 5; ++ch) {
        const int c = ch * 64 + lane, gx = x0 - h + c;
        const bool on = c < sw && rin && gx >= 0 && gx < W && (Mb[(int64_t)gy * W + gx] & 1);
        const uint64_t bal = __ballot(on);
        if (lane == 0) {
          sbits[r][2 * ch] = (uint32_t)bal;
          sbits[r][2 * ch + 1] = (uint32_t)(bal >> 32);
        }
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < sh * 8; t += 256) {  // horizontal: out bit c = OR of bits c .. c+2h
      const int r = t >> 3, w = t & 7;
      const uint64_t v = (uint64_t)sbits[r][w] | ((uint64_t)sbits[r][w + 1] << 32);
      uint64_t d = 0;
      for (int j = 0; j <= 2 * h; ++j) d |= v >> j;
      hbits[r][w] = (uint32_t)d;
    }
    __syncthreads();
    {  // vertical: rows ly .. ly+2h of the horizontal dilation
      const int ly = threadIdx.x >> 3, w = threadIdx.x & 7;
      if (ly < rows) {
        uint32_t d = 0;
        for (int i = 0; i <= 2 * h; ++i) d |= hbits[ly + i][w];
        dbits[ly][w] = d;
      }
    }
  }
  __syncthreads();
  const int lx = (threadIdx.x & 63) * 4, xb = x0 + lx;
  if (xb >= W) return;
  const bool full = xb + 4 <= W;
#pragma unroll 1
  for (int ly = threadIdx.x >> 6; ly < rows; ly += 4) {
    const int y = y0 + ly;
    const uint8_t* Srow = S + (int64_t)y * spitch + xb;
    uint8_t* Mrow = Mb + (int64_t)y * W + xb;
    uint32_t m4 = 0, s4 = 0;
    if (kSeeds) {
      const uint32_t nib = (dbits[ly][lx >> 5] >> (lx & 31)) & 0xfu;
      m4 = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
    }
    if (full && (((uintptr_t)Srow) & 3) == 0) {
      s4 = *reinterpret_cast<const uint32_t*>(Srow);
    } else {
      for (int q = 0; q < 4 && xb + q < W; ++q) s4 |= (uint32_t)Srow[q] << (8 * q);
    }
    uint32_t packed = s4;
    if (m4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!((m4 >> (8 * q)) & 0xff)) continue;
        uint32_t v;
        if (kDirect) {
          float sum = 0.f;
          for (int i = 0; i < k; ++i) sum = __builtin_fmaf((float)tile[ly + i][lx + q + i], kf, sum);
          const int r = (int)rintf(sum);
          v = (uint32_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        } else {
          int sum = 0;
          for (int i = 0; i < k; ++i) sum += tile[ly + i][lx + q + i];
          int qq = sum / k;
          const int rem = sum - qq * k;
          if (2 * rem > k || (2 * rem == k && (qq & 1))) ++qq;
          v = (uint32_t)(qq > 255 ? 255 : qq);
        }
        packed = (packed & ~(0xffu << (8 * q))) | (v << (8 * q));
      }
    }
    // mask byte: seed bit | dilated << 1 (k_mb_fix), or 0 without seeds
    const uint32_t mo = m4 << 1;
    uint8_t* D = dst + b * dstride + (int64_t)y * dpitch + xb;
    if (full && (((uintptr_t)D) & 3) == 0) {
      *reinterpret_cast<uint32_t*>(D) = packed;
    } else {
      for (int q = 0; q < 4 && xb + q < W; ++q) D[q] = (uint8_t)(packed >> (8 * q));
    }
    if (kSeeds) {  // only this block writes these bytes; neighbours read bit 0, which is kept (from sbits)
      const int cb = lx + h;  // seed-tile column of this thread's first pixel, row ly + h
      const uint64_t sv = (uint64_t)sbits[ly + h][cb >> 5] | ((uint64_t)sbits[ly + h][(cb >> 5) + 1] << 32);
      const uint32_t sn = (uint32_t)(sv >> (cb & 31)) & 0xfu;
      const uint32_t sd = (sn & 1u) | ((sn & 2u) << 7) | ((sn & 4u) << 14) | ((sn & 8u) << 21);
      if (full && (((uintptr_t)Mrow) & 3) == 0) {
        *reinterpret_cast<uint32_t*>(Mrow) = sd | mo;
      } else {
        for (int q = 0; q < 4 && xb + q < W; ++q) Mrow[q] = (uint8_t)(((sd | mo) >> (8 * q)) & 0xff);
      }
    } else if (full && (((uintptr_t)Mrow) & 3) == 0) {
      *reinterpret_cast<uint32_t*>(Mrow) = 0;
    } else {
      for (int q = 0; q < 4 && xb + q < W; ++q) Mrow[q] = 0;
    }
  }
}

}  // namespace

int motion_blur_run(fvo_ctx* ctx, const uint8_t* img, int batch, int64_t sstride, int spitch, int ksize,
                    const int32_t* centers, const int32_t* ncent, int cap, uint8_t* mask, uint8_t* out,
                    int64_t dstride, int dpitch, hipStream_t s) {
  const int W = ctx->cfg.width, H = ctx->cfg.height;
  const int64_t mstride = (int64_t)W * H;
  const int half = ksize / 2;
  const bool seeds = cap > 0;
  // k_mb_fix rewrites the mask a dword at a time: refuse a misaligned mask before any launch,
  // so an error never leaves the mask in its intermediate (seed / dilated bit) encoding
  if (seeds && (((uintptr_t)mask) & 3)) return fvo_fail(ctx, "motion blur: mask must be 4-byte aligned");
  if (seeds) {
    FVO_HIP(ctx, hipMemsetAsync(mask, 0, (size_t)mstride * batch, s));
    hipLaunchKernelGGL(k_mb_seed, dim3((cap + 255) / 256, batch), dim3(256), 0, s, centers, ncent, cap, mask, mstride,
                       W * H);
    FVO_LAUNCH_CHECK(ctx);
  }
  dim3 grid((W + kMbTileW - 1) / kMbTileW, (H + kMbTileH - 1) / kMbTileH, batch);
  const bool direct = ksize * ksize < 130;
  const float kf = (float)(1.0 / ksize);
#define FVO_MB(DIR, SEED)                                                                                    \
  hipLaunchKernelGGL((k_mb_blur<DIR, SEED>), grid, dim3(256), 0, s, img, sstride, spitch, mask, mstride, out, \
                     dstride, dpitch, W, H, ksize, half, kf)
  FVO_TIMED(ctx, KN_MOTION_BLUR, s, {
    if (direct) {
      if (seeds) FVO_MB(true, true); else FVO_MB(true, false);
    } else {
      if (seeds) FVO_MB(false, true); else FVO_MB(false, false);
    }
  });
#undef FVO_MB
  FVO_LAUNCH_CHECK(ctx);
  if (seeds) {
    const int64_t n = mstride * batch;
    hipLaunchKernelGGL(k_mb_fix, dim3((unsigned)((n / 4 + 256) / 256)), dim3(256), 0, s, mask, n);
    FVO_LAUNCH_CHECK(ctx);
  }
  return 0;
}
