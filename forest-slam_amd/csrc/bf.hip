// Cross-checked brute-force Hamming matcher for gfx950 — replaces
// cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True).match(d0, d1)
// (ros_ws/src/stereo_slam.py:85, :234, :242).
//
// k_bf_argmin: one thread per row descriptor (held in 8 VGPRs), the other set streamed
//   through LDS in 1024-descriptor tiles (32 KB, broadcast ds_read_b128); distance =
//   sum of v_bcnt(xor) over the 8 words; strict '<' in ascending column order, so the
//   first index wins ties exactly like batchDistance(K=1).  Both directions in one
//   launch (blockIdx.z).
// k_bf_finish: mutual-nearest check + ordered compaction (ascending queryIdx).
#include "fvo_device.h"

namespace {

constexpr int kTile = 1024;
constexpr int kRowsPerBlock = 256;

__global__ __launch_bounds__(kRowsPerBlock) void k_bf_argmin(const uint8_t* __restrict__ query,
                                                            const int32_t* __restrict__ nq,
                                                            const uint8_t* __restrict__ train,
                                                            const int32_t* __restrict__ nt, int cap,
                                                            int32_t* __restrict__ sidx, int32_t* __restrict__ sdist,
                                                            int32_t* __restrict__ tidx) {
  __shared__ uint4 tile[kTile * 2];
  const int b = blockIdx.y;
  const int dir = blockIdx.z;
  const uint8_t* rows = dir == 0 ? query : train;
  const uint8_t* cols = dir == 0 ? train : query;
  int nr = dir == 0 ? nq[b] : nt[b];
  int nc = dir == 0 ? nt[b] : nq[b];
  nr = nr < 0 ? 0 : (nr > cap ? cap : nr);
  nc = nc < 0 ? 0 : (nc > cap ? cap : nc);
  const int r = blockIdx.x * kRowsPerBlock + threadIdx.x;
  if ((int)(blockIdx.x * kRowsPerBlock) >= nr) return;  // uniform per block
  uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
  if (r < nr) {
    const uint4* p = reinterpret_cast<const uint4*>(rows + ((int64_t)b * cap + r) * 32);
    q0 = p[0];
    q1 = p[1];
  }
  int best = 0x7fffffff, bi = -1;
  const uint4* cb = reinterpret_cast<const uint4*>(cols + (int64_t)b * cap * 32);
  for (int t0 = 0; t0 < nc; t0 += kTile) {
    int tn = min(kTile, nc - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * tn; i += kRowsPerBlock) tile[i] = cb[2 * t0 + i];
    __syncthreads();
    if (r < nr) {
      for (int j = 0; j < tn; ++j) {
        uint4 a = tile[2 * j], c = tile[2 * j + 1];
        int d = __popc(q0.x ^ a.x) + __popc(q0.y ^ a.y) + __popc(q0.z ^ a.z) + __popc(q0.w ^ a.w) +
                __popc(q1.x ^ c.x) + __popc(q1.y ^ c.y) + __popc(q1.z ^ c.z) + __popc(q1.w ^ c.w);
        if (d < best) {
          best = d;
          bi = t0 + j;
        }
      }
    }
  }
  if (r < nr) {
    if (dir == 0) {
      sidx[(int64_t)b * cap + r] = bi;
      sdist[(int64_t)b * cap + r] = best;
    } else {
      tidx[(int64_t)b * cap + r] = bi;
    }
  }
}

__global__ void k_bf_finish(const int32_t* __restrict__ nq, const int32_t* __restrict__ nt, int cap,
                            const int32_t* __restrict__ sidx, const int32_t* __restrict__ sdist,
                            const int32_t* __restrict__ tidx, int32_t* __restrict__ matches,
                            int32_t* __restrict__ nmatch) {
  const int b = blockIdx.x;
  int n0 = nq[b], n1 = nt[b];
  n0 = n0 < 0 ? 0 : (n0 > cap ? cap : n0);
  n1 = n1 < 0 ? 0 : (n1 > cap ? cap : n1);
  if (n1 == 0) n0 = 0;
  __shared__ int s_w[16];
  __shared__ int s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int base = 0; base < n0; base += blockDim.x) {
    int q = base + threadIdx.x;
    int t = -1;
    bool keep = false;
    if (q < n0) {
      t = sidx[(int64_t)b * cap + q];
      keep = t >= 0 && tidx[(int64_t)b * cap + t] == q;
    }
    unsigned long long m = __ballot(keep);
    int pre = __popcll(m & ((1ull << wave_lane()) - 1ull));
    if (wave_lane() == 0) s_w[threadIdx.x >> 6] = __popcll(m);
    __syncthreads();
    int wpre = 0, tot = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      if (i < (int)(threadIdx.x >> 6)) wpre += s_w[i];
      tot += s_w[i];
    }
    if (keep) {
      int32_t* o = matches + ((int64_t)b * cap + s_carry + wpre + pre) * 3;
      o[0] = q;
      o[1] = t;
      o[2] = sdist[(int64_t)b * cap + q];
    }
    __syncthreads();
    if (threadIdx.x == 0) s_carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) nmatch[b] = s_carry;
}

}  // namespace

int bf_init(fvo_ctx* ctx) {
  const int64_t n = (int64_t)ctx->cfg.max_batch * ctx->kp_cap;
  int rc;
  if ((rc = fvo_alloc(ctx, &ctx->bf_sidx, n)) || (rc = fvo_alloc(ctx, &ctx->bf_sdist, n)) ||
      (rc = fvo_alloc(ctx, &ctx->bf_tidx, n)))
    return rc;
  return 0;
}

int bf_run(fvo_ctx* ctx, const uint8_t* q, const int32_t* nq, const uint8_t* t, const int32_t* nt, int batch, int cap,
           int32_t* matches, int32_t* nmatch, hipStream_t s) {
  if ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(t)) & 15)
    return fvo_fail(ctx, "descriptor buffers must be 16-byte aligned");
  FVO_TIMED(ctx, KN_BF_ARGMIN, s, hipLaunchKernelGGL(k_bf_argmin, dim3((cap + kRowsPerBlock - 1) / kRowsPerBlock, batch, 2), dim3(kRowsPerBlock), 0,
                     s, q, nq, t, nt, cap, ctx->bf_sidx, ctx->bf_sdist, ctx->bf_tidx));
  FVO_TIMED(ctx, KN_BF_FINISH, s, hipLaunchKernelGGL(k_bf_finish, dim3(batch), dim3(256), 0, s, nq, nt, cap, ctx->bf_sidx, ctx->bf_sdist, ctx->bf_tidx,
                     matches, nmatch));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
