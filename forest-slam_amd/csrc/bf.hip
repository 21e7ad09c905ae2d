// Cross-checked brute-force Hamming matcher for gfx950 — replaces
// cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True).match(d0, d1)
// (ros_ws/src/stereo_slam.py:85, :234, :242).
//
// One pass over the distance matrix gives both directions' nearest neighbours (r6; r1-r5 ran
// the two directions as separate grids, every popcount twice).  The minima are packed keys
// (distance << 16 | index): min over keys = smallest distance, then the smallest index, which
// is batchDistance(K=1)'s first-index-wins rule in either direction, independent of the order
// the distances are visited in.
// k_bf_pass: block = 4 waves x 64 query rows (one row descriptor per lane, 8 VGPRs) x a chunk of
//   kChunk train columns staged in LDS.  A wave walks each 64-column block of the chunk
//   diagonally: at step s lane i takes column (i + s) mod 64, so the 64 lanes touch 64 different
//   columns and a column's running minimum over the wave's rows travels with it -- one DPP
//   wave_rol:1 per step (folded into the v_min_u32) hands each lane the accumulator of the column
//   it takes next.  The row minimum stays in the lane.  Per distance: 8 xor + 8 v_bcnt, two key
//   builds, two mins -- no cross-lane argmin reduction, no second pass.  Column minima of the
//   block's 4 waves meet in LDS (ds_min), then one global atomicMin per column; row minima one
//   global atomicMin per row (blocks of other column chunks).
// k_bf_finish: mutual-nearest check + ordered compaction (ascending queryIdx); resets the key
//   arrays for the next call.
#include <type_traits>

#include "fvo_device.h"

namespace {

constexpr int kChunk = 256;  // train columns per block (4 column blocks of 64)
constexpr int kRows = 256;   // query rows per block (4 waves)
constexpr uint32_t kNoKey = 0xFFFFFFFFu;

// popcount accumulated in one instruction (v_bcnt_u32_b32 d, x, acc): the compiler otherwise
// turns a chain of popcount + add into separate counts and v_add3s
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
  return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Hamming distance of a row descriptor (a0, a1) and a column descriptor at p (LDS, 32 B: loaded
// as two whole 16-B vectors -- ds_read_b128 -- before the scalar popcounts take them apart)
__device__ __forceinline__ uint32_t hamming(const u32x4& a0, const u32x4& a1, const uint4* p) {
  const u32x4 b0 = *reinterpret_cast<const u32x4*>(p) ^ a0;
  const u32x4 b1 = *reinterpret_cast<const u32x4*>(p + 1) ^ a1;
  uint32_t d = bcnt_acc(b0.x, 0u);
  d = bcnt_acc(b0.y, d);
  d = bcnt_acc(b0.z, d);
  d = bcnt_acc(b0.w, d);
  d = bcnt_acc(b1.x, d);
  d = bcnt_acc(b1.y, d);
  d = bcnt_acc(b1.z, d);
  return bcnt_acc(b1.w, d);
}

// DPP wave_rol:1 -- lane i receives lane i + 1's value (lane 63 lane 0's)
__device__ __forceinline__ uint32_t wave_rol1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFFu, (int)v, 0x134, 0xF, 0xF, false);
}

__global__ __launch_bounds__(kRows) void k_bf_pass(const uint8_t* __restrict__ query, const int32_t* __restrict__ nq,
                                                   const uint8_t* __restrict__ train, const int32_t* __restrict__ nt,
                                                   int cap, uint32_t* __restrict__ rowkey,
                                                   uint32_t* __restrict__ colkey) {
  __shared__ uint4 s_desc[kChunk * 2];  // the chunk's train descriptors (32 B each)
  __shared__ uint32_t s_col[kChunk];    // column minima of the block's rows
  const int b = blockIdx.z;
  int nr = nq[b], nc = nt[b];
  nr = nr < 0 ? 0 : (nr > cap ? cap : nr);
  nc = nc < 0 ? 0 : (nc > cap ? cap : nc);
  const int r0 = blockIdx.x * kRows, c0 = blockIdx.y * kChunk;
  if (r0 >= nr || c0 >= nc) return;  // uniform per block
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ncols = min(kChunk, nc - c0);
  const uint4* cb = reinterpret_cast<const uint4*>(train + ((int64_t)b * cap + c0) * 32);
  for (int i = tid; i < 2 * kChunk; i += kRows) s_desc[i] = i < 2 * ncols ? cb[i] : make_uint4(0, 0, 0, 0);
  for (int i = tid; i < kChunk; i += kRows) s_col[i] = kNoKey;
  const int r = r0 + tid;
  const bool rv = r < nr;
  u32x4 q0 = {0, 0, 0, 0}, q1 = q0;
  if (rv) {
    const u32x4* p = reinterpret_cast<const u32x4*>(query + ((int64_t)b * cap + r) * 32);
    q0 = p[0];
    q1 = p[1];
  }
  // a row past the set's end contributes kNoKey to every column minimum: (d << 16) | ~0 = ~0
  const uint32_t rbits = rv ? (uint32_t)r : kNoKey;
  uint32_t rkey = kNoKey;
  __syncthreads();
  // one 64-column block (PART: the set's last, partial one -- its columns past the end never win a row)
  auto walk = [&](int cbk, auto part_t) {
    constexpr bool PART = decltype(part_t)::value;
    const uint32_t nv = (uint32_t)(ncols - cbk * 64);  // valid columns of the block
    uint32_t j = (uint32_t)lane;  // this lane's column in the block at step s: (lane + s) mod 64
    uint32_t acc = kNoKey, rk = kNoKey;
#pragma unroll 8
    for (int s = 0; s < 64; ++s) {
      const uint32_t d = hamming(q0, q1, &s_desc[(cbk * 64 + j) * 2]);
      uint32_t kr = (d << 16) | j;  // the block's column offset is added after the walk
      if constexpr (PART) kr = j < nv ? kr : kNoKey;
      rk = min(rk, kr);
      // the accumulator of column (lane + s) comes from lane + 1, which held it at step s - 1
      // (at s = 0 every lane's is still kNoKey, so the rotation is harmless there)
      acc = min(wave_rol1(acc), (d << 16) | rbits);
      j = (j + 1) & 63;
    }
    if (rk != kNoKey) rkey = min(rkey, rk | (uint32_t)(c0 + cbk * 64));
    // after step 63 lane i holds column i - 1's minimum: one more rotation puts column i on lane i
    atomicMin(&s_col[cbk * 64 + lane], wave_rol1(acc));
  };
  const int nfull = ncols >> 6;
  for (int cbk = 0; cbk < nfull; ++cbk) walk(cbk, std::false_type{});
  if (ncols & 63) walk(nfull, std::true_type{});
  if (rv && rkey != kNoKey) atomicMin(&rowkey[(int64_t)b * cap + r], rkey);
  __syncthreads();
  for (int i = tid; i < ncols; i += kRows)
    if (s_col[i] != kNoKey) atomicMin(&colkey[(int64_t)b * cap + c0 + i], s_col[i]);
}

__global__ void k_bf_finish(const int32_t* __restrict__ nq, const int32_t* __restrict__ nt, int cap,
                            uint32_t* __restrict__ rowkey, uint32_t* __restrict__ colkey,
                            int32_t* __restrict__ matches, int32_t* __restrict__ nmatch) {
  const int b = blockIdx.x;
  int n0 = nq[b], n1 = nt[b];
  n0 = n0 < 0 ? 0 : (n0 > cap ? cap : n0);
  n1 = n1 < 0 ? 0 : (n1 > cap ? cap : n1);
  const int r0 = n0, r1 = n1;  // the key entries the pass may have lowered
  if (n1 == 0) n0 = 0;
  __shared__ int s_w[16];
  __shared__ int s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  uint32_t* rk = rowkey + (int64_t)b * cap;
  uint32_t* ck = colkey + (int64_t)b * cap;
  for (int base = 0; base < n0; base += blockDim.x) {
    int q = base + threadIdx.x;
    uint32_t key = kNoKey;
    bool keep = false;
    if (q < n0) {
      key = rk[q];
      keep = key != kNoKey && (ck[key & 0xFFFFu] & 0xFFFFu) == (uint32_t)q;
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
      o[1] = (int32_t)(key & 0xFFFFu);
      o[2] = (int32_t)(key >> 16);
    }
    __syncthreads();
    if (threadIdx.x == 0) s_carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) nmatch[b] = s_carry;
  // every read of this set's keys is behind the loop's last barrier: reset them for the next call
  for (int i = threadIdx.x; i < r0; i += blockDim.x) rk[i] = kNoKey;
  for (int i = threadIdx.x; i < r1; i += blockDim.x) ck[i] = kNoKey;
}

}  // namespace

int bf_init(fvo_ctx* ctx) {
  const int64_t n = (int64_t)ctx->cfg.max_batch * ctx->kp_cap;
  if (ctx->kp_cap > 0xFFFF) return fvo_fail(ctx, "BF: kp_capacity must be <= 65535 (16-bit indices in the keys)");
  int rc;
  if ((rc = fvo_alloc(ctx, &ctx->bf_rowkey, n)) || (rc = fvo_alloc(ctx, &ctx->bf_colkey, n))) return rc;
  // the key arrays start (and are left by every k_bf_finish) at "no key"
  FVO_HIP(ctx, hipMemset(ctx->bf_rowkey, 0xFF, n * sizeof(uint32_t)));
  FVO_HIP(ctx, hipMemset(ctx->bf_colkey, 0xFF, n * sizeof(uint32_t)));
  return 0;
}

int bf_run(fvo_ctx* ctx, const uint8_t* q, const int32_t* nq, const uint8_t* t, const int32_t* nt, int batch, int cap,
           int32_t* matches, int32_t* nmatch, hipStream_t s) {
  if ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(t)) & 15)
    return fvo_fail(ctx, "descriptor buffers must be 16-byte aligned");
  const dim3 grid((cap + kRows - 1) / kRows, (cap + kChunk - 1) / kChunk, batch);
  FVO_TIMED(ctx, KN_BF_ARGMIN, s, hipLaunchKernelGGL(k_bf_pass, grid, dim3(kRows), 0, s, q, nq, t, nt, cap,
                                                     ctx->bf_rowkey, ctx->bf_colkey));
  FVO_TIMED(ctx, KN_BF_FINISH, s, hipLaunchKernelGGL(k_bf_finish, dim3(batch), dim3(256), 0, s, nq, nt, cap,
                                                     ctx->bf_rowkey, ctx->bf_colkey, matches, nmatch));
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
