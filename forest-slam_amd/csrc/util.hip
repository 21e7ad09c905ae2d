// Step bookkeeping in one launch each (no reference counterpart: the reference's per-frame loop
// keeps these as Python lists).  A batched front end's back stage otherwise issues a dozen
// small copies and elementwise ops per step; each is a dispatch that, beside the next step's
// disparity kernels, waits for a free register slot -- so they are batched here:
//   k_copy_regions  up to FVO_MAX_REGIONS device-to-device copies (block row = region,
//                   16-B vector moves when the region allows, else bytes)
//   k_count_guard   per frame: status = code where any keypoint count of the frame's sets is
//                   negative (ORB's overflow report), clamped counts out
#include <algorithm>

#include "fvo_device.h"

namespace {

// single-wave blocks: the back stage issues these beside the front stage's kernels, and a
// one-wave block needs one free wave slot, not four on the same CU
__global__ __launch_bounds__(64) void k_copy_regions(FvoRegions r) {
  const fvo_region g = r.r[blockIdx.y];
  const uint8_t* src = static_cast<const uint8_t*>(g.src);
  uint8_t* dst = static_cast<uint8_t*>(g.dst);
  const int64_t n = g.bytes;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)n) & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (int64_t i = t0; i < n / 16; i += step) d4[i] = s4[i];
  } else if ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)n) & 3) == 0) {
    const uint32_t* s1 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d1 = reinterpret_cast<uint32_t*>(dst);
    for (int64_t i = t0; i < n / 4; i += step) d1[i] = s1[i];
  } else {
    for (int64_t i = t0; i < n; i += step) dst[i] = src[i];
  }
}

__global__ void k_count_guard(const int32_t* __restrict__ cnt, const int32_t* __restrict__ q_cnt, int n, int sets,
                              int32_t* __restrict__ status, int32_t code, int32_t* __restrict__ nkp_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool over = false;
  for (int s = 0; s < sets; ++s) over |= cnt[s * n + i] < 0 || (q_cnt && q_cnt[s * n + i] < 0);
  if (status && over) status[i] = code;
  if (nkp_out) nkp_out[i] = max(cnt[i], 0);
}

}  // namespace

int copy_regions_run(fvo_ctx* ctx, int count, const fvo_region* regions, hipStream_t s) {
  FvoRegions r{};
  int64_t most = 0;
  for (int i = 0; i < count; ++i) {
    r.r[i] = regions[i];
    most = std::max(most, regions[i].bytes);
  }
  // enough blocks for the largest region at 16 B per thread, at most 4096 per region
  const int64_t bx = std::min<int64_t>(4096, std::max<int64_t>(1, (most / 16 + 63) / 64));
  hipLaunchKernelGGL(k_copy_regions, dim3((unsigned)bx, count), dim3(64), 0, s, r);
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

int count_guard_run(fvo_ctx* ctx, const int32_t* cnt, const int32_t* q_cnt, int n, int sets, int32_t* status,
                    int32_t code, int32_t* nkp_out, hipStream_t s) {
  hipLaunchKernelGGL(k_count_guard, dim3((n + 63) / 64), dim3(64), 0, s, cnt, q_cnt, n, sets, status, code, nkp_out);
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
