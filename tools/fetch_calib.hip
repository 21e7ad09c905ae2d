// FETCH_SIZE / WRITE_SIZE calibration for the SGBM row pass's access widths.
//
// MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for 16-B-per-lane streaming reads (it
// reports half the bytes); the row pass (csrc/sgbm.hip k_sg_rows) reads its volume with
// raw_buffer_load_b96 (D = 96: 12 B per lane, one 768-B block per 4-row column) plus b16 loads
// of the per-row minima.  Each kernel here streams a known byte count from a buffer far larger
// than the 256 MiB Infinity Cache, in one access pattern, so FETCH_SIZE per dispatch divided by
// the bytes gives that pattern's factor.  Patterns:
//   b128     16 B per lane, contiguous (the guide's calibrated case: expect 0.5)
//   b32      4 B per lane, contiguous
//   b96v     the row pass's V(y) read: wave per 4-row group, lane (r, q) reads 12 B at
//            column*768 + r*192 + q*12, columns in order; 64 pairs x 150 groups x 864 columns
//   b96vp    b96v plus the previous-row read (rows 1-3: row r-1 of the group, row 0: row 3 of
//            the previous group) -- the row pass's sweep-1 loads exactly
//   b64v     the D = 64 layout (8 B per lane, 512-B columns)
//   b16m     the per-row minima: lane (r, q) reads 2 B of the [group][x][4] u16 array at sub-row
//            r - 1 (row 0: sub-row 3 of the previous group)
//   st64     8-B-per-lane non-temporal stores in the cost pass's layout (WRITE_SIZE calibration)
//   st64t    the same with temporal stores
//   st128    the same volume written 16 B per lane, each column's 192-B row piece by 12 lanes
// Usage: fetch_calib [pattern ...]  (default: all); prints one JSON line per pattern with the
// bytes it moves and the time per launch (HIP events), so the rocprofv3 pass is joined by name.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

namespace {

constexpr int kPairs = 64, kGroups = 150, kCols = 864;  // 960x600, D = 96: 150 4-row groups, width1 864

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, (short)0, (int)__builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}
// the row pass's XCD-aware block order (csrc/fvo_device.h xcd_block): consecutive groups of a
// pair on one XCD, so a group's previous-row read can hit the L2 its neighbour filled
__device__ __forceinline__ int2 xcd_gb() {
  const int gx = gridDim.x, N = gx * gridDim.y;
  const int L = blockIdx.y * gx + blockIdx.x;
  const int per = N >> 3;
  const int lg = L < (per << 3) ? (L & 7) * per + (L >> 3) : L;
  return make_int2(lg % gx, lg / gx);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__global__ __launch_bounds__(256) void k_cal_b128(const uint4* __restrict__ src, size_t n4, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_cal_b32(const uint32_t* __restrict__ src, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= src[i];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// wave per (pair, group); PQ packed words per lane (2: D = 64, 3: D = 96); PREV adds the
// previous-row load of the row pass
template <int PQ, bool PREV>
__global__ __launch_bounds__(64, 4) void k_cal_rows(const uint16_t* __restrict__ vol, uint32_t* __restrict__ sink) {
  constexpr int D = PQ * 32, XS = 4 * D * 2;  // bytes per column of a group
  const int lane = threadIdx.x, q = lane & 15, r = lane >> 4;
  const int2 gb = xcd_gb();
  const int g = gb.x, b = gb.y;
  const uint64_t plane = (uint64_t)kCols * XS;
  const uint16_t* pb = vol + (uint64_t)b * kGroups * plane / 2;
  const __amdgpu_buffer_rsrc_t rs = rsrc(pb, (uint32_t)(kGroups * plane));
  const uint32_t voff = (uint32_t)(g * plane + r * (D * 2) + q * PQ * 4);
  const uint32_t poff = r > 0 ? voff - D * 2 : (g > 0 ? (uint32_t)((g - 1) * plane + 3 * D * 2 + q * PQ * 4) : 0x80000000u);
  uint32_t acc = 0;
#pragma unroll 4
  for (int x = 0; x < kCols; ++x) {
    const uint32_t so = uni((uint32_t)x * XS);
    if constexpr (PQ == 3) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, voff, so, 0);
      acc ^= v[0] ^ v[1] ^ v[2];
      if constexpr (PREV) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b96(rs, poff, so, 0);
        acc += w[0] ^ w[1] ^ w[2];
      }
    } else {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, so, 0);
      acc ^= v[0] ^ v[1];
      if constexpr (PREV) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b64(rs, poff, so, 0);
        acc += w[0] ^ w[1];
      }
    }
  }
  sink[((size_t)b * kGroups + g) * 64 + lane] = acc;
}

// the per-row minima [pair][group][x][4] u16, read as the row pass reads the previous row's
__global__ __launch_bounds__(64, 4) void k_cal_b16m(const uint16_t* __restrict__ mv, uint32_t* __restrict__ sink) {
  const int lane = threadIdx.x, r = lane >> 4;
  const int2 gb = xcd_gb();
  const int g = gb.x, b = gb.y;
  const uint16_t* pb = mv + (uint64_t)b * kGroups * kCols * 4;
  const __amdgpu_buffer_rsrc_t rs = rsrc(pb, (uint32_t)(kGroups * kCols * 8));
  const uint32_t off = r > 0 ? (uint32_t)(((uint64_t)g * kCols * 4 + r - 1) * 2)
                             : (g > 0 ? (uint32_t)(((uint64_t)(g - 1) * kCols * 4 + 3) * 2) : 0x80000000u);
  uint32_t acc = 0;
#pragma unroll 4
  for (int x = 0; x < kCols; ++x) acc += (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, off, uni((uint32_t)x * 8), 0);
  sink[((size_t)b * kGroups + g) * 64 + lane] = acc;
}

// the cost pass's V stores: 8 lanes per column, 12 disparities (24 B) per lane as three 8-B
// non-temporal stores per row; blocks of 32 columns walk the rows in order, so every byte of
// the [group][x][4][D] volume is written once
__global__ __launch_bounds__(256) void k_cal_st64(uint16_t* __restrict__ vol) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, q = tid & 7, col = tid >> 3;
  const int x = blockIdx.x * 32 + col, b = blockIdx.y;
  if (x >= kCols) return;
  constexpr int D = 96;
  const uint64_t plane = (uint64_t)kCols * 4 * D;
  uint16_t* pb = vol + (uint64_t)b * kGroups * plane;
  for (int y = 0; y < kGroups * 4; ++y) {
    u32x2* p = reinterpret_cast<u32x2*>(pb + (uint64_t)(y >> 2) * plane + (uint64_t)x * 4 * D + (y & 3) * D + q * 12);
#pragma unroll
    for (int i = 0; i < 3; ++i) __builtin_nontemporal_store(u32x2{(uint32_t)y, (uint32_t)x + i}, p + i);
  }
}

// the same volume with plain (temporal) 8-B stores, and with whole 16-B-per-lane row pieces: lane
// (c, k) of a 12-lane column group writes bytes [16k, 16k + 16) of the column's 192-B row piece
template <bool NT>
__global__ __launch_bounds__(256) void k_cal_st64t(uint16_t* __restrict__ vol) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, q = tid & 7, col = tid >> 3;
  const int x = blockIdx.x * 32 + col, b = blockIdx.y;
  if (x >= kCols) return;
  constexpr int D = 96;
  const uint64_t plane = (uint64_t)kCols * 4 * D;
  uint16_t* pb = vol + (uint64_t)b * kGroups * plane;
  for (int y = 0; y < kGroups * 4; ++y) {
    u32x2* p = reinterpret_cast<u32x2*>(pb + (uint64_t)(y >> 2) * plane + (uint64_t)x * 4 * D + (y & 3) * D + q * 12);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if constexpr (NT) __builtin_nontemporal_store(u32x2{(uint32_t)y, (uint32_t)x + i}, p + i);
      else p[i] = u32x2{(uint32_t)y, (uint32_t)x + i};
    }
  }
}
__global__ __launch_bounds__(192) void k_cal_st128(uint16_t* __restrict__ vol) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, k = tid % 12, col = tid / 12;  // 16 columns x 12 lanes
  const int x = blockIdx.x * 16 + col, b = blockIdx.y;
  if (x >= kCols) return;
  constexpr int D = 96;
  const uint64_t plane = (uint64_t)kCols * 4 * D;
  uint16_t* pb = vol + (uint64_t)b * kGroups * plane;
  for (int y = 0; y < kGroups * 4; ++y) {
    u32x4* p = reinterpret_cast<u32x4*>(pb + (uint64_t)(y >> 2) * plane + (uint64_t)x * 4 * D + (y & 3) * D) + k;
    __builtin_nontemporal_store(u32x4{(uint32_t)y, (uint32_t)x, 0u, 1u}, p);
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> pats;
  for (int i = 1; i < argc; ++i) pats.push_back(argv[i]);
  if (pats.empty()) pats = {"b128", "b32", "b96v", "b96vp", "b64v", "b16m", "st64", "st64t", "st128"};
  const size_t volBytes = (size_t)kPairs * kGroups * kCols * 768;  // 6.37 GB: the row pass's V at B = 64
  const size_t mBytes = (size_t)kPairs * kGroups * kCols * 8;
  uint8_t* vol;
  uint8_t* mv;
  uint32_t* sink;
  CK(hipMalloc(&vol, volBytes));
  CK(hipMalloc(&mv, mBytes));
  CK(hipMalloc(&sink, (size_t)kPairs * kGroups * 64 * 4 + (1 << 24)));
  CK(hipMemset(vol, 1, volBytes));
  CK(hipMemset(mv, 1, mBytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const auto& pt : pats) {
    double bytes = 0;  // unique bytes the pattern moves (read, or written for st64)
    auto launch = [&]() {
      if (pt == "b128") {
        bytes = (double)volBytes;
        hipLaunchKernelGGL(k_cal_b128, dim3(8192), dim3(256), 0, 0, (const uint4*)vol, volBytes / 16, sink);
      } else if (pt == "b32") {
        bytes = (double)volBytes;
        hipLaunchKernelGGL(k_cal_b32, dim3(8192), dim3(256), 0, 0, (const uint32_t*)vol, volBytes / 4, sink);
      } else if (pt == "b96v" || pt == "b96vp") {
        bytes = (double)volBytes;
        auto k = pt == "b96v" ? k_cal_rows<3, false> : k_cal_rows<3, true>;
        hipLaunchKernelGGL(k, dim3(kGroups, kPairs), dim3(64), 0, 0, (const uint16_t*)vol, sink);
      } else if (pt == "b64v") {
        bytes = (double)volBytes * 2 / 3;
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_cal_rows<2, false>), dim3(kGroups, kPairs), dim3(64), 0, 0, (const uint16_t*)vol, sink);
      } else if (pt == "b16m") {
        bytes = (double)mBytes;
        hipLaunchKernelGGL(k_cal_b16m, dim3(kGroups, kPairs), dim3(64), 0, 0, (const uint16_t*)mv, sink);
      } else if (pt == "st64t") {
        bytes = (double)volBytes;
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_cal_st64t<false>), dim3((kCols + 31) / 32, kPairs), dim3(256), 0, 0, (uint16_t*)vol);
      } else if (pt == "st128") {
        bytes = (double)volBytes;
        hipLaunchKernelGGL(k_cal_st128, dim3((kCols + 15) / 16, kPairs), dim3(192), 0, 0, (uint16_t*)vol);
      } else if (pt == "st64") {
        bytes = (double)volBytes;
        hipLaunchKernelGGL(k_cal_st64, dim3((kCols + 31) / 32, kPairs), dim3(256), 0, 0, (uint16_t*)vol);
      } else {
        fprintf(stderr, "unknown pattern %s\n", pt.c_str());
        exit(2);
      }
      CK(hipGetLastError());
    };
    launch();  // warm-up
    CK(hipDeviceSynchronize());
    const int reps = 5;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("{\"pattern\": \"%s\", \"bytes\": %.0f, \"ms\": %.4f, \"gbs\": %.1f}\n", pt.c_str(), bytes, ms, bytes / ms * 1e-6);
    fflush(stdout);
  }
  CK(hipFree(vol));
  CK(hipFree(mv));
  CK(hipFree(sink));
  return 0;
}
