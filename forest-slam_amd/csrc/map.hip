// Map accumulation for gfx950 — SURVEY.md §8f rank 4, the reference's per-frame map update:
//   stereo_slam.py:308-318   homogeneous = hstack(points3D, 1); pts = (cum @ homogeneous.T)[:3].T
//                            all_points_3D.append(pts); create_point_cloud(concat) (PointCloud2,
//                            x/y/z FLOAT32 fields, point_step 12)
//   mono_slam.py:144-164     points = np.dot(cum, vstack(points.T, 1))[:3].T,
//                            o3d PointCloud.voxel_down_sample(0.5), concatenated into the map,
//                            pc2.create_cloud_xyz32
//   gt_mapping.py:62-66      the same with the ground-truth pose
// Kernels:
//   k_map_xform   thread per point: x' = ((T00 x + T01 y) + T02 z) + T03 in fp64 (no contraction;
//                 numpy's dgemm order is unpinned), appended at the map's running count as
//                 f64 xyz and/or the PointCloud2 float32 xyz record; HBM-bound (12 B in, 24+12 out).
//   k_chain       the pose chain stereo_slam.py:306 on the device (fvo_chain_poses): the map's
//                 placing poses without a host round trip.
//   voxel_down_sample (Open3D PointCloud::VoxelDownSample): min bound by block partials, voxel
//                 keys floor((p - (min - v/2)) / v) packed 3x21 bits, stable radix sort of
//                 (key, index) (hipcub), segment heads + exclusive scan, then one thread per
//                 voxel sums its points in the original order (= Open3D's AccumulatedPoint
//                 insertion order, so the fp64 sums are bit-identical) and divides by the count.
//                 Output ordered by voxel key (Open3D's unordered_map order is unspecified).
// Specification: oracle/map_ref.cpp.
#include <hipcub/hipcub.hpp>

#include "fvo_device.h"

namespace {

__global__ __launch_bounds__(256) void k_map_xform(const float* __restrict__ pts, int stride, int64_t cap,
                                                   const int32_t* __restrict__ npts, int batch,
                                                   const double* __restrict__ T, const int32_t* __restrict__ count,
                                                   int64_t map_cap, double* __restrict__ out64,
                                                   float* __restrict__ out32) {
  const int b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = min((int64_t)npts[b], cap);
  if ((int64_t)blockIdx.x * 256 >= n) return;  // uniform: no point of set b in this block
  // the set's offset in the map: one wave sums the counts of the sets before it
  __shared__ int64_t s_base;
  if (threadIdx.x < 64) {
    int64_t part = 0;
    for (int j = threadIdx.x; j < b; j += 64) part += min((int64_t)npts[j], cap);
    part = wave_sum(part);
    if (threadIdx.x == 0) s_base = count[0] + part;
  }
  __syncthreads();
  if (i >= n) return;
  const int64_t o = s_base + i;
  if (o >= map_cap) return;
  const float* p = pts + ((int64_t)b * cap + i) * stride;
  const double x = p[0], y = p[1], z = p[2];
  const double* M = T + 16 * b;
  double r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) r[k] = ((M[4 * k] * x + M[4 * k + 1] * y) + M[4 * k + 2] * z) + M[4 * k + 3] * 1.0;
  if (out64) {
    out64[3 * o] = r[0];
    out64[3 * o + 1] = r[1];
    out64[3 * o + 2] = r[2];
  }
  if (out32) {
    out32[3 * o] = (float)r[0];
    out32[3 * o + 1] = (float)r[1];
    out32[3 * o + 2] = (float)r[2];
  }
}

__global__ void k_map_count(const int32_t* __restrict__ npts, int batch, int64_t cap, int32_t* __restrict__ count) {
  if (threadIdx.x != 0) return;
  int64_t t = count[0];
  for (int j = 0; j < batch; ++j) t += min((int64_t)npts[j], cap);
  count[0] = (int32_t)min(t, (int64_t)INT32_MAX);
}

// Pose chains (fvo_chain_poses): 16 lanes per sequence, lane (i, j) holds cum[i][j]; per frame
// in order, c'_ij = ((c_i0 t_0j + c_i1 t_1j) + c_i2 t_2j) + c_i3 t_3j with the row of cum from the
// sequence's lanes (stereo_slam.py:306, np.dot(cumulative, T)), applied when the frame is posed
// (status >= 0: the reference chained it, :292).  Four sequences per wave; the serial chain is
// ~n dependent 4-term dot products, a few microseconds per batch.
__global__ __launch_bounds__(64) void k_chain(const double* __restrict__ T, const int32_t* __restrict__ status,
                                              const int32_t* __restrict__ npts, int n_seq, int n,
                                              double* __restrict__ cum, double* __restrict__ cum_out,
                                              int32_t* __restrict__ npts_out) {
  const int lane = threadIdx.x, sq = blockIdx.x * 4 + (lane >> 4), e = lane & 15, i = e >> 2, j = e & 3;
  const bool live = sq < n_seq;
  const int sqc = live ? sq : n_seq - 1;  // lanes past the last sequence mirror it and store nothing
  const int row = (lane & ~15) + 4 * i;
  double c = cum[(int64_t)sqc * 16 + e];
  for (int f = 0; f < n; ++f) {
    const int64_t k = (int64_t)sqc * n + f;
    const int st = status[k];
    const double* M = T + k * 16;
    const double t0 = M[j], t1 = M[4 + j], t2 = M[8 + j], t3 = M[12 + j];
    const double c0 = __shfl(c, row, 64), c1 = __shfl(c, row + 1, 64), c2 = __shfl(c, row + 2, 64),
                 c3 = __shfl(c, row + 3, 64);
    const double nc = ((c0 * t0 + c1 * t1) + c2 * t2) + c3 * t3;
    if (st >= 0) c = nc;
    if (live) cum_out[k * 16 + e] = c;
    if (live && npts_out && e == 0) npts_out[k] = st >= 0 ? npts[k] : 0;
  }
  if (live) cum[(int64_t)sq * 16 + e] = c;
}

constexpr int kVxBlocks = 256;

__global__ __launch_bounds__(256) void k_vx_bounds(const double* __restrict__ p, int64_t n, double* __restrict__ part) {
  __shared__ double sm[6][256];
  double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double v = p[3 * i + k];
      mn[k] = fmin(mn[k], v);
      mx[k] = fmax(mx[k], v);
    }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    sm[k][threadIdx.x] = mn[k];
    sm[3 + k][threadIdx.x] = mx[k];
  }
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        sm[k][threadIdx.x] = fmin(sm[k][threadIdx.x], sm[k][threadIdx.x + s]);
        sm[3 + k][threadIdx.x] = fmax(sm[3 + k][threadIdx.x], sm[3 + k][threadIdx.x + s]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = sm[threadIdx.x][0];
}

// keys: min over the block partials (min/max are exact, any order), vmin = min - v*0.5 (Eigen
// `GetMinBound() - voxel_size3 * 0.5`), ref = (p - vmin) / v, index = int(floor(ref)).
__global__ __launch_bounds__(256) void k_vx_keys(const double* __restrict__ p, int64_t n, double voxel,
                                                 const double* __restrict__ part, int nparts,
                                                 uint64_t* __restrict__ keys, int32_t* __restrict__ idx,
                                                 int32_t* __restrict__ status) {
  __shared__ double vmin[3];
  if (threadIdx.x < 3) {
    double m = INFINITY;
    for (int j = 0; j < nparts; ++j) m = fmin(m, part[j * 6 + threadIdx.x]);
    vmin[threadIdx.x] = m - voxel * 0.5;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t key = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double ref = (p[3 * i + k] - vmin[k]) / voxel;
    const double f = floor(ref);
    int64_t v = (f >= 0.0 && f < 2097152.0) ? (int64_t)f : -1;
    if (v < 0) {
      status[0] = 1;  // outside the 21-bit key range: result invalid, reported
      v = 0;
    }
    key = (key << 21) | (uint64_t)v;
  }
  keys[i] = key;
  idx[i] = (int32_t)i;
}

__global__ __launch_bounds__(256) void k_vx_heads(const uint64_t* __restrict__ keys, int64_t n,
                                                  int32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_vx_starts(const int32_t* __restrict__ flag, const int32_t* __restrict__ pos,
                                                   int64_t n, int32_t* __restrict__ start,
                                                   int32_t* __restrict__ n_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (flag[i]) start[pos[i]] = (int32_t)i;
  if (i == n - 1) {
    const int32_t nv = pos[i] + flag[i];
    start[nv] = (int32_t)n;
    n_out[0] = nv;
  }
}

__global__ __launch_bounds__(256) void k_vx_average(const double* __restrict__ p, const int32_t* __restrict__ sidx,
                                                    const int32_t* __restrict__ start,
                                                    const int32_t* __restrict__ n_out, double* __restrict__ out) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n_out[0]) return;
  const int32_t s = start[v], e = start[v + 1];
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;  // AccumulatedPoint: point_ += points_[index], insertion order
  for (int32_t j = s; j < e; ++j) {
    const int64_t q = sidx[j];
    a0 = a0 + p[3 * q];
    a1 = a1 + p[3 * q + 1];
    a2 = a2 + p[3 * q + 2];
  }
  const double c = (double)(e - s);
  out[3 * v] = a0 / c;
  out[3 * v + 1] = a1 / c;
  out[3 * v + 2] = a2 / c;
}

struct VxLayout {
  size_t keys_a, keys_b, idx_a, idx_b, flag, pos, start, part, status, cub, total, sort_bytes, scan_bytes;
};

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

int vx_layout(int64_t n, VxLayout& L) {
  size_t sort_bytes = 0, scan_bytes = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                         (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 63) != hipSuccess)
    return -1;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n) !=
      hipSuccess)
    return -1;
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
  L.keys_a = take(8 * (size_t)n);
  L.keys_b = take(8 * (size_t)n);
  L.idx_a = take(4 * (size_t)n);
  L.idx_b = take(4 * (size_t)n);
  L.flag = take(4 * (size_t)n);
  L.pos = take(4 * (size_t)n);
  L.start = take(4 * ((size_t)n + 1));
  L.part = take(8 * 6 * kVxBlocks);
  L.status = take(4);
  L.sort_bytes = sort_bytes;
  L.scan_bytes = scan_bytes;
  L.cub = take(sort_bytes > scan_bytes ? sort_bytes : scan_bytes);
  L.total = o;
  return 0;
}

}  // namespace

int map_transform_run(fvo_ctx* ctx, const float* pts, int stride, const int32_t* npts, int batch, int64_t cap,
                      const double* T, int32_t* count, int64_t map_cap, double* out64, float* out32, hipStream_t s) {
  dim3 grid((unsigned)((cap + 255) / 256), batch);
  FVO_TIMED(ctx, KN_MAP_XFORM, s, {
    hipLaunchKernelGGL(k_map_xform, grid, dim3(256), 0, s, pts, stride, cap, npts, batch, T, count, map_cap, out64,
                       out32);
  });
  FVO_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_map_count, dim3(1), dim3(64), 0, s, npts, batch, cap, count);
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

int chain_poses_run(fvo_ctx* ctx, const double* T, const int32_t* status, const int32_t* npts, int n_seq, int n,
                    double* cum, double* cum_out, int32_t* npts_out, hipStream_t s) {
  hipLaunchKernelGGL(k_chain, dim3((n_seq + 3) / 4), dim3(64), 0, s, T, status, npts, n_seq, n, cum, cum_out,
                     npts_out);
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}

int64_t voxel_workspace_bytes(int64_t n) {
  VxLayout L;
  if (n < 1 || vx_layout(n, L)) return -1;
  return (int64_t)L.total;
}

int voxel_run(fvo_ctx* ctx, const double* pts, int64_t n, double voxel, void* ws, size_t ws_bytes, double* out,
              int32_t* n_out, int32_t* status, hipStream_t s) {
  VxLayout L;
  if (vx_layout(n, L)) return fvo_fail(ctx, "voxel_down_sample: workspace size query failed");
  if (ws_bytes < L.total) return fvo_fail(ctx, "voxel_down_sample: workspace too small");
  char* w = (char*)ws;
  uint64_t *ka = (uint64_t*)(w + L.keys_a), *kb = (uint64_t*)(w + L.keys_b);
  int32_t *ia = (int32_t*)(w + L.idx_a), *ib = (int32_t*)(w + L.idx_b);
  int32_t *flag = (int32_t*)(w + L.flag), *pos = (int32_t*)(w + L.pos), *start = (int32_t*)(w + L.start);
  double* part = (double*)(w + L.part);
  int32_t* st = status ? status : (int32_t*)(w + L.status);
  const unsigned g = (unsigned)((n + 255) / 256);
  const int nparts = (int)((g < (unsigned)kVxBlocks) ? g : kVxBlocks);
  FVO_HIP(ctx, hipMemsetAsync(st, 0, 4, s));
  FVO_TIMED(ctx, KN_VOXEL, s, {
    hipLaunchKernelGGL(k_vx_bounds, dim3(nparts), dim3(256), 0, s, pts, n, part);
    hipLaunchKernelGGL(k_vx_keys, dim3(g), dim3(256), 0, s, pts, n, voxel, part, nparts, ka, ia, st);
    size_t sb = L.sort_bytes;
    (void)hipcub::DeviceRadixSort::SortPairs(w + L.cub, sb, ka, kb, ia, ib, (int)n, 0, 63, s);
    hipLaunchKernelGGL(k_vx_heads, dim3(g), dim3(256), 0, s, kb, n, flag);
    size_t cb = L.scan_bytes;
    (void)hipcub::DeviceScan::ExclusiveSum(w + L.cub, cb, flag, pos, (int)n, s);
    hipLaunchKernelGGL(k_vx_starts, dim3(g), dim3(256), 0, s, flag, pos, n, start, n_out);
    hipLaunchKernelGGL(k_vx_average, dim3(g), dim3(256), 0, s, pts, ib, start, n_out, out);
  });
  FVO_LAUNCH_CHECK(ctx);
  return 0;
}
