// ORACLE — test infrastructure only. Never linked into the product.
//
// Restates the reference's map accumulation:
//   stereo_slam.py:308-318  homogeneous_points3D = np.hstack((points3D, ones))
//                           transformed = (cumulative_est_tf_mat @ homogeneous.T)[:3].T
//                           all_points_3D.append(...); create_point_cloud(np.concatenate(...))
//                           (PointCloud2 with FLOAT32 x/y/z: the fp64 values rounded to float)
//   mono_slam.py:144-164    points (pc2.read_points float32 -> Python float), np.dot(cum, ...)
//                           then Open3D 0.17 PointCloud::VoxelDownSample(0.5):
//                             voxel_min_bound = GetMinBound() - voxel_size3 * 0.5
//                             ref_coord = (points_[i] - voxel_min_bound) / voxel_size
//                             voxel_index = (int(floor(ref_coord(0))), ... )
//                             voxelindex_to_accpoint[voxel_index].AddPoint(*this, i)   (point_ += p)
//                             output: accpoint.GetAveragePoint() = point_ / double(num_of_points_)
// The 4x4 @ 4xN product is evaluated per element as ((T0 x + T1 y) + T2 z) + T3 (numpy's dgemm
// order/FMA use is BLAS-dependent: unpinned, within an ulp).  Open3D iterates an unordered_map;
// this restatement emits voxels in lexicographic (ix, iy, iz) order (the set is identical).
#include <cmath>
#include <cstdint>
#include <map>
#include <tuple>

extern "C" {

void ref_map_transform(const float* pts, int64_t n, int stride, const double* T, double* out64, float* out32) {
  for (int64_t i = 0; i < n; ++i) {
    const double x = pts[i * stride], y = pts[i * stride + 1], z = pts[i * stride + 2];
    for (int k = 0; k < 3; ++k) {
      const double r = ((T[4 * k] * x + T[4 * k + 1] * y) + T[4 * k + 2] * z) + T[4 * k + 3] * 1.0;
      out64[3 * i + k] = r;
      out32[3 * i + k] = (float)r;
    }
  }
}

int64_t ref_voxel_down_sample(const double* p, int64_t n, double voxel, double* out) {
  if (n == 0) return 0;
  double mn[3] = {p[0], p[1], p[2]};
  for (int64_t i = 1; i < n; ++i)
    for (int k = 0; k < 3; ++k) mn[k] = std::fmin(mn[k], p[3 * i + k]);
  double vmin[3];
  for (int k = 0; k < 3; ++k) vmin[k] = mn[k] - voxel * 0.5;
  struct Acc { double s[3] = {0, 0, 0}; int64_t c = 0; };
  std::map<std::tuple<int, int, int>, Acc> vox;
  for (int64_t i = 0; i < n; ++i) {
    int id[3];
    for (int k = 0; k < 3; ++k) id[k] = (int)std::floor((p[3 * i + k] - vmin[k]) / voxel);
    Acc& a = vox[std::make_tuple(id[0], id[1], id[2])];
    for (int k = 0; k < 3; ++k) a.s[k] += p[3 * i + k];
    a.c += 1;
  }
  int64_t o = 0;
  for (auto& kv : vox) {
    for (int k = 0; k < 3; ++k) out[3 * o + k] = kv.second.s[k] / (double)kv.second.c;
    ++o;
  }
  return o;
}

}  // extern "C"
