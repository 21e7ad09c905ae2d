// extern "C" entry points of libfvo.so (include/fvo.h).  Thin: argument checks, context
// lifetime, dispatch to the per-stage launchers.  No allocation in the hot calls.
#include <cstddef>
#include <cstdio>
#include <cstring>

#include "fvo_internal.h"

int fvo_fail(fvo_ctx* ctx, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return -1;
}

hipEvent_t fvo_event(fvo_ctx* ctx) {
  if (!ctx->tpool.empty()) {
    hipEvent_t e = ctx->tpool.back();
    ctx->tpool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// The ABI layout: 31 int32 / float fields, no padding (include/fvo.h).
static_assert(sizeof(fvo_config) == 31 * 4, "fvo_config layout changed: bump FVO_ABI_VERSION");
static_assert(offsetof(fvo_config, scale_factor) == 16 && offsetof(fvo_config, sgbm_max_batch) == 104 &&
                  offsetof(fvo_config, sgbm_handoff_us) == 120,
              "fvo_config field offsets changed: bump FVO_ABI_VERSION");

extern "C" {

int fvo_abi_version(void) { return FVO_ABI_VERSION; }

int32_t fvo_config_size(void) { return (int32_t)sizeof(fvo_config); }

int32_t fvo_config_offset(const char* f) {
  if (!f) return -1;
#define FVO_OFS(name) if (!std::strcmp(f, #name)) return (int32_t)offsetof(fvo_config, name);
  FVO_OFS(width) FVO_OFS(height) FVO_OFS(max_batch) FVO_OFS(nfeatures) FVO_OFS(scale_factor) FVO_OFS(nlevels)
  FVO_OFS(edge_threshold) FVO_OFS(first_level) FVO_OFS(wta_k) FVO_OFS(score_type) FVO_OFS(patch_size)
  FVO_OFS(fast_threshold) FVO_OFS(min_disparity) FVO_OFS(num_disparities) FVO_OFS(block_size) FVO_OFS(P1)
  FVO_OFS(P2) FVO_OFS(disp12_max_diff) FVO_OFS(pre_filter_cap) FVO_OFS(uniqueness_ratio) FVO_OFS(sgbm_stripes)
  FVO_OFS(kp_capacity) FVO_OFS(stages) FVO_OFS(ba_window) FVO_OFS(ba_max_landmarks) FVO_OFS(ba_max_obs)
  FVO_OFS(sgbm_max_batch) FVO_OFS(sgbm_mode) FVO_OFS(sgbm_lanes) FVO_OFS(sgbm_cols) FVO_OFS(sgbm_handoff_us)
#undef FVO_OFS
  return -1;
}

void fvo_config_default(fvo_config* c, int32_t width, int32_t height) {
  std::memset(c, 0, sizeof(*c));
  c->width = width;
  c->height = height;
  c->max_batch = 1;
  c->nfeatures = 500;
  c->scale_factor = 1.2f;
  c->nlevels = 8;
  c->edge_threshold = 31;
  c->first_level = 0;
  c->wta_k = 2;
  c->score_type = 0;
  c->patch_size = 31;
  c->fast_threshold = 20;
  c->min_disparity = 0;
  c->num_disparities = 6 * 16;
  c->block_size = 7;
  c->P1 = 8 * 7 * 7;
  c->P2 = 32 * 7 * 7;
  c->disp12_max_diff = 0;
  c->pre_filter_cap = 0;
  c->uniqueness_ratio = 0;
  c->sgbm_stripes = 4;
  c->kp_capacity = 0;
  c->stages = FVO_STAGE_ALL;
  c->ba_window = 10;
  c->ba_max_landmarks = 4096;
  c->ba_max_obs = 32768;
  c->sgbm_max_batch = 0;
  c->sgbm_mode = FVO_SGBM_CLASSIC;
  c->sgbm_lanes = 0;
  c->sgbm_cols = 0;
  c->sgbm_handoff_us = 0;
}

static void release(fvo_ctx* c) {
  void* ptrs[] = {c->pyr,        c->blur,      c->score,     c->cand,     c->hel,
                  c->ncand,      c->nsel1,     c->nsel2,     c->koff,     c->scratch, c->fast_rec, c->rt.xofs,  c->rt.xc1,
                  c->rt.yofs,    c->rt.yc1,    c->umax,      c->bf_rowkey, c->bf_colkey, c->sg_ckpt,
                  c->sg_V,      c->sg_M,      c->sg_raw,    c->sg_hand,   c->sg_ctl,    c->pnp_hyp,  c->pnp_good,
                  c->pnp_sub,    c->rs_table, c->pnp_models, c->pnp_ws, c->pnp_state, c->pnp_plan, c->pnp_pts, c->ba_ws,
                  c->em_x, c->em_models, c->em_good, c->em_nmod, c->em_state, c->em_ws};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->ba_s2) (void)hipStreamDestroy(c->ba_s2);

  if (c->ba_fork) (void)hipEventDestroy(c->ba_fork);
  if (c->ba_join) (void)hipEventDestroy(c->ba_join);
}

int fvo_create(int device, const fvo_config* cfg, fvo_ctx** out) {
  if (!cfg || !out) return -1;
  *out = nullptr;
  fvo_ctx* c = new fvo_ctx();
  c->device = device;
  c->cfg = *cfg;
  auto bail = [&](int rc) {
    std::fprintf(stderr, "fvo_create: %s\n", c->err.c_str());
    release(c);
    delete c;
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) { c->err = "hipSetDevice failed"; return bail(-1); }
  if (c->cfg.stages == 0) c->cfg.stages = FVO_STAGE_ALL;
  const int st = c->cfg.stages;
  if (st & ~FVO_STAGE_ALL) { c->err = "unknown bits in stages"; return bail(-1); }
  if (cfg->max_batch < 1) { c->err = "max_batch must be >= 1"; return bail(-1); }
  if ((st & (FVO_STAGE_ORB | FVO_STAGE_SGBM)) && (cfg->width < 64 || cfg->height < 64)) {
    c->err = "image size must be at least 64x64";
    return bail(-1);
  }
  if (!(st & FVO_STAGE_ORB) && (st & (FVO_STAGE_BF | FVO_STAGE_POSE | FVO_STAGE_BA | FVO_STAGE_MONO)) &&
      cfg->kp_capacity < 1) {
    c->err = "kp_capacity must be set when the ORB stage is not enabled";
    return bail(-1);
  }
  c->kp_cap = cfg->kp_capacity > 0 ? cfg->kp_capacity : 2 * cfg->nfeatures + 64;
  int rc = 0;
  if (((st & FVO_STAGE_ORB) && (rc = orb_init(c))) || ((st & FVO_STAGE_BF) && (rc = bf_init(c))) ||
      ((st & FVO_STAGE_SGBM) && (rc = sgbm_init(c))) || ((st & FVO_STAGE_POSE) && (rc = pose_init(c))) ||
      ((st & FVO_STAGE_BA) && (rc = ba_init(c))) || ((st & FVO_STAGE_MONO) && (rc = mono_init(c))))
    return bail(rc);
  *out = c;
  return 0;
}

void fvo_destroy(fvo_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (auto& r : c->trecs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  for (auto e : c->tpool) (void)hipEventDestroy(e);
  release(c);
  delete c;
}

const char* fvo_last_error(const fvo_ctx* c) { return c ? c->err.c_str() : "null context"; }
int fvo_kp_capacity(const fvo_ctx* c) { return c ? c->kp_cap : 0; }
int64_t fvo_workspace_bytes(const fvo_ctx* c) { return c ? c->ws_bytes : 0; }

static int check_batch(fvo_ctx* c, int32_t batch, int stage) {
  if (!c) return -1;
  if (!(c->cfg.stages & stage)) return fvo_fail(c, "stage not enabled in this context (fvo_config.stages)");
  if (batch < 0 || batch > c->cfg.max_batch) return fvo_fail(c, "batch exceeds max_batch");
  return 0;
}

int fvo_orb_detect_compute(fvo_ctx* c, const uint8_t* images, int32_t batch, int64_t image_stride, int32_t pitch,
                           float* keypoints, uint8_t* descriptors, int32_t* counts, int32_t cap, fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_ORB)) return -1;
  if (batch == 0) return 0;
  if (!images || !keypoints || !descriptors || !counts) return fvo_fail(c, "null pointer argument");
  if (pitch < c->cfg.width || image_stride < (int64_t)pitch * c->cfg.height) return fvo_fail(c, "bad pitch/stride");
  if (cap < 1) return fvo_fail(c, "cap must be >= 1");
  return orb_run(c, images, batch, image_stride, pitch, keypoints, descriptors, counts, cap, (hipStream_t)stream);
}

int fvo_bf_match(fvo_ctx* c, const uint8_t* query, const int32_t* n_query, const uint8_t* train,
                 const int32_t* n_train, int32_t batch, int32_t cap, int32_t* matches, int32_t* n_matches,
                 fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_BF)) return -1;
  if (batch == 0) return 0;
  if (!query || !n_query || !train || !n_train || !matches || !n_matches) return fvo_fail(c, "null pointer argument");
  if (cap < 1 || cap > c->kp_cap) return fvo_fail(c, "cap must be in [1, fvo_kp_capacity()]");
  return bf_run(c, query, n_query, train, n_train, batch, cap, matches, n_matches, (hipStream_t)stream);
}

int fvo_sgbm(fvo_ctx* c, const uint8_t* left, const uint8_t* right, int32_t batch, int64_t image_stride,
             int32_t pitch, int16_t* disparity, int32_t* status, fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_SGBM)) return -1;
  if (batch == 0) return 0;
  if (!left || !right || !disparity) return fvo_fail(c, "null pointer argument");
  if (pitch < c->cfg.width || image_stride < (int64_t)pitch * c->cfg.height) return fvo_fail(c, "bad pitch/stride");
  if (batch > (c->cfg.sgbm_max_batch > 0 ? c->cfg.sgbm_max_batch : c->cfg.max_batch))
    return fvo_fail(c, "batch exceeds sgbm_max_batch");
  return sgbm_run(c, left, right, batch, image_stride, pitch, disparity, status, (hipStream_t)stream);
}

int fvo_backproject(fvo_ctx* c, const int16_t* disparity, const float* kp0, const float* kp1, const int32_t* matches,
                    const int32_t* n_matches, int32_t batch, int32_t cap, const double* K, double baseline,
                    float* points3d, float* points2d, int32_t* n_points, fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_POSE)) return -1;
  if (batch == 0) return 0;
  if (!disparity || !kp0 || !kp1 || !matches || !n_matches || !K || !points3d || !points2d || !n_points)
    return fvo_fail(c, "null pointer argument");
  if (cap < 1) return fvo_fail(c, "cap must be >= 1");
  return backproject_run(c, disparity, kp0, kp1, matches, n_matches, batch, cap, K, baseline, points3d, points2d,
                         n_points, (hipStream_t)stream);
}

int fvo_pnp_ransac(fvo_ctx* c, const float* points3d, const float* points2d, const int32_t* n_points, int32_t batch,
                   int32_t cap, const double* K, const double* dist, float reprojection_error, double confidence,
                   int32_t iterations, double* rvec, double* tvec, double* T, int32_t* status, uint8_t* inliers,
                   fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_POSE)) return -1;
  if (batch == 0) return 0;
  if (!points3d || !points2d || !n_points || !K || !dist || !rvec || !tvec || !T || !status)
    return fvo_fail(c, "null pointer argument");
  if (cap < 1) return fvo_fail(c, "cap must be >= 1");
  if (iterations < 1 || iterations > c->pnp_max_iters) return fvo_fail(c, "iterations out of range");
  if (!(confidence > 0 && confidence < 1)) return fvo_fail(c, "confidence must be in (0,1)");
  return pnp_run(c, points3d, points2d, n_points, batch, cap, K, dist, reprojection_error, confidence, iterations,
                 rvec, tvec, T, status, inliers, (hipStream_t)stream);
}

int fvo_keypoint_stereo(fvo_ctx* c, const int16_t* disparity, const float* keypoints, const int32_t* n_keypoints,
                        int32_t batch, int32_t cap, const double* K, double baseline, float* stereo,
                        fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_BA)) return -1;
  if (batch == 0) return 0;
  if (!disparity || !keypoints || !n_keypoints || !K || !stereo) return fvo_fail(c, "null pointer argument");
  if (cap < 1 || cap > c->kp_cap) return fvo_fail(c, "cap must be in [1, fvo_kp_capacity()]");
  if (reinterpret_cast<uintptr_t>(stereo) & 15) return fvo_fail(c, "stereo buffer must be 16-byte aligned");
  return ba_stereo_run(c, disparity, keypoints, n_keypoints, batch, cap, K, baseline, stereo, (hipStream_t)stream);
}

int fvo_ba_windows(fvo_ctx* c, const float* keypoints, const int32_t* n_keypoints, const int32_t* matches,
                   const int32_t* n_matches, const float* stereo, const double* T_rel, int32_t n_frames,
                   int32_t cap, int32_t first_end, int32_t n_windows, int32_t first_valid, const double* K,
                   double baseline, const double* inv_sigma2, int32_t n_levels, int32_t iterations,
                   double* T_out, double* stats, fvo_stream stream) {
  if (check_batch(c, n_windows, FVO_STAGE_BA)) return -1;
  if (n_windows == 0) return 0;
  if (!keypoints || !n_keypoints || !matches || !n_matches || !stereo || !T_rel || !K || !inv_sigma2 || !T_out ||
      !stats)
    return fvo_fail(c, "null pointer argument");
  if (reinterpret_cast<uintptr_t>(stereo) & 15) return fvo_fail(c, "stereo buffer must be 16-byte aligned");
  return ba_run(c, keypoints, n_keypoints, matches, n_matches, stereo, T_rel, n_frames, cap, first_end, n_windows,
                first_valid, K, baseline, inv_sigma2, n_levels, iterations, T_out, stats, (hipStream_t)stream);
}

int fvo_ba_count_births(fvo_ctx* c, const int32_t* matches, const int32_t* n_matches, const float* stereo,
                        int32_t n_frames, int32_t cap, int32_t first_end, int32_t n_windows, int32_t first_valid,
                        fvo_stream stream) {
  if (check_batch(c, n_windows, FVO_STAGE_BA)) return -1;
  c->ba_births.valid = false;
  if (n_windows == 0) return 0;
  if (!matches || !n_matches || !stereo) return fvo_fail(c, "null pointer argument");
  if (reinterpret_cast<uintptr_t>(stereo) & 15) return fvo_fail(c, "stereo buffer must be 16-byte aligned");
  return ba_births_run(c, matches, n_matches, stereo, n_frames, cap, first_end, n_windows, first_valid,
                       (hipStream_t)stream);
}

int fvo_ba_landmarks(fvo_ctx* c, int32_t window, double* xyz, int32_t* count, fvo_stream stream) {
  if (check_batch(c, 1, FVO_STAGE_BA)) return -1;
  if (!xyz || !count) return fvo_fail(c, "null pointer argument");
  return ba_export_run(c, window, xyz, count, (hipStream_t)stream);
}

int fvo_gather_matches(fvo_ctx* c, const float* kp0, const float* kp1, const int32_t* matches,
                       const int32_t* n_matches, int32_t batch, int32_t cap, float* p0, float* p1, int32_t* n_points,
                       fvo_stream stream) {
  if (!c) return -1;
  if (batch < 0 || batch > c->cfg.max_batch) return fvo_fail(c, "batch exceeds max_batch");
  if (batch == 0) return 0;
  if (!kp0 || !kp1 || !matches || !n_matches || !p0 || !p1 || !n_points) return fvo_fail(c, "null pointer argument");
  if (cap < 1) return fvo_fail(c, "cap must be >= 1");
  return gather_run(c, kp0, kp1, matches, n_matches, batch, cap, p0, p1, n_points, (hipStream_t)stream);
}

int fvo_find_essential(fvo_ctx* c, const float* p0, const float* p1, const int32_t* n_points, int32_t batch,
                       int32_t cap, double focal, double cx, double cy, double prob, double threshold,
                       int32_t max_iters, double* E, uint8_t* mask, int32_t* status, fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_MONO)) return -1;
  if (batch == 0) return 0;
  if (!p0 || !p1 || !n_points || !E || !status) return fvo_fail(c, "null pointer argument");
  if (cap < 1 || cap > c->kp_cap) return fvo_fail(c, "cap must be in [1, fvo_kp_capacity()]");
  if (!(focal > 0.0)) return fvo_fail(c, "focal must be > 0");
  return essential_run(c, p0, p1, n_points, batch, cap, focal, cx, cy, prob, threshold, max_iters, E, mask, status,
                       (hipStream_t)stream);
}

int fvo_recover_pose(fvo_ctx* c, const double* E, const int32_t* e_status, const float* p0, const float* p1,
                     const int32_t* n_points, int32_t batch, int32_t cap, double focal, double cx, double cy,
                     double distance_thresh, double* R, double* t, double* T, int32_t* n_good, fvo_stream stream) {
  if (check_batch(c, batch, FVO_STAGE_MONO)) return -1;
  if (batch == 0) return 0;
  if (!E || !p0 || !p1 || !n_points || !R || !t || !T || !n_good) return fvo_fail(c, "null pointer argument");
  if (cap < 1 || cap > c->kp_cap) return fvo_fail(c, "cap must be in [1, fvo_kp_capacity()]");
  if (!(focal > 0.0)) return fvo_fail(c, "focal must be > 0");
  return recover_run(c, E, e_status, p0, p1, n_points, batch, cap, focal, cx, cy, distance_thresh, R, t, T, n_good,
                     (hipStream_t)stream);
}

int fvo_undistort_gray(fvo_ctx* c, const uint8_t* bgr, int32_t batch, int64_t src_stride, int32_t src_pitch,
                       const double* K, const double* dist, uint8_t* gray, int64_t dst_stride, int32_t dst_pitch,
                       fvo_stream stream) {
  if (!c) return -1;
  if (batch < 0 || batch > c->cfg.max_batch) return fvo_fail(c, "batch exceeds max_batch");
  if (batch == 0) return 0;
  if (!bgr || !K || !dist || !gray) return fvo_fail(c, "null pointer argument");
  const int W = c->cfg.width, H = c->cfg.height;
  if (src_pitch < 3 * W || src_stride < (int64_t)src_pitch * H || dst_pitch < W || dst_stride < (int64_t)dst_pitch * H)
    return fvo_fail(c, "bad pitch/stride");
  return ingest_run(c, bgr, batch, src_stride, src_pitch, K, dist, gray, dst_stride, dst_pitch, (hipStream_t)stream);
}

int fvo_motion_blur(fvo_ctx* c, const uint8_t* img, int32_t batch, int64_t src_stride, int32_t src_pitch,
                    int32_t ksize, double angle, const int32_t* centers, const int32_t* n_centers, int32_t centers_cap,
                    uint8_t* mask, uint8_t* out, int64_t dst_stride, int32_t dst_pitch, fvo_stream stream) {
  if (!c) return -1;
  if (batch < 0 || batch > c->cfg.max_batch) return fvo_fail(c, "batch exceeds max_batch");
  if (batch == 0) return 0;
  if (!img || !mask || !out || (centers_cap > 0 && (!centers || !n_centers))) return fvo_fail(c, "null pointer argument");
  if (angle != 0.0) return fvo_fail(c, "motion blur: only angle 0 is supported (the reference's value)");
  const int W = c->cfg.width, H = c->cfg.height;
  if (ksize < 1 || ksize > 31) return fvo_fail(c, "motion blur: ksize must be in [1, 31]");
  if (W <= ksize || H <= ksize) return fvo_fail(c, "motion blur: image smaller than the kernel");
  if (centers_cap < 0) return fvo_fail(c, "centers_cap < 0");
  if (src_pitch < W || src_stride < (int64_t)src_pitch * H || dst_pitch < W || dst_stride < (int64_t)dst_pitch * H)
    return fvo_fail(c, "bad pitch/stride");
  if (img == out) return fvo_fail(c, "motion blur: out must not alias img");
  return motion_blur_run(c, img, batch, src_stride, src_pitch, ksize, centers, n_centers, centers_cap, mask, out,
                         dst_stride, dst_pitch, (hipStream_t)stream);
}

int fvo_map_transform(fvo_ctx* c, const float* points, int32_t point_stride, const int32_t* n_points, int32_t batch,
                      int64_t cap, const double* T, int32_t* map_count, int64_t map_cap, double* map_xyz64,
                      float* map_xyz32, fvo_stream stream) {
  if (!c) return -1;
  if (batch < 0) return fvo_fail(c, "batch < 0");
  if (batch == 0) return 0;
  if (!points || !n_points || !T || !map_count || (!map_xyz64 && !map_xyz32)) return fvo_fail(c, "null pointer argument");
  if (point_stride < 3) return fvo_fail(c, "point_stride must be >= 3 floats");
  if (cap < 1 || cap > (int64_t)1 << 31) return fvo_fail(c, "cap must be in [1, 2^31]");
  if (map_cap < 0) return fvo_fail(c, "map_cap < 0");
  return map_transform_run(c, points, point_stride, n_points, batch, cap, T, map_count, map_cap, map_xyz64, map_xyz32,
                           (hipStream_t)stream);
}

int fvo_chain_poses(fvo_ctx* c, const double* T, const int32_t* status, const int32_t* n_points, int32_t n_seq,
                    int32_t n, double* cum_state, double* cum_out, int32_t* n_points_out, fvo_stream stream) {
  if (!c) return -1;
  if (n_seq < 0 || n < 0) return fvo_fail(c, "n_seq and n must be >= 0");
  if (n_seq == 0 || n == 0) return 0;
  if (!T || !status || !cum_state || !cum_out) return fvo_fail(c, "null pointer argument");
  if ((n_points == nullptr) != (n_points_out == nullptr)) return fvo_fail(c, "n_points and n_points_out: both or neither");
  return chain_poses_run(c, T, status, n_points, n_seq, n, cum_state, cum_out, n_points_out, (hipStream_t)stream);
}

int fvo_copy_regions(fvo_ctx* c, int32_t count, const fvo_region* regions, fvo_stream stream) {
  if (!c) return -1;
  if (count < 0 || count > FVO_MAX_REGIONS) return fvo_fail(c, "copy_regions: count out of [0, FVO_MAX_REGIONS]");
  if (count == 0) return 0;
  if (!regions) return fvo_fail(c, "null pointer argument");
  int used = 0;
  fvo_region live[FVO_MAX_REGIONS];
  for (int i = 0; i < count; ++i) {
    const fvo_region& g = regions[i];
    if (g.bytes < 0) return fvo_fail(c, "copy_regions: bytes < 0");
    if (g.bytes == 0) continue;
    if (!g.dst || !g.src) return fvo_fail(c, "copy_regions: null region pointer");
    live[used++] = g;
  }
  auto overlap = [](const void* a, const void* b, int64_t na, int64_t nb) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return x < y + (uintptr_t)nb && y < x + (uintptr_t)na;
  };
  for (int i = 0; i < used; ++i)
    for (int j = 0; j < used; ++j) {
      if (overlap(live[i].dst, live[j].src, live[i].bytes, live[j].bytes) ||
          (i != j && overlap(live[i].dst, live[j].dst, live[i].bytes, live[j].bytes)))
        return fvo_fail(c, "copy_regions: a destination overlaps a source or another destination");
    }
  if (used == 0) return 0;
  return copy_regions_run(c, used, live, (hipStream_t)stream);
}

int fvo_count_guard(fvo_ctx* c, const int32_t* counts, const int32_t* q_counts, int32_t n, int32_t sets,
                    int32_t* status, int32_t code, int32_t* counts_clamped, fvo_stream stream) {
  if (!c) return -1;
  if (n < 0 || sets < 1 || sets > 8) return fvo_fail(c, "count_guard: n < 0 or sets outside [1, 8]");
  if (n == 0) return 0;
  if (!counts) return fvo_fail(c, "null pointer argument");
  return count_guard_run(c, counts, q_counts, n, sets, status, code, counts_clamped, (hipStream_t)stream);
}

int64_t fvo_voxel_workspace_bytes(int64_t n_points) {
  if (n_points < 1 || n_points > INT32_MAX) return -1;
  return voxel_workspace_bytes(n_points);
}

int fvo_voxel_down_sample(fvo_ctx* c, const double* points, int64_t n_points, double voxel_size, void* workspace,
                          int64_t workspace_bytes, double* out, int32_t* n_out, int32_t* status, fvo_stream stream) {
  if (!c) return -1;
  if (!out || !n_out || (n_points > 0 && (!points || !workspace))) return fvo_fail(c, "null pointer argument");
  if (!(voxel_size > 0.0)) return fvo_fail(c, "voxel_size must be > 0");
  if (n_points < 0 || n_points > INT32_MAX) return fvo_fail(c, "n_points out of range");
  if (n_points == 0) {  // Open3D: an empty cloud downsamples to an empty cloud
    FVO_HIP(c, hipMemsetAsync(n_out, 0, 4, (hipStream_t)stream));
    if (status) FVO_HIP(c, hipMemsetAsync(status, 0, 4, (hipStream_t)stream));
    return 0;
  }
  if (workspace_bytes < 0) return fvo_fail(c, "workspace_bytes < 0");
  return voxel_run(c, points, n_points, voxel_size, workspace, (size_t)workspace_bytes, out, n_out, status,
                   (hipStream_t)stream);
}

int fvo_kernel_count(void) { return KN_COUNT; }

const char* fvo_kernel_name(int id) {
  static const char* names[KN_COUNT] = {
      "orb_copy_level0", "orb_resize", "orb_fast_score", "orb_nms_count", "orb_row_scan", "orb_nms_compact",
      "orb_select_fast", "orb_harris", "orb_select_harris", "orb_offsets", "orb_angle", "orb_blur", "orb_brief",
      "bf_argmin", "bf_finish", "sgbm_vert", "sgbm_rows", "sgbm_median", "backproject",
      "pnp_ransac", "ba_stereo", "ba_build", "ba_solve", "gather_matches", "essential_ransac", "recover_pose", "ingest_undistort_gray", "motion_blur", "map_transform", "voxel_down_sample"};
  return (id >= 0 && id < KN_COUNT) ? names[id] : "";
}

int fvo_timing_enable(fvo_ctx* c, uint64_t mask) {
  if (!c) return -1;
  c->tmask = mask;
  return 0;
}

int fvo_timing_read(fvo_ctx* c, double* ms, int32_t* launches) {
  if (!c || !ms || !launches) return -1;
  for (int i = 0; i < KN_COUNT; ++i) { ms[i] = 0.0; launches[i] = 0; }
  for (auto& r : c->trecs) {
    FVO_HIP(c, hipEventSynchronize(r.b));
    float t = 0.f;
    FVO_HIP(c, hipEventElapsedTime(&t, r.a, r.b));
    ms[r.id] += t;
    launches[r.id] += 1;
    c->tpool.push_back(r.a);
    c->tpool.push_back(r.b);
  }
  c->trecs.clear();
  return 0;
}

// Debug/test hook: device pointer + size of an internal workspace buffer of the last call.
// which: 0 pyramid, 1 blurred pyramid, 2 FAST score map (all [max_batch][total_px] u8),
//        3 per-level candidate counts, 4 after retainBest(2n), 5 after retainBest(n) (i32 [B][L]),
//        6 PnP RANSAC inlier count per iteration (i32 [B][1000]), 7 PnP hypotheses (f64 [B][1000][6]),
//        8 PnP RANSAC state (i32 [B][4]: best inlier count, iteration bound, best iteration, points).
int fvo_debug_buffer(fvo_ctx* c, int which, void** ptr, int64_t* bytes) {
  if (!c || !ptr || !bytes) return -1;
  const int64_t B = c->cfg.max_batch;
  switch (which) {
    case 0: *ptr = c->pyr; *bytes = B * c->g.total_px; return 0;
    case 1:  // computed on request from the last call's pyramid (not part of the hot path)
      if (orb_blur_debug(c)) return -1;
      *ptr = c->blur; *bytes = B * c->g.total_px; return 0;
    case 2:  // computed on request from the last call's pyramid (not part of the hot path)
      if (orb_score_debug(c)) return -1;
      *ptr = c->score; *bytes = B * c->g.total_px; return 0;
    case 3: *ptr = c->ncand; *bytes = B * c->g.nlevels * 4; return 0;
    case 4: *ptr = c->nsel1; *bytes = B * c->g.nlevels * 4; return 0;
    case 5: *ptr = c->nsel2; *bytes = B * c->g.nlevels * 4; return 0;
    case 6: *ptr = c->pnp_good; *bytes = B * c->pnp_max_iters * 4; return 0;
    case 7: *ptr = c->pnp_models; *bytes = B * c->pnp_max_iters * 6 * 8; return 0;
    case 8: *ptr = c->pnp_state; *bytes = B * 16; return 0;
    case 9:  // SGBM control words: ticket, generation, hand-off timeouts, per-pair failure flags
      if (!c->sg_ctl) return fvo_fail(c, "no SGBM workspace");
      *ptr = c->sg_ctl; *bytes = (4 + B) * 4; return 0;
    default: return fvo_fail(c, "unknown debug buffer");
  }
}

}  // extern "C"
