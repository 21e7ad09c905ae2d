// Argument / config validation of libfvo's C ABI (csrc/capi.cpp) exercised on the host under
// AddressSanitizer + UndefinedBehaviorSanitizer (tools/sanitize.sh, SURVEY.md §5 "Race
// detection / sanitizers").  Linked against tests/sanitize/host_stubs.cpp instead of the device
// layer: every entry point is called with good arguments (the stub launcher must be reached)
// and with each class of bad argument the boundary rejects (status < 0, fvo_last_error set,
// no launch).  Exit status 0 = all checks passed.
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/fvo.h"

extern std::string g_last_launch;

static int g_fail = 0, g_checks = 0;

#define CHECK(cond)                                                       \
  do {                                                                    \
    ++g_checks;                                                           \
    if (!(cond)) {                                                        \
      ++g_fail;                                                           \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                     \
  } while (0)

// rc must be < 0 with an error message and no launcher reached
static void rejected(fvo_ctx* c, int rc) {
  CHECK(rc < 0);
  CHECK(std::strlen(fvo_last_error(c)) > 0);
  CHECK(g_last_launch.empty());
}

static void reached(int rc, const char* launcher) {
  CHECK(rc == 0);
  CHECK(g_last_launch == launcher);
}

int main() {
  // ---- config
  fvo_config cfg;
  fvo_config_default(&cfg, 960, 600);
  CHECK(fvo_config_size() == (int32_t)sizeof(fvo_config));
  CHECK(cfg.nfeatures == 500 && cfg.num_disparities == 96 && cfg.P1 == 392 && cfg.P2 == 1568);
  const char* fields[] = {"width", "height", "max_batch", "nfeatures", "scale_factor", "nlevels", "edge_threshold",
                          "first_level", "wta_k", "score_type", "patch_size", "fast_threshold", "min_disparity",
                          "num_disparities", "block_size", "P1", "P2", "disp12_max_diff", "pre_filter_cap",
                          "uniqueness_ratio", "sgbm_stripes", "kp_capacity", "stages", "ba_window",
                          "ba_max_landmarks", "ba_max_obs", "sgbm_max_batch", "sgbm_mode", "sgbm_lanes",
                          "sgbm_cols", "sgbm_handoff_us"};
  for (size_t i = 0; i < sizeof(fields) / sizeof(fields[0]); ++i) CHECK(fvo_config_offset(fields[i]) == (int32_t)(4 * i));
  CHECK(fvo_config_offset("nope") == -1 && fvo_config_offset(nullptr) == -1);
  CHECK(fvo_abi_version() == FVO_ABI_VERSION);

  // ---- context creation
  fvo_ctx* c = nullptr;
  CHECK(fvo_create(0, nullptr, &c) < 0 && c == nullptr);
  CHECK(fvo_create(0, &cfg, nullptr) < 0);
  fvo_config bad = cfg;
  bad.max_batch = 0;
  CHECK(fvo_create(0, &bad, &c) < 0 && c == nullptr);
  bad = cfg;
  bad.width = 32;
  CHECK(fvo_create(0, &bad, &c) < 0);
  bad = cfg;
  bad.stages = 1 << 12;
  CHECK(fvo_create(0, &bad, &c) < 0);
  bad = cfg;
  bad.stages = FVO_STAGE_BF;  // no ORB stage and no kp_capacity
  CHECK(fvo_create(0, &bad, &c) < 0);
  bad = cfg;
  bad.block_size = 5;  // refused by the SGBM stage init: the context is released cleanly
  CHECK(fvo_create(0, &bad, &c) < 0 && c == nullptr);
  CHECK(fvo_create(99, &cfg, &c) < 0);
  cfg.max_batch = 4;
  CHECK(fvo_create(0, &cfg, &c) == 0 && c != nullptr);
  CHECK(fvo_kp_capacity(c) == 2 * 500 + 64 && fvo_kp_capacity(nullptr) == 0);
  CHECK(std::strcmp(fvo_last_error(nullptr), "null context") == 0);

  // host stand-ins for device buffers (the stubs never dereference them)
  static uint8_t u8[1 << 16];
  static int32_t i32[1 << 12];
  static float f32[1 << 12];
  static double f64[1 << 12];
  static int16_t i16[1 << 12];
  const int cap = fvo_kp_capacity(c), W = 960, H = 600;
  auto reset = [] { g_last_launch.clear(); };

  // ---- ORB
  reset(); rejected(c, fvo_orb_detect_compute(c, nullptr, 1, W * H, W, f32, u8, i32, cap, nullptr));
  reset(); rejected(c, fvo_orb_detect_compute(c, u8, 5, W * H, W, f32, u8, i32, cap, nullptr));
  reset(); rejected(c, fvo_orb_detect_compute(c, u8, -1, W * H, W, f32, u8, i32, cap, nullptr));
  reset(); rejected(c, fvo_orb_detect_compute(c, u8, 1, W * H, W - 1, f32, u8, i32, cap, nullptr));
  reset(); rejected(c, fvo_orb_detect_compute(c, u8, 1, W * H - 1, W, f32, u8, i32, cap, nullptr));
  reset(); rejected(c, fvo_orb_detect_compute(c, u8, 1, W * H, W, f32, u8, i32, 0, nullptr));
  reset(); CHECK(fvo_orb_detect_compute(c, u8, 0, W * H, W, f32, u8, i32, cap, nullptr) == 0 && g_last_launch.empty());
  reset(); reached(fvo_orb_detect_compute(c, u8, 4, W * H, W, f32, u8, i32, cap, nullptr), "orb_run");
  CHECK(fvo_orb_detect_compute(nullptr, u8, 1, W * H, W, f32, u8, i32, cap, nullptr) < 0);

  // ---- BF
  reset(); rejected(c, fvo_bf_match(c, u8, i32, nullptr, i32, 1, cap, i32, i32, nullptr));
  reset(); rejected(c, fvo_bf_match(c, u8, i32, u8, i32, 1, cap + 1, i32, i32, nullptr));
  reset(); rejected(c, fvo_bf_match(c, u8, i32, u8, i32, 1, 0, i32, i32, nullptr));
  reset(); reached(fvo_bf_match(c, u8, i32, u8, i32, 2, cap, i32, i32, nullptr), "bf_run");

  // ---- SGBM
  reset(); rejected(c, fvo_sgbm(c, u8, nullptr, 1, W * H, W, i16, nullptr, nullptr));
  reset(); rejected(c, fvo_sgbm(c, u8, u8, 1, W * H, W - 8, i16, nullptr, nullptr));
  reset(); rejected(c, fvo_sgbm(c, u8, u8, 9, W * H, W, i16, nullptr, nullptr));
  reset(); reached(fvo_sgbm(c, u8, u8, 4, W * H, W, i16, nullptr, nullptr), "sgbm_run");

  // ---- back-projection / PnP
  reset(); rejected(c, fvo_backproject(c, i16, f32, f32, i32, i32, 1, cap, nullptr, 0.25, f32, f32, i32, nullptr));
  reset(); rejected(c, fvo_backproject(c, i16, f32, f32, i32, i32, 1, 0, f64, 0.25, f32, f32, i32, nullptr));
  reset(); reached(fvo_backproject(c, i16, f32, f32, i32, i32, 1, cap, f64, 0.25, f32, f32, i32, nullptr),
                   "backproject_run");
  reset(); rejected(c, fvo_pnp_ransac(c, f32, f32, i32, 1, cap, f64, f64, 1.f, 0.99, 0, f64, f64, f64, i32, u8, nullptr));
  reset(); rejected(c, fvo_pnp_ransac(c, f32, f32, i32, 1, cap, f64, f64, 1.f, 0.99, 1001, f64, f64, f64, i32, u8,
                                      nullptr));
  reset(); rejected(c, fvo_pnp_ransac(c, f32, f32, i32, 1, cap, f64, f64, 1.f, 1.0, 1000, f64, f64, f64, i32, u8,
                                      nullptr));
  reset(); rejected(c, fvo_pnp_ransac(c, f32, f32, i32, 1, cap, f64, nullptr, 1.f, 0.99, 1000, f64, f64, f64, i32, u8,
                                      nullptr));
  reset(); reached(fvo_pnp_ransac(c, f32, f32, i32, 1, cap, f64, f64, 1.f, 0.99, 1000, f64, f64, f64, i32, u8, nullptr),
                   "pnp_run");

  // ---- BA
  float* unaligned = reinterpret_cast<float*>(reinterpret_cast<char*>(f32) + 4);
  reset(); rejected(c, fvo_keypoint_stereo(c, i16, f32, i32, 1, cap, f64, 0.25, unaligned, nullptr));
  reset(); rejected(c, fvo_keypoint_stereo(c, i16, f32, i32, 1, cap + 1, f64, 0.25, f32, nullptr));
  reset(); reached(fvo_keypoint_stereo(c, i16, f32, i32, 1, cap, f64, 0.25, f32, nullptr), "ba_stereo_run");
  reset(); rejected(c, fvo_ba_windows(c, f32, i32, i32, i32, f32, f64, 12, cap, 9, 5, 0, f64, 0.25, f64, 8, 10, f64,
                                      f64, nullptr));  // n_windows > max_batch
  reset(); rejected(c, fvo_ba_windows(c, f32, i32, i32, i32, f32, f64, 12, cap, 9, 2, 0, f64, 0.25, nullptr, 8, 10,
                                      f64, f64, nullptr));
  reset(); reached(fvo_ba_windows(c, f32, i32, i32, i32, f32, f64, 12, cap, 9, 2, 0, f64, 0.25, f64, 8, 10, f64, f64,
                                  nullptr), "ba_run");
  reset(); rejected(c, fvo_ba_count_births(c, nullptr, i32, f32, 12, cap, 9, 2, 0, nullptr));
  reset(); rejected(c, fvo_ba_count_births(c, i32, i32, unaligned, 12, cap, 9, 2, 0, nullptr));
  reset(); rejected(c, fvo_ba_count_births(c, i32, i32, f32, 12, cap, 9, 5, 0, nullptr));  // n_windows > max_batch
  reset(); reached(fvo_ba_count_births(c, i32, i32, f32, 12, cap, 9, 2, 0, nullptr), "ba_births_run");
  reset(); rejected(c, fvo_ba_landmarks(c, 0, nullptr, i32, nullptr));
  reset(); reached(fvo_ba_landmarks(c, 0, f64, i32, nullptr), "ba_export_run");

  // ---- mono
  reset(); rejected(c, fvo_gather_matches(c, f32, f32, i32, i32, 5, cap, f32, f32, i32, nullptr));
  reset(); reached(fvo_gather_matches(c, f32, f32, i32, i32, 2, cap, f32, f32, i32, nullptr), "gather_run");
  reset(); rejected(c, fvo_find_essential(c, f32, f32, i32, 1, cap, 0.0, 480, 300, 0.999, 1.0, 1000, f64, u8, i32,
                                          nullptr));
  reset(); rejected(c, fvo_find_essential(c, f32, f32, i32, 1, cap + 1, 640, 480, 300, 0.999, 1.0, 1000, f64, u8, i32,
                                          nullptr));
  reset(); reached(fvo_find_essential(c, f32, f32, i32, 1, cap, 640, 480, 300, 0.999, 1.0, 1000, f64, u8, i32, nullptr),
                   "essential_run");
  reset(); rejected(c, fvo_recover_pose(c, f64, i32, f32, f32, i32, 1, cap, 640, 480, 300, 50, nullptr, f64, f64, i32,
                                        nullptr));
  reset(); reached(fvo_recover_pose(c, f64, i32, f32, f32, i32, 1, cap, 640, 480, 300, 50, f64, f64, f64, i32, nullptr),
                   "recover_run");

  // ---- ingest / blur
  reset(); rejected(c, fvo_undistort_gray(c, u8, 1, 3 * W * H, 3 * W - 1, f64, f64, u8, W * H, W, nullptr));
  reset(); reached(fvo_undistort_gray(c, u8, 1, 3 * W * H, 3 * W, f64, f64, u8, W * H, W, nullptr), "ingest_run");
  reset(); rejected(c, fvo_motion_blur(c, u8, 1, W * H, W, 10, 0.5, i32, i32, 16, u8, u8 + 8, W * H, W, nullptr));
  reset(); rejected(c, fvo_motion_blur(c, u8, 1, W * H, W, 32, 0.0, i32, i32, 16, u8, u8 + 8, W * H, W, nullptr));
  reset(); rejected(c, fvo_motion_blur(c, u8, 1, W * H, W, 10, 0.0, i32, i32, 16, u8, u8, W * H, W, nullptr));
  reset(); reached(fvo_motion_blur(c, u8, 1, W * H, W, 10, 0.0, i32, i32, 16, u8, u8 + 8, W * H, W, nullptr),
                   "motion_blur_run");

  // ---- map
  reset(); rejected(c, fvo_map_transform(c, f32, 2, i32, 1, cap, f64, i32, 100, f64, f32, nullptr));
  reset(); rejected(c, fvo_map_transform(c, f32, 3, i32, 1, cap, f64, i32, 100, nullptr, nullptr, nullptr));
  reset(); reached(fvo_map_transform(c, f32, 3, i32, 1, cap, f64, i32, 100, f64, nullptr, nullptr), "map_transform_run");
  reset(); rejected(c, fvo_chain_poses(c, f64, i32, i32, 2, 3, f64, f64, nullptr, nullptr));
  reset(); rejected(c, fvo_chain_poses(c, f64, nullptr, nullptr, 2, 3, f64, f64, nullptr, nullptr));
  reset(); rejected(c, fvo_chain_poses(c, f64, i32, nullptr, -1, 3, f64, f64, nullptr, nullptr));
  reset(); CHECK(fvo_chain_poses(c, f64, i32, nullptr, 0, 3, f64, f64, nullptr, nullptr) == 0 && g_last_launch.empty());
  reset(); reached(fvo_chain_poses(c, f64, i32, i32, 2, 3, f64, f64, i32, nullptr), "chain_poses_run");
  {  // step bookkeeping: region count / overlap validation, count guard ranges
    static char buf[4096];
    fvo_region r[FVO_MAX_REGIONS + 1];
    for (int i = 0; i <= FVO_MAX_REGIONS; ++i) r[i] = fvo_region{buf + 64 * i, buf + 3000, 16};
    reset(); rejected(c, fvo_copy_regions(c, FVO_MAX_REGIONS + 1, r, nullptr));
    reset(); rejected(c, fvo_copy_regions(c, 2, nullptr, nullptr));
    reset(); CHECK(fvo_copy_regions(c, 0, nullptr, nullptr) == 0 && g_last_launch.empty());
    reset(); reached(fvo_copy_regions(c, 2, r, nullptr), "copy_regions_run");
    fvo_region ov[2] = {{buf, buf + 8, 16}, {buf + 100, buf + 200, 16}};  // own source overlaps
    reset(); rejected(c, fvo_copy_regions(c, 2, ov, nullptr));
    fvo_region dd[2] = {{buf, buf + 1000, 16}, {buf + 8, buf + 2000, 16}};  // destinations overlap
    reset(); rejected(c, fvo_copy_regions(c, 2, dd, nullptr));
    fvo_region xs[2] = {{buf, buf + 1000, 16}, {buf + 1000, buf + 2000, 16}};  // dst 0 = src 0? no: dst 1 = src 0
    reset(); rejected(c, fvo_copy_regions(c, 2, xs, nullptr));
    fvo_region nb[1] = {{buf, buf + 100, -1}};
    reset(); rejected(c, fvo_copy_regions(c, 1, nb, nullptr));
    fvo_region z[1] = {{nullptr, nullptr, 0}};  // empty regions are skipped
    reset(); CHECK(fvo_copy_regions(c, 1, z, nullptr) == 0 && g_last_launch.empty());
    reset(); rejected(c, fvo_count_guard(c, i32, i32, 4, 0, i32, -3, nullptr, nullptr));
    reset(); rejected(c, fvo_count_guard(c, nullptr, i32, 4, 1, i32, -3, nullptr, nullptr));
    reset(); CHECK(fvo_count_guard(c, i32, nullptr, 0, 1, nullptr, -3, nullptr, nullptr) == 0 && g_last_launch.empty());
    reset(); reached(fvo_count_guard(c, i32, nullptr, 4, 2, i32, -3, i32, nullptr), "count_guard_run");
  }
  CHECK(fvo_voxel_workspace_bytes(0) == -1 && fvo_voxel_workspace_bytes(10) > 0);
  reset(); rejected(c, fvo_voxel_down_sample(c, f64, 10, 0.0, u8, 1 << 16, f64, i32, i32, nullptr));
  reset(); rejected(c, fvo_voxel_down_sample(c, f64, 10, 0.5, u8, -1, f64, i32, i32, nullptr));
  reset(); CHECK(fvo_voxel_down_sample(c, nullptr, 0, 0.5, nullptr, 0, f64, i32, i32, nullptr) == 0);
  reset(); reached(fvo_voxel_down_sample(c, f64, 10, 0.5, u8, 1 << 16, f64, i32, i32, nullptr), "voxel_run");

  // ---- timing / debug / names
  CHECK(fvo_kernel_count() > 0 && std::strlen(fvo_kernel_name(0)) > 0 && fvo_kernel_name(-1)[0] == 0 &&
        fvo_kernel_name(fvo_kernel_count())[0] == 0);
  CHECK(fvo_timing_enable(c, ~0ull) == 0);
  double ms[64];
  int32_t launches[64];
  CHECK(fvo_timing_read(c, ms, launches) == 0 && fvo_timing_read(c, nullptr, launches) < 0);
  void* ptr = nullptr;
  int64_t bytes = 0;
  CHECK(fvo_debug_buffer(c, 99, &ptr, &bytes) < 0 && fvo_debug_buffer(c, 3, nullptr, &bytes) < 0);
  reset(); CHECK(fvo_debug_buffer(c, 2, &ptr, &bytes) == 0 && g_last_launch == "orb_score_debug");

  fvo_destroy(c);
  fvo_destroy(nullptr);

  // a context without the ORB stage: stage checks and kp_capacity handling
  fvo_config_default(&cfg, 960, 600);
  cfg.stages = FVO_STAGE_BF;
  cfg.kp_capacity = 64;
  CHECK(fvo_create(0, &cfg, &c) == 0);
  reset(); rejected(c, fvo_orb_detect_compute(c, u8, 1, W * H, W, f32, u8, i32, 64, nullptr));
  reset(); rejected(c, fvo_sgbm(c, u8, u8, 1, W * H, W, i16, nullptr, nullptr));
  reset(); reached(fvo_bf_match(c, u8, i32, u8, i32, 1, 64, i32, i32, nullptr), "bf_run");
  fvo_destroy(c);

  std::printf("capi_check: %d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
