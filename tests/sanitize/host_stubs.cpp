// Host-only test double of libfvo's device layer, for the sanitizer build of capi.cpp
// (tools/sanitize.sh): the per-stage init / launch functions and the few HIP runtime calls
// capi.cpp makes are replaced by functions that record which launcher the entry point reached
// and touch every pointer argument's first element on the host side where it is host memory
// in this test (nothing here runs on a GPU).  Test infrastructure only; never linked into
// libfvo.so.
#include <cstring>
#include <string>

#include "../../forest-slam_amd/csrc/fvo_internal.h"

std::string g_last_launch;
static int g_fake_event = 0;

static int hit(const char* name) {
  g_last_launch = name;
  return 0;
}

// --- HIP runtime calls made by capi.cpp
extern "C" {
hipError_t hipSetDevice(int d) { return d >= 0 && d < 8 ? hipSuccess : hipErrorInvalidDevice; }
hipError_t hipFree(void* p) {
  delete[] static_cast<char*>(p);
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) {
  *e = reinterpret_cast<hipEvent_t>(&g_fake_event);
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) {
  *ms = 1.0f;
  return hipSuccess;
}
hipError_t hipMemsetAsync(void*, int, size_t, hipStream_t) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "stub hip error"; }
}

// --- stage inits: one small host allocation each, released by capi.cpp's hipFree
int orb_init(fvo_ctx* c) { c->pyr = reinterpret_cast<uint8_t*>(new char[16]); return hit("orb_init"); }
int bf_init(fvo_ctx* c) { c->bf_rowkey = reinterpret_cast<uint32_t*>(new char[16]); return hit("bf_init"); }
int sgbm_init(fvo_ctx* c) {
  if (c->cfg.block_size != 7) return fvo_fail(c, "SGBM: only blockSize=7 is supported");
  c->sg_raw = reinterpret_cast<int16_t*>(new char[16]);
  return hit("sgbm_init");
}
int pose_init(fvo_ctx* c) { c->pnp_max_iters = 1000; return hit("pose_init"); }
int ba_init(fvo_ctx*) { return hit("ba_init"); }
int mono_init(fvo_ctx*) { return hit("mono_init"); }

// --- launchers
int orb_run(fvo_ctx*, const uint8_t*, int, int64_t, int, float*, uint8_t*, int32_t*, int, hipStream_t) {
  return hit("orb_run");
}
int bf_run(fvo_ctx*, const uint8_t*, const int32_t*, const uint8_t*, const int32_t*, int, int, int32_t*, int32_t*,
           hipStream_t) {
  return hit("bf_run");
}
int sgbm_run(fvo_ctx*, const uint8_t*, const uint8_t*, int, int64_t, int, int16_t*, int32_t*, hipStream_t) {
  return hit("sgbm_run");
}
int backproject_run(fvo_ctx*, const int16_t*, const float*, const float*, const int32_t*, const int32_t*, int, int,
                    const double*, double, float*, float*, int32_t*, hipStream_t) {
  return hit("backproject_run");
}
int pnp_run(fvo_ctx*, const float*, const float*, const int32_t*, int, int, const double*, const double*, float, double,
            int, double*, double*, double*, int32_t*, uint8_t*, hipStream_t) {
  return hit("pnp_run");
}
int ba_stereo_run(fvo_ctx*, const int16_t*, const float*, const int32_t*, int, int, const double*, double, float*,
                  hipStream_t) {
  return hit("ba_stereo_run");
}
int ba_run(fvo_ctx*, const float*, const int32_t*, const int32_t*, const int32_t*, const float*, const double*, int, int,
           int, int, int, const double*, double, const double*, int, int, double*, double*, hipStream_t) {
  return hit("ba_run");
}
int ba_export_run(fvo_ctx*, int, double*, int32_t*, hipStream_t) { return hit("ba_export_run"); }
int ba_births_run(fvo_ctx*, const int32_t*, const int32_t*, const float*, int, int, int, int, int, hipStream_t) {
  return hit("ba_births_run");
}
int gather_run(fvo_ctx*, const float*, const float*, const int32_t*, const int32_t*, int, int, float*, float*, int32_t*,
               hipStream_t) {
  return hit("gather_run");
}
int essential_run(fvo_ctx*, const float*, const float*, const int32_t*, int, int, double, double, double, double, double,
                  int, double*, uint8_t*, int32_t*, hipStream_t) {
  return hit("essential_run");
}
int recover_run(fvo_ctx*, const double*, const int32_t*, const float*, const float*, const int32_t*, int, int, double,
                double, double, double, double*, double*, double*, int32_t*, hipStream_t) {
  return hit("recover_run");
}
int ingest_run(fvo_ctx*, const uint8_t*, int, int64_t, int, const double*, const double*, uint8_t*, int64_t, int,
               hipStream_t) {
  return hit("ingest_run");
}
int motion_blur_run(fvo_ctx*, const uint8_t*, int, int64_t, int, int, const int32_t*, const int32_t*, int, uint8_t*,
                    uint8_t*, int64_t, int, hipStream_t) {
  return hit("motion_blur_run");
}
int map_transform_run(fvo_ctx*, const float*, int, const int32_t*, int, int64_t, const double*, int32_t*, int64_t,
                      double*, float*, hipStream_t) {
  return hit("map_transform_run");
}
int chain_poses_run(fvo_ctx*, const double*, const int32_t*, const int32_t*, int, int, double*, double*, int32_t*,
                    hipStream_t) {
  return hit("chain_poses_run");
}
int copy_regions_run(fvo_ctx*, int, const fvo_region*, hipStream_t) { return hit("copy_regions_run"); }
int count_guard_run(fvo_ctx*, const int32_t*, const int32_t*, int, int, int32_t*, int32_t, int32_t*, hipStream_t) {
  return hit("count_guard_run");
}
int64_t voxel_workspace_bytes(int64_t n) { return 64 * n + 4096; }
int voxel_run(fvo_ctx*, const double*, int64_t, double, void*, size_t, double*, int32_t*, int32_t*, hipStream_t) {
  return hit("voxel_run");
}
int orb_blur_debug(fvo_ctx*) { return hit("orb_blur_debug"); }
int orb_score_debug(fvo_ctx*) { return hit("orb_score_debug"); }
