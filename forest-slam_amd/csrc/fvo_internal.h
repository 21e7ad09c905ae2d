// Internal declarations shared by the HIP translation units of libfvo.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/fvo.h"

#define FVO_MAX_LEVELS 12

// Pyramid geometry computed on the host exactly as OpenCV's ORB does
// (orb.cpp detectAndCompute: getScale, cvRound(cols * (1.f/scale))).
struct OrbGeom {
  int nlevels;
  int w[FVO_MAX_LEVELS], h[FVO_MAX_LEVELS];
  float scale[FVO_MAX_LEVELS];         // layerScale
  int64_t off[FVO_MAX_LEVELS + 1];      // plane offsets inside one image's pyramid
  int row0[FVO_MAX_LEVELS + 1];         // first global row of each level
  int nfeat[FVO_MAX_LEVELS];            // nfeaturesPerLevel
  int64_t cand_off[FVO_MAX_LEVELS + 1]; // candidate-array offsets per level (per image)
  int64_t total_px;
  int total_rows;
  int64_t cand_total;
};

// Constant tables for the INTER_LINEAR_EXACT pyramid resize (per level, per axis).
struct ResizeTab {
  int32_t* xofs;  // per level l>=1: w[l] entries: source index, -1 left clamp, -2 right clamp
  int32_t* xc1;   // ufixedpoint16 weight of ofs+1 (weight of ofs is 256 - c1)
  int32_t* yofs;
  int32_t* yc1;
  int64_t xoff[FVO_MAX_LEVELS], yoff[FVO_MAX_LEVELS];
};

// Kernel ids for the optional per-launch event timing (fvo_timing_enable / _read).
enum FvoKernel {
  KN_ORB_COPY, KN_ORB_RESIZE, KN_ORB_FAST, KN_ORB_NMS_COUNT, KN_ORB_ROW_SCAN, KN_ORB_COMPACT, KN_ORB_SELECT1,
  KN_ORB_HARRIS, KN_ORB_SELECT2, KN_ORB_OFFSETS, KN_ORB_ANGLE, KN_ORB_BLUR, KN_ORB_BRIEF, KN_BF_ARGMIN,
  KN_BF_FINISH, KN_SG_VERT, KN_SG_ROWS, KN_SG_MEDIAN, KN_BACKPROJECT, KN_PNP, KN_BA_STEREO,
  KN_BA_BUILD, KN_BA_SOLVE, KN_GATHER, KN_ESSENTIAL, KN_RECOVER, KN_INGEST, KN_MOTION_BLUR, KN_MAP_XFORM, KN_VOXEL, KN_COUNT
};

struct TimingRec {
  int id;
  hipEvent_t a, b;
};

struct fvo_ctx {
  int device = 0;
  uint64_t tmask = 0;                 // kernels whose launches are bracketed by events
  std::vector<TimingRec> trecs;
  std::vector<hipEvent_t> tpool;
  fvo_config cfg{};
  OrbGeom g{};
  std::string err;
  int kp_cap = 0;
  int64_t ws_bytes = 0;
  // ORB workspace (per image b < max_batch)
  uint8_t* pyr = nullptr;     // [B][total_px]
  uint8_t* blur = nullptr;    // [B][total_px] debug only (orb_blur_debug), allocated on first use
  int orb_last_batch = 0;     // images of the last ORB call
  uint8_t* score = nullptr;   // [B][total_px]
  uint32_t* cand = nullptr;   // [B][cand_total] packed (score<<24 | y<<12 | x)
  uint64_t* hel = nullptr;    // [B][cand_total] (harris float bits << 32 | packed)
  int32_t* ncand = nullptr;   // [B][L]
  int32_t* nsel1 = nullptr;   // [B][L]
  int32_t* nsel2 = nullptr;   // [B][L]
  int32_t* koff = nullptr;    // [B][L+1]
  int32_t* scratch = nullptr; // [B*L][2*maxcand] selection position lists
  int64_t scratch_per = 0;
  ResizeTab rt{};
  int32_t* umax = nullptr;    // IC angle row extents
  // BF workspace
  uint32_t* bf_rowkey = nullptr;  // [B][cap] (distance << 16 | train index) minimum per query row
  uint32_t* bf_colkey = nullptr;  // [B][cap] (distance << 16 | query index) minimum per train column
  // SGBM workspace
  uint16_t* sg_V = nullptr;     // top-down path V, [B][HG4 + nstripes][width1][4][D] (4-row groups)
  uint16_t* sg_M = nullptr;     // min over d of each V row, [B][HG4 + nstripes][width1][4]
  uint32_t* sg_ckpt = nullptr;  // [B][4-row blocks][nck][64 lanes][ckw] left->right path checkpoints
  int16_t* sg_raw = nullptr;    // [B][H][W] pre-median disparity
  uint64_t* sg_hand = nullptr;  // [B][H][2][D/32][16] L-path hand-off granules (cost pass, column block to block)
  uint32_t* sg_ctl = nullptr;   // [4 + B] ticket, generation, hand-off timeouts, per-pair failure flags
  // fvo_ba_count_births's record: the window range whose birth counts are already in the BA
  // workspace (valid until the next BA call)
  struct {
    bool valid = false;
    const void* matches = nullptr;
    const void* stereo = nullptr;
    int nframes = 0, first_end = 0, nwin = 0, first_valid = 0;
  } ba_births;
  // pose workspace
  double* pnp_hyp = nullptr;      // [B][cap][2] normalised inlier points (refinement)
  int32_t* pnp_sub = nullptr;     // [B][cap] inlier indices
  int16_t* rs_table = nullptr;    // [cap+1][rs_table_iters][5] RNG(-1) RANSAC subsets per point count
  int32_t rs_table_iters = 0;     //   (shared by PnP and the essential-matrix RANSAC)
  double* pnp_models = nullptr;   // [B][max_iters][6] hypotheses (rvec, tvec)
  double* pnp_ws = nullptr;       // [B][max_iters][PNP_WS] EPnP null space + subset state between launches
  int32_t* pnp_good = nullptr;    // [B][max_iters] inlier counts
  void* pnp_state = nullptr;      // [B] PnpState
  float* pnp_pts = nullptr;        // [B][5 * cap] the refinement's compacted inliers past its LDS
  int32_t* pnp_plan = nullptr;    // [3][B + 1] round-2 work-unit prefix sums (units of 64, 8, 16 iterations)
  int32_t pnp_max_iters = 0;
  uint8_t* fast_rec = nullptr;    // [B][tiles][kTRec] per FAST tile: row keep words + prefixes + kept scores
  // local BA workspace (per window w < max_batch; strides in ba_* counts)
  void* ba_ws = nullptr;          // one allocation, carved per window (ba.hip)
  int64_t ba_win_bytes = 0;
  hipStream_t ba_s2 = nullptr;    // second stream: half of the windows' LM sequences (ba.hip)
  hipEvent_t ba_fork = nullptr, ba_join = nullptr;
  // mono (essential matrix) workspace
  double* em_x = nullptr;         // [B][cap][4] normalised (x1, y1, x2, y2)
  double* em_models = nullptr;    // [B][max_iters][10][9] 5-point solutions
  int32_t* em_good = nullptr;     // [B][max_iters][10] inlier counts
  int8_t* em_nmod = nullptr;      // [B][max_iters] solutions per subset
  double* em_ws = nullptr;        // [B][max_iters][EM_WS] per-subset solver stages (basis, 10x20, B(z), det)
  void* em_state = nullptr;       // [B] EmState
  int32_t em_max_iters = 0;
};

// Error helpers: set ctx->err and return negative status.
int fvo_fail(fvo_ctx* ctx, const std::string& msg);
#define FVO_HIP(ctx, expr)                                                                 \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) return fvo_fail(ctx, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define FVO_LAUNCH_CHECK(ctx) FVO_HIP(ctx, hipGetLastError())

hipEvent_t fvo_event(fvo_ctx* ctx);
// Launch `...` on stream `s`; when kernel `id` is in ctx->tmask, bracket it with events.
#define FVO_TIMED(ctx, id, s, ...)                               \
  do {                                                           \
    const bool t_ = ((ctx)->tmask >> (id)) & 1ull;               \
    hipEvent_t a_ = nullptr, b_ = nullptr;                       \
    if (t_) {                                                    \
      a_ = fvo_event(ctx);                                       \
      (void)hipEventRecord(a_, s);                               \
    }                                                            \
    __VA_ARGS__;                                                 \
    if (t_) {                                                    \
      b_ = fvo_event(ctx);                                       \
      (void)hipEventRecord(b_, s);                               \
      (ctx)->trecs.push_back(TimingRec{(int)(id), a_, b_});      \
    }                                                            \
  } while (0)

// Per-module init/launchers (defined in the .hip files).
int orb_init(fvo_ctx* ctx);
int orb_run(fvo_ctx* ctx, const uint8_t* images, int batch, int64_t image_stride, int pitch, float* kp, uint8_t* desc,
            int32_t* counts, int cap, hipStream_t s);
int bf_init(fvo_ctx* ctx);
int bf_run(fvo_ctx* ctx, const uint8_t* q, const int32_t* nq, const uint8_t* t, const int32_t* nt, int batch, int cap,
           int32_t* matches, int32_t* nmatch, hipStream_t s);
int sgbm_init(fvo_ctx* ctx);
int sgbm_run(fvo_ctx* ctx, const uint8_t* L, const uint8_t* R, int batch, int64_t image_stride, int pitch,
             int16_t* disp, int32_t* status, hipStream_t s);
int pose_init(fvo_ctx* ctx);
int ransac_table_init(fvo_ctx* ctx);
int orb_blur_debug(fvo_ctx* ctx);
int orb_score_debug(fvo_ctx* ctx);
int backproject_run(fvo_ctx* ctx, const int16_t* disp, const float* kp0, const float* kp1, const int32_t* matches,
                    const int32_t* nmatch, int batch, int cap, const double* K, double baseline, float* P3, float* p2,
                    int32_t* npts, hipStream_t s);
int pnp_run(fvo_ctx* ctx, const float* P3, const float* p2, const int32_t* npts, int batch, int cap, const double* K,
            const double* dist, float reproj, double conf, int iters, double* rvec, double* tvec, double* T,
            int32_t* status, uint8_t* inliers, hipStream_t s);

int ingest_run(fvo_ctx* ctx, const uint8_t* bgr, int batch, int64_t sstride, int spitch, const double* K,
               const double* dist, uint8_t* gray, int64_t dstride, int dpitch, hipStream_t s);
int motion_blur_run(fvo_ctx* ctx, const uint8_t* img, int batch, int64_t sstride, int spitch, int ksize,
                    const int32_t* centers, const int32_t* ncent, int cap, uint8_t* mask, uint8_t* out,
                    int64_t dstride, int dpitch, hipStream_t s);
int map_transform_run(fvo_ctx* ctx, const float* pts, int stride, const int32_t* npts, int batch, int64_t cap,
                      const double* T, int32_t* count, int64_t map_cap, double* out64, float* out32, hipStream_t s);
int chain_poses_run(fvo_ctx* ctx, const double* T, const int32_t* status, const int32_t* npts, int n_seq, int n,
                    double* cum, double* cum_out, int32_t* npts_out, hipStream_t s);
struct FvoRegions {
  fvo_region r[FVO_MAX_REGIONS];
};
int copy_regions_run(fvo_ctx* ctx, int count, const fvo_region* regions, hipStream_t s);
int count_guard_run(fvo_ctx* ctx, const int32_t* cnt, const int32_t* q_cnt, int n, int sets, int32_t* status,
                    int32_t code, int32_t* nkp_out, hipStream_t s);
int64_t voxel_workspace_bytes(int64_t n);
int voxel_run(fvo_ctx* ctx, const double* pts, int64_t n, double voxel, void* ws, size_t ws_bytes, double* out,
              int32_t* n_out, int32_t* status, hipStream_t s);
int mono_init(fvo_ctx* ctx);
int gather_run(fvo_ctx* ctx, const float* kp0, const float* kp1, const int32_t* matches, const int32_t* nmatch,
               int batch, int cap, float* p0, float* p1, int32_t* npts, hipStream_t s);
int essential_run(fvo_ctx* ctx, const float* p0, const float* p1, const int32_t* npts, int batch, int cap,
                  double focal, double cx, double cy, double prob, double threshold, int maxIters, double* E,
                  uint8_t* mask, int32_t* status, hipStream_t s);
int recover_run(fvo_ctx* ctx, const double* E, const int32_t* est, const float* p0, const float* p1,
                const int32_t* npts, int batch, int cap, double focal, double cx, double cy, double dist, double* R,
                double* t, double* T, int32_t* ngood, hipStream_t s);

int ba_init(fvo_ctx* ctx);
int ba_export_run(fvo_ctx* ctx, int window, double* xyz, int32_t* count, hipStream_t s);
int ba_births_run(fvo_ctx* ctx, const int32_t* matches, const int32_t* nmatch, const float* stereo, int nframes,
                  int cap, int first_end, int nwin, int first_valid, hipStream_t s);
int ba_stereo_run(fvo_ctx* ctx, const int16_t* disp, const float* kp, const int32_t* nkp, int batch, int cap,
                  const double* K, double baseline, float* stereo, hipStream_t s);
int ba_run(fvo_ctx* ctx, const float* kp, const int32_t* nkp, const int32_t* matches, const int32_t* nmatch,
           const float* stereo, const double* Trel, int nframes, int cap, int first_end, int nwin, int first_valid,
           const double* K, double baseline, const double* inv_sigma2, int nlev, int iters, double* Tout,
           double* stats, hipStream_t s);

template <typename T>
int fvo_alloc(fvo_ctx* ctx, T** p, size_t n) {
  size_t bytes = n * sizeof(T);
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc((void**)p, bytes);
  if (e != hipSuccess) return fvo_fail(ctx, std::string("hipMalloc failed: ") + hipGetErrorString(e));
  ctx->ws_bytes += (int64_t)bytes;
  return 0;
}
