/* fvo.h — C ABI of the MI355X stereo-VO hot path (forest-slam_amd, libfvo.so).
 *
 * Drop-in boundary for the OpenCV calls of si220/Forest-SLAM's ORB branch
 * (ros_ws/src/stereo_slam.py).  Every entry point replaces one reference call:
 *
 *   fvo_orb_detect_compute  <- cv2.ORB_create() + orb.detectAndCompute(img, None)
 *                              stereo_slam.py:84, :232-233, :240-241
 *   fvo_bf_match            <- cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True).match(d0, d1)
 *                              stereo_slam.py:85, :234, :242 (+ the :235-238 gather)
 *   fvo_sgbm                <- cv2.StereoSGBM_create(numDisparities=96, minDisparity=0,
 *                              blockSize=7, P1=392, P2=1568, mode=SGBM_3WAY).compute(L, R)
 *                              stereo_slam.py:108-117 (get_disparity_map)
 *   fvo_backproject         <- depth = fx*B/disp, Z = depth[int(y), int(x)], X/Y, 0.1<Z<1000
 *                              stereo_slam.py:117-121 (0/-1 -> 0.1) and :262-289
 *   fvo_pnp_ransac          <- cv2.solvePnPRansac(P, p, K0, dist_l, reprojectionError=1.0,
 *                              confidence=0.99, iterationsCount=1000, SOLVEPNP_ITERATIVE)
 *                              + cv2.Rodrigues + T assembly, stereo_slam.py:292-303
 *   fvo_ba_windows          <- (new) windowed local bundle adjustment, no reference counterpart
 *                              (+ fvo_keypoint_stereo, fvo_ba_landmarks)
 *   fvo_gather_matches      <- mkpts0 = kpts0[valid], mkpts1 = kpts1[matches[valid]]
 *                              mono_slam.py:106-108 (stereo_slam.py:235-238 for the BF DMatch list)
 *   fvo_find_essential      <- cv2.findEssentialMat(mkpts0, mkpts1, focal=K0[0,0], pp=(K0[0,2], K0[1,2]),
 *                              method=cv2.RANSAC, prob=0.999, threshold=1.0)   mono_slam.py:111
 *   fvo_recover_pose        <- cv2.recoverPose(E, mkpts0, mkpts1, focal=, pp=) + the [R|t] matrix
 *                              mono_slam.py:112-117
 *   fvo_undistort_gray      <- cv2.cvtColor(cv2.undistort(img, K, dist), cv2.COLOR_BGR2GRAY)
 *                              stereo_slam.py:184-186, :196-198; mono_slam.py:92-93
 *   fvo_motion_blur         <- apply_random_motion_blur(img, blur_percentage, kernel_size, angle=0)
 *                              (cv2.getRotationMatrix2D + warpAffine + filter2D + np.where)
 *                              forest_slam_ros/src/stereo_slam.py:142-178, :194, :206
 *   fvo_chain_poses         <- cumulative_est_tf_mat = np.dot(cumulative_est_tf_mat, T) per posed frame
 *                              (the len(points3D) >= 6 guard), stereo_slam.py:292, :306 — on the device
 *   fvo_map_transform       <- (cum @ hstack(points3D, 1).T)[:3].T appended to the map + PointCloud2
 *                              float32 packing: stereo_slam.py:308-318; mono_slam.py:148; gt_mapping.py
 *   fvo_voxel_down_sample   <- open3d PointCloud.voxel_down_sample(voxel_size=0.5)
 *                              mono_slam.py:151-155, gt_mapping.py:62-66
 *
 * Conventions
 *  - All array pointers are DEVICE pointers owned by the caller (e.g. torch tensors'
 *    data_ptr()).  Calls are asynchronous on `stream` (a hipStream_t, may be NULL for
 *    the default stream); counts and statuses are written to device memory.
 *  - Every call works on a BATCH of independent items (images / image pairs / frames);
 *    `batch` <= fvo_config.max_batch.
 *  - Return value: 0 on success, <0 on argument/launch error (see fvo_last_error()).
 *    No exceptions cross this boundary.  Data-dependent failures (too few points,
 *    capacity overflow) are reported per item in the status/count outputs.
 *  - A context is not re-entrant: one context per (device, host thread).  All device
 *    workspace is allocated by fvo_create(); hot calls do not allocate and can be
 *    captured into a hipGraph.
 */
#ifndef FVO_H_
#define FVO_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FVO_ABI_VERSION 7

typedef struct fvo_ctx fvo_ctx;
typedef void* fvo_stream; /* hipStream_t */

/* Keypoint record written by fvo_orb_detect_compute (8 x float32 per keypoint):
 * x, y (level-0 pixels), size, angle (deg), response (Harris), octave, class_id (-1), 0 */
#define FVO_KP_STRIDE 8
#define FVO_DESC_BYTES 32

typedef struct fvo_config {
  int32_t width, height; /* image size shared by every call on this context         */
  int32_t max_batch;     /* max images (ORB) / pairs (BF, SGBM) / frames (pose) per call */
  /* cv2.ORB_create() parameters; defaults = OpenCV defaults (stereo_slam.py:84) */
  int32_t nfeatures;       /* 500 */
  float scale_factor;      /* 1.2f */
  int32_t nlevels;         /* 8 */
  int32_t edge_threshold;  /* 31 */
  int32_t first_level;     /* 0 (only 0 supported) */
  int32_t wta_k;           /* 2 (only 2 supported) */
  int32_t score_type;      /* 0 = HARRIS_SCORE (only Harris supported) */
  int32_t patch_size;      /* 31 (only 31 supported: the rBRIEF table) */
  int32_t fast_threshold;  /* 20 */
  /* cv2.StereoSGBM_create() parameters used at stereo_slam.py:109-115 */
  int32_t min_disparity;    /* 0 */
  int32_t num_disparities;  /* 96, multiple of 16 */
  int32_t block_size;       /* 7 */
  int32_t P1, P2;           /* 392, 1568 */
  int32_t disp12_max_diff;  /* 0 (-> 1 as in OpenCV) */
  int32_t pre_filter_cap;   /* 0 (-> 15) */
  int32_t uniqueness_ratio; /* 0 (only 0 supported) */
  int32_t sgbm_stripes;     /* 4: OpenCV's fixed stripe count for MODE_SGBM_3WAY */
  int32_t kp_capacity;      /* per-image keypoint capacity of the ORB outputs (0 = auto) */
  int32_t stages;           /* FVO_STAGE_* mask of the workspaces to allocate (0 = all) */
  /* local bundle adjustment (no reference counterpart: BASELINE.json north_star) */
  int32_t ba_window;        /* frames per BA window K (10); max 21 */
  int32_t ba_max_landmarks; /* per-window landmark cap (4096) */
  int32_t ba_max_obs;       /* per-window observation cap (32768) */
  int32_t sgbm_max_batch;   /* max pairs per fvo_sgbm call (0 = max_batch): the SGBM path
                               volume (one u16 volume, ~100 MB per pair at 600p) is sized by it */
  /* SGBM schedule (every schedule and launch shape is bit-identical).  Chosen
   * here, at fvo_create, and nowhere else: the library reads no environment variables. */
  int32_t sgbm_mode;        /* FVO_SGBM_CLASSIC (0, default) or FVO_SGBM_LPATH */
  int32_t sgbm_lanes;       /* classic cost pass: lanes per column, 4 / 8 / 16 (0 = 8) */
  int32_t sgbm_cols;        /* classic cost pass: columns per block (0 = default; lanes 4: 32 or 64
                               (default 64), lanes 8: 16 or 32 (default 32), lanes 16: 32) */
  int32_t sgbm_handoff_us;  /* lpath: bound on one column-block hand-off wait in microseconds
                               (0 = 250000); -1 = test hook: every hand-off times out */
} fvo_config;

/* fvo_config.sgbm_mode */
#define FVO_SGBM_CLASSIC 0 /* cost pass + row pass running both horizontal sweeps */
#define FVO_SGBM_LPATH 1   /* left->right path inside the cost pass, handed between column blocks */
/* fvo_sgbm status values */
#define FVO_SGBM_OK 0
#define FVO_SGBM_HANDOFF_TIMEOUT (-1) /* lpath: a hand-off wait of the pair timed out; its disparity
                                         map is all invalid ((min_disparity-1)*16) */

/* fvo_config.stages: a context only serves the stages it was created for (e.g. a
 * BFMatcher-only context needs no image-sized workspace). */
#define FVO_STAGE_ORB 1
#define FVO_STAGE_BF 2
#define FVO_STAGE_SGBM 4
#define FVO_STAGE_POSE 8
#define FVO_STAGE_BA 16
#define FVO_STAGE_MONO 32
#define FVO_STAGE_ALL 63

/* Fill `cfg` with the reference's parameters for a width x height image. */
void fvo_config_default(fvo_config* cfg, int32_t width, int32_t height);

/* Layout of fvo_config as this library was compiled: sizeof, and offsetof(field) in bytes
 * (-1 for an unknown name).  A binding that declares the struct itself (ctypes, cffi, cgo)
 * checks its declaration against these before calling fvo_config_default / fvo_create. */
int32_t fvo_config_size(void);
int32_t fvo_config_offset(const char* field);

int fvo_create(int device, const fvo_config* cfg, fvo_ctx** out);
void fvo_destroy(fvo_ctx* ctx);
const char* fvo_last_error(const fvo_ctx* ctx);
int fvo_abi_version(void);
/* Per-image keypoint capacity (rows of the keypoint/descriptor outputs). */
int fvo_kp_capacity(const fvo_ctx* ctx);
/* Device workspace bytes held by the context. */
int64_t fvo_workspace_bytes(const fvo_ctx* ctx);

/* ORB detectAndCompute on `batch` grayscale u8 images.
 * images:      batch images, image b at images + b*image_stride, rows `pitch` bytes apart.
 * keypoints:   [batch][cap][FVO_KP_STRIDE] f32     descriptors: [batch][cap][32] u8
 * counts:      [batch] i32 = number of keypoints, or -(needed) if it exceeds `cap`
 *              (outputs then unspecified).  Keypoint order = OpenCV's output order. */
int fvo_orb_detect_compute(fvo_ctx* ctx, const uint8_t* images, int32_t batch, int64_t image_stride,
                           int32_t pitch, float* keypoints, uint8_t* descriptors, int32_t* counts,
                           int32_t cap, fvo_stream stream);

/* Cross-checked brute-force Hamming matching of `batch` (query, train) descriptor sets.
 * query/train: [batch][cap][32] u8 with per-item counts n_query/n_train [batch] (<=0: empty).
 * matches:     [batch][cap][3] i32 rows (queryIdx, trainIdx, distance), ascending queryIdx.
 * n_matches:   [batch] i32. */
int fvo_bf_match(fvo_ctx* ctx, const uint8_t* query, const int32_t* n_query, const uint8_t* train,
                 const int32_t* n_train, int32_t batch, int32_t cap, int32_t* matches, int32_t* n_matches,
                 fvo_stream stream);

/* StereoSGBM 3-way disparity (incl. the final 3x3 median) of `batch` rectified pairs.
 * disparity: [batch][height][width] i16, disparity*16, invalid = (min_disparity-1)*16.
 * status:    [batch] i32 (device, may be NULL): FVO_SGBM_OK, or FVO_SGBM_HANDOFF_TIMEOUT (only
 *            under FVO_SGBM_LPATH) when the pair's disparities were dropped. */
int fvo_sgbm(fvo_ctx* ctx, const uint8_t* left, const uint8_t* right, int32_t batch, int64_t image_stride,
             int32_t pitch, int16_t* disparity, int32_t* status, fvo_stream stream);

/* Matched-keypoint back-projection through the disparity map (stereo_slam.py:262-289).
 * kp0/kp1:   keypoint records of the previous / current left images ([batch][cap][8]).
 * matches:   fvo_bf_match output (query = previous, train = current).
 * K:         host double[9] row-major camera matrix; baseline in metres.
 * points3d:  [batch][cap][3] f32 valid points (0.1 < Z < 1000), compacted in match order.  f32
 *            because the reference's NumPy 1.x (Python 3.8) evaluates float64-scalar x
 *            float32-array expressions in float32 (value-based casting), DESIGN.md §Parity.
 * points2d:  [batch][cap][2] f32 matching current-image keypoints.  n_points: [batch]. */
int fvo_backproject(fvo_ctx* ctx, const int16_t* disparity, const float* kp0, const float* kp1,
                    const int32_t* matches, const int32_t* n_matches, int32_t batch, int32_t cap, const double* K,
                    double baseline, float* points3d, float* points2d, int32_t* n_points, fvo_stream stream);

/* solvePnPRansac(SOLVEPNP_ITERATIVE) + Rodrigues on `batch` independent frames.
 * K, dist:   host double[9] / double[5] (k1 k2 p1 p2 k3).
 * rvec/tvec: [batch][3] f64.   T: [batch][16] f64 row-major [R|t;0 0 0 1].
 * status:    [batch] i32: 1 pose valid, 0 RANSAC failed, -1 skipped (n_points < 6,
 *            the reference's `len(points3D) >= 6` guard, stereo_slam.py:292).
 * inliers:   [batch][cap] u8 RANSAC inlier mask (may be NULL). */
int fvo_pnp_ransac(fvo_ctx* ctx, const float* points3d, const float* points2d, const int32_t* n_points,
                   int32_t batch, int32_t cap, const double* K, const double* dist, float reprojection_error,
                   double confidence, int32_t iterations, double* rvec, double* tvec, double* T, int32_t* status,
                   uint8_t* inliers, fvo_stream stream);

/* Stereo point of every keypoint of `batch` left images: the back-projection of
 * fvo_backproject (same float32 arithmetic, stereo_slam.py:265-289) applied to all
 * keypoints instead of the matched ones.  stereo: [batch][cap][4] f32 (X, Y, Z, d) in
 * camera coordinates with d the disparity used; Z = 0 when 0.1 < Z < 1000 fails.
 * Feeds fvo_ba_windows (stage FVO_STAGE_BA). */
int fvo_keypoint_stereo(fvo_ctx* ctx, const int16_t* disparity, const float* keypoints, const int32_t* n_keypoints,
                        int32_t batch, int32_t cap, const double* K, double baseline, float* stereo,
                        fvo_stream stream);

/* Windowed local bundle adjustment (specification: oracle/ba_ref.py).
 * Frame arrays cover `n_frames` consecutive frames f of one sequence:
 *   keypoints [F][cap][8], n_keypoints [F]      left-image ORB records
 *   matches [F][cap][3], n_matches [F]          BF matches frame f -> f+1 (f < F-1)
 *   stereo [F][cap][4]                          fvo_keypoint_stereo of frame f (f < F-1)
 *   T_rel [F][16]                               camera f -> camera f+1 (PnP), f < F-1
 * Window w (0 <= w < n_windows) ends at frame e = first_end + w and spans frames
 * max(first_valid, e - ba_window + 1) .. e; windows of fewer than 3 frames copy T_rel.
 * inv_sigma2: host double[nlevels] = 1 / scale_factor^(2*octave) observation weights.
 * Outputs: T_out [n_windows][16] refined camera (e-1) -> camera e transform;
 *          stats [n_windows][6] f64: cost0, cost, landmarks, observations, frames, accepted. */
int fvo_ba_windows(fvo_ctx* ctx, const float* keypoints, const int32_t* n_keypoints, const int32_t* matches,
                   const int32_t* n_matches, const float* stereo, const double* T_rel, int32_t n_frames,
                   int32_t cap, int32_t first_end, int32_t n_windows, int32_t first_valid, const double* K,
                   double baseline, const double* inv_sigma2, int32_t n_levels, int32_t iterations,
                   double* T_out, double* stats, fvo_stream stream);

/* The first step of fvo_ba_windows -- counting each window's landmark births and observations
 * per birth frame -- issued ahead of it, e.g. on a side stream while PnP runs (it reads only the
 * match rows and the keypoints' stereo points, not T_rel or the keypoints).  Arguments as for
 * fvo_ba_windows.  The next fvo_ba_windows call on this context with the same matches, stereo,
 * n_frames, first_end, n_windows and first_valid skips that step; the caller orders the two calls
 * (the stream of fvo_ba_windows waits for this one's).  Any other BA call in between (or a
 * different window range) makes fvo_ba_windows count again itself.  A window range whose match
 * maps exceed the LDS budget (the serial construction) is counted by fvo_ba_windows regardless. */
int fvo_ba_count_births(fvo_ctx* ctx, const int32_t* matches, const int32_t* n_matches, const float* stereo,
                        int32_t n_frames, int32_t cap, int32_t first_end, int32_t n_windows, int32_t first_valid,
                        fvo_stream stream);

/* Refined landmarks of BA window `window` of the most recent fvo_ba_windows call (the
 * keyframe map a rank shares with the others): xyz [ba_max_landmarks][3] f64
 * in the window's first-camera frame, count [1] i32.  Device-side, no host sync. */
int fvo_ba_landmarks(fvo_ctx* ctx, int32_t window, double* xyz, int32_t* count, fvo_stream stream);

/* Matched keypoint coordinates of `batch` frame pairs (mono_slam.py:106-108):
 * p0[i] = kp0[matches[i].queryIdx].xy, p1[i] = kp1[matches[i].trainIdx].xy, f32 [batch][cap][2];
 * n_points [batch] = n_matches clamped to [0, cap]. */
int fvo_gather_matches(fvo_ctx* ctx, const float* kp0, const float* kp1, const int32_t* matches,
                       const int32_t* n_matches, int32_t batch, int32_t cap, float* p0, float* p1, int32_t* n_points,
                       fvo_stream stream);

/* cv2.findEssentialMat(p0, p1, focal, pp, cv2.RANSAC, prob, threshold, max_iters) on `batch`
 * frame pairs (stage FVO_STAGE_MONO; mono_slam.py:111).  5-point solver inside OpenCV's
 * RANSAC (RNG(-1) subsets, adaptive iterations, max_iters <= 1000).
 * E:      [batch][9] f64 row-major unit-norm essential matrix (zeros when status != 1).
 * mask:   [batch][cap] u8 inlier mask of E (may be NULL).
 * status: [batch] i32: 1 ok, 0 RANSAC found no model, -1 fewer than 5 points, -2 exactly 5
 *         points with several solutions (OpenCV returns a stacked 3k x 3 E that recoverPose rejects). */
int fvo_find_essential(fvo_ctx* ctx, const float* p0, const float* p1, const int32_t* n_points, int32_t batch,
                       int32_t cap, double focal, double cx, double cy, double prob, double threshold,
                       int32_t max_iters, double* E, uint8_t* mask, int32_t* status, fvo_stream stream);

/* cv2.recoverPose(E, p0, p1, focal=, pp=) (distanceThresh 50 for that overload) on `batch`
 * frame pairs, all points (the reference passes no mask, mono_slam.py:112), + T = [R|t].
 * e_status: fvo_find_essential status (may be NULL); frames with status != 1 get R = I, t = 0,
 *           T = I and n_good = -1 (the reference's cv2 call would raise there).
 * R [batch][9], t [batch][3], T [batch][16] f64; n_good [batch] i32 = cheirality inliers. */
int fvo_recover_pose(fvo_ctx* ctx, const double* E, const int32_t* e_status, const float* p0, const float* p1,
                     const int32_t* n_points, int32_t batch, int32_t cap, double focal, double cx, double cy,
                     double distance_thresh, double* R, double* t, double* T, int32_t* n_good, fvo_stream stream);

/* Image ingest of `batch` BGR8 camera images of one camera (any stage; no workspace):
 * cv2.undistort(img, K, dist) (new camera matrix = K, INTER_LINEAR remap, BORDER_CONSTANT 0)
 * followed by cv2.cvtColor(., COLOR_BGR2GRAY).  Image size = the context's width x height.
 * bgr:  [batch] images, image b at bgr + b*src_stride, rows src_pitch (>= 3*width) bytes apart.
 * K:    host double[9] row-major; dist: host double[5] (k1 k2 p1 p2 k3).
 * gray: [batch] u8 images at gray + b*dst_stride, rows dst_pitch bytes apart. */
int fvo_undistort_gray(fvo_ctx* ctx, const uint8_t* bgr, int32_t batch, int64_t src_stride, int32_t src_pitch,
                       const double* K, const double* dist, uint8_t* gray, int64_t dst_stride, int32_t dst_pitch,
                       fvo_stream stream);

/* Motion-blur ablation on `batch` gray images (any stage; no workspace), image size = the
 * context's width x height:  out = np.where(mask, cv2.filter2D(img, -1, diag(ones(k))/k), img)
 * where mask = union of the (2*(k//2)+1)^2 squares (clipped) centred on the sampled pixels.
 * ksize in [1, 31], smaller than the image; angle must be 0 (the only value the reference uses;
 * other angles return an error).  filter2D arithmetic: direct float path for k*k < 130, exact
 * S/k (the DFT path's value) otherwise — see csrc/ingest.hip.
 * centers: [batch][centers_cap] int32 flat pixel indices y*W+x (random.sample(range(H*W), n)),
 *          n_centers [batch] device counts (<= centers_cap); centers_cap 0 = no blur (mask empty).
 * mask:    [batch][H][W] u8 device buffer (4-byte aligned), written (0/1).
 * img/out: [batch] u8 images (b*stride, rows pitch bytes apart); out must not alias img. */
int fvo_motion_blur(fvo_ctx* ctx, const uint8_t* img, int32_t batch, int64_t src_stride, int32_t src_pitch,
                    int32_t ksize, double angle, const int32_t* centers, const int32_t* n_centers, int32_t centers_cap,
                    uint8_t* mask, uint8_t* out, int64_t dst_stride, int32_t dst_pitch, fvo_stream stream);

/* Map accumulation (any stage; no workspace).  For each of `batch` point sets b (float32 xyz,
 * point p of set b at points + (b*cap + p)*point_stride, n_points[b] device counts <= cap) and
 * its 4x4 row-major fp64 transform T[b] (device, [batch][16]):
 *   x' = ((T[0] x + T[1] y) + T[2] z) + T[3]   (likewise rows 1, 2; fp64, no contraction)
 * appended to the map in set order starting at *map_count (device), which is then advanced by
 * the total.  map_xyz64 (fp64, [map_cap][3]) and/or map_xyz32 (the PointCloud2 FLOAT32 x/y/z
 * record, [map_cap][3]) may be NULL (not both); points past map_cap are dropped while
 * *map_count still counts them (caller checks for overflow). */
int fvo_map_transform(fvo_ctx* ctx, const float* points, int32_t point_stride, const int32_t* n_points, int32_t batch,
                      int64_t cap, const double* T, int32_t* map_count, int64_t map_cap, double* map_xyz64,
                      float* map_xyz32, fvo_stream stream);

/* Pose chains of n_seq sequences advanced over one batch of n frames each (any stage; no
 * workspace) — stereo_slam.py:292-306 on the device, for the map of every posed frame:
 * for s < n_seq, i < n in order, a frame is posed when status[s*n + i] >= 0 (pose valid, or
 * RANSAC failure with its identity T; -1 = the len(points3D) >= 6 skip, other negatives =
 * padding / overflow: not posed).  A posed frame advances cum[s] = cum[s] @ T[s*n + i] (fp64,
 * C_ij = ((c_i0 t_0j + c_i1 t_1j) + c_i2 t_2j) + c_i3 t_3j, no contraction — NumPy's BLAS order
 * is unpinned, <= 1 ulp).  Outputs: cum_out[s*n + i] = cum[s] after frame i, n_points_out[s*n + i]
 * = n_points[s*n + i] for posed frames, 0 otherwise (so fvo_map_transform(points, n_points_out,
 * cum_out) appends exactly the posed frames' points3D, stereo_slam.py:308-314).
 * cum_state: [n_seq][16] fp64 row-major, read and advanced in place (identity at a sequence's
 * start).  T, cum_out: [n_seq*n][16] fp64; status, n_points, n_points_out: [n_seq*n] int32.
 * n_points may be NULL (n_points_out then NULL too). */
int fvo_chain_poses(fvo_ctx* ctx, const double* T, const int32_t* status, const int32_t* n_points, int32_t n_seq,
                    int32_t n, double* cum_state, double* cum_out, int32_t* n_points_out, fvo_stream stream);

/* Step bookkeeping in one launch each (no reference call: the reference keeps these per frame
 * as Python lists; a batched front end would otherwise issue a dozen small copies and
 * elementwise ops per step, each a separate dispatch).  Any stage; no workspace.
 * fvo_copy_regions: `count` (0..FVO_MAX_REGIONS) device-to-device copies of regions[i].bytes
 * from regions[i].src to regions[i].dst, in one launch.  No region's destination may overlap
 * another region's source or destination, or its own source (refused: copy through a
 * temporary).  The region array is host memory, read before the call returns.
 * fvo_count_guard: for i < n, status[i] = code when any of counts[s*n + i] or
 * q_counts[s*n + i] (s < sets; q_counts may be NULL) is negative -- ORB's -(needed) overflow
 * report; counts_clamped[i] = max(counts[i], 0) (status and counts_clamped may be NULL). */
#define FVO_MAX_REGIONS 32
typedef struct {
  void* dst;
  const void* src;
  int64_t bytes;
} fvo_region;
int fvo_copy_regions(fvo_ctx* ctx, int32_t count, const fvo_region* regions, fvo_stream stream);
int fvo_count_guard(fvo_ctx* ctx, const int32_t* counts, const int32_t* q_counts, int32_t n, int32_t sets,
                    int32_t* status, int32_t code, int32_t* counts_clamped, fvo_stream stream);

/* Open3D PointCloud::VoxelDownSample(voxel_size) of n_points fp64 xyz points (device [n][3]):
 * vmin = min_bound - voxel/2, voxel index floor((p - vmin)/voxel), per voxel the fp64 sum of
 * its points in input order divided by the count.  Output: out [<= n][3] fp64 ordered by
 * voxel index (x, then y, then z — Open3D's hash-map order is unspecified), *n_out (device).
 * workspace: device scratch of fvo_voxel_workspace_bytes(n_points) bytes (caller-owned).
 * status (device, may be NULL): 0 ok, 1 = a voxel index outside [0, 2^21) (result invalid). */
int64_t fvo_voxel_workspace_bytes(int64_t n_points);
int fvo_voxel_down_sample(fvo_ctx* ctx, const double* points, int64_t n_points, double voxel_size, void* workspace,
                          int64_t workspace_bytes, double* out, int32_t* n_out, int32_t* status, fvo_stream stream);

/* Test hook: KeyPointsFilter::retainBest on `n` float responses (device memory) with the
 * product's selection kernel.  idx_out [n] receives the surviving original indices in
 * OpenCV's output order, *n_out the survivor count.  Allocates (stream-ordered). */
int fvo_test_retain_best(fvo_ctx* ctx, const float* keys, int32_t n, int32_t keep, int32_t* idx_out, int32_t* n_out,
                         fvo_stream stream);

/* Per-kernel timing with HIP events recorded on the launch stream (measurement hooks for
 * bench.py).  mask: bit i brackets every launch of kernel i (0..fvo_kernel_count()-1,
 * names from fvo_kernel_name()).  fvo_timing_read synchronises on the recorded events,
 * writes the summed milliseconds and launch counts per kernel (arrays of
 * fvo_kernel_count() entries) and clears the record. */
int fvo_kernel_count(void);
const char* fvo_kernel_name(int id);
int fvo_timing_enable(fvo_ctx* ctx, uint64_t mask);
int fvo_timing_read(fvo_ctx* ctx, double* ms, int32_t* launches);

/* Debug hook: device pointer and byte size of an internal buffer of the most recent ORB
 * call (0 pyramid, 1 blurred pyramid, 2 FAST score map, 3/4/5 per-level counts before /
 * after the two retainBest passes, 6/7 PnP RANSAC per-iteration inlier counts / hypotheses of the
 * last fvo_pnp_ransac, 8 its per-frame RANSAC state: int32 best count, iteration bound, best
 * iteration, points, 9 the SGBM control words: u32 ticket, generation, L-path hand-off timeouts
 * (must stay 0), reserved, then one failure flag per pair).  For stage-by-stage parity tests only. */
int fvo_debug_buffer(fvo_ctx* ctx, int which, void** ptr, int64_t* bytes);

#ifdef __cplusplus
}
#endif

#endif /* FVO_H_ */
