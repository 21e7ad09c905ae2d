// placeholder replaced below
#include "fvo_internal.h"
int pose_init(fvo_ctx* ctx) { ctx->pnp_max_iters = 1000; return 0; }
int backproject_run(fvo_ctx* ctx, const int16_t*, const float*, const float*, const int32_t*, const int32_t*, int, int,
                    const double*, double, double*, float*, int32_t*, hipStream_t) { return fvo_fail(ctx, "todo"); }
int pnp_run(fvo_ctx* ctx, const double*, const float*, const int32_t*, int, int, const double*, const double*, float,
            double, int, double*, double*, double*, int32_t*, uint8_t*, hipStream_t) { return fvo_fail(ctx, "todo"); }
