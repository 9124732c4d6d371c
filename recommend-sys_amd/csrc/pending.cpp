// pending.cpp -- entry points declared in rsgpu.h whose kernels land in later commits.
#include "common.hpp"

extern "C" int rs_baseline_fit(rs_ctx* ctx, const rs_ratings*, int32_t, double, double, double*,
                               double*, double*) {
    return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "rs_baseline_fit: not built yet");
}
