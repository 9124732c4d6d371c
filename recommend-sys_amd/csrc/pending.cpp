// pending.cpp -- entry points declared in rsgpu.h whose kernels land in later commits.
#include "common.hpp"

extern "C" int rs_svdpp_fit(rs_ctx* ctx, const rs_ratings*, const rs_sgd_params*, double*, double*,
                            double*, double*, double*, double*) {
    return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "rs_svdpp_fit: not built yet");
}
extern "C" int rs_baseline_fit(rs_ctx* ctx, const rs_ratings*, int32_t, double, double, double*,
                               double*, double*) {
    return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "rs_baseline_fit: not built yet");
}
