// solvempc_amd/csrc/mpcq_admm_f64.hip — fp64 instantiations of the lane kernel (mpcq_admm.h).
#include "mpcq_admm.h"

extern "C" int mpcq_internal_caps(int n, int m, int *nc, int *mc)
{
    int best = -1, bnc = 0, bmc = 0;
#define MPCQ_PICK(NC_, MC_)                                              \
    if (n <= NC_ && m <= MC_ && (best < 0 || NC_ * (NC_ + MC_) < best)) { \
        best = NC_ * (NC_ + MC_);                                         \
        bnc = NC_;                                                        \
        bmc = MC_;                                                        \
    }
    MPCQ_CAPS(MPCQ_PICK)
#undef MPCQ_PICK
    if (best < 0) return -1;
    *nc = bnc;
    *mc = bmc;
    return 0;
}

extern "C" int mpcq_internal_admm_launch_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, hipStream_t s)
{
    return mpcq::launch_any<double>(*a, nc, mc, s);
}

extern "C" int mpcq_internal_warm_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, const double *x,
                                      const double *y, hipStream_t s)
{
    return mpcq::warm_any<double>(*a, nc, mc, x, y, s);
}

