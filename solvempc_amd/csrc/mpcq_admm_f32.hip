// solvempc_amd/csrc/mpcq_admm_f32.hip — fp32 instantiations of the lane kernel (mpcq_admm.h).
#include "mpcq_admm.h"

extern "C" int mpcq_internal_admm_launch_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, hipStream_t s)
{
    return mpcq::launch_any<float>(*a, nc, mc, s);
}

extern "C" int mpcq_internal_warm_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, const double *x,
                                      const double *y, hipStream_t s)
{
    return mpcq::warm_any<float>(*a, nc, mc, x, y, s);
}

