// solvempc_amd/csrc/mpcq_wave_f64.hip — f64 instantiations of the one-QP-per-wave kernel (mpcq_wave.h).
#include "mpcq_wave.h"

extern "C" int mpcq_internal_wave_launch_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, int grid, hipStream_t s)
{
    return mpcq::wave_launch_any<double>(*a, nc, mc, grid, s);
}

extern "C" int mpcq_internal_stream_launch_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, const mpcq::StreamArgs *sa,
                                              hipStream_t s)
{
    return mpcq::stream_launch_any<double>(*a, nc, mc, *sa, s);
}
