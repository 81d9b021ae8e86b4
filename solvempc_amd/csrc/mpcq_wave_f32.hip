// solvempc_amd/csrc/mpcq_wave_f32.hip — f32 instantiations of the one-QP-per-wave kernel (mpcq_wave.h).
#include "mpcq_wave.h"

extern "C" int mpcq_internal_wave_launch_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, int grid, hipStream_t s)
{
    return mpcq::wave_launch_any<float>(*a, nc, mc, grid, s);
}

extern "C" int mpcq_internal_stream_launch_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, const mpcq::StreamArgs *sa,
                                              hipStream_t s)
{
    return mpcq::stream_launch_any<float>(*a, nc, mc, *sa, s);
}
