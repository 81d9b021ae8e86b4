// solvempc_amd/csrc/mpcq_tile_f32.hip — fp32 instantiations of the tile (MFMA) ADMM kernel.
#include "mpcq_tile.h"

extern "C" int mpcq_internal_tile_launch_f32(const mpcq::AdmmArgs<float> *a, int KN, int KM, hipStream_t s)
{
    return mpcq::tile_launch_any<float>(*a, KN, KM, s);
}

extern "C" int mpcq_internal_tile_stream_launch_f32(const mpcq::AdmmArgs<float> *a, int KN, int KM, hipStream_t s)
{
    return mpcq::tile_stream_launch_any<float>(*a, KN, KM, s);
}

extern "C" int mpcq_internal_tile_publish_f32(const mpcq::AdmmArgs<float> *a, int KN, int KM, int paired, hipStream_t s)
{
    return mpcq::tile_publish_any<float>(*a, KN, KM, paired != 0, s);
}
