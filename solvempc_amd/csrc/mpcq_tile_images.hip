// solvempc_amd/csrc/mpcq_tile_images.hip — MFMA operand images of a shared plant (TileLayout,
// mpcq_internal.h), built once per setup from the fp64 operator block of mpcq_setup.hip.
#include "mpcq_tile.h"

namespace mpcq {

// One thread per image element of both image sets (the generic one, then the paired one).  M(r, c) of
// each image, from the row-major (nc x nc / mc x nc) operator arrays (zero outside n, m):  S = sigma W'W,
// Bt = B', B = A^ W, PW = P^ W, AhT = A^', W, Wt = W'; the paired set keeps the top halves of B, B', A^'
// and (f64) BS = [B~; S] (rows 0 .. 4 KN - 1 of B, then S).
template <typename T>
__global__ void tile_images_kernel(const double *ops, int nc, int mc, int KN, int KM, T *img)
{
    const int VEC = 16 / sizeof(T);
    const TileLayout LG = TileLayout::make(KN, KM, VEC, false), LP = TileLayout::make(KN, KM, VEC, true);
    const OpsLayout O = OpsLayout::make(nc, mc);
    const int is32 = sizeof(T) == 4;
    for (size_t e0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e0 < LG.total + LP.total;
         e0 += (size_t)gridDim.x * blockDim.x) {
        const bool pset = e0 >= LG.total;
        const TileLayout &L = pset ? LP : LG;
        const size_t e = pset ? e0 - LG.total : e0;
        // which image
        const size_t offs[8] = {L.S, L.Bt, L.B, L.PW, L.AhT, L.W, L.Wt, L.BS};
        int id = 7;
        while (id > 0 && e < offs[id]) id--;
        const bool out_m = id == 2 && !pset;                // B has m output rows
        const bool in_m = (id == 1 || id == 4) && !pset;    // Bt, AhT have m inputs
        const int KSP = in_m ? L.KMP : L.KNP;
        size_t r = e - offs[id];
        const int within = (int)(r % VEC);
        r /= VEC;
        const int lane = (int)(r % 64);
        r /= 64;
        const int sg = (int)(r % (KSP / VEC));
        const int t = (int)(r / (KSP / VEC));
        const int s = sg * VEC + within;
        const int row = 16 * t + tile_arow(is32, lane & 15);
        const int col = 4 * s + (lane >> 4);
        const int rows = out_m ? mc : (id == 7 ? 8 * KN : (pset && id == 2 ? 4 * KN : nc)), cols = in_m ? mc : nc;
        double v = 0.0;
        if (row < rows && col < cols && s < (in_m ? KM : KN)) {
            switch (id) {
            case 0: v = ops[O.sWtW + (size_t)row * nc + col]; break;
            case 1: v = ops[O.WtA + (size_t)col * nc + row]; break;
            case 2: v = ops[O.WtA + (size_t)row * nc + col]; break;
            case 3: v = ops[O.PW + (size_t)row * nc + col]; break;
            case 4: v = ops[O.Ah + (size_t)col * nc + row]; break;
            case 5: v = ops[O.W + (size_t)row * nc + col]; break;
            case 6: v = ops[O.W + (size_t)col * nc + row]; break;
            default:  // BS: B~ rows, then S rows from 4 KN on
                if (row < 4 * KN) v = row < nc ? ops[O.WtA + (size_t)row * nc + col] : 0.0;
                else v = row - 4 * KN < nc ? ops[O.sWtW + (size_t)(row - 4 * KN) * nc + col] : 0.0;
                break;
            }
        }
        img[e0] = (T)v;
    }
}

}  // namespace mpcq

extern "C" int mpcq_internal_tile_supported(int KN, int KM)
{
#define MPCQ_TRY(KN_, KM_) if (KN == KN_ && KM == KM_) return 1;
    MPCQ_TILE_SHAPES(MPCQ_TRY)
#undef MPCQ_TRY
    return 0;
}

extern "C" int mpcq_internal_tile_images(const double *ops, int nc, int mc, int KN, int KM, int is_f32, void *img,
                                         hipStream_t s)
{
    if (is_f32)
        hipLaunchKernelGGL(mpcq::tile_images_kernel<float>, dim3(64), dim3(256), 0, s, ops, nc, mc, KN, KM, (float *)img);
    else
        hipLaunchKernelGGL(mpcq::tile_images_kernel<double>, dim3(64), dim3(256), 0, s, ops, nc, mc, KN, KM, (double *)img);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
