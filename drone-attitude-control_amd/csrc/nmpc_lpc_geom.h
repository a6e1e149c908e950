// nmpc_lpc_geom.h — LDS / scratch geometry of the lane-per-component IPM kernel
// (nmpc_ipm_lpc.hip), shared with the dispatch table (nmpc_ipm.hip) and the allocator.
#pragma once

#include <stddef.h>

#include "nmpc_internal.h"

namespace nmpc {
namespace lpc {

template <typename T, int NX, int NU, int WPB>
struct Geom {
    static constexpr int NZ = NX + NU;
    static constexpr int IPW = 64 / NZ;             // instances per wavefront
    static constexpr int VS = (64 + NZ - 1) / NZ;   // lane groups incl. a partial (idle) one
    static constexpr int VW = 16 / (int)sizeof(T);
    static constexpr int rup(int n) { return (n + VW - 1) / VW * VW; }
    static constexpr int cmax(int a, int b) { return a > b ? a : b; }
    static constexpr int LDZ = rup(NZ), LDX = rup(NX), LDU = rup(NU);
    // workgroup constants: rows of [A B], columns of [A B], H, He, bounds [3][nz] (k = 0 / 0<k<N / N)
    static constexpr int C_ABR = 0, C_ABT = C_ABR + NX * LDZ, C_H = C_ABT + NZ * LDX, C_HE = C_H + NZ * LDZ,
                         C_LB = C_HE + NX * LDX, C_UB = C_LB + 3 * LDZ, C_TOT = C_UB + 3 * LDZ;
    // per lane group: stage z / dx broadcast, re, v, h_u, F_uu, M^T (aliased by the rows of
    // Y = L^{-1} F_ux in the factorisation and by the partial products K(u, j) dx_j in the forward sweeps)
    static constexpr int G_ZB = 0, G_RB = G_ZB + LDZ, G_VB = G_RB + LDX, G_HU = G_VB + LDX, G_FU = G_HU + LDU,
                         G_MT = G_FU + rup(NU * NU), MTW = cmax(NZ * LDX, NX * LDU), G_TOT = G_MT + MTW;
    static constexpr int LDS_ELEMS = C_TOT + WPB * VS * G_TOT;
    // per-instance scratch records: x-lane j: K(:, j), Pr_j, re_j; u-lane u: kff_u, F_uu^{-1}(u, :)
    static constexpr int XW = NU + 2, XPR = NU, XRE = NU + 1;
    static constexpr int UW = 1 + NU, UKFF = 0, UFI = 1;
    static_assert(IPW >= 1, "stage wider than a wavefront");
};

// per-instance scratch, stage-major: stage k owns one block of BLK elements holding, for every
// lane r of the instance, the element arrays (z, lambda_l, lambda_u, dz_aff, dz, G yref, g) and
// the x-lane / u-lane stage records; an access is (lane offset) + k BLK (one SGPR) + a
// compile-time immediate
template <int NX, int NU>
struct Layout {
    static constexpr int NZ = NX + NU;
    static constexpr int Z = 0, LL = NZ, LU = 2 * NZ, DZA = 3 * NZ, DZ = 4 * NZ, GC = 5 * NZ, GF = 6 * NZ;
    static constexpr int XREC = 7 * NZ;                       // [XW][NX]
    static constexpr int UREC = XREC + (NU + 2) * NX;         // [UW][NU]
    static constexpr int BLK = UREC + (1 + NU) * NU;
    __host__ __device__ static size_t slot(int N) { return ((size_t)(N + 1) * BLK + 31) & ~size_t(31); }
};

template <typename T, int NX, int NU, int WPB>
inline size_t scratch_elems(int B, int N)
{
    using Gm = Geom<T, NX, NU, WPB>;
    const size_t waves = (size_t)(B + Gm::IPW - 1) / Gm::IPW;
    const size_t blocks = (waves + WPB - 1) / WPB;
    return blocks * WPB * Gm::VS * Layout<NX, NU>::slot(N);
}

}  // namespace lpc

template <typename T, int NX, int NU, int WPB, int MW>
hipError_t launch_ipm_lpc(const IpmParams<T> &p, hipStream_t s);

}  // namespace nmpc
