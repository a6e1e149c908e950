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
    // Y = L^{-1} F_ux in the factorisation, by the partial products K(u, j) dx_j in the forward sweeps
    // and by the double-buffered stage exchanges of the certificate and the initial point); G_CL: fused
    // closed loop with the model plant — state, output z_0, yref row 0 (LDZ each) and 4 sums
    static constexpr int G_ZB = 0, G_RB = G_ZB + LDZ, G_VB = G_RB + LDX, G_HU = G_VB + LDX, G_FU = G_HU + LDU,
                         G_MT = G_FU + rup(NU * NU), MTW = cmax(cmax(NZ * LDX, NX * LDU), 4 * LDZ),
                         G_CL = G_MT + MTW, G_RAW = G_CL + 3 * LDZ + rup(4);
    // lane groups start 16 banks apart (mod 64 dword banks): with a 32-bank stride the first and
    // third instance of a wavefront collided on every per-instance LDS access (PMC: bank
    // conflicts were ~3/4 of LDS-active cycles)
    static constexpr int DW = (int)sizeof(T) / 4, GSTEP = 64 / DW;
    static constexpr int G_TOT = G_RAW + ((16 / DW - G_RAW % GSTEP) % GSTEP + GSTEP) % GSTEP;
    // the partial lane group of a wavefront (VS > IPW: lanes that carry no instance) works in one
    // dummy area shared by the whole workgroup (its results are never used)
    static constexpr int NGA = WPB * IPW + (VS > IPW ? 1 : 0);
    static constexpr int LDS_ELEMS = C_TOT + NGA * G_TOT;
    __host__ __device__ static constexpr int group_area(int wave, int grp) { return grp < IPW ? wave * IPW + grp : WPB * IPW; }
    static constexpr int XPR = NU;        // x record: K(:, r) in words 0..NU-1, Pr_r in word NU
    static constexpr int UKFF = 0, UFI = 1;   // u record: kff_u, F_uu^{-1}(u, :) in words 1..NU
    static_assert(IPW >= 1, "stage wider than a wavefront");
};

// Scratch, wave-interleaved and stage-major: a wavefront owns (N+1) stage blocks of NW words
// x LW lanes (LW = IPW * NZ, the lanes that carry an instance: 51 for quad13); word w of stage
// k for lane l sits at (k NW + w) LW + l. Every access of a wavefront is one contiguous run of
// LW elements (408 B for quad13 fp64) instead of one partial-line segment per instance, and
// consecutive words share their boundary cache lines; the idle lanes of a wavefront address
// beyond the buffer (no memory traffic). Words: the element arrays (z, lambda_l, lambda_u,
// dz_aff, dz, G yref and, for non-diagonal costs, g) of component r, then the stage record of
// the lane (x-lane r: K(:, r), Pr_r; u-lane u: kff_u, F_uu^{-1}(u, :)). The dynamics residual
// is recomputed by the forward sweeps from z (no record word).
template <int NX, int NU, bool HDIAG = false>
struct Layout {
    static constexpr int LW = (64 / (NX + NU)) * (NX + NU);
    static constexpr int Z = 0, LL = 1, LU = 2, DZA = 3, DZ = 4, GC = 5, GF = HDIAG ? -1 : 6, REC = HDIAG ? 6 : 7;
    static constexpr int RECW = NU + 1;
    // ACT: active flag of the last solve's solution (fused closed loop: the next step's finish
    // starts from it, shifted by one stage)
    static constexpr int ACT = REC + RECW;
    static constexpr int NW = ACT + 1;
    __host__ __device__ static size_t wave_elems(int N) { return ((size_t)(N + 1) * NW * LW + 15) & ~size_t(15); }
};

template <typename T, int NX, int NU, int WPB, bool HDIAG>
inline size_t scratch_elems(int B, int N)
{
    using Gm = Geom<T, NX, NU, WPB>;
    const size_t waves = (size_t)(B + Gm::IPW - 1) / Gm::IPW;
    const size_t blocks = (waves + WPB - 1) / WPB;
    return blocks * WPB * Layout<NX, NU, HDIAG>::wave_elems(N);
}

}  // namespace lpc

template <typename T, int NX, int NU, int WPB, int MW, class SP>
hipError_t launch_ipm_lpc(const IpmParams<T> &p, hipStream_t s);

// lane-per-instance kernels (nmpc_ipm_lpi.hip)
template <typename T, int NX, int NU, class SP>
hipError_t launch_ipm_lpi(const IpmParams<T> &p, hipStream_t s);
template <int NX, int NU>
size_t lpi_words();
int lpi_instances_per_wave(int B);

}  // namespace nmpc

namespace nmpc {
namespace lpc {

// ---------------------------------------------------------------------------------------
// Compile-time model structure for the structure-specialised LPC kernels — the GPU analogue
// of acados generating model-specific C code (force_model/ocp.py:95-96 builds one solver per
// model). rows[l] has bit c set where [A B](l, c) may be nonzero: the structural closure of
// the continuous model (any integrator's discrete map of an affine ODE stays inside it).
// hdiag: H and He diagonal (LINEAR_LS with selection Vx/Vu and diagonal W, as every
// reference model has). tests/test_structures.py recomputes the masks from models.py. The
// host selects such a kernel only when the handle's discrete [A B] is exactly zero outside
// the mask and H, He are diagonal (nmpc::ipm_refine); otherwise the dense kernel runs.
template <int NX, int NU>
struct DenseStructure {
    static constexpr int id = 0;
    static constexpr bool hdiag = false;
    static constexpr bool ab(int, int) { return true; }
    static constexpr int max_row_nnz = NX + NU;
    static constexpr int max_col_nnz = NX;
};

// the mask rows are a template pack (not an array in memory) so that ab(l, c) folds to a
// constant once the stage loops are unrolled
template <int NX, int NU, int ID, unsigned... ROWS>
struct MaskStructure {
    static_assert(sizeof...(ROWS) == NX, "one mask row per state");
    static constexpr int id = ID;
    static constexpr bool hdiag = true;
    static constexpr bool ab(int l, int c)
    {
        int i = 0;
        bool res = false;
        ((res = (i++ == l) ? ((ROWS >> c) & 1u) != 0 : res), ...);
        return res;
    }
    static constexpr int max_nnz()
    {
        int m = 0;
        for (int l = 0; l < NX; l++) {
            int n = 0;
            for (int c = 0; c < NX + NU; c++) n += ab(l, c) ? 1 : 0;
            m = n > m ? n : m;
        }
        return m;
    }
    static constexpr int max_col_nnz_()
    {
        int m = 0;
        for (int c = 0; c < NX + NU; c++) {
            int n = 0;
            for (int l = 0; l < NX; l++) n += ab(l, c) ? 1 : 0;
            m = n > m ? n : m;
        }
        return m;
    }
    static constexpr int max_row_nnz = max_nnz();
    static constexpr int max_col_nnz = max_col_nnz_();
};

// force_model (force_model/dynamics.py:32-37): x = [px, pz, vx, vz], u = [Fx, Fz]
using ForceStructure = MaskStructure<4, 2, 1, 0x15u, 0x2au, 0x14u, 0x28u>;
// jerk_model (jerk_model/dynamics.py:35-42): x = [px, pz, vx, vz, ax, az], u = [hx, hz]
using JerkStructure = MaskStructure<6, 2, 2, 0x55u, 0xaau, 0x54u, 0xa8u, 0x50u, 0xa0u>;
// quad13 (models.py quad13_model): x = [p, v, q, w], u = [aT, alpha]
using Quad13Structure = MaskStructure<13, 4, 3, 0x8909u, 0x4492u, 0x2024u, 0x8908u, 0x4490u, 0x2020u, 0x40u, 0x4480u,
                                      0x8900u, 0x11200u, 0x4400u, 0x8800u, 0x11000u>;

// host check: the model fits structure SP (exact zeros outside the mask, diagonal costs)
template <class SP, int NX, int NU>
inline bool structure_fits(const double *AB, const double *H, const double *He)
{
    constexpr int NZ = NX + NU;
    for (int l = 0; l < NX; l++)
        for (int c = 0; c < NZ; c++)
            if (!SP::ab(l, c) && AB[l * NZ + c] != 0.0) return false;
    if (SP::hdiag) {
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j < NZ; j++)
                if (i != j && H[i * NZ + j] != 0.0) return false;
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NX; j++)
                if (i != j && He[i * NX + j] != 0.0) return false;
    }
    return true;
}

}  // namespace lpc
}  // namespace nmpc
