// nmpc_cond_host.cpp — condensing of the stage-wise LQ-OCP for the condensed IPM kernels.
//
// What acados's PARTIAL_CONDENSING_HPIPM does with a single block (src/force_model/ocp.py:83):
// eliminate the states through the dynamics x_{k+1} = A x_k + B u_k + c,
//     x_k = Phi_k x0 + d_k + Gamma_k U,   Phi_k = A^k,  d_{k+1} = A d_k + c,
//     Gamma_{k+1} = A Gamma_k + [0 .. B (block k) .. 0],
// and collect the stage costs 1/2 z'H z + (G yref_k)' z (z_k = [x_k; u_k] = E_k U + e_k) and the
// terminal cost into
//     H0 = sum_k E_k' H E_k + Gamma_N' He Gamma_N,
//     f  = fc + Fx x0 + Fy yref   (every term affine in x0 and the yref window),
// plus the bounded state components of stages 1..N-1 (and N when terminal bounds exist) as
// rows of Gx = Gamma_x with offsets xf = Phx x0 + dx. Everything here is shared by all
// instances of a handle and computed once at nmpc_create in double precision.
#include <algorithm>
#include <cmath>
#include <vector>

#include "nmpc_internal.h"

namespace nmpc {

static bool hasb(double b) { return std::fabs(b) < 1e20; }

bool cond_build(int nx, int nu, int N, int ny, int ny_e, const std::vector<double> &A, const std::vector<double> &Bm,
                const std::vector<double> &c, const std::vector<double> &H, const std::vector<double> &G,
                const std::vector<double> &He, const std::vector<double> &Ge, const std::vector<double> &lbnd,
                const std::vector<double> &ubnd, CondHost &o)
{
    const int nz = nx + nu, n = N * nu;
    // state maps for k = 0..N: Gam[k] (nx x n), Phi[k] (nx x nx), d[k] (nx)
    std::vector<std::vector<double>> Gam(N + 1, std::vector<double>((size_t)nx * n, 0.0)),
        Phi(N + 1, std::vector<double>((size_t)nx * nx, 0.0)), d(N + 1, std::vector<double>(nx, 0.0));
    for (int i = 0; i < nx; i++) Phi[0][i * nx + i] = 1.0;
    for (int k = 0; k < N; k++) {
        for (int i = 0; i < nx; i++) {
            for (int j = 0; j < n; j++) {
                double s = 0.0;
                for (int l = 0; l < nx; l++) s += A[i * nx + l] * Gam[k][l * n + j];
                Gam[k + 1][i * n + j] = s;
            }
            for (int j = 0; j < nu; j++) Gam[k + 1][i * n + k * nu + j] += Bm[i * nu + j];
            for (int j = 0; j < nx; j++) {
                double s = 0.0;
                for (int l = 0; l < nx; l++) s += A[i * nx + l] * Phi[k][l * nx + j];
                Phi[k + 1][i * nx + j] = s;
            }
            double s = c[i];
            for (int l = 0; l < nx; l++) s += A[i * nx + l] * d[k][l];
            d[k + 1][i] = s;
        }
    }
    // bounded x rows, stage-major
    std::vector<int> rk, ri;
    for (int k = 1; k <= N; k++) {
        const int t = k < N ? 1 : 2;
        for (int i = 0; i < nx; i++)
            if (hasb(lbnd[t * nz + i]) || hasb(ubnd[t * nz + i])) {
                rk.push_back(k);
                ri.push_back(i);
            }
    }
    const int mx = (int)rk.size();
    if (n > 128 || n + mx > 512) return false;
    const int nb = (n + 15) / 16, np = 16 * nb, mxp = (mx + 3) & ~3;
    int ldg = std::max(mxp, 2);
    while (ldg % 32 != 2) ldg++;   // == 2 mod 32: conflict-free MFMA operand reads (nmpc_cond.hip)
    o.n = n;
    o.nb = nb;
    o.mx = mx;
    o.ldg = ldg;
    o.nY = N * ny + ny_e;
    o.Gx.assign((size_t)np * ldg, 0.0);
    o.Phx.assign((size_t)nx * std::max(mx, 1), 0.0);
    o.dx.assign(std::max(mx, 1), 0.0);
    o.lox.assign(std::max(mx, 1), -1e30);
    o.hix.assign(std::max(mx, 1), 1e30);
    o.xcols.assign(std::max(mx, 1), 0);
    for (int r = 0; r < mx; r++) {
        const int k = rk[r], i = ri[r], t = k < N ? 1 : 2;
        for (int j = 0; j < n; j++) o.Gx[(size_t)j * ldg + r] = Gam[k][i * n + j];
        for (int a = 0; a < nx; a++) o.Phx[(size_t)a * mx + r] = Phi[k][i * nx + a];
        o.dx[r] = d[k][i];
        o.lox[r] = lbnd[t * nz + i];
        o.hix[r] = ubnd[t * nz + i];
        o.xcols[r] = std::min(n, k * nu);
    }
    o.rstart.assign(n, mx);
    for (int i = 0; i < n; i++)
        for (int r = 0; r < mx; r++)
            if (rk[r] * nu > i) {
                o.rstart[i] = r;
                break;
            }
    o.ks.assign(nb, mxp / 4);
    for (int I = 0; I < nb; I++)
        for (int r = 0; r < mx; r++)
            if (rk[r] * nu > 16 * I) {
                o.ks[I] = r / 4;
                break;
            }
    // condensed cost: E_k = [Gamma_k; S_k] maps U to z_k
    o.H0.assign((size_t)n * n, 0.0);
    o.Fx.assign((size_t)nx * n, 0.0);
    o.fc.assign(n, 0.0);
    o.Fy.assign((size_t)o.nY * n, 0.0);
    std::vector<double> E((size_t)nz * n), HE((size_t)nz * n);
    for (int k = 0; k <= N; k++) {
        const bool term = k == N;
        const int m = term ? nx : nz;
        const std::vector<double> &Hk = term ? He : H;
        std::fill(E.begin(), E.end(), 0.0);
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < n; j++) E[(size_t)i * n + j] = Gam[k][i * n + j];
        if (!term)
            for (int i = 0; i < nu; i++) E[(size_t)(nx + i) * n + k * nu + i] = 1.0;
        // HE = Hk E (m x n)
        for (int i = 0; i < m; i++)
            for (int j = 0; j < n; j++) {
                double s = 0.0;
                for (int l = 0; l < m; l++) s += Hk[i * m + l] * E[(size_t)l * n + j];
                HE[(size_t)i * n + j] = s;
            }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                double s = 0.0;
                for (int l = 0; l < m; l++) s += E[(size_t)l * n + i] * HE[(size_t)l * n + j];
                o.H0[(size_t)j * n + i] += s;
            }
        // linear terms: E' Hk e_k with e_k = [Phi_k x0 + d_k; 0], and E' Gk yref_k
        for (int i = 0; i < n; i++) {
            for (int a = 0; a < nx; a++) {
                double s = 0.0;
                for (int l = 0; l < m; l++)
                    for (int q = 0; q < nx; q++) s += E[(size_t)l * n + i] * Hk[l * m + q] * Phi[k][q * nx + a];
                o.Fx[(size_t)a * n + i] += s;
            }
            double s = 0.0;
            for (int l = 0; l < m; l++)
                for (int q = 0; q < nx; q++) s += E[(size_t)l * n + i] * Hk[l * m + q] * d[k][q];
            o.fc[i] += s;
            const int nyk = term ? ny_e : ny, off = k * ny;
            const std::vector<double> &Gk = term ? Ge : G;
            for (int b = 0; b < nyk; b++) {
                double t = 0.0;
                for (int l = 0; l < m; l++) t += E[(size_t)l * n + i] * Gk[l * nyk + b];
                o.Fy[(size_t)(off + b) * n + i] = t;
            }
        }
    }
    // lower tiles of H0, column-major 16x16 each
    o.H0t.assign((size_t)nb * (nb + 1) / 2 * 256, 0.0);
    for (int I = 0; I < nb; I++)
        for (int J = 0; J <= I; J++)
            for (int cc = 0; cc < 16; cc++)
                for (int rr = 0; rr < 16; rr++) {
                    const int i = 16 * I + rr, j = 16 * J + cc;
                    if (i < n && j < n) o.H0t[(size_t)(I * (I + 1) / 2 + J) * 256 + cc * 16 + rr] = o.H0[(size_t)j * n + i];
                }
    // input bounds per column of U
    o.lou.assign(n, -1e30);
    o.hiu.assign(n, 1e30);
    for (int k = 0; k < N; k++)
        for (int i = 0; i < nu; i++) {
            const int t = k == 0 ? 0 : 1;
            o.lou[k * nu + i] = lbnd[t * nz + nx + i];
            o.hiu[k * nu + i] = ubnd[t * nz + nx + i];
        }
    // outputs
    const int nrow = (N + 1) * nx;
    o.Gall.assign((size_t)n * nrow, 0.0);
    o.Phall.assign((size_t)nx * nrow, 0.0);
    o.dall.assign(nrow, 0.0);
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < nx; i++) {
            const int r = k * nx + i;
            for (int j = 0; j < n; j++) o.Gall[(size_t)j * nrow + r] = Gam[k][i * n + j];
            for (int a = 0; a < nx; a++) o.Phall[(size_t)a * nrow + r] = Phi[k][i * nx + a];
            o.dall[r] = d[k][i];
        }
    return true;
}

}  // namespace nmpc
