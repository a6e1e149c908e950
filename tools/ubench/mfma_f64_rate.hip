// f64 MFMA issue rates on one wavefront (tuning aid, needs a GPU): cycles per instruction for chains of
// independent v_mfma_f64_4x4x4_4b_f64 / v_mfma_f64_16x16x4_f64, and for v_fma_f64 (s_memtime, one wave
// per SIMD, and two waves per SIMD)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
template <int K>
__global__ void r44(double *out, long long *cyc, int iters)
{
    double acc[K];
    const double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    for (int k = 0; k < K; k++) acc[k] = k;
    const long long t0 = clock64();
    for (int it = 0; it < iters; it++)
#pragma unroll
        for (int k = 0; k < K; k++) acc[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[k], 0, 0, 0);
    const long long t1 = clock64();
    double s = 0;
    for (int k = 0; k < K; k++) s += acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int K>
__global__ void r16(double *out, long long *cyc, int iters)
{
    v4d acc[K];
    const double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    for (int k = 0; k < K; k++) acc[k] = v4d{(double)k, 0, 0, 0};
    const long long t0 = clock64();
    for (int it = 0; it < iters; it++)
#pragma unroll
        for (int k = 0; k < K; k++) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    const long long t1 = clock64();
    double s = 0;
    for (int k = 0; k < K; k++) s += acc[k][0] + acc[k][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int K>
__global__ void rfma(double *out, long long *cyc, int iters)
{
    double acc[K];
    const double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    for (int k = 0; k < K; k++) acc[k] = k;
    const long long t0 = clock64();
    for (int it = 0; it < iters; it++)
#pragma unroll
        for (int k = 0; k < K; k++) acc[k] = fma(a, acc[k], b);
    const long long t1 = clock64();
    double s = 0;
    for (int k = 0; k < K; k++) s += acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <class F>
void run(const char *name, F kern, int per_iter, int wpb)
{
    double *o;
    long long *c;
    const int iters = 2000, blocks = 256;
    if (hipMalloc(&o, blocks * 64 * wpb * sizeof(double)) != hipSuccess || hipMalloc(&c, blocks * sizeof(long long)) != hipSuccess) return;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), 0, 0, o, c, iters);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), 0, 0, o, c, iters);
    long long h[256];
    if (hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return;
    double m = 0;
    for (int i = 0; i < blocks; i++) m += (double)h[i] / blocks;
    printf("%-24s waves/SIMD %d: %.1f cycles per instruction per wave\n", name, wpb / 4 > 0 ? wpb / 4 : 1, m / ((double)iters * per_iter));
    (void)hipFree(o);
    (void)hipFree(c);
}
// a dependent chain through a lane permute (the D -> B layout change of the sweeps): mfma, then the result
// through ds_bpermute, as the next mfma's B operand
__global__ void rchain(double *out, long long *cyc, int iters)
{
    double acc = threadIdx.x, x = 1.0;
    const double a = threadIdx.x * 1e-3;
    const int src = (threadIdx.x & 0x33) | (1 << 2);
    const long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a, x, acc, 0, 0, 0);
        x = __shfl(acc, src);
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main()
{
    for (int wpb : {4, 8}) {
        run("mfma_f64_4x4x4_4b x16", r44<16>, 16, wpb);
        run("mfma_f64_4x4x4_4b dep", r44<1>, 1, wpb);
        run("mfma_f64_16x16x4 x8", r16<8>, 8, wpb);
        run("mfma_f64_16x16x4 dep", r16<1>, 1, wpb);
        run("v_fma_f64 x16 indep", rfma<16>, 16, wpb);
        run("mfma4x4 -> bpermute dep", rchain, 1, wpb);
    }
    return 0;
}
