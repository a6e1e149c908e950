// Layout probe for the f64 MFMA shapes (tuning aid, needs a GPU): wave w sets B = one-hot at lane w and
// A[l] = l + 1, so D = A[:, k(w)] lands in column n(w) of w's block; the nonzero D lanes and their values
// (the A lane + 1 holding (i, k(w))) give the A / B / D lane maps. Prints one line per probe lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void probe44(double *out)
{
    const int l = threadIdx.x, w = blockIdx.x;
    const double a = l + 1, b = l == w ? 1.0 : 0.0;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[w * 64 + l] = d;
}
__global__ void probe16(double *out)
{
    const int l = threadIdx.x, w = blockIdx.x;
    const double a = l + 1, b = l == w ? 1.0 : 0.0;
    v4d d = {0, 0, 0, 0};
    d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
    for (int r = 0; r < 4; r++) out[(w * 64 + l) * 4 + r] = d[r];
}
int main()
{
    double *d;
    if (hipMalloc(&d, 64 * 64 * 4 * sizeof(double)) != hipSuccess) return 1;
    std::vector<double> h(64 * 64 * 4);
    hipLaunchKernelGGL(probe44, dim3(64), dim3(64), 0, 0, d);
    if (hipMemcpy(h.data(), d, 64 * 64 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("4x4x4_4b: probe B lane -> [(D lane, value = A lane + 1)]\n");
    for (int w = 0; w < 64; w++) {
        printf("B%02d:", w);
        for (int l = 0; l < 64; l++)
            if (h[w * 64 + l] != 0.0) printf(" (%d,%g)", l, h[w * 64 + l]);
        printf("\n");
    }
    hipLaunchKernelGGL(probe16, dim3(64), dim3(64), 0, 0, d);
    if (hipMemcpy(h.data(), d, 64 * 64 * 4 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("16x16x4: probe B lane -> [(D lane, reg, value = A lane + 1)]\n");
    for (int w = 0; w < 64; w++) {
        printf("B%02d:", w);
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < 4; r++)
                if (h[(w * 64 + l) * 4 + r] != 0.0) printf(" (%d,%d,%g)", l, r, h[(w * 64 + l) * 4 + r]);
        printf("\n");
    }
    hipFree(d);
    return 0;
}
