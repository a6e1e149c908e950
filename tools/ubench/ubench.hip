// Single-wavefront issue / latency micro-benchmarks on gfx950 (s_memtime cycles), to calibrate
// the per-stage cost model of the IPM kernels. One workgroup of 64 lanes.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256

__global__ void k_fma_indep(double *out, unsigned long long *cyc, double a, double b)
{
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; i++) {
#define F64(x) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b))
        F64(x0); F64(x1); F64(x2); F64(x3); F64(x4); F64(x5); F64(x6); F64(x7);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}
__global__ void k_fma_dep(double *out, unsigned long long *cyc, double a, double b)
{
    double x0 = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP * 8; i++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}
__global__ void k_f32_indep(double *out, unsigned long long *cyc, double a_, double b_)
{
    float a = a_, b = b_;
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; i++) {
#define F32(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b))
        F32(x0); F32(x1); F32(x2); F32(x3); F32(x4); F32(x5); F32(x6); F32(x7);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}
__global__ void k_rcp_indep(double *out, unsigned long long *cyc, double a, double b)
{
    double x0 = threadIdx.x + a, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; i++) {
#define RCP(x) asm volatile("v_rcp_f64 %0, %0" : "+v"(x))
        RCP(x0); RCP(x1); RCP(x2); RCP(x3); RCP(x4); RCP(x5); RCP(x6); RCP(x7);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}
__global__ void k_cnd_indep(double *out, unsigned long long *cyc, double a, double b)
{
    unsigned x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    const bool p = threadIdx.x & 1;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < REP; i++) {
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x0) : "v"(x1));
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x2) : "v"(x3));
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x4) : "v"(x5));
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x6) : "v"(x7));
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x1) : "v"(x0));
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x3) : "v"(x2));
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x5) : "v"(x4));
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x7) : "v"(x6));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + p;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}
// LDS round trip: write then dependent read of another lane's value, REP times
__global__ void k_lds_rt(double *out, unsigned long long *cyc, double a, double b)
{
    __shared__ double s[64];
    double x = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; i++) {
        s[threadIdx.x] = x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        x = s[(threadIdx.x + 1) & 63] * a;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}
// ds_bpermute round trip (dependent)
__global__ void k_bperm(double *out, unsigned long long *cyc, double a, double b)
{
    double x = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; i++) x = __shfl(x, (threadIdx.x + 1) & 63, 64) * a;
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}

__global__ void k_lds_rd(double *out, unsigned long long *cyc, double a, double b)
{
    __shared__ double s[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) s[i] = i;
    __syncthreads();
    double acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
    for (int i = 0; i < REP; i++) acc += s[(i * 8) & 1023];   // broadcast reads
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) { cyc[2 * (threadIdx.x >> 6)] = t0; cyc[2 * (threadIdx.x >> 6) + 1] = t1; }
}
typedef void (*kfn)(double *, unsigned long long *, double, double);
int main()
{
    double *out;
    unsigned long long *cyc, h;
    hipMalloc(&out, 1024 * 8);
    hipMalloc(&cyc, 64 * 8);
    struct { const char *name; kfn f; int ops; } ks[] = {
        {"v_fma_f64 independent (8 chains)", k_fma_indep, REP * 8},
        {"v_fma_f64 dependent chain", k_fma_dep, REP * 8},
        {"v_fma_f32 independent (8 chains)", k_f32_indep, REP * 8},
        {"v_rcp_f64 independent (8 chains)", k_rcp_indep, REP * 8},
        {"v_cndmask_b32 independent", k_cnd_indep, REP * 8},
        {"LDS write + dependent read (round trip)", k_lds_rt, REP},
        {"ds_read_b64 broadcast + add chain", k_lds_rd, REP},
        {"ds_bpermute f64 dependent (2 x b32)", k_bperm, REP},
    };
    for (auto &k : ks) {
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, out, cyc, 1.0000001, 1e-9);
        hipDeviceSynchronize();
        unsigned long long hc[2];
        hipMemcpy(hc, cyc, 16, hipMemcpyDeviceToHost);
        h = hc[1] - hc[0];
        std::printf("%-42s %8.2f cycles/op (one wave)\n", k.name, (double)h / k.ops);
    }
    // multi-wave throughput on one CU: 4 waves per SIMD (16 waves in one workgroup of 1024)
    for (int wps = 1; wps <= 4; wps++)
        for (auto &k : ks) {
            if (k.f != k_fma_indep && k.f != k_rcp_indep && k.f != k_f32_indep && k.f != k_cnd_indep) continue;
            for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k.f, dim3(1), dim3(256 * wps), 0, 0, out, cyc, 1.0000001, 1e-9);
            hipDeviceSynchronize();
            unsigned long long hc[64];
            const int nw = 4 * wps;
            hipMemcpy(hc, cyc, nw * 16, hipMemcpyDeviceToHost);
            unsigned long long lo = ~0ull, hi = 0;
            for (int i = 0; i < nw; i++) { lo = hc[2 * i] < lo ? hc[2 * i] : lo; hi = hc[2 * i + 1] > hi ? hc[2 * i + 1] : hi; }
            std::printf("%-42s %8.2f cycles/op per SIMD (%d waves per SIMD: all-wave span / ops / waves-per-SIMD)\n", k.name,
                        (double)(hi - lo) / k.ops / wps, wps);
        }
    return 0;
}
