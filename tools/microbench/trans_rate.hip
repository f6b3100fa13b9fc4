// Issue cost of fp64/fp32 transcendentals vs FMA on gfx950: 8 independent dependency chains per
// lane, 8 waves per SIMD; prints ns per wave-instruction per CU (cycles = ns * clock).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int kOp>
__global__ __launch_bounds__(256) void k(double* out, int iters) {
    double x[8];
    float y[8];
    for (int i = 0; i < 8; i++) x[i] = 1.0 + 1e-3 * (threadIdx.x + i), y[i] = (float)x[i];
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (kOp == 0) x[i] = __builtin_amdgcn_rsq(x[i]);
            if (kOp == 1) x[i] = __builtin_amdgcn_rcp(x[i]);
            if (kOp == 2) y[i] = __builtin_amdgcn_rsqf(y[i]);
            if (kOp == 3) x[i] = __builtin_fma(x[i], 0.999, 1e-3);
            if (kOp == 4) x[i] = (double)__builtin_amdgcn_rsqf((float)x[i]);
        }
    }
    double s = 0;
    for (int i = 0; i < 8; i++) s += x[i] + y[i];
    if (s == 12345.0) out[threadIdx.x] = s;
}

int main() {
    double* out;
    hipMalloc(&out, 4096);
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount, blocks = cus * 8, iters = 20000;  // 8 blocks of 4 waves per CU = 8 waves/SIMD
    const char* names[] = {"v_rsq_f64", "v_rcp_f64", "v_rsq_f32", "v_fma_f64", "cvt+rsq_f32+cvt"};
    for (int op = 0; op < 5; op++) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (op == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        // wave-instructions per SIMD: 8 waves x iters x 8 ops
        const double per_simd = 8.0 * iters * 8;
        printf("%-18s %.3f ms  %.2f ns per wave-op per SIMD (x clock GHz = cycles)\n", names[op], ms, ms * 1e6 / per_simd);
    }
    return 0;
}
