// Microbenchmark (dev tool): fp64 VALU issue cost per wave-instruction on gfx950 at 1..4 waves per SIMD, with
// CH independent chains per lane (each step: one v_mul_f64 + one v_add_f64, no FMA contraction).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench_fp64 tools/ubench_fp64.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH>
__global__ void k_chains(double *out, unsigned long long *cyc, int iters, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = x[c] * a + b;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
}

template <int CH>
void run(int wps, int iters) {
    const int blocks = 256, threads = 256 * wps;
    double *out;
    unsigned long long *cyc;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    hipMalloc(&cyc, 8);
    hipMemset(cyc, 0, 8);
    hipLaunchKernelGGL(k_chains<CH>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 16, 0.999, 1e-3);
    hipMemset(cyc, 0, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_chains<CH>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 0.999, 1e-3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double waves = blocks * threads / 64.0;
    const double instr = 2.0 * CH * iters;                       // per wave
    const double cyc_per_wave = c / waves;
    const double flops = 2.0 * CH * iters * blocks * threads;
    printf("CH=%2d waves/SIMD=%d: %.3f ms, %.2f cycles per fp64 wave-instr per wave, %.2f SIMD-cycles per instr, "
           "%.1f TFLOP/s, clock %.2f GHz\n",
           CH, wps, ms, cyc_per_wave / instr, cyc_per_wave / instr / wps, flops / (ms * 1e-3) / 1e12,
           cyc_per_wave / (ms * 1e-3) / 1e9);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    const int iters = 20000;
    for (int w = 1; w <= 4; w *= 2) {
        run<1>(w, iters);
        run<2>(w, iters);
        run<4>(w, iters);
        run<8>(w, iters);
    }
    return 0;
}
