// pass_bench.hip — microbenchmark of the streamed CSS objective pass (the inner loop of k_cg_fit), used to choose
// how a wave should stream its 64 series rows. Not part of the library.
//
// Workload: G = lanes in flight, each lane re-streams ONE series row P times in a row (as the optimizer does:
// ~50 passes per fit), computing the ARIMA(2,*,2)+c objective recursion (arima_device.hpp css_pass) with NCH
// independent coefficient chains per pass. Reports the row bytes streamed per second.
//
// Variants
//   lane  : every lane streams its own row with per-lane 16-B loads (the round-1 design; D chunks in flight)
//   glds  : the wave streams its 64 rows cooperatively: one global_load_lds_dwordx4 wave-instruction moves 8 rows x
//           128 B (fully coalesced) into an LDS ring slot; lanes read their row's 16 doubles with ds_read_b128 from
//           an XOR-swizzled image (swizzle applied on the global SOURCE address, image lane-linear)
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o pass_bench pass_bench.hip
// Run:   ./pass_bench [rows_in_flight_per_cu_scale]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../spark-timeseries_amd/csrc/arima_device.hpp"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

using namespace sts;

constexpr int P_ = 2, Q_ = 2, I_ = 1, K_ = 5;

// ---------------------------------------------------------------------------------------------------------------
// per-lane variant: css_pass_multi over the lane's own row (stream_elems, D = kPrefetchF chunks in flight)
template <int NCH, int W>
__global__ __launch_bounds__(64 * W) void k_lane(const double *__restrict__ y, int64_t ld, int n, int rows_per_lane,
                                                 int passes, double *__restrict__ out) {
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0.0;
    for (int rr = 0; rr < rows_per_lane; ++rr) {
        const double *row = y + (g + rr * G) * ld;
        for (int ps = 0; ps < passes; ++ps) {
            double c[NCH][K_], css[NCH];
#pragma unroll
            for (int h = 0; h < NCH; ++h) {
                c[h][0] = 8.2 + 1e-3 * ps;
                c[h][1] = 0.2 + 1e-4 * h;
                c[h][2] = 0.5;
                c[h][3] = 0.3;
                c[h][4] = 0.1 + 1e-5 * rr;
            }
            css_pass_multi<P_, Q_, I_, NCH>(row, n, c, css);
#pragma unroll
            for (int h = 0; h < NCH; ++h) acc += css[h];
        }
    }
    out[g] = acc;
}

// gradient pass (css_pass<..., G = true, smear>), one chain, per lane over its own row
template <int W>
__global__ __launch_bounds__(64 * W) void k_lane_g(const double *__restrict__ y, int64_t ld, int n, int rows_per_lane,
                                                   int passes, double *__restrict__ out) {
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0.0;
    for (int rr = 0; rr < rows_per_lane; ++rr) {
        const double *row = y + (g + rr * G) * ld;
        for (int ps = 0; ps < passes; ++ps) {
            double c[K_] = {8.2 + 1e-3 * ps, 0.2, 0.5, 0.3, 0.1 + 1e-5 * rr}, css, gr[K_];
            css_pass<P_, Q_, I_, true, true>(row, n, c, css, gr);
            acc += css;
#pragma unroll
            for (int j = 0; j < K_; ++j) acc += gr[j];
        }
    }
    out[g] = acc;
}

// ---------------------------------------------------------------------------------------------------------------
// cooperative variant: LDS ring of R slots per wave, one slot = 64 rows x 16 doubles (8 KB)
__device__ __forceinline__ void glds16(const void *g, void *lds) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)g,
                                     (void __attribute__((address_space(3))) *)lds, 16, 0, 0);
}

template <int NCH, int W, int R>
__global__ __launch_bounds__(64 * W) void k_glds(const double *__restrict__ y, int64_t ld, int n, int rows_per_lane,
                                                 int passes, double *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) double ring[W][R][64 * 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t wave_row0 = g - lane;       // the wave's 64 rows are consecutive (g - lane .. g - lane + 63)
    constexpr int M = 2;
    const int nch = (n + 15) / 16;            // chunks covering [0, n)
    double acc = 0.0;
    for (int rr = 0; rr < rows_per_lane; ++rr) {
        const int64_t rbase = wave_row0 + rr * G;
        // source addresses of this lane's 8 pieces: piece i covers rows 8i .. 8i+7; lane -> row 8i + lane/8,
        // LDS position lane%8 of that row holds segment (lane%8) ^ f(row), f(r) = (r >> 1) & 7
        const double *src[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = 8 * i + (lane >> 3);
            const int seg = (lane & 7) ^ ((r >> 1) & 7);
            src[i] = y + (rbase + r) * ld + seg * 2;
        }
        const int myseg_sw = (lane >> 1) & 7;
        for (int ps = 0; ps < passes; ++ps) {
            double c[NCH][K_], e1[NCH], e2[NCH], css[NCH], yh0[NCH];
#pragma unroll
            for (int h = 0; h < NCH; ++h) {
                c[h][0] = 8.2 + 1e-3 * ps;
                c[h][1] = 0.2 + 1e-4 * h;
                c[h][2] = 0.5;
                c[h][3] = 0.3;
                c[h][4] = 0.1 + 1e-5 * rr;
                e1[h] = e2[h] = css[h] = 0.0;
                yh0[h] = 0.0 + (double)I_ * c[h][0];
            }
            double yl0 = 0.0, yl1 = 0.0;
            // prologue: R - 1 chunks in flight
#pragma unroll
            for (int j = 0; j < R - 1; ++j) {
                if (j < nch) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) glds16(src[i] + j * 16, &ring[wave][j][i * 128]);
                }
            }
            for (int ch = 0; ch < nch; ++ch) {
                const int nx = ch + R - 1;
                if (nx < nch) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) glds16(src[i] + nx * 16, &ring[wave][nx % R][i * 128]);
                    // all but the (R - 1) * 8 youngest DMAs done => chunk ch has landed
                    if constexpr (R == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    else if constexpr (R == 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                const double *slot = &ring[wave][ch % R][lane * 16];
                double v[16];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const double2 t = *reinterpret_cast<const double2 *>(slot + 2 * (j ^ myseg_sw));
                    v[2 * j] = t.x;
                    v[2 * j + 1] = t.y;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int t = ch * 16 + u;
                    const double yi = v[u];
                    if (t >= M && t < n) {
#pragma unroll
                        for (int h = 0; h < NCH; ++h) {
                            double yh = yh0[h];
                            yh = yh + yl0 * c[h][1];
                            yh = yh + yl1 * c[h][2];
                            yh = yh + e1[h] * c[h][3];
                            yh = yh + e2[h] * c[h][4];
                            const double e = yi - yh;
                            css[h] = css[h] + e * e;
                            e2[h] = e1[h];
                            e1[h] = e;
                        }
                    }
                    yl1 = yl0;
                    yl0 = yi;
                }
            }
#pragma unroll
            for (int h = 0; h < NCH; ++h) acc += css[h];
        }
    }
    out[g] = acc;
}

__global__ void k_fill(double *y, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) {
        uint32_t x = (uint32_t)(i * 2654435761u) ^ 0x9e3779b9u;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        y[i] = (double)(x & 0xffff) / 65536.0 - 0.5;
    }
}

template <class KFn>
double run(const char *name, KFn kfn, int blocks, int threads, const double *y, int64_t ld, int n, int rpl,
           int passes, double *out, double bytes) {
    hipLaunchKernelGGL(kfn, dim3(blocks), dim3(threads), 0, 0, y, ld, n, rpl, 1, out);   // warm
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(kfn, dim3(blocks), dim3(threads), 0, 0, y, ld, n, rpl, passes, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-34s blocks %5d x %4d  %8.2f ms  %7.1f GB/s (row bytes streamed)\n", name, blocks, threads, ms,
           bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
    return ms;
}

int main(int argc, char **argv) {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int T = 1024, n = 1023;
    const int64_t ld = 1024;
    const int passes = argc > 1 ? atoi(argv[1]) : 20;
    const int64_t lanes_max = (int64_t)cus * 512;       // 8 waves per CU
    const int rpl = 2;                                  // rows per lane (sequentially)
    const int64_t rows = lanes_max * rpl;
    double *y, *out;
    CK(hipMalloc(&y, rows * ld * sizeof(double)));
    CK(hipMalloc(&out, lanes_max * sizeof(double)));
    hipLaunchKernelGGL(k_fill, dim3((rows * ld + 255) / 256), dim3(256), 0, 0, y, rows * ld);
    CK(hipDeviceSynchronize());
    printf("CUs %d, T %d, passes %d, rows per lane %d\n", cus, T, passes, rpl);
    auto bytes = [&](int64_t lanes) { return (double)lanes * rpl * passes * n * 8.0; };
#define RUN_LANE(NCH, W, BPC)                                                                            \
    run("lane NCH=" #NCH " W=" #W " blk/CU=" #BPC, k_lane<NCH, W>, cus * BPC, 64 * W, y, ld, n, rpl, passes, out, \
        bytes((int64_t)cus * BPC * 64 * W))
#define RUN_GLDS(NCH, W, R, BPC)                                                                         \
    run("glds NCH=" #NCH " W=" #W " R=" #R " blk/CU=" #BPC, k_glds<NCH, W, R>, cus * BPC, 64 * W, y, ld, n, rpl, \
        passes, out, bytes((int64_t)cus * BPC * 64 * W))
#define RUN_LANEG(W, BPC)                                                                                \
    run("laneG W=" #W " blk/CU=" #BPC, k_lane_g<W>, cus * BPC, 64 * W, y, ld, n, rpl, passes, out,               \
        bytes((int64_t)cus * BPC * 64 * W))
    // waves per SIMD = W * BPC / 4: the issue efficiency of one pass type at 1 / 2 waves per SIMD
    RUN_LANE(1, 4, 1);
    RUN_LANE(1, 4, 2);
    RUN_LANE(3, 4, 1);
    RUN_LANE(3, 4, 2);
    RUN_LANEG(4, 1);
    RUN_LANEG(4, 2);
    RUN_LANE(2, 4, 1);
    RUN_LANE(4, 4, 1);
    RUN_GLDS(1, 4, 2, 1);
    RUN_GLDS(1, 4, 3, 1);
    RUN_GLDS(1, 4, 4, 1);
    RUN_GLDS(1, 4, 2, 2);
    RUN_GLDS(2, 4, 3, 1);
    RUN_GLDS(4, 4, 3, 1);
    RUN_GLDS(4, 4, 4, 1);
    RUN_GLDS(1, 2, 4, 2);
    RUN_GLDS(1, 8, 2, 1);
    return 0;
}
