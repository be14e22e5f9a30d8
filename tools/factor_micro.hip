// Diagnostic micro-benchmark (not part of the library): the LBA reduced-system factorization + substitutions
// (lba_kernels.hip factor_reg / factor_body) alone on one workgroup, an SPD system of n rows, cycles from
// s_memtime (100 MHz constant clock on gfx950: x24 for 2.4 GHz shader cycles).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I sp-slam_amd/csrc -I include \
//         -o /tmp/factor_micro tools/factor_micro.hip
#include "lba_kernels.hip"

#include <cstdio>
#include <vector>

namespace spslam {
namespace lba {
template <int kVariant>
__global__ __launch_bounds__(kThreads) void fbench(double* S, double* bs, double* y, double* dd, LbaCtl* ctl, int n,
                                                   long long* cyc) {
    extern __shared__ double lds[];
    Ctx c{};
    c.S = S; c.bs = bs; c.y = y; c.dd = dd;
    __syncthreads();
    const long long t0 = wall_clock64();
    if (kVariant == 0) {
        if (n <= 64) factor_reg<1>(c, *ctl, lds, n);
        else factor_reg<2>(c, *ctl, lds, n);
    }
    else factor_body<true>(c, *ctl, lds, n);
    __syncthreads();
    const long long t1 = wall_clock64();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
// building blocks, 64 columns each: kOp 0 barrier only; 1 + an LDS read feeding a uniform branch; 2 + one
// wave's fp64 division and LDS store before the barrier
template <int kOp>
__global__ __launch_bounds__(kThreads) void bblock(double* out, long long* cyc) {
    __shared__ double buf[4096];
    const int t = threadIdx.x;
    for (int i = t; i < 4096; i += kThreads) buf[i] = 1.0 + i;
    __syncthreads();
    double acc = 0.0;
    const long long t0 = wall_clock64();
    for (int j = 0; j < 64; j++) {
        if (kOp >= 1) {
            const double d = buf[j];
            if (d == 0.0) break;
            acc += d;
        }
        if (kOp >= 2 && (t >> 6) == (j & 3)) buf[64 + j * 64 + (t & 63)] = buf[j * 64 + (t & 63)] / acc;
        __syncthreads();
    }
    const long long t1 = wall_clock64();
    out[t] = acc;
    if (t == 0) cyc[0] = t1 - t0;
}
}  // namespace lba
}  // namespace spslam

int main() {
    using namespace spslam::lba;
    const int ns[] = {24, 60, 78, 120};
    double *S, *bs, *y, *dd;
    spslam::LbaCtl* ctl;
    long long* cyc;
    (void)hipMalloc(&S, 140 * 140 * 8); (void)hipMalloc(&bs, 140 * 8); (void)hipMalloc(&y, 140 * 8);
    (void)hipMalloc(&dd, 140 * 8); (void)hipMalloc(&ctl, sizeof(spslam::LbaCtl)); (void)hipMalloc(&cyc, 64);
    (void)hipFuncSetAttribute((const void*)fbench<0>, hipFuncAttributeMaxDynamicSharedMemorySize, kFactorLds);
    (void)hipFuncSetAttribute((const void*)fbench<1>, hipFuncAttributeMaxDynamicSharedMemorySize, kFactorLds);
    {
        double* out;
        (void)hipMalloc(&out, 4096 * 8);
        for (int op = 0; op < 3; op++) {
            long long best = 1ll << 60;
            for (int rep = 0; rep < 4; rep++) {
                if (op == 0) hipLaunchKernelGGL(bblock<0>, dim3(1), dim3(kThreads), 0, 0, out, cyc);
                if (op == 1) hipLaunchKernelGGL(bblock<1>, dim3(1), dim3(kThreads), 0, 0, out, cyc);
                if (op == 2) hipLaunchKernelGGL(bblock<2>, dim3(1), dim3(kThreads), 0, 0, out, cyc);
                (void)hipDeviceSynchronize();
                long long cv = 0;
                (void)hipMemcpy(&cv, cyc, 8, hipMemcpyDeviceToHost);
                best = cv < best ? cv : best;
            }
            std::printf("64 columns of building block %d: %.2f us (%.0f ns per column)\n", op, best * 0.01,
                        best * 10.0 / 64);
        }
    }
    for (int n : ns) {
        std::vector<double> h(n * n), b(n);
        for (int i = 0; i < n; i++) {
            b[i] = 1.0 + 0.01 * i;
            for (int j = 0; j < n; j++) h[i * n + j] = (i == j ? 2.0 * n : 0.0) + 1.0 / (1 + i + j);
        }
        (void)hipMemcpy(bs, b.data(), n * 8, hipMemcpyHostToDevice);
        std::vector<double> yv[2];
        for (int v = 0; v < 2; v++) {
            long long best = 1ll << 60;
            for (int rep = 0; rep < 4; rep++) {
                (void)hipMemcpy(S, h.data(), n * n * 8, hipMemcpyHostToDevice);
                if (v == 0) hipLaunchKernelGGL(fbench<0>, dim3(1), dim3(kThreads), kFactorLds, 0, S, bs, y, dd, ctl, n, cyc);
                else hipLaunchKernelGGL(fbench<1>, dim3(1), dim3(kThreads), kFactorLds, 0, S, bs, y, dd, ctl, n, cyc);
                (void)hipDeviceSynchronize();
                long long cv = 0;
                (void)hipMemcpy(&cv, cyc, 8, hipMemcpyDeviceToHost);
                best = cv < best ? cv : best;
            }
            yv[v].resize(n);
            (void)hipMemcpy(yv[v].data(), y, n * 8, hipMemcpyDeviceToHost);
            std::printf("n %3d %-12s %8.1f us\n", n, v == 0 ? "factor_reg" : "factor_body", best * 0.01);
        }
        int diff = 0;
        for (int i = 0; i < n; i++) diff += yv[0][i] != yv[1][i];
        std::printf("n %3d solutions differing: %d\n", n, diff);
    }
    return 0;
}
