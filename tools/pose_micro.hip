// Diagnostic micro-benchmark (not part of the library): latency of the PoseOptimization building blocks on
// gfx950 -- one evaluation per lane, each fed from the previous one's result (a dependent chain), one wave per
// SIMD, cycles from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I sp-slam_amd/csrc -o /tmp/pose_micro tools/pose_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "g2o_device.h"

using namespace spslam;
using namespace spslam::g2od;

constexpr int kIt = 64;

template <int kOp>
__global__ void bench(double* out, long long* cyc, int kind) {
    const int l = threadIdx.x & 63;
    double a = 0.1 + 1e-3 * l, acc = 0;
    SE3 T{Q{0.99, 0.05, 0.07, 0.02}, V3{0.1, -0.2, 0.3}};
    q_normalize(T.r);
    const P4 w{{0.3, 0.5, 0.81, 1.5}}, m{{0.31, 0.49, 0.81, 1.2}};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIt; i++) {
        if (kOp == 0) {  // plane error, inlined
            T.t.x = a;
            const E3 e = plane_error3(kind, T, w, m);
            a = 0.1 + 1e-9 * (e.e0 + e.e1 + e.e2);
        } else if (kOp == 1) {  // plane error, out of line
            T.t.x = a;
            const E3 e = plane_error_call(kind, T, w, m);
            a = 0.1 + 1e-9 * (e.e0 + e.e1 + e.e2);
        } else if (kOp == 2) {  // one correctly rounded atan2
            a = 0.5 + 1e-9 * lm::atan2_(a, 0.7);
        } else if (kOp == 3) {  // two side by side
            double r0, r1;
            lm::atan2x2_(a, 0.7, 0.3, a, &r0, &r1);
            a = 0.5 + 1e-9 * (r0 + r1);
        } else if (kOp == 4) {  // one sincos
            double s, c;
            lm::sincos_(a, &s, &c);
            a = 0.5 + 1e-9 * (s + c);
        } else if (kOp == 5) {  // two side by side
            double s0, c0, s1, c1;
            lm::sincos2_(a, a + 0.25, &s0, &c0, &s1, &c1);
            a = 0.5 + 1e-9 * (s0 + c1);
        } else if (kOp == 6) {  // SE3Quat::exp
            const double u[6] = {a * 1e-3, 2e-3, -1e-3, 0.01, a * 0.01, 0.0};
            const SE3 E = se3_exp(u);
            a = 0.5 + 1e-9 * (E.r.w + E.t.y);
        } else if (kOp == 7) {  // exp(u) * T
            const double u[6] = {a * 1e-3, 2e-3, -1e-3, 0.01, a * 0.01, 0.0};
            const SE3 E = se3_mul(se3_exp(u), T);
            a = 0.5 + 1e-9 * (E.r.w + E.t.y);
        } else if (kOp == 8) {  // point projection error (mono), the pose kernel's expression
            const V3 p = q_rot(T.r, V3{a, 0.2, 2.0}) + T.t;
            const double e0 = 300.0 - (p.x / p.z * 500.0 + 320.0), e1 = 200.0 - (p.y / p.z * 500.0 + 240.0);
            a = 0.1 + 1e-9 * (e0 + e1);
        } else {  // quaternion normalisation (sqrt + 4 divisions)
            Q q{a, 0.1, 0.2, 0.3};
            q_normalize(q);
            a = 0.5 + 1e-3 * q.x;
        }
        acc += a;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}


// The ordered chain of the pose kernel: rows of kStride doubles in LDS, lane = column, 478 rows, one call
template <int kStride>
__device__ __forceinline__ void chain_seg(double& acc, const double* p, int cnt) {
    auto ld = [&](double (&v)[8], int i) __attribute__((always_inline)) {
        const double* q = p + i * kStride;
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = q[k * kStride];
    };
    auto add = [&](const double (&v)[8], int n) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k < n) acc += v[k];
    };
    const int full = cnt - cnt % 24;
    double a[8], b[8], c[8];
    ld(a, 0);
    ld(b, 8);
    ld(c, 16);
    for (int i = 0; i < full; i += 24) {
        add(a, 8);
        ld(a, i + 24);
        __builtin_amdgcn_sched_barrier(0);
        add(b, 8);
        ld(b, i + 32);
        __builtin_amdgcn_sched_barrier(0);
        add(c, 8);
        ld(c, i + 40);
        __builtin_amdgcn_sched_barrier(0);
    }
    const int r = cnt - full;
    add(a, r);
    add(b, r - 8);
    add(c, r - 16);
}
__global__ void chain_bench(double* out, long long* cyc, int rows, int nchain_waves) {
    __shared__ double ring[(512 + 48) * 29];
    for (int i = threadIdx.x; i < (512 + 48) * 29; i += blockDim.x) ring[i] = 1e-3 * (i % 97);
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double acc = 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (w < nchain_waves) {
        for (int rep = 0; rep < 8; rep++) chain_seg<29>(acc, ring + (lane < 28 ? lane : 28), rows);
    } else {  // a competing fp64 stream on the other waves
        double x = acc + lane;
        for (int i = 0; i < 4096; i++) x = fma(x, 0.999, 1e-3);
        acc = x;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double* d_out;
    long long* d_cyc;
    (void)hipMalloc(&d_out, 1 << 20);
    (void)hipMalloc(&d_cyc, 1 << 12);
    const char* names[] = {"plane_error inline", "plane_error call", "atan2 x1", "atan2 x2", "sincos x1",
                           "sincos x2", "se3_exp", "exp(u)*T", "point error", "q_normalize"};
    for (int op = 0; op < 10; op++)
        for (int kind = 0; kind < (op < 2 ? 3 : 1); kind++) {
            auto launch = [&] {
                const dim3 g(1), b(64);
                switch (op) {
                    case 0: hipLaunchKernelGGL(bench<0>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 1: hipLaunchKernelGGL(bench<1>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 2: hipLaunchKernelGGL(bench<2>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 3: hipLaunchKernelGGL(bench<3>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 4: hipLaunchKernelGGL(bench<4>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 5: hipLaunchKernelGGL(bench<5>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 6: hipLaunchKernelGGL(bench<6>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 7: hipLaunchKernelGGL(bench<7>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    case 8: hipLaunchKernelGGL(bench<8>, g, b, 0, 0, d_out, d_cyc, kind); break;
                    default: hipLaunchKernelGGL(bench<9>, g, b, 0, 0, d_out, d_cyc, kind); break;
                }
            };
            launch();
            (void)hipDeviceSynchronize();
            launch();
            long long c = 0;
            (void)hipMemcpy(&c, d_cyc, sizeof c, hipMemcpyDeviceToHost);
            std::printf("%-20s kind %d: %8.0f cycles per evaluation\n", names[op], kind, (double)c / kIt);
        }
    for (int cfg = 0; cfg < 4; cfg++) {
        const int threads = cfg == 0 ? 64 : cfg == 1 ? 256 : cfg == 2 ? 320 : 512, chainers = cfg == 1 ? 4 : 1;
        hipLaunchKernelGGL(chain_bench, dim3(1), dim3(threads), 0, 0, d_out, d_cyc, 478, chainers);
        (void)hipDeviceSynchronize();
        hipLaunchKernelGGL(chain_bench, dim3(1), dim3(threads), 0, 0, d_out, d_cyc, 478, chainers);
        long long c = 0;
        (void)hipMemcpy(&c, d_cyc, sizeof c, hipMemcpyDeviceToHost);
        std::printf("chain 478 rows x 28 cols, %d threads (%d chaining waves, the rest fp64 fma): %.1f cycles per row\n",
                    threads, chainers, (double)c / (8 * 478));
    }
    return 0;
}
