// Diagnostic micro-benchmark (not part of the library): dependent-chain latency of the fp64 operations the
// PoseOptimization chains are made of, one wave (and two waves) per SIMD, measured with s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -o build/f64_latency tools/f64_latency.hip && build/f64_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 4096;

template <int kOp>
__global__ void chain(double* out, long long* cyc, double a, double b) {
    double x = a + threadIdx.x * 1e-12, y = b;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < kN; i++) {
        if (kOp == 0) x = x + y;                // v_add_f64
        else if (kOp == 1) x = fma(x, y, 1e-3); // v_fma_f64
        else if (kOp == 2) x = x * y;           // v_mul_f64
        else if (kOp == 3) x = 1.0 / (x + 2.0); // division (v_div_scale / rcp / fma / fmas / fixup) + add
        else if (kOp == 4) x = sqrt(x + 1.0);   // v_sqrt_f64 + add
        else x = x + y * 1e-30;                 // mul + add, the add depends on x
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    double* d_out;
    long long* d_cyc;
    hipMalloc(&d_out, 1 << 20);
    hipMalloc(&d_cyc, 1 << 12);
    const char* names[] = {"v_add_f64", "v_fma_f64", "v_mul_f64", "div+add", "sqrt+add", "mul+add"};
    for (int waves : {1, 4, 8}) {
        for (int op = 0; op < 6; op++) {
            auto launch = [&] {
                const dim3 g(1), b(64 * waves);
                switch (op) {
                    case 0: hipLaunchKernelGGL(chain<0>, g, b, 0, 0, d_out, d_cyc, 1.0, 1e-9); break;
                    case 1: hipLaunchKernelGGL(chain<1>, g, b, 0, 0, d_out, d_cyc, 1.0, 0.999); break;
                    case 2: hipLaunchKernelGGL(chain<2>, g, b, 0, 0, d_out, d_cyc, 1.0, 1.0000001); break;
                    case 3: hipLaunchKernelGGL(chain<3>, g, b, 0, 0, d_out, d_cyc, 1.0, 0.0); break;
                    case 4: hipLaunchKernelGGL(chain<4>, g, b, 0, 0, d_out, d_cyc, 1.0, 0.0); break;
                    default: hipLaunchKernelGGL(chain<5>, g, b, 0, 0, d_out, d_cyc, 1.0, 1.0); break;
                }
            };
            launch();
            hipDeviceSynchronize();
            launch();
            long long c = 0;
            hipMemcpy(&c, d_cyc, sizeof c, hipMemcpyDeviceToHost);
            std::printf("%-10s waves/WG %d: %.1f cycles per dependent step (s_memtime)\n", names[op], waves,
                        (double)c / kN);
        }
    }
    return 0;
}
