// Calibration of rocprofv3's FETCH_SIZE on gfx950 for narrow loads (is level_kernel's
// 3.1x read ratio halo re-reads or the blanket x2 correction?).  Three kernels stream the same 256 MiB buffer
// once, with 16, 4 and 1 byte(s) per lane per load, coalesced.  Run under `rocprofv3 --pmc FETCH_SIZE
// --kernel-trace`: the true fetch is 256 MiB per dispatch, so FETCH_SIZE / 256 MiB is the counter's scale for
// each load width.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_probe.bin tools/fetch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr size_t kBytes = 256ull << 20;
constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void probe16(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kThreads) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // (keeps the loads)
}
__global__ __launch_bounds__(kThreads) void probe4(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kThreads) acc ^= p[i];
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}
__global__ __launch_bounds__(kThreads) void probe1(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kThreads) acc += p[i];
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}
int main() {
    void* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    if (hipMemset(buf, 1, kBytes) != hipSuccess) return 1;
    const int grid = 2048;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(probe16, dim3(grid), dim3(kThreads), 0, 0, (const uint4*)buf, kBytes / 16, out);
        hipLaunchKernelGGL(probe4, dim3(grid), dim3(kThreads), 0, 0, (const uint32_t*)buf, kBytes / 4, out);
        hipLaunchKernelGGL(probe1, dim3(grid), dim3(kThreads), 0, 0, (const uint8_t*)buf, kBytes, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("fetch_probe: 3 kernels x 3, %zu bytes each\n", kBytes);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
