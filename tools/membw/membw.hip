// HBM write / read / copy bandwidth on the GPU box (diagnostic for the
// headline's roofline: the bench step writes ~224 MB and reads ~150 MB).
// hipcc --offload-arch=gfx950 -O3 -o membw membw.hip && ./membw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void k_write(u32x4* dst, size_t n, int iters) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
        if (NT) __builtin_nontemporal_store(v, &dst[i]);
        else dst[i] = v;
    }
}
__global__ void k_read(const u32x4* src, size_t n, uint32_t* sink) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const u32x4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
template <bool NT>
__global__ void k_copy(const u32x4* src, u32x4* dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const u32x4 v = src[i];
        if (NT) __builtin_nontemporal_store(v, &dst[i]);
        else dst[i] = v;
    }
}

int main() {
    const size_t bytes = 1ull << 30, n = bytes / 16;
    u32x4 *a, *b;
    uint32_t* sink;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&sink, 4);
    hipMemset(a, 1, bytes);
    hipMemset(b, 2, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grids[] = {1024, 4096, 16384};
    for (int gi = 0; gi < 3; gi++) {
        const int grid = grids[gi];
        for (int rep = 0; rep < 2; rep++) {
            float ms;
            hipEventRecord(e0);
            for (int k = 0; k < 10; k++) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, a, n, 1);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            const double w_nt = 10.0 * bytes / (ms * 1e-3) / 1e12;
            hipEventRecord(e0);
            for (int k = 0; k < 10; k++) hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, a, n, 1);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            const double w = 10.0 * bytes / (ms * 1e-3) / 1e12;
            hipEventRecord(e0);
            for (int k = 0; k < 10; k++) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            const double r = 10.0 * bytes / (ms * 1e-3) / 1e12;
            hipEventRecord(e0);
            for (int k = 0; k < 10; k++) hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), 0, 0, a, b, n);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            const double c = 10.0 * 2 * bytes / (ms * 1e-3) / 1e12;
            printf("grid %5d: write NT %.2f TB/s, write %.2f TB/s, read %.2f TB/s, copy NT (r+w) %.2f TB/s\n", grid, w_nt, w, r, c);
        }
    }
    // the headline's sizes: 150 MB of writes per launch, repeated
    const size_t n2 = (150ull << 20) / 16;
    float ms;
    hipEventRecord(e0);
    for (int k = 0; k < 100; k++) hipLaunchKernelGGL(k_write<true>, dim3(4096), dim3(256), 0, 0, a, n2, 1);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("150 MB NT write: %.1f us per launch = %.2f TB/s\n", ms * 10.0, 100.0 * n2 * 16 / (ms * 1e-3) / 1e12);
    return 0;
}
