// First-use costs of the host-to-device paths a camera upload can take (one fresh process
// per mode): pageable hipMemcpy, pinned hipMemcpy, and a copy kernel reading mapped pinned
// memory. usage: dma_probe MODE BYTES  (MODE 0 pageable, 1 pinned, 2 kernel)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const size_t n = argc > 2 ? (size_t)atoll(argv[2]) : (400u << 10);
    double t = now_ms();
    void* d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess) return 1;
    (void)hipDeviceSynchronize();
    printf("init+malloc %.3f ms\n", now_ms() - t);
    std::vector<char> h(n, 1);
    for (int rep = 0; rep < 3; ++rep) {
        t = now_ms();
        if (mode == 0) {
            (void)hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice);
        } else {
            static void* p = nullptr;
            if (!p && hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return 2;
            const double t1 = now_ms();
            memcpy(p, h.data(), n);
            if (mode == 1) {
                (void)hipMemcpy(d, p, n, hipMemcpyHostToDevice);
            } else {
                hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, 0, (const uint4*)p, (uint4*)d, n / 16);
                (void)hipDeviceSynchronize();
            }
            if (rep == 0) printf("  (hostmalloc %.3f ms)\n", t1 - t);
        }
        printf("mode %d rep %d bytes %zu: %.3f ms\n", mode, rep, n, now_ms() - t);
    }
    return 0;
}
