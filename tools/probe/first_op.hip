// Probe (GPU box, diagnostic): the cost of a process's first GPU operations,
// each mode in a fresh process.  Which first operation pays the runtime's
// one-time setup (blit kernels, queues), and does a page-locked or
// kernel-side copy avoid it?  Usage: first_op <mode A..F>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_copy(const unsigned* __restrict__ src, unsigned* __restrict__ dst, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define T(label, expr)                                                                  \
    do {                                                                                \
        const double t0_ = now_ms();                                                    \
        hipError_t e_ = (expr);                                                         \
        std::printf("  %-34s %8.3f ms %s\n", label, now_ms() - t0_, e_ ? hipGetErrorString(e_) : ""); \
    } while (0)

int main(int argc, char** argv) {
    const char m = argc > 1 ? argv[1][0] : 'A';
    std::printf("mode %c\n", m);
    int n = 0;
    T("hipGetDeviceCount (init)", hipGetDeviceCount(&n));
    const int N = 1 << 18;   // 1 MiB
    std::vector<unsigned> h(N, 7u);
    unsigned *d = nullptr, *d2 = nullptr, *p = nullptr;
    hipStream_t st = nullptr;
    T("hipMalloc", hipMalloc(&d, N * 4));
    T("hipMalloc 2", hipMalloc(&d2, N * 4));
    T("hipStreamCreate", hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto launch = [&]() { hipLaunchKernelGGL(k_copy, dim3(64), dim3(256), 0, st, d, d2, N); return hipGetLastError(); };
    switch (m) {
        case 'A':   // pageable copy first
            T("memcpyAsync pageable (1st)", hipMemcpyAsync(d, h.data(), N * 4, hipMemcpyHostToDevice, st));
            T("sync", hipStreamSynchronize(st));
            T("memcpyAsync pageable (2nd)", hipMemcpyAsync(d, h.data(), N * 4, hipMemcpyHostToDevice, st));
            T("sync", hipStreamSynchronize(st));
            T("own kernel launch", launch());
            T("sync", hipStreamSynchronize(st));
            break;
        case 'B':   // own kernel first
            T("own kernel launch (1st)", launch());
            T("sync", hipStreamSynchronize(st));
            T("memcpyAsync pageable", hipMemcpyAsync(d, h.data(), N * 4, hipMemcpyHostToDevice, st));
            T("sync", hipStreamSynchronize(st));
            break;
        case 'C':   // page-locked copy first
            T("hipHostMalloc", hipHostMalloc(reinterpret_cast<void**>(&p), N * 4, hipHostMallocDefault));
            std::memcpy(p, h.data(), N * 4);
            T("memcpyAsync pinned (1st)", hipMemcpyAsync(d, p, N * 4, hipMemcpyHostToDevice, st));
            T("sync", hipStreamSynchronize(st));
            T("memcpyAsync pinned (2nd)", hipMemcpyAsync(d, p, N * 4, hipMemcpyHostToDevice, st));
            T("sync", hipStreamSynchronize(st));
            T("memcpyAsync pageable", hipMemcpyAsync(d, h.data(), N * 4, hipMemcpyHostToDevice, st));
            T("sync", hipStreamSynchronize(st));
            break;
        case 'D':   // own kernel reading page-locked host memory
            T("hipHostMalloc", hipHostMalloc(reinterpret_cast<void**>(&p), N * 4, hipHostMallocDefault));
            std::memcpy(p, h.data(), N * 4);
            {
                auto hl = [&]() { hipLaunchKernelGGL(k_copy, dim3(64), dim3(256), 0, st, p, d, N); return hipGetLastError(); };
                T("own copy kernel host->dev (1st)", hl());
            }
            T("sync", hipStreamSynchronize(st));
            T("memsetAsync", hipMemsetAsync(d2, 0, 4096, st));
            T("sync", hipStreamSynchronize(st));
            break;
        case 'E':   // memset first
            T("memsetAsync (1st)", hipMemsetAsync(d2, 0, 4096, st));
            T("sync", hipStreamSynchronize(st));
            T("own kernel launch", launch());
            T("sync", hipStreamSynchronize(st));
            break;
        case 'F':   // sync hipMemcpy pageable, large
        {
            std::vector<unsigned> big(4 * N, 3u);
            unsigned* db = nullptr;
            T("hipMalloc 4MiB", hipMalloc(&db, 16 * N));
            T("hipMemcpy pageable 4MiB (1st)", hipMemcpy(db, big.data(), 16 * N, hipMemcpyHostToDevice));
            T("hipMemcpy pageable 4MiB (2nd)", hipMemcpy(db, big.data(), 16 * N, hipMemcpyHostToDevice));
            break;
        }
    }
    return 0;
}
