// rt_kernels_f64.hip — the FP64 render kernels (namespace rtd): the parity
// path.  Device math follows the reference's double arithmetic step for step
// (DESIGN.md §Numerics).
#include "rt_device.hpp"
#include "rt_kernels.hpp"
#include "rt_test.h"

// ------------------------------------------------------------- test hook
// div3 (rt_device.hpp) against the compiler's own division on the device:
// out_div3[3i+k] = div3(a[3i..3i+2], b[i])[k], out_plain[3i+k] = a[3i+k] / b[i].
namespace {
__global__ void k_test_div3(const double* a, const double* b, int n, double* o3, double* op) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rtd::D3 q = rtd::div3(a[3 * i], a[3 * i + 1], a[3 * i + 2], b[i]);
    o3[3 * i] = q.x;
    o3[3 * i + 1] = q.y;
    o3[3 * i + 2] = q.z;
    op[3 * i] = a[3 * i] / b[i];
    op[3 * i + 1] = a[3 * i + 1] / b[i];
    op[3 * i + 2] = a[3 * i + 2] / b[i];
}
}  // namespace

extern "C" int rt_test_div3(const double* a_host, const double* b_host, int n, double* div3_host, double* plain_host) {
    if (n <= 0 || !a_host || !b_host || !div3_host || !plain_host) return RT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    double *a = nullptr, *b = nullptr, *o3 = nullptr, *op = nullptr;
    const size_t n3 = (size_t)n * 3 * sizeof(double);
    int rc = RT_OK;
    if (hipMalloc(&a, n3) != hipSuccess || hipMalloc(&b, (size_t)n * sizeof(double)) != hipSuccess ||
        hipMalloc(&o3, n3) != hipSuccess || hipMalloc(&op, n3) != hipSuccess)
        rc = RT_ERR_HIP;
    if (rc == RT_OK && (hipMemcpy(a, a_host, n3, hipMemcpyHostToDevice) != hipSuccess ||
                        hipMemcpy(b, b_host, (size_t)n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess))
        rc = RT_ERR_HIP;
    if (rc == RT_OK) {
        hipLaunchKernelGGL(k_test_div3, dim3((n + 255) / 256), dim3(256), 0, nullptr, a, b, n, o3, op);
        if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(div3_host, o3, n3, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(plain_host, op, n3, hipMemcpyDeviceToHost) != hipSuccess)
            rc = RT_ERR_HIP;
    }
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (o3) (void)hipFree(o3);
    if (op) (void)hipFree(op);
    return rc;
}
