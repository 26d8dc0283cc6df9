// Probe (GPU box, diagnostic): what a DPP row_ror read returns for a source
// lane that is disabled by EXEC (gfx950).  Prints, per active lane, the value
// read from lane (i+1)%16 of its row; the source's own value is 1000 + lane,
// and 7777 is what disabled lanes hold from an earlier full-exec write.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(int* out, int pattern) {
    const int lane = threadIdx.x;
    int v = 7777;
    asm volatile("v_mov_b32 %0, 7777" : "=v"(v));   // every lane
    int r = -1;
    const bool on = pattern == 0 ? (lane % 3 == 0) : (lane % 2 == 0);
    if (on) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(1000 + lane));
        r = __builtin_amdgcn_update_dpp(0, v, 0x121, 0xf, 0xf, true);   // row_ror:1, bound_ctrl
        out[lane] = r;
        out[64 + lane] = __builtin_amdgcn_update_dpp(0, v, 0x121, 0xf, 0xf, false);
    }
}

int main() {
    int* d;
    hipMalloc(&d, 128 * sizeof(int));
    for (int p = 0; p < 2; ++p) {
        hipMemset(d, 0xff, 128 * sizeof(int));
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, p);
        int h[128];
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("pattern %d\n", p);
        for (int i = 0; i < 64; ++i)
            if (h[i] != -1) printf("lane %2d src %2d : bound=%d nobound=%d\n", i, (i & ~15) | ((i + 15) & 15), h[i], h[64 + i]);
    }
    hipFree(d);
    return 0;
}
