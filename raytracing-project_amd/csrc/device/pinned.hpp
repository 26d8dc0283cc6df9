// pinned.hpp — page-locked host staging for a frame's small uploads.
//
// hipMemcpyAsync from pageable host memory goes through the runtime's own
// staging and can hold the calling thread until the copy has run in stream
// order: a rank of a split frame then enqueues its next row chunk only after
// the previous chunk's work reached the copy (profiles/r04i_*: 40-110 us
// holes between a rank's launches).  From page-locked memory the copy is a
// plain DMA descriptor and the call returns at once.  One arena per device
// workspace; a frame bump-allocates its uploads (rows, jitter job, paper
// lists) and the next frame reuses them: rt_frame_end has synchronised every
// stream the frame used before the workspace lock is released.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>
#include <utility>
#include <vector>

#include "rt_internal.hpp"

namespace rtamd {

struct PinnedArena {
    char* p = nullptr;
    size_t cap = 0, used = 0;
    std::vector<char*> old;   // outgrown blocks of the current frame (freed at the next reset)

    void reset() {
        for (char* b : old) (void)hipHostFree(b);
        old.clear();
        used = 0;
    }
    // A page-locked copy of src[0, n), or nullptr if no page-locked memory
    // could be had (the caller then copies from src itself).
    void* put(const void* src, size_t n) {
        const size_t need = (n + 255) & ~(size_t)255;
        if (used + need > cap) {
            if (p) old.push_back(p);
            cap = std::max<size_t>({2 * cap, need, (size_t)1 << 16});
            p = nullptr;
            used = 0;
            SetupTimer tm(kSetupPinned);
            if (hipHostMalloc(reinterpret_cast<void**>(&p), cap, hipHostMallocDefault) != hipSuccess) {
                p = nullptr;
                cap = 0;
                return nullptr;
            }
        }
        char* d = p + used;
        if (n) std::memcpy(d, src, n);
        used += need;
        return d;
    }
    void release() {
        reset();
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// dst[0, n) <- page-locked src[0, n) by a kernel on st (k_host_copy,
// rt_render.hip: the GPU reads the host memory over PCIe).  Both pointers
// 16-byte aligned, else hipMemcpyAsync.  A process's first copy-engine
// transfer costs ~8 ms of host time in the runtime (profiles/
// r06d_first_op.txt: pageable or page-locked alike; a kernel's own first
// launch ~0.3 ms), so a frame's uploads never use the copy engines.
hipError_t host_copy_async(void* dst, const void* src_pinned, size_t n, hipStream_t st);
// Once per process: a 1 MiB device-to-host read-back into pageable memory on
// st, so that the runtime's one-time set-up of that path (~8 ms of host time
// in the call, profiles/r06d_first_op.txt) runs while the frame's first trace
// executes instead of in front of the frame's read-back.
hipError_t warm_copy_engine(hipStream_t st);

// H2D through the arena: page-locked staging + k_host_copy (pageable
// hipMemcpyAsync if the arena has no room).
inline hipError_t upload_async(PinnedArena* a, void* dst, const void* src, size_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    const void* s = a ? a->put(src, n) : nullptr;
    if (s) return host_copy_async(dst, s, n, st);
    return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
}

// Wait for an event by polling it (yielding the core between polls; after
// ~20 ms, 50 us sleeps).  A blocking wait - the pageable counter copy
// rt_frame_end used to make - resumed the host ~115 us after the GPU had
// finished (profiles/r04t_api_timeline.txt): 1-2 % of an 8 ms frame, 10 % of
// a 1 ms rank share.
inline hipError_t spin_wait(hipEvent_t ev) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q != hipErrorNotReady) return q;
        if (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20))
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

}  // namespace rtamd
