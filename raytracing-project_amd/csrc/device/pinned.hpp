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

// hipMemcpyAsync H2D through the arena (pageable source if it has no room).
inline hipError_t upload_async(PinnedArena* a, void* dst, const void* src, size_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    const void* s = a ? a->put(src, n) : nullptr;
    return hipMemcpyAsync(dst, s ? s : src, n, hipMemcpyHostToDevice, st);
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
