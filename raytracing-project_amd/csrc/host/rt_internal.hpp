// rt_internal.hpp — helpers shared between librt_host and librtamd.
#pragma once

#include <chrono>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "rt.h"

namespace rtamd {
void set_last_error(const std::string& msg);
void clear_last_error();
bool validate_desc(const rt_scene_desc& d, std::string* why);
bool node_depth_ok(const rt_scene_desc& d, int idx, int level, int* maxdepth);
// Process-unique id of a scene handle (scenes are immutable after creation,
// so a device copy keyed by it never goes stale).
uint64_t scene_uid(const rt_scene* s);
// librtamd: free every per-device workspace of slot >= min_slot (rt_shutdown:
// all of them); returns an rt_status.
int release_device_workspaces(int min_slot = 0);
// librtamd: `chunks` contiguous pieces of [0, m), each a whole number of
// strips of S rows, of decreasing size (weights chunks, chunks-1, ..., 1:
// 4 chunks = 40/30/20/10 %).
std::vector<std::pair<int, int>> row_chunks(int m, int chunks, int S = 1);
// librtamd: row chunks of a one-GPU paper frame (RT_PAPER_CHUNKS_1GPU, default 4).
int paper_chunks_1gpu();
// librtamd: host costs reported by rt_setup_times.  Slots 4..6 accumulate
// over the process (device allocations, page-locked allocations, stream /
// event creation; scope timers around those calls); slots 7..10 hold the last
// frame's host split (rt_frame_begin, the rt_frame_trace calls, rt_frame_end
// including its wait for the device, and rt_render_multi's own setup before
// its frame: device group, output buffer).
enum {
    kSetupAlloc = 4, kSetupPinned = 5, kSetupStreams = 6,
    kLastBegin = 7, kLastTrace = 8, kLastEnd = 9, kLastGroup = 10, kSetupCopyEngine = 11, kSetupSlots = 12
};
void note_setup_ms(int slot, double ms);   // slots 4..6: add; 7..10: set (kLastTrace adds within a frame)
struct SetupTimer {
    int slot;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit SetupTimer(int s) : slot(s) {}
    ~SetupTimer() {
        note_setup_ms(slot, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};
// librtamd: the workspace slot of the calling thread's frames (0: the
// process's own; rt_test_dist_threads gives each simulated rank its own).
void set_workspace_slot(int slot);
// librtamd: rt_frame_trace of a paper-mode FP64 frame that writes one
// paper-code byte per pixel (rtamd::paper_code_value) instead of FP64 rows:
// the distributed frame's gather payload (rt_dist.hip).
int frame_trace_paper_codes(rt_frame* f, int ri0, int ri1, uint8_t* codes_rows_dev, void* hip_stream);

}  // namespace rtamd
