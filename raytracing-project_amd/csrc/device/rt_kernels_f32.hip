// rt_kernels_f32.hip — the FP32 render kernels (namespace rtf), selected by
// RT_FLAG_FP32: SURVEY.md §8f row 3, the optional non-parity fast path.  The
// algorithm, op order and culling are the FP64 path's; only the arithmetic
// type of the scene records and the trace differs.
#define RT_REAL float
#define RT_NS rtf
#define RT_NO_PLAIN   // (no plain kernel variants in the FP32 diagnostic build)
#include "rt_device.hpp"
#include "rt_kernels.hpp"
