// rt_kernels_big.hip — the FP64 general kernels again, with large per-lane
// stacks in scratch memory (namespace rtdb): scenes whose reflection /
// refraction recursion, transform nesting inside CSG operands or CSG operand
// depth exceed the common kernels' stacks (rt_launch.hpp kBig*) run here
// instead of being refused.  Same arithmetic as rt_kernels_f64.hip.
#define RT_REAL double
#define RT_NS rtdb
#define RT_BIG_STACKS 1
#define RT_GENERAL_ONLY 1
#include "rt_device.hpp"
#include "rt_kernels.hpp"
