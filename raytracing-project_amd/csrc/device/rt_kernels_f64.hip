// rt_kernels_f64.hip — the FP64 render kernels (namespace rtd): the parity
// path.  Device math follows the reference's double arithmetic step for step
// (DESIGN.md §Numerics).
#include "rt_device.hpp"
#include "rt_kernels.hpp"
