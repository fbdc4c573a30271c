// sorted-path kernels for N <= 16, one lane per pixel (see stack_sorted_impl.h)
#include "stack_sorted_inst.h"
SGPU_DEFINE_SORTED_LAUNCHER(16, 1, SGPU_LAUNCH_CASE(16, 1, LINEARFIT) SGPU_LAUNCH_CASE(16, 1, GESDT))
