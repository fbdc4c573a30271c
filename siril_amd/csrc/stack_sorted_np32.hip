// sorted-path kernels for N <= 32, one lane per pixel (see stack_sorted_impl.h)
#include "stack_sorted_inst.h"
SGPU_DEFINE_SORTED_LAUNCHER(32, 1, SGPU_LAUNCH_CASE(32, 1, LINEARFIT) SGPU_LAUNCH_CASE(32, 1, GESDT))
