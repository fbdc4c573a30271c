// sorted-path kernels for N <= 64, 2 lanes per pixel (see stack_sorted_impl.h)
#include "stack_sorted_inst.h"
SGPU_DEFINE_SORTED_LAUNCHER(64, 2, )
