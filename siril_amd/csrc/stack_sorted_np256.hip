// sorted-path kernels for N <= 256, 8 lanes per pixel (see stack_sorted_impl.h)
#include "stack_sorted_inst.h"
SGPU_DEFINE_SORTED_LAUNCHER(256, 8, )
