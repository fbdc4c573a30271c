// sorted-path kernels for N <= 1024, 32 lanes per pixel (see stack_sorted_impl.h)
#include "stack_sorted_inst.h"
SGPU_DEFINE_SORTED_LAUNCHER(1024, 32, )
