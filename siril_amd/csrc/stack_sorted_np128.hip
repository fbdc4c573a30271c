// sorted-path kernels for N <= 128, 4 lanes per pixel (see stack_sorted_impl.h)
#include "stack_sorted_inst.h"
#ifndef SGPU_G128
#define SGPU_G128 4
#endif
SGPU_DEFINE_SORTED_LAUNCHER(128, SGPU_G128, )
