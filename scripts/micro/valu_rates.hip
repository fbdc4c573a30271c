// Microbenchmark: issue cost of the VALU instructions of the stack kernel's
// inner loops on gfx950 (v_cvt_f64_f32, v_add_f64, v_med3_f32, v_pk_add_f32,
// v_add_u32), 8 independent chains per lane, occupancy W waves per SIMD.
// Prints cycles per wave-instruction per SIMD (clock from s_memrealtime is
// not needed: we report ns per wave-instruction per SIMD and the ratio).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define ITERS 4096
template <int OP>
__global__ __launch_bounds__(256) void k(float *out, float a, float b) {
    float f[8];
    double d[8];
    unsigned u[8];
    for (int i = 0; i < 8; i++) { f[i] = a + threadIdx.x * 1e-7f + i; d[i] = f[i]; u[i] = threadIdx.x + i; }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (OP == 0) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[i]) : "v"(f[i]));
            if constexpr (OP == 1) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
            if constexpr (OP == 2) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(a), "v"(b));
            if constexpr (OP == 3) { typedef float f2 __attribute__((ext_vector_type(2))); f2 x = {f[i], f[(i+1)&7]}; asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(x)); f[i] = x.x + 0.f; }
            if constexpr (OP == 4) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            if constexpr (OP == 5) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(f[(i + 1) & 7]));
            if constexpr (OP == 6) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[i]) : "v"(d[i]));
            if constexpr (OP == 7) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
        }
    }
    float s = 0.f;
    for (int i = 0; i < 8; i++) s += f[i] + (float)d[i] + (float)u[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int OP> float run(int blocks) {
    float *o; hipMalloc(&o, 1024 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, 1.f, 2.f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, 1.f, 2.f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipFree(o);
    // wave-instructions issued per SIMD: blocks*4 waves * ITERS*8 / 1024 SIMDs, per launch
    double wi = (double)blocks * 4 * ITERS * 8 / 1024.0;
    return (float)(ms / 5 * 1e6 / wi);   // ns per wave-instruction per SIMD
}

int main() {
    const char *names[] = {"v_cvt_f64_f32", "v_add_f64", "v_med3_f32", "v_pk_add_f32(+v_add)", "v_add_u32", "v_add_f32", "v_cvt_f32_f64", "v_fma_f64"};
    for (int w : {1, 2, 4, 8}) {
        int blocks = 256 * w;   // w waves per SIMD (4 waves per block, 1 block per CU per w)
        float r[8] = {run<0>(blocks), run<1>(blocks), run<2>(blocks), run<3>(blocks), run<4>(blocks), run<5>(blocks), run<6>(blocks), run<7>(blocks)};
        for (int i = 0; i < 8; i++) printf("waves/SIMD %d  %-22s %.3f ns/wave-inst/SIMD (= %.2f cycles @2.4GHz)\n", w, names[i], r[i], r[i] * 2.4);
    }
    return 0;
}
