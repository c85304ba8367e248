// Microbenchmark: issue cost of f64 vs 64-bit integer vs f32 VALU ops on gfx950 (8 waves/SIMD, independent
// chains per lane so issue, not latency, bounds).  usage: ./issue_rates  -> ns per op per wave
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int N_ITER = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(double* out, uint64_t* outi, float* outf, double seed) {
    double a0 = seed + threadIdx.x, a1 = a0 * 1.5, a2 = a0 * 2.5, a3 = a0 * 3.5;
    const double b = 1e-9 * (1 + (threadIdx.x & 3));
    uint64_t i0 = (uint64_t)threadIdx.x * 977, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3;
    const uint64_t ib = 12345 + (threadIdx.x & 7);
    float f0 = (float)a0, f1 = f0 * 1.5f, f2 = f0 * 2.5f, f3 = f0 * 3.5f;
    const float fb = 1e-3f;
    uint32_t cnt = 0;
    for (int it = 0; it < N_ITER; it++) {
        if (OP == 0) { a0 += b; a1 += b; a2 += b; a3 += b; }                       // v_add_f64
        if (OP == 1) { i0 += ib; i1 += ib; i2 += ib; i3 += ib; }                   // 64-bit int add (2 ops)
        if (OP == 2) { f0 += fb; f1 += fb; f2 += fb; f3 += fb; }                   // v_add_f32
        if (OP == 3) { cnt += (a0 < a1) + (a1 < a2) + (a2 < a3) + (a3 < a0); a0 += b; }  // v_cmp_f64 (+1 add)
        if (OP == 4) { cnt += (i0 < i1) + (i1 < i2) + (i2 < i3) + (i3 < i0); i0 += ib; } // v_cmp_u64 (+int add)
        if (OP == 5) { a0 = __builtin_fma(b, a1, a0); a1 = __builtin_fma(b, a2, a1); a2 = __builtin_fma(b, a3, a2); a3 = __builtin_fma(b, a0, a3); }
        asm volatile("" :: "v"(a0), "v"(i0), "v"(f0));
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
    outi[blockIdx.x * 256 + threadIdx.x] = i0 + i1 + i2 + i3 + cnt;
    outf[blockIdx.x * 256 + threadIdx.x] = f0 + f1 + f2 + f3;
}

template <int OP>
float run(int blocks, double* o, uint64_t* oi, float* of) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, oi, of, 1.0);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, oi, of, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
    double* o;
    uint64_t* oi;
    float* of;
    hipMalloc(&o, blocks * 256 * 8);
    hipMalloc(&oi, blocks * 256 * 8);
    hipMalloc(&of, blocks * 256 * 4);
    const char* names[] = {"4x v_add_f64", "4x u64 add", "4x v_add_f32", "4x v_cmp_f64 + 1 add_f64", "4x v_cmp_u64 + 1 u64 add", "4x v_fma_f64"};
    float t[6] = {run<0>(blocks, o, oi, of), run<1>(blocks, o, oi, of), run<2>(blocks, o, oi, of), run<3>(blocks, o, oi, of),
                  run<4>(blocks, o, oi, of), run<5>(blocks, o, oi, of)};
    const double waves_per_simd = blocks * 4.0 / 1024.0;
    for (int i = 0; i < 6; i++) {
        // cycles per loop iteration per wave at 2.4 GHz, per SIMD: t / (N_ITER * waves_per_simd)
        printf("%-28s %8.3f ms  %6.2f SIMD-cycles per iteration per wave\n", names[i], t[i], t[i] * 1e-3 * 2.4e9 / (N_ITER * waves_per_simd));
    }
    return 0;
}
