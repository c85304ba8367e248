// Exhaustive check: is v_rcp_f32 + one FMA Newton step (e = fma(-x, r, 1), r' = fma(e, r, r)) the
// correctly rounded f32 reciprocal, i.e. (float)(1.0 / (double)x), for every positive normal x whose
// reciprocal is normal (both signs)?  One count per block (no atomics); the host sums.  usage: ./rcp_check
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

__global__ __launch_bounds__(256) void k(uint32_t lo, uint32_t n, uint32_t* bad, uint32_t* first) {
    __shared__ uint32_t cnt[256], fst[256];
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    uint32_t b = 0u, f = 0xFFFFFFFFu;
    if (i < n) {
        const uint32_t u = lo + i;  // (lo may carry the sign bit)
        const float x = __uint_as_float(u);
        const float r0 = __builtin_amdgcn_rcpf(x);
        const float e = __builtin_fmaf(-x, r0, 1.0f);
        const float r1 = __builtin_fmaf(e, r0, r0);
        const float ref = (float)(1.0 / (double)x);
        if (__float_as_uint(r1) != __float_as_uint(ref)) { b = 1u; f = u; }
    }
    cnt[threadIdx.x] = b;
    fst[threadIdx.x] = f;
    __syncthreads();
    for (uint32_t s = 128u; s > 0u; s >>= 1) {
        if (threadIdx.x < s) {
            cnt[threadIdx.x] += cnt[threadIdx.x + s];
            fst[threadIdx.x] = min(fst[threadIdx.x], fst[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        bad[blockIdx.x] = cnt[0];
        first[blockIdx.x] = fst[0];
    }
}

int main() {
    const uint32_t lo = 0x00800000u, hi = 0x7E800000u;  // x normal and 1/x normal (x < 2^126)
    const uint32_t chunk = 1u << 26, nb = chunk / 256u;
    uint32_t *dbad, *dfirst;
    hipMalloc(&dbad, nb * 4);
    hipMalloc(&dfirst, nb * 4);
    uint32_t* hbad = (uint32_t*)malloc(nb * 4);
    uint32_t* hfirst = (uint32_t*)malloc(nb * 4);
    uint64_t total = 0, checked = 0;
    uint32_t firsts[8];
    int nf = 0;
    for (uint32_t sign = 0u; sign <= 0x80000000u; sign += 0x80000000u) {
        for (uint64_t s = lo; s < hi; s += chunk) {
            const uint32_t n = (uint32_t)((hi - s) < chunk ? (hi - s) : chunk);
            hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, (uint32_t)s | sign, n, dbad, dfirst);
            hipMemcpy(hbad, dbad, ((n + 255) / 256) * 4, hipMemcpyDeviceToHost);
            hipMemcpy(hfirst, dfirst, ((n + 255) / 256) * 4, hipMemcpyDeviceToHost);
            for (uint32_t j = 0; j < (n + 255) / 256; j++) {
                total += hbad[j];
                if (hbad[j] && nf < 8) firsts[nf++] = hfirst[j];
            }
            checked += n;
        }
        if (sign) break;
    }
    printf("checked %llu floats, mismatches %llu\n", (unsigned long long)checked, (unsigned long long)total);
    for (int i = 0; i < nf; i++) printf("  e.g. x = 0x%08x (%g)\n", firsts[i], (double)*(float*)&firsts[i]);
    return 0;
}
