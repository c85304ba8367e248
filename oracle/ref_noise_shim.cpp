// ORACLE (test infrastructure only): a C entry point onto the reference's own OpenSimplex class,
// compiled together with /root/reference/include/OpenSimplexNoise.cpp into oracle/_ref/.
// Nothing here restates or replaces reference code; it only calls Noise(seed).eval(x, y).
#include "OpenSimplexNoise.h"
#include <cstdint>

extern "C" __attribute__((visibility("default"))) void ref_noise2_batch(int64_t seed, const double* x, const double* y, double* out,
                                                                        long n) {
    OpenSimplexNoise::Noise noise(seed);
    for (long i = 0; i < n; i++) out[i] = noise.eval(x[i], y[i]);
}
