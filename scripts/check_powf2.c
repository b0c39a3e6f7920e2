/* Exhaustive host check of walker_gym_amd/csrc/powf2.h against the image's libm powf (tests/test_powf2.py):
 * for every non-negative finite float32 x (and its negation), pw_pow2(x) must equal powf(x, 2.0f) bit for bit, and
 * whenever pw_pow2_fast(x) claims RN(x*x) it must equal powf(x, 2.0f) too.  powf is called through a volatile
 * function pointer: compilers fold powf(x, 2.0f) into x*x, which is exactly what numpy does NOT get.
 * Build: gcc -O2 -fopenmp -ffp-contract=off -fno-builtin -I walker_gym_amd/csrc scripts/check_powf2.c -lm */
#include <stdio.h>
#include <stdlib.h>
#include "powf2.h"

typedef float (*powf_fn)(float, float);

int main(int argc, char **argv) {
    unsigned long long step = argc > 1 ? strtoull(argv[1], 0, 0) : 1;   /* 1 = every float */
    volatile powf_fn P = powf;
    powf_fn pf = P;
    unsigned long long bad = 0, bad_fast = 0, slow = 0, n = 0;
    unsigned int first = 0;
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : bad, bad_fast, slow, n)
    for (long long u = 0; u < 0x7f800000ll; u += (long long)step) {
        for (int sgn = 0; sgn < 2; sgn++) {
            const float x = pw_asfloat((unsigned int)u | (sgn ? 0x80000000u : 0u));
            const float ref = pf(x, 2.0f), emu = pw_pow2(x);
            float f;
            n++;
            if (pw_asu32(ref) != pw_asu32(emu)) {
                bad++;
#pragma omp critical
                if (!first) first = (unsigned int)u;
            }
            if (pw_pow2_fast(x, &f)) {
                if (pw_asu32(f) != pw_asu32(ref)) bad_fast++;
            } else {
                slow++;
            }
        }
    }
    printf("{\"inputs\": %llu, \"mismatch\": %llu, \"fast_mismatch\": %llu, \"slow_path\": %llu, \"first_bad\": %u}\n",
           n, bad, bad_fast, slow, first);
    return (bad || bad_fast) ? 1 : 0;
}
