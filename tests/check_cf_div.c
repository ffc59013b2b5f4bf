/* Exhaustive check behind cf_per_kw (dgen_amd/csrc/dgen_hip.hip): for every
 * integer |x| <= 2e7, fma(fma(-q, 1e6, x), inv, q) with q = x * inv and
 * inv = RN(1 / 1e6) equals the IEEE quotient x / 1e6.  Prints the number of
 * mismatches (0 expected). */
#include <math.h>
#include <stdio.h>
int main(void) {
    const double inv = 1.0 / 1e6;
    long bad = 0;
    for (long x = -20000000; x <= 20000000; x++) {
        const double a = (double)x;
        const double q = a * inv;
        const double r = fma(-q, 1e6, a);
        if (fma(r, inv, q) != a / 1e6) bad++;
    }
    printf("%ld\n", bad);
    return 0;
}
