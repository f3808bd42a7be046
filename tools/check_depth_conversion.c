// Exhaustive check of the kernels' u16 millimetre -> metres conversion against NumPy's
// astype(float)/1000. for every m in [0, 65535]: the kernels compute fma(m, C_HI, m * C_LO) with
// C_HI = RN(1/1000) = 0.001 and C_LO = RN(1/1000 - C_HI) (a two-term 1/1000: one multiply and one
// FMA).  The plain product m*0.001 is NOT exact, nor is the other association fma(m, C_LO, m*C_HI).
// gcc -O2 -ffp-contract=off tools/check_depth_conversion.c -lm && ./a.out
#include <math.h>
#include <stdio.h>
int main() {
    const double c_hi = 0.001, c_lo = -2.0858186326137145e-20;
    const long double lo_exact = 1.0L / 1000.0L - (long double)c_hi;
    int bad_mul = 0, bad_two = 0, bad_swap = 0;
    for (int m = 0; m < 65536; m++) {
        const double ref = (double)m / 1000.0, dm = (double)m;
        if (dm * c_hi != ref) bad_mul++;
        if (fma(dm, c_hi, dm * c_lo) != ref) bad_two++;
        if (fma(dm, c_lo, dm * c_hi) != ref) bad_swap++;
    }
    printf("C_LO %s RN(1/1000 - C_HI)\n", (double)lo_exact == c_lo ? "==" : "!=");
    printf("mul-only mismatches %d, two-term mismatches %d, swapped mismatches %d\n", bad_mul, bad_two, bad_swap);
    return 0;
}
