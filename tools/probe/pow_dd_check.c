/* pow_spec (rt_device.hpp): the unnormalised double-double x^k against the renormalised one and glibc pow
 * over random (x, k); host-only check.  gcc -O2 -ffp-contract=off pow_dd_check.c -lm && ./a.out 50000000 */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static double pow_dd(double x, int k) {
    if (k == 0) return 1.0;
    int top = 31 - __builtin_clz(k);
    double h = x, l = 0.0;
    for (int i = top - 1; i >= 0; --i) {
        double p = h * h; double e = fma(h, h, -p); e = e + (2.0 * h) * l; h = p + e; l = e - (h - p);
        if ((k >> i) & 1) { p = h * x; e = fma(h, x, -p); e = e + l * x; h = p + e; l = e - (h - p); }
    }
    return h + l;
}
static double pow_un(double x, int k) {
    if (k == 0) return 1.0;
    int top = 31 - __builtin_clz(k);
    double h = x, l = 0.0;
    for (int i = top - 1; i >= 0; --i) {
        double p = h * h; double e = fma(h, h, -p); l = fma(h + h, l, e); h = p;
        if ((k >> i) & 1) { p = h * x; e = fma(h, x, -p); l = fma(l, x, e); h = p; }
    }
    return h + l;
}
static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 10000000;
    long diff = 0, diffg = 0, diffg0 = 0;
    for (long i = 0; i < n; ++i) {
        int k = (i & 1) ? (int)(rnd() % 1024) : (int)(1 + rnd() % 128);
        double x;
        uint64_t r = rnd();
        if (i % 3 == 0) x = (double)(r >> 11) * 0x1p-53;               /* [0,1) */
        else if (i % 3 == 1) x = 1.0 - (double)(r >> 11) * 0x1p-60;   /* near 1 */
        else { x = (double)(r >> 11) * 0x1p-53 * 4.0; }                /* [0,4) */
        double a = pow_dd(x, k), b = pow_un(x, k), g = pow(x, (double)k);
        if (memcmp(&a, &b, 8) && fabs(a) > 0x1p-1000) { if (diff < 10) printf("diff x=%a k=%d dd=%a un=%a g=%a\n", x, k, a, b, g); ++diff; }
        if (memcmp(&b, &g, 8)) ++diffg;
        if (memcmp(&a, &g, 8)) ++diffg0;
    }
    printf("n=%ld dd!=un %ld  un!=glibc %ld  dd!=glibc %ld\n", n, diff, diffg, diffg0);
    return 0;
}
