/* check_fastdiv.c -- CPU evidence for the exact short sequences used by the
 * two-column stream kernel (lbm-graphcore_amd/csrc/lbm_stream2.hip).
 *
 * 1. x / d for d = 9, 36 (D2Q9) and 3, 18 (D3Q19): q = RN(x*y), r = fma(-d, q, x), q' = fma(r, y, q),
 *    y = RN(1/d).  Checked against IEEE x / d for EVERY float x in 41
 *    binades [2^-20, 2^21) -- the check depends only on the significand while
 *    no result is subnormal, so this covers every normal x of interest.
 * 2. n / d with the LLVM AMDGPU IEEE expansion minus v_div_scale/v_div_fixup:
 *    r = rcp(d); e = fma(-d, r, 1); r = fma(e, r, r); q = n*r;
 *    q = fma(fma(-d, q, n), r, q); q = fma(fma(-d, q, n), r, q).
 *    v_rcp_f32 is accurate to 1 ulp; each random (n, d) pair is checked with
 *    the three candidates RN(1/d) - 1 ulp, RN(1/d), RN(1/d) + 1 ulp.
 * Build: gcc -O2 -ffp-contract=off -mfma check_fastdiv.c -lm
 * Exit status 0 iff no mismatch.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t rs = 88172645463325252ull;
static uint64_t xr(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }

static float div_const(float x, float d, float y) {
    float q = x * y;
    float r = fmaf(-d, q, x);
    return fmaf(r, y, q);
}

static float div_seq(float n, float d, float r0) {
    float e = fmaf(-d, r0, 1.0f);
    float r = fmaf(e, r0, r0);
    float q = n * r;
    q = fmaf(fmaf(-d, q, n), r, q);
    return fmaf(fmaf(-d, q, n), r, q);
}

int main(int argc, char **argv) {
    long pairs = argc > 1 ? atol(argv[1]) : 20000000L;
    long bad = 0, total = 0;
    const float ds[4] = {9.0f, 36.0f, 3.0f, 18.0f};  /* D2Q9 weights; D3Q19 adds 1/3, 1/18 */
    for (int di = 0; di < 4; ++di) {
        volatile float one = 1.0f, d = ds[di];
        const float y = one / d;
        for (int e = -20; e <= 20; ++e)
            for (uint32_t m = 0; m < (1u << 23); ++m) {
                const float x = bits_f(((uint32_t)(127 + e) << 23) | m);
                volatile float vx = x;
                const float ref = vx / d, got = div_const(x, d, y);
                ++total;
                if (f_bits(ref) != f_bits(got)) {
                    if (bad < 5) printf("const d=%g x=%a ref=%a got=%a\n", (double)d, x, ref, got);
                    ++bad;
                }
            }
    }
    printf("constant divisors: %ld mismatches of %ld\n", bad, total);
    long bad2 = 0;
    for (long i = 0; i < pairs; ++i) {
        /* d in [2^-12, 2^8) (densities), n in +-[2^-100, 2^8) (momenta) */
        const float d = bits_f(((uint32_t)(127 - 12 + (xr() % 20)) << 23) | (uint32_t)(xr() & 0x7fffff));
        const float n = bits_f(((uint32_t)(127 - 100 + (xr() % 108)) << 23) | (uint32_t)(xr() & 0x7fffff) |
                               (uint32_t)((xr() & 1) << 31));
        volatile float vn = n, one = 1.0f;
        const float ref = vn / d, rr = one / d;
        for (int k = -1; k <= 1; ++k) {
            const float got = div_seq(n, d, bits_f(f_bits(rr) + (uint32_t)k));
            if (f_bits(ref) != f_bits(got)) {
                if (bad2 < 5) printf("pair n=%a d=%a k=%d ref=%a got=%a\n", n, d, k, ref, got);
                ++bad2;
            }
        }
    }
    printf("variable divisor: %ld mismatches in %ld pairs x 3 reciprocals\n", bad2, pairs);
    return (bad || bad2) ? 1 : 0;
}
