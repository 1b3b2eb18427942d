/*
 * gen_rsqrtps_lut.c -- TEST INFRASTRUCTURE (oracle side). Measures the x86
 * `rsqrtps` approximation on the CPU it runs on and writes it as a 2x1024
 * lookup table.
 *
 * Why: the reference normalises the ray direction (and the hit normal) with
 * `_mm256_rsqrt_ps` + one Newton-Raphson step (reference
 * sphereflake/SIMD_AVX.h:170-180). The approximation is implementation
 * defined; on the Intel CPU the parity fixtures were generated on it is a pure
 * function of (exponent parity, top 10 mantissa bits), and scaling the input
 * by 4 halves the output exactly. This program VERIFIES both
 * claims exhaustively over every positive normal float before writing the
 * table, so the table is data measured from the instruction, not derived from
 * reference code.
 *
 * Table layout (little-endian uint32 bit patterns, 2048 entries):
 *   key = ((E & 1) << 10) | (mantissa >> 13), E = biased exponent of x
 *   LUT[key] = bits of rsqrtps(x0) where x0 has the same key and biased
 *              exponent E0 = 127 (E odd) or 128 (E even), i.e. x0 in [1,4).
 * Emulation for a normal x:  out_bits = LUT[key] - (((E - E0) / 2) << 23).
 *
 * Build: gcc -O2 -msse2 gen_rsqrtps_lut.c -o gen_rsqrtps_lut
 * Usage: gen_rsqrtps_lut <out.bin>     (prints a JSON summary on stdout)
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static uint32_t lut[2048];

static uint32_t emulate(uint32_t xb)
{
    uint32_t E = (xb >> 23) & 0xffu;
    uint32_t key = ((E & 1u) << 10) | ((xb & 0x7fffffu) >> 13);
    int32_t E0 = (E & 1u) ? 127 : 128;
    int32_t k = ((int32_t)E - E0) / 2;
    return (uint32_t)((int32_t)lut[key] - (k << 23));
}

int main(int argc, char** argv)
{
    if (argc < 2) { fprintf(stderr, "usage: %s out.bin\n", argv[0]); return 2; }

    /* 1. table from x in [1,4), and the "low 13 mantissa bits do not matter" check */
    uint64_t low_bits_violations = 0;
    for (uint32_t par = 0; par < 2; ++par) {
        uint32_t E0 = par ? 127u : 128u;
        for (uint32_t hi = 0; hi < 1024; ++hi) {
            uint32_t key = (par << 10) | hi;
            uint32_t base = (E0 << 23) | (hi << 13);
            float xs[8];
            uint32_t first = 0;
            for (uint32_t lo = 0; lo < 8192; lo += 8) {
                for (int j = 0; j < 8; ++j) xs[j] = u2f(base | (lo + j));
                __m128 a = _mm_loadu_ps(xs), b = _mm_loadu_ps(xs + 4);
                float ra[4], rb[4];
                _mm_storeu_ps(ra, _mm_rsqrt_ps(a));
                _mm_storeu_ps(rb, _mm_rsqrt_ps(b));
                if (lo == 0) first = f2u(ra[0]);
                for (int j = 0; j < 4; ++j) {
                    if (f2u(ra[j]) != first) ++low_bits_violations;
                    if (f2u(rb[j]) != first) ++low_bits_violations;
                }
            }
            lut[key] = first;
        }
    }

    /* 2. exhaustive check of the emulation over every positive normal float */
    uint64_t checked = 0, mismatches = 0;
    for (uint32_t xb = 0x00800000u; xb < 0x7f800000u; xb += 4) {
        float xs[4] = { u2f(xb), u2f(xb + 1), u2f(xb + 2), u2f(xb + 3) };
        float r[4];
        _mm_storeu_ps(r, _mm_rsqrt_ps(_mm_loadu_ps(xs)));
        for (int j = 0; j < 4; ++j) {
            ++checked;
            if (f2u(r[j]) != emulate(xb + j)) ++mismatches;
        }
    }

    /* 3. special inputs: record what the instruction does (the emulators copy this) */
    float sp_in[8] = { 0.0f, -0.0f, u2f(0x00000001u), u2f(0x007fffffu),
                       u2f(0x7f800000u), -1.0f, u2f(0x7fc00000u), u2f(0x7fa00000u) };
    float sp_out[8];
    _mm_storeu_ps(sp_out, _mm_rsqrt_ps(_mm_loadu_ps(sp_in)));
    _mm_storeu_ps(sp_out + 4, _mm_rsqrt_ps(_mm_loadu_ps(sp_in + 4)));

    FILE* f = fopen(argv[1], "wb");
    if (!f) { perror("fopen"); return 1; }
    fwrite(lut, 4, 2048, f);
    fclose(f);

    char vendor[13] = {0};
    {
        unsigned a, b, c, d;
        __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(0));
        memcpy(vendor, &b, 4); memcpy(vendor + 4, &d, 4); memcpy(vendor + 8, &c, 4);
    }
    printf("{\"cpu_vendor\": \"%s\", \"low_bits_violations\": %llu, \"checked\": %llu, "
           "\"mismatches\": %llu, \"special\": {",
           vendor, (unsigned long long)low_bits_violations,
           (unsigned long long)checked, (unsigned long long)mismatches);
    for (int j = 0; j < 8; ++j)
        printf("%s\"0x%08x\": \"0x%08x\"", j ? ", " : "", f2u(sp_in[j]), f2u(sp_out[j]));
    printf("}}\n");
    return (low_bits_violations || mismatches) ? 1 : 0;
}
