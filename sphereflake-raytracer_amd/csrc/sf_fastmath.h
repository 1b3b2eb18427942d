// sf_fastmath.h -- correctly rounded fp32 reciprocal and square root on gfx950 for arguments inside the ranges where
// the IEEE sequences' range scaling and special-case fixups are idle, so the short forms return the same bits.
//
// The compiler's IEEE forms (-fhip-fp32-correctly-rounded-divide-sqrt): 1.0f / x is v_div_scale x2, v_rcp, five
// FMAs, v_div_fmas and v_div_fixup; sqrtf(x) scales tiny arguments by 2^32, takes v_sqrt, tests the neighbours
// s - 1 ulp and s + 1 ulp by FMA residuals, and patches 0 / inf / NaN with a class test. Inside the ranges below the
// scales are 1 and the fixups pass the value through: what is left is the core of each sequence. Both are checked
// against the IEEE operation for EVERY float of their range (tests/hip/fastmath_check.hip,
// tests/test_gpu_post.py::test_fastmath_matches_ieee_on_every_float); callers send other arguments to the IEEE form.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

// range of rcp_rn_mid: 2^-124 <= |x| <= 2^124 (and the quotient is normal)
#define SF_RCP_MID_LO 0x1p-124f
#define SF_RCP_MID_HI 0x1p124f
// range of sqrt_rn_mid: 2^-96 <= x < +inf (no scaling of tiny arguments), and x == 0
#define SF_SQRT_MID_LO 0x1p-96f

// 1/x: v_rcp (within 1 ulp) and one Newton step by FMA. The compiler's division runs two more residual
// corrections of the quotient; over the range they change nothing: this form equals the IEEE 1/x on every float of
// the range (4 160 749 570 arguments, 0 mismatches; the bare v_rcp differs on part of them -- tests/hip).
__device__ __forceinline__ float rcp_rn_mid(float x)
{
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
}

// sqrt(x): v_sqrt, then the neighbour whose residual says it is the correctly rounded root
__device__ __forceinline__ float sqrt_rn_mid(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    const float t = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : t;
}
