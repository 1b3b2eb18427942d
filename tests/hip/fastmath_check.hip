// Test kernel (not product code): sf_fastmath.h's short forms against the IEEE operations for every float of their
// ranges. Built by __graft_entry__.build() into tests/hip/build/libsf_fastmath_check.so; called by
// tests/test_gpu_post.py::test_fastmath_matches_ieee_on_every_float.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sf_fastmath.h"

namespace {

// out[0]: reciprocal mismatches, out[1]: square-root mismatches, out[2]: reciprocal arguments checked, out[3]: root
// arguments checked, out[4] / out[5]: mismatches of the bare v_rcp / v_sqrt (what
// the refinements are for); every 32-bit pattern once
// (grid-stride over 2^32)
__global__ void __launch_bounds__(256) check_all(unsigned long long* out)
{
    unsigned long long bad_r = 0, bad_s = 0, n_r = 0, n_s = 0, bad_1 = 0, bad_2 = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const float x = __uint_as_float((uint32_t)i);
        const float ax = __builtin_fabsf(x);
        if (ax >= SF_RCP_MID_LO && ax <= SF_RCP_MID_HI) {
            ++n_r;
            const float ref = 1.0f / x;
            bad_r += __float_as_uint(rcp_rn_mid(x)) != __float_as_uint(ref);
            bad_1 += __float_as_uint(__builtin_amdgcn_rcpf(x)) != __float_as_uint(ref);
        }
        if ((x >= SF_SQRT_MID_LO && x <= 3.402823466e38f) || (uint32_t)i == 0u) {
            ++n_s;
            const float ref = sqrtf(x);
            bad_s += __float_as_uint(sqrt_rn_mid(x)) != __float_as_uint(ref);
            bad_2 += __float_as_uint(__builtin_amdgcn_sqrtf(x)) != __float_as_uint(ref);
        }
    }
    atomicAdd(&out[0], bad_r);
    atomicAdd(&out[1], bad_s);
    atomicAdd(&out[2], n_r);
    atomicAdd(&out[3], n_s);
    atomicAdd(&out[4], bad_1);
    atomicAdd(&out[5], bad_2);
}

}  // namespace

extern "C" int sf_fastmath_check(unsigned long long* counts)
{
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 6 * sizeof *d) != hipSuccess) return -1;
    int rc = 0;
    if (hipMemset(d, 0, 6 * sizeof *d) != hipSuccess) rc = -2;
    if (!rc) {
        hipLaunchKernelGGL(check_all, dim3(8192), dim3(256), 0, 0, d);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -3;
    }
    if (!rc && hipMemcpy(counts, d, 6 * sizeof *d, hipMemcpyDeviceToHost) != hipSuccess) rc = -4;
    (void)hipFree(d);
    return rc;
}
