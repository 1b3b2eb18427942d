// Diagnostic kernel (not product code): how long a small kernel on a second stream waits for a wave slot while
// a persistent trace grid fills the GPU -- the rehearsal of rank 0's RCCL receive posted beside its own trace
// (csrc/sf_dist.hip; VERDICT r4 "residency hazard"). One workgroup of one wave stores s_memrealtime (100 MHz) when
// it starts; the caller compares it with the host's launch time and the trace kernel's own start.
// Built by __graft_entry__.build() into tests/hip/build/libsf_slot_probe.so; used by scripts/slot_residency_probe.py.
#include <hip/hip_runtime.h>

#include <cstdint>

__global__ void __launch_bounds__(64) stamp(unsigned long long* out)
{
    if (threadIdx.x == 0) *out = __builtin_amdgcn_s_memrealtime();
}

// the same clock read on the device right now (one tiny kernel, waited for): host <-> device clock pairing
extern "C" int sf_probe_stamp(unsigned long long* dev_out, void* stream)
{
    hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, (hipStream_t)stream, dev_out);
    return (int)hipGetLastError();
}
