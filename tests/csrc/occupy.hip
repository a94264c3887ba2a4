// Test hook (never in libskyrl_hip.so): `blocks` workgroups of `threads` threads that each spin on
// the 100 MHz constant clock for base_ticks + (block % 64) * step_ticks, holding their CU slots.
// tests/test_gpu_policy_train_split.py runs the split training pass beside it on another stream, so
// the pieces of a row are dispatched far apart (a piece whose partner is late computes that
// partner's state itself).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void occupy_kernel(int64_t base, int64_t step) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t until = (uint64_t)(base + (int64_t)(blockIdx.x % 64) * step);
    while (__builtin_amdgcn_s_memrealtime() - t0 < until) __builtin_amdgcn_s_sleep(8);
}

extern "C" int skyrl_test_occupy(int32_t blocks, int32_t threads, int64_t base_ticks, int64_t step_ticks, void* stream) {
    if (blocks < 1 || blocks > 65536 || threads < 64 || threads > 1024 || threads % 64) return 1;
    if (base_ticks < 0 || step_ticks < 0 || base_ticks + 64 * step_ticks > 100000000) return 1;  // at most 1 s
    hipLaunchKernelGGL(occupy_kernel, dim3(blocks), dim3(threads), 0, reinterpret_cast<hipStream_t>(stream), base_ticks,
                       step_ticks);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
