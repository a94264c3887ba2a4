// Last-arriver hand-offs for in-launch reductions (gfx950, 8 XCDs with private L2s).
//
// Producer side, every form (MI355X_MICROARCH.md, "Valid forms", split-K seam, write-through):
// the block's (or wave's) partial record is stored WRITE-THROUGH with agent-scope relaxed atomic
// stores (global_store ... sc1, st_wt below) by ONE lane, which then drains them
// (s_waitcnt vmcnt(0)) and draws a ticket with a relaxed agent-scope fetch_add on one counter.
// No release fence: a per-block buffer_wbl2 over thousands of workgroups was the dominant cost
// (SQ_WAIT_ANY 82 % of wave cycles in the sampler). The counter lives in caller-owned workspace
// zeroed once at allocation; the consumer re-arms it (rearm).
//
// Consumer side: the workgroup (or wave) whose add returned total - 1 reads every record with
// agent-scope relaxed loads (global_load ... sc1) after ONE agent acquire (buffer_inv sc1 +
// vmcnt(0)): arrive_last() for block-level records, handoff_acquire() where the merging wave
// tested the ticket itself (the sampler's split merge, the fused pass's plan and fold). The
// guide's row 1 would allow the sc1 loads without the acquire, but it was measured at one
// workgroup per CU; these launches put several on a CU, so the acquire stays. The
// sc1 form alone is still what the tests exercise hardest: tests/test_gpu_sampler_splits.py runs
// every split shape for many decode steps against the oracle's tokens (a stale record would show
// as a wrong token or logprob), and the fold / plan tests compare every micro-batch's loss.
#ifndef SKYRL_HANDOFF_ACQUIRE  // probe builds A/B its cost
#define SKYRL_HANDOFF_ACQUIRE 1
#endif
#pragma once
#include "common.h"

namespace skyrl {

template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) {  // write-through (sc1) store of a partial
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every partial of this block must have been stored with st_wt() by threadIdx.x == 0.
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned total, int* lds_flag) {
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (prev == total - 1u);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *lds_flag = last;
    }
    __syncthreads();
    return *lds_flag != 0;
}

// the merging wave's acquire before it loads the other producers' records (see the header)
__device__ __forceinline__ void handoff_acquire() {
#if SKYRL_HANDOFF_ACQUIRE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}

__device__ __forceinline__ void rearm(unsigned* counter) {
    if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-wide sum of NV doubles (fixed tree, deterministic). lds: NW*NV doubles.
template <int NW, int NV>
__device__ __forceinline__ void block_sum_d(double (&v)[NV], double* lds) {
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
    }
    __syncthreads();
    double s[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) s[k] = 0.0;
#pragma unroll 1
    for (int j = 0; j < NW; ++j) {  // same per-quantity order; not unrolled (16 waves x 6 doubles spilled)
#pragma unroll
        for (int k = 0; k < NV; ++k) s[k] += lds[j * NV + k];
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = s[k];
    __syncthreads();
}

// fp64 wave sum without LDS: DPP moves of the two 32-bit halves (quad_perm xor 1, xor 2, then
// row_ror 4 and 8 inside each 16-lane row), then the four row sums read with v_readlane and added
// as (r0 + r1) + (r2 + r3). A fixed tree, so the result is deterministic and wave-uniform; it
// replaces the xor butterfly of __shfl_xor, whose 64-bit ds_bpermute pairs cost six LDS round
// trips per value (the loss finish's block reduction measured 0.8 us of its 1.1 us fold).
// Requires all 64 lanes active.
template <int CTRL>
__device__ __forceinline__ double dpp_mov_f64(double x) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u & 0xffffffffull), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double readlane_f64(double x, int lane) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += dpp_mov_f64<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
    v += dpp_mov_f64<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
    v += dpp_mov_f64<0x124>(v);  // row_ror 4
    v += dpp_mov_f64<0x128>(v);  // row_ror 8: lane 16r holds row r's sum
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// fp32 wave sum, the same DPP tree (quad_perm xor 1, xor 2, row_ror 4, 8, then the four row sums
// read with v_readlane as (r0 + r1) + (r2 + r3)); wave-uniform. Requires all 64 lanes active.
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
    auto rl = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
    return (rl(0) + rl(16)) + (rl(32) + rl(48));
}

}  // namespace skyrl
