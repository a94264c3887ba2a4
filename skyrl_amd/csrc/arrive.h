// Last-arriver election for in-launch reductions (gfx950, 8 XCDs with private L2s).
//
// Producer side (guide: split-K seam, write-through form): the block's partial record is
// stored WRITE-THROUGH with agent-scope relaxed atomic stores (global_store ... sc1) by
// the single storing thread, which then drains (s_waitcnt vmcnt(0)) and draws a ticket
// with a relaxed agent-scope fetch_add. No release fence: a per-block buffer_wbl2 over
// thousands of workgroups was the dominant cost (SQ_WAIT_ANY 82% of wave cycles in the
// sampler). The block drawing the last ticket does one agent-scope ACQUIRE (invalidates
// this CU's L1) before a block barrier, then reads every partial, and re-arms the counter.
// The counter lives in caller-owned workspace zeroed once at allocation.
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

}  // namespace skyrl
