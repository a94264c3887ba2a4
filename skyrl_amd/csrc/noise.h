// The sampler's noise model and decision helpers, shared by sampler.hip (a1, logits in HBM) and
// lmhead_gemm.hip (the same decision fused into the lm_head GEMM epilogue). Every float op on
// the decision path is an IEEE basic op or an explicit fmaf with contraction off, so
// oracle/sampler_ref.c reproduces the decisions bit for bit.
#pragma once
#include "common.h"

#pragma clang fp contract(off)

namespace skyrl {

__host__ __device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// Per-element noise hash of pair index p (two 16-bit halves, one per element). Built from
// 24-bit multiplies (v_mad_u32_u24 / v_mul_u32_u24 issue at the full VALU rate, v_mul_lo_u32 at a
// quarter of it) and 16-bit xor-shifts (one SDWA op each); the two row keys enter at two rounds, so
// that an additive collision of the first round between rows is broken by the second.
// Bit-identical in oracle/sampler_ref.c.
__host__ __device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) { return (a & 0xffffffu) * (b & 0xffffffu); }
__host__ __device__ __forceinline__ uint32_t ehash(uint32_t ka, uint32_t kb, uint32_t p) {
    uint32_t h = mul24(p, 0x9e3779u) + ka;
    h ^= h >> 16;
    h = mul24(h, 0x85ebcau) + kb;
    h ^= h >> 16;
    h = mul24(h, 0xc2b2aeu);
    h ^= h >> 16;
    return h;
}

__host__ __device__ __forceinline__ uint32_t row_key(uint64_t seed, int64_t seq, int64_t step) {
    uint32_t k = hash32((uint32_t)seed ^ 0x9e3779b9u);
    k = hash32(k ^ (uint32_t)(seed >> 32));
    k = hash32(k ^ (uint32_t)((uint64_t)seq));
    k = hash32(k ^ (uint32_t)((uint64_t)seq >> 32));
    k = hash32(k ^ (uint32_t)((uint64_t)step));
    k = hash32(k ^ (uint32_t)((uint64_t)step >> 32));
    return k;
}

// Deterministic natural log for normal positive floats (branch-free): ix = bits - bits(2/3),
// e = ix >> 23 (arithmetic), mantissa rebased into [2/3, 4/3), ln(1+z) = z*P6(z) by fmaf
// Horner (|err| < 1.1e-6). Bit-identical in oracle/sampler_ref.c (same ops, contraction off).
__host__ __device__ __forceinline__ float det_ln(float y) {
    const uint32_t ix = __builtin_bit_cast(uint32_t, y) - 0x3f2aaaabu;
    const int e = (int)ix >> 23;
    const float m = __builtin_bit_cast(float, (ix & 0x007fffffu) + 0x3f2aaaabu);
    const float z = m - 1.0f;
    float p = 0.16302786767482758f;
    p = fmaf(p, z, -0.18978701531887054f);
    p = fmaf(p, z, 0.19917640089988708f);
    p = fmaf(p, z, -0.24900923669338226f);
    p = fmaf(p, z, 0.3333371579647064f);
    p = fmaf(p, z, -0.5000061392784119f);
    p = fmaf(p, z, 1.0f);
    return fmaf((float)e, 0.693147180559945f, z * p);
}

// Group-of-8 exponential race (the noise model, see sample_kernel): group hash h gives the
// group's smallest Exp(1) draw E_g = -ln(u_g)/8 at slot h & 7; every other slot v adds
// -ln U_v with U_v from hash32(key2 ^ v phi). score = x/T - ln E_v.
constexpr float kNoiseU24 = 5.9604644775390625e-8f;
__host__ __device__ __forceinline__ float group_min_e(uint32_t h) {
    const uint32_t t16 = (h >> 16) ^ 0xffffu;
    const float ug = (float)(((t16 << 8) | ((h >> 8) & 0xffu)) | 1u) * kNoiseU24;
    return -det_ln(ug) * 0.125f;
}
// score = x/T - ln E_v of element v (group hash h, group minimum Eg); the body, for a caller that
// keeps ONE inlined site (a loop over candidates) instead of a call
__host__ __device__ __forceinline__ float noise_score_inl(float xk, float inv_t, int v, uint32_t h, float Eg,
                                                          uint32_t key2) {
    float E = Eg;
    if (((uint32_t)v & 7u) != (h & 7u)) {
        const uint32_t hu = hash32(key2 ^ ((uint32_t)v * 0x9e3779b1u));
        const float U = (float)((hu >> 8) | 1u) * kNoiseU24;
        E = Eg + (-det_ln(U));
    }
    return xk * inv_t + (-det_ln(E));
}
// Inlined (SKYRL_NOISE_INLINE 2, the product): r06 tried the exact score out of line to shrink
// the T > 0 kernels' code (51-108 KB vs greedy's 9 KB), and every T > 0 launch got slower (512 /
// 64 / 1 rows at T = 1: 32.5 -> 39.7, 14.5 -> 20.4, 8.9 -> 13.8 us; profiles/r06_sampler_inline_ab.json):
// a callee starts with s_waitcnt vmcnt(0), so each call drained the loads the streaming loop had
// in flight. The callers keep the code small instead with one inlined copy of the scoring per
// visit site (a loop over the slots that need it; eval_slots in sampler.hip).
#ifndef SKYRL_NOISE_INLINE  // probe builds (scripts/probe/sampler_ab.py) A/B the inlining
#define SKYRL_NOISE_INLINE 2
#endif
#if SKYRL_NOISE_INLINE
#define SKYRL_NOISE_ATTR __attribute__((always_inline))
#else
#define SKYRL_NOISE_ATTR __attribute__((noinline))
#endif
inline __host__ __device__ SKYRL_NOISE_ATTR float noise_score(float xk, float inv_t, int v, uint32_t h, float Eg,
                                                              uint32_t key2) {
    return noise_score_inl(xk, inv_t, v, h, Eg, key2);
}
// Group bound: an element of group hash h can reach an exact score `bar` only if
//   xmax - (T ln2 2^-23) bits(float(h >> 16)) >= (bar - kNoiseC) T     (see sample_kernel)
constexpr float kNoiseC = 146.0f * 0.6931471805599453f + 0.01f;
__device__ __forceinline__ float noise_bits(uint32_t h) { return (float)(int)__float_as_uint((float)(h >> 16)); }
__host__ __device__ __forceinline__ uint32_t noise_key2(uint32_t key) { return hash32(key ^ 0x5bd1e995u); }
__host__ __device__ __forceinline__ uint32_t noise_keyb(uint32_t key) { return hash32(key ^ 0x27d4eb2fu); }

struct Best {
    float score;
    int idx;
};
__device__ __forceinline__ bool better(float s, int i, const Best& b) {
    return s > b.score || (s == b.score && i < b.idx);
}

}  // namespace skyrl
