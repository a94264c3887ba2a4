// Shared row-softmax machinery for the vocabulary-streaming kernels (logprob.hip, lmhead.hip):
// bf16/f32 element access with the reference's in-dtype temperature division, and the online
// softmax state (m, S, W) in log2 units with its wave-level merge.
#pragma once
#include "common.h"

namespace skyrl {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kDLow = -1.0e30f;  // floor for x - m so that -inf logits give e=0, e*d=0

template <typename T> struct Elem;
template <> struct Elem<uint16_t> {
    static constexpr int kVec = 8;
    __device__ static float load(const uint16_t* p) { return bf16_to_f32(*p); }
    __device__ static float apply_t(float x, float t, bool has_t) {
        // logits.div_(T) in bf16: fp32 divide, round to bf16.
        return has_t ? bf16_to_f32(f32_to_bf16(x / t)) : x;
    }
    __device__ static void unpack(const uint4& v, float (&x)[8]) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[2 * k] = __uint_as_float(w[k] << 16);
            x[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        }
    }
    __device__ static uint4 pack(const float (&x)[8]) {
        return make_uint4(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                          pack_bf16x2(x[6], x[7]));
    }
    __device__ static void store(uint16_t* p, float x) { *p = f32_to_bf16(x); }
};
template <> struct Elem<float> {
    static constexpr int kVec = 4;
    __device__ static float load(const float* p) { return *p; }
    __device__ static float apply_t(float x, float t, bool has_t) { return has_t ? x / t : x; }
    __device__ static void unpack(const uint4& v, float (&x)[4]) {
        x[0] = __uint_as_float(v.x); x[1] = __uint_as_float(v.y);
        x[2] = __uint_as_float(v.z); x[3] = __uint_as_float(v.w);
    }
    __device__ static uint4 pack(const float (&x)[4]) {
        return make_uint4(__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3]));
    }
    __device__ static void store(float* p, float x) { *p = x; }
};

// Online softmax state in log2 units: m = running max of x, S = sum 2^y, W = sum 2^y * y
// with y = (x - m) * log2(e) >= -1e30 (finite even for x = -inf, so e*y = 0, never NaN).
// lse = m + ln(S); H = ln(S) - ln(2) * W / S.
struct SoftState {
    float m, s, w;
};

__device__ __forceinline__ void state_init(SoftState& st) {
    st.m = -3.402823466e38f;
    st.s = 0.f;
    st.w = 0.f;
}

// Fold a group of values (already temperature-applied) into the state.
template <int K>
__device__ __forceinline__ void state_add(SoftState& st, const float (&x)[K]) {
    float mx = x[0];
#pragma unroll
    for (int k = 1; k < K; ++k) mx = fmaxf(mx, x[k]);
    const float mn = fmaxf(st.m, mx);
    const float dy = fmaxf((st.m - mn) * kLog2e, kDLow);  // first fold: -FLT_MAX*log2e would be -inf
    const float a = fast_exp2(dy);
    st.w = a * fmaf(dy, st.s, st.w);
    st.s = a * st.s;
    st.m = mn;
    const float c = -mn * kLog2e;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const float y = fmaxf(fmaf(x[k], kLog2e, c), kDLow);
        const float e = fast_exp2(y);
        st.s += e;
        st.w = fmaf(e, y, st.w);
    }
}

__device__ __forceinline__ void state_merge(SoftState& a, const SoftState& b) {
    const float mn = fmaxf(a.m, b.m);
    const float da = fmaxf((a.m - mn) * kLog2e, kDLow), db = fmaxf((b.m - mn) * kLog2e, kDLow);
    const float ea = fast_exp2(da), eb = fast_exp2(db);
    a.w = ea * fmaf(da, a.s, a.w) + eb * fmaf(db, b.s, b.w);
    a.s = ea * a.s + eb * b.s;
    a.m = mn;
}

__device__ __forceinline__ SoftState wave_merge(SoftState st) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        SoftState o;
        o.m = __shfl_xor(st.m, off, kWave);
        o.s = __shfl_xor(st.s, off, kWave);
        o.w = __shfl_xor(st.w, off, kWave);
        state_merge(st, o);
    }
    return st;
}

// logp = x_label - lse, H = ln S - ln2 W / S and lse of a token's final state (lmhead.hip's chunk
// path and lmhead_gemm.hip's tile path)
__device__ __forceinline__ void finalize_row(const SoftState& st, float xl, int64_t r, float* __restrict__ logp_out,
                                             float* __restrict__ ent_out, float* __restrict__ lse_out) {
    const float logs = fast_log2(st.s) * kLn2;
    const float lse = st.m + logs;
    logp_out[r] = xl - lse;  // NaN for a label outside [0, V), as logprob.hip
    if (ent_out) ent_out[r] = logs - kLn2 * (st.w / st.s);
    if (lse_out) lse_out[r] = lse;
}

// Streaming 16-B load of data read once per pass (159 GB per pass >> L2/MALL): nontemporal.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_stream(const uint4* p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

}  // namespace skyrl
