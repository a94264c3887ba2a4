// Shared device helpers for the gfx950 hot-path kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/skyrl_hip.h"

namespace skyrl {

constexpr int kWave = 64;

// ---- error plumbing (host) -------------------------------------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

#define SKYRL_REQUIRE(cond, msg)                                   \
    do {                                                           \
        if (!(cond)) return ::skyrl::fail(SKYRL_ERR_INVALID, msg); \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- dtype helpers (device) ------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
    return __uint_as_float(static_cast<uint32_t>(h) << 16);
}
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// f32 -> bf16, round-to-nearest-even, NaN kept a NaN: one v_cvt_pk_bf16_f32 (gfx950).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
    f32x2_t f = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
}

// Raw v_exp_f32 / v_log_f32 (base 2): no range-reduction wrapper. Inputs on the hot
// paths are <= 0 (softmax numerators) or normal positives (sums), where the bare
// instruction is accurate to ~1 ulp; exp2f()/log2f() add 4-5 VALU ops of denormal
// handling per call.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

// Mask element as float, for every mask dtype the reference uses
// (int64 response_mask, f32 loss_mask, bool).
__device__ __forceinline__ float load_mask(const void* m, int dtype, int64_t i) {
    switch (dtype) {
        case SKYRL_F32: return reinterpret_cast<const float*>(m)[i];
        case SKYRL_I64: return static_cast<float>(reinterpret_cast<const int64_t*>(m)[i]);
        case SKYRL_I32: return static_cast<float>(reinterpret_cast<const int32_t*>(m)[i]);
        case SKYRL_U8: return static_cast<float>(reinterpret_cast<const uint8_t*>(m)[i]);
        default: return 0.f;
    }
}

// Four consecutive mask values loaded raw and converted later, so the load stays in flight past
// the code between (a float conversion right after the load makes the compiler wait for it,
// and with it for every load issued before).
struct Mask4Raw {
    uint4 a, b;
};
template <int MDT>
__device__ __forceinline__ Mask4Raw load_mask4_raw(const void* m, int64_t idx) {
    Mask4Raw r;
    r.b = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (MDT == SKYRL_I64) {
        const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const int64_t*>(m) + idx);
        r.a = p[0];
        r.b = p[1];
    } else if constexpr (MDT == SKYRL_U8) {
        r.a = make_uint4(*reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(m) + idx), 0u, 0u, 0u);
    } else {
        r.a = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint32_t*>(m) + idx);
    }
    return r;
}
template <int MDT>
__device__ __forceinline__ void mask4_to_float(const Mask4Raw& r, float (&o)[4]) {
    if constexpr (MDT == SKYRL_I64) {
        o[0] = (float)(int64_t)(((uint64_t)r.a.y << 32) | r.a.x);
        o[1] = (float)(int64_t)(((uint64_t)r.a.w << 32) | r.a.z);
        o[2] = (float)(int64_t)(((uint64_t)r.b.y << 32) | r.b.x);
        o[3] = (float)(int64_t)(((uint64_t)r.b.w << 32) | r.b.z);
    } else if constexpr (MDT == SKYRL_F32) {
        o[0] = __uint_as_float(r.a.x); o[1] = __uint_as_float(r.a.y);
        o[2] = __uint_as_float(r.a.z); o[3] = __uint_as_float(r.a.w);
    } else if constexpr (MDT == SKYRL_I32) {
        o[0] = (float)(int)r.a.x; o[1] = (float)(int)r.a.y; o[2] = (float)(int)r.a.z; o[3] = (float)(int)r.a.w;
    } else {
        o[0] = (float)(r.a.x & 0xffu); o[1] = (float)((r.a.x >> 8) & 0xffu);
        o[2] = (float)((r.a.x >> 16) & 0xffu); o[3] = (float)(r.a.x >> 24);
    }
}

// ---- wave / block reductions ------------------------------------------------
// Four consecutive mask values from a 16-B-aligned (f32/i64/i32) or 4-B-aligned (u8) address.
__device__ __forceinline__ void load_mask4(const void* m, int dtype, int64_t idx, float (&o)[4]) {
    switch (dtype) {
        case SKYRL_F32: {
            float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(m) + idx);
            o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
            break;
        }
        case SKYRL_I64: {
            const longlong2* p = reinterpret_cast<const longlong2*>(reinterpret_cast<const int64_t*>(m) + idx);
            longlong2 a = p[0], b = p[1];
            o[0] = (float)a.x; o[1] = (float)a.y; o[2] = (float)b.x; o[3] = (float)b.y;
            break;
        }
        case SKYRL_I32: {
            int4 v = *reinterpret_cast<const int4*>(reinterpret_cast<const int32_t*>(m) + idx);
            o[0] = (float)v.x; o[1] = (float)v.y; o[2] = (float)v.z; o[3] = (float)v.w;
            break;
        }
        default: {
            uchar4 v = *reinterpret_cast<const uchar4*>(reinterpret_cast<const uint8_t*>(m) + idx);
            o[0] = (float)v.x; o[1] = (float)v.y; o[2] = (float)v.z; o[3] = (float)v.w;
            break;
        }
    }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
    return v;
}

// Wave-wide max broadcast as a wave-uniform value, without LDS: DPP quad_perm xor1/xor2 and
// row_ror 4/8 give every lane its 16-lane row max (out-of-row sources keep -inf), then the
// four row maxima are read with v_readlane. Requires all 64 lanes active.
__device__ __forceinline__ float wave_max_uniform(float v) {
    auto step = [](float x, int ctrl) -> float {
        constexpr int kNegInf = (int)0xff800000u;
        int y;
        switch (ctrl) {  // dpp control must be an immediate
            case 0: y = __builtin_amdgcn_update_dpp(kNegInf, __float_as_int(x), 0xB1, 0xF, 0xF, false); break;
            case 1: y = __builtin_amdgcn_update_dpp(kNegInf, __float_as_int(x), 0x4E, 0xF, 0xF, false); break;
            case 2: y = __builtin_amdgcn_update_dpp(kNegInf, __float_as_int(x), 0x124, 0xF, 0xF, false); break;
            default: y = __builtin_amdgcn_update_dpp(kNegInf, __float_as_int(x), 0x128, 0xF, 0xF, false); break;
        }
        return fmaxf(x, __int_as_float(y));
    };
    v = step(v, 0);
    v = step(v, 1);
    v = step(v, 2);
    v = step(v, 3);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// Sum of NV values across a block of NW waves; result valid in every thread.
// `lds` needs NW*NV floats. Deterministic (fixed tree).
template <int NW, int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* lds) {
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < NW; ++j) s += lds[j * NV + k];
        v[k] = s;
    }
    __syncthreads();
}

}  // namespace skyrl
