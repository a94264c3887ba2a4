// §8(f)2 decode loop: the elementwise glue of a Qwen2/Llama decoder layer, fused.
//
// HF Qwen2DecoderLayer / LlamaDecoderLayer (transformers) run, per layer,
//   residual + attn_out -> RMSNorm -> MLP(gate, up) -> residual + mlp_out -> next RMSNorm
// as ~14 small PyTorch kernels (f32 upcast, pow, mean, rsqrt, mul, downcast, weight mul, add,
// silu, mul). At decode batch sizes every one of them is a launch-bound pass over a [n, H]
// row block; these two kernels do the same arithmetic in 2 launches per half-layer.
//
// skyrl_add_rmsnorm: h = bf16(h + delta) (the residual stream, rounded as HF's bf16 add),
//   y = bf16(h_f32 * rsqrt(mean(h_f32^2) + eps)), out = bf16(w * y) — HF Qwen2RMSNorm:
//   variance in f32, normalise in f32, cast, then scale in the model dtype.
// skyrl_silu_mul: out = bf16(bf16(silu(gate)) * up) — act_fn(gate_proj(x)) * up_proj(x) with
//   the bf16 rounding of each PyTorch op.
#include "common.h"

namespace skyrl {
namespace {

constexpr int kNT = 256;

__device__ __forceinline__ float2 bf2_to_f2(uint32_t v) {
    return make_float2(__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u));
}
__device__ __forceinline__ float round_bf16(float x) { return bf16_to_f32(f32_to_bf16(x)); }

// One block per row; each thread owns H / (4 * kNT) groups of 4 contiguous elements held in
// registers across the reduction (H <= 4 * kNT * kMaxV).
template <int kMaxV>
__global__ __launch_bounds__(kNT) void add_rmsnorm_kernel(const uint16_t* __restrict__ delta,
                                                          uint16_t* __restrict__ h, const uint16_t* __restrict__ w,
                                                          int H, float eps, uint16_t* __restrict__ out) {
    __shared__ float s_red[kNT / kWave];
    const int64_t row = blockIdx.x;
    const int nv = H >> 2;  // 4-element groups
    float x[kMaxV][4];
    float ss = 0.f;
    uint16_t* hr = h + row * H;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
        const int v = threadIdx.x + k * kNT;
        if (v < nv) {
            const uint2 hv = reinterpret_cast<const uint2*>(hr)[v];
            float2 a = bf2_to_f2(hv.x), b = bf2_to_f2(hv.y);
            float t[4] = {a.x, a.y, b.x, b.y};
            if (delta) {
                const uint2 dv = reinterpret_cast<const uint2*>(delta + row * H)[v];
                const float2 c = bf2_to_f2(dv.x), d = bf2_to_f2(dv.y);
                t[0] = round_bf16(t[0] + c.x);
                t[1] = round_bf16(t[1] + c.y);
                t[2] = round_bf16(t[2] + d.x);
                t[3] = round_bf16(t[3] + d.y);
                reinterpret_cast<uint2*>(hr)[v] = make_uint2(pack_bf16x2(t[0], t[1]), pack_bf16x2(t[2], t[3]));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                x[k][j] = t[j];
                ss += t[j] * t[j];
            }
        }
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x / kWave] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int j = 0; j < kNT / kWave; ++j) tot += s_red[j];
    const float r = rsqrtf(tot / (float)H + eps);
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
        const int v = threadIdx.x + k * kNT;
        if (v < nv) {
            const uint2 wv = reinterpret_cast<const uint2*>(w)[v];
            const float2 wa = bf2_to_f2(wv.x), wb = bf2_to_f2(wv.y);
            const float y0 = wa.x * round_bf16(x[k][0] * r), y1 = wa.y * round_bf16(x[k][1] * r);
            const float y2 = wb.x * round_bf16(x[k][2] * r), y3 = wb.y * round_bf16(x[k][3] * r);
            reinterpret_cast<uint2*>(out + row * H)[v] = make_uint2(pack_bf16x2(y0, y1), pack_bf16x2(y2, y3));
        }
    }
}

// grid-stride over n * I / 4 groups of 4 outputs; gu is [n, 2I] (gate | up).
__global__ __launch_bounds__(kNT) void silu_mul_kernel(const uint16_t* __restrict__ gu, int64_t n, int I,
                                                       uint16_t* __restrict__ out) {
    const int iv = I >> 2;
    const int64_t total = n * iv;
    for (int64_t e = (int64_t)blockIdx.x * kNT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kNT) {
        const int64_t row = e / iv;
        const int c = (int)(e - row * iv);
        const uint2 g = reinterpret_cast<const uint2*>(gu + row * 2 * I)[c];
        const uint2 u = reinterpret_cast<const uint2*>(gu + row * 2 * I + I)[c];
        const float2 g0 = bf2_to_f2(g.x), g1 = bf2_to_f2(g.y), u0 = bf2_to_f2(u.x), u1 = bf2_to_f2(u.y);
        auto act = [](float a) { return round_bf16(a / (1.f + expf(-a))); };
        reinterpret_cast<uint2*>(out + row * I)[c] =
            make_uint2(pack_bf16x2(act(g0.x) * u0.x, act(g0.y) * u0.y), pack_bf16x2(act(g1.x) * u1.x, act(g1.y) * u1.y));
    }
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" int skyrl_add_rmsnorm(const void* delta, void* hidden, const void* weight, int32_t n, int32_t H, float eps,
                                 void* out, void* stream) {
    SKYRL_REQUIRE(n >= 0 && H > 0 && H % 4 == 0 && H <= 4 * kNT * 8, "add_rmsnorm: H must be a multiple of 4, <= 8192");
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(hidden && weight && out, "add_rmsnorm: null pointer");
    auto* d = reinterpret_cast<const uint16_t*>(delta);
    auto* h = reinterpret_cast<uint16_t*>(hidden);
    auto* w = reinterpret_cast<const uint16_t*>(weight);
    auto* o = reinterpret_cast<uint16_t*>(out);
    const int nv = H / 4;
    if (nv <= kNT * 2)
        hipLaunchKernelGGL(add_rmsnorm_kernel<2>, dim3(n), dim3(kNT), 0, as_stream(stream), d, h, w, H, eps, o);
    else if (nv <= kNT * 4)
        hipLaunchKernelGGL(add_rmsnorm_kernel<4>, dim3(n), dim3(kNT), 0, as_stream(stream), d, h, w, H, eps, o);
    else
        hipLaunchKernelGGL(add_rmsnorm_kernel<8>, dim3(n), dim3(kNT), 0, as_stream(stream), d, h, w, H, eps, o);
    return check_launch("add_rmsnorm_kernel");
}

extern "C" int skyrl_silu_mul(const void* gate_up, int64_t n, int32_t I, void* out, void* stream) {
    SKYRL_REQUIRE(n >= 0 && I > 0 && I % 4 == 0, "silu_mul: I must be a positive multiple of 4");
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(gate_up && out, "silu_mul: null pointer");
    const int64_t groups = n * (I / 4);
    int64_t blocks = (groups + kNT - 1) / kNT;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(silu_mul_kernel, dim3((unsigned)blocks), dim3(kNT), 0, as_stream(stream),
                       reinterpret_cast<const uint16_t*>(gate_up), n, I, reinterpret_cast<uint16_t*>(out));
    return check_launch("silu_mul_kernel");
}
