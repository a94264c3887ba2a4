// a2/a3: per-token logprob + entropy over the vocabulary, forward and backward.
//
// Reference semantics (skyrl-train/skyrl_train/):
//   HFModelWrapper.forward      model_wrapper.py:313-363 (logits.div_(T) in the
//                               logits dtype, then logprobs + chunked entropy)
//   logprobs_from_logits        utils/torch_utils.py:115-177 (flash-attn CE:
//                               fp32 LSE of the logits minus the label logit)
//   chunked_entropy_from_logits utils/torch_utils.py:59-111
//
// Design (HBM-bound, 2 B/element bf16): one wave64 per token row, 4 rows per
// 256-thread workgroup, thousands of workgroups per launch. Each lane streams
// 16-B vectors (8 bf16) of its row with 4 loads in flight and keeps an online
// softmax state (m, S = sum e^(x-m), W = sum e^(x-m)(x-m)) in registers; the
// wave folds the 64 lane states with shuffles. Nothing is staged in LDS: the
// row is read exactly once, the label logit with one extra scalar load.
// H = log S - W/S avoids the lse - E[x] cancellation.
// Backward streams the row again and writes dlogits (2 B/element):
//   d/dx_v = (g_lp*(1[v=label] - p_v) - g_ent*p_v*(logp_v + H)) / T.
#include "softmax.h"
#include "variant.h"

namespace skyrl {
namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerBlock = kThreads / kWave;
template <typename T, int kUnroll, bool kNT>
__global__ __launch_bounds__(kThreads) void logprob_fwd_kernel(
    const T* __restrict__ logits, int64_t sb, int64_t st_, int nt, int64_t rows, int V,
    const int64_t* __restrict__ labels, int64_t lsb, int64_t lst, float temp, bool has_t,
    float* __restrict__ logp_out, float* __restrict__ ent_out, float* __restrict__ lse_out) {
    using E = Elem<T>;
    constexpr int VEC = E::kVec;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
    if (r >= rows) return;
    const int64_t b = r / nt, t = r % nt;
    const T* row = logits + b * sb + t * st_;

    SoftState st;
    state_init(st);
    const bool vec_ok = (reinterpret_cast<uintptr_t>(row) % 16) == 0;
    int done = 0;
    if (vec_ok) {
        const int nvec = V / VEC;
        const uint4* rv = reinterpret_cast<const uint4*>(row);
        int i = lane;
        for (; i + (kUnroll - 1) * kWave < nvec; i += kUnroll * kWave) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) v[u] = kNT ? ld_stream(rv + i + u * kWave) : rv[i + u * kWave];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                float x[VEC];
                E::unpack(v[u], x);
                if (has_t) {
#pragma unroll
                    for (int k = 0; k < VEC; ++k) x[k] = E::apply_t(x[k], temp, true);
                }
                state_add<VEC>(st, x);
            }
        }
        for (; i < nvec; i += kWave) {
            float x[VEC];
            E::unpack(kNT ? ld_stream(rv + i) : rv[i], x);
            if (has_t) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) x[k] = E::apply_t(x[k], temp, true);
            }
            state_add<VEC>(st, x);
        }
        done = nvec * VEC;
    }
    for (int i = done + lane; i < V; i += kWave) {
        float x[1] = {E::apply_t(E::load(row + i), temp, has_t)};
        state_add<1>(st, x);
    }
    st = wave_merge(st);
    if (lane == 0) {
        const float logs = fast_log2(st.s) * kLn2;
        const float lse = st.m + logs;
        const int64_t lab = labels[b * lsb + t * lst];
        float xl;
        if (lab >= 0 && lab < V) xl = E::apply_t(E::load(row + lab), temp, has_t);
        else xl = __builtin_nanf("");
        logp_out[r] = xl - lse;
        if (ent_out) ent_out[r] = logs - kLn2 * (st.w / st.s);
        if (lse_out) lse_out[r] = lse;
    }
}

template <typename T, int kUnroll, bool kNT>
__global__ __launch_bounds__(kThreads) void logprob_bwd_kernel(
    const T* __restrict__ logits, int64_t sb, int64_t st_, int nt, int64_t rows, int V,
    const int64_t* __restrict__ labels, int64_t lsb, int64_t lst, float temp, bool has_t,
    const float* __restrict__ lse, const float* __restrict__ ent, const float* __restrict__ g_lp,
    const float* __restrict__ g_ent, T* __restrict__ dx) {
    using E = Elem<T>;
    constexpr int VEC = E::kVec;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
    if (r >= rows) return;
    const int64_t b = r / nt, t = r % nt;
    const T* row = logits + b * sb + t * st_;
    T* out = dx + r * (int64_t)V;
    const float L = lse[r];
    const float H = g_ent ? ent[r] : 0.f;
    const float glp = g_lp[r];
    const float gent = g_ent ? g_ent[r] : 0.f;
    const float inv_t = has_t ? 1.f / temp : 1.f;
    const int64_t lab = labels[b * lsb + t * lst];
    auto grad = [&](float x, int64_t v) -> float {
        const float lp = x - L;
        const float p = fast_exp2(lp * kLog2e);
        float g = -glp * p - gent * p * (lp + H);
        if (v == lab) g += glp;
        return has_t ? g * inv_t : g;
    };
    const bool vec_ok = (reinterpret_cast<uintptr_t>(row) % 16) == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0;
    int done = 0;
    if (vec_ok) {
        const int nvec = V / VEC;
        const uint4* rv = reinterpret_cast<const uint4*>(row);
        uint4* ov = reinterpret_cast<uint4*>(out);
        int i = lane;
        for (; i + (kUnroll - 1) * kWave < nvec; i += kUnroll * kWave) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) v[u] = kNT ? ld_stream(rv + i + u * kWave) : rv[i + u * kWave];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                float x[VEC];
                E::unpack(v[u], x);
                const int64_t v0 = (int64_t)(i + u * kWave) * VEC;
#pragma unroll
                for (int k = 0; k < VEC; ++k) x[k] = grad(E::apply_t(x[k], temp, has_t), v0 + k);
                ov[i + u * kWave] = E::pack(x);
            }
        }
        for (; i < nvec; i += kWave) {
            float x[VEC];
            E::unpack(kNT ? ld_stream(rv + i) : rv[i], x);
            const int64_t v0 = (int64_t)i * VEC;
#pragma unroll
            for (int k = 0; k < VEC; ++k) x[k] = grad(E::apply_t(x[k], temp, has_t), v0 + k);
            ov[i] = E::pack(x);
        }
        done = nvec * VEC;
    }
    for (int i = done + lane; i < V; i += kWave) {
        E::store(out + i, grad(E::apply_t(E::load(row + i), temp, has_t), i));
    }
}


template <typename T, int U, bool NT>
int launch_fwd_v(const void* logits, int64_t sb, int64_t st, int nb, int nt, int V, const int64_t* labels, int64_t lsb,
               int64_t lst, float temp, float* logp, float* ent, float* lse, hipStream_t s) {
    const int64_t rows = (int64_t)nb * nt;
    const int64_t blocks = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
    const bool has_t = temp != 1.0f;
    hipLaunchKernelGGL((logprob_fwd_kernel<T, U, NT>), dim3((unsigned)blocks), dim3(kThreads), 0, s,
                       reinterpret_cast<const T*>(logits), sb, st, nt, rows, V, labels, lsb, lst, temp, has_t, logp,
                       ent, lse);
    return check_launch("logprob_fwd_kernel");
}

template <typename T, int U, bool NT>
int launch_bwd_v(const void* logits, int64_t sb, int64_t st, int nb, int nt, int V, const int64_t* labels, int64_t lsb,
               int64_t lst, float temp, const float* lse, const float* ent, const float* glp, const float* gent,
               void* dx, hipStream_t s) {
    const int64_t rows = (int64_t)nb * nt;
    const int64_t blocks = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
    const bool has_t = temp != 1.0f;
    hipLaunchKernelGGL((logprob_bwd_kernel<T, U, NT>), dim3((unsigned)blocks), dim3(kThreads), 0, s,
                       reinterpret_cast<const T*>(logits), sb, st, nt, rows, V, labels, lsb, lst, temp, has_t, lse,
                       ent, glp, gent, reinterpret_cast<T*>(dx));
    return check_launch("logprob_bwd_kernel");
}

template <typename T>
int launch_fwd(const void* logits, int64_t sb, int64_t st, int nb, int nt, int V, const int64_t* labels, int64_t lsb,
               int64_t lst, float temp, float* logp, float* ent, float* lse, hipStream_t s) {
    const bool nt_ = knobs().logprob_nt != 0;
    if (knobs().logprob_unroll == 8)
        return nt_ ? launch_fwd_v<T, 8, true>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, logp, ent, lse, s)
                   : launch_fwd_v<T, 8, false>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, logp, ent, lse, s);
    return nt_ ? launch_fwd_v<T, 4, true>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, logp, ent, lse, s)
               : launch_fwd_v<T, 4, false>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, logp, ent, lse, s);
}

template <typename T>
int launch_bwd(const void* logits, int64_t sb, int64_t st, int nb, int nt, int V, const int64_t* labels, int64_t lsb,
               int64_t lst, float temp, const float* lse, const float* ent, const float* glp, const float* gent,
               void* dx, hipStream_t s) {
    const bool nt_ = knobs().logprob_nt != 0;
    if (knobs().logprob_unroll == 8)
        return nt_ ? launch_bwd_v<T, 8, true>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, lse, ent, glp, gent, dx, s)
                   : launch_bwd_v<T, 8, false>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, lse, ent, glp, gent, dx, s);
    return nt_ ? launch_bwd_v<T, 4, true>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, lse, ent, glp, gent, dx, s)
               : launch_bwd_v<T, 4, false>(logits, sb, st, nb, nt, V, labels, lsb, lst, temp, lse, ent, glp, gent, dx, s);
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" int skyrl_logprob_fwd(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t nb,
                                 int32_t nt, int32_t V, const int64_t* labels, int64_t lstride_b, int64_t lstride_t,
                                 float temperature, float* logp_out, float* entropy_out, float* lse_out,
                                 void* stream) {
    SKYRL_REQUIRE(nb >= 0 && nt >= 0 && V > 0, "logprob_fwd: bad sizes");
    if ((int64_t)nb * nt == 0) return SKYRL_OK;
    SKYRL_REQUIRE(logits && labels && logp_out, "logprob_fwd: null pointer");
    SKYRL_REQUIRE(temperature > 0.f, "logprob_fwd: temperature must be > 0");
    if (dtype == SKYRL_BF16)
        return launch_fwd<uint16_t>(logits, stride_b, stride_t, nb, nt, V, labels, lstride_b, lstride_t, temperature,
                                    logp_out, entropy_out, lse_out, as_stream(stream));
    if (dtype == SKYRL_F32)
        return launch_fwd<float>(logits, stride_b, stride_t, nb, nt, V, labels, lstride_b, lstride_t, temperature,
                                 logp_out, entropy_out, lse_out, as_stream(stream));
    return fail(SKYRL_ERR_INVALID, "logprob_fwd: logits dtype must be bf16 or f32");
}

extern "C" int skyrl_logprob_bwd(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t nb,
                                 int32_t nt, int32_t V, const int64_t* labels, int64_t lstride_b, int64_t lstride_t,
                                 float temperature, const float* lse, const float* entropy, const float* grad_logp,
                                 const float* grad_entropy, void* grad_logits, void* stream) {
    SKYRL_REQUIRE(nb >= 0 && nt >= 0 && V > 0, "logprob_bwd: bad sizes");
    if ((int64_t)nb * nt == 0) return SKYRL_OK;
    SKYRL_REQUIRE(logits && labels && lse && grad_logp && grad_logits, "logprob_bwd: null pointer");
    SKYRL_REQUIRE(!grad_entropy || entropy, "logprob_bwd: grad_entropy needs entropy");
    SKYRL_REQUIRE(temperature > 0.f, "logprob_bwd: temperature must be > 0");
    if (dtype == SKYRL_BF16)
        return launch_bwd<uint16_t>(logits, stride_b, stride_t, nb, nt, V, labels, lstride_b, lstride_t, temperature,
                                    lse, entropy, grad_logp, grad_entropy, grad_logits, as_stream(stream));
    if (dtype == SKYRL_F32)
        return launch_bwd<float>(logits, stride_b, stride_t, nb, nt, V, labels, lstride_b, lstride_t, temperature,
                                 lse, entropy, grad_logp, grad_entropy, grad_logits, as_stream(stream));
    return fail(SKYRL_ERR_INVALID, "logprob_bwd: logits dtype must be bf16 or f32");
}
