// a9: experience pack (ragged CSR -> padded training tensors) fused with
// pad_batch, plus small utilities (gradient bucket scaling / sum of squares,
// scalar-scaled copies for autograd backward).
//
// Reference: convert_prompts_responses_to_batch_tensors
// (skyrl-train/skyrl_train/dataset/preprocess.py:28-132): left-padded prompt |
// right-padded response, int64 sequences/attention/response masks, f32
// rewards/loss masks, rollout logprobs zero-padded; pad_batch
// (trainer.py:872-907): rows N..N+pad-1 clone rows 0..pad-1, loss_mask 0.
//
// Pure byte movement (HBM-bound, ~23 MB at N=512, P=512, R=1024): grid =
// (output row, 1024-column tile); each thread writes four adjacent columns of every
// output with 16-B stores when the row widths allow it.
#include "common.h"

namespace skyrl {
namespace {

constexpr int kThreads = 256;
constexpr int kQ = 4;                  // columns per thread
constexpr int kCols = kThreads * kQ;   // columns per workgroup

// Output row i (< N: sample i; >= N: pad row cloning sample i - N with loss_mask 0). Each
// thread produces kQ adjacent columns; with VEC (row widths multiple of kQ, 16-B aligned
// bases) every output is written with full 16-B stores, one instruction per array and
// thread, so each wave store covers whole cache lines.
template <bool VEC>
__global__ __launch_bounds__(kThreads) void pack_kernel(skyrl_pack_inputs in, int N, int P, int R, int64_t pad_id,
                                                        int64_t* __restrict__ seq, int64_t* __restrict__ att,
                                                        int64_t* __restrict__ rmask, float* __restrict__ rew,
                                                        float* __restrict__ lmask, float* __restrict__ rlp,
                                                        float* __restrict__ lm_rowsum, float* __restrict__ rw_rowsum) {
    const int i = blockIdx.x;
    const int src = i < N ? i : i - N;
    const bool is_pad = i >= N;
    const int S = P + R;
    const int64_t p0 = in.prompt_off[src];
    const int plen = (int)(in.prompt_off[src + 1] - p0);
    const int lpad = P - plen;
    const int64_t r0 = in.response_off[src];
    const int rlen = (int)(in.response_off[src + 1] - r0);
    const int64_t w0 = in.reward_off[src];
    const int wl = (int)(in.reward_off[src + 1] - w0);
    const int64_t m0 = in.loss_mask_off[src];
    const int ml = is_pad ? 0 : (int)(in.loss_mask_off[src + 1] - m0);
    const int64_t l0 = rlp ? in.logprob_off[src] : 0;
    const int ll = rlp ? (int)(in.logprob_off[src + 1] - l0) : 0;
    const int c0 = blockIdx.y * kCols + threadIdx.x * kQ;
    const int64_t so = (int64_t)i * S;
    const int64_t ro = (int64_t)i * R;
    int64_t tk[kQ], at[kQ], rm[kQ];
    float rw[kQ], lm[kQ], lp[kQ];
#pragma unroll
    for (int k = 0; k < kQ; ++k) {
        const int c = c0 + k;
        if (c < P) {
            const bool real = c >= lpad;
            tk[k] = real ? in.prompt_tokens[p0 + (c - lpad)] : pad_id;
            at[k] = real;
        } else {
            const int j = c - P;
            const bool real = j < rlen && c < S;
            tk[k] = real ? in.response_tokens[r0 + j] : pad_id;
            at[k] = real;
        }
        rm[k] = c < rlen;
        rw[k] = c < wl ? in.reward_vals[w0 + c] : 0.f;
        lm[k] = c < ml ? in.loss_mask_vals[m0 + c] : 0.f;
        lp[k] = c < ll ? in.logprob_vals[l0 + c] : 0.f;
    }
    if (lm_rowsum && blockIdx.y == 0) {  // per-row loss-mask sum for the loss's reduction scales
        __shared__ float s_red[kThreads / kWave];
        float acc[1] = {0.f};
        for (int c = threadIdx.x; c < ml && c < R; c += kThreads) acc[0] += in.loss_mask_vals[m0 + c];
        block_sum<kThreads / kWave, 1>(acc, s_red);
        if (threadIdx.x == 0) lm_rowsum[i] = acc[0];
    }
    if (rw_rowsum && blockIdx.y == 0 && threadIdx.x < kWave) {
        // GRPO score = sum of the padded reward row, summed in grpo.hip's order (row_sum_wave: lane
        // l adds the 4-element groups l, l + 64, ... as (x0 + x1) + (x2 + x3), then the wave tree),
        // so skyrl_grpo_advantage / skyrl_grpo_ppo_loss_fwd given these scores produce what they
        // compute from the padded rewards themselves
        const int lane = threadIdx.x;
        const int lim = wl < R ? wl : R;
        float acc = 0.f;
        for (int q = lane; 4 * q < lim; q += kWave) {
            float x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = 4 * q + k < lim ? in.reward_vals[w0 + 4 * q + k] : 0.f;
            acc += (x[0] + x[1]) + (x[2] + x[3]);
        }
        acc = wave_sum(acc);
        if (lane == 0) rw_rowsum[i] = acc;
    }
    if (VEC) {
        if (c0 < S) {
            longlong2* s2 = reinterpret_cast<longlong2*>(seq + so + c0);
            longlong2* a2 = reinterpret_cast<longlong2*>(att + so + c0);
            s2[0] = make_longlong2(tk[0], tk[1]);
            s2[1] = make_longlong2(tk[2], tk[3]);
            a2[0] = make_longlong2(at[0], at[1]);
            a2[1] = make_longlong2(at[2], at[3]);
        }
        if (c0 < R) {
            longlong2* m2 = reinterpret_cast<longlong2*>(rmask + ro + c0);
            m2[0] = make_longlong2(rm[0], rm[1]);
            m2[1] = make_longlong2(rm[2], rm[3]);
            *reinterpret_cast<float4*>(rew + ro + c0) = make_float4(rw[0], rw[1], rw[2], rw[3]);
            *reinterpret_cast<float4*>(lmask + ro + c0) = make_float4(lm[0], lm[1], lm[2], lm[3]);
            if (rlp) *reinterpret_cast<float4*>(rlp + ro + c0) = make_float4(lp[0], lp[1], lp[2], lp[3]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kQ; ++k) {
            const int c = c0 + k;
            if (c < S) {
                seq[so + c] = tk[k];
                att[so + c] = at[k];
            }
            if (c < R) {
                rmask[ro + c] = rm[k];
                rew[ro + c] = rw[k];
                lmask[ro + c] = lm[k];
                if (rlp) rlp[ro + c] = lp[k];
            }
        }
    }
}

__global__ void scale_sumsq_kernel(float* __restrict__ g, int64_t n, float scale, float* __restrict__ sumsq) {
    float acc = 0.f;
    const int64_t n4 = n / 4;
    float4* g4 = reinterpret_cast<float4*>(g);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        float4 v = g4[i];
        v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
        g4[i] = v;
        acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = g[i] * scale;
        g[i] = v;
        acc += v * v;
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0 && sumsq) atomicAdd(sumsq, acc);
}

__global__ void scale_by_scalar_kernel(const float* __restrict__ s, const float* __restrict__ in,
                                       float* __restrict__ out, int64_t n) {
    const float g = s[0];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = g * in[i];
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" int skyrl_pack_experience(const skyrl_pack_inputs* in, int32_t N, int32_t pad, int32_t P, int32_t R,
                                     int64_t pad_token_id, int64_t* sequences, int64_t* attention_mask,
                                     int64_t* response_mask, float* rewards, float* loss_mask,
                                     float* rollout_logprobs, float* loss_mask_row_sum, float* reward_row_sum,
                                     void* stream) {
    SKYRL_REQUIRE(in, "pack: inputs is null");
    SKYRL_REQUIRE(N > 0 && pad >= 0 && pad <= N && P >= 0 && R >= 0, "pack: bad sizes");
    SKYRL_REQUIRE(in->prompt_tokens && in->prompt_off && in->response_tokens && in->response_off && in->reward_vals &&
                      in->reward_off && in->loss_mask_vals && in->loss_mask_off,
                  "pack: null input pointer");
    SKYRL_REQUIRE(!rollout_logprobs || (in->logprob_vals && in->logprob_off), "pack: logprobs requested but absent");
    SKYRL_REQUIRE(sequences && attention_mask && response_mask && rewards && loss_mask, "pack: null output pointer");
    const int S = P + R;
    int cols = S > R ? S : R;
    if (cols == 0 && !loss_mask_row_sum && !reward_row_sum) return SKYRL_OK;
    if (cols == 0) cols = 1;
    dim3 grid(N + pad, (cols + kCols - 1) / kCols);
    auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool vec = S % kQ == 0 && R % kQ == 0 && a16(sequences) && a16(attention_mask) && a16(response_mask) &&
                     a16(rewards) && a16(loss_mask) && (!rollout_logprobs || a16(rollout_logprobs));
    if (vec)
        hipLaunchKernelGGL(pack_kernel<true>, grid, dim3(kThreads), 0, as_stream(stream), *in, N, P, R, pad_token_id,
                           sequences, attention_mask, response_mask, rewards, loss_mask, rollout_logprobs,
                           loss_mask_row_sum, reward_row_sum);
    else
        hipLaunchKernelGGL(pack_kernel<false>, grid, dim3(kThreads), 0, as_stream(stream), *in, N, P, R, pad_token_id,
                           sequences, attention_mask, response_mask, rewards, loss_mask, rollout_logprobs,
                           loss_mask_row_sum, reward_row_sum);
    return check_launch("pack_kernel");
}

extern "C" int skyrl_scale_and_sumsq(float* grads, int64_t n, float scale, float* sumsq_out, void* stream) {
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(grads && (reinterpret_cast<uintptr_t>(grads) % 16) == 0, "scale_and_sumsq: null/misaligned grads");
    int64_t blocks = (n / 4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(scale_sumsq_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), grads, n, scale,
                       sumsq_out);
    return check_launch("scale_sumsq_kernel");
}

extern "C" int skyrl_scale_by_device_scalar(const float* g, const float* in, float* out, int64_t n, void* stream) {
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(g && in && out, "scale_by_device_scalar: null pointer");
    int64_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(scale_by_scalar_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), g, in, out, n);
    return check_launch("scale_by_scalar_kernel");
}
