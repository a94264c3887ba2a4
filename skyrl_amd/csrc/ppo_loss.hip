// a6/a7/a8: approximate KL, fused clipped policy loss (+KL-to-ref, +entropy
// term) forward/backward, reward KL penalty, clipped value loss.
//
// References (skyrl-train/skyrl_train/):
//   compute_approx_kl            utils/ppo_utils.py:88-124
//   ppo_policy_loss              utils/ppo_utils.py:548-586
//   reduce_loss                  utils/ppo_utils.py:984-1009
//   masked_mean / safe_exp_delta utils/torch_utils.py:180-192
//   loss assembly                workers/worker.py:810-876
//   apply_reward_kl_penalty      trainer.py:981-1035
//   ppo_critic_loss              utils/ppo_utils.py:175-193
//
// Layout: all per-token tensors f32 [n,R] row-major. Forward: grid (row, 1024-column chunk),
// one token per thread; it reads 20 B/token (logp, old, adv, mask, ref), writes the per-token
// gradient numerator (4 B/token) and a 5-float record per block; a one-block fold launch
// folds the records into the scalar loss,
// the metric vector and the per-row gradient scale. The backward is then a
// 12 B/token elementwise pass (numerator, scale, upstream grad).
#include "arrive.h"

// Phase timestamps for scripts/probe/phase_probe (compiled only there, never in the product).
#ifdef SKYRL_PHASE_PROBE
__device__ uint64_t g_phase[8192 * 8];
#define PHASE(k)                                                                                           \
    do {                                                                                                   \
        if (threadIdx.x == 0)                                                                              \
            g_phase[(blockIdx.x + blockIdx.y * gridDim.x) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PHASE(k) \
    do {         \
    } while (0)
#endif

namespace skyrl {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kChunk = kThreads * 4;  // columns per block
constexpr int kNP = 5;                // partials: sum l*m, m, clip*m, kl*m*m, ent*m
constexpr int kRec = 8;               // partial record stride (floats): two 16-B loads per record
constexpr int kPre = 1;               // rows per thread whose records the epilogue loads at once (1024 threads)

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// compute_approx_kl on one element (before the mask multiply).
__device__ __forceinline__ float approx_kl(float lp, float base, int kl_type) {
    switch (kl_type) {
        case 0: return lp - base;
        case 1: return fabsf(lp - base);
        case 2: { float d = lp - base; return 0.5f * (d * d); }
        default: {
            float kl = clampf(base - lp, -20.f, 20.f);
            float r = expf(kl);
            return clampf((r - kl) - 1.f, -10.f, 10.f);
        }
    }
}

struct TokenOut {
    float loss;   // per-token policy loss (before mask)
    float dldlp;  // d loss / d logp (before mask and reduction scale)
    float clip;   // (-surr2 > -surr1)
};

// ppo_policy_loss for one token, with torch-autograd gradient semantics.
__device__ __forceinline__ TokenOut ppo_token(float lp, float old, float A, float lo, float hi, float c,
                                              int dual_clip) {
    const float delta = lp - old;
    const float ratio = expf(clampf(delta, -20.f, 20.f));
    const float dratio = (delta >= -20.f && delta <= 20.f) ? ratio : 0.f;
    const float surr1 = ratio * A;
    const float rc = clampf(ratio, lo, hi);
    const float surr2 = rc * A;
    const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
    float loss1, d1;  // loss1 = -min(surr1, surr2); d1 = d loss1 / d ratio
    if (surr1 < surr2) {
        loss1 = -surr1;
        d1 = -A;
    } else if (surr2 < surr1) {
        loss1 = -surr2;
        d1 = -A * inr;
    } else {  // tie: torch.min splits the gradient in half
        loss1 = -surr1;
        d1 = -(0.5f * A + 0.5f * A * inr);
    }
    TokenOut o;
    o.clip = (-surr2 > -surr1) ? 1.f : 0.f;
    o.loss = loss1;
    float d = d1;
    if (dual_clip && A < 0.f) {
        const float pg3 = -A * c;
        if (pg3 < loss1) {
            o.loss = pg3;
            d = 0.f;
        } else if (loss1 == pg3) {
            d = 0.5f * d1;
        }
    }
    o.dldlp = d * dratio;
    return o;
}

// Grid (row, 1024-column chunk), 256 threads x 4 tokens: every thread issues its 16-B loads
// of all inputs at once, and the 4 independent tokens give the PPO/KL arithmetic (two
// accurate expf, clamps, selects) ILP within the wave. Measured at [512, 1024]: this 4-wave
// shape beats one token per thread in 1024-thread blocks (16-wave fold tail per block) and a
// wave-per-row shape (16 tokens per lane, 1 wave per SIMD).
constexpr int kFT = kThreads * 4;  // columns per block
constexpr int kFW = kThreads / kWave;

__global__ __launch_bounds__(kThreads) void ppo_loss_fwd_kernel(
    const float* __restrict__ lp, const float* __restrict__ old, const float* __restrict__ adv,
    const float* __restrict__ mask, const float* __restrict__ ref, const float* __restrict__ ent, int n,
    int R, skyrl_ppo_params p, bool vec4, float* __restrict__ gnum, float* __restrict__ partials) {
    __shared__ float s_red[kFW * kNP];
    PHASE(0);
    const int row = blockIdx.x;
    const int chunk = blockIdx.y;
    const int nchunks = gridDim.y;
    const float lo = (float)(1.0 - (double)p.eps_clip_low);
    const float hi = (float)(1.0 + (double)p.eps_clip_high);
    const int64_t rbase = (int64_t)row * R;
    float acc[kNP] = {0.f, 0.f, 0.f, 0.f, 0.f};
    auto tok = [&](float L, float O, float A, float M, float RF, float E) -> float {
        const TokenOut t = ppo_token(L, O, A, lo, hi, p.clip_ratio_c, p.dual_clip);
        acc[0] += t.loss * M;
        acc[1] += M;
        acc[2] += t.clip * M;
        if (p.use_kl_loss) acc[3] += (approx_kl(L, RF, p.kl_type) * M) * M;
        acc[4] += E * M;
        return t.dldlp * M;
    };
    const int c0 = chunk * kFT + threadIdx.x * 4;
    if (vec4) {
        if (c0 + 3 < R) {  // R % 4 == 0 on this path
            const int64_t e = rbase + c0;
            const float4 l4 = *reinterpret_cast<const float4*>(lp + e);
            const float4 o4 = *reinterpret_cast<const float4*>(old + e);
            const float4 a4 = *reinterpret_cast<const float4*>(adv + e);
            const float4 m4 = mask ? *reinterpret_cast<const float4*>(mask + e) : make_float4(1.f, 1.f, 1.f, 1.f);
            const float4 r4 = p.use_kl_loss ? *reinterpret_cast<const float4*>(ref + e) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 e4 = ent ? *reinterpret_cast<const float4*>(ent + e) : make_float4(0.f, 0.f, 0.f, 0.f);
            float4 g;
            g.x = tok(l4.x, o4.x, a4.x, m4.x, r4.x, e4.x);
            g.y = tok(l4.y, o4.y, a4.y, m4.y, r4.y, e4.y);
            g.z = tok(l4.z, o4.z, a4.z, m4.z, r4.z, e4.z);
            g.w = tok(l4.w, o4.w, a4.w, m4.w, r4.w, e4.w);
            *reinterpret_cast<float4*>(gnum + e) = g;
        }
    } else {
        for (int c = chunk * kFT + threadIdx.x; c < R && c < (chunk + 1) * kFT; c += kThreads) {
            const int64_t e = rbase + c;
            gnum[e] = tok(lp[e], old[e], adv[e], mask ? mask[e] : 1.f, p.use_kl_loss ? ref[e] : 0.f,
                          ent ? ent[e] : 0.f);
        }
    }
    PHASE(1);
    block_sum<kFW, kNP>(acc, s_red);
    if (threadIdx.x < kNP) partials[((int64_t)row * nchunks + chunk) * kRec + threadIdx.x] = acc[threadIdx.x];
    PHASE(2);
}

// The fold runs as its own one-block launch: the kernel boundary publishes every record.
// (An in-kernel last-arriver fold measured 13-16 us at n=512: each block drained its
// stores before ticking, and the folding block's tail sat behind all of that.)
constexpr int kFoldT = 256;
__global__ __launch_bounds__(kFoldT) void ppo_loss_fold_kernel(int n, int nchunks, skyrl_ppo_params p,
                                                               const float* __restrict__ partials,
                                                               float* __restrict__ loss_out, float* __restrict__ metrics,
                                                               float* __restrict__ row_scale) {
    __shared__ double s_redd[(kFoldT / kWave) * 6];
    PHASE(3);
    // ---- epilogue: one block folds the n*nchunks partials ---------------------
    // tot: 0 sum l*m, 1 sum m, 2 sum clip*m, 3 sum_rows row-reduced loss (seq modes),
    //      4 sum_rows kl_row, 5 sum ent*m
    double tot[6] = {0, 0, 0, 0, 0, 0};
    // Each thread loads the chunk-0 records of kPre rows before the first wait (one
    // dependent round trip for n <= kPre * kThreads rows), further chunks after.
    for (int r0 = threadIdx.x; r0 < n; r0 += kFoldT * kPre) {
        float4 rec[kPre][2];
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
            const int r = r0 + u * kFoldT;
            if (r < n) {
                const float4* src = reinterpret_cast<const float4*>(partials + (int64_t)r * nchunks * kRec);
                rec[u][0] = src[0];
                rec[u][1] = src[1];
            }
        }
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
            const int r = r0 + u * kFoldT;
            if (r >= n) break;
            double rs[kNP] = {rec[u][0].x, rec[u][0].y, rec[u][0].z, rec[u][0].w, rec[u][1].x};
            for (int c = 1; c < nchunks; ++c) {
                const float* src = partials + ((int64_t)r * nchunks + c) * kRec;
#pragma unroll
                for (int k = 0; k < kNP; ++k) rs[k] += (double)src[k];
            }
            const double mrow = rs[1] > 1.0 ? rs[1] : 1.0;  // mask.sum(-1).clamp(min=1)
            tot[0] += rs[0];
            tot[1] += rs[1];
            tot[2] += rs[2];
            tot[4] += rs[3] / mrow;
            tot[5] += rs[4];
            if (p.loss_reduction == 1) {
                tot[3] += rs[0] / mrow;
                row_scale[r] = (float)(1.0 / ((double)n * mrow));
            } else if (p.loss_reduction == 2) {
                tot[3] += rs[0] / (double)p.max_seq_len;
                row_scale[r] = (float)(1.0 / ((double)n * (double)p.max_seq_len));
            }
        }
    }
    PHASE(4);
    block_sum_d<kFoldT / kWave, 6>(tot, s_redd);
    const double msum = tot[1] > 1.0 ? tot[1] : 1.0;
    if (p.loss_reduction == 0) {
        const float sc = (float)(1.0 / msum);
        for (int r = threadIdx.x; r < n; r += kFoldT) row_scale[r] = sc;
    }
    if (threadIdx.x == 0) {
        float pg;
        if (p.loss_reduction == 0) pg = (float)(tot[0] / msum);
        else pg = (float)(tot[3] / (double)n);
        const float clip_ratio = (float)(tot[2] / msum);
        const float kl = p.use_kl_loss ? (float)(tot[4] / (double)n) : 0.f;
        const float entropy = (float)(tot[5] / msum);
        float final_loss = pg + kl * p.kl_loss_coef;
        if (p.use_entropy_loss) final_loss = final_loss - entropy * p.entropy_loss_coef;
        loss_out[0] = final_loss;
        metrics[SKYRL_M_FINAL_LOSS] = final_loss;
        metrics[SKYRL_M_POLICY_LOSS] = pg;
        metrics[SKYRL_M_ENTROPY] = entropy;
        metrics[SKYRL_M_KL] = kl;
        metrics[SKYRL_M_CLIP_RATIO] = clip_ratio;
        metrics[SKYRL_M_MASK_SUM] = (float)tot[1];
        metrics[6] = 0.f;
        metrics[7] = 0.f;
    }
    PHASE(5);
}

__global__ __launch_bounds__(kThreads) void ppo_loss_bwd_kernel(
    const float* __restrict__ gout, const float* __restrict__ gnum, const float* __restrict__ row_scale,
    const float* __restrict__ mask, const float* __restrict__ metrics, int R, int use_ent, float ent_coef,
    bool vec4, float* __restrict__ glp, float* __restrict__ gent) {
    const int row = blockIdx.x;
    const float g = gout[0];
    const float s = g * row_scale[row];
    float es = 0.f;
    if (use_ent) {
        const float ms = metrics[SKYRL_M_MASK_SUM];
        es = -(g * ent_coef) / (ms > 1.f ? ms : 1.f);
    }
    const int64_t rbase = (int64_t)row * R;
    const int c0 = blockIdx.y * kChunk + threadIdx.x * 4;
    if (vec4) {
        if (c0 + 3 < R) {
            float4 u = *reinterpret_cast<const float4*>(gnum + rbase + c0);
            *reinterpret_cast<float4*>(glp + rbase + c0) = make_float4(u.x * s, u.y * s, u.z * s, u.w * s);
            if (use_ent) {
                float4 m = mask ? *reinterpret_cast<const float4*>(mask + rbase + c0) : make_float4(1.f, 1.f, 1.f, 1.f);
                *reinterpret_cast<float4*>(gent + rbase + c0) = make_float4(es * m.x, es * m.y, es * m.z, es * m.w);
            }
        }
    } else {
        for (int c = blockIdx.y * kChunk + threadIdx.x; c < R && c < (blockIdx.y + 1) * kChunk; c += kThreads) {
            glp[rbase + c] = gnum[rbase + c] * s;
            if (use_ent) gent[rbase + c] = es * (mask ? mask[rbase + c] : 1.f);
        }
    }
}

// ---- compute_approx_kl, elementwise ---------------------------------------------
__global__ void approx_kl_kernel(const float* __restrict__ lp, const float* __restrict__ base,
                                 const void* __restrict__ mask, int mask_dtype, int64_t n, int kl_type,
                                 float* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float k = approx_kl(lp[i], base[i], kl_type);
        if (mask) k = k * load_mask(mask, mask_dtype, i);
        out[i] = k;
    }
}

// ---- apply_reward_kl_penalty: one block per row + last-arriver metrics ---------
__global__ __launch_bounds__(kThreads) void reward_kl_kernel(
    const float* __restrict__ rewards, const float* __restrict__ lp, const float* __restrict__ base,
    const float* __restrict__ mask, int N, int R, int kl_type, float coef, float* __restrict__ out,
    float* __restrict__ partials) {
    __shared__ float s_red[kWaves * 2];
    __shared__ float s_max[kWaves];
    const int row = blockIdx.x;
    const int64_t rbase = (int64_t)row * R;
    const float c = coef > 0.f ? coef : 0.f;  // max(0, kl_loss_coef)
    float acc[2] = {0.f, 0.f};                // sum (kl*m)*m, sum m
    float kmax = 0.f;                         // max |kl*m|
    for (int t = threadIdx.x; t < R; t += kThreads) {
        const float m = mask[rbase + t];
        const float k = approx_kl(lp[rbase + t], base[rbase + t], kl_type) * m;
        out[rbase + t] = rewards[rbase + t] - k * c;
        acc[0] += k * m;
        acc[1] += m;
        kmax = fmaxf(kmax, fabsf(k));
    }
    kmax = wave_max(kmax);
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x / kWave] = kmax;
    block_sum<kWaves, 2>(acc, s_red);  // contains __syncthreads
    if (threadIdx.x == 0) {
        float mx = s_max[0];
        for (int j = 1; j < kWaves; ++j) mx = fmaxf(mx, s_max[j]);
        partials[row * 2 + 0] = acc[0] / (acc[1] > 1.f ? acc[1] : 1.f);
        partials[row * 2 + 1] = mx;
    }
}

// One-block fold of the per-row records of reward_kl_kernel / critic_loss_kernel (its own
// launch: the kernel boundary publishes the records; see ppo_loss_fold_kernel).
// mode 0 (reward KL): metrics[0] = mean_rows rec0, metrics[1] = mean_rows rec1.
// mode 1 (critic):    out0 = 0.5 * mean_rows rec0, out1 = clip ? sum rec1 / max(sum rec2, 1) : 0.
template <int K>
__global__ __launch_bounds__(kThreads) void rows_fold_kernel(const float* __restrict__ partials, int n, int mode,
                                                            int clip, float* __restrict__ out0,
                                                            float* __restrict__ out1) {
    __shared__ double s_redd[kWaves * K];
    double tot[K];
#pragma unroll
    for (int k = 0; k < K; ++k) tot[k] = 0.0;
    for (int r = threadIdx.x; r < n; r += kThreads) {
#pragma unroll
        for (int k = 0; k < K; ++k) tot[k] += (double)partials[r * K + k];
    }
    block_sum_d<kWaves, K>(tot, s_redd);
    if (threadIdx.x != 0) return;
    if (mode == 0) {
        out0[0] = (float)(tot[0] / (double)n);
        out0[1] = (float)(tot[1] / (double)n);
    } else {
        out0[0] = 0.5f * (float)(tot[0] / (double)n);
        out1[0] = clip ? (float)(tot[1] / (tot[K - 1] > 1.0 ? tot[K - 1] : 1.0)) : 0.f;
    }
}

// ---- ppo_critic_loss -----------------------------------------------------------
__global__ __launch_bounds__(kThreads) void critic_loss_kernel(
    const float* __restrict__ V, const float* __restrict__ Vold, const float* __restrict__ ret,
    const float* __restrict__ mask, int n, int R, float vclip, float* __restrict__ gv,
    float* __restrict__ partials) {
    __shared__ float s_red[kWaves * 3];
    const int row = blockIdx.x;
    const int64_t rbase = (int64_t)row * R;
    const bool clip = vclip >= 0.f;
    float acc[3] = {0.f, 0.f, 0.f};  // sum loss*m, sum m, sum (s1>s2)*m
    for (int t = threadIdx.x; t < R; t += kThreads) {
        const int64_t i = rbase + t;
        const float m = mask ? mask[i] : 1.f;
        const float v = V[i], r = ret[i];
        float l, d, cf = 0.f;
        const float s2 = (v - r) * (v - r);
        const float ds2 = 2.f * (v - r);
        if (clip) {
            const float dv = v - Vold[i];
            const float vc = Vold[i] + clampf(dv, -vclip, vclip);
            const float s1 = (vc - r) * (vc - r);
            const float ds1 = (dv >= -vclip && dv <= vclip) ? 2.f * (vc - r) : 0.f;
            if (s1 > s2) { l = s1; d = ds1; cf = 1.f; }
            else if (s2 > s1) { l = s2; d = ds2; }
            else { l = s1; d = 0.5f * (ds1 + ds2); }
        } else {
            l = s2;
            d = ds2;
        }
        acc[0] += l * m;
        acc[1] += m;
        acc[2] += cf * m;
        gv[i] = d * m;  // scaled by 0.5/(n*max(row m,1)) below
    }
    block_sum<kWaves, 3>(acc, s_red);
    const float mrow = acc[1] > 1.f ? acc[1] : 1.f;
    const float sc = 0.5f / ((float)n * mrow);
    for (int t = threadIdx.x; t < R; t += kThreads) gv[rbase + t] *= sc;
    if (threadIdx.x == 0) {
        partials[row * 3 + 0] = acc[0] / mrow;
        partials[row * 3 + 1] = acc[2];
        partials[row * 3 + 2] = acc[1];
    }
}

inline bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % 16) == 0; }

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" size_t skyrl_ppo_loss_workspace_bytes(int32_t n, int32_t R) {
    const size_t nchunks = (size_t)((R + kFT - 1) / kFT);
    const size_t parts = (size_t)(n > 0 ? n : 1) * (nchunks ? nchunks : 1) * kRec * sizeof(float);
    return 256 + ((parts + 255) / 256) * 256;  // [counter | pad][partials]
}

extern "C" int skyrl_ppo_loss_fwd(const float* log_probs, const float* old_log_probs, const float* advantages,
                                  const float* loss_mask, const float* ref_log_probs, const float* entropy,
                                  int32_t n, int32_t R, const skyrl_ppo_params* params, float* loss_out,
                                  float* metrics_out, float* grad_num, float* row_scale, void* workspace,
                                  void* stream) {
    SKYRL_REQUIRE(params, "ppo_loss_fwd: params is null");
    SKYRL_REQUIRE(n > 0 && R > 0, "ppo_loss_fwd: empty batch");
    SKYRL_REQUIRE(log_probs && old_log_probs && advantages && loss_out && metrics_out && grad_num && row_scale &&
                      workspace,
                  "ppo_loss_fwd: null pointer");
    SKYRL_REQUIRE(!params->use_kl_loss || ref_log_probs, "ppo_loss_fwd: use_kl_loss needs ref_log_probs");
    SKYRL_REQUIRE(params->loss_reduction >= 0 && params->loss_reduction <= 2, "ppo_loss_fwd: bad loss_reduction");
    SKYRL_REQUIRE(params->loss_reduction != 2 || params->max_seq_len > 0.f,
                  "ppo_loss_fwd: seq_mean_token_sum_norm needs max_seq_len");
    SKYRL_REQUIRE(params->kl_type >= 0 && params->kl_type <= 3, "ppo_loss_fwd: bad kl_type");
    float* partials = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + 256);
    const bool vec4 = (R % 4) == 0 && aligned16(log_probs) && aligned16(old_log_probs) && aligned16(advantages) &&
                      aligned16(loss_mask) && aligned16(ref_log_probs) && aligned16(entropy) && aligned16(grad_num);
    dim3 grid(n, (R + kFT - 1) / kFT);
    hipLaunchKernelGGL(ppo_loss_fwd_kernel, grid, dim3(kThreads), 0, as_stream(stream), log_probs, old_log_probs,
                       advantages, loss_mask, ref_log_probs, entropy, n, R, *params, vec4, grad_num, partials);
    int rc = check_launch("ppo_loss_fwd_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(ppo_loss_fold_kernel, dim3(1), dim3(kFoldT), 0, as_stream(stream), n, (int)grid.y, *params,
                       partials, loss_out, metrics_out, row_scale);
    return check_launch("ppo_loss_fold_kernel");
}

extern "C" int skyrl_ppo_loss_bwd(const float* grad_out, const float* grad_num, const float* row_scale,
                                  const float* loss_mask, const float* metrics, int32_t n, int32_t R,
                                  const skyrl_ppo_params* params, float* grad_logp, float* grad_entropy,
                                  void* stream) {
    SKYRL_REQUIRE(params && grad_out && grad_num && row_scale && grad_logp && metrics, "ppo_loss_bwd: null pointer");
    SKYRL_REQUIRE(n > 0 && R > 0, "ppo_loss_bwd: empty batch");
    const int use_ent = params->use_entropy_loss && grad_entropy != nullptr;
    const bool vec4 = (R % 4) == 0 && aligned16(grad_num) && aligned16(grad_logp) && aligned16(loss_mask) &&
                      aligned16(grad_entropy);
    dim3 grid(n, (R + kChunk - 1) / kChunk);
    hipLaunchKernelGGL(ppo_loss_bwd_kernel, grid, dim3(kThreads), 0, as_stream(stream), grad_out, grad_num, row_scale,
                       loss_mask, metrics, R, use_ent, params->entropy_loss_coef, vec4, grad_logp, grad_entropy);
    return check_launch("ppo_loss_bwd_kernel");
}

extern "C" int skyrl_approx_kl(const float* log_probs, const float* log_probs_base, const void* loss_mask,
                               int mask_dtype, int64_t n, int32_t kl_type, float* kl_out, void* stream) {
    SKYRL_REQUIRE(kl_type >= 0 && kl_type <= 3, "approx_kl: bad kl_type");
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(log_probs && log_probs_base && kl_out, "approx_kl: null pointer");
    const int threads = 256;
    int64_t blocks = (n + threads - 1) / threads;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(approx_kl_kernel, dim3((unsigned)blocks), dim3(threads), 0, as_stream(stream), log_probs,
                       log_probs_base, loss_mask, mask_dtype, n, kl_type, kl_out);
    return check_launch("approx_kl_kernel");
}

extern "C" size_t skyrl_reward_kl_workspace_bytes(int32_t N) {
    return 256 + (((size_t)N * 2 * sizeof(float) + 255) / 256) * 256;
}

extern "C" int skyrl_reward_kl_penalty(const float* rewards, const float* action_log_probs,
                                          const float* base_action_log_probs, const float* loss_mask, int32_t N,
                                          int32_t R, int32_t kl_type, float kl_coef, float* rewards_out,
                                          float* metrics_out, void* workspace, void* stream) {
    SKYRL_REQUIRE(N > 0 && R > 0, "reward_kl_penalty: empty batch");
    SKYRL_REQUIRE(rewards && action_log_probs && base_action_log_probs && loss_mask && rewards_out && metrics_out &&
                      workspace,
                  "reward_kl_penalty: null pointer");
    SKYRL_REQUIRE(kl_type >= 0 && kl_type <= 3, "reward_kl_penalty: bad kl_type");
    float* partials = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + 256);
    hipLaunchKernelGGL(reward_kl_kernel, dim3(N), dim3(kThreads), 0, as_stream(stream), rewards, action_log_probs,
                       base_action_log_probs, loss_mask, N, R, kl_type, kl_coef, rewards_out, partials);
    int rc = check_launch("reward_kl_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(rows_fold_kernel<2>, dim3(1), dim3(kThreads), 0, as_stream(stream), partials, N, 0, 0,
                       metrics_out, nullptr);
    return check_launch("reward_kl_kernel");
}

extern "C" size_t skyrl_critic_loss_workspace_bytes(int32_t n, int32_t R) {
    (void)R;
    return 256 + (((size_t)n * 3 * sizeof(float) + 255) / 256) * 256;
}

extern "C" int skyrl_critic_loss_fwd(const float* values, const float* old_values, const float* returns,
                                     const float* loss_mask, int32_t n, int32_t R, float value_clip, float* loss_out,
                                     float* clipfrac_out, float* grad_values, void* workspace, void* stream) {
    SKYRL_REQUIRE(n > 0 && R > 0, "critic_loss: empty batch");
    SKYRL_REQUIRE(values && returns && loss_out && clipfrac_out && grad_values && workspace,
                  "critic_loss: null pointer");
    SKYRL_REQUIRE(value_clip < 0.f || old_values, "critic_loss: value_clip needs old_values");
    float* partials = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + 256);
    hipLaunchKernelGGL(critic_loss_kernel, dim3(n), dim3(kThreads), 0, as_stream(stream), values, old_values, returns,
                       loss_mask, n, R, value_clip, grad_values, partials);
    int rc = check_launch("critic_loss_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(rows_fold_kernel<3>, dim3(1), dim3(kThreads), 0, as_stream(stream), partials, n, 1,
                       value_clip >= 0.f ? 1 : 0, loss_out, clipfrac_out);
    return check_launch("critic_loss_kernel");
}
