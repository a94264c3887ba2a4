// Fused policy training pass (a2 + a3 + a6 + a7): logprob/entropy forward, the PPO
// clipped loss + KL(ref) + entropy term, and the logprob backward in ONE sweep pair over
// the vocabulary per token.
//
// Why fusable: for regular/dual_clip PPO the gradient of the micro-batch loss w.r.t.
// logp_t is dl/dlogp(logp_t, old_t, adv_t) * m_t * scale(row), where scale depends only
// on the loss mask (token_mean: 1/max(sum m,1); sequence_mean: 1/(n*max(row sum,1));
// seq_mean_token_sum_norm: 1/(n*max_seq_len)), and the entropy-loss gradient is
// -coef * m_t / max(sum m, 1); the KL term has no gradient (compute_approx_kl is
// @torch.no_grad(), ppo_utils.py:87). So dlogits for a unit upstream gradient are known
// as soon as the row's logsumexp is; a non-unit upstream gradient rescales them after.
// Reference semantics: model_wrapper.py:313-370, ppo_utils.py:88-124,548-586,984-1009,
// workers/worker.py:810-876, torch_utils.py:59-192.
//
// Launches per micro-batch:
//   1. train_scales_kernel   (1 block): mask sums -> per-row gradient scale, D
//   2. policy_train_kernel   (1 block of 1024 threads per token): sweep 1 reads the
//      row from HBM (online max / sum-exp / entropy, label logit), the token's loss terms
//      and gradient coefficients, sweep 2 re-reads the row -- 300 KB, issued right after
//      sweep 1, with <= 2 rows in flight per CU (<= 154 MB chip-wide), so it is served by
//      the 256 MB Infinity Cache -- and writes dlogits (bf16).
//   3. train_epilogue_kernel (1 block): folds the per-token terms into the loss scalar
//      and the metric vector (same layout as skyrl_ppo_loss_fwd).
// HBM traffic per token: V*2 (read) + V*2 (write) vs V*2 + V*2 + V*2 unfused.
#include <utility>

#include "arrive.h"
#include "variant.h"

// Phase timestamps for scripts/probe/train_phase_probe (compiled only there, never in the product).
#ifdef SKYRL_TRAIN_PHASE_PROBE
__device__ uint64_t g_tphase[16384 * 8];
#define TPHASE(k)                                                                                       \
    do {                                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < 16384) {                                                   \
            g_tphase[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                          \
            if ((k) == 0) g_tphase[blockIdx.x * 8 + 7] = (uint64_t)__smid();                            \
        }                                                                                               \
    } while (0)
#else
#define TPHASE(k) \
    do {          \
    } while (0)
#endif

namespace skyrl {
namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / kWave;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kDLow = -1.0e30f;

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// dlogits are written once and not re-read here: optionally non-temporal (the variant field train_ntstore)
__device__ __forceinline__ void st_out(uint4* p, uint4 v, bool nts) {
    if (nts) __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(p));
    else *p = v;
}

__device__ __forceinline__ void unpack8(const uint4& v, float (&x)[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        x[2 * k] = __uint_as_float(w[k] << 16);
        x[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
}

struct St {
    float m, s, w;
};
__device__ __forceinline__ void st_add8(St& st, const float (&x)[8]) {
    float mx = x[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) mx = fmaxf(mx, x[k]);
    const float mn = fmaxf(st.m, mx);
    const float dy = fmaxf((st.m - mn) * kLog2e, kDLow);
    const float a = fast_exp2(dy);
    st.w = a * fmaf(dy, st.s, st.w);
    st.s = a * st.s;
    st.m = mn;
    const float c = -mn * kLog2e;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float y = fmaxf(fmaf(x[k], kLog2e, c), kDLow);
        const float e = fast_exp2(y);
        st.s += e;
        st.w = fmaf(e, y, st.w);
    }
}
__device__ __forceinline__ void st_merge(St& a, const St& b) {
    const float mn = fmaxf(a.m, b.m);
    const float da = fmaxf((a.m - mn) * kLog2e, kDLow), db = fmaxf((b.m - mn) * kLog2e, kDLow);
    const float ea = fast_exp2(da), eb = fast_exp2(db);
    a.w = ea * fmaf(da, a.s, a.w) + eb * fmaf(db, b.s, b.w);
    a.s = ea * a.s + eb * b.s;
    a.m = mn;
}

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

// ppo_policy_loss per token with torch-autograd gradient semantics (see ppo_loss.hip).
__device__ __forceinline__ void ppo_token(float lp, float old, float A, float lo, float hi, float c, int dual,
                                          float& loss, float& dldlp, float& clip) {
    const float delta = lp - old;
    const float ratio = expf(clampf(delta, -20.f, 20.f));
    const float dratio = (delta >= -20.f && delta <= 20.f) ? ratio : 0.f;
    const float surr1 = ratio * A;
    const float surr2 = clampf(ratio, lo, hi) * A;
    const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
    float l1, d1;
    if (surr1 < surr2) { l1 = -surr1; d1 = -A; }
    else if (surr2 < surr1) { l1 = -surr2; d1 = -A * inr; }
    else { l1 = -surr1; d1 = -(0.5f * A + 0.5f * A * inr); }
    clip = (-surr2 > -surr1) ? 1.f : 0.f;
    loss = l1;
    float d = d1;
    if (dual && A < 0.f) {
        const float pg3 = -A * c;
        if (pg3 < l1) { loss = pg3; d = 0.f; }
        else if (l1 == pg3) { d = 0.5f * d1; }
    }
    dldlp = d * dratio;
}

// ---- 1. mask statistics -> gradient scales -------------------------------------------
// Sum of one loss-mask row by one wave: lane l takes the 16-B vectors l, l + 64, ... as
// (x + y) + (z + w) in vector order (scalars t = l, l + 64, ... when the row is not 16-B aligned
// or R % 4 != 0), then the wave's xor-butterfly sum; a NULL mask counts R. The per-call scales and
// the step plan both sum rows this way, and total a micro-batch's rows in row order (fp64), so
// they derive the same bits.
__device__ __forceinline__ float mask_row_sum(const float* __restrict__ row, int R) {
    const int lane = threadIdx.x & 63;
    if (!row) return (float)R;
    float acc = 0.f;
    if ((R & 3) == 0 && (reinterpret_cast<uintptr_t>(row) & 15) == 0) {
        const float4* r4 = reinterpret_cast<const float4*>(row);
#pragma unroll 4
        for (int i = lane; i < (R >> 2); i += kWave) {
            const float4 v = r4[i];
            acc += (v.x + v.y) + (v.z + v.w);
        }
    } else {
#pragma unroll 8
        for (int t = lane; t < R; t += kWave) acc += row[t];
    }
    return wave_sum(acc);
}
__device__ __forceinline__ float row_scale_of(const skyrl_ppo_params& p, float acc, int n) {
    const double mrow = acc > 1.f ? acc : 1.0;
    if (p.loss_reduction == 1) return (float)(1.0 / ((double)n * mrow));
    return (float)(1.0 / ((double)n * (double)p.max_seq_len));  // (reduction 2; token_mean is set from D)
}
// scal[0] = sum m, scal[1] = entropy-gradient scale (-coef / D or 0), scal[2] = 1 / D with
// D = max(sum m, 1); row_scale[b] = 1 / D (token_mean) or the per-row scale.
__device__ __forceinline__ void write_scales(const skyrl_ppo_params& p, double all, float* __restrict__ scal) {
    const double d = all > 1.0 ? all : 1.0;
    scal[0] = (float)all;
    scal[1] = p.use_entropy_loss ? (float)(-(double)p.entropy_loss_coef / d) : 0.f;
    scal[2] = (float)(1.0 / d);
}

// One block: rows strided over the 16 waves; the row sums staged in row_scale, totalled by
// thread 0 in row order, then every row's scale.
// Header word 16 is the split kernel's exchange tag for the launch(es) these scales serve:
// the single-call entries advance it by one per launch; the step plan (skyrl_policy_train_plan)
// gives micro-batch k the tag (c << 12) | k with c its slot's own counter, so every launch of
// every step carries a tag no other launch that shares the granules carries.
__device__ __forceinline__ void scales_body(const float* __restrict__ mask, int n, int R, const skyrl_ppo_params& p,
                                            float* __restrict__ row_scale, float* __restrict__ scal, int step_k) {
    __shared__ double s_all;
    const int lane = threadIdx.x & 63, w = threadIdx.x / kWave;
    for (int b = w; b < n; b += kWaves) {
        const float acc = mask_row_sum(mask ? mask + (int64_t)b * R : nullptr, R);
        if (lane == 0) row_scale[b] = acc;
    }
    __threadfence_block();
    __syncthreads();
    if (threadIdx.x == 0) {
        double all = 0.0;
        for (int b = 0; b < n; ++b) all += (double)row_scale[b];
        s_all = all;
        write_scales(p, all, scal);
        // this launch's tag for the split kernel's exchange granules (header word 16, see
        // skyrl_policy_train_fwd); the previous launch's granules carry the previous tag
        unsigned* epoch = reinterpret_cast<unsigned*>(scal) + 16;
        epoch[0] = step_k < 0 ? epoch[0] + 1u : ((((epoch[0] >> 12) + 1u) << 12) | (unsigned)step_k);
    }
    __syncthreads();
    const double d = s_all > 1.0 ? s_all : 1.0;
    for (int b = threadIdx.x; b < n; b += kThreads)
        row_scale[b] = p.loss_reduction == 0 ? (float)(1.0 / d) : row_scale_of(p, row_scale[b], n);
}

__global__ __launch_bounds__(kThreads) void train_scales_kernel(const float* __restrict__ mask, int n, int R,
                                                                skyrl_ppo_params p, float* __restrict__ row_scale,
                                                                float* __restrict__ scal) {
    scales_body(mask, n, R, p, row_scale, scal, -1);
}

constexpr int kStepSlot = 256;
// micro slot words (kStepSlot bytes each): 0..2 scal floats, 16 the exchange tag, 32 the error
// flag, 33 recomputed partner states (diagnostics), 40 / 41 the plan's / fold's arrival counters
constexpr int kSlotPlanCtr = 40, kSlotFoldCtr = 41;
constexpr int kStepRows = 2;  // rows (one wave each) per block of the step plan and fold

// The step plan: one wave per row of the mini-batch (2 rows per block: n_total / 2 blocks). A row's
// wave sums its loss mask (mask_row_sum), stores it write-through and adds to its micro-batch's
// counter; the wave whose add comes last totals the micro-batch's rows in row order (fp64, the
// per-call scales' order and bits), writes the micro slot's scalars and tag and every row scale.
// Hand-off without an acquire (MI355X_MICROARCH.md's valid sc1 form: sc1 stores by the adding
// lane, drained; the last adder's wave reads them with sc1 loads).
// With GRPO (scores != NULL, contiguous groups of G rows): the wave also writes its row's advantages,
// adv = (score - mean) / (std + eps) (fp64 group stats in j order, compute_grpo_outcome_advantage,
// ppo_utils.py:1132-1182, the same arithmetic as grpo_adv_contig_kernel) times the response mask.
template <int MDT>
__global__ __launch_bounds__(kStepRows * kWave) void train_plan_kernel(
    const float* __restrict__ mask, int n_total, int R, int mb, skyrl_ppo_params p, float* __restrict__ row_scale,
    float* __restrict__ rsum, char* __restrict__ slots, const float* __restrict__ scores,
    const void* __restrict__ rmask, int G, float eps, int norm_by_std, float* __restrict__ adv,
    const float* __restrict__ pack_rsum) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * kStepRows + threadIdx.x / kWave;
    if (b >= n_total) return;
    const int k = b / mb;
    const int r0 = k * mb;
    const int n = min(n_total, r0 + mb) - r0;
    float* scal = reinterpret_cast<float*>(slots + (size_t)k * kStepSlot);
    unsigned* ctr = reinterpret_cast<unsigned*>(scal) + kSlotPlanCtr;
    // pack_rsum (skyrl_pack_experience's loss-mask row sums): every wave totals its micro-batch's
    // rows itself (row order, fp64): no mask read and no arrival; else the row's own sum here
    // (micro-batches of up to 64 rows: one load of all its row sums, first)
    const float vrow = pack_rsum && n <= kWave ? pack_rsum[r0 + min(lane, n - 1)] : 0.f;
    const float acc = pack_rsum ? (n <= kWave ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vrow), b - r0))
                                              : pack_rsum[b])
                                : mask_row_sum(mask + (int64_t)b * R, R);
    unsigned prev = 0;
    if (pack_rsum) {
        if (lane == 0 && p.loss_reduction != 0) row_scale[b] = row_scale_of(p, acc, n);
    } else if (lane == 0) {
        if (p.loss_reduction != 0) row_scale[b] = row_scale_of(p, acc, n);
        st_wt(rsum + b, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (scores) {  // GRPO: this row's advantages (overlaps the arrival's round trip)
        const int g0 = b - b % G;
        const float sj = lane < G ? scores[g0 + lane] : 0.f;
        // the response mask's loads (up to R = 1024) issued with the scores', before the group
        // statistics they do not depend on (clamped indices: unconditional loads)
        constexpr int kPre = 4;
        const int nq = R >> 2;
        const bool pre = (R & 3) == 0 && nq <= kPre * kWave;
        float mm[kPre][4];
        if (pre) {
#pragma unroll
            for (int u = 0; u < kPre; ++u) load_mask4(rmask, MDT, (int64_t)b * R + 4 * min(lane + u * kWave, nq - 1), mm[u]);
        }
        auto lane_score = [&](int j) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sj), j)); };
        float mean_f, denom_f;
        if (G <= 1) {
            mean_f = 0.f;  // singleton group: mean 0, std 1 (ppo_utils.py:1167-1169)
            denom_f = norm_by_std ? (1.f + eps) : 1.f;
        } else {  // fp64 like torch.std on CPU, j in order
            double sum = 0.0;
            for (int j = 0; j < G; ++j) sum += (double)lane_score(j);
            const double mean = sum / (double)G;
            double m2 = 0.0;
            for (int j = 0; j < G; ++j) {
                const double d = (double)lane_score(j) - mean;
                m2 += d * d;
            }
            mean_f = (float)mean;
            const float std_f = (float)sqrt(m2 / (double)(G - 1));
            denom_f = norm_by_std ? (std_f + eps) : 1.f;
        }
        const float sc = lane_score(b - g0);
        const float a = norm_by_std ? (sc - mean_f) / denom_f : (sc - mean_f);
        float* orow = adv + (int64_t)b * R;
        if (pre) {
            float4* o4 = reinterpret_cast<float4*>(orow);
#pragma unroll
            for (int u = 0; u < kPre; ++u)
                if (lane + u * kWave < nq) o4[lane + u * kWave] = make_float4(a * mm[u][0], a * mm[u][1], a * mm[u][2], a * mm[u][3]);
        } else if ((R & 3) == 0) {
            float4* o4 = reinterpret_cast<float4*>(orow);
#pragma unroll 4
            for (int i = lane; i < (R >> 2); i += kWave) {
                float mm[4];
                load_mask4(rmask, MDT, (int64_t)b * R + 4 * i, mm);
                o4[i] = make_float4(a * mm[0], a * mm[1], a * mm[2], a * mm[3]);
            }
        } else {
            for (int t = lane; t < R; t += kWave) orow[t] = a * load_mask(rmask, MDT, (int64_t)b * R + t);
        }
    }
    double all = 0.0;
    if (pack_rsum) {  // every wave: the micro-batch's total; the wave of its first row writes the slot
        if (n <= kWave) {
            for (int j = 0; j < n; ++j) all += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(vrow), j));
        } else {
            for (int j0 = 0; j0 < n; j0 += kWave) {
                const float v = j0 + lane < n ? pack_rsum[r0 + j0 + lane] : 0.f;
                for (int j = 0; j < kWave && j0 + j < n; ++j)
                    all += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
            }
        }
        if (p.loss_reduction == 0 && lane == 0) row_scale[b] = (float)(1.0 / (all > 1.0 ? all : 1.0));
        if (b != r0) return;
        if (lane == 0) {
            write_scales(p, all, scal);
            unsigned* epoch = reinterpret_cast<unsigned*>(scal) + 16;
            epoch[0] = (((epoch[0] >> 12) + 1u) << 12) | (unsigned)k;
        }
        return;
    }
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev != (unsigned)n - 1u) return;
    handoff_acquire();
    // the micro-batch's last row: total in row order, scalars, tag, token_mean scales
    for (int j0 = 0; j0 < n; j0 += kWave) {
        const float v = j0 + lane < n ? __hip_atomic_load(rsum + r0 + j0 + lane, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        for (int j = 0; j < kWave && j0 + j < n; ++j)
            all += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
    }
    if (lane == 0) {
        write_scales(p, all, scal);
        unsigned* epoch = reinterpret_cast<unsigned*>(scal) + 16;
        epoch[0] = (((epoch[0] >> 12) + 1u) << 12) | (unsigned)k;
        __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    if (p.loss_reduction == 0) {
        const double d = all > 1.0 ? all : 1.0;
        for (int j = lane; j < n; j += kWave) row_scale[r0 + j] = (float)(1.0 / d);
    }
}

// ---- 2. fused sweep pair per token ------------------------------------------------------
// tok[r*4 + {0,1,2,3}] = loss*m, clip*m, kl*m*m, ent*m
__global__ __launch_bounds__(kThreads) void policy_train_kernel(
    const uint16_t* __restrict__ logits, int64_t sb, int64_t st_, int R, int64_t rows, int V,
    const int64_t* __restrict__ labels, int64_t lsb, int64_t lst, float temp, bool has_t,
    const float* __restrict__ old, const float* __restrict__ adv, const float* __restrict__ mask,
    const float* __restrict__ ref, const float* __restrict__ row_scale, const float* __restrict__ scal,
    skyrl_ppo_params p, float* __restrict__ logp_out, float* __restrict__ ent_out, float* __restrict__ tok,
    uint16_t* __restrict__ dx, int64_t gsb, int64_t gst, bool nts) {
    __shared__ St s_st[kWaves];
    __shared__ float s_g[3];  // lse, g_lp, g_ent*... (see below)
    __shared__ float s_h;
    const int64_t r = blockIdx.x;
    const int64_t b = r / R, t = r % R;
    const uint16_t* row = logits + b * sb + t * st_;
    uint16_t* out = dx + b * gsb + t * gst;
    const int lane = threadIdx.x & 63;
    const int nvec = V / 8;
    const bool vec_ok = (reinterpret_cast<uintptr_t>(row) % 16) == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0;
    auto tval = [&](float x) { return has_t ? bf16_to_f32(f32_to_bf16(x / temp)) : x; };

    // ---- sweep 1: online softmax state
    St st{-3.402823466e38f, 0.f, 0.f};
    int done = 0;
    if (vec_ok) {
        const uint4* rv = reinterpret_cast<const uint4*>(row);
        int i = threadIdx.x;
        for (; i + 3 * kThreads < nvec; i += 4 * kThreads) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = rv[i + u * kThreads];  // default policy: keep for sweep 2
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float x[8];
                unpack8(v[u], x);
                if (has_t) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) x[k] = tval(x[k]);
                }
                st_add8(st, x);
            }
        }
        for (; i < nvec; i += kThreads) {
            float x[8];
            unpack8(rv[i], x);
            if (has_t) {
#pragma unroll
                for (int k = 0; k < 8; ++k) x[k] = tval(x[k]);
            }
            st_add8(st, x);
        }
        done = nvec * 8;
    }
    for (int v = done + threadIdx.x; v < V; v += kThreads) {
        float x[8];
        const float xv = tval(bf16_to_f32(row[v]));
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = k == 0 ? xv : -INFINITY;
        st_add8(st, x);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        St o{__shfl_xor(st.m, off, kWave), __shfl_xor(st.s, off, kWave), __shfl_xor(st.w, off, kWave)};
        st_merge(st, o);
    }
    if (lane == 0) s_st[threadIdx.x / kWave] = st;
    __syncthreads();
    if (threadIdx.x == 0) {
        St a = s_st[0];
        for (int j = 1; j < kWaves; ++j) st_merge(a, s_st[j]);
        const float logs = fast_log2(a.s) * kLn2;
        const float lse = a.m + logs;
        const float H = logs - kLn2 * (a.w / a.s);
        const int64_t lab = labels[b * lsb + t * lst];
        const float xl = (lab >= 0 && lab < V) ? tval(bf16_to_f32(row[lab])) : __builtin_nanf("");
        const float lp = xl - lse;
        const float m = mask ? mask[r] : 1.f;
        const float lo = (float)(1.0 - (double)p.eps_clip_low), hi = (float)(1.0 + (double)p.eps_clip_high);
        float loss, dl, clip;
        ppo_token(lp, old[r], adv[r], lo, hi, p.clip_ratio_c, p.dual_clip, loss, dl, clip);
        const float kl = p.use_kl_loss ? (approx_kl(lp, ref[r], p.kl_type) * m) * m : 0.f;
        logp_out[r] = lp;
        if (ent_out) ent_out[r] = H;
        *reinterpret_cast<float4*>(tok + r * 4) = make_float4(loss * m, clip * m, kl, H * m);
        s_g[0] = lse;
        s_g[1] = (dl * m) * row_scale[b];        // dL/dlogp for unit upstream gradient
        s_g[2] = scal[1] * m;                    // dL/dH
        s_h = H;
        (void)lab;
    }
    __syncthreads();
    const float L = s_g[0], glp = s_g[1], gent = s_g[2], H = s_h;
    const int64_t lab = labels[b * lsb + t * lst];
    const float inv_t = has_t ? 1.f / temp : 1.f;
    auto grad = [&](float x, int64_t v) -> float {
        const float lpv = x - L;
        const float pv = fast_exp2(lpv * kLog2e);
        float g = -glp * pv - gent * pv * (lpv + H);
        if (v == lab) g += glp;
        return has_t ? g * inv_t : g;
    };
    // ---- sweep 2: dlogits (row re-read is MALL-resident)
    if (vec_ok) {
        const uint4* rv = reinterpret_cast<const uint4*>(row);
        uint4* ov = reinterpret_cast<uint4*>(out);
        int i = threadIdx.x;
        for (; i + 3 * kThreads < nvec; i += 4 * kThreads) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = ld_nt(rv + i + u * kThreads);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float x[8];
                unpack8(v[u], x);
                const int64_t v0 = (int64_t)(i + u * kThreads) * 8;
#pragma unroll
                for (int k = 0; k < 8; ++k) x[k] = grad(tval(x[k]), v0 + k);
                st_out(ov + i + u * kThreads, make_uint4(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]),
                                                         pack_bf16x2(x[4], x[5]), pack_bf16x2(x[6], x[7])), nts);
            }
        }
        for (; i < nvec; i += kThreads) {
            float x[8];
            unpack8(ld_nt(rv + i), x);
            const int64_t v0 = (int64_t)i * 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = grad(tval(x[k]), v0 + k);
            st_out(ov + i, make_uint4(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                                      pack_bf16x2(x[6], x[7])), nts);
        }
    }
    for (int v = done + threadIdx.x; v < V; v += kThreads) out[v] = f32_to_bf16(grad(tval(bf16_to_f32(row[v])), v));
}

// ---- 2b. register-resident variant: the row is loaded ONCE into registers (NV 16-B
// vectors per thread, NT threads: 1024 x 19 covers V <= 155,648, Qwen2.5's 151,936 and
// 152,064; 1024 x 16 Llama-3's 128,256; 1024 x 7 GPT-2's 50,257), so sweep 2 needs no
// memory reads at all: HBM traffic per token is exactly V*2 read + V*2 written. One block
// per CU; the per-token scalars (old/adv/mask/ref, row scale, label) are scalar loads issued
// up front, the label logit one broadcast load by thread 0.
// Any row alignment: the row is read as the 16-B vectors of its aligned-down span (h = the
// row start's element offset within 16 B, 0 for Qwen/Llama rows; GPT-2's odd V makes it vary
// per row), slots outside [0, V) read as bf16 -inf (e = 0 in the softmax). dlogits rows share
// the logits rows' alignment (host check), so full vectors are stored whole and only a row's
// first and last vectors go element by element.
template <int NT, int NV, bool HAS_T, bool EDGE>
__global__ __launch_bounds__(NT) void policy_train_resident_kernel(
    const uint16_t* __restrict__ logits, int64_t sb, int64_t st_, int R, int V, const int64_t* __restrict__ labels,
    int64_t lsb, int64_t lst, float temp, const float* __restrict__ old, const float* __restrict__ adv,
    const float* __restrict__ mask, const float* __restrict__ ref, const float* __restrict__ row_scale,
    const float* __restrict__ scal, skyrl_ppo_params p, float* __restrict__ logp_out, float* __restrict__ ent_out,
    float* __restrict__ tok, uint16_t* __restrict__ dx, int64_t gsb, int64_t gst, bool nts) {
    __shared__ St s_st[NT / 64];
    __shared__ float s_g[4];
    TPHASE(0);
    const int64_t r = blockIdx.x;
    const int64_t b = r / R, t = r % R;
    const uint16_t* row = logits + b * sb + t * st_;
    uint16_t* out = dx + b * gsb + t * gst;
    const int lane = threadIdx.x & 63;
    // EDGE = false: 16-B-aligned rows and V % 8 == 0 (Qwen, Llama): no partial vectors, and the
    // edge logic below compiles away (it costs ~20 VGPRs and spills at NV >= 16)
    const int h = EDGE ? (int)((reinterpret_cast<uintptr_t>(row) >> 1) & 7) : 0;  // uniform per block
    const int nvec = EDGE ? (h + V + 7) >> 3 : V >> 3;                           // vectors of the span
    const uint4* rv = reinterpret_cast<const uint4*>(row - h);
    auto tval = [&](float x) { return HAS_T ? bf16_to_f32(f32_to_bf16(x / temp)) : x; };

    // The token's scalars sit at block-uniform addresses: every thread loads them, so they
    // become scalar loads into SGPRs, issued ahead of the row and costing no VGPRs (the row
    // itself holds 4*NV VGPRs across the whole kernel).
    const int64_t lab = labels[b * lsb + t * lst];
    const float o_old = old[r];
    const float o_adv = adv[r];
    const float o_m = mask ? mask[r] : 1.f;
    const float o_ref = p.use_kl_loss ? ref[r] : 0.f;
    const float o_rs = row_scale[b];
    const float o_ge = scal[1];
    float xl = 0.f;
    if (threadIdx.x == 0) xl = (lab >= 0 && lab < V) ? bf16_to_f32(row[lab]) : __builtin_nanf("");
    constexpr uint32_t kNinf2 = 0xff80ff80u;  // two bf16 -inf: contribute e = 0
    uint4 v[NV];
    // !EDGE: the host guarantees (NV-1)*NT < nvec <= NV*NT, so only the last vector can be out of
    // range and the others load unconditionally (one address live at a time, as few VGPRs as the
    // row itself needs)
    if constexpr (!EDGE) {
#pragma unroll
        for (int k = 0; k < NV - 1; ++k) v[k] = ld_nt(rv + threadIdx.x + k * NT);
        const int idx = threadIdx.x + (NV - 1) * NT;
        const bool ok = idx < nvec;
        const uint4 t4 = ld_nt(rv + (ok ? idx : nvec - 1));
        v[NV - 1] = make_uint4(ok ? t4.x : kNinf2, ok ? t4.y : kNinf2, ok ? t4.z : kNinf2, ok ? t4.w : kNinf2);
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int idx = threadIdx.x + k * NT;
            const bool ok = idx < nvec;
            const uint4 t4 = ld_nt(rv + (ok ? idx : 0));
            v[k] = make_uint4(ok ? t4.x : kNinf2, ok ? t4.y : kNinf2, ok ? t4.z : kNinf2, ok ? t4.w : kNinf2);
        }
    }
    // the span's first and last vectors may hold slots outside the row: -inf them (only the
    // lanes holding those two vectors take the branch)
#pragma unroll
    for (int k = 0; k < (EDGE ? NV : 0); ++k) {
        const int idx = threadIdx.x + k * NT;
        const int lo = h - 8 * idx, hi = V + h - 8 * idx;  // valid slots: lo <= j < hi
        if (idx < nvec && (lo > 0 || hi < 8)) {
            uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < lo || j >= hi) {
                    const uint32_t keep = (j & 1) ? 0x0000ffffu : 0xffff0000u;
                    w[j >> 1] = (w[j >> 1] & keep) | (kNinf2 & ~keep);
                }
            }
            v[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    St st{-3.402823466e38f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float x[8];
        unpack8(v[k], x);  // padding slots are bf16 -inf: contribute e = 0
        if constexpr (HAS_T) {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = tval(x[j]);
        }
        st_add8(st, x);
        __builtin_amdgcn_sched_barrier(0);  // one vector at a time: bounds register pressure
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        St o{__shfl_xor(st.m, off, kWave), __shfl_xor(st.s, off, kWave), __shfl_xor(st.w, off, kWave)};
        st_merge(st, o);
    }
    TPHASE(1);
    if (lane == 0) s_st[threadIdx.x / kWave] = st;
    __syncthreads();
    TPHASE(2);
    // wave 0 merges the NT/64 wave states as a shuffle tree (a serial lane-0 fold of 12 states
    // sat on every row's critical path), then lane 0 evaluates the token's loss terms
    static_assert(NT / 64 <= 16, "wave-state tree covers 16 waves");
    if (threadIdx.x < kWave) {
        St a = threadIdx.x < NT / 64 ? s_st[threadIdx.x] : St{-3.402823466e38f, 0.f, 0.f};
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) {
            St o{__shfl_xor(a.m, off, kWave), __shfl_xor(a.s, off, kWave), __shfl_xor(a.w, off, kWave)};
            st_merge(a, o);
        }
        if (threadIdx.x == 0) {
        const float logs = fast_log2(a.s) * kLn2;
        const float lse = a.m + logs;
        const float H = logs - kLn2 * (a.w / a.s);
        const float lp = tval(xl) - lse;
        const float lo = (float)(1.0 - (double)p.eps_clip_low), hi = (float)(1.0 + (double)p.eps_clip_high);
        float loss, dl, clip;
        ppo_token(lp, o_old, o_adv, lo, hi, p.clip_ratio_c, p.dual_clip, loss, dl, clip);
        const float kl = p.use_kl_loss ? (approx_kl(lp, o_ref, p.kl_type) * o_m) * o_m : 0.f;
        logp_out[r] = lp;
        if (ent_out) ent_out[r] = H;
        *reinterpret_cast<float4*>(tok + r * 4) = make_float4(loss * o_m, clip * o_m, kl, H * o_m);
        s_g[0] = lse;
        s_g[1] = (dl * o_m) * o_rs;
        s_g[2] = o_ge * o_m;
        s_g[3] = H;
        }
    }
    __syncthreads();
    TPHASE(3);
    const float L = s_g[0], glp = s_g[1], gent = s_g[2], H = s_g[3];
    const int lab_s = (lab >= 0 && lab < V) ? (int)lab + h : -1;  // label's slot in the aligned-down span
#pragma unroll
    for (int k = 0; k < NV; ++k)  // new values: no reuse of sweep-1 unpacks across the barrier
        asm volatile("" : "+v"(v[k].x), "+v"(v[k].y), "+v"(v[k].z), "+v"(v[k].w));
    const float inv_t = HAS_T ? 1.f / temp : 1.f;
    uint4* ov = reinterpret_cast<uint4*>(out - h);

#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int idx = threadIdx.x + k * NT;
        if ((!EDGE && k < NV - 1) || idx < nvec) {
            float x[8];
            unpack8(v[k], x);
            const int v0 = idx * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float lpv = tval(x[j]) - L;
                const float pv = fast_exp2(lpv * kLog2e);
                float g = -glp * pv - gent * pv * (lpv + H);
                if (v0 + j == lab_s) g += glp;
                x[j] = HAS_T ? g * inv_t : g;
            }
            const int lo = h - v0, hi = V + h - v0;
            if (!EDGE || (lo <= 0 && hi >= 8)) {
                st_out(ov + idx, make_uint4(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]),
                                            pack_bf16x2(x[4], x[5]), pack_bf16x2(x[6], x[7])), nts);
            } else {  // the row's first / last vector: only its own slots
                uint16_t* o16 = reinterpret_cast<uint16_t*>(ov + idx);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (j >= lo && j < hi) o16[j] = f32_to_bf16(x[j]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    TPHASE(4);
}

// ---- 2c. split rows: each row is cut into P contiguous pieces (P = 8 by default: 128-thread
// workgroups; 4: 256 threads), NV 16-B vectors per thread held in registers across both
// sweeps, so HBM still sees V*2 read + V*2 written per token. Several pieces of DIFFERENT rows
// share a CU at different phases (eighths: 6 workgroups of 143 VGPRs; quarters: 4 of 115):
// one piece's barrier and store drain overlap the others' loads, where the one-row-per-CU
// resident kernel left its CU without loads in flight for about half of each row
// (profiles/r02_policy_train_phases.log). Measured per 16 x 1024 tokens at V = 151,936
// (profiles/r03_kbench_split.json, one box): eighths 1.71 ms = 5.83 TB/s, quarters 1.74 ms,
// sixteenths 1.99 ms, resident 1.94 ms. Copy-shaped probe: split rows 5.76 TB/s vs 5.13
// resident (profiles/r03_rw_split_probe.log).
// The pieces exchange their online-softmax states (m, s, w) as epoch-tagged 64-bit granules
// (write-through agent-scope stores, polled with agent-scope loads: the pieces sit on
// different XCDs, whose L2s are not coherent); every piece merges the P states in piece
// order, so all derive bit-identical lse / entropy / loss terms, and piece 0 writes the
// token's outputs. The epoch is advanced once per launch by train_scales_kernel, so a piece
// never mistakes the previous launch's granules for its partners'. The pieces of a row are
// consecutive blocks (blocks are dispatched in order, so a waiting piece's partners are
// resident or next to be), every poll is bounded, and a timeout raises the error word
// (metrics[6] = 1 via the epilogue; ops.check_loss_metrics raises) and leaves NaN in that
// row's terms instead of hanging.
constexpr int kSplitMaxP = 12;  // most pieces per row of any built shape (split_shapes below)
// how long a piece waits for a partner's published state, on the 100 MHz constant clock
// (s_memrealtime): partners are consecutive blocks, resident or next to be dispatched, and
// publish within microseconds; past this bound (other streams' kernels holding the CUs, a grid
// larger than what is resident) the piece computes the partner's state itself (no deadlock, no
// error path, the same bits). The bound is knobs().train_split_wait (default 5000 ticks = 50 us;
// tests shorten it through the variant).

typedef __attribute__((address_space(1))) unsigned long long ptr_gu64;
typedef __attribute__((address_space(1))) unsigned ptr_gu32;

template <int NV, bool HAS_T, int P, bool EDGE, int W, int NT>
__global__ __launch_bounds__(NT, W) void policy_train_split_kernel(
    const uint16_t* __restrict__ logits, int64_t sb, int64_t st_, int R, int V, const int64_t* __restrict__ labels,
    int64_t lsb, int64_t lst, float temp, const float* __restrict__ old, const float* __restrict__ adv,
    const float* __restrict__ mask, const float* __restrict__ ref, const float* __restrict__ row_scale,
    const float* __restrict__ scal, skyrl_ppo_params p, float* __restrict__ logp_out, float* __restrict__ ent_out,
    float* __restrict__ tok, uint16_t* __restrict__ dx, int64_t gsb, int64_t gst, bool nts,
    unsigned long long* __restrict__ gran, unsigned* __restrict__ err_word, const int32_t* __restrict__ tpos,
    unsigned wait_ticks) {
    static_assert(P <= 16 && NT % 64 == 0 && NT <= 1024, "split shape");
    __shared__ St s_st[NT / 64];
    __shared__ float s_g[4];
    __shared__ float s_part[P * 3];
    __shared__ unsigned s_missing;  // partners whose state this piece computes itself
    // block -> (row, piece): consecutive blocks. (Placing a row's pieces on one XCD, so the
    // exchange stays in that XCD's L2, measured slower: 2.05 vs 1.71 ms per 16 x 1024 tokens,
    // profiles/r03_kbench_split.json; so did longer sleeps between polls, no change.)
    // tpos (ragged launches, skyrl_policy_train_ragged_fwd): token q of the launch has logits row
    // q (stride st_ / gst) and sits at [n, R] position tpos[q] of the per-token arrays
    const int64_t q = blockIdx.x / P;
    const int part = blockIdx.x % P;
    const int64_t r = tpos ? (int64_t)tpos[q] : q;
    const int64_t b = r / R, t = r % R;
    const uint16_t* row = tpos ? logits + q * st_ : logits + b * sb + t * st_;
    uint16_t* out = tpos ? dx + q * gst : dx + b * gsb + t * gst;
    const int lane = threadIdx.x & 63;
    // EDGE: rows not 16-B aligned or V % 8 != 0 (GPT-2's 50,257): the row's aligned-down span
    // (h slots before it) is what is cut into pieces; its first and last vectors are partial
    const int h = EDGE ? (int)((reinterpret_cast<uintptr_t>(row) >> 1) & 7) : 0;
    const int nvec = EDGE ? (h + V + 7) >> 3 : V >> 3;
    // host (split_nv / split_nv_edge): per <= NV*NT, every piece non-empty, and without EDGE
    // (NV-1)*NT < the last piece's length
    const int per = (nvec + P - 1) / P;
    const int lo = part * per;
    const int hi = min(nvec, lo + per);
    const uint4* rv = reinterpret_cast<const uint4*>(row - h) + lo;
    auto tval = [&](float x) { return HAS_T ? bf16_to_f32(f32_to_bf16(x / temp)) : x; };
    const unsigned epoch = __hip_atomic_load((const ptr_gu32*)(reinterpret_cast<const unsigned*>(scal) + 16),
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t lab = tpos ? labels[q * lst] : labels[b * lsb + t * lst];
    const float o_old = old[r];
    const float o_adv = adv[r];
    const float o_m = mask ? mask[r] : 1.f;
    const float o_ref = p.use_kl_loss ? ref[r] : 0.f;
    const float o_rs = row_scale[b];
    const float o_ge = scal[1];
    float xl = 0.f;
    if (threadIdx.x == 0) xl = (lab >= 0 && lab < V) ? bf16_to_f32(row[lab]) : __builtin_nanf("");
    constexpr uint32_t kNinf2 = 0xff80ff80u;
    uint4 v[NV];
    const int nq = hi - lo;
    if constexpr (!EDGE) {
#pragma unroll
        for (int k = 0; k < NV - 1; ++k) v[k] = ld_nt(rv + threadIdx.x + k * NT);
        const int idx = threadIdx.x + (NV - 1) * NT;
        const bool ok = idx < nq;
        const uint4 t4 = ld_nt(rv + (ok ? idx : nq - 1));
        v[NV - 1] = make_uint4(ok ? t4.x : kNinf2, ok ? t4.y : kNinf2, ok ? t4.z : kNinf2, ok ? t4.w : kNinf2);
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int idx = threadIdx.x + k * NT;
            const bool ok = idx < nq;
            const uint4 t4 = ld_nt(rv + (ok ? idx : 0));
            v[k] = make_uint4(ok ? t4.x : kNinf2, ok ? t4.y : kNinf2, ok ? t4.z : kNinf2, ok ? t4.w : kNinf2);
        }
        // the span's first and last vectors hold slots of the neighbouring rows: -inf them
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int idx = threadIdx.x + k * NT;
            const int sl = h - 8 * (lo + idx), sh = V + h - 8 * (lo + idx);  // own slots: sl <= j < sh
            if (idx < nq && (sl > 0 || sh < 8)) {
                uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (j < sl || j >= sh) {
                        const uint32_t keep = (j & 1) ? 0x0000ffffu : 0xffff0000u;
                        w[j >> 1] = (w[j >> 1] & keep) | (kNinf2 & ~keep);
                    }
                }
                v[k] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
    }
    St st{-3.402823466e38f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float x[8];
        unpack8(v[k], x);
        if constexpr (HAS_T) {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = tval(x[j]);
        }
        st_add8(st, x);
        __builtin_amdgcn_sched_barrier(0);
    }
    // a piece's state from its threads' states: the xor butterfly in each wave, then (wave 0) an
    // xor tree over the NT/64 wave states, at least 4 lanes wide so lanes 0..2, which publish
    // m, s, w, all hold it. Shared by this piece's own state and a partner state recomputed
    // below, so both give the same bits.
    auto wave_fold = [&](St x) -> St {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            St o{__shfl_xor(x.m, off, kWave), __shfl_xor(x.s, off, kWave), __shfl_xor(x.w, off, kWave)};
            st_merge(x, o);
        }
        return x;
    };
    auto piece_tree = [&]() -> St {  // wave 0, after the barrier that follows the s_st writes
        St a = threadIdx.x < NT / 64 ? s_st[threadIdx.x] : St{-3.402823466e38f, 0.f, 0.f};
#pragma unroll
        for (int off = (NT / 128 > 2 ? NT / 128 : 2); off > 0; off >>= 1) {
            St o{__shfl_xor(a.m, off, kWave), __shfl_xor(a.s, off, kWave), __shfl_xor(a.w, off, kWave)};
            st_merge(a, o);
        }
        return a;
    };
    st = wave_fold(st);
    if (lane == 0) s_st[threadIdx.x / kWave] = st;
    if (threadIdx.x == 0) s_missing = 0u;
    __syncthreads();
    if (threadIdx.x < kWave) {
        const St a = piece_tree();
        unsigned long long* g = gran + r * (P * 3);
        // lanes 0..2 publish (m, s, w) of this piece; lanes 3q..3q+2 of the other pieces poll
        const int q = lane / 3, f = lane % 3;
        const float mine = f == 0 ? a.m : (f == 1 ? a.s : a.w);
        if (lane < 3) {
            s_part[part * 3 + f] = mine;
            __hip_atomic_store((ptr_gu64*)(g + part * 3 + f),
                               ((unsigned long long)epoch << 32) | __float_as_uint(mine), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane < P * 3 && q != part) {
            unsigned long long x = 0;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                x = __hip_atomic_load((const ptr_gu64*)(g + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((unsigned)(x >> 32) == epoch) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > wait_ticks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if ((unsigned)(x >> 32) == epoch) s_part[lane] = __uint_as_float((unsigned)x);
            else atomicOr(&s_missing, 1u << q);  // LDS
        }
    }
    __syncthreads();
    const unsigned missing = s_missing;  // workgroup-uniform
    if (missing != 0u) {
        // A partner not published within the bound (not resident: other streams' kernels hold
        // the CUs, or the grid outgrew what is resident at once): this workgroup computes that
        // partner's state itself from the partner's slice of the row, with the partner's own
        // loads, masking, summation order and trees, so the bits are the ones the partner
        // publishes (or already did). No piece ever waits on a partner being dispatched.
        for (int pp = 0; pp < P; ++pp) {
            if (!((missing >> pp) & 1u)) continue;
            const int plo = pp * per;
            const int pnq = min(nvec, plo + per) - plo;
            const uint4* prv = reinterpret_cast<const uint4*>(row - h) + plo;
            St ps{-3.402823466e38f, 0.f, 0.f};
#pragma unroll 1
            for (int k = 0; k < NV; ++k) {
                const int idx = threadIdx.x + k * NT;
                const bool ok = idx < pnq;
                uint4 w4;
                if (!EDGE && k < NV - 1) {
                    w4 = ld_nt(prv + idx);
                } else {
                    const uint4 t4 = ld_nt(prv + (ok ? idx : (EDGE ? 0 : pnq - 1)));
                    w4 = make_uint4(ok ? t4.x : kNinf2, ok ? t4.y : kNinf2, ok ? t4.z : kNinf2, ok ? t4.w : kNinf2);
                }
                if constexpr (EDGE) {
                    const int sl = h - 8 * (plo + idx), sh = V + h - 8 * (plo + idx);
                    if (ok && (sl > 0 || sh < 8)) {
                        uint32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            if (j < sl || j >= sh) {
                                const uint32_t keep = (j & 1) ? 0x0000ffffu : 0xffff0000u;
                                wv[j >> 1] = (wv[j >> 1] & keep) | (kNinf2 & ~keep);
                            }
                        }
                        w4 = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                    }
                }
                float x[8];
                unpack8(w4, x);
                if constexpr (HAS_T) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) x[j] = tval(x[j]);
                }
                st_add8(ps, x);
            }
            ps = wave_fold(ps);
            __syncthreads();  // s_st is free again (the previous tree has been read)
            if (lane == 0) s_st[threadIdx.x / kWave] = ps;
            __syncthreads();
            if (threadIdx.x < kWave) {
                const St a = piece_tree();
                if (lane < 3) s_part[pp * 3 + lane] = lane == 0 ? a.m : (lane == 1 ? a.s : a.w);
            }
        }
        if (threadIdx.x == 0)  // diagnostics (tests): partner states recomputed, header word 33
            __hip_atomic_fetch_add((ptr_gu32*)(err_word + 1), (unsigned)__popc(missing), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }
    if (threadIdx.x < kWave) {
        // the row's state: a fixed xor tree over lanes 0..P-1 (lane j holds piece j), the same
        // operations on the same values in every piece, so all pieces get the same bits (a
        // serial fold in lane 0 held 3P more VGPRs across the exchange)
        constexpr int kTop = P > 8 ? 8 : P > 4 ? 4 : P > 2 ? 2 : 1;
        St m = lane < P ? St{s_part[3 * lane], s_part[3 * lane + 1], s_part[3 * lane + 2]}
                        : St{-3.402823466e38f, 0.f, 0.f};
#pragma unroll
        for (int off = kTop; off > 0; off >>= 1) {
            St o{__shfl_xor(m.m, off, kWave), __shfl_xor(m.s, off, kWave), __shfl_xor(m.w, off, kWave)};
            st_merge(m, o);
        }
        if (threadIdx.x == 0) {
            const float logs = fast_log2(m.s) * kLn2;
            const float lse = m.m + logs;
            const float H = logs - kLn2 * (m.w / m.s);
            const float lp = tval(xl) - lse;
            const float lo_c = (float)(1.0 - (double)p.eps_clip_low), hi_c = (float)(1.0 + (double)p.eps_clip_high);
            float loss, dl, clip;
            ppo_token(lp, o_old, o_adv, lo_c, hi_c, p.clip_ratio_c, p.dual_clip, loss, dl, clip);
            const float kl = p.use_kl_loss ? (approx_kl(lp, o_ref, p.kl_type) * o_m) * o_m : 0.f;
            if (part == 0) {
                logp_out[r] = lp;
                if (ent_out) ent_out[r] = H;
                *reinterpret_cast<float4*>(tok + r * 4) = make_float4(loss * o_m, clip * o_m, kl, H * o_m);
            }
            s_g[0] = lse;
            s_g[1] = (dl * o_m) * o_rs;
            s_g[2] = o_ge * o_m;
            s_g[3] = H;
        }
    }
    __syncthreads();
    const float L = s_g[0], glp = s_g[1], gent = s_g[2], H = s_g[3];
    const int lab_s = (lab >= 0 && lab < V) ? (int)lab + h - 8 * lo : -1;  // label's slot in this piece
    const int lab_v = lab_s >= 0 ? lab_s >> 3 : -1, lab_j = lab_s & 7;
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(v[k].x), "+v"(v[k].y), "+v"(v[k].z), "+v"(v[k].w));
    const float inv_t = HAS_T ? 1.f / temp : 1.f;
    // dL/dz = glp (onehot - p) - gent p (logp + H) with logp = z - L and p = 2^((z - L) log2e):
    //   gg = p (ca z + cb), ca = -gent, cb = -glp - gent (H - L); the label's element adds glp.
    // Two packed fma, one exp2 and one multiply per element (the per-element label compare and the
    // separate subtract / scale are gone): the sweep is less VALU per byte, which matters when the
    // chip's clock drops under sustained HBM load (policy_train)
    const float cy = -L * kLog2e;
    const float ca = -gent, cb = -glp - gent * (H - L);
    uint4* ov = reinterpret_cast<uint4*>(out - h) + lo;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int idx = threadIdx.x + k * NT;
        if ((!EDGE && k < NV - 1) || idx < nq) {
            float x[8];
            unpack8(v[k], x);
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 l2 = {kLog2e, kLog2e}, c2 = {cy, cy}, a2 = {ca, ca}, b2 = {cb, cb};
#pragma unroll
            for (int j = 0; j < 8; j += 2) {  // packed fma pairs (v_pk_fma_f32)
                const f2 z = {tval(x[j]), tval(x[j + 1])};
                const f2 y = __builtin_elementwise_fma(z, l2, c2);
                const f2 t = __builtin_elementwise_fma(a2, z, b2);
                const f2 pv = {fast_exp2(y.x), fast_exp2(y.y)};
                const f2 g = pv * t;
                x[j] = g.x;
                x[j + 1] = g.y;
            }
            if (idx == lab_v) {  // one lane of the row
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (j == lab_j) x[j] += glp;
            }
            if constexpr (HAS_T) {
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] *= inv_t;
            }
            const int sl = h - 8 * (lo + idx), sh = V + h - 8 * (lo + idx);
            if (!EDGE || (sl <= 0 && sh >= 8)) {
                st_out(ov + idx, make_uint4(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]),
                                            pack_bf16x2(x[4], x[5]), pack_bf16x2(x[6], x[7])), nts);
            } else {  // the span's first / last vector: only this row's slots
                uint16_t* o16 = reinterpret_cast<uint16_t*>(ov + idx);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (j >= sl && j < sh) o16[j] = f32_to_bf16(x[j]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ---- 3. loss scalar + metrics ---------------------------------------------------------
// Per row (one wave): a0 = sum l*m, a1 = sum kl*m*m, am = sum m (fp32, lane order then the
// butterfly), clip*m and ent*m per lane in fp64 then the butterfly; the row's record is
// (a0, a0 / mrow | a0 / max_seq_len, a1 / mrow, clip, ent) in fp64. A micro-batch's terms are its
// rows' records summed in row order (the per-call epilogue and the step fold alike, so their
// loss and metrics are the same bits); same metric layout as skyrl_ppo_loss_fwd. MASKED (the step
// fold): a position whose loss mask is 0 contributes nothing, which lets a packed micro-batch leave
// the records of positions no token maps to unwritten (every record is premultiplied by m, so for
// finite terms the sums are the same bits).
struct RowRec {
    double tl, pg, kl, tc, te;
};
template <bool MASKED>
__device__ __forceinline__ RowRec row_record(const float* __restrict__ tok, const float* __restrict__ mask, int R,
                                             const skyrl_ppo_params& p) {
    const int lane = threadIdx.x & 63;
    float a0 = 0.f, a1 = 0.f, am = 0.f;
    double tc = 0.0, te = 0.0;
    constexpr int kU = 16;  // a lane's positions per batch: every load of the batch in flight at once
    for (int t0 = 0; t0 < R; t0 += kU * kWave) {
        float4 v[kU];
        float mm[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {  // clamped addresses: the loads are unconditional
            const int t = min(t0 + u * kWave + lane, R - 1);
            v[u] = *reinterpret_cast<const float4*>(tok + (int64_t)t * 4);
            mm[u] = mask ? mask[t] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {  // in position order, as one position at a time would
            if (t0 + u * kWave + lane >= R) continue;
            float4 x = v[u];
            const float m = mm[u];
            if (MASKED && m == 0.f) x = make_float4(0.f, 0.f, 0.f, 0.f);
            a0 += x.x;
            a1 += x.z;
            tc += x.y;
            te += x.w;
            am += m;
        }
    }
    a0 = wave_sum_dpp(a0);  // (DPP trees, no LDS round trips: the fold's wave is latency-bound)
    a1 = wave_sum_dpp(a1);
    am = wave_sum_dpp(am);
    tc = wave_sum_dpp(tc);
    te = wave_sum_dpp(te);
    const double mrow = am > 1.f ? am : 1.0;
    RowRec r{a0, 0.0, a1 / mrow, tc, te};
    if (p.loss_reduction == 1) r.pg = a0 / mrow;
    else if (p.loss_reduction == 2) r.pg = a0 / (double)p.max_seq_len;
    return r;
}
__device__ __forceinline__ void rec_add(RowRec& a, const RowRec& b) {
    a.tl += b.tl;
    a.pg += b.pg;
    a.kl += b.kl;
    a.tc += b.tc;
    a.te += b.te;
}
// the micro-batch's loss and metrics from its summed records (n rows)
__device__ __forceinline__ void finish_metrics(const RowRec& v, int n, const skyrl_ppo_params& p,
                                               const float* __restrict__ scal, float* __restrict__ loss_out,
                                               float* __restrict__ metrics) {
    const double msum = scal[0] > 1.f ? (double)scal[0] : 1.0;
    const float pg = p.loss_reduction == 0 ? (float)(v.tl / msum) : (float)(v.pg / (double)n);
    const float kl = p.use_kl_loss ? (float)(v.kl / (double)n) : 0.f;
    const float entropy = (float)(v.te / msum);
    float final_loss = pg + kl * p.kl_loss_coef;
    if (p.use_entropy_loss) final_loss = final_loss - entropy * p.entropy_loss_coef;
    loss_out[0] = final_loss;
    metrics[SKYRL_M_FINAL_LOSS] = final_loss;
    metrics[SKYRL_M_POLICY_LOSS] = pg;
    metrics[SKYRL_M_ENTROPY] = entropy;
    metrics[SKYRL_M_KL] = kl;
    metrics[SKYRL_M_CLIP_RATIO] = (float)(v.tc / msum);
    metrics[SKYRL_M_MASK_SUM] = scal[0];
    unsigned* err = reinterpret_cast<unsigned*>(const_cast<float*>(scal)) + 32;  // header word 32
    metrics[6] = err[0] ? 1.f : 0.f;  // split-row exchange failure (not produced since r05)
    metrics[7] = 0.f;
    err[0] = 0u;
}

// One block over n rows: 16 rows (one per wave) at a time, their records summed by thread 0 in
// row order.
template <bool MASKED>
__device__ __forceinline__ void epilogue_body(const float* __restrict__ tok, const float* __restrict__ mask, int n,
                                              int R, const skyrl_ppo_params& p, const float* __restrict__ scal,
                                              float* __restrict__ loss_out, float* __restrict__ metrics) {
    __shared__ RowRec s_rec[kWaves];
    const int lane = threadIdx.x & 63, w = threadIdx.x / kWave;
    RowRec tot{0.0, 0.0, 0.0, 0.0, 0.0};
    for (int b0 = 0; b0 < n; b0 += kWaves) {
        const int b = b0 + w;
        if (b < n) {
            const RowRec r = row_record<MASKED>(tok + (int64_t)b * R * 4, mask ? mask + (int64_t)b * R : nullptr, R, p);
            if (lane == 0) s_rec[w] = r;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int j = 0; j < kWaves && b0 + j < n; ++j) rec_add(tot, s_rec[j]);
        __syncthreads();
    }
    if (threadIdx.x == 0) finish_metrics(tot, n, p, scal, loss_out, metrics);
}

__global__ __launch_bounds__(kThreads) void train_epilogue_kernel(const float* __restrict__ tok,
                                                                  const float* __restrict__ mask, int n, int R,
                                                                  skyrl_ppo_params p, const float* __restrict__ scal,
                                                                  float* __restrict__ loss_out,
                                                                  float* __restrict__ metrics) {
    epilogue_body<false>(tok, mask, n, R, p, scal, loss_out, metrics);
}

// The step fold: one wave per row (2 rows per block), the row's record (row_record, MASKED) stored
// write-through, one arrival per row on the micro-batch's counter; the last row's wave sums the
// micro-batch's records in row order (the per-call epilogue's order and bits, for finite terms)
// and writes its loss and metrics (the plan's hand-off form).
__global__ __launch_bounds__(kStepRows * kWave) void train_fold_kernel(
    const float* __restrict__ tok, const float* __restrict__ mask, int n_total, int R, int mb, skyrl_ppo_params p,
    char* __restrict__ slots, double* __restrict__ recs, float* __restrict__ loss_out, float* __restrict__ metrics) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * kStepRows + threadIdx.x / kWave;
    if (b >= n_total) return;
    const int k = b / mb;
    const int r0 = k * mb;
    const int n = min(n_total, r0 + mb) - r0;
    float* scal = reinterpret_cast<float*>(slots + (size_t)k * kStepSlot);
    unsigned* ctr = reinterpret_cast<unsigned*>(scal) + kSlotFoldCtr;
    const RowRec r = row_record<true>(tok + (int64_t)b * R * 4, mask + (int64_t)b * R, R, p);
    unsigned prev = 0;
    if (lane == 0) {
        double* d = recs + (size_t)b * 5;
        st_wt(d + 0, r.tl);
        st_wt(d + 1, r.pg);
        st_wt(d + 2, r.kl);
        st_wt(d + 3, r.tc);
        st_wt(d + 4, r.te);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev != (unsigned)n - 1u) return;
    handoff_acquire();
    RowRec tot{0.0, 0.0, 0.0, 0.0, 0.0};
    for (int j0 = 0; j0 < n; j0 += kWave) {
        double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        if (j0 + lane < n) {
            const double* d = recs + (size_t)(r0 + j0 + lane) * 5;
#pragma unroll
            for (int f = 0; f < 5; ++f) v[f] = __hip_atomic_load(d + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int j = 0; j < kWave && j0 + j < n; ++j)
            rec_add(tot, RowRec{readlane_f64(v[0], j), readlane_f64(v[1], j), readlane_f64(v[2], j),
                                readlane_f64(v[3], j), readlane_f64(v[4], j)});
    }
    if (lane == 0) {
        finish_metrics(tot, n, p, scal, loss_out + k, metrics + (size_t)k * SKYRL_M_COUNT);
        __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
}

// dlogits *= g (skipped when g == 1: the common loss.backward() case)
__global__ void scale_bf16_kernel(const float* __restrict__ g, uint16_t* __restrict__ x, int64_t n) {
    const float s = g[0];
    if (s == 1.0f) return;
    uint4* x4 = reinterpret_cast<uint4*>(x);
    const int64_t n8 = n / 8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8];
        unpack8(x4[i], v);
        x4[i] = make_uint4(pack_bf16x2(v[0] * s, v[1] * s), pack_bf16x2(v[2] * s, v[3] * s),
                           pack_bf16x2(v[4] * s, v[5] * s), pack_bf16x2(v[6] * s, v[7] * s));
    }
    for (int64_t i = n8 * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = f32_to_bf16(bf16_to_f32(x[i]) * s);
}

}  // namespace


}  // namespace skyrl

using namespace skyrl;

// Workspace: [0, 256) header (scal[0..2] floats; word 16: the split kernel's exchange epoch;
// word 32: its timeout flag), row scales (n floats, 256-B padded), per-token terms (n*R x 16 B,
// 256-B padded), the split kernel's exchange granules (n*R x kSplitMaxP x 3 x 8 B). Zeroed once at
// allocation; the kernels keep it consistent from launch to launch.
namespace {
size_t pt_pad(size_t x) { return (x + 255) / 256 * 256; }
size_t pt_tok_off(int32_t n) { return 256 + pt_pad((size_t)n * 4); }
size_t pt_gran_off(int32_t n, int32_t R) { return pt_tok_off(n) + pt_pad((size_t)n * R * 16); }
}  // namespace

extern "C" size_t skyrl_policy_train_workspace_bytes(int32_t n, int32_t R) {
    if (n <= 0 || R <= 0) return 256;
    return pt_gran_off(n, R) + (size_t)n * R * kSplitMaxP * 3 * 8;
}

namespace {
// Register-resident instantiations (1024 threads): NV vectors per thread cover spans up to
// NV * 8192 elements. The host takes the smallest NV that covers the row's aligned-down span.
using TrainKernel = void (*)(const uint16_t*, int64_t, int64_t, int, int, const int64_t*, int64_t, int64_t, float,
                             const float*, const float*, const float*, const float*, const float*, const float*,
                             skyrl_ppo_params, float*, float*, float*, uint16_t*, int64_t, int64_t, bool);
template <int NV, bool EDGE>
TrainKernel pick_resident(bool has_t) {
    return has_t ? policy_train_resident_kernel<1024, NV, true, EDGE> : policy_train_resident_kernel<1024, NV, false, EDGE>;
}
// rows with partial vectors (EDGE): the smallest listed NV covering the span; NV <= 14 fits
// the edge logic without spills
constexpr int kEdgeNV[] = {2, 4, 6, 7, 8, 10, 12, 14};
TrainKernel resident_edge_for(int nv, bool has_t) {
    switch (nv) {
        case 2: return pick_resident<2, true>(has_t);
        case 4: return pick_resident<4, true>(has_t);
        case 6: return pick_resident<6, true>(has_t);
        case 7: return pick_resident<7, true>(has_t);
        case 8: return pick_resident<8, true>(has_t);
        case 10: return pick_resident<10, true>(has_t);
        case 12: return pick_resident<12, true>(has_t);
        default: return pick_resident<14, true>(has_t);
    }
}
using SplitKernel = void (*)(const uint16_t*, int64_t, int64_t, int, int, const int64_t*, int64_t, int64_t, float,
                             const float*, const float*, const float*, const float*, const float*, const float*,
                             skyrl_ppo_params, float*, float*, float*, uint16_t*, int64_t, int64_t, bool,
                             unsigned long long*, unsigned*, const int32_t*, unsigned);
// Split shapes: P pieces per row of NT threads each, W waves per SIMD (the __launch_bounds__
// occupancy target, i.e. the VGPR cap 512 / W in granules of 8 the compiler schedules the
// piece's registers under). the variant field train_split_shape = i picks one; 0 = by vocabulary.
template <int P, bool EDGE, int W, int NT, int NV>
SplitKernel pick_split(bool has_t) {
    return has_t ? policy_train_split_kernel<NV, true, P, EDGE, W, NT>
                 : policy_train_split_kernel<NV, false, P, EDGE, W, NT>;
}
// aligned rows need NV exactly (the first NV-1 loads are unconditional); EDGE rows take the
// smallest listed NV >= nv
template <int P, bool EDGE, int W, int NT, int... NVs>
SplitKernel split_table(int nv, bool has_t, std::integer_sequence<int, NVs...>) {
    SplitKernel k = nullptr;
    ((k = (k == nullptr && (EDGE ? nv <= NVs : nv == NVs)) ? pick_split<P, EDGE, W, NT, NVs>(has_t) : k), ...);
    return k;
}
using AlignedNV = std::integer_sequence<int, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19>;
// the edge logic costs VGPRs: NV <= 14 (V <= 114,688 at 1024 threads per row)
using EdgeNV = std::integer_sequence<int, 1, 2, 4, 7, 10, 14>;
constexpr int kSplitEdgeNV[] = {1, 2, 4, 7, 10, 14};
struct SplitShape {
    int parts, threads, waves;
};
constexpr SplitShape kSplitShapes[] = {
    {0, 0, 0},       // 0: by vocabulary (split_plan)
    {8, 128, 3},     // 1
    {4, 256, 4},     // 2
    {2, 512, 2},     // 3
    {5, 256, 4},     // 4
    {6, 256, 5},     // 5
};
static_assert(sizeof(kSplitShapes) / sizeof(kSplitShapes[0]) == 6, "variant.hip accepts train_split_shape 0..5");
SplitKernel split_for(int nv, bool has_t, int shape, bool edge) {
    if (edge) {  // EDGE forms are built for the power-of-two shapes only
        switch (shape) {
            case 1: return split_table<8, true, 3, 128>(nv, has_t, EdgeNV{});
            case 2: return split_table<4, true, 4, 256>(nv, has_t, EdgeNV{});
            case 3: return split_table<2, true, 2, 512>(nv, has_t, EdgeNV{});
            default: return nullptr;
        }
    }
    switch (shape) {
        case 1: return split_table<8, false, 3, 128>(nv, has_t, AlignedNV{});
        case 2: return split_table<4, false, 4, 256>(nv, has_t, AlignedNV{});
        case 3: return split_table<2, false, 2, 512>(nv, has_t, AlignedNV{});
        case 4: return split_table<5, false, 4, 256>(nv, has_t, AlignedNV{});
        case 5: return split_table<6, false, 5, 256>(nv, has_t, AlignedNV{});
        default: return nullptr;
    }
}
// EDGE layout: a row's span is (h + V + 7) / 8 vectors for its offset h = 0..7 within 16 B, so
// two span lengths occur; both must give pieces of at most NV*NT vectors and a non-empty last
// piece. Returns the listed NV, or 0.
int split_nv_edge(int V, int parts, int nt) {
    const int spans[2] = {(V + 7) / 8, (V + 14) / 8};
    int need = 0;
    for (int nvec : spans) {
        const int per = (nvec + parts - 1) / parts;
        if (nvec - (parts - 1) * per < 1) return 0;
        need = max(need, (per + nt - 1) / nt);
    }
    for (int cand : kSplitEdgeNV)
        if (need <= cand) return cand;
    return 0;
}
// the split kernel's vectors per thread for nvec row vectors cut into `parts` pieces of
// nt threads, or 0 if its layout does not fit: pieces of per = ceil(nvec / parts)
// vectors, NV = ceil(per / threads) <= 19, and the last piece still covers the NV-1
// unconditional loads of every thread
int split_nv(int nvec, int parts, int nt) {
    const int per = (nvec + parts - 1) / parts;
    const int nv = (per + nt - 1) / nt;
    const int last = nvec - (parts - 1) * per;
    if (nv < 1 || nv > 19 || last <= (nv - 1) * nt) return 0;
    return nv;
}
// the split launch for a vocabulary: the variant field train_split_shape if set, else by V
struct SplitPlan {
    SplitKernel kern = nullptr;
    int parts = 0, threads = 0;
};
SplitPlan split_plan(int V, bool aligned, bool has_t) {
    SplitPlan sp;
    // by vocabulary (profiles/r03_split_shapes.json, 16 x 1024 tokens per launch): rows over
    // 128 KB in six 256-thread pieces (13 vectors per thread at V = 151,936: 79 VGPRs, so 6
    // waves per SIMD and 6 pieces per CU in flight), shorter rows and rows with partial
    // vectors (GPT-2) in four
    const int shape = knobs().train_split_shape ? knobs().train_split_shape : (aligned && V > 65536 ? 5 : 2);
    const SplitShape& sh = kSplitShapes[shape];
    const int nv = aligned ? split_nv(V / 8, sh.parts, sh.threads) : split_nv_edge(V, sh.parts, sh.threads);
    if (nv > 0) sp.kern = split_for(nv, has_t, shape, !aligned);
    sp.parts = sh.parts;
    sp.threads = sh.threads;
    return sp;
}
// aligned rows: NV = ceil(nvec / 1024) exactly, 1..19 (V <= 155,648)
TrainKernel resident_aligned_for(int nv, bool has_t) {
    switch (nv) {
        case 1: return pick_resident<1, false>(has_t);
        case 2: return pick_resident<2, false>(has_t);
        case 3: return pick_resident<3, false>(has_t);
        case 4: return pick_resident<4, false>(has_t);
        case 5: return pick_resident<5, false>(has_t);
        case 6: return pick_resident<6, false>(has_t);
        case 7: return pick_resident<7, false>(has_t);
        case 8: return pick_resident<8, false>(has_t);
        case 9: return pick_resident<9, false>(has_t);
        case 10: return pick_resident<10, false>(has_t);
        case 11: return pick_resident<11, false>(has_t);
        case 12: return pick_resident<12, false>(has_t);
        case 13: return pick_resident<13, false>(has_t);
        case 14: return pick_resident<14, false>(has_t);
        case 15: return pick_resident<15, false>(has_t);
        case 16: return pick_resident<16, false>(has_t);
        case 17: return pick_resident<17, false>(has_t);
        case 18: return pick_resident<18, false>(has_t);
        default: return pick_resident<19, false>(has_t);
    }
}
}  // namespace

extern "C" int skyrl_policy_train_fwd(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t n,
                                      int32_t R, int32_t V, const int64_t* labels, int64_t lstride_b,
                                      int64_t lstride_t, float temperature, const float* old_log_probs,
                                      const float* advantages, const float* loss_mask, const float* ref_log_probs,
                                      const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                                      float* logp_out, float* entropy_out, void* grad_logits, int64_t gstride_b,
                                      int64_t gstride_t, void* workspace, void* stream) {
    SKYRL_REQUIRE(params && logits && labels && old_log_probs && advantages && loss_out && metrics_out && logp_out &&
                      grad_logits && workspace,
                  "policy_train_fwd: null pointer");
    SKYRL_REQUIRE(dtype == SKYRL_BF16, "policy_train_fwd: logits must be bf16");
    SKYRL_REQUIRE(n > 0 && R > 0 && V > 0, "policy_train_fwd: bad sizes");
    SKYRL_REQUIRE(gstride_t >= V && (n == 1 || gstride_b >= (int64_t)(R - 1) * gstride_t + V),
                  "policy_train_fwd: grad_logits rows overlap");
    SKYRL_REQUIRE(temperature > 0.f, "policy_train_fwd: temperature must be > 0");
    SKYRL_REQUIRE(!params->use_kl_loss || ref_log_probs, "policy_train_fwd: use_kl_loss needs ref_log_probs");
    SKYRL_REQUIRE(params->loss_reduction >= 0 && params->loss_reduction <= 2, "policy_train_fwd: bad loss_reduction");
    SKYRL_REQUIRE(params->loss_reduction != 2 || params->max_seq_len > 0.f,
                  "policy_train_fwd: seq_mean_token_sum_norm needs max_seq_len");
    char* w = reinterpret_cast<char*>(workspace);
    float* scal = reinterpret_cast<float*>(w);
    float* row_scale = reinterpret_cast<float*>(w + 256);
    float* tok = reinterpret_cast<float*>(w + pt_tok_off(n));
    auto* gran = reinterpret_cast<unsigned long long*>(w + pt_gran_off(n, R));
    unsigned* err_word = reinterpret_cast<unsigned*>(w) + 32;
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(train_scales_kernel, dim3(1), dim3(kThreads), 0, s, loss_mask, n, R, *params, row_scale, scal);
    int rc = check_launch("train_scales_kernel");
    if (rc) return rc;
    const bool has_t = temperature != 1.0f;
    const int nvec = V / 8;
    auto* out = reinterpret_cast<uint16_t*>(grad_logits);
    const auto* in = reinterpret_cast<const uint16_t*>(logits);
    // dlogits rows must share the logits rows' position within 16 B (then every row's
    // aligned-down span maps slot for slot); both 2-byte aligned.
    const bool same_align = ((reinterpret_cast<uintptr_t>(out) - reinterpret_cast<uintptr_t>(in)) % 16) == 0 &&
                            ((gstride_b - stride_b) % 8) == 0 && ((gstride_t - stride_t) % 8) == 0 &&
                            (reinterpret_cast<uintptr_t>(in) % 2) == 0;
    // Qwen2.5's V = 151,936 at 768 threads x 25 vectors (the variant field train_resident_nt = 768)
    const bool use768 = knobs().train_resident_nt == 768 && nvec <= 25 * 768 && nvec > 24 * 768;
    // rows without partial vectors: 16-B-aligned logits and dlogits rows, V % 8 == 0
    const bool aligned = (V % 8) == 0 && (reinterpret_cast<uintptr_t>(in) % 16) == 0 && (stride_b % 8) == 0 &&
                         (stride_t % 8) == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0 &&
                         (gstride_b % 8) == 0 && (gstride_t % 8) == 0;
    int nv = 0;
    if (aligned) {
        nv = (nvec + 1023) / 1024;
        if (nv > 19) nv = 0;
    } else {
        const int span = (V + 7 + 7) / 8;  // aligned-down span in vectors, worst-case row offset
        for (int cand : kEdgeNV)
            if (span <= cand * 1024) { nv = cand; break; }
    }
    const bool resident_ok = knobs().train_resident && same_align && nv > 0;
    const SplitPlan sp = split_plan(V, aligned, has_t);
    if (knobs().train_split && knobs().train_resident && same_align && sp.kern && (int64_t)n * R * sp.parts < (1ll << 31)) {
        hipLaunchKernelGGL(sp.kern, dim3((unsigned)((int64_t)n * R * sp.parts)), dim3(sp.threads), 0, s, in,
                           stride_b, stride_t, R, V, labels, lstride_b, lstride_t, temperature, old_log_probs,
                           advantages, loss_mask, ref_log_probs, row_scale, scal, *params, logp_out, entropy_out, tok,
                           out, gstride_b, gstride_t, knobs().train_ntstore != 0, gran, err_word, nullptr, (unsigned)knobs().train_split_wait);
    } else if (knobs().train_resident && use768 && aligned) {
        auto kern = has_t ? policy_train_resident_kernel<768, 25, true, false>
                          : policy_train_resident_kernel<768, 25, false, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)((int64_t)n * R)), dim3(768), 0, s, in, stride_b, stride_t, R, V, labels,
                           lstride_b, lstride_t, temperature, old_log_probs, advantages, loss_mask, ref_log_probs,
                           row_scale, scal, *params, logp_out, entropy_out, tok, out, gstride_b, gstride_t,
                           knobs().train_ntstore != 0);
    } else if (resident_ok) {
        hipLaunchKernelGGL(aligned ? resident_aligned_for(nv, has_t) : resident_edge_for(nv, has_t),
                           dim3((unsigned)((int64_t)n * R)), dim3(1024), 0, s, in, stride_b, stride_t, R, V, labels,
                           lstride_b, lstride_t, temperature, old_log_probs, advantages, loss_mask, ref_log_probs,
                           row_scale, scal, *params, logp_out, entropy_out, tok, out, gstride_b, gstride_t,
                           knobs().train_ntstore != 0);
    } else
    hipLaunchKernelGGL(policy_train_kernel, dim3((unsigned)((int64_t)n * R)), dim3(kThreads), 0, s, in, stride_b,
                       stride_t, R, (int64_t)n * R, V, labels, lstride_b, lstride_t, temperature, has_t, old_log_probs,
                       advantages, loss_mask, ref_log_probs, row_scale, scal, *params, logp_out, entropy_out, tok, out,
                       gstride_b, gstride_t, knobs().train_ntstore != 0);
    rc = check_launch("policy_train_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(train_epilogue_kernel, dim3(1), dim3(kThreads), 0, s, tok, loss_mask, n, R, *params, scal,
                       loss_out, metrics_out);
    return check_launch("train_epilogue_kernel");
}

// Ragged (sample-packed) form: ntok tokens whose logits rows are dense [ntok, V] (row q at
// logits + q * ld), token q standing at [n, R] position token_pos[q] of the per-token arrays
// (old / adv / mask / ref / logp_out / entropy_out, all [n, R]); positions no token maps to must
// carry mask 0 (the padding of a packed batch). Loss, metrics and per-row scales are those of
// the dense call on the padded [n, R] batch; dlogits rows are [ntok, V] at grad_logits + q * ld_grad.
// Runs the split-row kernel only (its EDGE form for rows not 16-B aligned or V % 8 != 0).
extern "C" int skyrl_policy_train_ragged_fwd(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V,
                                             const int64_t* labels, const int32_t* token_pos, int32_t n, int32_t R,
                                             float temperature, const float* old_log_probs, const float* advantages,
                                             const float* loss_mask, const float* ref_log_probs,
                                             const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                                             float* logp_out, float* entropy_out, void* grad_logits, int64_t ld_grad,
                                             void* workspace, void* stream) {
    SKYRL_REQUIRE(params && logits && labels && token_pos && old_log_probs && advantages && loss_mask && loss_out &&
                      metrics_out && logp_out && grad_logits && workspace,
                  "policy_train_ragged_fwd: null pointer");
    SKYRL_REQUIRE(dtype == SKYRL_BF16, "policy_train_ragged_fwd: logits must be bf16");
    SKYRL_REQUIRE(ntok > 0 && n > 0 && R > 0 && V > 0 && (int64_t)ntok <= (int64_t)n * R,
                  "policy_train_ragged_fwd: bad sizes");
    SKYRL_REQUIRE(temperature > 0.f, "policy_train_ragged_fwd: temperature must be > 0");
    SKYRL_REQUIRE(!params->use_kl_loss || ref_log_probs, "policy_train_ragged_fwd: use_kl_loss needs ref_log_probs");
    SKYRL_REQUIRE(params->loss_reduction >= 0 && params->loss_reduction <= 2,
                  "policy_train_ragged_fwd: bad loss_reduction");
    SKYRL_REQUIRE(params->loss_reduction != 2 || params->max_seq_len > 0.f,
                  "policy_train_ragged_fwd: seq_mean_token_sum_norm needs max_seq_len");
    const auto lgp = reinterpret_cast<uintptr_t>(logits), grp = reinterpret_cast<uintptr_t>(grad_logits);
    // rows without partial vectors take the plain split kernel, others (GPT-2's odd V) its EDGE
    // form; either way every dlogits row must sit at its logits row's offset within 16 B
    const bool aligned = (V % 8) == 0 && (ld % 8) == 0 && (ld_grad % 8) == 0 && lgp % 16 == 0 && grp % 16 == 0;
    const SplitPlan sp = split_plan(V, aligned, temperature != 1.0f);
    SKYRL_REQUIRE(sp.kern != nullptr, "policy_train_ragged_fwd: V outside the split kernel's range (V <= 155,648, or "
                           "114,688 for rows not 16-B aligned)");
    SKYRL_REQUIRE(ld >= V && ld_grad >= V && lgp % 2 == 0 && (grp - lgp) % 16 == 0 && (ld_grad - ld) % 8 == 0,
                  "policy_train_ragged_fwd: dlogits rows must share the logits rows' offset within 16 B");
    SKYRL_REQUIRE((int64_t)ntok * sp.parts < (1ll << 31), "policy_train_ragged_fwd: too many tokens for one launch");
    char* w = reinterpret_cast<char*>(workspace);
    float* scal = reinterpret_cast<float*>(w);
    float* row_scale = reinterpret_cast<float*>(w + 256);
    float* tok = reinterpret_cast<float*>(w + pt_tok_off(n));
    auto* gran = reinterpret_cast<unsigned long long*>(w + pt_gran_off(n, R));
    unsigned* err_word = reinterpret_cast<unsigned*>(w) + 32;
    hipStream_t s = as_stream(stream);
    // positions no token maps to are folded by the epilogue with mask 0: their terms must be 0
    SKYRL_REQUIRE(hipMemsetAsync(tok, 0, (size_t)n * R * 16, s) == hipSuccess, "policy_train_ragged_fwd: memset");
    hipLaunchKernelGGL(train_scales_kernel, dim3(1), dim3(kThreads), 0, s, loss_mask, n, R, *params, row_scale, scal);
    int rc = check_launch("train_scales_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(sp.kern, dim3((unsigned)((int64_t)ntok * sp.parts)), dim3(sp.threads), 0, s, reinterpret_cast<const uint16_t*>(logits), (int64_t)0, ld, R, V,
                       labels, (int64_t)0, (int64_t)1, temperature, old_log_probs, advantages, loss_mask, ref_log_probs,
                       row_scale, scal, *params, logp_out, entropy_out, tok, reinterpret_cast<uint16_t*>(grad_logits),
                       (int64_t)0, ld_grad, knobs().train_ntstore != 0, gran, err_word, token_pos, (unsigned)knobs().train_split_wait);
    rc = check_launch("policy_train_split_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(train_epilogue_kernel, dim3(1), dim3(kThreads), 0, s, tok, loss_mask, n, R, *params, scal,
                       loss_out, metrics_out);
    return check_launch("train_epilogue_kernel");
}

extern "C" int skyrl_scale_bf16_by_device_scalar(const float* g, void* x, int64_t n, void* stream) {
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(g && x && (reinterpret_cast<uintptr_t>(x) % 16) == 0, "scale_bf16: null/misaligned pointer");
    int64_t blocks = (n / 8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(scale_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), g,
                       reinterpret_cast<uint16_t*>(x), n);
    return check_launch("scale_bf16_kernel");
}

// ---- step form (ABI 8): one plan and one fold per mini-batch instead of two single-workgroup
// launches per micro-batch. The reference's micro-batch loop (workers/worker.py:731-900) reads
// loss and metrics only after the mini-batch's backward passes (optim_step, :900-925), so the
// per-micro-batch fold can wait until then; the scales depend only on the loss mask, so one plan
// launch computes every micro-batch's before the first pass.
// Step workspace: [0, 256) header, micro slots (kStepSlot B each: scal[0..2], word 16 the launch's
// exchange tag, word 32 its timeout flag), row scales (n_total floats), per-token records
// (n_total * R x 16 B), the exchange granules of one micro-batch (reused by every launch; the
// tags keep launches apart). Zeroed once at allocation.
namespace {
constexpr int kStepMaxMicro = 4096;  // the tag's low 12 bits
int step_micro_count(int32_t n_total, int32_t mb) { return (n_total + mb - 1) / mb; }
size_t st_rows_off(int nm) { return 256 + pt_pad((size_t)nm * kStepSlot); }
size_t st_rsum_off(int32_t n_total, int nm) { return st_rows_off(nm) + pt_pad((size_t)n_total * 4); }
size_t st_recs_off(int32_t n_total, int nm) { return st_rsum_off(n_total, nm) + pt_pad((size_t)n_total * 4); }
size_t st_tok_off(int32_t n_total, int nm) { return st_recs_off(n_total, nm) + pt_pad((size_t)n_total * 5 * 8); }
size_t st_gran_off(int32_t n_total, int32_t R, int nm) { return st_tok_off(n_total, nm) + pt_pad((size_t)n_total * R * 16); }
const char* step_check(int32_t n_total, int32_t R, int32_t mb, const skyrl_ppo_params* params) {
    if (n_total <= 0 || R <= 0 || mb <= 0) return "bad sizes";
    if (step_micro_count(n_total, mb) > kStepMaxMicro) return "more than 4096 micro-batches";
    if (!params) return "null params";
    if (params->loss_reduction < 0 || params->loss_reduction > 2) return "bad loss_reduction";
    if (params->loss_reduction == 2 && !(params->max_seq_len > 0.f)) return "seq_mean_token_sum_norm needs max_seq_len";
    return nullptr;
}
}  // namespace

extern "C" size_t skyrl_policy_train_step_workspace_bytes(int32_t n_total, int32_t R, int32_t micro_rows) {
    if (n_total <= 0 || R <= 0 || micro_rows <= 0) return 256;
    const int nm = step_micro_count(n_total, micro_rows);
    return st_gran_off(n_total, R, nm) + (size_t)min(micro_rows, n_total) * R * kSplitMaxP * 3 * 8;
}

namespace {
int launch_plan(const float* loss_mask, int32_t n_total, int32_t R, int32_t micro_rows, const skyrl_ppo_params* params,
                const float* scores, const void* rmask, int mask_dtype, int32_t G, float eps, int32_t norm_by_std,
                float* adv, const float* pack_rsum, void* workspace, hipStream_t stream) {
    char* w = reinterpret_cast<char*>(workspace);
    const int nm = step_micro_count(n_total, micro_rows);
    float* rows = reinterpret_cast<float*>(w + st_rows_off(nm));
    float* rsum = reinterpret_cast<float*>(w + st_rsum_off(n_total, nm));
    const dim3 grid((unsigned)((n_total + kStepRows - 1) / kStepRows));
    auto k = mask_dtype == SKYRL_I64   ? train_plan_kernel<SKYRL_I64>
             : mask_dtype == SKYRL_F32 ? train_plan_kernel<SKYRL_F32>
             : mask_dtype == SKYRL_I32 ? train_plan_kernel<SKYRL_I32>
                                       : train_plan_kernel<SKYRL_U8>;
    hipLaunchKernelGGL(k, grid, dim3(kStepRows * kWave), 0, stream, loss_mask, n_total, R, micro_rows, *params, rows,
                       rsum, w + 256, scores, rmask, G, eps, norm_by_std, adv, pack_rsum);
    return check_launch("train_plan_kernel");
}
}  // namespace

extern "C" int skyrl_policy_train_plan(const float* loss_mask, int32_t n_total, int32_t R, int32_t micro_rows,
                                       const skyrl_ppo_params* params, void* workspace, void* stream) {
    SKYRL_REQUIRE(loss_mask && workspace, "policy_train_plan: null pointer");
    const char* bad = step_check(n_total, R, micro_rows, params);
    SKYRL_REQUIRE(bad == nullptr, bad ? bad : "");
    return launch_plan(loss_mask, n_total, R, micro_rows, params, nullptr, nullptr, SKYRL_F32, 1, 0.f, 0, nullptr,
                       nullptr, workspace, as_stream(stream));
}

extern "C" int skyrl_policy_train_plan_grpo(const float* loss_mask, int32_t n_total, int32_t R, int32_t micro_rows,
                                            const skyrl_ppo_params* params, const float* scores,
                                            const void* response_mask, int mask_dtype, int32_t group_size,
                                            float epsilon, int32_t norm_by_std, float* advantages,
                                            const float* loss_mask_row_sum, void* workspace, void* stream) {
    SKYRL_REQUIRE(loss_mask && workspace && scores && response_mask && advantages,
                  "policy_train_plan_grpo: null pointer");
    const char* bad = step_check(n_total, R, micro_rows, params);
    SKYRL_REQUIRE(bad == nullptr, bad ? bad : "");
    SKYRL_REQUIRE(group_size >= 1 && group_size <= kWave && n_total % group_size == 0,
                  "policy_train_plan_grpo: contiguous groups of 1..64 rows dividing the rows");
    SKYRL_REQUIRE(mask_dtype == SKYRL_F32 || mask_dtype == SKYRL_I64 || mask_dtype == SKYRL_I32 ||
                      mask_dtype == SKYRL_U8,
                  "policy_train_plan_grpo: unsupported mask dtype");
    SKYRL_REQUIRE((R % 4) != 0 || ((reinterpret_cast<uintptr_t>(advantages) | reinterpret_cast<uintptr_t>(response_mask)) % 16) == 0,
                  "policy_train_plan_grpo: advantages / response mask must be 16-B aligned");
    return launch_plan(loss_mask, n_total, R, micro_rows, params, scores, response_mask, mask_dtype, group_size,
                       epsilon, norm_by_std, advantages, loss_mask_row_sum, workspace, as_stream(stream));
}

extern "C" int skyrl_policy_train_micro_fwd(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V,
                                            const int64_t* labels, int64_t label_stride_b, int64_t label_stride_t,
                                            const int32_t* token_pos, int32_t micro, int32_t n_total, int32_t R,
                                            int32_t micro_rows, float temperature, const float* old_log_probs,
                                            const float* advantages, const float* loss_mask,
                                            const float* ref_log_probs, const skyrl_ppo_params* params,
                                            float* logp_out, float* entropy_out, void* grad_logits, int64_t ld_grad,
                                            void* workspace, void* stream) {
    SKYRL_REQUIRE(logits && labels && old_log_probs && advantages && loss_mask && logp_out && grad_logits && workspace,
                  "policy_train_micro_fwd: null pointer");
    const char* bad = step_check(n_total, R, micro_rows, params);
    SKYRL_REQUIRE(bad == nullptr, bad ? bad : "");
    SKYRL_REQUIRE(dtype == SKYRL_BF16, "policy_train_micro_fwd: logits must be bf16");
    const int nm = step_micro_count(n_total, micro_rows);
    SKYRL_REQUIRE(micro >= 0 && micro < nm, "policy_train_micro_fwd: micro-batch index out of range");
    const int32_t r0 = micro * micro_rows;
    const int32_t n = min(n_total, r0 + micro_rows) - r0;
    SKYRL_REQUIRE(ntok > 0 && (int64_t)ntok <= (int64_t)n * R && (token_pos || (int64_t)ntok == (int64_t)n * R),
                  "policy_train_micro_fwd: bad token count (dense launches cover the micro-batch's n x R positions)");
    SKYRL_REQUIRE(temperature > 0.f, "policy_train_micro_fwd: temperature must be > 0");
    SKYRL_REQUIRE(!params->use_kl_loss || ref_log_probs, "policy_train_micro_fwd: use_kl_loss needs ref_log_probs");
    const auto lgp = reinterpret_cast<uintptr_t>(logits), grp = reinterpret_cast<uintptr_t>(grad_logits);
    const bool aligned = (V % 8) == 0 && (ld % 8) == 0 && (ld_grad % 8) == 0 && lgp % 16 == 0 && grp % 16 == 0;
    const SplitPlan sp = split_plan(V, aligned, temperature != 1.0f);
    SKYRL_REQUIRE(sp.kern != nullptr, "policy_train_micro_fwd: V outside the split kernel's range (V <= 155,648, or "
                           "114,688 for rows not 16-B aligned)");
    SKYRL_REQUIRE(ld >= V && ld_grad >= V && lgp % 2 == 0 && (grp - lgp) % 16 == 0 && (ld_grad - ld) % 8 == 0,
                  "policy_train_micro_fwd: dlogits rows must share the logits rows' offset within 16 B");
    SKYRL_REQUIRE((int64_t)ntok * sp.parts < (1ll << 31), "policy_train_micro_fwd: too many tokens for one launch");
    char* w = reinterpret_cast<char*>(workspace);
    float* scal = reinterpret_cast<float*>(w + 256 + (size_t)micro * kStepSlot);
    float* row_scale = reinterpret_cast<float*>(w + st_rows_off(nm)) + r0;
    float* tok = reinterpret_cast<float*>(w + st_tok_off(n_total, nm)) + (int64_t)r0 * R * 4;
    auto* gran = reinterpret_cast<unsigned long long*>(w + st_gran_off(n_total, R, nm));
    unsigned* err_word = reinterpret_cast<unsigned*>(scal) + 32;
    const int64_t o = (int64_t)r0 * R;
    // dense: position (b, t) of the micro-batch is logits row b * R + t; packed: row q is token q
    const int64_t sb = token_pos ? 0 : (int64_t)R * ld, gsb = token_pos ? 0 : (int64_t)R * ld_grad;
    const int64_t lsb = token_pos ? 0 : label_stride_b;
    hipLaunchKernelGGL(sp.kern, dim3((unsigned)((int64_t)ntok * sp.parts)), dim3(sp.threads), 0, as_stream(stream),
                       reinterpret_cast<const uint16_t*>(logits), sb, ld, R, V, labels, lsb, label_stride_t,
                       temperature, old_log_probs + o, advantages + o, loss_mask + o,
                       ref_log_probs ? ref_log_probs + o : nullptr, row_scale, scal, *params, logp_out + o,
                       entropy_out ? entropy_out + o : nullptr, tok, reinterpret_cast<uint16_t*>(grad_logits), gsb,
                       ld_grad, knobs().train_ntstore != 0, gran, err_word, token_pos, (unsigned)knobs().train_split_wait);
    return check_launch("policy_train_split_kernel");
}

extern "C" int skyrl_policy_train_fold(const float* loss_mask, int32_t n_total, int32_t R, int32_t micro_rows,
                                       const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                                       void* workspace, void* stream) {
    SKYRL_REQUIRE(loss_mask && loss_out && metrics_out && workspace, "policy_train_fold: null pointer");
    const char* bad = step_check(n_total, R, micro_rows, params);
    SKYRL_REQUIRE(bad == nullptr, bad ? bad : "");
    char* w = reinterpret_cast<char*>(workspace);
    const int nm = step_micro_count(n_total, micro_rows);
    hipLaunchKernelGGL(train_fold_kernel, dim3((unsigned)((n_total + kStepRows - 1) / kStepRows)),
                       dim3(kStepRows * kWave), 0, as_stream(stream),
                       reinterpret_cast<const float*>(w + st_tok_off(n_total, nm)), loss_mask, n_total, R,
                       micro_rows, *params, w + 256, reinterpret_cast<double*>(w + st_recs_off(n_total, nm)), loss_out,
                       metrics_out);
    return check_launch("train_fold_kernel");
}

// 1 when the packed / step forms (split kernel) take vocabulary V: rows 16-B aligned with
// V % 8 == 0 (aligned = 1) or otherwise (the EDGE form), at this temperature; the same plan
// the launches make, so a host that asks first never gets their range error.
extern "C" int skyrl_policy_train_supports(int32_t V, int32_t aligned, float temperature) {
    if (V <= 0 || !(temperature > 0.f)) return 0;
    return split_plan(V, aligned != 0 && (V % 8) == 0, temperature != 1.0f).kern != nullptr ? 1 : 0;
}


