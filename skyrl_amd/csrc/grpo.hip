// a4: GRPO outcome advantage (reference: utils/ppo_utils.py:1132-1182).
//
// One launch over the whole [N,R] batch. Grid = (group, 256-column slice). Two kernels:
// grpo_adv_contig_kernel for contiguous equal-size groups (the trainer's layout, no index
// loads) and grpo_adv_kernel for arbitrary CSR groups.
// Every block of a group recomputes the group's row sums (the rewards of one
// group are G*R*4 B = 32 KB at G=8, R=1024: re-read from L2/MALL, not HBM), so
// no inter-workgroup hand-off is needed; slice s then writes its 256 columns
// of adv*mask for all rows of the group. Row sums use a fixed reduction tree,
// so every slice sees bit-identical scores. Group stats in fp64 (torch.std on
// CPU accumulates in double), the normalisation itself in fp32 as the
// reference does.
#include "arrive.h"
#include "variant.h"

namespace skyrl {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kSlice = 256;          // columns written per block
constexpr int kMaxCachedRows = 1024; // scores cached in LDS; larger groups recompute

// Sum of one reward row by one wave (all lanes get the result).
__device__ float row_sum_wave(const float* __restrict__ row, int R, bool vec4) {
    const int lane = threadIdx.x & (kWave - 1);
    float acc = 0.f;
    if (vec4) {
        const float4* r4 = reinterpret_cast<const float4*>(row);
        const int n4 = R >> 2;
        for (int i = lane; i < n4; i += kWave) {
            float4 v = r4[i];
            acc += (v.x + v.y) + (v.z + v.w);
        }
    } else {
        for (int i = lane; i < R; i += kWave) acc += row[i];
    }
    return wave_sum(acc);
}

__global__ __launch_bounds__(kThreads) void grpo_adv_kernel(
    const float* __restrict__ rewards, const float* __restrict__ scores_in, const void* __restrict__ mask, int mask_dtype,
    const int32_t* __restrict__ group_off, const int32_t* __restrict__ group_rows, int R,
    float epsilon, int norm_by_std, bool vec4, float* __restrict__ out, float* __restrict__ scores_out) {
    __shared__ float s_scores[kMaxCachedRows];
    __shared__ float s_stat[2];  // mean, denom (std + eps) or 1

    const int g = blockIdx.x;
    const int slice = blockIdx.y;
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    const int beg = group_off[g];
    const int n = group_off[g + 1] - beg;

    // Phase 1: row sums (score = token_level_rewards.sum(-1), ppo_utils.py:1156).
    for (int j = w; j < n && j < kMaxCachedRows; j += kWaves) {
        const int row = group_rows[beg + j];
        float s = scores_in ? scores_in[row] : row_sum_wave(rewards + (int64_t)row * R, R, vec4);
        if (lane == 0) {
            s_scores[j] = s;
            if (scores_out && slice == 0) scores_out[row] = s;
        }
    }
    __syncthreads();

    // Phase 2: group mean / unbiased std (ppo_utils.py:1164-1175), wave 0.
    if (w == 0) {
        auto score_of = [&](int j) -> float {
            if (j < kMaxCachedRows) return s_scores[j];
            const int row = group_rows[beg + j];
            if (scores_in) return scores_in[row];
            const float* r = rewards + (int64_t)row * R;
            float acc = 0.f;
            for (int i = 0; i < R; ++i) acc += r[i];
            return acc;
        };
        float mean_f, denom_f;
        if (n <= 1) {
            mean_f = 0.f;   // singleton group: mean 0, std 1 (ppo_utils.py:1167-1169)
            denom_f = norm_by_std ? (1.f + epsilon) : 1.f;
        } else {
            double sum = 0.0;
            for (int j = lane; j < n; j += kWave) sum += (double)score_of(j);
            sum = wave_sum(sum);
            const double mean = sum / (double)n;
            double m2 = 0.0;
            for (int j = lane; j < n; j += kWave) {
                double d = (double)score_of(j) - mean;
                m2 += d * d;
            }
            m2 = wave_sum(m2);
            mean_f = (float)mean;
            const float std_f = (float)sqrt(m2 / (double)(n - 1));
            denom_f = norm_by_std ? (std_f + epsilon) : 1.f;
        }
        if (lane == 0) {
            s_stat[0] = mean_f;
            s_stat[1] = denom_f;
        }
    }
    __syncthreads();
    const float mean = s_stat[0];
    const float denom = s_stat[1];

    // Phase 3: out[row, slice cols] = ((score - mean) / denom) * mask.
    const int col0 = slice * kSlice + lane * 4;
    for (int j = w; j < n; j += kWaves) {
        const int row = group_rows[beg + j];
        float score;
        if (j < kMaxCachedRows) {
            score = s_scores[j];
        } else {
            score = scores_in ? scores_in[row] : row_sum_wave(rewards + (int64_t)row * R, R, vec4);
        }
        const float a = norm_by_std ? (score - mean) / denom : (score - mean);
        const int64_t base = (int64_t)row * R;
        if (vec4 && col0 + 3 < R) {
            float m[4];
            load_mask4(mask, mask_dtype, base + col0, m);
            float4 o = make_float4(a * m[0], a * m[1], a * m[2], a * m[3]);
            *reinterpret_cast<float4*>(out + base + col0) = o;
        } else {
            for (int c = col0; c < col0 + 4 && c < R; ++c) out[base + c] = a * load_mask(mask, mask_dtype, base + c);
        }
    }
}

// Contiguous uniform groups (rows [g*G, (g+1)*G), the layout generators/utils.py:373-393
// produces, G <= kMaxFastG): one block per group, one wave per row, no index loads. Each
// wave issues its whole row (rewards and mask) before the first wait, sums the rewards (same
// per-lane order and wave tree as row_sum_wave, so scores are bit-identical to the CSR
// kernel), and after ONE barrier every wave derives the group stats from the G scores in LDS
// and writes its row. One dependent memory round trip plus the stores; few, wide blocks keep
// the dispatch ramp short (phase probe: 512 small blocks take ~4.6 us just to dispatch).
constexpr int kMaxFastG = 16;
constexpr int kFastUnroll = 4;  // 16-B vectors per lane issued together

template <int MDT>
__global__ __launch_bounds__(kMaxFastG * kWave) void grpo_adv_contig_kernel(
    const float* __restrict__ rewards, const float* __restrict__ scores_in, const void* __restrict__ mask, int G, int R,
    float epsilon, int norm_by_std, float* __restrict__ out, float* __restrict__ scores_out) {
    __shared__ float s_scores[kMaxFastG];
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;  // row within the group
    const int64_t row = (int64_t)blockIdx.x * G + w;
    const float* rrow = rewards + row * R;
    const int n4 = R >> 2;
    float acc = 0.f;
    float m[kFastUnroll][4];
    int i0 = lane;
    if (scores_in) {  // given scores: only the mask is read
        acc = scores_in[row];
#pragma unroll
        for (int u = 0; u < kFastUnroll; ++u) {
            const int i = i0 + u * kWave;
            if (i < n4) load_mask4(mask, MDT, row * R + 4 * i, m[u]);
        }
    } else {
        // first kFastUnroll vectors of rewards and mask in flight together (R = 1024: the whole row)
        {
            float4 v[kFastUnroll];
#pragma unroll
            for (int u = 0; u < kFastUnroll; ++u) {
                const int i = i0 + u * kWave;
                v[u] = i < n4 ? reinterpret_cast<const float4*>(rrow)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
                if (i < n4) load_mask4(mask, MDT, row * R + 4 * i, m[u]);
            }
#pragma unroll
            for (int u = 0; u < kFastUnroll; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
        }
        for (int i = i0 + kFastUnroll * kWave; i < n4; i += kWave) {  // longer rows (same per-lane order)
            const float4 v = reinterpret_cast<const float4*>(rrow)[i];
            acc += (v.x + v.y) + (v.z + v.w);
        }
        acc = wave_sum(acc);
    }
    if (lane == 0) {
        s_scores[w] = acc;
        if (scores_out) scores_out[row] = acc;
    }
    __syncthreads();
    float mean_f, denom_f;
    if (G <= 1) {
        mean_f = 0.f;  // singleton group: mean 0, std 1 (ppo_utils.py:1167-1169)
        denom_f = norm_by_std ? (1.f + epsilon) : 1.f;
    } else {  // fp64 like torch.std on CPU
        double sum = 0.0;
        for (int j = 0; j < G; ++j) sum += (double)s_scores[j];
        const double mean = sum / (double)G;
        double m2 = 0.0;
        for (int j = 0; j < G; ++j) {
            const double d = (double)s_scores[j] - mean;
            m2 += d * d;
        }
        mean_f = (float)mean;
        const float std_f = (float)sqrt(m2 / (double)(G - 1));
        denom_f = norm_by_std ? (std_f + epsilon) : 1.f;
    }
    const float sc = s_scores[w];
    const float a = norm_by_std ? (sc - mean_f) / denom_f : (sc - mean_f);
    float4* orow = reinterpret_cast<float4*>(out + row * R);
#pragma unroll
    for (int u = 0; u < kFastUnroll; ++u) {
        const int i = i0 + u * kWave;
        if (i < n4) orow[i] = make_float4(a * m[u][0], a * m[u][1], a * m[u][2], a * m[u][3]);
    }
    for (int i = i0 + kFastUnroll * kWave; i < n4; i += kWave) {
        float mm[4];
        load_mask4(mask, MDT, row * R + 4 * i, mm);
        orow[i] = make_float4(a * mm[0], a * mm[1], a * mm[2], a * mm[3]);
    }
}


// Contiguous uniform groups spread over S column slices per group (S in {2, 4}): a block per
// (group, slice), one wave per row. Every block of a group sums the group's whole reward rows
// (same per-lane order and tree as above, so all slices see bit-identical scores) but reads
// the mask and writes the advantages of its own R/S columns only. The slices of a group are
// placed on the same XCD (blocks are dispatched round-robin over the 8 XCDs, so block b runs
// on XCD b % 8): their repeated reward reads hit that XCD's L2, and 4x as many CUs stream the
// mask/advantage bytes as in the one-block-per-group form.
template <int MDT, int S>
__global__ __launch_bounds__(kMaxFastG * kWave) void grpo_adv_sliced_kernel(
    const float* __restrict__ rewards, const float* __restrict__ scores_in, const void* __restrict__ mask,
    int num_groups, int G, int R, float epsilon, int norm_by_std, float* __restrict__ out,
    float* __restrict__ scores_out) {
    __shared__ float s_scores[kMaxFastG];
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int k = b >> 3;
    const int slice = k % S;
    const int group = (k / S) * 8 + xcd;
    if (group >= num_groups) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    const int64_t row = (int64_t)group * G + w;
    const float* rrow = rewards + row * R;
    const int n4 = R >> 2;
    const int sw = (n4 + S - 1) / S;  // 16-B vectors per slice
    const int s0 = slice * sw, s1 = (s0 + sw < n4) ? s0 + sw : n4;
    // this lane's slice vector (the common R = 1024, S = 4 case: exactly one) and its reward
    // vectors, all issued before the first wait
    const int vi = s0 + lane;
    float m[4] = {0.f, 0.f, 0.f, 0.f};
    if (vi < s1) load_mask4(mask, MDT, row * R + 4 * vi, m);
    float acc = 0.f;
    if (scores_in) {
        acc = scores_in[row];
    } else {
        {
            float4 v[kFastUnroll];
#pragma unroll
            for (int u = 0; u < kFastUnroll; ++u) {
                const int i = lane + u * kWave;
                v[u] = i < n4 ? reinterpret_cast<const float4*>(rrow)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < kFastUnroll; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
        }
        for (int i = lane + kFastUnroll * kWave; i < n4; i += kWave) {
            const float4 v = reinterpret_cast<const float4*>(rrow)[i];
            acc += (v.x + v.y) + (v.z + v.w);
        }
        acc = wave_sum(acc);
    }
    if (lane == 0) {
        s_scores[w] = acc;
        if (scores_out && slice == 0) scores_out[row] = acc;
    }
    __syncthreads();
    float mean_f, denom_f;
    if (G <= 1) {
        mean_f = 0.f;
        denom_f = norm_by_std ? (1.f + epsilon) : 1.f;
    } else {
        double sum = 0.0;
        for (int j = 0; j < G; ++j) sum += (double)s_scores[j];
        const double mean = sum / (double)G;
        double m2 = 0.0;
        for (int j = 0; j < G; ++j) {
            const double d = (double)s_scores[j] - mean;
            m2 += d * d;
        }
        mean_f = (float)mean;
        const float std_f = (float)sqrt(m2 / (double)(G - 1));
        denom_f = norm_by_std ? (std_f + epsilon) : 1.f;
    }
    const float sc = s_scores[w];
    const float a = norm_by_std ? (sc - mean_f) / denom_f : (sc - mean_f);
    float4* orow = reinterpret_cast<float4*>(out + row * R);
    if (vi < s1) orow[vi] = make_float4(a * m[0], a * m[1], a * m[2], a * m[3]);
    for (int i = vi + kWave; i < s1; i += kWave) {
        float mm[4];
        load_mask4(mask, MDT, row * R + 4 * i, mm);
        orow[i] = make_float4(a * mm[0], a * mm[1], a * mm[2], a * mm[3]);
    }
}

// ---- advantage_batch_normalize (ppo_utils.py:127-145, called at trainer.py:275-276) -----------
// mean over EVERY element (unmasked), masked sum of squared deviations / mask sum, rstd =
// rsqrt(clamp(., 1e-8)), out = (adv - mean) * rstd (not re-masked). Two launches so that a DP
// caller can all-reduce the five fp64 sums in between (one all-reduce of scalars):
//   stats: per block fp64 (sum a, sum m, sum a m, sum a^2 m) over a contiguous range, the last
//          arriving block folds the block records in block order (deterministic) and appends
//          the element count; sum (a - mu)^2 m = sum a^2 m - 2 mu sum a m + mu^2 sum m in fp64
//   apply: mean / rstd from the sums (every block, scalar loads), one streaming pass.
constexpr int kNormThreads = 256;
constexpr int kNormMaxBlocks = 512;

template <int MDT>
__global__ __launch_bounds__(kNormThreads) void adv_norm_stats_kernel(const float* __restrict__ adv,
                                                                     const void* __restrict__ mask, int64_t n,
                                                                     int64_t per_block, bool vec4,
                                                                     double* __restrict__ parts,
                                                                     unsigned* __restrict__ counter,
                                                                     double* __restrict__ sums_out) {
    __shared__ double s_red[(kNormThreads / kWave) * 4];
    __shared__ int s_last;
    const int64_t b0 = (int64_t)blockIdx.x * per_block;
    const int64_t b1 = min(n, b0 + per_block);
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    auto add = [&](float a, float m) {
        const double ad = a, md = m;
        v[0] += ad;
        v[1] += md;
        v[2] += ad * md;
        v[3] += ad * ad * md;
    };
    if (vec4) {  // b0, b1 multiples of 4 (per_block is), n % 4 == 0
        for (int64_t i = b0 + 4 * (int64_t)threadIdx.x; i < b1; i += 4 * kNormThreads) {
            const float4 a = *reinterpret_cast<const float4*>(adv + i);
            float m[4];
            mask4_to_float<MDT>(load_mask4_raw<MDT>(mask, i), m);
            add(a.x, m[0]);
            add(a.y, m[1]);
            add(a.z, m[2]);
            add(a.w, m[3]);
        }
    } else {
        for (int64_t i = b0 + threadIdx.x; i < b1; i += kNormThreads) add(adv[i], load_mask(mask, MDT, i));
    }
    block_sum_d<kNormThreads / kWave, 4>(v, s_red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) st_wt(parts + (int64_t)blockIdx.x * 4 + k, v[k]);
    }
    if (!arrive_last(counter, gridDim.x, &s_last)) return;
    if (threadIdx.x < kWave) {  // wave 0: lane l folds blocks l, l+64, ... in order, then a fixed tree
        double t[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = threadIdx.x; j < (int)gridDim.x; j += kWave) {
#pragma unroll
            for (int k = 0; k < 4; ++k) t[k] += __hip_atomic_load(parts + (int64_t)j * 4 + k, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = wave_sum_dpp(t[k]);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) sums_out[k] = t[k];
            sums_out[4] = (double)n;
            rearm(counter);
        }
    }
}

__global__ __launch_bounds__(kNormThreads) void adv_norm_apply_kernel(const float* __restrict__ adv, int64_t n,
                                                                      const double* __restrict__ sums, bool vec4,
                                                                      float* __restrict__ out) {
    // torch: mean = adv.mean() (f32), ss = ((adv - mean)^2 * m).sum(), rstd = (ss / m.sum()).clamp(1e-8).rsqrt()
    const double cnt = sums[4];
    const float mean_f = (float)(sums[0] / cnt);
    const double mu = (double)mean_f;
    const double ss = sums[3] - 2.0 * mu * sums[2] + mu * mu * sums[1];
    double var = ss / sums[1];      // mask sum 0: nan (0/0) or inf, as the reference's
    if (var < 1e-8) var = 1e-8;     // clamp(min=1e-8); a NaN stays NaN (torch.clamp propagates it)
    const float rstd = (float)(1.0 / sqrt(var));
    const int64_t stride = (int64_t)gridDim.x * kNormThreads;
    if (vec4) {
        const int64_t n4 = n >> 2;
        for (int64_t i = (int64_t)blockIdx.x * kNormThreads + threadIdx.x; i < n4; i += stride) {
            float4 a = reinterpret_cast<const float4*>(adv)[i];
            a.x = (a.x - mean_f) * rstd;
            a.y = (a.y - mean_f) * rstd;
            a.z = (a.z - mean_f) * rstd;
            a.w = (a.w - mean_f) * rstd;
            reinterpret_cast<float4*>(out)[i] = a;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNormThreads + threadIdx.x; i < n; i += stride)
            out[i] = (adv[i] - mean_f) * rstd;
    }
}

}  // namespace

}  // namespace skyrl

extern "C" size_t skyrl_adv_norm_workspace_bytes(void) {
    using namespace skyrl;
    return 256 + (size_t)kNormMaxBlocks * 4 * sizeof(double);
}

extern "C" int skyrl_adv_norm_stats(const float* advantages, const void* response_mask, int mask_dtype, int64_t n,
                                    double* sums_out, void* workspace, void* stream) {
    using namespace skyrl;
    SKYRL_REQUIRE(n >= 0, "adv_norm: negative size");
    SKYRL_REQUIRE(advantages && response_mask && sums_out && workspace, "adv_norm: null pointer");
    SKYRL_REQUIRE(mask_dtype == SKYRL_F32 || mask_dtype == SKYRL_I64 || mask_dtype == SKYRL_I32 ||
                      mask_dtype == SKYRL_U8,
                  "adv_norm: unsupported mask dtype");
    SKYRL_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "adv_norm: workspace must be 16-B aligned");
    const size_t mbytes = mask_dtype == SKYRL_I64 ? 8 : mask_dtype == SKYRL_U8 ? 1 : 4;
    const bool vec4 = (n % 4) == 0 && (reinterpret_cast<uintptr_t>(advantages) % 16) == 0 &&
                      (reinterpret_cast<uintptr_t>(response_mask) % (4 * mbytes < 16 ? 4 * mbytes : 16)) == 0;
    // blocks of >= 8 float4 per thread, at most kNormMaxBlocks; a multiple of 4 elements each
    int64_t per = (n + kNormMaxBlocks - 1) / kNormMaxBlocks;
    const int64_t minper = (int64_t)kNormThreads * 32;
    per = per < minper ? minper : per;
    per = (per + 3) / 4 * 4;
    const int blocks = n == 0 ? 1 : (int)((n + per - 1) / per);
    unsigned* counter = reinterpret_cast<unsigned*>(workspace);
    double* parts = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) + 256);
    auto k = mask_dtype == SKYRL_I64   ? adv_norm_stats_kernel<SKYRL_I64>
             : mask_dtype == SKYRL_F32 ? adv_norm_stats_kernel<SKYRL_F32>
             : mask_dtype == SKYRL_I32 ? adv_norm_stats_kernel<SKYRL_I32>
                                       : adv_norm_stats_kernel<SKYRL_U8>;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(kNormThreads), 0, as_stream(stream), advantages, response_mask, n, per,
                       vec4, parts, counter, sums_out);
    return check_launch("adv_norm_stats_kernel");
}

extern "C" int skyrl_adv_norm_apply(const float* advantages, int64_t n, const double* sums, float* out, void* stream) {
    using namespace skyrl;
    SKYRL_REQUIRE(n >= 0, "adv_norm: negative size");
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(advantages && sums && out, "adv_norm: null pointer");
    const bool vec4 = (n % 4) == 0 && (reinterpret_cast<uintptr_t>(advantages) % 16) == 0 &&
                      (reinterpret_cast<uintptr_t>(out) % 16) == 0;
    const int64_t work = vec4 ? n / 4 : n;
    int64_t blocks = (work + kNormThreads - 1) / kNormThreads;
    blocks = blocks > 2048 ? 2048 : blocks;
    hipLaunchKernelGGL(adv_norm_apply_kernel, dim3((unsigned)blocks), dim3(kNormThreads), 0, as_stream(stream),
                       advantages, n, sums, vec4, out);
    return check_launch("adv_norm_apply_kernel");
}

extern "C" int skyrl_grpo_advantage(const float* rewards, const float* scores_in, const void* response_mask,
                                    int mask_dtype,
                                    const int32_t* group_off, const int32_t* group_rows,
                                    int32_t num_groups, int32_t N, int32_t R, float epsilon,
                                    int32_t norm_by_std, float* advantages, float* scores_out,
                                    void* stream) {
    using namespace skyrl;
    SKYRL_REQUIRE(N >= 0 && R >= 0 && num_groups >= 0, "grpo: negative size");
    if (N == 0 || R == 0 || num_groups == 0) return SKYRL_OK;
    SKYRL_REQUIRE((rewards || scores_in) && response_mask && advantages, "grpo: null pointer");
    SKYRL_REQUIRE(mask_dtype == SKYRL_F32 || mask_dtype == SKYRL_I64 || mask_dtype == SKYRL_I32 ||
                      mask_dtype == SKYRL_U8,
                  "grpo: unsupported mask dtype");
    const bool vec4 = (R % 4) == 0 && (reinterpret_cast<uintptr_t>(rewards) % 16) == 0 &&  // (NULL is aligned)
                      (reinterpret_cast<uintptr_t>(advantages) % 16) == 0 &&
                      (reinterpret_cast<uintptr_t>(response_mask) % 16) == 0;
    dim3 grid(num_groups, (R + kSlice - 1) / kSlice);
    if (!group_off && !group_rows) {  // contiguous uniform groups of N / num_groups rows
        SKYRL_REQUIRE(N % num_groups == 0, "grpo: contiguous groups need N % num_groups == 0");
        const int G = N / num_groups;
        if (vec4 && G <= kMaxFastG && knobs().grpo_slices > 1) {
            const int S = knobs().grpo_slices;
            auto pick = [&](auto k2, auto k4) { return S == 2 ? k2 : k4; };
            auto k = mask_dtype == SKYRL_I64   ? pick(grpo_adv_sliced_kernel<SKYRL_I64, 2>, grpo_adv_sliced_kernel<SKYRL_I64, 4>)
                     : mask_dtype == SKYRL_F32 ? pick(grpo_adv_sliced_kernel<SKYRL_F32, 2>, grpo_adv_sliced_kernel<SKYRL_F32, 4>)
                     : mask_dtype == SKYRL_I32 ? pick(grpo_adv_sliced_kernel<SKYRL_I32, 2>, grpo_adv_sliced_kernel<SKYRL_I32, 4>)
                                               : pick(grpo_adv_sliced_kernel<SKYRL_U8, 2>, grpo_adv_sliced_kernel<SKYRL_U8, 4>);
            const int ngp = (num_groups + 7) / 8 * 8;
            hipLaunchKernelGGL(k, dim3(ngp * S), dim3(G * kWave), 0, as_stream(stream), rewards, scores_in,
                               response_mask, num_groups, G, R, epsilon, norm_by_std, advantages, scores_out);
            return check_launch("grpo_adv_sliced_kernel");
        }
        if (vec4 && G <= kMaxFastG) {
            auto k = mask_dtype == SKYRL_I64   ? grpo_adv_contig_kernel<SKYRL_I64>
                     : mask_dtype == SKYRL_F32 ? grpo_adv_contig_kernel<SKYRL_F32>
                     : mask_dtype == SKYRL_I32 ? grpo_adv_contig_kernel<SKYRL_I32>
                                               : grpo_adv_contig_kernel<SKYRL_U8>;
            hipLaunchKernelGGL(k, dim3(num_groups), dim3(G * kWave), 0, as_stream(stream), rewards, scores_in,
                               response_mask, G, R, epsilon, norm_by_std, advantages, scores_out);
            return check_launch("grpo_adv_contig_kernel");
        }
        return fail(SKYRL_ERR_INVALID, "grpo: contiguous form needs R % 4 == 0, 16-B alignment and G <= 16; "
                                       "pass CSR groups otherwise");
    }
    SKYRL_REQUIRE(group_off && group_rows, "grpo: group_off and group_rows are both given or both NULL");
    hipLaunchKernelGGL(grpo_adv_kernel, grid, dim3(kThreads), 0, as_stream(stream), rewards, scores_in,
                       response_mask, mask_dtype, group_off, group_rows, R, epsilon, norm_by_std, vec4,
                       advantages, scores_out);
    return check_launch("grpo_adv_kernel");
}
