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
// Layout: all per-token tensors f32 [n,R] row-major. The policy loss is ONE launch: grid
// (row, 1024-column chunk), 4 tokens per thread; it reads 20 B/token (logp, old, adv, mask,
// ref), writes the final dL/dlogp for a unit upstream gradient (4 B/token) and a 5-float
// record per block, and the last-arriving block folds the records into the scalar loss and
// the metric vector. The backward rescales in place only when the upstream gradient != 1.
// Deferred form (SKYRL_LOSS_DEFER_FOLD): the forward only writes the records, and the
// backward launch (skyrl_ppo_loss_finish) folds them stream-ordered -- no polling -- and
// rescales; loss and metrics are valid once that launch has run.
#include "arrive.h"
#include "variant.h"

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
constexpr int kNP = 5;                // partials: sum l*m, m, clip*m, kl*m*m, ent*m

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// compute_approx_kl on one element (before the mask multiply). Branch-free: every estimator is
// evaluated and the uniform kl_type selects one, so a token's code is one basic block and the
// compiler can interleave the tokens of a thread (a switch split each token into blocks that
// serialised them). Same operations on the same inputs as the switch: identical bits.
__device__ __forceinline__ float approx_kl(float lp, float base, int kl_type) {
    // every operand computed first: a conditional operator over plain values becomes a select,
    // one over expressions (or a call) becomes branches that serialise the thread's tokens
    const float d = lp - base;
    const float k1a = fabsf(d);
    const float k2 = 0.5f * (d * d);
    const float k3x = clampf(base - lp, -20.f, 20.f);
    const float k3 = clampf((expf(k3x) - k3x) - 1.f, -10.f, 10.f);
    const float k23 = kl_type == 2 ? k2 : k3;
    const float k123 = kl_type == 1 ? k1a : k23;
    return kl_type == 0 ? d : k123;
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
    // Branch-free (selects only, so the tokens of a thread interleave; divergent if / else here
    // serialised them): loss1 = -min(surr1, surr2), d1 = d loss1 / d ratio, a tie splitting the
    // gradient in half as torch.min does; the same operations as the branchy form.
    const bool lt = surr1 < surr2, gt = surr2 < surr1;
    const float ns1 = -surr1, ns2 = -surr2;
    const float loss1 = gt ? ns2 : ns1;
    const float d_lt = -A, d_gt = -A * inr, d_tie = -(0.5f * A + 0.5f * A * inr);
    const float d_ge = gt ? d_gt : d_tie;
    const float d1 = lt ? d_lt : d_ge;
    TokenOut o;
    o.clip = (ns2 > ns1) ? 1.f : 0.f;
    const float pg3 = -A * c;
    const bool neg = dual_clip && A < 0.f;
    const bool take3 = neg && pg3 < loss1;
    const bool tie3 = neg && !(pg3 < loss1) && loss1 == pg3;
    o.loss = take3 ? pg3 : loss1;
    const float half_d1 = 0.5f * d1;
    const float d_nt = tie3 ? half_d1 : d1;
    const float d = take3 ? 0.f : d_nt;
    o.dldlp = d * dratio;
    return o;
}

// ---- fused loss: ONE launch writes dL/dlogp (unit upstream gradient) + loss/metrics ----
// Grid (row, 1024-column chunk), 256 threads x 4 tokens: every thread issues its 16-B loads
// of all inputs at once, and the 4 independent tokens give the PPO/KL arithmetic (two
// accurate expf, clamps, selects) ILP within the wave. The reduction scale of every token is
// known before the loss is: it depends on the loss mask only (token_mean 1/max(sum m, 1),
// sequence_mean 1/(n*max(row m, 1)), seq_mean_token_sum_norm 1/(n*max_seq_len)), and the
// per-row mask sums come in with the batch (pack emits them). So the gradient is final when
// written: 4 B/token out for 20 B/token in.
//
// The scalar loss and the metrics come out of the same launch, and they need no per-row
// state at fold time: with the row sums known up front, every reported quantity is a LINEAR
// sum of per-token terms -- sum l*m*w_row (w = 1, 1/max(row m, 1) or 1/max_seq_len by
// reduction), sum clip*m, sum kl*m*m/max(row m, 1), sum ent*m, sum m -- so each block
// reduces its tokens to 5 numbers. Those are folded without any atomic read-modify-write
// (one ticket counter hit by every block serialises at the L2, about 10 ns per block
// measured: +5 us at 512 blocks, +80 us at 8192): each block publishes its 5 partials as
// 8-byte {epoch, value} granules (one write-through 64-bit store each, untorn: guide G16
// R2), laid out value-major so the folder's loads coalesce, and ONE designated block (the last
// of the grid, after its own tokens) waits in a fixed order until every tag carries this
// launch's epoch, then sums them in fp64. (A dedicated folder block polling from the start
// measured slower: its sc1 polls slowed the workers' streams, 11.6 vs 8.4 us at 512 rows.) The epoch lives in the workspace and the folder advances it
// at the end, so a replayed graph never mistakes the previous launch's granules for this
// launch's. Every spin is bounded: on timeout the loss and the metrics are NaN and
// metrics[6] = 1.
constexpr int kFT = kThreads * 4;  // columns per work unit (one row chunk)
constexpr int kFW = kThreads / kWave;
constexpr int kInlineTotalRows = 1024;  // token_mean total summed by every block up to this n
constexpr int kMaxGranPerThread = 8;    // folder: granule loads per thread per poll (x kNP)
constexpr unsigned kMaxPolls = 1u << 22;

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void store_granule(unsigned long long* g, unsigned epoch, float v) {
    __hip_atomic_store((gu64*)g, ((unsigned long long)epoch << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long load_granule(const unsigned long long* g) {
    return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NW>
__device__ void fold_finalize(double (&tot)[kNP], int any_timeout, int n, const skyrl_ppo_params& p, double* s_redd,
                              float* __restrict__ loss_out, float* __restrict__ metrics);

// Sum the nb blocks' granules (value-major [kNP][nb]) into the loss and the metric vector;
// run by the whole folding block. Thread t owns blocks t, t + kThreads, ... (fixed order).
// NW = waves of the calling block (its threads >= kThreads hold zeros and only join the
// barriers, so the fold order and the result are those of a kThreads block).
template <int NW = kThreads / kWave>
__device__ void fold_granules(const unsigned long long* gran, unsigned epoch, int nb, int n,
                              const skyrl_ppo_params& p, double* s_redd, float* __restrict__ loss_out,
                              float* __restrict__ metrics) {
    double tot[kNP] = {0, 0, 0, 0, 0};  // sum l*m*w, sum m, sum clip*m, sum kl*m*m/mrow, sum ent*m
    bool timed_out = false;
    for (int b0 = threadIdx.x; b0 < nb && !timed_out && threadIdx.x < kThreads; b0 += kThreads * kMaxGranPerThread) {
        float v[kMaxGranPerThread][kNP];
        for (unsigned polls = 0;; ++polls) {
            bool ok = true;
#pragma unroll
            for (int u = 0; u < kMaxGranPerThread; ++u) {
                const int b = b0 + u * kThreads;
                if (b < nb) {
#pragma unroll
                    for (int k = 0; k < kNP; ++k) {
                        const unsigned long long x = load_granule(gran + (int64_t)k * nb + b);
                        v[u][k] = __uint_as_float((unsigned)x);
                        ok = ok && (unsigned)(x >> 32) == epoch;
                    }
                }
            }
            if (ok) break;
            if (polls >= kMaxPolls) {
                timed_out = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int u = 0; u < kMaxGranPerThread; ++u)
            if (b0 + u * kThreads < nb)
#pragma unroll
                for (int k = 0; k < kNP; ++k) tot[k] += (double)v[u][k];
    }
    const int any_timeout = __syncthreads_or(timed_out ? 1 : 0);
    fold_finalize<NW>(tot, any_timeout, n, p, s_redd, loss_out, metrics);
}

__device__ void fold_write(const double (&tot)[kNP], int any_timeout, int n, const skyrl_ppo_params& p,
                           float* __restrict__ loss_out, float* __restrict__ metrics);

// fp64 per-thread totals -> the loss and the metric vector: each wave's DPP tree
// (wave_sum_dpp), the NW wave sums added in wave order by thread 0, which writes. Every fold of
// the loss records (in-launch, deferred finish, no-grad) goes through here, so they agree bit
// for bit. s_redd: NW * kNP doubles.
template <int NW>
__device__ void fold_finalize(double (&tot)[kNP], int any_timeout, int n, const skyrl_ppo_params& p, double* s_redd,
                              float* __restrict__ loss_out, float* __restrict__ metrics) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    double ws[kNP];
#pragma unroll
    for (int k = 0; k < kNP; ++k) ws[k] = wave_sum_dpp(tot[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < kNP; ++k) s_redd[w * kNP + k] = ws[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        double t[kNP];
#pragma unroll
        for (int k = 0; k < kNP; ++k) {
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < NW; ++j) acc += s_redd[j * kNP + k];
            t[k] = acc;
        }
        fold_write(t, any_timeout, n, p, loss_out, metrics);
    }
}

// the folded sums -> loss and metrics (one thread)
__device__ void fold_write(const double (&tot)[kNP], int any_timeout, int n, const skyrl_ppo_params& p,
                           float* __restrict__ loss_out, float* __restrict__ metrics) {
    {
        const double msum = tot[1] > 1.0 ? tot[1] : 1.0;
        float pg = p.loss_reduction == 0 ? (float)(tot[0] / msum) : (float)(tot[0] / (double)n);
        float clip_ratio = (float)(tot[2] / msum);
        float kl = p.use_kl_loss ? (float)(tot[3] / (double)n) : 0.f;
        float entropy = (float)(tot[4] / msum);
        float final_loss = pg + kl * p.kl_loss_coef;
        if (p.use_entropy_loss) final_loss = final_loss - entropy * p.entropy_loss_coef;
        float mask_sum = (float)tot[1];
        if (any_timeout) pg = clip_ratio = kl = entropy = final_loss = mask_sum = __int_as_float(0x7fc00000);
        loss_out[0] = final_loss;
        metrics[SKYRL_M_FINAL_LOSS] = final_loss;
        metrics[SKYRL_M_POLICY_LOSS] = pg;
        metrics[SKYRL_M_ENTROPY] = entropy;
        metrics[SKYRL_M_KL] = kl;
        metrics[SKYRL_M_CLIP_RATIO] = clip_ratio;
        metrics[SKYRL_M_MASK_SUM] = mask_sum;
        metrics[6] = any_timeout ? 1.f : 0.f;  // fold timed out
        metrics[7] = 0.f;
    }
}

// Deferred form: the forward left plain fp32 records (value-major [kNP][nb], nb in the
// workspace header); the kernel boundary has published them, so block 0 of this launch sums
// them in the order fold_granules does (thread t: records t, t + kThreads, ... in fp64) and
// the result is bit-identical to the one-launch fold. The other blocks rescale the gradients
// when the upstream gradient is not 1 (the autograd backward); at 1 they exit at once.
// Records are laid out [kNP][units] (units = n * ceil(R / 1024), the most a forward writes) and
// a forward with nb < units records zeroes the slots [nb, units), so the fold sums every slot:
// no dependent load of nb before the record loads, and the added zeros leave the fp64 sums
// bit-identical to summing the nb records.
__global__ __launch_bounds__(kThreads) void loss_finish_kernel(const float* __restrict__ g,
                                                               const float* __restrict__ parts,
                                                               const int* __restrict__ nb_word, int n, int units,
                                                               skyrl_ppo_params p, float* __restrict__ loss_out,
                                                               float* __restrict__ metrics, float* __restrict__ glp,
                                                               float* __restrict__ gent, int64_t numel, int mode) {
    if (blockIdx.x == 0) {
        __shared__ double s_redd[kFW * kNP];
        if (mode == 2) return;  // timing probe only (the variant field finish_mode = 2): no fold
        double tot[kNP] = {0, 0, 0, 0, 0};
        if (mode == 0) {  // two records per thread in flight per pass (512 units: one pass); clamped
            // indices, no branch around a load (its end would wait for every load before it)
            for (int b = threadIdx.x; b < units; b += 2 * kThreads) {
                const int b2 = b + kThreads < units ? b + kThreads : b;
                float v0[kNP], v1[kNP];
#pragma unroll
                for (int k = 0; k < kNP; ++k) {
                    v0[k] = parts[(int64_t)k * units + b];
                    v1[k] = parts[(int64_t)k * units + b2];
                }
#pragma unroll
                for (int k = 0; k < kNP; ++k) tot[k] += (double)v0[k];
                if (b + kThreads < units)
#pragma unroll
                    for (int k = 0; k < kNP; ++k) tot[k] += (double)v1[k];
            }
        } else {  // nb first, then the records (the variant A/B'd against mode 0)
            const int nb = *nb_word;
            for (int b = threadIdx.x; b < nb; b += kThreads)
#pragma unroll
                for (int k = 0; k < kNP; ++k) tot[k] += (double)parts[(int64_t)k * units + b];
        }
        if (mode == 3) {  // timing probe only: no block reduction (thread 0's own sums)
            if (threadIdx.x == 0) fold_write(tot, 0, n, p, loss_out, metrics);
            return;
        }
        if (mode == 4) {  // timing probe only: block reduction, raw sums written (no divisions)
            block_sum_d<kFW, kNP>(tot, s_redd);
            if (threadIdx.x < kNP) metrics[threadIdx.x] = (float)tot[threadIdx.x];
            return;
        }
        fold_finalize<kFW>(tot, 0, n, p, s_redd, loss_out, metrics);
        return;
    }
    if (!g) return;
    const float sc = g[0];
    if (sc == 1.0f) return;
    const int64_t stride = (int64_t)(gridDim.x - 1) * blockDim.x;
    for (int64_t i = (int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x; i < numel; i += stride) {
        glp[i] *= sc;
        if (gent) gent[i] *= sc;
    }
}

// token_mean total over n <= kInlineTotalRows loss-mask row sums, computed by every wave that
// needs it, identically in ppo_loss_grad_kernel and grpo_loss_grad_kernel (so the two-call and
// the one-launch paths scale their gradients by the same bits): lane l adds the 4-row groups l,
// l + 64, l + 128, l + 192 as (r0 + r1) + (r2 + r3) (rows >= n read as 0), then the wave tree.
// Four 16-B loads per lane when the row sums are 16-B aligned and n % 4 == 0, else 16 scalar
// loads; every address is clamped in bounds, so the loads carry no divergent branch.
struct TotalLoads {
    float4 v[kInlineTotalRows / (4 * kWave)];
};
__device__ __forceinline__ void total_issue(const float* __restrict__ rms, int n, bool vec, TotalLoads& t) {
    const int lane = threadIdx.x & (kWave - 1);
    const int nv = (n + 3) >> 2;
#pragma unroll
    for (int u = 0; u < kInlineTotalRows / (4 * kWave); ++u) {
        const int vi = lane + u * kWave;
        const int vc = vi < nv ? vi : nv - 1;
        if (vec) {
            t.v[u] = reinterpret_cast<const float4*>(rms)[vc];
        } else {
            const int r = 4 * vc;
            t.v[u].x = rms[r < n ? r : n - 1];
            t.v[u].y = rms[r + 1 < n ? r + 1 : n - 1];
            t.v[u].z = rms[r + 2 < n ? r + 2 : n - 1];
            t.v[u].w = rms[r + 3 < n ? r + 3 : n - 1];
        }
    }
}
__device__ __forceinline__ float total_sum(const TotalLoads& t, int n) {
    const int lane = threadIdx.x & (kWave - 1);
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < kInlineTotalRows / (4 * kWave); ++u) {
        const int r = 4 * (lane + u * kWave);
        const float x = r < n ? t.v[u].x : 0.f, y = r + 1 < n ? t.v[u].y : 0.f;
        const float z = r + 2 < n ? t.v[u].z : 0.f, w = r + 3 < n ? t.v[u].w : 0.f;
        acc += (x + y) + (z + w);
    }
    return wave_sum(acc);
}

// Per-row sums of the loss mask (one wave per row), for callers that do not carry them.
__global__ __launch_bounds__(kThreads) void mask_row_sum_kernel(const float* __restrict__ mask, int n, int R,
                                                                float* __restrict__ out) {
    const int row = blockIdx.x * kFW + threadIdx.x / kWave;
    if (row >= n) return;
    const int lane = threadIdx.x & (kWave - 1);
    const float* m = mask + (int64_t)row * R;
    float acc = 0.f;
    for (int t = lane; t < R; t += kWave) acc += m[t];
    acc = wave_sum(acc);
    if (lane == 0) out[row] = acc;
}

// token_mean total: sum of n row sums in fp64 in a fixed order (bit-identical in every block).
__global__ __launch_bounds__(kThreads) void mask_total_kernel(const float* __restrict__ row_msum, int n,
                                                              float* __restrict__ total) {
    __shared__ double s[kFW];
    double t[1] = {0.0};
    for (int r = threadIdx.x; r < n; r += kThreads) t[0] += (double)row_msum[r];
    block_sum_d<kFW, 1>(t, s);
    if (threadIdx.x == 0) total[0] = (float)t[0];
}

// Work unit = one 1024-column chunk of one row; block b takes units [b*U, b*U + U). U = 1 up
// to 2048 units (512 rows: 8.4 us vs 10.1 at U = 2 and 13.6 at U = 4, measured), U = 4 above
// (8192 rows: 63 us vs 80 at U = 1: a quarter of the granules to fold).
template <bool VEC4, int U, bool DEFER>
__global__ __launch_bounds__(kThreads) void ppo_loss_grad_kernel(
    const float* __restrict__ lp, const float* __restrict__ old, const float* __restrict__ adv,
    const float* __restrict__ mask, const float* __restrict__ ref, const float* __restrict__ ent,
    const float* __restrict__ row_msum, const float* __restrict__ msum_total, int n, int R, int nchunks,
    skyrl_ppo_params p, float* __restrict__ glp, float* __restrict__ gent, unsigned long long* __restrict__ gran,
    unsigned* __restrict__ epoch_word, int* __restrict__ nb_word, float* __restrict__ loss_out,
    float* __restrict__ metrics) {
    __shared__ float s_red[kFW * kNP];
    __shared__ double s_redd[DEFER ? 1 : kFW * kNP];
    __shared__ unsigned s_epoch;
    PHASE(0);
    if (!DEFER && threadIdx.x == 0)
        s_epoch = __hip_atomic_load((gu32*)epoch_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const int units = n * nchunks;
    const int nb = gridDim.x;
    const int wb = blockIdx.x;
    const float lo = (float)(1.0 - (double)p.eps_clip_low);
    const float hi = (float)(1.0 + (double)p.eps_clip_high);
    // issue every 16-B load of all U units first (R % 4 == 0 on the VEC4 path)
    // Loads are unconditional from addresses valid for every thread (a dead unit reads element 0
    // and drops it): a load under a divergent branch makes the compiler wait for it, and for
    // every load before it, at the branch's end, which serialised the round trips.
    float4 l4[U], o4[U], a4[U], m4[U], r4[U], e4[U];
    int row_u[U];
    bool live[U];
    float mrow_u[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int unit = wb * U + u;
        row_u[u] = unit < units ? unit / nchunks : 0;
        const int c0 = (unit - row_u[u] * nchunks) * kFT + threadIdx.x * 4;
        live[u] = VEC4 && unit < units && c0 + 3 < R;
        l4[u] = o4[u] = a4[u] = r4[u] = e4[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        m4[u] = make_float4(1.f, 1.f, 1.f, 1.f);
        if (VEC4) {
            const int64_t e = live[u] ? (int64_t)row_u[u] * R + c0 : 0;
            l4[u] = *reinterpret_cast<const float4*>(lp + e);
            o4[u] = *reinterpret_cast<const float4*>(old + e);
            a4[u] = *reinterpret_cast<const float4*>(adv + e);
            if (mask) m4[u] = *reinterpret_cast<const float4*>(mask + e);
            if (p.use_kl_loss) r4[u] = *reinterpret_cast<const float4*>(ref + e);
            if (ent) e4[u] = *reinterpret_cast<const float4*>(ent + e);
        }
        mrow_u[u] = row_msum[row_u[u]];
    }
    // the mask-only scales while the loads are in flight
    const bool need_total = p.loss_reduction == 0 || (p.use_entropy_loss && gent);
    // every wave sums the n row sums itself (same lanes, same order, xor tree: the same value
    // in every wave of every block), so no barrier stands between the loads and the math; the
    // loads are issued together (a dependent per-iteration loop serialised them)
    float total = 0.f;
    if (need_total) {
        if (msum_total) {
            total = msum_total[0];
        } else {  // n <= kInlineTotalRows
            TotalLoads tl;
            total_issue(row_msum, n, (n & 3) == 0 && (reinterpret_cast<uintptr_t>(row_msum) & 15) == 0, tl);
            total = total_sum(tl, n);
        }
    }
    const float tok_scale = 1.f / (total > 1.f ? total : 1.f);  // token_mean
    const float escale = need_total ? -(p.entropy_loss_coef / (total > 1.f ? total : 1.f)) : 0.f;
    PHASE(4);

    float acc[kNP] = {0.f, 0.f, 0.f, 0.f, 0.f};  // sum l*m*w, m, clip*m, kl*m*m/mrow, ent*m
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int unit = wb * U + u;
        if (unit >= units) break;
        const int row = row_u[u];
        const double mr = (double)mrow_u[u];
        // 1 / max(mrow, 1) in fp32: the correctly rounded fp32 quotient equals the fp64 one
        // rounded to fp32 (53 >= 2 * 24 + 2: double rounding is innocuous for division), so the
        // bits are those of (float)(1.0 / mr) without the fp64 division on the critical path
        const float inv_mrow = 1.f / (mrow_u[u] > 1.f ? mrow_u[u] : 1.f);
        float scale, w;  // gradient scale; weight of the row's l*m in the pg sum
        if (p.loss_reduction == 0) { scale = tok_scale; w = 1.f; }
        else if (p.loss_reduction == 1) { scale = (float)(1.0 / ((double)n * (mr > 1.0 ? mr : 1.0))); w = inv_mrow; }
        else { scale = (float)(1.0 / ((double)n * (double)p.max_seq_len)); w = (float)(1.0 / (double)p.max_seq_len); }
        float a[kNP] = {0.f, 0.f, 0.f, 0.f, 0.f};
        auto tok = [&](float L, float O, float A, float M, float RF, float E) -> float {
            const TokenOut t = ppo_token(L, O, A, lo, hi, p.clip_ratio_c, p.dual_clip);
            a[0] += t.loss * M;
            a[1] += M;
            a[2] += t.clip * M;
            const float klm = (approx_kl(L, RF, p.kl_type) * M) * M;
            a[3] += p.use_kl_loss ? klm : 0.f;
            a[4] += E * M;
            return (t.dldlp * M) * scale;
        };
        const int64_t rbase = (int64_t)row * R;
        const int chunk = unit - row * nchunks;
        if (VEC4) {
            if (live[u]) {
                const int64_t e = rbase + chunk * kFT + threadIdx.x * 4;
                float4 g;
                g.x = tok(l4[u].x, o4[u].x, a4[u].x, m4[u].x, r4[u].x, e4[u].x);
                g.y = tok(l4[u].y, o4[u].y, a4[u].y, m4[u].y, r4[u].y, e4[u].y);
                g.z = tok(l4[u].z, o4[u].z, a4[u].z, m4[u].z, r4[u].z, e4[u].z);
                g.w = tok(l4[u].w, o4[u].w, a4[u].w, m4[u].w, r4[u].w, e4[u].w);
                *reinterpret_cast<float4*>(glp + e) = g;
                if (gent) *reinterpret_cast<float4*>(gent + e) =
                    make_float4(escale * m4[u].x, escale * m4[u].y, escale * m4[u].z, escale * m4[u].w);
            }
        } else {
            for (int c = chunk * kFT + threadIdx.x; c < R && c < (chunk + 1) * kFT; c += kThreads) {
                const int64_t e = rbase + c;
                const float M = mask ? mask[e] : 1.f;
                glp[e] = tok(lp[e], old[e], adv[e], M, p.use_kl_loss ? ref[e] : 0.f, ent ? ent[e] : 0.f);
                if (gent) gent[e] = escale * M;
            }
        }
        acc[0] += a[0] * w;
        acc[1] += a[1];
        acc[2] += a[2];
        acc[3] += a[3] * inv_mrow;
        acc[4] += a[4];
    }
    PHASE(1);
    block_sum<kFW, kNP>(acc, s_red);  // (its barrier also publishes s_epoch)
    if constexpr (DEFER) {  // plain records, folded by loss_finish_kernel after the kernel boundary
        float* parts = reinterpret_cast<float*>(gran);  // [kNP][units]: see loss_finish_kernel
        if (threadIdx.x < kNP) {
            parts[(int64_t)threadIdx.x * units + wb] = acc[threadIdx.x];
            for (int z = nb + wb; z < units; z += nb) parts[(int64_t)threadIdx.x * units + z] = 0.f;  // U > 1
        }
        if (wb == 0 && threadIdx.x == 0) *nb_word = nb;
        return;
    }
    const unsigned epoch = s_epoch;
    if (threadIdx.x < kNP) store_granule(gran + (int64_t)threadIdx.x * nb + wb, epoch, acc[threadIdx.x]);
    if (wb != nb - 1) return;
    PHASE(2);
    fold_granules(gran, epoch, nb, n, p, s_redd, loss_out, metrics);
    if (threadIdx.x == 0) __hip_atomic_store((gu32*)epoch_word, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    PHASE(3);
}

// ---- a4 + a7 in ONE launch: GRPO advantage inside the loss launch ----------------------
// For a batch that is one micro-batch (the north_star's advantage+loss leg), the GRPO
// advantage (grpo.hip) and the loss above are two dependent launches joined by a 4 B/token
// advantage round trip. Here every loss block derives its own row's advantage: it sums the
// reward rows of its group (contiguous uniform groups of G <= 16 rows, the trainer's layout,
// generators/utils.py:373-393) with the per-lane order and wave tree of grpo.hip's
// grpo_adv_contig_kernel, so the scores, the fp64 group stats and the fp32 normalisation are
// bit-identical to skyrl_grpo_advantage's; it writes adv*response_mask for its own chunk (the
// product output, kept in the batch like the reference's advantages) and feeds the same
// values to ppo_token. The G*nchunks blocks of a group sit on one XCD (block b runs on XCD
// b % 8), so the group's repeated reward reads (G*R*4 B) hit that XCD's L2.
constexpr int kGroupMax = 16;

// RPB row chunks per block (RPB x 256 threads, one chunk per 256-thread half): the group's
// reward rows are read once per RPB units, each wave sums fewer of them, and every half
// still publishes its own unit's granules (same fp32 partials, same fold as RPB = 1).
// scores (f32 [n], the per-row reward sums skyrl_pack_experience emits, in grpo.hip's summation
// order) replace the group's reward-row reads: the block then loads G floats instead of G*R*4 B.
// DEFER: plain records for loss_finish_kernel instead of the in-launch fold.
template <int MDT, int RPB, bool DEFER>
__global__ __launch_bounds__(kThreads * RPB) void grpo_loss_grad_kernel(
    const float* __restrict__ rewards, const float* __restrict__ scores, const void* __restrict__ resp_mask,
    int num_groups, int G, float epsilon, int norm_by_std, int xcd_map, const float* __restrict__ lp,
    const float* __restrict__ old, const float* __restrict__ mask, const float* __restrict__ ref,
    const float* __restrict__ ent, const float* __restrict__ row_msum, int n, int R, int nchunks, skyrl_ppo_params p,
    float* __restrict__ adv_out, float* __restrict__ glp, float* __restrict__ gent,
    unsigned long long* __restrict__ gran, unsigned* __restrict__ epoch_word, int* __restrict__ nb_word,
    float* __restrict__ loss_out, float* __restrict__ metrics) {
    constexpr int kW = kFW * RPB;  // waves per block
    __shared__ float s_red[kW * kNP];
    __shared__ double s_redd[DEFER ? 1 : kW * kNP];
    __shared__ float s_scores[kGroupMax];  // summed from the reward rows
    __shared__ float s_given[kGroupMax];   // the given scores, written by every wave (see below)
    __shared__ unsigned s_epoch;
    PHASE(0);
    if (!DEFER && threadIdx.x == 0)
        s_epoch = __hip_atomic_load((gu32*)epoch_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const int nb = gridDim.x * RPB;  // granule sets = units
    const int half = threadIdx.x / kThreads;
    const int tid = threadIdx.x % kThreads;
    const int wb = blockIdx.x * RPB + half;  // this half's granule slot
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int gb = G * nchunks / RPB;  // blocks per group
    int group, local;
    if (xcd_map) {
        const int k = blockIdx.x >> 3;
        group = (k / gb) * 8 + (blockIdx.x & 7);
        local = (k % gb) * RPB + half;
    } else {
        group = blockIdx.x / gb;
        local = (blockIdx.x % gb) * RPB + half;
    }
    const bool unit_live = group < num_groups;
    const int row = unit_live ? group * G + local / nchunks : 0;
    const int chunk = local % nchunks;
    const int c0 = chunk * kFT + tid * 4;
    const bool live = unit_live && c0 < R;  // R % 4 == 0 on this path
    // Every load below is unconditional, from an address valid for every thread (dead threads
    // read element 0 and drop it): a load under a divergent branch makes the compiler wait for
    // it (and for every load before it) at the branch's end, which serialised the round trips.
    const int64_t e = live ? (int64_t)row * R + c0 : 0;
    float4 l4 = make_float4(0.f, 0.f, 0.f, 0.f), o4 = l4, r4 = l4, e4 = l4, m4 = make_float4(1.f, 1.f, 1.f, 1.f);
    // response mask NULL (only with adv_out NULL): the row's advantage on every token, exact
    // wherever the loss mask is nonzero when the loss mask is 0 outside the response (pack's layout)
    // The same loads on every path (absent inputs read lp instead and are replaced after the
    // barrier): with a path-dependent number of loads in flight the compiler's wait counts go
    // conservative and wait for nearly everything at the first use.
    Mask4Raw rm_raw;
    const float mrow_in = row_msum[row];  // issued with the loads, not after the barrier
    auto issue_loss_loads = [&]() {
        l4 = *reinterpret_cast<const float4*>(lp + e);
        o4 = *reinterpret_cast<const float4*>(old + e);
        m4 = *reinterpret_cast<const float4*>((mask ? mask : lp) + e);
        r4 = *reinterpret_cast<const float4*>((p.use_kl_loss ? ref : lp) + e);
        e4 = *reinterpret_cast<const float4*>((ent ? ent : lp) + e);
        rm_raw = load_mask4_raw<MDT>(resp_mask ? resp_mask : (const void*)lp, resp_mask ? e : 0);  // converted later
    };
    // token_mean total: this lane's row sums (n <= kInlineTotalRows on this path) issued with
    // the other loads, summed after the barrier in ppo_loss_grad_kernel's order
    const bool need_total = p.loss_reduction == 0 || (p.use_entropy_loss && gent);
    TotalLoads tl;
    const bool tot_vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(row_msum) & 15) == 0;
    auto issue_total_loads = [&]() { total_issue(row_msum, n, tot_vec, tl); };
    // group scores: wave wv sums rows wv, wv + kFW, ... (grpo_adv_contig_kernel's lane order).
    // One load sequence for both sources: the score (scores given; from rewards otherwise, where
    // it is dropped), the total and the loss inputs, then the reward vectors; the reward-first
    // order of r02 measured the same (11.02 vs 11.07 us).
    const int n4 = R >> 2;
    const int g0 = unit_live ? group * G : 0;
    const int si = threadIdx.x & (kGroupMax - 1);
    const float sc = (scores ? scores : rewards)[g0 + (si < G ? si : G - 1)];
    issue_total_loads();
    issue_loss_loads();
    // group stats (grpo.hip, ppo_utils.py:1164-1175): fp64 mean / unbiased std, fp32 normalisation
    auto group_adv = [&](auto score_of) -> float {
        float mean_f, denom_f;
        if (G <= 1) {
            mean_f = 0.f;
            denom_f = norm_by_std ? (1.f + epsilon) : 1.f;
        } else {
            double sum = 0.0;
            for (int j = 0; j < G; ++j) sum += (double)score_of(j);
            const double mean = sum / (double)G;
            double m2 = 0.0;
            for (int j = 0; j < G; ++j) {
                const double d = (double)score_of(j) - mean;
                m2 += d * d;
            }
            mean_f = (float)mean;
            const float std_f = (float)sqrt(m2 / (double)(G - 1));
            denom_f = norm_by_std ? (std_f + epsilon) : 1.f;
        }
        const float s = score_of(row - group * G);
        return norm_by_std ? (s - mean_f) / denom_f : (s - mean_f);
    };
    // given scores: every wave writes all 16 slots of s_given (lane l writes slot l & 15; equal
    // values per slot whichever wave writes), so each wave reads back slots it wrote itself (LDS
    // operations of one wave complete in order): no block barrier, and the advantage is derived
    // while the loss inputs are in flight. Every lane executes the write, so the score load is
    // not sunk into a branch (whose end would wait for every load issued after it).
    s_given[si] = sc;
    __builtin_amdgcn_wave_barrier();
    float adv_row = 0.f;
    if (scores) {
#ifdef SKYRL_PROBE_NOSTATS  // scripts/probe/phase_probe_deferred only: timing, wrong advantages
        const float a = s_given[0];
#else
        const float a = group_adv([&](int j) { return s_given[j]; });
#endif
        if (unit_live) adv_row = a;
    }
    if (!scores && unit_live && n4 <= 4 * kWave) {
        // R <= 1024: every reward vector of the wave's (up to 4) rows in flight at once (clamped
        // addresses, dropped after the loads)
        float4 v[kGroupMax / kW][4];
#pragma unroll
        for (int q = 0; q < kGroupMax / kW; ++q) {
            const int j = wv + q * kW;
            const float4* rrow =
                reinterpret_cast<const float4*>(rewards + (int64_t)(group * G + (j < G ? j : G - 1)) * R);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = lane + u * kWave;
                v[q][u] = rrow[i < n4 ? i : n4 - 1];
                if (!(j < G && i < n4)) v[q][u] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int q = 0; q < kGroupMax / kW; ++q) {
            const int j = wv + q * kW;
            if (j < G) {
                float acc = 0.f;
#pragma unroll
                for (int u = 0; u < 4; ++u) acc += (v[q][u].x + v[q][u].y) + (v[q][u].z + v[q][u].w);
                acc = wave_sum(acc);
                if (lane == 0) s_scores[j] = acc;
            }
        }
    }
    if (!scores && unit_live && n4 > 4 * kWave) {
        for (int j = wv; j < G; j += kW) {
            const float4* rrow = reinterpret_cast<const float4*>(rewards + (int64_t)(group * G + j) * R);
            float acc = 0.f;
            int i = lane;
            for (; i + 3 * kWave < n4; i += 4 * kWave) {
                const float4 v0 = rrow[i], v1 = rrow[i + kWave], v2 = rrow[i + 2 * kWave], v3 = rrow[i + 3 * kWave];
                acc += (v0.x + v0.y) + (v0.z + v0.w);
                acc += (v1.x + v1.y) + (v1.z + v1.w);
                acc += (v2.x + v2.y) + (v2.z + v2.w);
                acc += (v3.x + v3.y) + (v3.z + v3.w);
            }
            for (; i < n4; i += kWave) {
                const float4 v = rrow[i];
                acc += (v.x + v.y) + (v.z + v.w);
            }
            acc = wave_sum(acc);
            if (lane == 0) s_scores[j] = acc;
        }
    }
    if (!scores) __syncthreads();  // (kernel-uniform)
    PHASE(5);
    const float total = need_total ? total_sum(tl, n) : 0.f;
    const float tok_scale = 1.f / (total > 1.f ? total : 1.f);
    const float escale = need_total ? -(p.entropy_loss_coef / (total > 1.f ? total : 1.f)) : 0.f;
    float rm[4] = {1.f, 1.f, 1.f, 1.f};
    if (resp_mask) mask4_to_float<MDT>(rm_raw, rm);
    if (!mask) m4 = make_float4(1.f, 1.f, 1.f, 1.f);
    if (!p.use_kl_loss) r4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!ent) e4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!scores && unit_live) adv_row = group_adv([&](int j) { return s_scores[j]; });
    const float4 a4 = make_float4(adv_row * rm[0], adv_row * rm[1], adv_row * rm[2], adv_row * rm[3]);
    const float lo = (float)(1.0 - (double)p.eps_clip_low);
    const float hi = (float)(1.0 + (double)p.eps_clip_high);
    float acc[kNP] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (live) {
        if (adv_out) *reinterpret_cast<float4*>(adv_out + e) = a4;
        const double mr = (double)mrow_in;
        const float inv_mrow = 1.f / (mrow_in > 1.f ? mrow_in : 1.f);  // = (float)(1.0 / mr), see above
        float scale, w;
        if (p.loss_reduction == 0) { scale = tok_scale; w = 1.f; }
        else if (p.loss_reduction == 1) { scale = (float)(1.0 / ((double)n * (mr > 1.0 ? mr : 1.0))); w = inv_mrow; }
        else { scale = (float)(1.0 / ((double)n * (double)p.max_seq_len)); w = (float)(1.0 / (double)p.max_seq_len); }
        float a[kNP] = {0.f, 0.f, 0.f, 0.f, 0.f};
        auto tok = [&](float L, float O, float A, float M, float RF, float E) -> float {
#ifdef SKYRL_PROBE_NOMATH  // scripts/probe/phase_probe_deferred only: timing, wrong values
            a[0] += L * M;
            a[1] += M;
            a[3] += RF * M;
            return (O + A) * scale;
#else
            const TokenOut t = ppo_token(L, O, A, lo, hi, p.clip_ratio_c, p.dual_clip);
            a[0] += t.loss * M;
            a[1] += M;
            a[2] += t.clip * M;
            const float klm = (approx_kl(L, RF, p.kl_type) * M) * M;
            a[3] += p.use_kl_loss ? klm : 0.f;
            a[4] += E * M;
            return (t.dldlp * M) * scale;
#endif
        };
        float4 g;
        g.x = tok(l4.x, o4.x, a4.x, m4.x, r4.x, e4.x);
        g.y = tok(l4.y, o4.y, a4.y, m4.y, r4.y, e4.y);
        g.z = tok(l4.z, o4.z, a4.z, m4.z, r4.z, e4.z);
        g.w = tok(l4.w, o4.w, a4.w, m4.w, r4.w, e4.w);
        *reinterpret_cast<float4*>(glp + e) = g;
        if (gent) *reinterpret_cast<float4*>(gent + e) = make_float4(escale * m4.x, escale * m4.y, escale * m4.z, escale * m4.w);
        acc[0] = a[0] * w;
        acc[1] = a[1];
        acc[2] = a[2];
        acc[3] = a[3] * inv_mrow;
        acc[4] = a[4];
    }
    PHASE(1);
    // per-half reduction: block_sum<kFW>'s wave tree and order over the half's own waves
#pragma unroll
    for (int k = 0; k < kNP; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < kNP; ++k) s_red[wv * kNP + k] = acc[k];
    __syncthreads();
    const unsigned epoch = s_epoch;
    if (tid < kNP) {
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < kFW; ++j) sum += s_red[(half * kFW + j) * kNP + tid];
        if constexpr (DEFER) reinterpret_cast<float*>(gran)[(int64_t)tid * nb + wb] = sum;  // nb == units here
        else store_granule(gran + (int64_t)tid * nb + wb, epoch, sum);
    }
    if constexpr (DEFER) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *nb_word = nb;
        PHASE(6);
        return;
    }
    if (blockIdx.x != gridDim.x - 1) return;
    PHASE(2);
    fold_granules<kW>(gran, epoch, nb, n, p, s_redd, loss_out, metrics);
    if (threadIdx.x == 0) __hip_atomic_store((gu32*)epoch_word, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    PHASE(3);
}

// In-place x *= g[0] (the autograd backward of the fused loss); nothing is touched when g == 1.
__global__ void rescale_kernel(const float* __restrict__ g, float* __restrict__ x, float* __restrict__ y, int64_t n) {
    const float s = g[0];
    if (s == 1.0f) return;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        x[i] *= s;
        if (y) y[i] *= s;
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

__global__ void fill_kernel(float* __restrict__ x, int n, float v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = v;
}

inline bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % 16) == 0; }

}  // namespace
}  // namespace skyrl

using namespace skyrl;

// Loss variants (skyrl_variant, per call): loss_units (row chunks per loss block, 0 auto), grpo_loss_rpb
// (row chunks per fused GRPO+loss block; 2 measured slower: 12.1 vs 11.0 us), loss_bwd_blocks (grid cap
// of the backward rescale), finish_mode (0 block tree, 1 nb first; timing probes with wrong values: 2 no
// fold, 3 no block reduction, 4 no divisions; a one-wave fold standing for the 256 threads (no LDS /
// barrier) measured slower: 4.02 vs 3.05 us, profiles/r03_adv_leg_finish_one_wave.log).

extern "C" size_t skyrl_ppo_loss_workspace_bytes(int32_t n, int32_t R) {
    const size_t nchunks = (size_t)((R + kFT - 1) / kFT);
    const size_t nn = (size_t)(n > 0 ? n : 1);
    const size_t parts = nn * (nchunks ? nchunks : 1) * kNP * sizeof(unsigned long long);
    const size_t rows = ((nn * sizeof(float) + 255) / 256) * 256;
    // [epoch | total | pad][granules][row mask sums]
    return 256 + ((parts + 255) / 256) * 256 + rows;
}

// workspace header: [0] epoch word (in-launch fold), [64] token_mean total, [128] record count nb
// (deferred fold), then the records from byte 256
static int* nb_word_of(void* workspace) { return reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + 128); }

extern "C" int skyrl_ppo_loss_fwd(const float* log_probs, const float* old_log_probs, const float* advantages,
                                  const float* loss_mask, const float* ref_log_probs, const float* entropy,
                                  const float* row_mask_sum, int32_t n, int32_t R, const skyrl_ppo_params* params,
                                  float* loss_out, float* metrics_out, float* grad_logp, float* grad_entropy,
                                  int32_t flags, void* workspace, void* stream) {
    SKYRL_REQUIRE(params, "ppo_loss_fwd: params is null");
    SKYRL_REQUIRE(n > 0 && R > 0, "ppo_loss_fwd: empty batch");
    SKYRL_REQUIRE(log_probs && old_log_probs && advantages && loss_out && metrics_out && grad_logp && workspace,
                  "ppo_loss_fwd: null pointer");
    SKYRL_REQUIRE(!params->use_kl_loss || ref_log_probs, "ppo_loss_fwd: use_kl_loss needs ref_log_probs");
    SKYRL_REQUIRE(params->loss_reduction >= 0 && params->loss_reduction <= 2, "ppo_loss_fwd: bad loss_reduction");
    SKYRL_REQUIRE(params->loss_reduction != 2 || params->max_seq_len > 0.f,
                  "ppo_loss_fwd: seq_mean_token_sum_norm needs max_seq_len");
    SKYRL_REQUIRE(params->kl_type >= 0 && params->kl_type <= 3, "ppo_loss_fwd: bad kl_type");
    SKYRL_REQUIRE(!grad_entropy || params->use_entropy_loss, "ppo_loss_fwd: grad_entropy needs use_entropy_loss");
    SKYRL_REQUIRE((flags & ~SKYRL_LOSS_DEFER_FOLD) == 0, "ppo_loss_fwd: unknown flags");
    const bool defer = (flags & SKYRL_LOSS_DEFER_FOLD) != 0;
    const int nchunks = (R + kFT - 1) / kFT;
    char* w = reinterpret_cast<char*>(workspace);
    unsigned* epoch_word = reinterpret_cast<unsigned*>(w);
    float* total = reinterpret_cast<float*>(w + 64);
    unsigned long long* gran = reinterpret_cast<unsigned long long*>(w + 256);
    const size_t parts = (size_t)n * nchunks * kNP * sizeof(unsigned long long);
    float* rows_ws = reinterpret_cast<float*>(w + 256 + ((parts + 255) / 256) * 256);
    hipStream_t s = as_stream(stream);
    const float* rows = row_mask_sum;
    if (!rows) {  // the caller does not carry the loss-mask row sums: one extra launch
        if (loss_mask) {
            hipLaunchKernelGGL(mask_row_sum_kernel, dim3((n + kFW - 1) / kFW), dim3(kThreads), 0, s, loss_mask, n, R,
                               rows_ws);
            int rc = check_launch("mask_row_sum_kernel");
            if (rc) return rc;
        } else {
            hipLaunchKernelGGL(fill_kernel, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, rows_ws, n,
                               (float)R);
            int rc = check_launch("fill_kernel");
            if (rc) return rc;
        }
        rows = rows_ws;
    }
    const bool need_total = params->loss_reduction == 0 || (params->use_entropy_loss && grad_entropy);
    const float* tot = nullptr;
    if (need_total && n > kInlineTotalRows) {
        hipLaunchKernelGGL(mask_total_kernel, dim3(1), dim3(kThreads), 0, s, rows, n, total);
        int rc = check_launch("mask_total_kernel");
        if (rc) return rc;
        tot = total;
    }
    const bool vec4 = (R % 4) == 0 && aligned16(log_probs) && aligned16(old_log_probs) && aligned16(advantages) &&
                      aligned16(loss_mask) && aligned16(ref_log_probs) && aligned16(entropy) && aligned16(grad_logp) &&
                      aligned16(grad_entropy);
    const int units = n * nchunks;
    int U = knobs().loss_units > 0 ? knobs().loss_units : (units > 2048 ? 4 : 1);
    if (!vec4) U = 1;
    const int nb = (units + U - 1) / U;
    auto pick = [&](auto kd, auto kf) { return defer ? kd : kf; };
    auto k = !vec4    ? pick(ppo_loss_grad_kernel<false, 1, true>, ppo_loss_grad_kernel<false, 1, false>)
             : U == 1 ? pick(ppo_loss_grad_kernel<true, 1, true>, ppo_loss_grad_kernel<true, 1, false>)
             : U == 2 ? pick(ppo_loss_grad_kernel<true, 2, true>, ppo_loss_grad_kernel<true, 2, false>)
                      : pick(ppo_loss_grad_kernel<true, 4, true>, ppo_loss_grad_kernel<true, 4, false>);
    hipLaunchKernelGGL(k, dim3(nb), dim3(kThreads), 0, s, log_probs, old_log_probs, advantages, loss_mask, ref_log_probs,
                       entropy, rows, tot, n, R, nchunks, *params, grad_logp, grad_entropy, gran, epoch_word,
                       nb_word_of(workspace), loss_out, metrics_out);
    return check_launch("ppo_loss_grad_kernel");
}

extern "C" int skyrl_grpo_ppo_loss_fwd(const float* rewards, const float* scores, const void* response_mask,
                                       int mask_dtype, int32_t num_groups, float epsilon, int32_t norm_by_std,
                                       const float* log_probs, const float* old_log_probs, const float* loss_mask,
                                       const float* ref_log_probs, const float* entropy, const float* row_mask_sum,
                                       int32_t n, int32_t R, const skyrl_ppo_params* params, float* advantages,
                                       float* loss_out, float* metrics_out, float* grad_logp, float* grad_entropy,
                                       int32_t flags, void* workspace, void* stream) {
    SKYRL_REQUIRE(params, "grpo_ppo_loss_fwd: params is null");
    SKYRL_REQUIRE(n > 0 && R > 0 && num_groups > 0, "grpo_ppo_loss_fwd: empty batch");
    SKYRL_REQUIRE(n % num_groups == 0, "grpo_ppo_loss_fwd: contiguous groups need n % num_groups == 0");
    SKYRL_REQUIRE((rewards || scores) && (response_mask || !advantages) && log_probs && old_log_probs && loss_out &&
                      metrics_out && grad_logp && workspace,
                  "grpo_ppo_loss_fwd: null pointer");
    SKYRL_REQUIRE((flags & ~SKYRL_LOSS_DEFER_FOLD) == 0, "grpo_ppo_loss_fwd: unknown flags");
    const bool defer = (flags & SKYRL_LOSS_DEFER_FOLD) != 0;
    SKYRL_REQUIRE(mask_dtype == SKYRL_F32 || mask_dtype == SKYRL_I64 || mask_dtype == SKYRL_I32 ||
                      mask_dtype == SKYRL_U8,
                  "grpo_ppo_loss_fwd: unsupported mask dtype");
    const int G = n / num_groups;
    const int nchunks = (R + kFT - 1) / kFT;
    const int units = n * nchunks;
    const bool need_total = params->loss_reduction == 0 || (params->use_entropy_loss && grad_entropy);
    const bool one_launch = row_mask_sum && G <= kGroupMax && (R % 4) == 0 && units <= 2048 &&
                            !(need_total && n > kInlineTotalRows) && aligned16(rewards) && aligned16(scores) &&
                            aligned16(response_mask) &&
                            aligned16(log_probs) && aligned16(old_log_probs) && aligned16(loss_mask) &&
                            aligned16(ref_log_probs) && aligned16(entropy) && aligned16(advantages) &&
                            aligned16(grad_logp) && aligned16(grad_entropy);
    if (!one_launch) {  // larger batches (the fold would dominate) or other layouts: the two launches
        SKYRL_REQUIRE(advantages && response_mask,
                      "grpo_ppo_loss_fwd: this layout runs two launches and needs advantages and response_mask");
        int rc = skyrl_grpo_advantage(rewards, scores, response_mask, mask_dtype, nullptr, nullptr, num_groups, n, R,
                                      epsilon, norm_by_std, advantages, nullptr, stream);
        if (rc) return rc;
        return skyrl_ppo_loss_fwd(log_probs, old_log_probs, advantages, loss_mask, ref_log_probs, entropy,
                                  row_mask_sum, n, R, params, loss_out, metrics_out, grad_logp, grad_entropy, flags,
                                  workspace, stream);
    }
    SKYRL_REQUIRE(!params->use_kl_loss || ref_log_probs, "grpo_ppo_loss_fwd: use_kl_loss needs ref_log_probs");
    SKYRL_REQUIRE(params->loss_reduction >= 0 && params->loss_reduction <= 2, "grpo_ppo_loss_fwd: bad loss_reduction");
    SKYRL_REQUIRE(params->loss_reduction != 2 || params->max_seq_len > 0.f,
                  "grpo_ppo_loss_fwd: seq_mean_token_sum_norm needs max_seq_len");
    SKYRL_REQUIRE(params->kl_type >= 0 && params->kl_type <= 3, "grpo_ppo_loss_fwd: bad kl_type");
    SKYRL_REQUIRE(!grad_entropy || params->use_entropy_loss, "grpo_ppo_loss_fwd: grad_entropy needs use_entropy_loss");
    char* w = reinterpret_cast<char*>(workspace);
    unsigned* epoch_word = reinterpret_cast<unsigned*>(w);
    unsigned long long* gran = reinterpret_cast<unsigned long long*>(w + 256);
    const int xcd_map = (num_groups % 8) == 0 ? 1 : 0;  // grid stays n * nchunks blocks either way
    const int rpb = (knobs().grpo_loss_rpb == 2 && (G * nchunks) % 2 == 0) ? 2 : 1;
    using KT = decltype(&grpo_loss_grad_kernel<SKYRL_I64, 1, false>);
    KT k = nullptr;
#define SKYRL_GL_PICK(MDT)                                                                              \
    k = defer ? (rpb == 2 ? grpo_loss_grad_kernel<MDT, 2, true> : grpo_loss_grad_kernel<MDT, 1, true>) \
              : (rpb == 2 ? grpo_loss_grad_kernel<MDT, 2, false> : grpo_loss_grad_kernel<MDT, 1, false>)
    if (mask_dtype == SKYRL_I64) SKYRL_GL_PICK(SKYRL_I64);
    else if (mask_dtype == SKYRL_F32) SKYRL_GL_PICK(SKYRL_F32);
    else if (mask_dtype == SKYRL_I32) SKYRL_GL_PICK(SKYRL_I32);
    else SKYRL_GL_PICK(SKYRL_U8);
#undef SKYRL_GL_PICK
    hipLaunchKernelGGL(k, dim3(units / rpb), dim3(kThreads * rpb), 0, as_stream(stream), rewards, scores, response_mask,
                       num_groups, G, epsilon, norm_by_std, xcd_map, log_probs, old_log_probs, loss_mask, ref_log_probs,
                       entropy, row_mask_sum, n, R, nchunks, *params, advantages, grad_logp, grad_entropy, gran,
                       epoch_word, nb_word_of(workspace), loss_out, metrics_out);
    return check_launch("grpo_loss_grad_kernel");
}

extern "C" int skyrl_ppo_loss_finish(const float* grad_out, float* grad_logp, float* grad_entropy, int32_t n,
                                     int32_t R, const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                                     void* workspace, void* stream) {
    SKYRL_REQUIRE(params && loss_out && metrics_out && workspace, "ppo_loss_finish: null pointer");
    SKYRL_REQUIRE(n > 0 && R > 0, "ppo_loss_finish: bad sizes");
    SKYRL_REQUIRE(!grad_out || grad_logp, "ppo_loss_finish: grad_out needs grad_logp");
    const int64_t numel = (int64_t)n * R;
    const int units = n * ((R + kFT - 1) / kFT);
    int64_t blocks = grad_out ? (numel + kThreads - 1) / kThreads : 0;
    if (blocks > knobs().loss_bwd_blocks) blocks = knobs().loss_bwd_blocks;
    const float* parts = reinterpret_cast<const float*>(reinterpret_cast<char*>(workspace) + 256);
    hipLaunchKernelGGL(loss_finish_kernel, dim3((unsigned)(1 + blocks)), dim3(kThreads), 0, as_stream(stream), grad_out,
                       parts, nb_word_of(workspace), n, units, *params, loss_out, metrics_out, grad_logp, grad_entropy,
                       numel, knobs().finish_mode);
    return check_launch("loss_finish_kernel");
}

extern "C" int skyrl_ppo_loss_bwd(const float* grad_out, int64_t numel, float* grad_logp, float* grad_entropy,
                                  void* stream) {
    SKYRL_REQUIRE(grad_out && grad_logp, "ppo_loss_bwd: null pointer");
    SKYRL_REQUIRE(numel >= 0, "ppo_loss_bwd: negative size");
    if (numel == 0) return SKYRL_OK;
    // a small grid: at unit upstream gradient (the common case) the launch only dispatches
    int64_t blocks = (numel + kThreads - 1) / kThreads;
    if (blocks > knobs().loss_bwd_blocks) blocks = knobs().loss_bwd_blocks;
    hipLaunchKernelGGL(rescale_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, as_stream(stream), grad_out,
                       grad_logp, grad_entropy, numel);
    return check_launch("rescale_kernel");
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
