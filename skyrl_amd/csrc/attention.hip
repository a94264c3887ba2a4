// §8(f)2: rollout decode loop kernels — rotary embedding fused with the paged KV-cache
// write, and single-token (decode) attention over the paged cache with MFMA.
//
// Replaces the attention inside vLLM's decode step that the reference drives through
// VLLMInferenceEngine.generate (skyrl_train/inference_engines/vllm/vllm_engine.py:196-218);
// model semantics follow HF Qwen2/Llama (apply_rotary_pos_emb with rotate_half, GQA with
// num_key_value_heads, softmax(q.k / sqrt(D)) v).
//
// Cache layout (one layer; the host keeps one pair per layer):
//   K: bf16 [num_blocks, nkv, 16, D]   — a (block, head) tile is 16 token rows of D
//   V: bf16 [num_blocks, nkv, D, 16]   — transposed: 16 tokens contiguous per dim
// A slot is block * 16 + offset. The V transpose makes both MFMA operands of the P.V
// product 8-byte loads (below).
//
// Decode attention: one wave per (partition of <= part_tokens context tokens, kv head,
// sequence). Per 16-token block the wave computes S^T[token x head] = K[16 x D] . Q^T[D x 16]
// with D/32 mfma_f32_16x16x32_bf16 (the <= 16 query heads of the kv head's GQA group are the
// 16 MFMA columns; unused columns are zero), so every lane holds 4 tokens of ONE head: the
// online-softmax statistics are per lane, the block max is 2 xor-shuffles, and the exp'd
// scores are already the B operand of O^T[d x head] += V^T[d x 16] . P^T[16 x head]
// (D/16 mfma_f32_16x16x16_bf16, no lane movement, no LDS). K and V stream straight from
// HBM into VGPRs (guide: decode attention, M <= 16 rows per kv head). Partitions are
// merged by a small reduce kernel when a sequence spans more than one.
#include "common.h"
#include "variant.h"

namespace skyrl {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBS = 16;  // tokens per KV-cache block

// Per-sequence split of a context of ctx tokens over at most nparts waves, each partition at
// least part_min tokens (a multiple of 16): part = max(part_min, ceil16(ceil(ctx / nparts))).
// Both the attention and the merge kernel derive it from the device-resident context length,
// so one launch shape (fixed nparts, e.g. a captured graph) adapts to every context.
__device__ __forceinline__ void seq_split(int ctx, int part_min, int nparts, int& part, int& np) {
    int p = (ctx + nparts - 1) / nparts;
    p = (p + kBS - 1) / kBS * kBS;
    part = p > part_min ? p : part_min;
    np = (ctx + part - 1) / part;
}

// ---- rotary embedding + KV-cache write ----------------------------------------------
// grid (T, nh + 2*nkv), one wave per (token, head). Heads [0, nh) are query heads (rotated
// into q_out), [nh, nh+nkv) key heads (rotated into the K cache at the token's slot, and
// into k_out if given), [nh+nkv, nh+2nkv) value heads (copied into the V cache). qkv is the
// fused projection output [T, (nh+2nkv)*D] with row stride qkv_stride (elements).
// cos_sin: f32 [max_pos, D]: cos in [0, D/2), sin in [D/2, D) (HF's duplicated halves
// collapse to one copy). Rotation in f32, one rounding to bf16.
template <int D>
__global__ __launch_bounds__(64) void rope_kv_write_kernel(
    const uint16_t* __restrict__ qkv, int64_t qkv_stride, const int64_t* __restrict__ positions,
    const int64_t* __restrict__ slots, const float* __restrict__ cos_sin, int nh, int nkv,
    uint16_t* __restrict__ q_out, uint16_t* __restrict__ k_out, uint16_t* __restrict__ kc,
    uint16_t* __restrict__ vc) {
    const int t = blockIdx.x;
    const int hh = blockIdx.y;
    const int lane = threadIdx.x;
    const uint16_t* src = qkv + (int64_t)t * qkv_stride + (int64_t)hh * D;
    constexpr int H2 = D / 2;
    if (hh >= nh + nkv) {  // value head: copy into the transposed V tile
        const int64_t slot = slots[t];
        if (slot < 0) return;
        const int kvh = hh - nh - nkv;
        const int64_t blk = slot / kBS;
        const int off = (int)(slot % kBS);
        uint16_t* dst = vc + ((blk * nkv + kvh) * D) * kBS + off;
        for (int d = lane; d < D; d += kWave) dst[(int64_t)d * kBS] = src[d];
        return;
    }
    const int64_t pos = positions[t];
    const float* cs = cos_sin + pos * D;
    for (int i = lane; i < H2; i += kWave) {
        const float x1 = bf16_to_f32(src[i]);
        const float x2 = bf16_to_f32(src[i + H2]);
        const float c = cs[i], s = cs[H2 + i];
        const uint16_t y1 = f32_to_bf16(x1 * c - x2 * s);
        const uint16_t y2 = f32_to_bf16(x2 * c + x1 * s);
        if (hh < nh) {
            uint16_t* dq = q_out + ((int64_t)t * nh + hh) * D;
            dq[i] = y1;
            dq[i + H2] = y2;
        } else {
            const int kvh = hh - nh;
            if (k_out) {
                uint16_t* dk = k_out + ((int64_t)t * nkv + kvh) * D;
                dk[i] = y1;
                dk[i + H2] = y2;
            }
            const int64_t slot = slots[t];
            if (slot >= 0) {
                const int64_t blk = slot / kBS;
                const int off = (int)(slot % kBS);
                uint16_t* dk = kc + ((blk * nkv + kvh) * kBS + off) * D;
                dk[i] = y1;
                dk[i + H2] = y2;
            }
        }
    }
}

// Per-wave timestamps for scripts/probe/attn_phase_probe (compiled only there, never in the product).
#ifdef SKYRL_ATTN_PHASE_PROBE
__device__ uint64_t g_aphase[8192 * 8];
#define APHASE(k, extra)                                                                                    \
    do {                                                                                                    \
        const unsigned wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                \
        if (threadIdx.x == 0 && wg_ < 8192) {                                                               \
            g_aphase[wg_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                                     \
            if ((k) == 0) g_aphase[wg_ * 8 + 7] = (uint64_t)__smid() | ((uint64_t)__builtin_amdgcn_s_getreg(20 | (3 << 11)) << 32); \
            if ((k) == 0) g_aphase[wg_ * 8 + 6] = (uint64_t)(extra);                                        \
        }                                                                                                   \
    } while (0)
#else
#define APHASE(k, extra) \
    do {                 \
    } while (0)
#endif

// ---- decode attention over the paged cache -------------------------------------------
// Attention of one kv head's query group over context tokens [t0, t1) of one sequence, one
// wave: o[n][i] = unnormalised O^T[dim 16n + 4g + i][head c], m / l this lane's running max
// and its share of the row sum (log2 domain). PF blocks in flight (see the ring below).
template <int D, int PF>
__device__ __forceinline__ void attend_range(const uint16_t* __restrict__ q, int64_t q_stride,
                                             const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
                                             const int32_t* __restrict__ bt_row, int seq, int kvh, int t0, int t1,
                                             int nkv, int qpk, float scale_log2, f32x4 (&o)[D / 16], float& m,
                                             float& l) {
    constexpr int KS = D / 32;  // k-steps of the Q.K^T MFMA
    constexpr int NT = D / 16;  // 16-dim output tiles of the P.V MFMA
    const int lane = threadIdx.x;
    const int c = lane & 15;  // MFMA column: query head within the GQA group / token row of K
    const int g = lane >> 4;  // lane group: k-slice of the operands, 4-row slice of the result
    const int h = kvh * qpk + c;
    const bool hv = c < qpk;

    s16x8 qf[KS];
    const uint16_t* qrow = q + (int64_t)seq * q_stride + (int64_t)(hv ? h : 0) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        qf[s] = *reinterpret_cast<const s16x8*>(qrow + 32 * s + 8 * g);
        if (!hv) qf[s] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    m = -INFINITY;
    l = 0.f;

    // Block ids of this partition: one vector load of up to 64 table entries (one per lane),
    // read back with readlane, so the per-block address chain has no dependent table load.
    const int32_t* bt = bt_row + t0 / kBS;
    const int nb = (t1 - t0 + kBS - 1) / kBS;
    int tbl = lane < nb ? bt[lane] : 0;
    const int64_t head_tile = (int64_t)kBS * D;
    const int64_t blk_stride = (int64_t)nkv * head_tile;
    const uint16_t* kbase = kc + kvh * head_tile + c * D + 8 * g;
    const uint16_t* vbase = vc + kvh * head_tile + c * kBS + 4 * g;
    auto load_blk = [&](int jb, s16x8 (&kd)[KS], s16x4 (&vd)[NT]) {
        const int64_t blk = __builtin_amdgcn_readlane(tbl, jb & 63);
#pragma unroll
        for (int s = 0; s < KS; ++s) kd[s] = *reinterpret_cast<const s16x8*>(kbase + blk * blk_stride + 32 * s);
#pragma unroll
        for (int n = 0; n < NT; ++n) vd[n] = *reinterpret_cast<const s16x4*>(vbase + blk * blk_stride + 16 * n * kBS);
    };
    // One block step: S^T = K.Q^T, online softmax, O^T += V^T.P^T.
    auto step = [&](int j, const s16x8 (&kf)[KS], s16x4 (&vf)[NT]) {
        const int tb = t0 + j * kBS;
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[s], qf[s], sacc, 0, 0, 0);
        if (j == 0) APHASE(1, 0);  // first block's K has arrived
        // sacc[i] = S[token tb + 4g + i][head c]; tokens past the partition end are masked
        // (their K/V slots hold stale data: select, never multiply).
        const int nv = t1 - (tb + 4 * g);  // valid tokens among this lane's 4
        float sv[4];
        float bm = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            sv[i] = (i < nv) ? sacc[i] * scale_log2 : -INFINITY;
            bm = fmaxf(bm, sv[i]);
        }
        bm = fmaxf(bm, __shfl_xor(bm, 16, kWave));
        bm = fmaxf(bm, __shfl_xor(bm, 32, kWave));
        const float mn = fmaxf(m, bm);
        const float alpha = fast_exp2(m - mn);  // m = -inf on the first block: 0
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = fast_exp2(sv[i] - mn);
        l = l * alpha + ((p[0] + p[1]) + (p[2] + p[3]));
        m = mn;
        if (nv < 4) {  // zero the V columns of masked tokens: stale V times p = 0 must not be NaN
#pragma unroll
            for (int n = 0; n < NT; ++n) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i >= nv) vf[n][i] = 0;
            }
        }
        s16x4 pf;
        const uint32_t p01 = pack_bf16x2(p[0], p[1]);
        const uint32_t p23 = pack_bf16x2(p[2], p[3]);
        pf[0] = (short)(p01 & 0xffff);
        pf[1] = (short)(p01 >> 16);
        pf[2] = (short)(p23 & 0xffff);
        pf[3] = (short)(p23 >> 16);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            o[n] = o[n] * alpha;
            o[n] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf[n], pf, o[n], 0, 0, 0);
        }
    };
    // PF blocks in flight per wave (the current one + PF - 1 prefetched) in a register ring;
    // the loop is unrolled by PF so every ring slot is a static register set (no moves). A
    // wave is bound by its loads' latency (bytes in flight / latency), so the depth sets the
    // per-wave stream rate; the launch's ~1024 waves fit one per SIMD, where the extra
    // registers cost no occupancy.
    s16x8 kb[PF][KS];
    s16x4 vb[PF][NT];
#pragma unroll
    for (int i = 0; i < PF - 1; ++i)
        if (i < nb) load_blk(i, kb[i], vb[i]);
    for (int j0 = 0; j0 < nb; j0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int j = j0 + u;
            if (j < nb) {
                const int jn = j + PF - 1;
                if (jn < nb) {
                    if ((jn & 63) == 0) tbl = (jn + lane < nb) ? bt[jn + lane] : 0;
                    load_blk(jn, kb[(u + PF - 1) % PF], vb[(u + PF - 1) % PF]);
                }
                step(j, kb[u], vb[u]);
            }
        }
    }
}

template <int D, int PF, int MINW>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MINW, 8))) void paged_decode_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int32_t* __restrict__ block_tables, int64_t bt_stride,
    const int32_t* __restrict__ ctx_lens, int nh, int nkv, int qpk, float scale_log2, int part_min,
    int nparts, uint16_t* __restrict__ out, int64_t out_stride, float* __restrict__ ws_o,
    float* __restrict__ ws_ml) {
    constexpr int NT = D / 16;  // 16-dim output tiles of the P.V MFMA
    const int seq = blockIdx.z;
    const int kvh = blockIdx.y;
    const int part = blockIdx.x;
    const int ctx = ctx_lens[seq];
    int part_tokens, np;
    seq_split(ctx, part_min, nparts, part_tokens, np);
    if (part >= np) return;
    const int t0 = part * part_tokens;
    const int t1 = min(ctx, t0 + part_tokens);
    APHASE(0, t1 - t0);
    const int lane = threadIdx.x;
    const int c = lane & 15;
    const int g = lane >> 4;
    const int h = kvh * qpk + c;
    const bool hv = c < qpk;
    f32x4 o[NT];
    float m, l;
    attend_range<D, PF>(q, q_stride, kc, vc, block_tables + (int64_t)seq * bt_stride, seq, kvh, t0, t1, nkv, qpk,
                        scale_log2, o, m, l);
    APHASE(2, 0);
    // o[n][i] = O^T[dim 16n + 4g + i][head c]; l is this lane's share of the row sum
    l += __shfl_xor(l, 16, kWave);
    l += __shfl_xor(l, 32, kWave);
    if (!hv) return;
    if (np == 1) {  // the whole context in this wave: final output, the merge skips this sequence
        const float inv = 1.f / l;
        uint16_t* orow = out + (int64_t)seq * out_stride + (int64_t)h * D;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            uint2 w;
            w.x = pack_bf16x2(o[n][0] * inv, o[n][1] * inv);
            w.y = pack_bf16x2(o[n][2] * inv, o[n][3] * inv);
            *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g) = w;
        }
    } else {
        const int64_t rec = ((int64_t)seq * nh + h) * nparts + part;
        float* wo = ws_o + rec * D;
#pragma unroll
        for (int n = 0; n < NT; ++n) *reinterpret_cast<f32x4*>(wo + 16 * n + 4 * g) = o[n];
        if (g == 0) {
            ws_ml[rec * 2 + 0] = m;
            ws_ml[rec * 2 + 1] = l;
        }
    }
}

// Merge the partitions of one (sequence, head): grid (nh, nseq), D threads.
template <int D>
__global__ __launch_bounds__(D) void paged_decode_reduce_kernel(const float* __restrict__ ws_o,
                                                                const float* __restrict__ ws_ml,
                                                                const int32_t* __restrict__ ctx_lens, int nh,
                                                                int part_min, int nparts,
                                                                uint16_t* __restrict__ out, int64_t out_stride) {
    const int h = blockIdx.x;
    const int seq = blockIdx.y;
    const int d = threadIdx.x;
    const int ctx = ctx_lens[seq];
    int part_tokens, np;
    seq_split(ctx, part_min, nparts, part_tokens, np);
    if (np == 1) return;  // written directly by the attention kernel
    const int64_t rec0 = ((int64_t)seq * nh + h) * nparts;
    float M = -INFINITY;
    for (int p = 0; p < np; ++p) M = fmaxf(M, ws_ml[(rec0 + p) * 2]);
    float L = 0.f, acc = 0.f;
    for (int p = 0; p < np; ++p) {
        const float w = fast_exp2(ws_ml[(rec0 + p) * 2] - M);
        L += w * ws_ml[(rec0 + p) * 2 + 1];
        acc += w * ws_o[(rec0 + p) * D + d];
    }
    out[(int64_t)seq * out_stride + (int64_t)h * D + d] = f32_to_bf16(np > 0 ? acc / L : 0.f);
}

// ---- balanced decode: every wave streams the same number of cache blocks ------------------
// The per-sequence split above gives a wave a whole context (or a fixed share of one), so on a
// ragged batch the waves' work differs by up to 90x and the CUs that drew the long contexts set
// the launch time (per-wave timeline: CU end time follows CU token count, correlation 0.79).
// Here the blocks of all sequences of one kv head are laid end to end (sequence-major) and wave
// w of W takes blocks [floor(w B / W), floor((w+1) B / W)) of that list: every wave streams
// B / W blocks whatever the context mix. A wave walks the sequences its range touches; a
// sequence wholly inside one wave is written directly, a split one leaves (o, m, l) records
// for the merge. A wave has at most two split segments (its first and its last), so records
// are addressed by (wave, 0 = first segment / 1 = last segment). Plan: one workgroup scans
// the block counts (pre[s] = blocks before sequence s) and finds each wave's first sequence.
constexpr int kPlanThreads = 1024;
constexpr int kPlanMaxSeqs = 8192;  // LDS prefix array (32 KB)

__device__ __forceinline__ int64_t wave_start(int w, int64_t B, int W) { return (int64_t)w * B / W; }
// the non-empty wave whose range holds block x: the largest w with wave_start(w) <= x
__device__ __forceinline__ int wave_of(int64_t x, int64_t B, int W) { return (int)(((x + 1) * W + B - 1) / B - 1); }

__global__ __launch_bounds__(kPlanThreads) void decode_plan_kernel(const int32_t* __restrict__ ctx_lens, int nseq,
                                                                   int W, int32_t* __restrict__ pre,
                                                                   int32_t* __restrict__ wave_seq) {
    __shared__ int32_t s_pre[kPlanMaxSeqs + 1];
    __shared__ int32_t s_wsum[kPlanThreads / kWave];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wid = tid / kWave;
    const int per = (nseq + kPlanThreads - 1) / kPlanThreads;
    const int lo = min(nseq, tid * per), hi = min(nseq, lo + per);
    int sum = 0;
    for (int i = lo; i < hi; ++i) sum += (ctx_lens[i] + kBS - 1) / kBS;
    int incl = sum;  // inclusive scan over the wave
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int v = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += v;
    }
    if (lane == kWave - 1) s_wsum[wid] = incl;
    __syncthreads();
    int base = incl - sum;
    for (int k = 0; k < wid; ++k) base += s_wsum[k];
    for (int i = lo; i < hi; ++i) {
        s_pre[i] = base;
        base += (ctx_lens[i] + kBS - 1) / kBS;
    }
    if (tid == kPlanThreads - 1) s_pre[nseq] = base;  // the last thread's running sum is the total
    __syncthreads();
    for (int i = tid; i <= nseq; i += kPlanThreads) pre[i] = s_pre[i];
    const int64_t B = s_pre[nseq];
    for (int w = tid; w < W; w += kPlanThreads) {
        const int64_t x = wave_start(w, B, W);
        int a = 0, b = nseq - 1;  // largest s with s_pre[s] <= x (contexts are >= 1 token)
        while (a < b) {
            const int mid = (a + b + 1) >> 1;
            if (s_pre[mid] <= x) a = mid;
            else b = mid - 1;
        }
        wave_seq[w] = x < B ? a : nseq;
    }
}

template <int D, int PF, int MINW>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MINW, 8))) void paged_decode_balanced_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int32_t* __restrict__ block_tables, int64_t bt_stride,
    const int32_t* __restrict__ ctx_lens, const int32_t* __restrict__ pre, const int32_t* __restrict__ wave_seq,
    int nseq, int W, int nh, int nkv, int qpk, float scale_log2, uint16_t* __restrict__ out, int64_t out_stride,
    float* __restrict__ ws_o, float* __restrict__ ws_ml) {
    constexpr int NT = D / 16;
    const int w = blockIdx.x;
    const int kvh = blockIdx.y;
    const int64_t B = pre[nseq];
    int64_t x0 = wave_start(w, B, W);
    const int64_t x1 = wave_start(w + 1, B, W);
    if (x0 >= x1) return;
    int s = wave_seq[w];
    const int lane = threadIdx.x;
    const int c = lane & 15;
    const int g = lane >> 4;
    const int h = kvh * qpk + c;
    const bool hv = c < qpk;
    int slot = 0;
    while (x0 < x1) {
        const int64_t ps = pre[s], pe = pre[s + 1];
        const int a = (int)(x0 - ps);
        const int b = (int)((x1 < pe ? x1 : pe) - ps);
        const int ctx = ctx_lens[s];
        const int t0 = a * kBS;
        const int t1 = min(ctx, b * kBS);
        f32x4 o[NT];
        float m, l;
        attend_range<D, PF>(q, q_stride, kc, vc, block_tables + (int64_t)s * bt_stride, s, kvh, t0, t1, nkv, qpk,
                            scale_log2, o, m, l);
        l += __shfl_xor(l, 16, kWave);
        l += __shfl_xor(l, 32, kWave);
        if (hv) {
            if (a == 0 && ps + b == pe) {  // the whole context in this wave
                const float inv = 1.f / l;
                uint16_t* orow = out + (int64_t)s * out_stride + (int64_t)h * D;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    uint2 v;
                    v.x = pack_bf16x2(o[n][0] * inv, o[n][1] * inv);
                    v.y = pack_bf16x2(o[n][2] * inv, o[n][3] * inv);
                    *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g) = v;
                }
            } else {
                const int64_t rec = ((int64_t)w * 2 + slot) * nh + h;
                float* wo = ws_o + rec * D;
#pragma unroll
                for (int n = 0; n < NT; ++n) *reinterpret_cast<f32x4*>(wo + 16 * n + 4 * g) = o[n];
                if (g == 0) {
                    ws_ml[rec * 2 + 0] = m;
                    ws_ml[rec * 2 + 1] = l;
                }
            }
        }
        x0 = pe;
        ++s;
        slot = 1;
    }
}

// Merge the split sequences' records: grid (nh, nseq), D threads; sequences inside one wave exit.
template <int D>
__global__ __launch_bounds__(D) void paged_decode_balanced_merge_kernel(
    const float* __restrict__ ws_o, const float* __restrict__ ws_ml, const int32_t* __restrict__ pre,
    const int32_t* __restrict__ wave_seq, int nseq, int W, int nh, uint16_t* __restrict__ out, int64_t out_stride) {
    const int h = blockIdx.x;
    const int s = blockIdx.y;
    const int d = threadIdx.x;
    const int64_t B = pre[nseq];
    const int64_t ps = pre[s], pe = pre[s + 1];
    const int wf = wave_of(ps, B, W), wl = wave_of(pe - 1, B, W);
    if (wf == wl) return;
    auto rec_of = [&](int w) -> int64_t { return ((int64_t)w * 2 + ((w == wf && wave_seq[w] != s) ? 1 : 0)) * nh + h; };
    float M = -INFINITY;
    for (int w = wf; w <= wl; ++w)
        if (wave_start(w, B, W) < wave_start(w + 1, B, W)) M = fmaxf(M, ws_ml[rec_of(w) * 2]);
    float L = 0.f, acc = 0.f;
    for (int w = wf; w <= wl; ++w) {
        if (wave_start(w, B, W) == wave_start(w + 1, B, W)) continue;
        const int64_t r = rec_of(w);
        const float e = fast_exp2(ws_ml[r * 2] - M);
        L += e * ws_ml[r * 2 + 1];
        acc += e * ws_o[r * D + d];
    }
    out[(int64_t)s * out_stride + (int64_t)h * D + d] = f32_to_bf16(acc / L);
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" int skyrl_rope_kv_write(const void* qkv, int64_t qkv_stride, int32_t T, int32_t nh, int32_t nkv,
                                   int32_t head_dim, const int64_t* positions, const int64_t* slot_mapping,
                                   const float* cos_sin, void* q_out, void* k_out, void* k_cache, void* v_cache,
                                   void* stream) {
    SKYRL_REQUIRE(T >= 0 && nh > 0 && nkv > 0 && nh % nkv == 0, "rope_kv_write: bad head counts");
    SKYRL_REQUIRE(head_dim == 64 || head_dim == 128, "rope_kv_write: head_dim must be 64 or 128");
    if (T == 0) return SKYRL_OK;
    SKYRL_REQUIRE(qkv && positions && slot_mapping && cos_sin && q_out && k_cache && v_cache,
                  "rope_kv_write: null pointer");
    SKYRL_REQUIRE(qkv_stride >= (int64_t)(nh + 2 * nkv) * head_dim, "rope_kv_write: qkv_stride too small");
    dim3 grid(T, nh + 2 * nkv);
    auto* src = reinterpret_cast<const uint16_t*>(qkv);
    auto* qo = reinterpret_cast<uint16_t*>(q_out);
    auto* ko = reinterpret_cast<uint16_t*>(k_out);
    auto* kcp = reinterpret_cast<uint16_t*>(k_cache);
    auto* vcp = reinterpret_cast<uint16_t*>(v_cache);
    if (head_dim == 128)
        hipLaunchKernelGGL(rope_kv_write_kernel<128>, grid, dim3(64), 0, as_stream(stream), src, qkv_stride,
                           positions, slot_mapping, cos_sin, nh, nkv, qo, ko, kcp, vcp);
    else
        hipLaunchKernelGGL(rope_kv_write_kernel<64>, grid, dim3(64), 0, as_stream(stream), src, qkv_stride,
                           positions, slot_mapping, cos_sin, nh, nkv, qo, ko, kcp, vcp);
    return check_launch("rope_kv_write_kernel");
}

extern "C" size_t skyrl_paged_decode_workspace_bytes(int32_t nseq, int32_t nh, int32_t head_dim, int32_t nparts) {
    if (nparts <= 1) return 0;
    const size_t recs = (size_t)(nseq > 0 ? nseq : 1) * (size_t)nh * (size_t)nparts;
    return recs * ((size_t)head_dim + 2) * sizeof(float);
}

namespace skyrl {
}

extern "C" int skyrl_paged_decode(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                                  const int32_t* block_tables, int64_t bt_stride, const int32_t* context_lens,
                                  int32_t nseq, int32_t nh, int32_t nkv, int32_t head_dim, float scale,
                                  int32_t part_tokens, int32_t nparts, void* out, int64_t out_stride, void* workspace,
                                  void* stream) {
    SKYRL_REQUIRE(nseq >= 0 && nh > 0 && nkv > 0 && nh % nkv == 0, "paged_decode: bad head counts");
    SKYRL_REQUIRE(nh / nkv <= 16, "paged_decode: more than 16 query heads per kv head");
    SKYRL_REQUIRE(head_dim == 64 || head_dim == 128, "paged_decode: head_dim must be 64 or 128");
    SKYRL_REQUIRE(part_tokens > 0 && part_tokens % kBS == 0,
                  "paged_decode: part_tokens (minimum partition) must be a multiple of 16");
    SKYRL_REQUIRE(nparts >= 1, "paged_decode: nparts must be >= 1");
    if (nseq == 0) return SKYRL_OK;
    SKYRL_REQUIRE(q && k_cache && v_cache && block_tables && context_lens && out, "paged_decode: null pointer");
    SKYRL_REQUIRE(nparts == 1 || workspace, "paged_decode: nparts > 1 needs the workspace");
    SKYRL_REQUIRE(q_stride >= (int64_t)nh * head_dim && out_stride >= (int64_t)nh * head_dim,
                  "paged_decode: row stride smaller than nh * head_dim");
    SKYRL_REQUIRE((reinterpret_cast<uintptr_t>(q) % 16) == 0 && (q_stride % 8) == 0,
                  "paged_decode: q must be 16-B aligned with a row stride multiple of 8");
    const float scale_log2 = scale * 1.4426950408889634f;
    const int qpk = nh / nkv;
    float* ws_o = reinterpret_cast<float*>(workspace);
    float* ws_ml = ws_o ? ws_o + (size_t)nseq * nh * nparts * head_dim : nullptr;
    dim3 grid(nparts, nkv, nseq);
    auto* qp = reinterpret_cast<const uint16_t*>(q);
    auto* kp = reinterpret_cast<const uint16_t*>(k_cache);
    auto* vp = reinterpret_cast<const uint16_t*>(v_cache);
    auto* op = reinterpret_cast<uint16_t*>(out);
    // D = 128: 4 blocks in flight (205 VGPRs, 2 waves / SIMD). Measured on the ragged rollout mix
    // (512 x U[17,1536]): 92 us vs 101 for the earlier 3-deep loop; 6 and 8 deep (1 wave / SIMD,
    // ring partly in AGPRs) 94-96 us; 3 deep in this unrolled form spills at 3 waves / SIMD.
    const int pf = knobs().attn_pf > 0 ? knobs().attn_pf : 4;
#define SKYRL_PD_LAUNCH(DD, PF, MINW)                                                                          \
    hipLaunchKernelGGL((paged_decode_kernel<DD, PF, MINW>), grid, dim3(64), 0, as_stream(stream), qp, q_stride, kp, \
                       vp, block_tables, bt_stride, context_lens, nh, nkv, qpk, scale_log2, part_tokens, nparts, op, \
                       out_stride, ws_o, ws_ml)
    if (head_dim == 128) {
        switch (pf) {
            case 6: SKYRL_PD_LAUNCH(128, 6, 1); break;
            case 8: SKYRL_PD_LAUNCH(128, 8, 1); break;
            default: SKYRL_PD_LAUNCH(128, 4, 2); break;
        }
    } else {
        SKYRL_PD_LAUNCH(64, 3, 3);
    }
#undef SKYRL_PD_LAUNCH
    int rc = check_launch("paged_decode_kernel");
    if (rc || nparts == 1) return rc;
    dim3 rgrid(nh, nseq);
    if (head_dim == 128)
        hipLaunchKernelGGL(paged_decode_reduce_kernel<128>, rgrid, dim3(128), 0, as_stream(stream), ws_o, ws_ml,
                           context_lens, nh, part_tokens, nparts, op, out_stride);
    else
        hipLaunchKernelGGL(paged_decode_reduce_kernel<64>, rgrid, dim3(64), 0, as_stream(stream), ws_o, ws_ml,
                           context_lens, nh, part_tokens, nparts, op, out_stride);
    return check_launch("paged_decode_reduce_kernel");
}

extern "C" size_t skyrl_paged_decode_balanced_workspace_bytes(int32_t nseq, int32_t nh, int32_t head_dim,
                                                              int32_t waves) {
    const size_t ints = (((size_t)(nseq > 0 ? nseq : 0) + 1 + (size_t)(waves > 0 ? waves : 0)) * 4 + 255) / 256 * 256;
    const size_t recs = (size_t)(waves > 0 ? waves : 0) * 2 * (size_t)nh;
    return ints + recs * (size_t)head_dim * 4 + recs * 2 * 4;
}

extern "C" int skyrl_paged_decode_balanced(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                                           const int32_t* block_tables, int64_t bt_stride,
                                           const int32_t* context_lens, int32_t nseq, int32_t nh, int32_t nkv,
                                           int32_t head_dim, float scale, int32_t waves, void* out,
                                           int64_t out_stride, void* workspace, void* stream) {
    SKYRL_REQUIRE(nseq >= 0 && nseq <= kPlanMaxSeqs, "paged_decode_balanced: nseq must be in [0, 8192]");
    SKYRL_REQUIRE(nh > 0 && nkv > 0 && nh % nkv == 0 && nh / nkv <= 16, "paged_decode_balanced: bad head counts");
    SKYRL_REQUIRE(head_dim == 64 || head_dim == 128, "paged_decode_balanced: head_dim must be 64 or 128");
    SKYRL_REQUIRE(waves >= 1, "paged_decode_balanced: waves must be >= 1");
    if (nseq == 0) return SKYRL_OK;
    SKYRL_REQUIRE(q && k_cache && v_cache && block_tables && context_lens && out && workspace,
                  "paged_decode_balanced: null pointer");
    SKYRL_REQUIRE(q_stride >= (int64_t)nh * head_dim && out_stride >= (int64_t)nh * head_dim,
                  "paged_decode_balanced: row stride smaller than nh * head_dim");
    SKYRL_REQUIRE((reinterpret_cast<uintptr_t>(q) % 16) == 0 && (q_stride % 8) == 0,
                  "paged_decode_balanced: q must be 16-B aligned with a row stride multiple of 8");
    const float scale_log2 = scale * 1.4426950408889634f;
    const int qpk = nh / nkv;
    char* wsb = reinterpret_cast<char*>(workspace);
    int32_t* pre = reinterpret_cast<int32_t*>(wsb);
    int32_t* wave_seq = pre + nseq + 1;
    const size_t ints = (((size_t)nseq + 1 + (size_t)waves) * 4 + 255) / 256 * 256;
    float* ws_o = reinterpret_cast<float*>(wsb + ints);
    float* ws_ml = ws_o + (size_t)waves * 2 * nh * head_dim;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(decode_plan_kernel, dim3(1), dim3(kPlanThreads), 0, st, context_lens, nseq, waves, pre,
                       wave_seq);
    int rc = check_launch("decode_plan_kernel");
    if (rc) return rc;
    auto* qp = reinterpret_cast<const uint16_t*>(q);
    auto* kp = reinterpret_cast<const uint16_t*>(k_cache);
    auto* vp = reinterpret_cast<const uint16_t*>(v_cache);
    auto* op = reinterpret_cast<uint16_t*>(out);
    dim3 grid(waves, nkv);
    if (head_dim == 128)
        hipLaunchKernelGGL((paged_decode_balanced_kernel<128, 4, 2>), grid, dim3(64), 0, st, qp, q_stride, kp, vp,
                           block_tables, bt_stride, context_lens, pre, wave_seq, nseq, waves, nh, nkv, qpk,
                           scale_log2, op, out_stride, ws_o, ws_ml);
    else
        hipLaunchKernelGGL((paged_decode_balanced_kernel<64, 3, 3>), grid, dim3(64), 0, st, qp, q_stride, kp, vp,
                           block_tables, bt_stride, context_lens, pre, wave_seq, nseq, waves, nh, nkv, qpk,
                           scale_log2, op, out_stride, ws_o, ws_ml);
    rc = check_launch("paged_decode_balanced_kernel");
    if (rc) return rc;
    dim3 rgrid(nh, nseq);
    if (head_dim == 128)
        hipLaunchKernelGGL(paged_decode_balanced_merge_kernel<128>, rgrid, dim3(128), 0, st, ws_o, ws_ml, pre,
                           wave_seq, nseq, waves, nh, op, out_stride);
    else
        hipLaunchKernelGGL(paged_decode_balanced_merge_kernel<64>, rgrid, dim3(64), 0, st, ws_o, ws_ml, pre,
                           wave_seq, nseq, waves, nh, op, out_stride);
    return check_launch("paged_decode_balanced_merge_kernel");
}
