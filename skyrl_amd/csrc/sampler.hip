// a1: rollout token sampling with sampled-token logprob.
//
// Replaces the vLLM sampler behind VLLMInferenceEngine.generate
// (skyrl-train/skyrl_train/inference_engines/vllm/vllm_engine.py:196-218,
// logprob extraction :139-149; params inference_engines/utils.py:15-42,
// defaults config/ppo_base_config.yaml:316-324). Filter semantics follow
// skyrl-tx/tx/utils/generator.py:213-227,398-449: temperature first, then
// top_k (exactly k: the k largest, equal values in index order, as lax.top_k + the first-k
// mask of apply_top_k_batch :410-418), then min_p, then top_p; T == 0 is greedy
// over the raw logits; the returned logprob is log_softmax(raw logits)[token].
//
// Sampling is Gumbel-max, argmax_v (x_v/T - ln E_v) with E_v iid Exp(1), drawn per group of 8
// elements through their order statistics (see the noise model in sample_kernel) from
// counter-based integer hashes of (seed, seq_id, step, v). Every float
// operation on the decision path is an IEEE basic op or an explicit fmaf and
// contraction is off in this file, so the token is a pure function of the
// inputs and oracle/sampler_ref.c reproduces it bit for bit.
//
// Layout: grid = (sequence, vocab split); each 256-thread workgroup streams
// its split of the row (16-B bf16 vectors), keeps per lane the best
// (score, index) and the raw online (max, sum-exp), reduces in the wave and
// workgroup, and the last-arriving split of the row (arrive.h) folds the
// partials in split order (lowest index wins ties).
#include "arrive.h"
#include "noise.h"
#include "variant.h"

#include <type_traits>

#pragma clang fp contract(off)

namespace skyrl {
// Sampler variants (skyrl_variant, per call; the defaults are the tuned choices): sampler_row (1 =
// progress-priority row kernel, 0 = plain), sampler_split_rows (rows split over workgroups below
// this), sampler_split_wgs (workgroups a split launch aims at: 4 per CU at 256 threads),
// sampler_split_nt (threads per split workgroup), sampler_split_gran (split chunks are multiples of
// this many elements), sampler_topk_fast (0 = top_k on the pre-pass + MODE 2 kernels),
// sampler_topp_fast (0 = top_p / min_p
// alone on the pre-pass + MODE 2 kernels; 1 = the one-pass kernel, except min_p without top_p below
// the row-mode batch, where the pre-pass and the split MODE 2 sampler measured faster (32 / 64 / 128
// rows: 26.2 / 33.0 / 43.2 vs 43.8 / 44.8 / 47.4 us; 256 rows: 68.1 vs 49.6; same tokens;
// profiles/r05_topp_rows.json); 2 = always the one-pass kernel), topp_probe (timing probes: 1 pass 1
// alone, 2 pass 1 + the cut, 3 / 4 + a bare re-read (tokens invalid); 5 every row through pass 2
// (valid tokens); 6 / 7 min_p's in-row pass 2 timed per row (tokens = ticks; 7 without the visits);
// 11 per row, the cut's and pass 1's times in the outputs).
#ifndef SKYRL_TP_PROBE0  // scripts/probe/topp_variants.py builds with another default; the product: 0
#define SKYRL_TP_PROBE0 0
#endif
namespace {

constexpr int kThreads = 256;
constexpr int kMaxSplitRows = 1024;  // split mode is never used at or above this many rows
// Workspace: a fixed-size region of per-row arrival counters first (only split mode uses them),
// so that the counters sit at the same place for every batch size and never overlap another
// call's row filters or partials in a reused workspace (a split-mode call after one with fewer
// rows would otherwise read that call's partials as counters): every counter is zero at
// allocation and re-armed by its user.
constexpr size_t kCounterBytes = (size_t)kMaxSplitRows * 4;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// order-preserving unsigned keys
__device__ __forceinline__ uint32_t okey_bf16(uint16_t h) {
    return (h & 0x8000u) ? (uint32_t)(uint16_t)~h : (uint32_t)(h | 0x8000u);
}
__device__ __forceinline__ uint32_t okey_f32(uint32_t u) { return (u & 0x80000000u) ? ~u : (u | 0x80000000u); }

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// logits rows are read once per decode step: non-temporal streaming loads
__device__ __forceinline__ uint4 ld_stream(const uint4* p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

struct Part {  // per (row, split) partial
    float score;
    int idx;
    float m;
    float s;
    float xb;  // raw logit of idx (the logprob needs no re-load of the winner)
};

// Fold partial b into a: best (score desc, index asc) with its raw logit, and the raw online
// (max, sum-exp). Every fold below runs in a fixed order, so the result is deterministic.
__device__ __forceinline__ void part_merge(Part& a, const Part& b) {
    const Best ab{a.score, a.idx};
    if (better(b.score, b.idx, ab)) {
        a.score = b.score;
        a.idx = b.idx;
        a.xb = b.xb;
    }
    const float mn = fmaxf(a.m, b.m);
    a.s = a.s * fast_exp2((a.m - mn) * kLog2e) + b.s * fast_exp2((b.m - mn) * kLog2e);
    a.m = mn;
}
template <int CTRL>
__device__ __forceinline__ void part_dpp_step(Part& p) {
    auto mv = [](float x) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false)); };
    const Part o{mv(p.score), __builtin_amdgcn_update_dpp(0, p.idx, CTRL, 0xF, 0xF, false), mv(p.m), mv(p.s), mv(p.xb)};
    part_merge(p, o);
}
__device__ __forceinline__ Part part_readlane(const Part& p, int l) {
    auto rl = [l](float x) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l)); };
    return Part{rl(p.score), __builtin_amdgcn_readlane(p.idx, l), rl(p.m), rl(p.s), rl(p.xb)};
}
// Wave-wide fold on DPP (quad_perm xor 1 / xor 2, row_ror 4 / 8 inside each 16-lane row) and the
// four row results read with v_readlane, no LDS round trips; the result is wave-uniform.
// Requires all 64 lanes active.
__device__ __forceinline__ Part wave_reduce_part(Part p) {
    part_dpp_step<0xB1>(p);
    part_dpp_step<0x4E>(p);
    part_dpp_step<0x124>(p);
    part_dpp_step<0x128>(p);
    Part r0 = part_readlane(p, 0), r2 = part_readlane(p, 32);
    part_merge(r0, part_readlane(p, 16));
    part_merge(r2, part_readlane(p, 48));
    part_merge(r0, r2);
    return r0;
}

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<uint16_t>(uint16_t v) { return bf16_to_f32(v); }
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <typename T>
__device__ __forceinline__ uint32_t okey(T v);
template <> __device__ __forceinline__ uint32_t okey<uint16_t>(uint16_t v) { return okey_bf16(v); }
template <> __device__ __forceinline__ uint32_t okey<float>(float v) { return okey_f32(__float_as_uint(v)); }

// inverse of okey: the logit value of a key
template <typename T>
__device__ __forceinline__ float from_key(uint32_t k);
template <> __device__ __forceinline__ float from_key<uint16_t>(uint32_t k) {
    return bf16_to_f32((uint16_t)((k & 0x8000u) ? (k & 0x7fffu) : (~k & 0xffffu)));
}
template <> __device__ __forceinline__ float from_key<float>(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Deterministic 2^y for y <= 0 (0 below -126): floor split, degree-6 fit of 2^f on [0, 1)
// (max rel. err 6e-8), exponent added in the bit pattern. Bit-identical in sampler_ref.c.
__host__ __device__ __forceinline__ float det_exp2(float y) {
    const float yc = y >= -126.0f ? y : -126.0f;
    const float fi = floorf(yc);
    const float f = yc - fi;
    float p = 2.170088992e-04f;
    p = fmaf(p, f, 1.243957202e-03f);
    p = fmaf(p, f, 9.678921662e-03f);
    p = fmaf(p, f, 5.548325926e-02f);
    p = fmaf(p, f, 2.402298748e-01f);
    p = fmaf(p, f, 6.931470037e-01f);
    p = fmaf(p, f, 1.0f);
    const float r = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, p) + ((uint32_t)(int)fi << 23));
    return y >= -126.0f ? r : 0.0f;
}
// top_p mass of a logit in fixed point: 2^31 * e^((x - max) / T), as an integer so that every
// sum is exact and order-independent (the oracle makes the same decisions bit for bit)
__host__ __device__ __forceinline__ uint32_t mass_q(float x, float mx, float inv_t) {
    const float y = ((x - mx) * inv_t) * 1.4426950408889634f;
    return (uint32_t)(det_exp2(y) * 2147483648.0f);
}

struct RowFilter {  // per row, written by the filter pre-pass
    float rmax;     // raw max logit
    uint32_t tk;    // top_k: keep keys > tk, and key == tk at indices <= ik
    int32_t ik;
    uint32_t kc;    // top_p: keep keys > kc, and key == kc at indices <= ic
    int32_t ic;
};
// a key at index i inside a (key, index) cut: keys above it, or equal at an index up to it
__device__ __forceinline__ bool in_cut(uint32_t kk, int i, uint32_t kcut, int icut) {
    return kk > kcut || (kk == kcut && i <= icut);
}

// ---- filter pre-pass: one 1024-thread workgroup per row ---------------------------------
// top_k (tx generator.py:398-420: lax.top_k keeps exactly k, equal logits in index order, the
// fixture tests/utils/test_generator.py:197-207) and top_p (tx generator.py:424-449 on the
// top_k- and min_p-filtered distribution: tokens in descending order, equal logits in index
// order (a stable argsort), are kept while the probability mass strictly before them is < p,
// the top token always) by MSB-first radix selection over d = key(max) - key with 8-bit digits
// (2 levels for bf16, 4 for f32): a 256-bin LDS histogram of counts (top_k) or of the
// fixed-point masses (top_p) per level. The tie group at either cut is resolved by an
// index-ordered count: the cut is a (key, last index) pair.
constexpr int kFT = 1024;
// One row's cuts with FT threads (the pre-pass kernel: 1024; the top_k fast path's fallback: 512).
template <typename T, int FT>
__device__ __forceinline__ void filter_row(const T* __restrict__ logits, int64_t ld, int V, int top_k, int use_minp,
                                           float inv_t, float ln_min_p, float top_p, RowFilter* __restrict__ dst,
                                           const int row_i) {
    constexpr int NW = FT / kWave;
    constexpr int KB = sizeof(T) * 8;
    __shared__ unsigned long long hist[256];
    __shared__ unsigned long long s_red[NW], s_red2[NW];
    __shared__ unsigned long long s_fine[FT];
    __shared__ uint32_t s_u[NW];
    __shared__ uint32_t s_sel[2];               // selected d, found flag
    __shared__ unsigned long long s_below, s_at;
    __shared__ int s_ic;
    const T* row = logits + (int64_t)row_i * ld;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    constexpr int VEC = 16 / sizeof(T);
    // every pass visits the row in 16-B vectors where aligned (VEC elements per thread per
    // step), the unaligned head/tail element-wise; fn(raw, index)
    const int head = (int)((16 - (reinterpret_cast<uintptr_t>(row) & 15)) & 15) / (int)sizeof(T);
    const int h0 = head < V ? head : V;
    const int nv = (V - h0) / VEC;
    const int t0 = h0 + nv * VEC;
    auto for_each = [&](auto fn) {
        if ((reinterpret_cast<uintptr_t>(row) & (sizeof(T) - 1)) == 0) {
            for (int i = threadIdx.x; i < h0; i += FT) fn(row[i], i);
            const uint4* rv = reinterpret_cast<const uint4*>(row + h0);
            for (int j = threadIdx.x; j < nv; j += FT) {
                const uint4 pk = rv[j];
                T vals[VEC];
                __builtin_memcpy(vals, &pk, 16);
#pragma unroll
                for (int k = 0; k < VEC; ++k) fn(vals[k], h0 + j * VEC + k);
            }
            for (int i = t0 + threadIdx.x; i < V; i += FT) fn(row[i], i);
        } else {
            for (int i = threadIdx.x; i < V; i += FT) fn(row[i], i);
        }
    };

    // pass 0: max key (an integer max, exact)
    uint32_t km = 0u;
    for_each([&](T raw, int) { km = max(km, okey<T>(raw)); });
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) km = max(km, (uint32_t)__shfl_xor((int)km, off, kWave));
    if (lane == 0) s_u[w] = km;
    __syncthreads();
    uint32_t kmax = s_u[0];
#pragma unroll
    for (int j = 1; j < NW; ++j) kmax = max(kmax, s_u[j]);
    const float mx = from_key<T>(kmax);
    const float mthr = mx * inv_t + ln_min_p;
    __syncthreads();

    // MSB-first radix selection: smallest d with (sum of weights over d' <= d) >= target
    auto radix = [&](auto weight, double target) {
        uint32_t prefix = 0u;
        unsigned long long below = 0ull, at = 0ull;
        for (int lvl = 0; lvl < KB / 8; ++lvl) {
            const int shift = KB - 8 * (lvl + 1);
            for (int j = threadIdx.x; j < 256; j += FT) hist[j] = 0ull;
            __syncthreads();
            for_each([&](T raw, int i) {
                const uint32_t d = kmax - okey<T>(raw);
                if (lvl > 0 && (d >> (shift + 8)) != prefix) return;
                const unsigned long long wt = weight(raw, i);
                if (wt) atomicAdd(&hist[(d >> shift) & 255u], wt);
            });
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned long long cum = below;
                int dg = 0;
                for (; dg < 255; ++dg) {
                    if ((double)(cum + hist[dg]) >= target) break;
                    cum += hist[dg];
                }
                s_below = cum;
                s_at = hist[dg];
                s_sel[0] = (prefix << 8) | (uint32_t)dg;
            }
            __syncthreads();
            prefix = s_sel[0];
            below = s_below;
            at = s_at;
            __syncthreads();
        }
        struct R { uint32_t d; unsigned long long below, at; };
        return R{prefix, below, at};
    };

    // bf16 fast path: one pass with a full-resolution histogram of d < kFine (every bf16 value
    // within kFine steps of the max has its own bin; the rest is summed in registers), then a
    // block-wide scan of the bins. Falls back to the radix passes when the target is not
    // reached inside the window.
    constexpr int kFine = FT;
    struct Sel { bool ok; uint32_t d; unsigned long long below, at, total; };
    auto fine = [&](auto weight, double target, bool want_total) -> Sel {
        unsigned long long* fh = reinterpret_cast<unsigned long long*>(s_fine);
        fh[threadIdx.x] = 0ull;
        __syncthreads();
        unsigned long long rest = 0ull;
        for_each([&](T raw, int i) {
            const unsigned long long wt = weight(raw, i);
            if (!wt) return;
            const uint32_t d = kmax - okey<T>(raw);
            if (d < (uint32_t)kFine) atomicAdd(&fh[d], wt);
            else rest += wt;
        });
        __syncthreads();
        // inclusive scan over the kFine bins (bin = thread), plus the out-of-window total
        const unsigned long long mine = fh[threadIdx.x];
        unsigned long long incl = mine;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const unsigned long long o = (unsigned long long)__shfl_up((long long)incl, off, kWave);
            if (lane >= off) incl += o;
        }
        if (want_total) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) rest += (unsigned long long)__shfl_xor((long long)rest, off, kWave);
        }
        if (lane == kWave - 1) s_red[w] = incl;
        if (lane == 0) s_red2[w] = rest;
        if (threadIdx.x == 0) s_sel[1] = 0u;
        __syncthreads();
        unsigned long long off_w = 0ull, win = 0ull, tot_rest = 0ull;
        for (int j = 0; j < NW; ++j) {
            if (j < w) off_w += s_red[j];
            win += s_red[j];
            tot_rest += s_red2[j];
        }
        const unsigned long long total = win + tot_rest;
        const double tgt = target < 0.0 ? (double)top_p * (double)total : target;  // top_p: p * Z
        const unsigned long long cum_in = off_w + incl, cum_before = cum_in - mine;
        if (mine && (double)cum_before < tgt && (double)cum_in >= tgt) {
            s_sel[0] = threadIdx.x;
            s_sel[1] = 1u;
            s_below = cum_before;
            s_at = mine;
        }
        __syncthreads();
        Sel r{s_sel[1] != 0u, s_sel[0], s_below, s_at, total};
        __syncthreads();
        return r;
    };

    // index of the c-th (1-based) element in index order with pred(raw, i): rounds of FT
    // contiguous chunks of CH elements (thread t owns [base + t*CH, base + (t+1)*CH))
    auto nth_index = [&](auto pred, long long c) -> int {
        constexpr int CH = 16;
        if (threadIdx.x == 0) s_ic = 0x7fffffff;
        long long seen = 0;
        for (int base = 0; base < V; base += FT * CH) {
            const int i0 = base + threadIdx.x * CH;
            int cntt = 0;
            for (int k = 0; k < CH; ++k) {
                const int i = i0 + k;
                if (i < V && pred(row[i], i)) ++cntt;
            }
            // block exclusive scan of cntt (wave scan + per-wave totals)
            int incl = cntt;
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const int o = __shfl_up(incl, off, kWave);
                if (lane >= off) incl += o;
            }
            if (lane == kWave - 1) s_u[w] = (uint32_t)incl;
            __syncthreads();
            long long off_w = 0, tot = 0;
            for (int j = 0; j < NW; ++j) {
                if (j < w) off_w += s_u[j];
                tot += s_u[j];
            }
            const long long before = seen + off_w + (incl - cntt);
            if (cntt > 0 && before < c && before + cntt >= c) {  // the c-th is in my chunk
                long long r2 = before;
                for (int k = 0; k < CH; ++k) {
                    const int i = i0 + k;
                    if (i < V && pred(row[i], i) && ++r2 == c) s_ic = i;
                }
            }
            seen += tot;
            __syncthreads();
            if (seen >= c) break;
        }
        const int r = s_ic;
        __syncthreads();
        return r;
    };

    uint32_t tk = 0u;
    int ik = 0x7fffffff;
    if (top_k > 0 && top_k < V) {
        bool done = false;
        unsigned long long kbelow = 0ull, kat = 0ull;
        if constexpr (sizeof(T) == 2) {
            const Sel f = fine([&](T, int) -> unsigned long long { return 1ull; }, (double)top_k, false);
            if (f.ok) {
                tk = kmax - f.d;
                kbelow = f.below;
                kat = f.at;
                done = true;
            }
        }
        if (!done) {
            const auto r = radix([&](T, int) -> unsigned long long { return 1ull; }, (double)top_k);
            tk = kmax - r.d;
            kbelow = r.below;
            kat = r.at;
        }
        // exactly k: the first (k - #above) of the tk tie group in index order
        const long long c = (long long)top_k - (long long)kbelow;
        if (c < (long long)kat) ik = nth_index([&](T raw, int) -> bool { return okey<T>(raw) == tk; }, c);
    }
    uint32_t kc = 0u;
    int ic = 0x7fffffff;
    if (top_p < 1.0f) {
        auto kept = [&](T raw, int i) -> bool {
            return in_cut(okey<T>(raw), i, tk, ik) && (!use_minp || to_f<T>(raw) * inv_t >= mthr);
        };
        auto wmass = [&](T raw, int i) -> unsigned long long {
            return kept(raw, i) ? (unsigned long long)mass_q(to_f<T>(raw), mx, inv_t) : 0ull; };
        uint32_t dsel = 0u;
        unsigned long long below = 0ull, at = 0ull, Z = 0ull;
        double target = 0.0;
        bool done = false;
        if constexpr (sizeof(T) == 2) {  // Z and the cut in one pass (target = p * Z inside)
            const Sel f = fine(wmass, -1.0, true);
            Z = f.total;
            target = (double)top_p * (double)Z;
            if (f.ok) {
                dsel = f.d;
                below = f.below;
                at = f.at;
                done = true;
            }
        }
        if (!done) {
            if (Z == 0ull) {  // Z: exact integer sum of the kept masses
                unsigned long long z = 0ull;
                for_each([&](T raw, int i) { z += wmass(raw, i); });
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) z += (unsigned long long)__shfl_xor((long long)z, off, kWave);
                if (lane == 0) s_red[w] = z;
                __syncthreads();
#pragma unroll
                for (int j = 0; j < NW; ++j) Z += s_red[j];
                __syncthreads();
                target = (double)top_p * (double)Z;
            }
            const auto r = radix(wmass, target);
            dsel = r.d;
            below = r.below;
            at = r.at;
        }
        struct { uint32_t d; unsigned long long below, at; } r{dsel, below, at};
        kc = kmax - r.d;
        const unsigned long long qc = mass_q(from_key<T>(kc), mx, inv_t);
        const unsigned long long A = r.below;
        if (qc != 0ull) {
            // c = number of tie ranks j >= 0 with A + j qc < target (the first always for the top key)
            const double jd = (target - (double)A) / (double)qc;
            long long c = jd > 0.0 ? (long long)jd : 0;
            while (c > 0 && (double)(A + (unsigned long long)(c - 1) * qc) >= target) --c;
            while ((double)(A + (unsigned long long)c * qc) < target) ++c;
            if (kc == kmax && c < 1) c = 1;
            const long long cnt = (long long)(r.at / qc);
            if (c < cnt)
                ic = nth_index([&](T raw, int i) -> bool { return okey<T>(raw) == kc && kept(raw, i); }, c);
        }
    }
    if (threadIdx.x == 0) *dst = RowFilter{mx, tk, ik, kc, ic};
}
template <typename T>
__global__ __launch_bounds__(kFT) void sample_filter_kernel(const T* __restrict__ logits, int64_t ld, int V, int top_k,
                                                            int use_minp, float inv_t, float ln_min_p, float top_p,
                                                            RowFilter* __restrict__ out) {
    filter_row<T, kFT>(logits, ld, V, top_k, use_minp, inv_t, ln_min_p, top_p, out + blockIdx.x, blockIdx.x);
}

// MODE: 0 greedy (T == 0), 1 Gumbel-max without filters, 2 Gumbel-max with top_k / min_p,
// 3 Gumbel-max without filters at T == 1 in row mode (the bound test reuses the lse exponentials).
// NT threads per workgroup. Grid (row, split): with one split the workgroup owns the whole
// row and finishes it alone; with several, the last-arriving split folds the partials.
// Phase timestamps for scripts/probe/sampler_phase_probe (compiled only there, never in the product).
#ifdef SKYRL_SAMPLER_PHASE_PROBE
__device__ uint64_t g_sphase[4096 * 8];
#define SPHASE(k)                                                                              \
    do {                                                                                       \
        const unsigned lin_ = blockIdx.y * gridDim.x + blockIdx.x;                             \
        if (threadIdx.x == 0 && lin_ < 4096) {                                                 \
            g_sphase[lin_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                       \
            if ((k) == 0) g_sphase[lin_ * 8 + 7] = (uint64_t)__smid();                         \
            if ((k) == 0) g_sphase[lin_ * 8 + 6] = __builtin_amdgcn_s_getreg(20 | (3 << 11));  \
        }                                                                                      \
    } while (0)
#else
#define SPHASE(k) \
    do {          \
    } while (0)
#endif

// PRIO: the waves raise their issue priority with the fraction of their row still to stream
// (3 in the first quarter ... 0 in the last), so of the two row workgroups sharing a CU the one
// behind is issued first and both finish together (otherwise age priority lets the first-
// dispatched one finish ~9 us ahead at T = 1 and the other streams its tail alone).
// One work unit: split `split` of `nsplit` of row row_i (the whole row when nsplit == 1).
// TieSink (the top_p kernel's pass 2, TIES = true): elements whose key is `kc` are taken out of
// the decision and appended to an LDS list with their exact scores (the caller ranks them by
// index: the cut keeps the first c); a kc no key equals (> 0xffff) disables it at run time.
// the top_p kernel's pass-1 bar: 1 publishes only when a lane improved (product), 0 after every
// candidate vector (probe builds, scripts/probe/sampler_ab.py)
#ifndef SKYRL_TP_BAR_FORM
#define SKYRL_TP_BAR_FORM 1
#endif
// the same for the top_p pass-2 kernel's pieces (1, product; the form measured 65 -> 80 us in the
// in-row min_p pass 2, which keeps publishing after every candidate vector:
// profiles/r05_topp2_bar_form_ab.json)
#ifndef SKYRL_TP2_BAR_FORM
#define SKYRL_TP2_BAR_FORM 1
#endif
// the top_p kernel's pass-1 bar (top_p only; min_p alone keeps the best record): R = 1 the best
// exact score so far; R > 1 the R-th largest of the 8 waves' best scores, a lower bound on the
// row's R-th best score, so pass 1 certifies a row unless its R best elements are all outside the
// kept set (about (1 - top_p)^R of the rows). R = 3 (product): 0.05 rows of 512 left to pass 2
// at top_p 0.95 against 27 with R = 1; pass 1 costs 49 -> 59 us (the lower bar lets ~2x the
// candidate events through) and whole calls 77.7 / 70.3 / 80.0 -> 66.5 / 65.6 / 73.7 us at top_p
// 0.95 T = 1 / 0.6 and top_p 0.9 (R = 2: 73.2 / 71.9 / 84.5, R = 4 slower than 3; tokens bit-exact;
// profiles/r06v_topp_rbar_ab.json, scripts/probe/topp_rbar_ab.py)
#ifndef SKYRL_TP_RBAR
#define SKYRL_TP_RBAR 3
#endif
// pass 1 ranks the split cut key's records that beat e* by a scan of the row prefix (1, product:
// with R = 3 these were most of the rows left, 9 of 11 over 20 steps) or leaves the row to pass 2 (0)
#ifndef SKYRL_TP_TIERES
#define SKYRL_TP_TIERES 1
#endif
// min_p alone (sample_topp_kernel<T, false>): pass 1 lists every element with x/T >= (a lower
// bound of the row max)/T + ln min_p -- a superset of the kept set -- instead of running the race,
// and decides the row from the list once the max is known (1, product: every row decided in pass 1
// against ~32 % with the race; min_p 0.05 at 512 x 151,936: 66.3 -> 50.7 us at T = 1, 60.7 -> 43.4
// at T = 0.6, min_p 0.1 64.9 -> 45.8; tokens bit-exact; profiles/r06x_minp_list_ab.json); or the
// race + certificate (0)
#ifndef SKYRL_MP_LIST
#define SKYRL_MP_LIST 1
#endif
#ifndef SKYRL_TP_RBAR_VEC  // R > 1: the waves' bests read by two 16-B LDS loads (1) or 8 atomic loads (0)
#define SKYRL_TP_RBAR_VEC 1
#endif
static_assert(SKYRL_TP_BAR_FORM || SKYRL_TP_RBAR == 1, "the R-th-best bar is built on the publish-on-improvement form");
struct TieSink {
    int32_t* idx;
    float* sc;
    uint32_t* n;
    int cap;
    uint32_t kc;
};

// Exact scores of the slots in `needm` of one vector (elements v0 + k, group hash h): the best
// (score desc; ascending k, so a strict '>' keeps the lowest index, as the caller's ascending visit
// order requires) starting from b. Inlined, with one copy of the scoring per site (a loop over
// the needed slots): a call would drain the caller's loads in flight (noise.h).
struct Slots8 {
    float v[8];
};
struct SlotBest {
    float s;
    int i;
    float x;
};
__device__ SKYRL_NOISE_ATTR SlotBest eval_slots(Slots8 xs, unsigned needm, int v0, uint32_t h, float inv_t,
                                                uint32_t key2, SlotBest b) {
    const float Eg = group_min_e(h);
#if SKYRL_NOISE_INLINE == 2  // one copy of the scoring per site: a loop over the needed slots
    for (unsigned m = needm; m; m &= m - 1) {
        const int k = __builtin_ctz(m);
        const float x01 = (k & 1) ? xs.v[1] : xs.v[0], x23 = (k & 1) ? xs.v[3] : xs.v[2];
        const float x45 = (k & 1) ? xs.v[5] : xs.v[4], x67 = (k & 1) ? xs.v[7] : xs.v[6];
        const float x03 = (k & 2) ? x23 : x01, x47 = (k & 2) ? x67 : x45;
        const float x = (k & 4) ? x47 : x03;
        const float sc = noise_score_inl(x, inv_t, v0 + k, h, Eg, key2);
        if (sc > b.s) b = SlotBest{sc, v0 + k, x};  // ascending k: a strict '>' keeps the lowest index
    }
#else
    for (int k = 0; k < 8; ++k) {
        if ((needm >> k) & 1u) {
            const float sc = noise_score(xs.v[k], inv_t, v0 + k, h, Eg, key2);
            if (sc > b.s) b = SlotBest{sc, v0 + k, xs.v[k]};
        }
    }
#endif
    return b;
}

template <typename T, int MODE, int NT, bool PRIO, bool TIES = false>
__device__ __forceinline__ void sample_unit(
    const T* __restrict__ logits, int64_t ld, int V, int chunk, float inv_t, int use_topk_rt,
    int use_minp_rt, float ln_min_p, uint64_t seed, const int64_t* __restrict__ seq_ids, int64_t step,
    int use_topp_rt, const RowFilter* __restrict__ filt, int32_t* __restrict__ tokens,
    float* __restrict__ logp_out, Part* __restrict__ parts, unsigned* __restrict__ counters, const int row_i,
    const int split, const int nsplit, const int frow, const TieSink* ties = nullptr, Part* result = nullptr) {
    constexpr int NW = NT / kWave;
    SPHASE(0);
    __shared__ Part s_part[NW];
    __shared__ int s_last;
    __shared__ float s_bar;  // best exact score found by any wave of this workgroup
    const int lane = threadIdx.x & (kWave - 1);
    const T* row = logits + (int64_t)row_i * ld;
    const int v_beg = split * chunk;
    const int v_end = max(v_beg, min(V, v_beg + chunk));  // (an empty split contributes the identity)
    const uint32_t key = row_key(seed, seq_ids ? seq_ids[row_i] : (int64_t)row_i, step);  // per (seed, seq, step)
    constexpr bool greedy = MODE == 0;
    const bool use_topk = MODE == 2 && use_topk_rt;
    const bool use_minp = MODE == 2 && use_minp_rt;
    const bool use_topp = MODE == 2 && use_topp_rt;
    const uint32_t tk = use_topk ? filt[frow].tk : 0u;  // frow: this row's filter (row_i, or 0 of a local copy)
    const int ik = use_topk ? filt[frow].ik : 0;
    const float mthr = use_minp ? filt[frow].rmax * inv_t + ln_min_p : 0.f;
    const uint32_t kc = use_topp ? filt[frow].kc : 0u;
    const int ic = use_topp ? filt[frow].ic : 0;
    // the filtered distribution's support (MODE 2): top_k, min_p, top_p
    auto admissible = [&](T rawk, float xk, int v) -> bool {
        bool keep = true;
        const uint32_t kk = okey<T>(rawk);
        if (use_topk) keep = keep && in_cut(kk, v, tk, ik);
        if (use_minp) keep = keep && xk * inv_t >= mthr;
        if (use_topp) keep = keep && in_cut(kk, v, kc, ic);
        return keep;
    };
    if (!greedy) {
        if (threadIdx.x == 0) s_bar = -INFINITY;
        __syncthreads();
    }

    // Per lane: best (score, index) over the elements it visits in ascending index order
    // (so a strict '>' keeps the lowest index on ties) and the raw online (max, sum-exp).
    float best_s = -INFINITY;
    int best_i = 0x7fffffff;
    float best_x = 0.f;  // raw logit of best_i
    const uint32_t key2 = noise_key2(key);  // per-element uniforms (candidates only)
    const uint32_t keyb = noise_keyb(key);  // second-round key of ehash
    // raw online (max, sum-exp) for the sampled token's logprob; finite start so that an
    // all-padding vector never forms inf - inf
    float m = -1e30f, s = 0.f;
    // Noise model (group-of-8 exponential race). Gumbel-max argmax_v (x_v/T - ln E_v) with E_v iid
    // Exp(1) draws the 8 E's of group g = v >> 3 through their order statistics: the minimum
    // E_g = -ln(u_g)/8 ~ Exp(8) sits at slot p, uniform, and the other slots are E_g + e_k with
    // e_k = -ln U_k ~ Exp(1) (memorylessness), so every E_v is exactly Exp(1) and independent. One
    // hash h = ehash(g) per 8 elements gives h16 = h >> 16, u_g = (((h16 ^ 0xffff) << 8) | lo8 |
    // 1) 2^-24 with lo8 = (h >> 8) & 0xff, and p = h & 7; U_k comes from hash32(key2 ^ v phi),
    // evaluated for candidates only.
    // Bound: E_v >= E_g >= 1 - u_g > h16 2^-19, so -ln E_v < ln2 (19 - log2 h16) <= ln2 (146 -
    // bits(float(h16)) 2^-23) (a float's bit pattern is a piecewise-linear lower bound of
    // 2^23 (log2 + 127)). With margin 0.01 (>> the det_ln error) a group can hold an element that
    // beats an exact score `bar` already found in this row only if
    //   xmax/T + 146 ln2 + 0.01 - ln2 2^-23 bits >= bar  <=>  xmax - (T ln2 2^-23) bits >= (bar - C) T,
    // one max over the vector, one fma and one compare per 8 elements. Decisions are unchanged:
    // the filter only skips elements whose exact score is provably below a score already found.
    const float temp = greedy ? 1.f : 1.0f / inv_t;
    const float kT = 0.6931471805599453f * 1.1920928955078125e-7f * temp;
    constexpr float kC = kNoiseC;
    float thr = -INFINITY;   // (bar - C) * T, wave-uniform
    float bar = -INFINITY;   // best exact score known to this wave (wave-uniform)
    bool seeded = greedy;    // first vector: one exact score per lane sets the bar
    constexpr int VEC = 16 / sizeof(T);  // 8 bf16 (one group) or 4 f32 (half a group)

    // E_g of group hash h (the group's smallest Exp(1) draw)
    auto group_e = [&](uint32_t h) -> float { return group_min_e(h); };
    // exact score of element v of the group with hash h and minimum E_g
    auto exact = [&](float xk, int v, uint32_t h, float Eg) -> float { return noise_score(xk, inv_t, v, h, Eg, key2); };
    // Every element of a candidate vector that can still reach the bar through the group bound
    // (the additive form per element; a tie with the bar is evaluated): eval_slots loops over the
    // slots some bound could not rule out (usually one or two per candidate vector).
    auto eval_vec = [&](const float (&x)[VEC], const bool (&ok)[VEC], int v0, uint32_t h) {
        const float bits = (float)(int)__float_as_uint((float)(h >> 16));
        unsigned needm = 0u;
#pragma unroll
        for (int k = 0; k < VEC; ++k)
            if (ok[k] && !(fmaf(bits, -kT, x[k]) - thr < 0.f)) needm |= 1u << k;
        if (!needm) return;
        Slots8 xs;
#pragma unroll
        for (int k = 0; k < 8; ++k) xs.v[k] = k < VEC ? x[k] : 0.f;
        const SlotBest r = eval_slots(xs, needm, v0, h, inv_t, key2, SlotBest{best_s, best_i, best_x});
        best_s = r.s;
        best_i = r.i;
        best_x = r.x;
    };
    // MODE 3 (T == 1) bound in multiplicative form, reusing the lse exponentials ex = e^(x - m):
    // h16 <= 2^19 e^(xmax - bar + 0.01) <=> h16 <= exmax * Q, Q = 2^19 e^(m - bar + 0.01) per lane.
    // While some lane has m - bar > 70 (Q near overflow; an ex that underflowed, x < m - 87,
    // could then still matter) the wave falls back to the additive bits form (qbad). Q is
    // clamped below at FLT_MIN so that an overflowed ex (inf) stays a candidate.
    float Q = 0.f;
    bool qbad = true;
    auto recompute_q = [&]() {
        const float d = m - bar + 0.01f;
        Q = fmaxf(fast_exp2(fmaf(fminf(d, 70.f), kLog2e, 19.0f)), 1.17549435e-38f);
        qbad = __builtin_amdgcn_ballot_w64(!(d <= 70.f)) != 0;
    };
    auto raise_bar = [&]() {  // publish the wave's best, read the workgroup's
        const float wb = wave_max_uniform(best_s);
        if (lane == 0 && wb > -INFINITY)
            __hip_atomic_fetch_max(&s_bar, wb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const float sb = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s_bar)));
        bar = fmaxf(wb, sb);
        thr = (bar - kC) * temp;
        if constexpr (MODE == 3) recompute_q();
    };
    // adopt the workgroup's bar (after the seeding barrier; a per-iteration refresh measured slower:
    // the LDS round trip stalls every wave at the same point of its iteration)
    auto refresh_bar = [&]() {
        const float sb = __int_as_float(__builtin_amdgcn_readfirstlane(
            __float_as_int(__hip_atomic_load(&s_bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))));
        if (sb > bar) {
            bar = sb;
            thr = (bar - kC) * temp;
            if constexpr (MODE == 3) recompute_q();
        }
    };
    // after a candidate vector: publish the wave's best and read the workgroup's when some lane
    // improved on the bar, else only read the workgroup's (the wave max and the LDS max skipped:
    // 512 / 128 / 64 rows at T = 1 33.28 / 17.78 / 14.22 vs 34.44 / 18.59 / 14.80 us, same tokens;
    // profiles/r05_sampler_eval_form_ab.json, form 1)
    auto after_eval = [&]() {
        if (__builtin_amdgcn_ballot_w64(best_s > bar) != 0) raise_bar();
        else refresh_bar();
    };
    // additive bound test of a vector whose largest admissible logit is xm
    auto cand_add = [&](float xm, uint32_t h) -> bool {
        const float bits = (float)(int)__float_as_uint((float)(h >> 16));
        return !(fmaf(bits, -kT, xm) - thr < 0.f);
    };
    // once per wave, before any filtering: the exact score of each lane's largest admissible
    // element of its first vector sets the bar (one exact evaluation per lane instead of VEC)
    auto seed_vec = [&](const float (&x)[VEC], const bool (&ok)[VEC], int v0, uint32_t h) {
        seeded = true;
        float xb = -INFINITY;
        int kb = -1;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            if (ok[k] && x[k] > xb) {
                xb = x[k];
                kb = k;
            }
        }
        if (kb >= 0) {
            Slots8 xs;
#pragma unroll
            for (int k = 0; k < 8; ++k) xs.v[k] = k < VEC ? x[k] : 0.f;
            const SlotBest r = eval_slots(xs, 1u << kb, v0, h, inv_t, key2, SlotBest{best_s, best_i, best_x});
            best_s = r.s;
            best_i = r.i;
            best_x = r.x;
        }
        raise_bar();
    };
    // lse of the raw logits over one vector (not on the decision path); leaves exp(x - mn) in ex
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    auto lse_vec = [&](const float (&x)[VEC], float vmax, float (&ex)[VEC]) -> float {
        const float mn = fmaxf(m, vmax);
        s *= fast_exp2((m - mn) * kLog2e);
        const f32x2 c2 = {-mn * kLog2e, -mn * kLog2e};
        const f32x2 l2 = {kLog2e, kLog2e};
        f32x2 acc = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k < VEC; k += 2) {
            const f32x2 xv = {x[k], x[k + 1]};
            const f32x2 y = __builtin_elementwise_fma(xv, l2, c2);
            ex[k] = fast_exp2(y.x);
            ex[k + 1] = fast_exp2(y.y);
            const f32x2 e2 = {ex[k], ex[k + 1]};
            acc += e2;
        }
        s += acc.x + acc.y;
        m = mn;
        return mn;
    };
    // One vector of VEC elements starting at v0 (v0 % VEC == 0, so inside one group); cnt < VEC
    // only on the ragged tail (FULL = false).
    auto visit_vec = [&](const T (&raw)[VEC], int v0, int cnt, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        float x[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = (FULL || k < cnt) ? to_f<T>(raw[k]) : -INFINITY;
        float vmax = x[0];
#pragma unroll
        for (int k = 1; k < VEC; ++k) vmax = fmaxf(vmax, x[k]);
        float ex[VEC];
        lse_vec(x, vmax, ex);
        if constexpr (greedy) {
            if (vmax > best_s) {  // first index of the new maximum (ascending visit order)
                int kk = VEC - 1;
#pragma unroll
                for (int k = VEC - 2; k >= 0; --k) kk = (x[k] == vmax) ? k : kk;
                best_s = vmax;
                best_i = v0 + kk;
                best_x = vmax;
            }
            return;
        }
        bool ok[VEC];
        float xm = -INFINITY;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            ok[k] = FULL || k < cnt;
            if constexpr (MODE == 2) ok[k] = ok[k] && admissible(raw[k], x[k], v0 + k);
            xm = fmaxf(xm, ok[k] ? x[k] : -INFINITY);
        }
        const uint32_t h = ehash(key, keyb, (uint32_t)v0 >> 3);
        if constexpr (TIES) {  // the cut key's elements: exact scores into the caller's list
            bool tie[VEC];
            bool anyt = false;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                tie[k] = (FULL || k < cnt) && okey<T>(raw[k]) == ties->kc;
                anyt = anyt || tie[k];
            }
            if (__builtin_amdgcn_ballot_w64(anyt) != 0 && anyt) {
                const float Eg = group_e(h);
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    if (tie[k]) {
                        const uint32_t pos = atomicAdd(ties->n, 1u);
                        if (pos < (uint32_t)ties->cap) {
                            ties->idx[pos] = v0 + k;
                            ties->sc[pos] = exact(x[k], v0 + k, h, Eg);
                        }
                    }
                }
            }
        }
        if constexpr (!FULL) {
            if (!seeded) seed_vec(x, ok, v0, h);
        }
        const bool cand = xm > -INFINITY && cand_add(xm, h);
        if (__builtin_amdgcn_ballot_w64(cand) == 0) return;  // wave-uniform: rare once the bar is up
        if (cand) eval_vec(x, ok, v0, h);
        after_eval();
    };
    // MODE 3 full vector, lagged lse offset m (exps accumulate into acc2; the caller checks
    // for overflow once per iteration)
    auto visit3 = [&](const uint4& dw4, int v0, f32x2& acc2) {
        T raw[VEC];
        __builtin_memcpy(raw, &dw4, 16);
        float x[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = to_f<T>(raw[k]);
        const f32x2 l2 = {kLog2e, kLog2e};
        const f32x2 c2 = {-m * kLog2e, -m * kLog2e};
        float ex[VEC];
#pragma unroll
        for (int k = 0; k < VEC; k += 2) {
            const f32x2 xv = {x[k], x[k + 1]};
            const f32x2 y = __builtin_elementwise_fma(xv, l2, c2);
            ex[k] = fast_exp2(y.x);
            ex[k + 1] = fast_exp2(y.y);
            acc2 += f32x2{ex[k], ex[k + 1]};
        }
#ifdef SKYRL_SV_NOHASH  // scripts/probe/sampler_variants only: timing, not correct tokens
        const uint32_t h = 0x80000000u ^ (uint32_t)v0;
#else
        const uint32_t h = ehash(key, keyb, (uint32_t)v0 >> 3);
#endif
        bool cand;
        if (!qbad) {
            float em = fmaxf(fmaxf(ex[0], ex[1]), ex[2]);
#pragma unroll
            for (int k = 3; k + 1 < VEC; k += 2) em = fmaxf(fmaxf(em, ex[k]), ex[k + 1]);
            if constexpr (VEC % 2 == 0) em = fmaxf(em, ex[VEC - 1]);
            cand = fmaf(em, Q, -(float)(h >> 16)) >= 0.f;
        } else {
            float xm = x[0];
#pragma unroll
            for (int k = 1; k < VEC; ++k) xm = fmaxf(xm, x[k]);
            cand = cand_add(xm, h);
        }
#ifdef SKYRL_SV_NOCAND
        cand = false;
#endif
#if defined(SKYRL_SV_NOCAND_LIVE) && SKYRL_SV_NOCAND_LIVE  // probe: the bound test computed, nothing evaluated
        asm volatile("" ::"v"((int)cand));
        cand = false;
#endif
        if (__builtin_amdgcn_ballot_w64(cand) == 0) return;
        if (cand) {
            bool ok[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) ok[k] = true;
            eval_vec(x, ok, v0, h);
        }
        after_eval();
    };
    // lse of one iteration redone with a fresh offset after an overflow of the lagged one
    auto lse_refresh = [&](const uint4 (&dw)[4]) {
        float mx = m;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            T raw[VEC];
            __builtin_memcpy(raw, &dw[u], 16);
#pragma unroll
            for (int k = 0; k < VEC; ++k) mx = fmaxf(mx, to_f<T>(raw[k]));
        }
        s *= fast_exp2((m - mx) * kLog2e);
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            T raw[VEC];
            __builtin_memcpy(raw, &dw[u], 16);
#pragma unroll
            for (int k = 0; k < VEC; ++k) acc += fast_exp2((to_f<T>(raw[k]) - mx) * kLog2e);
        }
        s += acc;
        m = mx;
    };
    const std::integral_constant<bool, true> kFull{};
    const std::integral_constant<bool, false> kPart{};
    const bool vec_ok = (reinterpret_cast<uintptr_t>(row + v_beg) % 16) == 0;
    int v0 = v_beg;
    if (vec_ok) {
        const int nvec = (v_end - v_beg) / VEC;
        const uint4* rv = reinterpret_cast<const uint4*>(row + v_beg);
        constexpr int kStep = 4 * NT;  // 4 x 16 B per lane per iteration
        const int nfull = (nvec / kStep) * kStep;
        // full iterations, software-pipelined: the next iteration's loads are issued before the
        // current one is processed
        uint4 cur[4], nxt[4];
        if (nfull > 0) {
#pragma unroll
            for (int u = 0; u < 4; ++u) cur[u] = ld_stream(rv + u * NT + threadIdx.x);
            // Drain the first iteration's loads here. Otherwise the loop header merges "cur
            // pending" (this path) with "cur in registers" (the back edge), and the waitcnt pass
            // puts vmcnt(2)/(1)/(0) before cur[1..3] in EVERY iteration: those counts then wait for
            // the next iteration's prefetch, and the last vector is processed with nothing in flight.
            __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
            if constexpr (!greedy) {  // seed from this lane's first two vectors
                float x[2][VEC];
                bool ok[2][VEC];
                float xb[2] = {-INFINITY, -INFINITY};
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    T vals[VEC];
                    __builtin_memcpy(vals, &cur[u], 16);
                    const int v0s = v_beg + (u * NT + threadIdx.x) * VEC;
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        x[u][k] = to_f<T>(vals[k]);
                        ok[u][k] = true;
                        if constexpr (MODE == 2) ok[u][k] = admissible(vals[k], x[u][k], v0s + k);
                        xb[u] = fmaxf(xb[u], ok[u][k] ? x[u][k] : -INFINITY);
                    }
                }
                if constexpr (MODE == 3) m = fmaxf(xb[0], xb[1]);  // lagged lse offset: this lane's first max
                const bool us = xb[1] > xb[0];
                float xs[VEC];
                bool oks[VEC];
#pragma unroll
                for (int k = 0; k < VEC; ++k) {  // selects, not a dynamically indexed array (scratch)
                    xs[k] = us ? x[1][k] : x[0][k];
                    oks[k] = us ? ok[1][k] : ok[0][k];
                }
                const int v0s = v_beg + ((us ? NT : 0) + threadIdx.x) * VEC;
                seed_vec(xs, oks, v0s, ehash(key, keyb, (uint32_t)v0s >> 3));
                // every wave starts from the best of the workgroup's 2 x NT seeds
                __syncthreads();
                refresh_bar();
            }
            SPHASE(1);
        }
        for (int base = 0; base < nfull; base += kStep) {
            const bool more = base + kStep < nfull;
            if constexpr (PRIO) {
                switch (((nfull - base) * 4 - 1) / nfull) {  // quarter of the row still ahead
                    case 3: __builtin_amdgcn_s_setprio(3); break;
                    case 2: __builtin_amdgcn_s_setprio(2); break;
                    case 1: __builtin_amdgcn_s_setprio(1); break;
                    default: __builtin_amdgcn_s_setprio(0); break;
                }
            }
            if (more) {
#pragma unroll
                for (int u = 0; u < 4; ++u) nxt[u] = ld_stream(rv + base + kStep + u * NT + threadIdx.x);
            }
            if constexpr (MODE == 3) {
                f32x2 acc2 = {0.f, 0.f};
#pragma unroll
                for (int u = 0; u < 4; ++u) visit3(cur[u], v_beg + (base + u * NT + threadIdx.x) * VEC, acc2);
                const float acc = acc2.x + acc2.y;
                const bool ovf = !(acc < 1e30f);  // a value far above the lagged offset m
                if (ovf) lse_refresh(cur);
                else s += acc;
                if (__builtin_amdgcn_ballot_w64(ovf) != 0) recompute_q();
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    T vals[VEC];
                    __builtin_memcpy(vals, &cur[u], 16);
                    visit_vec(vals, v_beg + (base + u * NT + threadIdx.x) * VEC, VEC, kFull);
                }
            }
            if (more) {
#pragma unroll
                for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
            }
        }
        // the partial iteration: same trip count in every thread (out-of-range slots are -inf
        // padding with cnt = 0), so the wave-wide max inside visit_vec never reads an inactive lane
        if (nfull < nvec) {
            uint4 pk[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = nfull + u * NT + threadIdx.x;
                pk[u] = i < nvec ? ld_stream(rv + i) : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = nfull + u * NT + threadIdx.x;
                T vals[VEC];
                __builtin_memcpy(vals, &pk[u], 16);
                visit_vec(vals, v_beg + i * VEC, i < nvec ? VEC : 0, kPart);
            }
        }
        v0 = v_beg + nvec * VEC;
    }
    // unaligned rows or the ragged tail: VEC-element groups, the last one partial
    for (int gb = v0; gb < v_end; gb += NT * VEC) {
        const int g0 = gb + threadIdx.x * VEC;
        const int cnt = max(0, min(VEC, v_end - g0));
        T vals[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) vals[k] = k < cnt ? row[g0 + k] : row[v_beg];
        visit_vec(vals, g0, cnt, kPart);
    }
    SPHASE(2);

    // wave fold on DPP: best (score desc, idx asc) with its raw logit, and (m, s)
    const Part wp = wave_reduce_part(Part{best_s, best_i, m, s, best_x});
    if (lane == 0) s_part[threadIdx.x / kWave] = wp;
    __syncthreads();
    SPHASE(3);
    Part p;
    if (threadIdx.x == 0) {
        p = s_part[0];
        for (int j = 1; j < NW; ++j) part_merge(p, s_part[j]);
    }
    if (nsplit > 1) {
        // Hand-off without an acquire (MI355X_MICROARCH.md, the valid sc1 form: one lane stores
        // the whole record write-through, drains, adds to the row's counter; the workgroup whose
        // add returned last reads every record with sc1 loads after the barrier its adding wave
        // joins): the last split's wave 0 loads the nsplit records in parallel, one per lane,
        // and folds them on DPP in a fixed tree.
        if (threadIdx.x == 0) {
            float* dst = reinterpret_cast<float*>(parts + (int64_t)row_i * nsplit + split);
            st_wt(dst + 0, p.score);
            st_wt(reinterpret_cast<int*>(dst) + 1, p.idx);
            st_wt(dst + 2, p.m);
            st_wt(dst + 3, p.s);
            st_wt(dst + 4, p.xb);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned prev = __hip_atomic_fetch_add(counters + row_i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = prev == (unsigned)nsplit - 1u;
            SPHASE(5);
        }
        __syncthreads();
        if (!s_last || threadIdx.x >= kWave) return;
        handoff_acquire();
        Part q{-INFINITY, 0x7fffffff, -1e30f, 0.f, 0.f};  // identity for lanes past nsplit
        if (lane < nsplit) {
            const float* src = reinterpret_cast<const float*>(parts + (int64_t)row_i * nsplit + lane);
            q.score = __hip_atomic_load(src + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            q.idx = __hip_atomic_load(reinterpret_cast<const int*>(src) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            q.m = __hip_atomic_load(src + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            q.s = __hip_atomic_load(src + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            q.xb = __hip_atomic_load(src + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        p = wave_reduce_part(q);
    }
    if (result) {  // the caller decides (the top_p kernel: ties at the cut still to rank)
        if (threadIdx.x == 0) *result = p;
        return;
    }
    if (threadIdx.x == 0) {
        SPHASE(4);
        tokens[row_i] = p.idx;
        if (logp_out) {
            const float lse = p.m + fast_log2(p.s) * kLn2;
            logp_out[row_i] = (p.idx >= 0 && p.idx < V) ? p.xb - lse : __builtin_nanf("");
        }
        if (nsplit > 1) rearm(counters + row_i);
    }
}

#define SKYRL_SAMPLE_ARGS                                                                                     \
    const T *__restrict__ logits, int64_t ld, int V, int chunk, float inv_t, int use_topk_rt, int use_minp_rt, \
        float ln_min_p, uint64_t seed, const int64_t *__restrict__ seq_ids, int64_t step, int use_topp_rt,     \
        const RowFilter *__restrict__ filt, int32_t *__restrict__ tokens, float *__restrict__ logp_out,         \
        Part *__restrict__ parts, unsigned *__restrict__ counters
#define SKYRL_SAMPLE_PASS                                                                                   \
    logits, ld, V, chunk, inv_t, use_topk_rt, use_minp_rt, ln_min_p, seed, seq_ids, step, use_topp_rt, filt, \
        tokens, logp_out, parts, counters

// Static grid: block (row, split).
#ifndef SKYRL_SPLIT_WPE  // waves per SIMD the split (256-thread) instances are built for; probe builds vary it
#define SKYRL_SPLIT_WPE 4
#endif
template <typename T, int MODE, int NT, bool PRIO = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 ? SKYRL_SPLIT_WPE : 4))) void sample_kernel(SKYRL_SAMPLE_ARGS) {
    sample_unit<T, MODE, NT, PRIO>(SKYRL_SAMPLE_PASS, blockIdx.x, blockIdx.y, gridDim.y, blockIdx.x);
}

// ---- top_k fast path: the whole filtered decision in one pass over the row ------------------
// With top_k set (k <= kFastK) every filter and the decision live in the row's k largest logits.
// One 512-thread workgroup per row streams the row ONCE:
//   * B: with the row's first 4 NT vectors in registers (the next 4 NT in flight), the k-th
//     largest of the threads' maxima over them (4-bit radix select by wave ballots). At least k
//     elements are >= B, so all of the row's top k are.
//   * The pass: the raw online (max, sum-exp) for the logprob, and every element >= B appended
//     to an LDS candidate list (about k V / (4 NT VEC) elements: 464 at k = 50, V = 151,936).
//   * On chip: the k-th largest candidate key (a 256-bin histogram of kmax - key, or a radix
//     select by wave ballots when the candidates span more keys); the candidates at or
//     above it ranked in the exact (key desc, index asc) order; top_k = rank < k; min_p = x/T >=
//     max/T + ln min_p; top_p = the fixed-point masses (mass_q) summed exactly in rank order,
//     kept while the mass before is < p Z (rank 0 always); the Gumbel-max decision over the
//     admissible elements (noise_score, lowest index on ties).
// These are the pre-pass's cut rules and MODE 2's exact scores on the same elements, so tokens
// are those of the two-kernel path (and of oracle/sampler_ref.c) bit for bit. A row whose lists
// overflow (tie-heavy rows, mostly -inf rows) runs the two-kernel path's code in this workgroup
// (filter_row with 512 threads, then sample_unit MODE 2 on the row).
constexpr int kFastNT = 512;
constexpr int kFastK = 128;      // largest top_k served here
constexpr int kFastCap = 4096;   // candidates >= B
constexpr int kFastCap2 = 512;   // candidates at or above the k-th largest key
constexpr int32_t kRowDone = -2;      // RowFilter.ik markers (for tests): the row was decided by the fast path,
constexpr int32_t kRowFallback = -3;  // or by its in-kernel fallback (the pre-pass's cuts + MODE 2)

template <typename T>
__device__ __attribute__((noinline)) void topk_fallback(const T* __restrict__ logits, int64_t ld, int V, int top_k,
                                                        float inv_t, int use_minp, float ln_min_p, int use_topp,
                                                        float top_p, uint64_t seed, const int64_t* __restrict__ seq_ids,
                                                        int64_t step, int32_t* __restrict__ tokens,
                                                        float* __restrict__ logp_out, RowFilter* rf, int row_i) {
    filter_row<T, kFastNT>(logits, ld, V, top_k, use_minp, inv_t, ln_min_p, use_topp ? top_p : 1.0f, rf, row_i);
    __syncthreads();
    sample_unit<T, 2, kFastNT, false>(logits, ld, V, V, inv_t, 1, use_minp, ln_min_p, seed, seq_ids, step, use_topp, rf,
                                      tokens, logp_out, nullptr, nullptr, row_i, 0, 1, 0);
}

template <typename T>
__global__ __launch_bounds__(kFastNT) __attribute__((amdgpu_waves_per_eu(4))) void sample_topk_kernel(const T* __restrict__ logits, int64_t ld, int V, int top_k,
                                                              float inv_t, int use_minp, float ln_min_p, int use_topp,
                                                              float top_p, uint64_t seed,
                                                              const int64_t* __restrict__ seq_ids, int64_t step,
                                                              int32_t* __restrict__ tokens, float* __restrict__ logp_out,
                                                              RowFilter* __restrict__ filt) {
    constexpr int NT = kFastNT, NW = NT / kWave, VEC = 16 / sizeof(T), KB = sizeof(T) * 8;
    constexpr uint32_t KTOP = KB == 16 ? 0xffffu : 0xffffffffu;  // d = KTOP - key: smallest d = largest key
    __shared__ float s_m[NW], s_s[NW];
    __shared__ uint32_t s_kmax[NW];
    __shared__ uint32_t s_rc[2][NW][16];
    __shared__ uint32_t s_ckey[kFastCap];
    __shared__ int32_t s_cidx[kFastCap];
    __shared__ __attribute__((aligned(16))) uint32_t s_fkey[kFastCap2];
    __shared__ __attribute__((aligned(16))) int32_t s_fidx[kFastCap2];
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[256];
    __shared__ uint32_t s_sel;
    __shared__ int32_t s_frank[kFastCap2];
    __shared__ uint32_t s_mass[kFastK];
    __shared__ unsigned long long s_before[kFastK];
    __shared__ unsigned long long s_wsum[NW];
    __shared__ uint32_t s_cc, s_fc;
    __shared__ float s_bs[NW];
    __shared__ int32_t s_bi[NW];
    __shared__ RowFilter s_rf;
    const int row_i = blockIdx.x;
    SPHASE(0);
    // a row the candidate lists cannot settle: the pre-pass's cuts and the MODE 2 decision, here
    // (a call, not inlined: its registers would otherwise crowd the streaming loop)
    auto fallback = [&]() {
        topk_fallback<T>(logits, ld, V, top_k, inv_t, use_minp, ln_min_p, use_topp, top_p, seed, seq_ids, step, tokens,
                         logp_out, &s_rf, row_i);
        if (threadIdx.x == 0) filt[row_i].ik = kRowFallback;
    };
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const T* row = logits + (int64_t)row_i * ld;
    if (threadIdx.x == 0) {
        s_cc = 0u;
        s_fc = 0u;
    }
    if (threadIdx.x < 256) s_hist[threadIdx.x] = 0u;

    // ---- prologue: the first 4 NT vectors (the next 4 NT in flight) and their per-thread max
    const uint4* rv = reinterpret_cast<const uint4*>(row);  // 16-B aligned (host check)
    const int nvec = V / VEC;
    constexpr int kStep = 4 * NT;
    const int nfull = (nvec / kStep) * kStep;
    uint4 cur[4], nxt[4];
    if (nfull > 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = ld_stream(rv + u * NT + threadIdx.x);
        if (kStep < nfull) {
#pragma unroll
            for (int u = 0; u < 4; ++u) nxt[u] = ld_stream(rv + kStep + u * NT + threadIdx.x);
        }
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = u * NT + threadIdx.x;
            cur[u] = i < nvec ? ld_stream(rv + i) : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    uint32_t km0 = 0u;
    bool has0 = false;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (u * NT + (int)threadIdx.x < nvec) {
            has0 = true;
            T raw[VEC];
            __builtin_memcpy(raw, &cur[u], 16);
#pragma unroll
            for (int k = 0; k < VEC; ++k) km0 = max(km0, okey<T>(raw[k]));
        }
    }
    // the k-th smallest d among the wave counts' 256 histogram bins (wave 0; s_sel = d, or
    // 0xffffffff when the k-th is beyond the bins)
    auto hist_pick = [&](uint32_t k) {
        if (w == 0) {
            const uint4 hb = reinterpret_cast<const uint4*>(s_hist)[lane];  // bins 4 lane .. 4 lane + 3
            const uint32_t tot = hb.x + hb.y + hb.z + hb.w;
            uint32_t incl = tot;
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const uint32_t o = (uint32_t)__shfl_up((int)incl, off, kWave);
                if (lane >= off) incl += o;
            }
            const uint64_t hit = __builtin_amdgcn_ballot_w64(incl >= k);
            if (!hit) {
                if (lane == 0) s_sel = 0xffffffffu;
            } else if (lane == __builtin_ctzll(hit)) {
                uint32_t cum = incl - tot, d = 4u * lane;
                if (cum + hb.x < k) {
                    cum += hb.x;
                    ++d;
                    if (cum + hb.y < k) {
                        cum += hb.y;
                        ++d;
                        if (cum + hb.z < k) ++d;
                    }
                }
                s_sel = d;
            }
        }
    };
    // B = the k-th largest of km0 over the threads that hold a vector: a 256-bin histogram of
    // kmax0 - km0 (the last bin saturates), or a radix select by wave ballots when the k-th
    // lands in the saturated bin. Fewer than k threads holding a vector: no bound.
    uint32_t kw = has0 ? km0 : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) kw = max(kw, (uint32_t)__shfl_xor((int)kw, off, kWave));
    if (lane == 0) s_kmax[w] = kw;
    const int n_ne = __syncthreads_count(has0);
    uint32_t kmax0 = s_kmax[0];
#pragma unroll
    for (int j = 1; j < NW; ++j) kmax0 = max(kmax0, s_kmax[j]);
    uint32_t bkey = 0u;
    if (n_ne >= top_k) {
        if (has0) atomicAdd(&s_hist[min(kmax0 - km0, 255u)], 1u);
        __syncthreads();
        hist_pick((uint32_t)top_k);
        __syncthreads();
        const uint32_t dsel = s_sel;
        if (threadIdx.x < 256) s_hist[threadIdx.x] = 0u;  // again for the candidates (barriers between)
        if (dsel < 255u) {
            bkey = kmax0 - dsel;
        } else {
            const uint32_t d0 = has0 ? KTOP - km0 : 0xffffffffu;
            uint32_t P = 0u;
            int below = 0;
#pragma unroll
            for (int st = 0; st < KB / 4; ++st) {
                const int sh = KB - 4 * (st + 1);
                const bool match = st == 0 ? (KB == 32 ? has0 : d0 <= 0xffffu) : ((d0 >> (sh + 4)) == P);
                const uint32_t dig = (d0 >> sh) & 15u;
                uint32_t mine = 0u;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const uint32_t c = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(match && dig == (uint32_t)q));
                    if (lane == q) mine = c;
                }
                if (lane < 16) s_rc[st & 1][w][lane] = mine;
                __syncthreads();
                uint32_t tq = 0u;  // lane q: the workgroup's count of digit q
                if (lane < 16) {
#pragma unroll
                    for (int j = 0; j < NW; ++j) tq += s_rc[st & 1][j][lane];
                }
                uint32_t incl = tq;
#pragma unroll
                for (int off = 1; off < 16; off <<= 1) {
                    const uint32_t o = (uint32_t)__shfl_up((int)incl, off, kWave);
                    if (lane >= off) incl += o;
                }
                const uint64_t hit = __builtin_amdgcn_ballot_w64(lane < 16 && below + (int)incl >= top_k);
                const int q = hit ? __builtin_ctzll(hit) : 15;
                below += (int)__shfl((int)(incl - tq), q, kWave);
                P = (P << 4) | (uint32_t)q;
            }
            bkey = KTOP - P;
        }
    }
    const float bf = n_ne < top_k ? -INFINITY : from_key<T>(bkey);
    SPHASE(1);

    // ---- the pass: lse of the raw logits; every element >= B into the candidate list
    float m = has0 ? fmaxf(from_key<T>(km0), -1e30f) : -1e30f, s = 0.f;
    uint32_t kmx = 0u;
    auto append = [&](uint32_t kk, int idx) {
        const uint32_t pos = atomicAdd(&s_cc, 1u);
        if (pos < (uint32_t)kFastCap) {
            s_ckey[pos] = kk;
            s_cidx[pos] = idx;
        }
        kmx = max(kmx, kk);
    };
    auto visit = [&](const uint4& pk, int v0) {
        T raw[VEC];
        __builtin_memcpy(raw, &pk, 16);
        float x[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = to_f<T>(raw[k]);
        float vmax = x[0];
#pragma unroll
        for (int k = 1; k < VEC; ++k) vmax = fmaxf(vmax, x[k]);
        // lagged lse offset (the thread's prologue max): rescaled only when a value rises 64
        // above it, so the exponentials of one vector never overflow
        if (vmax > m + 64.f) {
            s *= fast_exp2((m - vmax) * kLog2e);
            m = vmax;
        }
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc += fast_exp2((x[k] - m) * kLog2e);
        s += acc;
        if (vmax >= bf) {  // a float compare admits every key >= key(B) (-0 beside +0 as well)
#pragma unroll
            for (int k = 0; k < VEC; ++k)
                if (x[k] >= bf) append(okey<T>(raw[k]), v0 + k);
        }
    };
    if (nfull > 0) {
        for (int base = 0; base < nfull; base += kStep) {
            const bool more = base + kStep < nfull;
            switch (((nfull - base) * 4 - 1) / nfull) {  // progress priority, as the row-mode sampler
                case 3: __builtin_amdgcn_s_setprio(3); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                default: __builtin_amdgcn_s_setprio(0); break;
            }
            if (more && base > 0) {
#pragma unroll
                for (int u = 0; u < 4; ++u) nxt[u] = ld_stream(rv + base + kStep + u * NT + threadIdx.x);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) visit(cur[u], (base + u * NT + threadIdx.x) * VEC);
            if (more) {
#pragma unroll
                for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
            }
        }
        for (int i = nfull + threadIdx.x; i < nvec; i += NT) visit(ld_stream(rv + i), i * VEC);
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (u * NT + (int)threadIdx.x < nvec) visit(cur[u], (u * NT + threadIdx.x) * VEC);
    }
    for (int i = nvec * VEC + threadIdx.x; i < V; i += NT) {  // ragged tail, one element per thread
        const float x = to_f<T>(row[i]);
        const float mn = fmaxf(m, x);
        s = s * fast_exp2((m - mn) * kLog2e) + fast_exp2((x - mn) * kLog2e);
        m = mn;
        if (x >= bf) append(okey<T>(row[i]), i);
    }

    SPHASE(2);
    // ---- row lse and max key (the max element is a candidate)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float om = __shfl_xor(m, off, kWave);
        const float os = __shfl_xor(s, off, kWave);
        const float mn = fmaxf(m, om);
        s = s * fast_exp2((m - mn) * kLog2e) + os * fast_exp2((om - mn) * kLog2e);
        m = mn;
        kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, off, kWave));
    }
    if (lane == 0) {
        s_m[w] = m;
        s_s[w] = s;
        s_kmax[w] = kmx;
    }
    __syncthreads();
    float M = s_m[0], S = s_s[0];
    uint32_t kmax = s_kmax[0];
#pragma unroll
    for (int j = 1; j < NW; ++j) {
        const float mn = fmaxf(M, s_m[j]);
        S = S * fast_exp2((M - mn) * kLog2e) + s_s[j] * fast_exp2((s_m[j] - mn) * kLog2e);
        M = mn;
        kmax = max(kmax, s_kmax[j]);
    }
    SPHASE(5);
    const float lse = M + fast_log2(S) * kLn2;
    const float mx = from_key<T>(kmax);
    const int C = (int)s_cc;
    if (C > kFastCap || C < top_k) {
        fallback();
        return;
    }

    // ---- the k-th largest candidate key. Candidates lie within kmax - key(B) of the max: when
    //      that span is under 256 keys (bf16 rows: usually), one histogram of d = kmax - key and
    //      a scan by one wave; otherwise a radix select by wave ballots over rounds of NT
    //      candidates (per-wave digit counts summed through LDS)
    const int rounds = (C + NT - 1) / NT;
    uint32_t tkey;
    if (n_ne >= top_k && kmax - bkey < 256u) {
        for (int i = threadIdx.x; i < C; i += NT) {
            // a -0 admitted beside a bound of +0 lies one key below it: never in the top k
            const uint32_t dd = kmax - s_ckey[i];
            if (dd < 256u) atomicAdd(&s_hist[dd], 1u);
        }
        __syncthreads();
        hist_pick((uint32_t)top_k);
        __syncthreads();
        tkey = kmax - s_sel;
    } else {
    uint32_t Pc = 0u;
    int above = 0;
#pragma unroll
    for (int st = 0; st < KB / 4; ++st) {
        const int sh = KB - 4 * (st + 1);
        uint32_t mine = 0u;
        for (int rd = 0; rd < rounds; ++rd) {
            const int i = rd * NT + threadIdx.x;
            const uint32_t d = i < C ? KTOP - s_ckey[i] : 0u;
            const bool match = i < C && (st == 0 || (d >> (sh + 4)) == Pc);
            const uint32_t dig = (d >> sh) & 15u;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint32_t c = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(match && dig == (uint32_t)q));
                if (lane == q) mine += c;
            }
        }
        if (lane < 16) s_rc[st & 1][w][lane] = mine;
        __syncthreads();
        uint32_t tq = 0u;
        if (lane < 16) {
#pragma unroll
            for (int j = 0; j < NW; ++j) tq += s_rc[st & 1][j][lane];
        }
        uint32_t incl = tq;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)incl, off, kWave);
            if (lane >= off) incl += o;
        }
        const uint64_t hit = __builtin_amdgcn_ballot_w64(lane < 16 && above + (int)incl >= top_k);
        const int q = hit ? __builtin_ctzll(hit) : 15;
        above += (int)__shfl((int)(incl - tq), q, kWave);
        Pc = (Pc << 4) | (uint32_t)q;
    }
    tkey = KTOP - Pc;  // the k-th largest key; `above` candidates are larger
    }
    SPHASE(3);

    // ---- candidates at or above it (ballot compaction, one LDS atomic per wave and round),
    //      ranked in (key desc, index asc) order
    for (int rd = 0; rd < rounds; ++rd) {
        const int i = rd * NT + threadIdx.x;
        const uint32_t kk = i < C ? s_ckey[i] : 0u;
        const bool keep = i < C && kk >= tkey;
        const uint64_t bal = __builtin_amdgcn_ballot_w64(keep);
        uint32_t wbase = 0u;
        if (lane == 0 && bal) wbase = atomicAdd(&s_fc, (uint32_t)__builtin_popcountll(bal));
        wbase = (uint32_t)__shfl((int)wbase, 0, kWave);
        if (keep) {
            const uint32_t pos = wbase + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
            if (pos < (uint32_t)kFastCap2) {
                s_fkey[pos] = kk;
                s_fidx[pos] = s_cidx[i];
            }
        }
    }
    for (int r = threadIdx.x; r < top_k; r += NT) s_mass[r] = 0u;
    __syncthreads();
    const int F = (int)s_fc;
    if (F > kFastCap2 - 4) {  // a tie group too large for the exact ranking here
        fallback();
        return;
    }
    // pad to whole 16-B groups with entries that precede nothing (key 0, the last index)
    const int F4 = (F + 3) & ~3;
    if ((int)threadIdx.x < F4 - F) {
        s_fkey[F + threadIdx.x] = 0u;
        s_fidx[F + threadIdx.x] = 0x7fffffff;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < F; i += NT) {
        const uint32_t ki = s_fkey[i];
        const int ii = s_fidx[i];
        int r = 0;
        for (int j = 0; j < F4 / 4; ++j) {
            const uint4 kq = reinterpret_cast<const uint4*>(s_fkey)[j];
            const int4 iq = reinterpret_cast<const int4*>(s_fidx)[j];
            r += (kq.x > ki || (kq.x == ki && iq.x < ii)) ? 1 : 0;
            r += (kq.y > ki || (kq.y == ki && iq.y < ii)) ? 1 : 0;
            r += (kq.z > ki || (kq.z == ki && iq.z < ii)) ? 1 : 0;
            r += (kq.w > ki || (kq.w == ki && iq.w < ii)) ? 1 : 0;
        }
        s_frank[i] = r;
    }
    __syncthreads();

    // ---- filters on the ranked candidates
    const float mthr = mx * inv_t + ln_min_p;
    unsigned long long Z = 0ull;
    if (use_topp) {
        for (int i = threadIdx.x; i < F; i += NT) {
            const int r = s_frank[i];
            if (r < top_k) {
                const float x = from_key<T>(s_fkey[i]);
                if (!use_minp || x * inv_t >= mthr) s_mass[r] = mass_q(x, mx, inv_t);
            }
        }
        __syncthreads();
        // exclusive scan of the masses in rank order (ranks < k <= NT: one per thread)
        const unsigned long long mine = (int)threadIdx.x < top_k ? (unsigned long long)s_mass[threadIdx.x] : 0ull;
        unsigned long long incl = mine;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const unsigned long long o = (unsigned long long)__shfl_up((long long)incl, off, kWave);
            if (lane >= off) incl += o;
        }
        if (lane == kWave - 1) s_wsum[w] = incl;
        __syncthreads();
        unsigned long long off_w = 0ull;
        for (int j = 0; j < NW; ++j) {
            if (j < w) off_w += s_wsum[j];
            Z += s_wsum[j];
        }
        if ((int)threadIdx.x < top_k) s_before[threadIdx.x] = off_w + incl - mine;
        __syncthreads();
    }
    const double target = (double)top_p * (double)Z;
    const uint32_t key = row_key(seed, seq_ids ? seq_ids[row_i] : (int64_t)row_i, step);
    const uint32_t key2 = noise_key2(key), keyb = noise_keyb(key);
    Best best{-INFINITY, 0x7fffffff};
    for (int i = threadIdx.x; i < F; i += NT) {
        const int r = s_frank[i];
        if (r >= top_k) continue;
        const float x = from_key<T>(s_fkey[i]);
        if (use_minp && !(x * inv_t >= mthr)) continue;
        if (use_topp && r != 0 && !((double)s_before[r] < target)) continue;
        const int v = s_fidx[i];
        const uint32_t h = ehash(key, keyb, (uint32_t)v >> 3);
        const float sc = noise_score(x, inv_t, v, h, group_min_e(h), key2);
        if (better(sc, v, best)) best = Best{sc, v};
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float os = __shfl_xor(best.score, off, kWave);
        const int oi = __shfl_xor(best.idx, off, kWave);
        if (better(os, oi, best)) best = Best{os, oi};
    }
    if (lane == 0) {
        s_bs[w] = best.score;
        s_bi[w] = best.idx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        SPHASE(4);
        Best b{s_bs[0], s_bi[0]};
        for (int j = 1; j < NW; ++j)
            if (better(s_bs[j], s_bi[j], b)) b = Best{s_bs[j], s_bi[j]};
        tokens[row_i] = b.idx;
        if (logp_out) logp_out[row_i] = to_f<T>(row[b.idx]) - lse;
        filt[row_i].ik = kRowDone;
    }
}

// ---- top_p / min_p without top_k: the row streamed twice by one workgroup ---------------------
// (With top_k set, sample_topk_kernel above.) A top_p cut needs the row max before any mass is
// known, and the kept set can run to thousands of tokens (13k at p = 0.95 on N(0, 3^2) rows), so:
//  * pass 1 (HBM; cached loads, so that pass 2 finds the row in the Infinity Cache): the row max
//    and an LDS histogram of COUNTS per exact bf16 key over |x| in [2^-16, 2^16)
//    (8192 bins: every key of that range has its own), +0 and -0 two more; keys below the window
//    (0 < |x| < 2^-16) go to a short list; NaN, +inf, x >= 2^16 or a full list send the row to
//    the fallback.
//  * on chip: with the max known, a bin's mass is its count x mass_q(value, max) -- the pre-pass's
//    fixed-point masses, exactly, without a det_exp2 per element; Z is their exact sum (+ the
//    list's); block scans over the bins in descending key order (positive window, then the
//    negative one) find the cut key kc, and filter_row's tie rule the number c of its elements
//    (index order) that are kept.
//  * pass 2 (re-read): sample_unit's MODE 2 (group bound, exact noise_score, lse) over the keys
//    above kc (min_p alone: x/T >= max/T + ln min_p); when the cut splits kc's tie group, kc's
//    elements go to an LDS list with their exact scores instead, ranked by index afterwards: the
//    first c are admissible.
// The pre-pass's cuts and MODE 2's scores on the same elements: the tokens (and the logprobs)
// of the two-kernel path, and of oracle/sampler_ref.c, bit for bit. Rows outside these bounds
// (the cut among the values below 2^-16 or the zeros, more than kPTieCap ties at the cut) run
// the two-kernel path's code in this workgroup, as the top_k kernel's fallback does.
constexpr int kPNT = 512;
constexpr int kPE0 = 111;       // window: bf16 exponent fields 111..142, |x| in [2^-16, 2^16)
constexpr int kPHalf = 4096;    // keys per sign in the window
constexpr int kPSlowCap = 512;  // elements below the window
constexpr int kPTieCap = 1024;  // elements at a split cut key
constexpr int kPTieRes = 64;    // pass 1 ranks at most this many cut-key records (else pass 2)
constexpr int kPCandCap = 2048; // pass 1's exactly scored elements (seeds + bound survivors)
constexpr int32_t kRowPending = -4;  // RowFilter.ik between the two top_p kernels: pass 2 to run
constexpr int kP2Splits = 8;         // workgroups per left row in sample_topp_pass2_kernel
struct ToppPending {  // a row pass 1 did not decide, for sample_topp_pass2_kernel
    float xlo, xc, lse, mx;  // admissibility bound, the cut key's value, the raw lse, the raw max
    float e_s;               // e*: pass 1's best admissible record (score, index)
    int e_i;
    int split;
    uint32_t kc;
    long long c;             // the split cut key's kept tie ranks
};

// uniform (scalar) copy of a wave-uniform float, so the hot loops keep it in an SGPR
__device__ __forceinline__ float uni(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

template <typename T, bool TOPP>
__global__ __launch_bounds__(kPNT) __attribute__((amdgpu_waves_per_eu(4))) void sample_topp_kernel(
    const T* __restrict__ logits, int64_t ld, int V, float inv_t, int use_minp, float ln_min_p, float top_p,
    uint64_t seed, const int64_t* __restrict__ seq_ids, int64_t step, int32_t* __restrict__ tokens,
    float* __restrict__ logp_out, RowFilter* __restrict__ filt, ToppPending* __restrict__ pend,
    unsigned* __restrict__ pend_nt, int probe) {
    static_assert(sizeof(T) == 2, "bf16 rows");
    constexpr int NT = kPNT, NW = NT / kWave, VEC = 8;
    constexpr int kDummy = 2 * kPHalf;  // 64 words taking the out-of-window elements' increments (no branch)
    __shared__ uint32_t s_hist[2 * kPHalf + kWave];
    __shared__ uint16_t s_slow[kPSlowCap];
    __shared__ uint32_t s_nslow, s_bad, s_nt, s_zero[2];
    __shared__ float s_vmax[NW], s_bar;
    __shared__ double s_wexp[NW];
    __shared__ unsigned long long s_wpos[NW], s_wneg[NW], s_woth[NW];
    __shared__ unsigned long long s_cut_a;
    __shared__ int s_cut_j;
    __shared__ int32_t s_tidx[kPTieCap];
    __shared__ float s_cs[kPCandCap];     // pass 1's exactly scored elements: score, index, key
    __shared__ int32_t s_ci[kPCandCap];
    __shared__ uint16_t s_ck[kPCandCap];
    __shared__ uint32_t s_nc, s_ntie, s_trn;
#ifdef SKYRL_TP_COUNT
    __shared__ uint32_t s_cnt[2];
    if (threadIdx.x < 2) s_cnt[threadIdx.x] = 0u;
#endif
    __shared__ int32_t s_tri[kPTieRes];  // pass 1's cut-key records that beat e* (SKYRL_TP_TIERES)
    __shared__ float s_trs[kPTieRes];
    __shared__ float s_bar1, s_runmax;
    __shared__ __attribute__((aligned(16))) float s_wbest[NW];  // R > 1: each wave's best exact score
    constexpr int kRBar = TOPP ? SKYRL_TP_RBAR : 1;
    __shared__ float s_bs[NW];
    __shared__ int32_t s_bi[NW];
    __shared__ int s_icut;
    __shared__ RowFilter s_rf;
    const int row_i = blockIdx.x;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const T* row = logits + (int64_t)row_i * ld;
    const uint4* rv = reinterpret_cast<const uint4*>(row);  // 16-B aligned (host check)
    const int nvec = V / VEC;
    constexpr int kStep = 4 * NT;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();  // (probes 5 / 6: per-row phase times)
    const int nfull = (nvec / kStep) * kStep;
    uint4 cur[4], nxt[4];
    if (nfull > 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = rv[u * NT + threadIdx.x];
    }
    if (threadIdx.x == 0) {
        s_nslow = 0u;
        s_bad = 0u;
        s_nt = 0u;
        s_cut_j = -1;
        s_zero[0] = s_zero[1] = 0u;
        s_nc = 0u;

        s_ntie = 0u;
        s_bar1 = -INFINITY;  // the workgroup's best exact score so far
        s_runmax = -INFINITY;  // list mode: the largest wave maximum published so far
    }
    if (threadIdx.x < NW) s_wbest[threadIdx.x] = -INFINITY;
    for (int j = threadIdx.x; j < 2 * kPHalf + kWave; j += NT) s_hist[j] = 0u;
    __syncthreads();

    // ---- pass 1: the row max; top_p: the count histogram (one LDS add per element, no branch;
    //      elements outside the window take a uniform slow path), min_p: the raw lse
    float vmx = -INFINITY;
    bool bad = false;
    // The decision in the same pass: MODE 2's noise (group hash, group bound, exact noise_score)
    // against the workgroup's bar = the best exact score computed so far (the unfiltered sampler's
    // race over the whole row). Admissibility is unknown until the cut, so every element the bound
    // lets through is scored exactly and recorded (s_cs / s_ci / s_ck); an element the bound skips
    // scored below the bar at its visit, so below the final bar. After the cut, the best admissible
    // record e* is the row's decision when it is the best record (the unfiltered winner lies in the
    // kept set, so it wins the filtered race too) and no unranked element of a split cut key beats
    // it -- the certificate, which holds with probability about the kept mass (>= top_p); the other
    // rows take pass 2 (the re-read), with e* as its starting bar. (A margin below the bar, which
    // certifies more rows, made pass 1 slower than the re-reads it saved: DESIGN §3 "Filters".)
    // top_p with SKYRL_TP_RBAR = R > 1: the bar is the R-th largest of the waves' best scores, so
    // the certificate (e* >= that final bar) fails only when the row's R best elements are all cut
    // (about (1 - top_p)^R), and recorded cut-key ties above e* are ranked in pass 1 (SKYRL_TP_TIERES).
    const uint32_t key = row_key(seed, seq_ids ? seq_ids[row_i] : (int64_t)row_i, step);
    const uint32_t key2 = noise_key2(key), keyb = noise_keyb(key);
    const float temp = 1.0f / inv_t;
    const float kT = 0.6931471805599453f * 1.1920928955078125e-7f * temp;
    constexpr bool kList = !TOPP && SKYRL_MP_LIST;
    float thr_run = -INFINITY;  // list mode: (a lower bound of the row max) / T + ln min_p, wave-uniform
    float thr1 = -INFINITY;  // (bar - C) T, wave-uniform
    int seed_v = -1;         // this lane's seed element (scored once: no duplicate record)
    auto record = [&](float sc, int v, uint32_t b) {
#ifdef SKYRL_TP_NOREC  // (probe builds only)
        asm volatile("" ::"v"(sc), "v"(v), "v"(b));
        return;
#endif
        const uint32_t p = atomicAdd(&s_nc, 1u);
        if (p < (uint32_t)kPCandCap) {
            s_cs[p] = sc;
            s_ci[p] = v;
            s_ck[p] = (uint16_t)b;
        }
    };
    // R > 1: the R-th largest of the waves' published bests (insertion into R sorted slots)
    auto rbar = [&]() -> float {
        float t[kRBar];
#pragma unroll
        for (int r = 0; r < kRBar; ++r) t[r] = -INFINITY;
#if SKYRL_TP_RBAR_VEC  // two 16-B LDS reads (the other waves' stores seen at the next read: a
                       // compiler barrier keeps the loads here)
        asm volatile("" ::: "memory");
        const float4 q0 = reinterpret_cast<const float4*>(s_wbest)[0], q1 = reinterpret_cast<const float4*>(s_wbest)[1];
        const float wv[NW] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#endif
#pragma unroll
        for (int j = 0; j < NW; ++j) {
#if SKYRL_TP_RBAR_VEC
            float v = wv[j];
#else
            float v = __hip_atomic_load(&s_wbest[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
#pragma unroll
            for (int r = 0; r < kRBar; ++r) {
                const float hi = fmaxf(t[r], v);
                v = fminf(t[r], v);
                t[r] = hi;
            }
        }
        return uni(t[kRBar - 1]);
    };
    float wbest = -INFINITY;  // R > 1: this wave's best exact score (wave-uniform)
#if SKYRL_TP_BAR_FORM
    // publish the wave's best new score and read the workgroup's when a lane beat the wave's bar,
    // else only read the workgroup's (as the unfiltered sampler's after_eval). s_bar1 stays the
    // best record: an unpublished score is <= bar1 <= s_bar1.
    float bar1 = -INFINITY;
    auto bar_merge = [&](float best_new) {
        if constexpr (kRBar > 1) {  // every skipped element scores below the bar at its visit,
                                    // which is at most the final R-th largest wave best
            if (__builtin_amdgcn_ballot_w64(best_new > wbest) != 0) {
                wbest = fmaxf(wbest, wave_max_uniform(best_new));
                if (lane == 0) __hip_atomic_store(&s_wbest[w], wbest, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            thr1 = (rbar() - kNoiseC) * temp;
            return;
        }
        if (__builtin_amdgcn_ballot_w64(best_new > bar1) != 0) {
            const float wb = wave_max_uniform(best_new);
            if (lane == 0 && wb > -INFINITY)
                __hip_atomic_fetch_max(&s_bar1, wb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            bar1 = fmaxf(wb, uni(s_bar1));
        } else {
            bar1 = fmaxf(bar1, uni(s_bar1));
        }
        thr1 = (bar1 - kNoiseC) * temp;
    };
#else
    auto bar_merge = [&](float best_new) {  // publish the wave's best new score, read the workgroup's
        const float wb = wave_max_uniform(best_new);
        if (lane == 0 && wb > -INFINITY)
            __hip_atomic_fetch_max(&s_bar1, wb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        thr1 = (fmaxf(wb, uni(s_bar1)) - kNoiseC) * temp;
    };
#endif
    // the group bound and the exact scores of one group's elements (x[k] at v0 + k, raw bits b[k])
    auto gumbel = [&](const float (&x)[VEC], const uint16_t (&b)[VEC], float vm, int v0, int cnt) {
        const uint32_t h = ehash(key, keyb, (uint32_t)v0 >> 3);
        const float bits = noise_bits(h);
        const bool cand = !(fmaf(bits, -kT, vm) - thr1 < 0.f);
        if (__builtin_amdgcn_ballot_w64(cand) == 0) return;
#ifdef SKYRL_TP_COUNT  // (probe builds: candidate events per row, exact scores per row)
        if (lane == 0) atomicAdd(&s_cnt[0], 1u);
        {
            uint32_t nsc = 0u;
            for (int k = 0; k < VEC; ++k)
                nsc += (cand && k < cnt && v0 + k != seed_v && !(fmaf(bits, -kT, x[k]) - thr1 < 0.f)) ? 1u : 0u;
            if (nsc) atomicAdd(&s_cnt[1], nsc);
        }
#endif
        float bn = -INFINITY;
        if (cand) {
            const float Eg = group_min_e(h);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                if (k < cnt && v0 + k != seed_v && !(fmaf(bits, -kT, x[k]) - thr1 < 0.f)) {
                    const float sc = noise_score(x[k], inv_t, v0 + k, h, Eg, key2);
                    record(sc, v0 + k, b[k]);
                    bn = fmaxf(bn, sc);
                }
            }
        }
        bar_merge(bn);
    };
    // list mode: the vector's elements that can be kept (x/T >= thr_run) into s_cs (values) / s_ci;
    // after a vector that listed any, the wave publishes its running max and reads the workgroup's
    auto collect = [&](const float (&x)[VEC], float vm, int v0, int cnt) {
        const bool any = !(vm * inv_t < thr_run);
        if (__builtin_amdgcn_ballot_w64(any) == 0) return;
        if (any) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                if (k < cnt && !(x[k] * inv_t < thr_run)) {
                    const uint32_t p = atomicAdd(&s_nc, 1u);
                    if (p < (uint32_t)kPCandCap) {
                        s_cs[p] = x[k];
                        s_ci[p] = v0 + k;
                    }
                }
            }
        }
        const float wm = wave_max_uniform(vmx);
        if (lane == 0) __hip_atomic_fetch_max(&s_runmax, wm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        thr_run = fmaxf(wm, uni(s_runmax)) * inv_t + ln_min_p;
    };
    auto rare_elem = [&](uint32_t b) {  // an element outside the window (top_p)
        const uint32_t a = b & 0x7fffu;
        if (a == 0u) {
            atomicAdd(&s_zero[b >> 15], 1u);  // +-0: their own counters (exact zeros may be many)
        } else if (a < (uint32_t)(kPE0 << 7)) {
            const uint32_t pos = atomicAdd(&s_nslow, 1u);
            if (pos < (uint32_t)kPSlowCap) s_slow[pos] = (uint16_t)b;
        } else {  // |x| >= 2^16: -inf and large negatives weigh nothing; NaN, +inf, x >= 2^16: fallback
            bad |= !(b == 0xff80u || ((b & 0x8000u) && a < 0x7f80u));
        }
    };
    auto visit1 = [&](const uint4& pk, int v0) {
        uint16_t raw[VEC];
        __builtin_memcpy(raw, &pk, 16);
        float x[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = bf16_to_f32(raw[k]);
        float vm = x[0];
#pragma unroll
        for (int k = 1; k < VEC; ++k) vm = fmaxf(vm, x[k]);
        vmx = fmaxf(vmx, vm);
#ifndef SKYRL_TP_NORACE  // (probe builds only: timing attribution, tokens invalid)
        if constexpr (kList) collect(x, vm, v0, VEC);
        else gumbel(x, raw, vm, v0, VEC);
#endif
        {
            bool rare = false;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const uint32_t b = raw[k];
                const int wi = (int)(b & 0x7fffu) - (kPE0 << 7);
                const bool in = (unsigned)wi < (unsigned)kPHalf;
                const int bin = (b & 0x8000u) ? kPHalf - 1 - wi : kPHalf + wi;
#ifndef SKYRL_TP_NOHIST  // (probe builds only)
                atomicAdd(&s_hist[in ? bin : kDummy + lane], 1u);
#else
                asm volatile("" ::"v"(bin), "v"(in));
#endif
                rare |= !in;  // (bitwise: a short-circuit || becomes branches)
            }
            if (__builtin_amdgcn_ballot_w64(rare) != 0 && rare) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const int wi = (int)(raw[k] & 0x7fffu) - (kPE0 << 7);
                    if (!((unsigned)wi < (unsigned)kPHalf)) rare_elem(raw[k]);
                }
            }
        }
    };
    if (nfull > 0) {
        if constexpr (kList) {  // the first threshold: the maximum of every lane's first 4 vectors
            float m0 = -INFINITY;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint16_t raw[VEC];
                __builtin_memcpy(raw, &cur[u], 16);
#pragma unroll
                for (int k = 0; k < VEC; ++k) m0 = fmaxf(m0, bf16_to_f32(raw[k]));
            }
            m0 = wave_max_uniform(m0);
            if (lane == 0) __hip_atomic_fetch_max(&s_runmax, m0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            thr_run = uni(s_runmax) * inv_t + ln_min_p;
        } else
        // the wave's first bar: each lane's exact score of the largest element of its first vector
        {
            uint16_t raw[VEC];
            __builtin_memcpy(raw, &cur[0], 16);
            float xb = bf16_to_f32(raw[0]);
            int kb = 0;
#pragma unroll
            for (int k = 1; k < VEC; ++k) {
                const float xk = bf16_to_f32(raw[k]);
                kb = xk > xb ? k : kb;
                xb = fmaxf(xb, xk);
            }
            const int vb = (int)threadIdx.x * VEC + kb;
            const uint32_t h = ehash(key, keyb, (uint32_t)vb >> 3);
            const float sc = noise_score(xb, inv_t, vb, h, group_min_e(h), key2);
            uint16_t bb = raw[0];
#pragma unroll
            for (int k = 1; k < VEC; ++k) bb = k == kb ? raw[k] : bb;
            record(sc, vb, bb);
            seed_v = vb;
            bar_merge(sc);
            if constexpr (kRBar > 1) {  // every wave's seed published before the stream: an early
                                        // visit against an unpublished (-inf) slot scores everything
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                thr1 = (rbar() - kNoiseC) * temp;
            }
        }
        for (int base = 0; base < nfull; base += kStep) {
            const bool more = base + kStep < nfull;
            switch (((nfull - base) * 4 - 1) / nfull) {  // progress priority, as the row-mode sampler
                case 3: __builtin_amdgcn_s_setprio(3); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                default: __builtin_amdgcn_s_setprio(0); break;
            }
            if (more) {
#pragma unroll
                for (int u = 0; u < 4; ++u) nxt[u] = rv[base + kStep + u * NT + threadIdx.x];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                visit1(cur[u], (base + u * NT + (int)threadIdx.x) * VEC);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (more) {
#pragma unroll
                for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
            }
        }
        __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (kList) {
        if (nfull == 0) {  // a short row: the first threshold from every lane's first vector
            float m0 = -INFINITY;
            if ((int)threadIdx.x < nvec) {
                const uint4 pk = rv[threadIdx.x];
                uint16_t raw[VEC];
                __builtin_memcpy(raw, &pk, 16);
#pragma unroll
                for (int k = 0; k < VEC; ++k) m0 = fmaxf(m0, bf16_to_f32(raw[k]));
            }
            m0 = wave_max_uniform(m0);
            if (lane == 0) __hip_atomic_fetch_max(&s_runmax, m0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            thr_run = uni(s_runmax) * inv_t + ln_min_p;
        }
    }
    for (int i0 = nfull; i0 < nvec; i0 += NT) {  // same trip count in every thread (wave ballots inside)
        const int i = i0 + (int)threadIdx.x;
        if (i < nvec) {
            visit1(rv[i], i * VEC);
        } else {  // an idle lane joins the ballots with nothing to score
            const uint16_t nb[VEC] = {0xff80u, 0xff80u, 0xff80u, 0xff80u, 0xff80u, 0xff80u, 0xff80u, 0xff80u};
            const float nx[VEC] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY, -INFINITY, -INFINITY, -INFINITY, -INFINITY};
            if constexpr (kList) collect(nx, -INFINITY, 0, 0);
            else gumbel(nx, nb, -INFINITY, 0, 0);
        }
    }
    if (nvec * VEC < V) {  // the ragged tail: one partial group, lanes 0 .. cnt-1 one element each
        const int t0 = nvec * VEC, cnt = V - t0;
        uint16_t tb[VEC];
        float tx[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            tb[k] = threadIdx.x == 0 && k < cnt ? row[t0 + k] : (uint16_t)0xff80u;
            tx[k] = bf16_to_f32(tb[k]);
        }
        float tm = tx[0];
#pragma unroll
        for (int k = 1; k < VEC; ++k) tm = fmaxf(tm, tx[k]);
        if constexpr (kList) collect(tx, tm, t0, threadIdx.x == 0 ? cnt : 0);
        else gumbel(tx, tb, tm, t0, threadIdx.x == 0 ? cnt : 0);
    }
    for (int i = nvec * VEC + threadIdx.x; i < V; i += NT) {  // ragged tail, one element per thread
        const uint16_t b = row[i];
        const float x = bf16_to_f32(b);
        vmx = fmaxf(vmx, x);
        const int wi = (int)(b & 0x7fffu) - (kPE0 << 7);
        if ((unsigned)wi < (unsigned)kPHalf) atomicAdd(&s_hist[(b & 0x8000u) ? kPHalf - 1 - wi : kPHalf + wi], 1u);
        else rare_elem(b);
    }
    vmx = wave_max(vmx);
    if (bad) s_bad = 1u;
    if (lane == 0) s_vmax[w] = vmx;
    __syncthreads();
    float mx = s_vmax[0];
#pragma unroll
    for (int j = 1; j < NW; ++j) mx = fmaxf(mx, s_vmax[j]);
    mx = uni(mx);
    const uint32_t kmax = okey_bf16(f32_to_bf16(mx));  // the max is a bf16 value: exact
    const float mthr = uni(mx * inv_t + ln_min_p);
    if (probe == 1) return;  // timing probe (variant field topp_probe): pass 1 only
    const uint64_t t_p1 = __builtin_amdgcn_s_memrealtime();  // (probe 11: the cut's time per row)

    bool fb = s_bad != 0u || s_nslow > (uint32_t)kPSlowCap;  // block-uniform
    // the raw logits' sum-exp for the logprob, from the counts (another summation order than a
    // streaming lse: equal to float rounding)
    float lse = 0.f;
    if (!fb) {
        double se = 0.0;
        auto sexp = [&](uint32_t bits, uint32_t n) {
            if (n) se += (double)n * (double)fast_exp2((bf16_to_f32((uint16_t)bits) - mx) * kLog2e);
        };
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int p8 = 8 * (int)threadIdx.x + q;
            sexp((uint32_t)((kPE0 << 7) + p8), s_hist[kPHalf + p8]);
            sexp(0x8000u | (uint32_t)((kPE0 << 7) + p8), s_hist[kPHalf - 1 - p8]);
        }
        for (int i = threadIdx.x; i < (int)s_nslow; i += NT) sexp(s_slow[i], 1u);
        if (threadIdx.x < 2) sexp(threadIdx.x ? 0x8000u : 0u, s_zero[threadIdx.x]);
        se = wave_sum(se);
        if (lane == 0) s_wexp[w] = se;
        __syncthreads();
        double S = 0.0;
        for (int j = 0; j < NW; ++j) S += s_wexp[j];
        lse = mx + fast_log2((float)S) * kLn2;
    }

    // ---- on chip (top_p): bin masses (once per bin, kept in registers), Z, the raw lse, the cut
    //      key and its tie count
    uint32_t kc = 0u;
    bool split = false;
    long long c = 0;
    long long cut_cnt = 0;  // the cut key's element count (top_p)
    int ic = 0x7fffffff;
    if constexpr (TOPP) {
        if (!fb) {
            // thread t: the positive bins at descending positions p = 8t .. 8t+7 (value offset 4095 - p),
            // the negative bins at ascending |x| (offset p), the list entries t, t + NT, ...
            auto mass_of = [&](uint32_t bits, uint32_t n) -> unsigned long long {
                const float x = bf16_to_f32((uint16_t)bits);
                if (n == 0u || (use_minp && !(x * inv_t >= mthr))) return 0ull;
                return (unsigned long long)n * (unsigned long long)mass_q(x, mx, inv_t);
            };
            unsigned long long pm[8], nm[8];
            unsigned long long pos = 0ull, neg = 0ull, mid = 0ull;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int p8 = 8 * (int)threadIdx.x + q;
                const uint32_t pb = (uint32_t)((kPE0 << 7) + kPHalf - 1 - p8), nb = 0x8000u | (uint32_t)((kPE0 << 7) + p8);
                const uint32_t pc = s_hist[2 * kPHalf - 1 - p8], nc = s_hist[kPHalf - 1 - p8];
                pm[q] = mass_of(pb, pc);
                nm[q] = mass_of(nb, nc);
                pos += pm[q];
                neg += nm[q];
            }
            for (int i = threadIdx.x; i < (int)s_nslow; i += NT) mid += mass_of(s_slow[i], 1u);
            if (threadIdx.x < 2) mid += mass_of(threadIdx.x ? 0x8000u : 0u, s_zero[threadIdx.x]);
            unsigned long long ip = pos, in = neg;
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const unsigned long long op = (unsigned long long)__shfl_up((long long)ip, off, kWave);
                const unsigned long long on = (unsigned long long)__shfl_up((long long)in, off, kWave);
                if (lane >= off) {
                    ip += op;
                    in += on;
                }
            }
            unsigned long long wm = mid;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) wm += (unsigned long long)__shfl_xor((long long)wm, off, kWave);
            if (lane == kWave - 1) {
                s_wpos[w] = ip;
                s_wneg[w] = in;
            }
            if (lane == 0) s_woth[w] = wm;
            __syncthreads();
            unsigned long long offp = 0ull, offn = 0ull, Zp = 0ull, Zn = 0ull, Zm = 0ull;
            for (int j = 0; j < NW; ++j) {
                if (j < w) {
                    offp += s_wpos[j];
                    offn += s_wneg[j];
                }
                Zp += s_wpos[j];
                Zn += s_wneg[j];
                Zm += s_woth[j];
            }
            const double target = (double)top_p * (double)(Zp + Zm + Zn);
            // the cut: the bin where the mass before it is < p Z and the mass through it reaches it (the
            // first weighted bin also when target <= 0: top_p = 0 keeps the top token, as filter_row's
            // radix select, whose first bin is the max's); cut_j < 4096: positive bin (descending
            // position), >= 4096: negative bin 4096 + |x| offset
            auto scan8 = [&](unsigned long long cum, const unsigned long long (&m)[8], int base) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    if (m[q] && (cum == 0ull || (double)cum < target) && (double)(cum + m[q]) >= target) {
                        s_cut_j = base + 8 * (int)threadIdx.x + q;
                        s_cut_a = cum;
                    }
                    cum += m[q];
                }
            };
            scan8(offp + ip - pos, pm, 0);
            __syncthreads();
            if (s_cut_j < 0 && (double)(Zp + Zm) < target) {  // past the positive window and the middle
                scan8(Zp + Zm + offn + in - neg, nm, kPHalf);
                __syncthreads();
            }
            if (s_cut_j < 0) {  // the cut among the values below 2^-16 / the zeros (or not reached)
                fb = true;
            } else {
                const int cj = s_cut_j;
                const bool cut_neg = cj >= kPHalf;
                const int cb = cut_neg ? cj - kPHalf : kPHalf - 1 - cj;  // window offset of the cut value
                kc = okey_bf16((uint16_t)((cut_neg ? 0x8000u : 0u) | (uint32_t)((kPE0 << 7) + cb)));
                const long long cnt = (long long)s_hist[cut_neg ? kPHalf - 1 - cb : kPHalf + cb];
                cut_cnt = cnt;
                const unsigned long long qc = mass_q(from_key<T>(kc), mx, inv_t);
                const unsigned long long A = s_cut_a;
                // filter_row's rule: c = number of tie ranks j >= 0 with A + j qc < target (the first
                // always for the top key)
                const double jd = (target - (double)A) / (double)qc;
                c = jd > 0.0 ? (long long)jd : 0;
                while (c > 0 && (double)(A + (unsigned long long)(c - 1) * qc) >= target) --c;
                while ((double)(A + (unsigned long long)c * qc) < target) ++c;
                if (kc == kmax && c < 1) c = 1;
                if (c < cnt) {
                    if (cnt > kPTieCap) fb = true;
                    split = true;
                    ic = -1;
                }
            }
        }
    }
    // the cut as wave-uniform scalars (SGPRs through pass 2)
    kc = (uint32_t)__builtin_amdgcn_readfirstlane((int)kc);
    split = __builtin_amdgcn_readfirstlane((int)split) != 0;
    c = (long long)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)c >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c));
    ic = __builtin_amdgcn_readfirstlane(ic);
    lse = uni(lse);
    if (!fb) {  // (the fallback's call site stays after the hot loops: the register allocation of
                // the passes does not see it)
#ifdef SKYRL_TP_COUNT
    if (probe == 2 && threadIdx.x == 0) {
        tokens[row_i] = (int)s_cnt[0];
        if (logp_out) logp_out[row_i] = (float)s_cnt[1];
    }
#endif
    if (probe == 2) return;  // timing probe: pass 1 + the cut
    if (probe == 11) {  // timing probe: per row, the cut's and pass 1's times (10-ns ticks; tokens invalid)
        if (threadIdx.x == 0) {
            tokens[row_i] = (int)(__builtin_amdgcn_s_memrealtime() - t_p1);
            if (logp_out) logp_out[row_i] = (float)(t_p1 - t_start);
        }
        return;
    }

    // ---- pass 2: the Gumbel-max decision (MODE 2's noise, group bound and exact scores) over the
    //      admissible elements x >= xlo: top_p, the value above the cut key when the cut splits its
    //      tie group, else the cut key's value (value and key order agree off +-0, which no window
    //      bin holds); min_p alone, the smallest bf16 value with x/T >= max/T + ln min_p; the cut
    //      key's elements, when split, into the tie list (indices: their value is xc)
    const float xc = uni(TOPP ? from_key<T>(kc) : 0.f);
    float xlo;
    if constexpr (TOPP) {
        xlo = uni(split ? from_key<T>(kc + 1u) : xc);
    } else {
        // min_p as a value bound: the smallest bf16 x with x/T >= mthr (x * inv_t is monotone in x),
        // by bisection over the keys between -inf (never) and +inf (always)
        uint32_t lo = 0x007fu, hi = 0xff80u;
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (from_key<T>(mid) * inv_t >= mthr) hi = mid;
            else lo = mid;
        }
        xlo = uni(from_key<T>(hi));
    }
    // ---- pass 1's decision: the best admissible record e*, certified when it reaches the final
    //      bar (the best record; R > 1: the R-th largest wave best) and no unranked element of a split
    //      cut key beats it: an element the bound skipped scored below the bar at its visit, so below
    //      the final bar, so below e*; otherwise pass 2 decides, starting from e*
    Best e0{-INFINITY, 0x7fffffff};
#ifdef SKYRL_TP_REASON
    uint32_t why = 16u;
#endif
    if constexpr (kList) {
        // list mode: every kept element (x >= xlo) is listed when the list did not overflow; their
        // exact scores decide the row (the max is kept, so the list holds at least one). Overflow:
        // the in-row pass 2 below, from no bar
        if (probe != 5 && s_nc <= (uint32_t)kPCandCap) {
            const int nc = (int)s_nc;
            Best e{-INFINITY, 0x7fffffff};
            for (int i = threadIdx.x; i < nc; i += NT) {
                const float xv = s_cs[i];
                if (xv >= xlo) {
                    const int v = s_ci[i];
                    const uint32_t h = ehash(key, keyb, (uint32_t)v >> 3);
                    const float sc = noise_score(xv, inv_t, v, h, group_min_e(h), key2);
                    if (better(sc, v, e)) e = Best{sc, v};
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const float os = __shfl_xor(e.score, off, kWave);
                const int oi = __shfl_xor(e.idx, off, kWave);
                if (better(os, oi, e)) e = Best{os, oi};
            }
            if (lane == 0) {
                s_bs[w] = e.score;
                s_bi[w] = e.idx;
            }
            __syncthreads();
            Best es{s_bs[0], s_bi[0]};
            for (int j = 1; j < NW; ++j)
                if (better(s_bs[j], s_bi[j], es)) es = Best{s_bs[j], s_bi[j]};
            if (es.idx != 0x7fffffff) {  // (block-uniform)
                if (threadIdx.x == 0) {
                    tokens[row_i] = es.idx;
                    if (logp_out) logp_out[row_i] = to_f<T>(row[es.idx]) - lse;
                    filt[row_i] = RowFilter{mx, 1u, kRowDone, kc, ic};
                }
                return;
            }
            __syncthreads();  // s_bs reused below
        }
    } else {
        const int nc = (int)min(s_nc, (uint32_t)kPCandCap);
        const bool complete = s_nc <= (uint32_t)kPCandCap;
        auto cls = [&](int i) -> int {  // 1 admissible, 0 inadmissible, 2 an element of the split cut key
            const uint32_t kk = okey_bf16(s_ck[i]);
            if constexpr (TOPP) {
                if (kk > kc || (!split && kk == kc)) return 1;
                return (split && kk == kc) ? 2 : 0;
            } else {
                return bf16_to_f32(s_ck[i]) >= xlo ? 1 : 0;
            }
        };
        Best e{-INFINITY, 0x7fffffff};
        for (int i = threadIdx.x; i < nc; i += NT)
            if (cls(i) == 1 && better(s_cs[i], s_ci[i], e)) e = Best{s_cs[i], s_ci[i]};
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float os = __shfl_xor(e.score, off, kWave);
            const int oi = __shfl_xor(e.idx, off, kWave);
            if (better(os, oi, e)) e = Best{os, oi};
        }
        if (lane == 0) {
            s_bs[w] = e.score;
            s_bi[w] = e.idx;
        }
        __syncthreads();
        Best es{s_bs[0], s_bi[0]};
        for (int j = 1; j < NW; ++j)
            if (better(s_bs[j], s_bi[j], es)) es = Best{s_bs[j], s_bi[j]};
        e0 = es;
        uint32_t ntie = 0u;
        if (TOPP && split)
            for (int i = threadIdx.x; i < nc; i += NT) ntie += (better(s_cs[i], s_ci[i], es) && cls(i) == 2) ? 1u : 0u;
        if (ntie) atomicAdd(&s_ntie, ntie);
        __syncthreads();
        const float bar_end = kRBar > 1 ? rbar() : s_bar1;  // (after the barriers above: final)
        bool ties_ok = s_ntie == 0u;
#ifdef SKYRL_TP_REASON
        why |= (complete ? 0u : 1u) | (es.idx == 0x7fffffff ? 2u : 0u) | (s_ntie ? 4u : 0u) | (es.score < bar_end ? 8u : 0u);
#endif
#if SKYRL_TP_TIERES
        // recorded elements of the split cut key that beat e*: kept iff fewer than c elements of that
        // key precede them (filter_row's index order), so rank them here by a scan of the row prefix
        // (cached: the row was just read) for the key's indices, instead of leaving the row to pass 2.
        // The unrecorded ones scored below the bar, so below e*: the decision is the best of e* and the
        // kept listed records.
        if (TOPP && split && !ties_ok && s_ntie <= (uint32_t)kPTieRes && probe != 5 && complete &&
            es.idx != 0x7fffffff && es.score >= bar_end) {
            if (threadIdx.x == 0) s_trn = 0u;
            __syncthreads();
            for (int i = threadIdx.x; i < nc; i += NT)
                if (cls(i) == 2 && better(s_cs[i], s_ci[i], es)) {
                    const uint32_t p = atomicAdd(&s_trn, 1u);  // < kPTieRes (s_ntie counted the same set)
                    s_tri[p] = s_ci[i];
                    s_trs[p] = s_cs[i];
                }
            __syncthreads();
            const int nr = (int)s_trn;
            int imin = 0x7fffffff, imax = 0;
            for (int j = 0; j < nr; ++j) {
                imin = min(imin, s_tri[j]);
                imax = max(imax, s_tri[j]);
            }
            // the shorter side: the key's indices below imax (rank = those below the record), or
            // from imin on (rank = the key's count - those at or above the record)
            const bool suffix = V - imin < imax;
            const int e0 = suffix ? imin : 0, e1 = suffix ? V : imax;
            const int vb = min((e0 + VEC - 1) / VEC, nvec), ve = max(vb, min(e1 / VEC, nvec));
            auto tie_vec = [&](const uint4& pk, int i) {
                uint16_t raw[VEC];
                __builtin_memcpy(raw, &pk, 16);
                uint32_t n = 0u;
#pragma unroll
                for (int k = 0; k < VEC; ++k) n += bf16_to_f32(raw[k]) == xc ? 1u : 0u;
                if (n) {
                    uint32_t p = atomicAdd(&s_nt, n);
#pragma unroll
                    for (int k = 0; k < VEC; ++k)
                        if (bf16_to_f32(raw[k]) == xc) s_tidx[p++] = i * VEC + k;  // (<= the key's count <= kPTieCap)
                }
            };
            constexpr int kScanDepth = 8;  // loads in flight per lane (a lone workgroup: latency-bound)
            for (int i0 = vb + (int)threadIdx.x; i0 < ve; i0 += kScanDepth * NT) {
                uint4 pk[kScanDepth];
#pragma unroll
                for (int u = 0; u < kScanDepth; ++u) {
                    const int i = i0 + u * NT;
                    pk[u] = i < ve ? rv[i] : make_uint4(0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u);
                }
#pragma unroll
                for (int u = 0; u < kScanDepth; ++u) tie_vec(pk[u], i0 + u * NT);
            }
            {  // the elements outside whole vectors: [e0, vb VEC) and [ve VEC, e1)
                const int a1 = min(vb * VEC, e1), b0 = max(max(ve * VEC, a1), e0);
                for (int i = e0 + (int)threadIdx.x; i < a1; i += NT)
                    if (to_f<T>(row[i]) == xc) s_tidx[atomicAdd(&s_nt, 1u)] = i;
                for (int i = b0 + (int)threadIdx.x; i < e1; i += NT)
                    if (to_f<T>(row[i]) == xc) s_tidx[atomicAdd(&s_nt, 1u)] = i;
            }
            __syncthreads();
            const int n = (int)s_nt;
            Best tb{-INFINITY, 0x7fffffff};
            if ((int)threadIdx.x < nr) {
                const int ii = s_tri[threadIdx.x];
                long long r = 0;
                if (suffix) {
                    for (int j = 0; j < n; ++j) r += s_tidx[j] >= ii ? 1 : 0;
                    r = cut_cnt - r;
                } else {
                    for (int j = 0; j < n; ++j) r += s_tidx[j] < ii ? 1 : 0;
                }
                if (r < c) tb = Best{s_trs[threadIdx.x], ii};
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const float os = __shfl_xor(tb.score, off, kWave);
                const int oi = __shfl_xor(tb.idx, off, kWave);
                if (better(os, oi, tb)) tb = Best{os, oi};
            }
            if (lane == 0) {
                s_bs[w] = tb.score;
                s_bi[w] = tb.idx;
            }
            __syncthreads();
            for (int j = 0; j < NW; ++j)
                if (better(s_bs[j], s_bi[j], es)) es = Best{s_bs[j], s_bi[j]};
            ties_ok = true;
        }
#endif
        const bool certified = probe != 5 && complete && es.idx != 0x7fffffff && ties_ok && es.score >= bar_end;
        if (certified) {
            if (threadIdx.x == 0) {
                tokens[row_i] = es.idx;
                if (logp_out) logp_out[row_i] = to_f<T>(row[es.idx]) - lse;
                // (tk = 1: decided in pass 1; ic unresolved: not needed)
                filt[row_i] = RowFilter{mx, 1u, kRowDone, kc, split ? -1 : ic};
            }
            return;
        }
        __syncthreads();  // s_bs reused below
    }
    if constexpr (TOPP) {
        // top_p: a row pass 1 did not decide goes to sample_topp_pass2_kernel (launched next), cut
        // into kP2Splits workgroups: few rows are left (~5 %), and one alone on this workgroup's CU
        // spends ~20 us in the visits' VALU. min_p alone leaves most rows (~70 %): the in-row pass 2
        // below, at full occupancy, is the better form there.
        if (probe < 3 || probe > 4) {
            if (threadIdx.x == 0) {
                pend[row_i] = ToppPending{xlo, xc, lse, mx, e0.score, e0.idx, split ? 1 : 0, kc, c};
                pend_nt[2 * row_i] = 0u;      // the row's tie count and its pieces' arrival counter (the
                pend_nt[2 * row_i + 1] = 0u;  // workspace layout moves with the batch size: not left re-armed)
#ifdef SKYRL_TP_REASON  // (probe builds: why pass 1 left the row, kept through pass 2)
                filt[row_i] = RowFilter{mx, why, kRowPending, kc, ic};
#else
                filt[row_i] = RowFilter{mx, 0u, kRowPending, kc, ic};
#endif
            }
            return;
        }
    }
    const uint64_t t_p2 = __builtin_amdgcn_s_memrealtime();
    // e* (admissible, exactly scored) is the starting best and bar: only elements that beat it
    // are scored exactly
    float bar = uni(e0.score);
    float thr = (bar - kNoiseC) * temp;
    float best_s = e0.score;
    int best_i = e0.idx;
    if (threadIdx.x == 0) s_bar = e0.score;
    auto adm = [&](float x) -> bool { return x >= xlo; };
    auto raise_bar = [&]() {  // publish the wave's best, read the workgroup's
        const float wb = wave_max_uniform(best_s);
        if (lane == 0 && wb > -INFINITY)
            __hip_atomic_fetch_max(&s_bar, wb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        bar = fmaxf(wb, uni(s_bar));
        thr = (bar - kNoiseC) * temp;
    };
    // one vector of up to VEC elements at v0 (one noise group; padding slots are -inf); a vector
    // without admissible elements in the whole wave costs no hash
    auto visit2 = [&](const uint4& pk, int v0) {
        uint16_t raw[VEC];
        __builtin_memcpy(raw, &pk, 16);
        float x[VEC];
        float xm = -INFINITY;
        bool anyt = false;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            x[k] = bf16_to_f32(raw[k]);
            xm = fmaxf(xm, adm(x[k]) ? x[k] : -INFINITY);
            if constexpr (TOPP) anyt |= x[k] == xc;  // (gated by split at the ballot)
        }
        if constexpr (TOPP) {
            if (split && __builtin_amdgcn_ballot_w64(anyt) != 0 && anyt) {
                uint32_t nt = 0u;
#pragma unroll
                for (int k = 0; k < VEC; ++k) nt += x[k] == xc ? 1u : 0u;
                uint32_t p = atomicAdd(&s_nt, nt);
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    if (x[k] == xc) {
                        if (p < (uint32_t)kPTieCap) s_tidx[p] = v0 + k;
                        ++p;
                    }
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(xm > -INFINITY) == 0) return;
        const uint32_t h = ehash(key, keyb, (uint32_t)v0 >> 3);
        const float bits = noise_bits(h);
        const bool cand = !(fmaf(bits, -kT, xm) - thr < 0.f);
        if (__builtin_amdgcn_ballot_w64(cand) == 0) return;
        if (cand) {
            const float Eg = group_min_e(h);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                if (adm(x[k]) && !(fmaf(bits, -kT, x[k]) - thr < 0.f)) {
                    const float sc = noise_score(x[k], inv_t, v0 + k, h, Eg, key2);
                    if (better(sc, v0 + k, Best{best_s, best_i})) {
                        best_s = sc;
                        best_i = v0 + k;
                    }
                }
            }
        }
        raise_bar();
    };
    // four vectors (a stage) at once: one ballot per decision instead of one per vector, and the
    // four group hashes independent of each other (a row left to pass 2 runs alone on its CU at the
    // end of the launch, bound by its waves' dependent chains, not by bandwidth)
    auto visit2x4 = [&](const uint4 (&pk)[4], int vbase) {  // vector u at (vbase + u NT) VEC
        float xm[4];
        bool anyt = false, anya = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint16_t raw[VEC];
            __builtin_memcpy(raw, &pk[u], 16);
            xm[u] = -INFINITY;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const float x = bf16_to_f32(raw[k]);
                xm[u] = fmaxf(xm[u], adm(x) ? x : -INFINITY);
                if constexpr (TOPP) anyt |= x == xc;  // (gated by split at the ballot)
            }
            anya |= xm[u] > -INFINITY;
        }
        if constexpr (TOPP) {
            // the cut key's elements into the tie list: ONE LDS add per lane for all its ties (an
            // add per element would wait on its return in each of the 32 slots, exec-masked or not:
            // 2/3 of the pass's time before this)
            if (split && __builtin_amdgcn_ballot_w64(anyt) != 0) {
                uint32_t nt = 0u;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    uint16_t raw[VEC];
                    __builtin_memcpy(raw, &pk[u], 16);
#pragma unroll
                    for (int k = 0; k < VEC; ++k) nt += bf16_to_f32(raw[k]) == xc ? 1u : 0u;
                }
                if (nt) {
                    uint32_t p = atomicAdd(&s_nt, nt);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        uint16_t raw[VEC];
                        __builtin_memcpy(raw, &pk[u], 16);
#pragma unroll
                        for (int k = 0; k < VEC; ++k) {
                            if (bf16_to_f32(raw[k]) == xc) {
                                if (p < (uint32_t)kPTieCap) s_tidx[p] = (vbase + u * NT) * VEC + k;
                                ++p;
                            }
                        }
                    }
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(anya) == 0) return;
        uint32_t h[4];
        bool cand[4], anyc = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            h[u] = ehash(key, keyb, (uint32_t)(vbase + u * NT));  // (the group index: vector index)
            cand[u] = !(fmaf(noise_bits(h[u]), -kT, xm[u]) - thr < 0.f);
            anyc |= cand[u];
        }
        if (__builtin_amdgcn_ballot_w64(anyc) == 0) return;
        if (anyc) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (cand[u]) {
                    uint16_t raw[VEC];
                    __builtin_memcpy(raw, &pk[u], 16);
                    const float bits = noise_bits(h[u]);
                    const float Eg = group_min_e(h[u]);
                    const int v0 = (vbase + u * NT) * VEC;
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        const float x = bf16_to_f32(raw[k]);
                        if (adm(x) && !(fmaf(bits, -kT, x) - thr < 0.f)) {
                            const float sc = noise_score(x, inv_t, v0 + k, h[u], Eg, key2);
                            if (better(sc, v0 + k, Best{best_s, best_i})) {
                                best_s = sc;
                                best_i = v0 + k;
                            }
                        }
                    }
                }
            }
        }
        raise_bar();
    };
    constexpr uint32_t kPadNinf = 0xff80ff80u;  // -inf bf16 pairs: never admissible, never a tie
    if (probe == 3) {  // timing probe: pass 2's re-read alone (loads consumed by an xor)
        uint32_t acc = 0u;
        for (int i = threadIdx.x; i < nvec; i += NT) {
            const uint4 v = ld_stream(rv + i);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        if (acc == 0x12345678u) tokens[row_i] = -7;
        return;
    }
    if (probe == 4) {  // timing probe: the same re-read with cached loads
        uint32_t acc = 0u;
        for (int i = threadIdx.x; i < nvec; i += NT) {
            const uint4 v = rv[i];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        if (acc == 0x12345678u) tokens[row_i] = -7;
        return;
    }
    // pass 2's stream: kP2Depth stages of 4 NT vectors, each refilled right after it is visited, so
    // that (kP2Depth - 1) x 4 loads per lane stay in flight (a row re-read alone on its CU at the end
    // of the launch is latency-bound; cached loads: the row is in the Infinity Cache)
    constexpr int kP2Depth = 3;
    const int nit = nfull / kStep;
    uint4 stg[kP2Depth][4];
#pragma unroll
    for (int d = 0; d < kP2Depth; ++d)
        if (d < nit) {
#pragma unroll
            for (int u = 0; u < 4; ++u) stg[d][u] = rv[d * kStep + u * NT + threadIdx.x];
        }
    __syncthreads();  // s_bar
    if (nfull > 0) {
        // the bar from this lane's first two vectors (one exact score: the best admissible element)
        float xb = -INFINITY;
        int vb = -1;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            uint16_t raw[VEC];
            __builtin_memcpy(raw, &stg[0][u], 16);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const float x = bf16_to_f32(raw[k]);
                if (adm(x) && x > xb) {
                    xb = x;
                    vb = (u * NT + (int)threadIdx.x) * VEC + k;
                }
            }
        }
        if (vb >= 0) {
            const uint32_t h = ehash(key, keyb, (uint32_t)vb >> 3);
            const float sc = noise_score(xb, inv_t, vb, h, group_min_e(h), key2);
            if (better(sc, vb, Best{best_s, best_i})) {
                best_s = sc;
                best_i = vb;
            }
        }
        raise_bar();
        __syncthreads();
        bar = fmaxf(bar, uni(s_bar));
        thr = (bar - kNoiseC) * temp;
        for (int it0 = 0; it0 < nit; it0 += kP2Depth) {
            switch (((nit - it0) * 4 - 1) / nit) {
                case 3: __builtin_amdgcn_s_setprio(3); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                default: __builtin_amdgcn_s_setprio(0); break;
            }
#pragma unroll
            for (int d = 0; d < kP2Depth; ++d) {  // stage d in place (no register rotation: a move
                const int it = it0 + d;           // would wait for the loads in flight)
                if (it < nit) {
                    if (probe == 7) {  // timing probe: the stage loop's loads without the visits
                        uint32_t acc = 0u;
#pragma unroll
                        for (int u = 0; u < 4; ++u) acc ^= stg[d][u].x ^ stg[d][u].y ^ stg[d][u].z ^ stg[d][u].w;
                        if (acc == 0x12345678u) s_nt = acc;
                    } else {
                        visit2x4(stg[d], it * kStep + (int)threadIdx.x);
                    }
                    if (it + kP2Depth < nit) {
#pragma unroll
                        for (int u = 0; u < 4; ++u) stg[d][u] = rv[(it + kP2Depth) * kStep + u * NT + threadIdx.x];
                    }
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
    }
    // the rest: whole vectors (same trip count in every thread: the wave ballots inside), then the
    // ragged tail's partial group, read element-wise by thread 0
    for (int i0 = nfull; i0 < nvec; i0 += NT) {
        const int i = i0 + (int)threadIdx.x;
        visit2(i < nvec ? rv[i] : make_uint4(kPadNinf, kPadNinf, kPadNinf, kPadNinf), i * VEC);
    }
    if (nvec * VEC < V) {
        const int t0 = nvec * VEC, cnt = V - t0;
        uint16_t t[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) t[k] = (threadIdx.x == 0 && k < cnt) ? row[t0 + k] : (uint16_t)0xff80u;
        uint4 pk;
        __builtin_memcpy(&pk, t, 16);
        visit2(pk, t0);
    }
    // the best admissible element: lanes, waves; then the cut key's kept ties
    Best best{best_s, best_i};
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float os = __shfl_xor(best.score, off, kWave);
        const int oi = __shfl_xor(best.idx, off, kWave);
        if (better(os, oi, best)) best = Best{os, oi};
    }
    if (lane == 0) {
        s_bs[w] = best.score;
        s_bi[w] = best.idx;
    }
    __syncthreads();
    Best b{s_bs[0], s_bi[0]};
    for (int j = 1; j < NW; ++j)
        if (better(s_bs[j], s_bi[j], b)) b = Best{s_bs[j], s_bi[j]};
    int icut = ic;
    if (TOPP && split) {  // rank kc's elements by index: the first c are admissible, scored exactly here
        const int n = (int)min(s_nt, (uint32_t)kPTieCap);
        Best tb{-INFINITY, 0x7fffffff};
        for (int i = threadIdx.x; i < n; i += NT) {
            const int ii = s_tidx[i];
            int r = 0;
            for (int j = 0; j < n; ++j) r += s_tidx[j] < ii ? 1 : 0;
            if (r < c) {
                const uint32_t h = ehash(key, keyb, (uint32_t)ii >> 3);
                const float sc = noise_score(xc, inv_t, ii, h, group_min_e(h), key2);
                if (better(sc, ii, tb)) tb = Best{sc, ii};
            }
            if (r == c - 1) s_icut = ii;  // the cut's last kept index (filter_row's ic)
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float os = __shfl_xor(tb.score, off, kWave);
            const int oi = __shfl_xor(tb.idx, off, kWave);
            if (better(os, oi, tb)) tb = Best{os, oi};
        }
        __syncthreads();
        if (lane == 0) {
            s_bs[w] = tb.score;
            s_bi[w] = tb.idx;
        }
        __syncthreads();
        for (int j = 0; j < NW; ++j)
            if (better(s_bs[j], s_bi[j], b)) b = Best{s_bs[j], s_bi[j]};
        icut = s_icut;
    }
    if (threadIdx.x == 0) {
        tokens[row_i] = b.idx;
        if (logp_out)
            logp_out[row_i] = (b.idx >= 0 && b.idx < V) ? to_f<T>(row[b.idx]) - lse : __builtin_nanf("");
        filt[row_i] = RowFilter{mx, 0u, kRowDone, kc, icut};
        if (probe >= 6) {  // timing probes (6, 7): pass 2's and the row's time before it, 10-ns ticks
            tokens[row_i] = (int)(__builtin_amdgcn_s_memrealtime() - t_p2);
            if (logp_out) logp_out[row_i] = (float)(t_p2 - t_start);
        }
    }
    return;
    }
    // the two-kernel path's code in this workgroup (one call site)
    topk_fallback<T>(logits, ld, V, 0, inv_t, use_minp, ln_min_p, TOPP ? 1 : 0, top_p, seed, seq_ids, step, tokens,
                     logp_out, &s_rf, row_i);
    if (threadIdx.x == 0) filt[row_i].ik = kRowFallback;
}

// Pass 2 of the rows sample_topp_kernel left pending (RowFilter.ik = kRowPending), each row cut into
// kP2Splits workgroups of contiguous vectors (a fixed partition: the split-mode sampler's pattern).
// (Measured and dropped in r05: a (slots x 8) grid over the left rows only, 25.6 vs 24 us; pass 2
// inside pass 1's launch with the left rows' pieces claimed by the workgroups that finished -- a
// CAS-claimed queue head ~1.4 ms, a row-by-row walk ~120 us, tickets ~88-91 vs 80-82 us a launch:
// a piece claimed after the row's cut waits out the same latency chain as a launch, plus the claim.)
// MODE 2 over the admissible elements x >= xlo of the piece, bar and best starting from e*; the
// split cut key's indices appended to the row's tie list (one agent-scope add per lane). The last
// arriving piece (arrive_last) merges the pieces' bests, ranks the ties by index (the first c are
// admissible, scored exactly) and writes token, logprob and cut. The other rows' workgroups exit.
template <typename T, bool TOPP>
__global__ __launch_bounds__(kPNT) void sample_topp_pass2_kernel(
    const T* __restrict__ logits, int64_t ld, int V, float inv_t, uint64_t seed, const int64_t* __restrict__ seq_ids,
    int64_t step, int32_t* __restrict__ tokens, float* __restrict__ logp_out, RowFilter* __restrict__ filt,
    const ToppPending* __restrict__ pend, unsigned* __restrict__ pend_nt, int32_t* __restrict__ ties,
    Best* __restrict__ parts) {
    constexpr int NT = kPNT, NW = NT / kWave, VEC = 8, kPer = 8;  // up to kPer vectors per lane
    const int row_i = blockIdx.x, piece = blockIdx.y;
    if (filt[row_i].ik != kRowPending) return;  // (workgroup-uniform)
    __shared__ float s_bar, s_bs[NW];
    __shared__ int32_t s_bi[NW];
    __shared__ int s_last, s_icut;
    __shared__ int32_t s_tidx[kPTieCap];
    const ToppPending st = pend[row_i];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const T* row = logits + (int64_t)row_i * ld;
    const uint4* rv = reinterpret_cast<const uint4*>(row);
    const int nvec = V / VEC;
    const int cs = (nvec + kP2Splits - 1) / kP2Splits;  // host check: cs <= kPer NT
    const int c0 = min(nvec, piece * cs), c1 = min(nvec, c0 + cs);
    const uint32_t key = row_key(seed, seq_ids ? seq_ids[row_i] : (int64_t)row_i, step);
    const uint32_t key2 = noise_key2(key), keyb = noise_keyb(key);
    const float temp = 1.0f / inv_t;
    const float kT = 0.6931471805599453f * 1.1920928955078125e-7f * temp;
    const float xlo = uni(st.xlo), xc = uni(st.xc);
    const bool split = st.split != 0;
    // the piece's vectors, all loads in flight at once
    constexpr uint32_t kPadNinf = 0xff80ff80u;  // -inf bf16 pairs: never admissible, never a tie
    uint4 v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int i = c0 + u * NT + (int)threadIdx.x;
        v[u] = i < c1 ? rv[i] : make_uint4(kPadNinf, kPadNinf, kPadNinf, kPadNinf);
    }
    if (threadIdx.x == 0) s_bar = st.e_s;
    __syncthreads();
    float bar = uni(st.e_s);
    float thr = (bar - kNoiseC) * temp;
    float best_s = st.e_s;
    int best_i = st.e_i;
    uint32_t nt = 0u;
    // ties first (one add per lane), then MODE 2 per vector
    if constexpr (TOPP) {
        if (split) {
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                uint16_t raw[VEC];
                __builtin_memcpy(raw, &v[u], 16);
#pragma unroll
                for (int k = 0; k < VEC; ++k) nt += bf16_to_f32(raw[k]) == xc ? 1u : 0u;
            }
            if (nt) {
                uint32_t p = __hip_atomic_fetch_add(pend_nt + 2 * row_i, nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int u = 0; u < kPer; ++u) {
                    uint16_t raw[VEC];
                    __builtin_memcpy(raw, &v[u], 16);
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        if (bf16_to_f32(raw[k]) == xc) {
                            if (p < (uint32_t)kPTieCap)
                                st_wt(ties + (int64_t)row_i * kPTieCap + p, (c0 + u * NT + (int)threadIdx.x) * VEC + k);
                            ++p;
                        }
                    }
                }
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        if (c0 + u * NT >= c1) break;  // (uniform)
        const int v0 = (c0 + u * NT + (int)threadIdx.x) * VEC;
        uint16_t raw[VEC];
        __builtin_memcpy(raw, &v[u], 16);
        float xm = -INFINITY;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const float x = bf16_to_f32(raw[k]);
            xm = fmaxf(xm, x >= xlo ? x : -INFINITY);
        }
        if (__builtin_amdgcn_ballot_w64(xm > -INFINITY) == 0) continue;
        const uint32_t h = ehash(key, keyb, (uint32_t)v0 >> 3);
        const float bits = noise_bits(h);
        const bool cand = !(fmaf(bits, -kT, xm) - thr < 0.f);
        if (__builtin_amdgcn_ballot_w64(cand) == 0) continue;
        if (cand) {
            const float Eg = group_min_e(h);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const float x = bf16_to_f32(raw[k]);
                if (x >= xlo && !(fmaf(bits, -kT, x) - thr < 0.f)) {
                    const float sc = noise_score(x, inv_t, v0 + k, h, Eg, key2);
                    if (better(sc, v0 + k, Best{best_s, best_i})) {
                        best_s = sc;
                        best_i = v0 + k;
                    }
                }
            }
        }
#if SKYRL_TP2_BAR_FORM
        if (__builtin_amdgcn_ballot_w64(best_s > bar) != 0) {  // publish only when a lane improved
            const float wb = wave_max_uniform(best_s);
            if (lane == 0 && wb > bar) __hip_atomic_fetch_max(&s_bar, wb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            bar = fmaxf(wb, uni(s_bar));
        } else {
            bar = fmaxf(bar, uni(s_bar));
        }
#else
        const float wb = wave_max_uniform(best_s);
        if (lane == 0 && wb > bar) __hip_atomic_fetch_max(&s_bar, wb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        bar = fmaxf(wb, uni(s_bar));
#endif
        thr = (bar - kNoiseC) * temp;
    }
    if (piece == kP2Splits - 1 && nvec * VEC < V) {  // the ragged tail's partial group, by thread 0
        const int t0 = nvec * VEC, cnt = V - t0;
        if (threadIdx.x == 0) {
            float xs[VEC];
            float xm = -INFINITY;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                xs[k] = k < cnt ? to_f<T>(row[t0 + k]) : -INFINITY;
                xm = fmaxf(xm, xs[k] >= xlo ? xs[k] : -INFINITY);
            }
            const uint32_t h = ehash(key, keyb, (uint32_t)t0 >> 3);
            if constexpr (TOPP) {
                if (split) {
                    uint32_t n2 = 0u;
#pragma unroll
                    for (int k = 0; k < VEC; ++k) n2 += xs[k] == xc ? 1u : 0u;
                    if (n2) {
                        uint32_t p = __hip_atomic_fetch_add(pend_nt + 2 * row_i, n2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                        for (int k = 0; k < VEC; ++k)
                            if (xs[k] == xc) {
                                if (p < (uint32_t)kPTieCap) st_wt(ties + (int64_t)row_i * kPTieCap + p, t0 + k);
                                ++p;
                            }
                    }
                }
            }
            if (xm > -INFINITY) {
                const float Eg = group_min_e(h);
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    if (xs[k] >= xlo) {
                        const float sc = noise_score(xs[k], inv_t, t0 + k, h, Eg, key2);
                        if (better(sc, t0 + k, Best{best_s, best_i})) {
                            best_s = sc;
                            best_i = t0 + k;
                        }
                    }
            }
        }
    }
    // the piece's best: lanes, waves; stored write-through, every storing wave drained, then the
    // arrival (the last piece merges)
    Best best{best_s, best_i};
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float os = __shfl_xor(best.score, off, kWave);
        const int oi = __shfl_xor(best.idx, off, kWave);
        if (better(os, oi, best)) best = Best{os, oi};
    }
    if (lane == 0) {
        s_bs[w] = best.score;
        s_bi[w] = best.idx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        Best b{s_bs[0], s_bi[0]};
        for (int j = 1; j < NW; ++j)
            if (better(s_bs[j], s_bi[j], b)) b = Best{s_bs[j], s_bi[j]};
        Best* dst = parts + (int64_t)row_i * kP2Splits + piece;
        st_wt(&dst->score, b.score);
        st_wt(&dst->idx, b.idx);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (every wave that stored ties)
    __syncthreads();
    if (!arrive_last(pend_nt + 2 * row_i + 1, (unsigned)kP2Splits, &s_last)) return;
    Best b{-INFINITY, 0x7fffffff};
    if (threadIdx.x == 0) {
        for (int j = 0; j < kP2Splits; ++j) {
            const Best q = parts[(int64_t)row_i * kP2Splits + j];
            if (better(q.score, q.idx, b)) b = q;
        }
    }
    int icut = split ? -1 : 0x7fffffff;
    if (TOPP && split) {  // rank kc's elements by index: the first c are admissible, scored exactly here
        const int n = (int)min(pend_nt[2 * row_i], (uint32_t)kPTieCap);
        for (int i = threadIdx.x; i < n; i += NT) s_tidx[i] = ties[(int64_t)row_i * kPTieCap + i];
        if (threadIdx.x == 0) s_icut = -1;
        __syncthreads();
        Best tb{-INFINITY, 0x7fffffff};
        for (int i = threadIdx.x; i < n; i += NT) {
            const int ii = s_tidx[i];
            int r = 0;
            for (int j = 0; j < n; ++j) r += s_tidx[j] < ii ? 1 : 0;
            if (r < st.c) {
                const uint32_t h = ehash(key, keyb, (uint32_t)ii >> 3);
                const float sc = noise_score(xc, inv_t, ii, h, group_min_e(h), key2);
                if (better(sc, ii, tb)) tb = Best{sc, ii};
            }
            if (r == st.c - 1) s_icut = ii;  // the cut's last kept index (filter_row's ic)
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float os = __shfl_xor(tb.score, off, kWave);
            const int oi = __shfl_xor(tb.idx, off, kWave);
            if (better(os, oi, tb)) tb = Best{os, oi};
        }
        if (lane == 0) {
            s_bs[w] = tb.score;
            s_bi[w] = tb.idx;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int j = 0; j < NW; ++j)
                if (better(s_bs[j], s_bi[j], b)) b = Best{s_bs[j], s_bi[j]};
        icut = s_icut;
    }
    if (threadIdx.x == 0) {
        tokens[row_i] = b.idx;
        if (logp_out) logp_out[row_i] = (b.idx >= 0 && b.idx < V) ? to_f<T>(row[b.idx]) - st.lse : __builtin_nanf("");
#ifdef SKYRL_TP_REASON
        filt[row_i] = RowFilter{st.mx, filt[row_i].tk, kRowDone, st.kc, icut};
#else
        filt[row_i] = RowFilter{st.mx, 0u, kRowDone, st.kc, icut};
#endif
    }
}

constexpr int kMaxSplits = 64;

// Splits per row: below knobs().sampler_split_rows rows the row is cut into chunks of a multiple of
// knobs().sampler_split_gran elements (default 8192 = one full streaming iteration of a 256-thread
// split, so every split runs the pipelined main loop, not the ragged-tail path) for about
// knobs().sampler_split_wgs workgroups in all; at or above it one 512-thread workgroup owns a row.
int splits_for(int nseq, int V) {
    if (nseq <= 0 || V <= 0 || nseq >= knobs().sampler_split_rows || nseq >= kMaxSplitRows) return 1;
    const int s0 = (knobs().sampler_split_wgs + nseq - 1) / nseq;
    const int64_t g = knobs().sampler_split_gran;
    int64_t chunk = ((int64_t)(V + s0 - 1) / s0 + g - 1) / g * g;
    if ((V + chunk - 1) / chunk > kMaxSplits) chunk = ((int64_t)(V + kMaxSplits - 1) / kMaxSplits + g - 1) / g * g;
    const int s = (int)((V + chunk - 1) / chunk);  // every split non-empty (launch_sample's chunk is <= this one)
    return s < 1 ? 1 : s;
}

size_t ws_align(size_t b) { return (b + 255) / 256 * 256; }
// the split partials' region: sized for the most splits any setting gives, so a workspace
// allocated once stays valid under every variant
size_t parts_bytes(int nseq) { return ws_align((size_t)nseq * kMaxSplits * sizeof(Part)); }

template <typename T, int MODE>
void launch_mode(dim3 grid, bool row_mode, hipStream_t stream, const T* lg, int64_t ld, int V, int chunk, float inv_t,
                 int use_topk, int use_minp, float ln_min_p, uint64_t seed, const int64_t* seq_ids, int64_t step,
                 int use_topp, const RowFilter* filt, int32_t* tokens, float* logp, Part* parts, unsigned* counters) {
    if (row_mode && knobs().sampler_row == 1)
        hipLaunchKernelGGL((sample_kernel<T, MODE, 512, true>), grid, dim3(512), 0, stream, lg, ld, V, chunk, inv_t,
                           use_topk, use_minp, ln_min_p, seed, seq_ids, step, use_topp, filt, tokens, logp, parts,
                           counters);
    else if (row_mode || knobs().sampler_split_nt == 512)
        hipLaunchKernelGGL((sample_kernel<T, MODE, 512>), grid, dim3(512), 0, stream, lg, ld, V, chunk, inv_t, use_topk,
                           use_minp, ln_min_p, seed, seq_ids, step, use_topp, filt, tokens, logp, parts, counters);
    else
        hipLaunchKernelGGL((sample_kernel<T, MODE, kThreads>), grid, dim3(kThreads), 0, stream, lg, ld, V, chunk, inv_t,
                           use_topk, use_minp, ln_min_p, seed, seq_ids, step, use_topp, filt, tokens, logp, parts,
                           counters);
}

// T = 1 in row mode takes the multiplicative bound on the lse exponentials (MODE 3); split
// launches take the additive form (MODE 1), which measured faster there (64 / 128 rows: 14.85 /
// 18.31 vs 15.14 / 18.64 us; 512 rows in row mode: 35.67 vs 33.35 us, same tokens;
// profiles/r05_sampler_t1mode_ab.json). Probe builds set SKYRL_T1_MODE to 1 to time row mode
// through the additive form.
#ifndef SKYRL_T1_MODE
#define SKYRL_T1_MODE 3
#endif
template <typename T>
int launch_sample(const void* logits, int64_t ld, int nseq, int V, float temperature, int top_k, float top_p,
                  float min_p, uint64_t seed, const int64_t* seq_ids, int64_t step, int32_t* tokens, float* logp,
                  void* ws, hipStream_t stream) {
    const int nsplit = splits_for(nseq, V);
    int chunk = (V + nsplit - 1) / nsplit;
    chunk = nsplit > 1 ? (chunk + knobs().sampler_split_gran - 1) / knobs().sampler_split_gran * knobs().sampler_split_gran
                       : (chunk + 15) & ~15;
    char* w = reinterpret_cast<char*>(ws);
    unsigned* counters = reinterpret_cast<unsigned*>(w);
    size_t off = kCounterBytes;
    RowFilter* filt = reinterpret_cast<RowFilter*>(w + off);
    off += ws_align((size_t)nseq * sizeof(RowFilter));
    Part* parts = reinterpret_cast<Part*>(w + off);
    const int greedy = temperature == 0.f;
    const int use_topk = !greedy && top_k > 0 && top_k < V;
    const int use_minp = !greedy && min_p > 0.f;
    const int use_topp = !greedy && top_p < 1.f;
    const float inv_t = greedy ? 1.f : 1.0f / temperature;
    const float ln_min_p = use_minp ? det_ln(min_p) : 0.f;
    const T* lg = reinterpret_cast<const T*>(logits);
    // top_k <= kFastK on 16-B aligned rows: the one-pass kernel alone (rows its candidate lists
    // cannot settle run the pre-pass's and MODE 2's code inside it)
    const bool fast = knobs().sampler_topk_fast && use_topk && top_k <= kFastK &&
                      (reinterpret_cast<uintptr_t>(logits) & 15) == 0 && ((ld * (int64_t)sizeof(T)) & 15) == 0;
    if (fast) {
        hipLaunchKernelGGL(sample_topk_kernel<T>, dim3(nseq), dim3(kFastNT), 0, stream, lg, ld, V, top_k, inv_t, use_minp,
                           ln_min_p, use_topp, use_topp ? top_p : 1.0f, seed, seq_ids, step, tokens, logp, filt);
        return check_launch("sample_topk_kernel");
    }
    // top_p / min_p without top_k on 16-B aligned bf16 rows: the two-pass kernel alone
    if constexpr (sizeof(T) == 2) {
        const int probe = knobs().topp_probe ? knobs().topp_probe : SKYRL_TP_PROBE0;
        if (knobs().sampler_topp_fast && !use_topk &&
            (use_topp || (use_minp && (knobs().sampler_topp_fast == 2 || nseq >= knobs().sampler_split_rows))) &&
            V <= kP2Splits * 8 * kPNT * 8 &&
            (reinterpret_cast<uintptr_t>(logits) & 15) == 0 &&
            ((ld * (int64_t)sizeof(T)) & 15) == 0) {
            // the pass-2 kernel's per-row state after the split sampler's parts (never used by this path)
            char* pw = w + off + parts_bytes(nseq);
            ToppPending* pend = reinterpret_cast<ToppPending*>(pw);
            pw += ws_align((size_t)nseq * sizeof(ToppPending));
            unsigned* pend_nt = reinterpret_cast<unsigned*>(pw);  // per row: tie count, arrival counter
            pw += ws_align((size_t)nseq * 2 * sizeof(unsigned));
            Best* pparts = reinterpret_cast<Best*>(pw);
            pw += ws_align((size_t)nseq * kP2Splits * sizeof(Best));
            int32_t* pties = reinterpret_cast<int32_t*>(pw);
            if (use_topp)
                hipLaunchKernelGGL((sample_topp_kernel<T, true>), dim3(nseq), dim3(kPNT), 0, stream, lg, ld, V, inv_t,
                                   use_minp, ln_min_p, top_p, seed, seq_ids, step, tokens, logp, filt, pend, pend_nt,
                                   probe);
            else
                hipLaunchKernelGGL((sample_topp_kernel<T, false>), dim3(nseq), dim3(kPNT), 0, stream, lg, ld, V, inv_t,
                                   use_minp, ln_min_p, 1.0f, seed, seq_ids, step, tokens, logp, filt, pend, pend_nt,
                                   probe);
            int rc = check_launch("sample_topp_kernel");
            if (rc || !use_topp || (probe >= 1 && probe <= 4) || probe == 11) return rc;  // (probes 1-4, 11)
            hipLaunchKernelGGL((sample_topp_pass2_kernel<T, true>), dim3(nseq, kP2Splits), dim3(kPNT), 0, stream, lg, ld,
                               V, inv_t, seed, seq_ids, step, tokens, logp, filt, pend, pend_nt, pties, pparts);
            return check_launch("sample_topp_pass2_kernel");
        }
    }
    if (use_topk || use_minp || use_topp) {
        hipLaunchKernelGGL(sample_filter_kernel<T>, dim3(nseq), dim3(kFT), 0, stream, lg, ld, V, use_topk ? top_k : 0,
                           use_minp, inv_t, ln_min_p, use_topp ? top_p : 1.0f, filt);
        int rc = check_launch("sample_filter_kernel");
        if (rc) return rc;
    }
    const dim3 grid(nseq, nsplit);
    const bool row_mode = nsplit == 1 && nseq >= knobs().sampler_split_rows;
    if (greedy)
        launch_mode<T, 0>(grid, row_mode, stream, lg, ld, V, chunk, inv_t, 0, 0, ln_min_p, seed, seq_ids, step, 0,
                          filt, tokens, logp, parts, counters);
    else if (use_topk || use_minp || use_topp)
        launch_mode<T, 2>(grid, row_mode, stream, lg, ld, V, chunk, inv_t, use_topk, use_minp, ln_min_p, seed, seq_ids,
                          step, use_topp, filt, tokens, logp, parts, counters);
    else if (temperature == 1.0f && row_mode)
        launch_mode<T, SKYRL_T1_MODE>(grid, row_mode, stream, lg, ld, V, chunk, inv_t, 0, 0, ln_min_p, seed, seq_ids, step, 0,
                          filt, tokens, logp, parts, counters);
    else
        launch_mode<T, 1>(grid, row_mode, stream, lg, ld, V, chunk, inv_t, 0, 0, ln_min_p, seed, seq_ids, step, 0,
                          filt, tokens, logp, parts, counters);
    return check_launch("sample_kernel");
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" size_t skyrl_sample_workspace_bytes(int32_t nseq, int32_t V) {
    return kCounterBytes + ws_align((size_t)nseq * sizeof(RowFilter)) +
           parts_bytes(nseq) + ws_align((size_t)nseq * sizeof(ToppPending)) +
           ws_align((size_t)nseq * 2 * sizeof(unsigned)) + ws_align((size_t)nseq * kP2Splits * sizeof(Best)) +
           (size_t)nseq * kPTieCap * sizeof(int32_t) + 256;
}

extern "C" int skyrl_sample(const void* logits, int dtype, int64_t ld, int32_t nseq, int32_t V, float temperature,
                            int32_t top_k, float top_p, float min_p, uint64_t seed, const int64_t* seq_ids,
                            int64_t step, int32_t* tokens_out, float* logp_out, void* workspace, void* stream) {
    SKYRL_REQUIRE(nseq >= 0 && V > 0, "sample: bad sizes");
    if (nseq == 0) return SKYRL_OK;
    SKYRL_REQUIRE(logits && tokens_out && workspace, "sample: null pointer");
    SKYRL_REQUIRE(temperature >= 0.f, "sample: temperature must be >= 0");
    SKYRL_REQUIRE(min_p >= 0.f && min_p <= 1.f, "sample: min_p must be in [0,1]");
    SKYRL_REQUIRE(top_p >= 0.f && top_p <= 1.f, "sample: top_p must be in [0,1]");
    if (dtype == SKYRL_BF16)
        return launch_sample<uint16_t>(logits, ld, nseq, V, temperature, top_k, top_p, min_p, seed, seq_ids, step,
                                       tokens_out, logp_out, workspace, as_stream(stream));
    if (dtype == SKYRL_F32)
        return launch_sample<float>(logits, ld, nseq, V, temperature, top_k, top_p, min_p, seed, seq_ids, step,
                                    tokens_out, logp_out, workspace, as_stream(stream));
    return fail(SKYRL_ERR_INVALID, "sample: logits dtype must be bf16 or f32");
}
