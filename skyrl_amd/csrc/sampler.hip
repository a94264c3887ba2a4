// a1: rollout token sampling with sampled-token logprob.
//
// Replaces the vLLM sampler behind VLLMInferenceEngine.generate
// (skyrl-train/skyrl_train/inference_engines/vllm/vllm_engine.py:196-218,
// logprob extraction :139-149; params inference_engines/utils.py:15-42,
// defaults config/ppo_base_config.yaml:316-324). Filter semantics follow
// skyrl-tx/tx/utils/generator.py:213-227,398-449: temperature first, then
// top_k (keep values >= k-th largest, ties kept), then min_p; T == 0 is greedy
// over the raw logits; the returned logprob is log_softmax(raw logits)[token].
//
// Sampling is Gumbel-max, argmax_v (x_v/T + g_v), with g = -ln(-ln u) and u
// from a counter-based integer hash of (seed, seq_id, step, v). Every float
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

#pragma clang fp contract(off)

namespace skyrl {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kGumbelMax = 17.0f;  // > -ln(-ln(1-2^-24)) = 16.64: bound for the skip test

__host__ __device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ uint32_t row_key(uint64_t seed, int64_t seq, int64_t step) {
    uint32_t k = hash32((uint32_t)seed ^ 0x9e3779b9u);
    k = hash32(k ^ (uint32_t)(seed >> 32));
    k = hash32(k ^ (uint32_t)((uint64_t)seq));
    k = hash32(k ^ (uint32_t)((uint64_t)seq >> 32));
    k = hash32(k ^ (uint32_t)((uint64_t)step));
    k = hash32(k ^ (uint32_t)((uint64_t)step >> 32));
    return k;
}

// Deterministic natural log for normal positive floats: exponent/mantissa split,
// mantissa in [sqrt(.5), sqrt(2)), ln(1+z) = z*P7(z) by fmaf Horner.
__host__ __device__ __forceinline__ float det_ln(float y) {
    const uint32_t bits = __builtin_bit_cast(uint32_t, y);
    int e = (int)(bits >> 23) - 127;
    uint32_t mb = (bits & 0x007fffffu) | 0x3f800000u;
    float m = __builtin_bit_cast(float, mb);
    if (m > 1.41421356f) {
        m = m * 0.5f;
        e += 1;
    }
    const float z = m - 1.0f;
    float p = 0.11931054294109344f;
    p = fmaf(p, z, -0.1868075132369995f);
    p = fmaf(p, z, 0.20491759479045868f);
    p = fmaf(p, z, -0.24908289313316345f);
    p = fmaf(p, z, 0.33314675092697144f);
    p = fmaf(p, z, -0.5000114440917969f);
    p = fmaf(p, z, 1.0000009536743164f);
    const float r = z * p;
    return fmaf((float)e, 0.693147180559945f, r);
}

__device__ __forceinline__ float gumbel(uint32_t key, uint32_t v) {
    const uint32_t r = hash32(key ^ (v * 0x9e3779b1u));
    const float u = (float)((r >> 8) | 1u) * 5.9604644775390625e-8f;  // odd / 2^24, exact
    const float E = -det_ln(u);
    return -det_ln(E);
}

// order-preserving unsigned keys
__device__ __forceinline__ uint32_t okey_bf16(uint16_t h) {
    return (h & 0x8000u) ? (uint32_t)(uint16_t)~h : (uint32_t)(h | 0x8000u);
}
__device__ __forceinline__ uint32_t okey_f32(uint32_t u) { return (u & 0x80000000u) ? ~u : (u | 0x80000000u); }

struct Best {
    float score;
    int idx;
};
__device__ __forceinline__ bool better(float s, int i, const Best& b) {
    return s > b.score || (s == b.score && i < b.idx);
}

struct Part {  // per (row, split) partial
    float score;
    int idx;
    float m;
    float s;
};

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<uint16_t>(uint16_t v) { return bf16_to_f32(v); }
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <typename T>
__device__ __forceinline__ uint32_t okey(T v);
template <> __device__ __forceinline__ uint32_t okey<uint16_t>(uint16_t v) { return okey_bf16(v); }
template <> __device__ __forceinline__ uint32_t okey<float>(float v) { return okey_f32(__float_as_uint(v)); }

// ---- pre-pass: per-row top_k key threshold (radix select) and raw max --------
template <typename T>
__global__ __launch_bounds__(kThreads) void sample_filter_kernel(const T* __restrict__ logits, int64_t ld, int V,
                                                                 int top_k, uint32_t* __restrict__ thr_key,
                                                                 float* __restrict__ row_max) {
    __shared__ unsigned hist[256];
    __shared__ uint32_t s_prefix, s_k;
    __shared__ float s_max[kWaves];
    const T* row = logits + (int64_t)blockIdx.x * ld;
    float mx = -3.402823466e38f;
    for (int i = threadIdx.x; i < V; i += kThreads) mx = fmaxf(mx, to_f<T>(row[i]));
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x / kWave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = s_max[0];
        for (int j = 1; j < kWaves; ++j) m = fmaxf(m, s_max[j]);
        row_max[blockIdx.x] = m;
    }
    if (top_k <= 0 || top_k >= V) {
        if (threadIdx.x == 0) thr_key[blockIdx.x] = 0u;  // keep everything
        return;
    }
    constexpr int kBits = sizeof(T) * 8;
    if (threadIdx.x == 0) {
        s_prefix = 0u;
        s_k = (uint32_t)top_k;
    }
    for (int shift = kBits - 8; shift >= 0; shift -= 8) {
        for (int j = threadIdx.x; j < 256; j += kThreads) hist[j] = 0u;
        __syncthreads();
        const uint32_t prefix = s_prefix;
        const uint32_t hi_mask = (shift + 8 >= 32) ? 0u : (0xffffffffu << (shift + 8));
        for (int i = threadIdx.x; i < V; i += kThreads) {
            const uint32_t k = okey<T>(row[i]);
            if ((k & hi_mask) == (prefix & hi_mask)) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t need = s_k, cum = 0u;
            int d = 255;
            for (; d > 0; --d) {
                if (cum + hist[d] >= need) break;
                cum += hist[d];
            }
            s_k = need - cum;
            s_prefix = prefix | ((uint32_t)d << shift);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) thr_key[blockIdx.x] = s_prefix;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void sample_kernel(
    const T* __restrict__ logits, int64_t ld, int V, int chunk, float inv_t, int greedy, int use_topk,
    int use_minp, float ln_min_p, uint64_t seed, const int64_t* __restrict__ seq_ids, int64_t step,
    const uint32_t* __restrict__ thr_key, const float* __restrict__ row_max, int32_t* __restrict__ tokens,
    float* __restrict__ logp_out, Part* __restrict__ parts, unsigned* __restrict__ counters) {
    __shared__ Part s_part[kWaves];
    __shared__ int s_last;
    const int row_i = blockIdx.x;
    const int split = blockIdx.y;
    const int nsplit = gridDim.y;
    const int lane = threadIdx.x & (kWave - 1);
    const T* row = logits + (int64_t)row_i * ld;
    const int v_beg = split * chunk;
    const int v_end = min(V, v_beg + chunk);
    const uint32_t key = row_key(seed, seq_ids ? seq_ids[row_i] : (int64_t)row_i, step);
    const uint32_t tk = use_topk ? thr_key[row_i] : 0u;
    const float mthr = use_minp ? row_max[row_i] * inv_t + ln_min_p : 0.f;

    Best best{-INFINITY, 0x7fffffff};
    float m = -3.402823466e38f, s = 0.f;  // raw online softmax for the logprob
    auto visit = [&](T raw, int v) {
        const float x = to_f<T>(raw);
        {  // lse of the raw logits (not on the decision path)
            const float mn = fmaxf(m, x);
            s = s * exp2f((m - mn) * kLog2e) + exp2f(fmaxf(x - mn, -1e30f) * kLog2e);
            m = mn;
        }
        if (greedy) {
            if (better(x, v, best)) best = Best{x, v};
            return;
        }
        const float xs = x * inv_t;
        if (use_topk && okey<T>(raw) < tk) return;
        if (use_minp && xs < mthr) return;
        // Skip the noise when it cannot win: fl(xs+g) <= fl(xs+17) <= best, and a
        // tie loses on index because a thread visits its elements in ascending v.
        if (best.score != -INFINITY && xs + kGumbelMax <= best.score) return;
        const float sc = xs + gumbel(key, (uint32_t)v);
        if (better(sc, v, best)) best = Best{sc, v};
    };
    constexpr int VEC = 16 / sizeof(T);
    const bool vec_ok = (reinterpret_cast<uintptr_t>(row + v_beg) % 16) == 0;
    int v0 = v_beg;
    if (vec_ok) {
        const int nvec = (v_end - v_beg) / VEC;
        const uint4* rv = reinterpret_cast<const uint4*>(row + v_beg);
        for (int i = threadIdx.x; i < nvec; i += kThreads) {
            uint4 pk = rv[i];
            T vals[VEC];
            memcpy(vals, &pk, 16);
#pragma unroll
            for (int k = 0; k < VEC; ++k) visit(vals[k], v_beg + i * VEC + k);
        }
        v0 = v_beg + nvec * VEC;
    }
    for (int v = v0 + threadIdx.x; v < v_end; v += kThreads) visit(row[v], v);

    // wave reduce: best (score desc, idx asc) and (m, s)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float os = __shfl_xor(best.score, off, kWave);
        const int oi = __shfl_xor(best.idx, off, kWave);
        if (better(os, oi, best)) best = Best{os, oi};
        const float om = __shfl_xor(m, off, kWave);
        const float oss = __shfl_xor(s, off, kWave);
        const float mn = fmaxf(m, om);
        s = s * exp2f((m - mn) * kLog2e) + oss * exp2f((om - mn) * kLog2e);
        m = mn;
    }
    if (lane == 0) s_part[threadIdx.x / kWave] = Part{best.score, best.idx, m, s};
    __syncthreads();
    if (threadIdx.x == 0) {
        Part p = s_part[0];
        for (int j = 1; j < kWaves; ++j) {
            const Part q = s_part[j];
            Best b{p.score, p.idx};
            if (better(q.score, q.idx, b)) {
                p.score = q.score;
                p.idx = q.idx;
            }
            const float mn = fmaxf(p.m, q.m);
            p.s = p.s * exp2f((p.m - mn) * kLog2e) + q.s * exp2f((q.m - mn) * kLog2e);
            p.m = mn;
        }
        parts[(int64_t)row_i * nsplit + split] = p;
    }
    if (nsplit > 1) {
        if (!arrive_last(counters + row_i, (unsigned)nsplit, &s_last)) return;
    } else {
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        Part p = parts[(int64_t)row_i * nsplit];
        for (int j = 1; j < nsplit; ++j) {
            const Part q = parts[(int64_t)row_i * nsplit + j];
            Best b{p.score, p.idx};
            if (better(q.score, q.idx, b)) {
                p.score = q.score;
                p.idx = q.idx;
            }
            const float mn = fmaxf(p.m, q.m);
            p.s = p.s * exp2f((p.m - mn) * kLog2e) + q.s * exp2f((q.m - mn) * kLog2e);
            p.m = mn;
        }
        tokens[row_i] = p.idx;
        if (logp_out) {
            const float lse = p.m + log2f(p.s) * kLn2;
            logp_out[row_i] = (p.idx >= 0 && p.idx < V) ? to_f<T>(row[p.idx]) - lse : __builtin_nanf("");
        }
    }
    if (nsplit > 1) rearm(counters + row_i);
}

int splits_for(int nseq, int V) {
    int s = (2048 + nseq - 1) / nseq;
    const int max_s = (V + 4095) / 4096;  // at least 4096 elements per split
    if (s > max_s) s = max_s;
    if (s > 64) s = 64;
    return s < 1 ? 1 : s;
}

template <typename T>
int launch_sample(const void* logits, int64_t ld, int nseq, int V, float temperature, int top_k, float min_p,
                  uint64_t seed, const int64_t* seq_ids, int64_t step, int32_t* tokens, float* logp, void* ws,
                  hipStream_t stream) {
    const int nsplit = splits_for(nseq, V);
    int chunk = (V + nsplit - 1) / nsplit;
    chunk = (chunk + 15) & ~15;
    char* w = reinterpret_cast<char*>(ws);
    unsigned* counters = reinterpret_cast<unsigned*>(w);
    size_t off = (((size_t)nseq * 4 + 255) / 256) * 256;
    uint32_t* thr = reinterpret_cast<uint32_t*>(w + off);
    off += (((size_t)nseq * 4 + 255) / 256) * 256;
    float* rmax = reinterpret_cast<float*>(w + off);
    off += (((size_t)nseq * 4 + 255) / 256) * 256;
    Part* parts = reinterpret_cast<Part*>(w + off);
    const int greedy = temperature == 0.f;
    const int use_topk = !greedy && top_k > 0 && top_k < V;
    const int use_minp = !greedy && min_p > 0.f;
    const float inv_t = greedy ? 1.f : 1.0f / temperature;
    const float ln_min_p = use_minp ? det_ln(min_p) : 0.f;
    const T* lg = reinterpret_cast<const T*>(logits);
    if (use_topk || use_minp) {
        hipLaunchKernelGGL(sample_filter_kernel<T>, dim3(nseq), dim3(kThreads), 0, stream, lg, ld, V,
                           use_topk ? top_k : 0, thr, rmax);
        int rc = check_launch("sample_filter_kernel");
        if (rc) return rc;
    }
    hipLaunchKernelGGL(sample_kernel<T>, dim3(nseq, nsplit), dim3(kThreads), 0, stream, lg, ld, V, chunk, inv_t,
                       greedy, use_topk, use_minp, ln_min_p, seed, seq_ids, step, thr, rmax, tokens, logp, parts,
                       counters);
    return check_launch("sample_kernel");
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" size_t skyrl_sample_workspace_bytes(int32_t nseq, int32_t V) {
    const size_t a = (((size_t)nseq * 4 + 255) / 256) * 256;
    return 3 * a + (size_t)nseq * splits_for(nseq, V) * sizeof(Part) + 256;
}

extern "C" int skyrl_sample(const void* logits, int dtype, int64_t ld, int32_t nseq, int32_t V, float temperature,
                            int32_t top_k, float min_p, uint64_t seed, const int64_t* seq_ids, int64_t step,
                            int32_t* tokens_out, float* logp_out, void* workspace, void* stream) {
    SKYRL_REQUIRE(nseq >= 0 && V > 0, "sample: bad sizes");
    if (nseq == 0) return SKYRL_OK;
    SKYRL_REQUIRE(logits && tokens_out && workspace, "sample: null pointer");
    SKYRL_REQUIRE(temperature >= 0.f, "sample: temperature must be >= 0");
    SKYRL_REQUIRE(min_p >= 0.f && min_p <= 1.f, "sample: min_p must be in [0,1]");
    if (dtype == SKYRL_BF16)
        return launch_sample<uint16_t>(logits, ld, nseq, V, temperature, top_k, min_p, seed, seq_ids, step, tokens_out,
                                       logp_out, workspace, as_stream(stream));
    if (dtype == SKYRL_F32)
        return launch_sample<float>(logits, ld, nseq, V, temperature, top_k, min_p, seed, seq_ids, step, tokens_out,
                                    logp_out, workspace, as_stream(stream));
    return fail(SKYRL_ERR_INVALID, "sample: logits dtype must be bf16 or f32");
}
