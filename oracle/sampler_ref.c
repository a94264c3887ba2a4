/*
 * sampler_ref.c — sequential CPU restatement of the skyrl_sample algorithm
 * (TEST INFRASTRUCTURE ONLY: the checker for skyrl_amd/csrc/sampler.hip).
 *
 * The reference's rollout sampler is vLLM 0.13.0 (skyrl-train/pyproject.toml:135),
 * third-party and absent here; its token stream is not pinned by any reference test
 * (tests/gpu/utils.py:222-236 compares text similarity only). The build therefore
 * defines its own counter-based sampler with the reference's filter semantics
 * (skyrl-tx/tx/utils/generator.py:213-227,398-449: temperature, top_k keeping values
 * >= the k-th largest, min_p relative to the max probability, greedy at T == 0,
 * logprob of the sampled token from the raw logits), and this file is its oracle:
 * one thread, elements in index order, every decision-path float operation an IEEE
 * basic op or fmaf, compiled with -ffp-contract=off. Tokens must match bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

static uint32_t row_key(uint64_t seed, int64_t seq, int64_t step) {
    uint32_t k = hash32((uint32_t)seed ^ 0x9e3779b9u);
    k = hash32(k ^ (uint32_t)(seed >> 32));
    k = hash32(k ^ (uint32_t)((uint64_t)seq));
    k = hash32(k ^ (uint32_t)((uint64_t)seq >> 32));
    k = hash32(k ^ (uint32_t)((uint64_t)step));
    k = hash32(k ^ (uint32_t)((uint64_t)step >> 32));
    return k;
}

/* ln for positive normal floats, branch-free: ix = bits - bits(2/3), e = ix >> 23,
 * mantissa rebased into [2/3, 4/3), ln(1+z) = z*P6(z). */
static float det_ln(float y) {
    uint32_t bits, ix, mb;
    float m, z, p;
    int e;
    memcpy(&bits, &y, 4);
    ix = bits - 0x3f2aaaabu;
    e = (int32_t)ix >> 23;
    mb = (ix & 0x007fffffu) + 0x3f2aaaabu;
    memcpy(&m, &mb, 4);
    z = m - 1.0f;
    p = 0.16302786767482758f;
    p = fmaf(p, z, -0.18978701531887054f);
    p = fmaf(p, z, 0.19917640089988708f);
    p = fmaf(p, z, -0.24900923669338226f);
    p = fmaf(p, z, 0.3333371579647064f);
    p = fmaf(p, z, -0.5000061392784119f);
    p = fmaf(p, z, 1.0f);
    return fmaf((float)e, 0.693147180559945f, z * p);
}

/* Element v's uniform: u = ((t16 << 8) | lo8 | 1) * 2^-24, t16 = 65535 - h16 with h16 =
 * half (v & 1) of hash32(key ^ (v >> 1) * phi), lo8 = top byte of hash32(key2 ^ v * phi),
 * key2 = hash32(key ^ 0x5bd1e995). g = -ln(-ln u). */
static float gumbel(uint32_t key, uint32_t v) {
    uint32_t key2 = hash32(key ^ 0x5bd1e995u);
    uint32_t t16 = ((hash32(key ^ ((v >> 1) * 0x9e3779b1u)) >> (16 * (v & 1))) & 0xffffu) ^ 0xffffu;
    uint32_t lo8 = hash32(key2 ^ (v * 0x9e3779b1u)) >> 24;
    float u = (float)(((t16 << 8) | lo8) | 1u) * 5.9604644775390625e-8f;
    float E = -det_ln(u);
    return -det_ln(E);
}

static float bf16f(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static uint32_t okey_bf16(uint16_t h) { return (h & 0x8000u) ? (uint32_t)(uint16_t)~h : (uint32_t)(h | 0x8000u); }
static uint32_t okey_f32(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

/* k-th largest key (1-based k): sort a copy descending. */
static int cmp_desc(const void* a, const void* b) {
    const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return (x < y) - (x > y);
}
static uint32_t kth_key(uint32_t* keys, int V, int k) {
    qsort(keys, (size_t)V, sizeof(uint32_t), cmp_desc);
    return keys[k - 1];
}

/*
 * logits: nseq rows of V elements, row stride ld; is_bf16 selects uint16 bf16 vs f32.
 * keys: scratch uint32[V]. tokens/logp: outputs.
 */
void sampler_ref(const void* logits, int is_bf16, int64_t ld, int nseq, int V, float temperature, int top_k,
                 float min_p, uint64_t seed, const int64_t* seq_ids, int64_t step, int32_t* tokens, float* logp,
                 uint32_t* keys) {
    int i, v;
    for (i = 0; i < nseq; ++i) {
        const uint16_t* rb = is_bf16 ? (const uint16_t*)logits + (int64_t)i * ld : NULL;
        const float* rf = is_bf16 ? NULL : (const float*)logits + (int64_t)i * ld;
#define X(vv) (is_bf16 ? bf16f(rb[vv]) : rf[vv])
        const int greedy = temperature == 0.0f;
        const int use_topk = !greedy && top_k > 0 && top_k < V;
        const int use_minp = !greedy && min_p > 0.0f;
        const float inv_t = greedy ? 1.0f : 1.0f / temperature;
        const uint32_t key = row_key(seed, seq_ids ? seq_ids[i] : (int64_t)i, step);
        uint32_t tk = 0;
        float mthr = 0.0f, mx = -3.402823466e38f, best = -INFINITY;
        int best_i = 0x7fffffff;
        double s = 0.0;
        for (v = 0; v < V; ++v) mx = fmaxf(mx, X(v));
        if (use_topk) {
            for (v = 0; v < V; ++v) keys[v] = is_bf16 ? okey_bf16(rb[v]) : okey_f32(rf[v]);
            tk = kth_key(keys, V, top_k);
        }
        if (use_minp) mthr = mx * inv_t + det_ln(min_p);
        for (v = 0; v < V; ++v) {
            const float x = X(v);
            float sc;
            s += exp((double)x - (double)mx);
            if (greedy) {
                sc = x;
            } else {
                const float xs = x * inv_t;
                if (use_topk && (is_bf16 ? okey_bf16(rb[v]) : okey_f32(rf[v])) < tk) continue;
                if (use_minp && xs < mthr) continue;
                sc = xs + gumbel(key, (uint32_t)v);
            }
            if (sc > best || (sc == best && v < best_i)) {
                best = sc;
                best_i = v;
            }
        }
        tokens[i] = best_i;
        if (logp) logp[i] = (float)((double)X(best_i) - ((double)mx + log(s)));
#undef X
    }
}
