/*
 * sampler_ref.c — sequential CPU restatement of the skyrl_sample algorithm
 * (TEST INFRASTRUCTURE ONLY: the checker for skyrl_amd/csrc/sampler.hip).
 *
 * The reference's rollout sampler is vLLM 0.13.0 (skyrl-train/pyproject.toml:135),
 * third-party and absent here; its token stream is not pinned by any reference test
 * (tests/gpu/utils.py:222-236 compares text similarity only). The build therefore
 * defines its own counter-based sampler with the reference's filter semantics
 * (skyrl-tx/tx/utils/generator.py:213-227,398-449: temperature; top_k keeping exactly k
 * tokens, the k largest with equal values taken in index order (lax.top_k + the first-k
 * mask, :410-418; fixture skyrl-tx/tests/utils/test_generator.py:197-207); min_p relative
 * to the max probability (vLLM's, not in tx); top_p on the top_k-filtered distribution
 * keeping tokens in descending order (stable argsort, ties in index order) while the mass
 * strictly before them is < p, the top token always (:433-449; fixture :210-238); greedy at
 * T == 0; logprob of the sampled token from the raw logits),
 * and this file is its oracle:
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

/* Pair hash from 24-bit products (restates ehash in skyrl_amd/csrc/sampler.hip). */
static uint32_t mul24(uint32_t a, uint32_t b) { return (a & 0xffffffu) * (b & 0xffffffu); }
static uint32_t ehash(uint32_t ka, uint32_t kb, uint32_t p) {
    uint32_t h = mul24(p, 0x9e3779u) + ka;
    h ^= h >> 16;
    h = mul24(h, 0x85ebcau) + kb;
    h ^= h >> 16;
    h = mul24(h, 0xc2b2aeu);
    h ^= h >> 16;
    return h;
}

/* Element v's noise -ln E_v, E_v ~ Exp(1) drawn per group g = v >> 3 through the order
 * statistics of 8 draws (restates the noise model of sample_kernel): h = ehash(key, keyb, g),
 * the group minimum E_g = -ln(u_g) / 8 with u_g = (((h >> 16 ^ 0xffff) << 8) | (h >> 8 & 0xff)
 * | 1) 2^-24 sits at slot p = h & 7; any other slot is E_g + (-ln U_v) with U_v = ((hash32(key2
 * ^ v phi) >> 8) | 1) 2^-24. key2 = hash32(key ^ 0x5bd1e995), keyb = hash32(key ^ 0x27d4eb2f). */
static float gumbel(uint32_t key, uint32_t v) {
    uint32_t key2 = hash32(key ^ 0x5bd1e995u);
    uint32_t keyb = hash32(key ^ 0x27d4eb2fu);
    uint32_t h = ehash(key, keyb, v >> 3);
    uint32_t t16 = (h >> 16) ^ 0xffffu;
    float ug = (float)(((t16 << 8) | ((h >> 8) & 0xffu)) | 1u) * 5.9604644775390625e-8f;
    float E = -det_ln(ug) * 0.125f;
    if ((v & 7u) != (h & 7u)) {
        uint32_t hu = hash32(key2 ^ (v * 0x9e3779b1u));
        float U = (float)((hu >> 8) | 1u) * 5.9604644775390625e-8f;
        E = E + (-det_ln(U));
    }
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


/* deterministic 2^y for y <= 0 (0 below -126): same operations as det_exp2 in sampler.hip */
static float det_exp2(float y) {
    const float yc = y >= -126.0f ? y : -126.0f;
    const float fi = floorf(yc);
    const float f = yc - fi;
    float p = 2.170088992e-04f, r;
    uint32_t b;
    p = fmaf(p, f, 1.243957202e-03f);
    p = fmaf(p, f, 9.678921662e-03f);
    p = fmaf(p, f, 5.548325926e-02f);
    p = fmaf(p, f, 2.402298748e-01f);
    p = fmaf(p, f, 6.931470037e-01f);
    p = fmaf(p, f, 1.0f);
    memcpy(&b, &p, 4);
    b += (uint32_t)(int)fi << 23;
    memcpy(&r, &b, 4);
    return y >= -126.0f ? r : 0.0f;
}
/* fixed-point top_p mass 2^31 e^((x - max)/T) */
static uint32_t mass_q(float x, float mx, float inv_t) {
    const float y = ((x - mx) * inv_t) * 1.4426950408889634f;
    return (uint32_t)(det_exp2(y) * 2147483648.0f);
}

typedef struct {
    uint32_t key;
    int idx;
    uint32_t q;
} kept_t;
static int cmp_kept(const void* a, const void* b) {
    const kept_t* x = (const kept_t*)a;
    const kept_t* y = (const kept_t*)b;
    if (x->key != y->key) return x->key < y->key ? 1 : -1; /* key descending */
    return (x->idx > y->idx) - (x->idx < y->idx);          /* index ascending */
}

/* top_k cut (1-based k): sort (key, index) by key descending / index ascending, keep the
 * first k; the cut is the k-th entry's (key, index), and a key equal to the cut key stays
 * only at an index <= the cut index (INT_MAX when the whole tie group fits in k). */
static void topk_cut(kept_t* all, int V, int k, uint32_t* tk, int* ik) {
    qsort(all, (size_t)V, sizeof(kept_t), cmp_kept);
    *tk = all[k - 1].key;
    *ik = (k < V && all[k].key == all[k - 1].key) ? all[k - 1].idx : 0x7fffffff;
}
static int in_cut(uint32_t kk, int v, uint32_t kcut, int icut) { return kk > kcut || (kk == kcut && v <= icut); }

/* The filtered support of one row (temperature, top_k, min_p, top_p): a token v stays iff
 * in_cut(key, v, tk, ik) (top_k), x/T >= mthr (min_p) and in_cut(key, v, kc, ic) (top_p). */
typedef struct {
    int use_topk, use_minp, use_topp;
    uint32_t tk, kc;
    int ik, ic;
    float inv_t, mthr, mx;
} row_filter_t;

static float row_x(const uint16_t* rb, const float* rf, int v) { return rb ? bf16f(rb[v]) : rf[v]; }
static uint32_t row_key_of(const uint16_t* rb, const float* rf, int v) { return rb ? okey_bf16(rb[v]) : okey_f32(rf[v]); }

static row_filter_t row_filter(const uint16_t* rb, const float* rf, int V, float temperature, int top_k, float top_p,
                               float min_p, kept_t* kept) {
    row_filter_t f;
    int v;
    const int greedy = temperature == 0.0f;
    f.use_topk = !greedy && top_k > 0 && top_k < V;
    f.use_minp = !greedy && min_p > 0.0f;
    f.use_topp = !greedy && top_p < 1.0f;
    f.tk = 0;
    f.ik = 0x7fffffff;
    f.kc = 0;
    f.ic = 0x7fffffff;
    f.inv_t = greedy ? 1.0f : 1.0f / temperature;
    f.mthr = 0.0f;
    f.mx = -3.402823466e38f;
    for (v = 0; v < V; ++v) f.mx = fmaxf(f.mx, row_x(rb, rf, v));
    if (f.use_topk) {
        for (v = 0; v < V; ++v) {
            kept[v].key = row_key_of(rb, rf, v);
            kept[v].idx = v;
            kept[v].q = 0;
        }
        topk_cut(kept, V, top_k, &f.tk, &f.ik);
    }
    if (f.use_minp) f.mthr = f.mx * f.inv_t + det_ln(min_p);
    if (f.use_topp) {
        /* kept set (top_k and min_p), sorted by key desc / index asc; first key group whose
         * cumulative mass reaches p*Z is the cut; its first c tokens (index order) stay */
        int nk = 0, g;
        uint64_t Z = 0, cum = 0;
        double target;
        for (v = 0; v < V; ++v) {
            const uint32_t kk = row_key_of(rb, rf, v);
            const float x = row_x(rb, rf, v);
            if (f.use_topk && !in_cut(kk, v, f.tk, f.ik)) continue;
            if (f.use_minp && x * f.inv_t < f.mthr) continue;
            kept[nk].key = kk;
            kept[nk].idx = v;
            kept[nk].q = mass_q(x, f.mx, f.inv_t);
            Z += kept[nk].q;
            ++nk;
        }
        qsort(kept, (size_t)nk, sizeof(kept_t), cmp_kept);
        target = (double)top_p * (double)Z;
        for (g = 0; g < nk;) {
            uint64_t gm = 0;
            int e = g;
            while (e < nk && kept[e].key == kept[g].key) gm += kept[e++].q;
            if ((double)(cum + gm) >= target || e == nk) {
                const uint64_t qc = kept[g].q;
                long long c;
                f.kc = kept[g].key;
                if (qc == 0) {
                    c = e - g;
                } else {
                    c = 0;
                    while ((double)(cum + (uint64_t)c * qc) < target) ++c;
                }
                if (g == 0 && c < 1) c = 1;
                if (c < e - g) f.ic = kept[g + c - 1].idx;
                break;
            }
            cum += gm;
            g = e;
        }
    }
    return f;
}

static int row_keeps(const row_filter_t* f, const uint16_t* rb, const float* rf, int v) {
    const uint32_t kk = row_key_of(rb, rf, v);
    if (f->use_topk && !in_cut(kk, v, f->tk, f->ik)) return 0;
    if (f->use_minp && row_x(rb, rf, v) * f->inv_t < f->mthr) return 0;
    if (f->use_topp && !in_cut(kk, v, f->kc, f->ic)) return 0;
    return 1;
}

/*
 * The filtered support as a 0/1 mask per element (keep: uint8 [nseq, V]); the -inf pattern of
 * apply_top_k_batch / apply_top_p_batch, checked against tx's fixtures by the CPU tests.
 */
void sampler_ref_support(const void* logits, int is_bf16, int64_t ld, int nseq, int V, float temperature, int top_k,
                         float top_p, float min_p, uint8_t* keep) {
    int i, v;
    kept_t* kept = (kept_t*)malloc(sizeof(kept_t) * (size_t)V);
    for (i = 0; i < nseq; ++i) {
        const uint16_t* rb = is_bf16 ? (const uint16_t*)logits + (int64_t)i * ld : NULL;
        const float* rf = is_bf16 ? NULL : (const float*)logits + (int64_t)i * ld;
        const row_filter_t f = row_filter(rb, rf, V, temperature, top_k, top_p, min_p, kept);
        for (v = 0; v < V; ++v) keep[(int64_t)i * V + v] = (uint8_t)(temperature == 0.0f || row_keeps(&f, rb, rf, v));
    }
    free(kept);
}

/*
 * logits: nseq rows of V elements, row stride ld; is_bf16 selects uint16 bf16 vs f32.
 * keys: unused (kept for the binding's signature). tokens/logp: outputs.
 */
void sampler_ref(const void* logits, int is_bf16, int64_t ld, int nseq, int V, float temperature, int top_k,
                 float top_p, float min_p, uint64_t seed, const int64_t* seq_ids, int64_t step, int32_t* tokens,
                 float* logp, uint32_t* keys) {
    int i, v;
    kept_t* kept = (kept_t*)malloc(sizeof(kept_t) * (size_t)V);
    (void)keys;
    for (i = 0; i < nseq; ++i) {
        const uint16_t* rb = is_bf16 ? (const uint16_t*)logits + (int64_t)i * ld : NULL;
        const float* rf = is_bf16 ? NULL : (const float*)logits + (int64_t)i * ld;
        const int greedy = temperature == 0.0f;
        const uint32_t key = row_key(seed, seq_ids ? seq_ids[i] : (int64_t)i, step);
        const row_filter_t f = row_filter(rb, rf, V, temperature, top_k, top_p, min_p, kept);
        float best = -INFINITY;
        int best_i = 0x7fffffff;
        double s = 0.0;
        for (v = 0; v < V; ++v) {
            const float x = row_x(rb, rf, v);
            float sc;
            s += exp((double)x - (double)f.mx);
            if (greedy) {
                sc = x;
            } else {
                if (!row_keeps(&f, rb, rf, v)) continue;
                sc = x * f.inv_t + gumbel(key, (uint32_t)v);
            }
            if (sc > best || (sc == best && v < best_i)) {
                best = sc;
                best_i = v;
            }
        }
        tokens[i] = best_i;
        if (logp) logp[i] = (float)((double)row_x(rb, rf, best_i) - ((double)f.mx + log(s)));
    }
    free(kept);
}
