/* Sanitizer driver for sampler_ref.c (TEST INFRASTRUCTURE ONLY): built by `make -C oracle
 * sanitize` with -fsanitize=address,undefined and run by tests/test_oracle_sanitizer.py. It drives
 * the C restatement over bf16 and f32 rows at odd and tiny vocabularies, with every filter
 * combination, strided rows and greedy, and checks the invariants every decision must hold
 * (token in range and admissible, logprob <= 0, greedy = the first maximum). Any out-of-bounds
 * access, use after free or undefined behaviour aborts the run. */
#include "sampler_ref.c"

#include <stdio.h>
#include <string.h>

static uint32_t rng_state = 12345u;
static uint32_t rng(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 17;
    rng_state ^= rng_state << 5;
    return rng_state;
}
static float frand(void) { return (float)(rng() >> 8) * (1.0f / 16777216.0f); }
static uint16_t to_bf16(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return (uint16_t)(u >> 16);
}

static int check(int V, int nseq, int is_bf16, int64_t ld, float T, int top_k, float top_p, float min_p) {
    const size_t elems = (size_t)ld * (size_t)nseq;
    void* logits = malloc(elems * (is_bf16 ? 2 : 4));
    int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * (size_t)nseq);
    int32_t* tok = (int32_t*)malloc(sizeof(int32_t) * (size_t)nseq);
    float* lp = (float*)malloc(sizeof(float) * (size_t)nseq);
    uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)V);
    int i, v, bad = 0;
    for (i = 0; i < nseq; ++i) ids[i] = 3 * i + 1;
    for (size_t e = 0; e < elems; ++e) {
        const float x = (frand() - 0.5f) * 12.0f;
        const float q = (rng() & 7u) == 0u ? 1.5f : x;  /* some ties */
        if (is_bf16) ((uint16_t*)logits)[e] = to_bf16(q);
        else ((float*)logits)[e] = q;
    }
    sampler_ref(logits, is_bf16, ld, nseq, V, T, top_k, top_p, min_p, 77u, ids, 5, tok, lp, keys);
    for (i = 0; i < nseq; ++i) {
        if (tok[i] < 0 || tok[i] >= V) { bad = 1; break; }
        if (!(lp[i] <= 1e-6f)) { bad = 1; break; }
        if (T == 0.0f) {  /* greedy: the first maximum */
            float best = -INFINITY;
            int bi = -1;
            for (v = 0; v < V; ++v) {
                const float x = is_bf16 ? bf16f(((uint16_t*)logits)[(size_t)i * ld + v]) : ((float*)logits)[(size_t)i * ld + v];
                if (x > best) { best = x; bi = v; }
            }
            if (tok[i] != bi) { bad = 1; break; }
        }
    }
    free(logits);
    free(ids);
    free(tok);
    free(lp);
    free(keys);
    if (bad) fprintf(stderr, "invariant failed: V=%d nseq=%d bf16=%d T=%g k=%d p=%g minp=%g\n", V, nseq, is_bf16, T, top_k,
                     top_p, min_p);
    return bad;
}

int main(void) {
    static const int vocabs[] = {1, 2, 7, 8, 9, 63, 257, 1031, 4100};
    static const float temps[] = {0.0f, 1.0f, 0.7f};
    int fails = 0, a, b, f;
    for (a = 0; a < (int)(sizeof(vocabs) / sizeof(vocabs[0])); ++a) {
        for (b = 0; b < 3; ++b) {
            for (f = 0; f < 4; ++f) {
                const int V = vocabs[a];
                const int top_k = f == 1 ? (V > 3 ? 3 : 1) : -1;
                const float top_p = f == 2 ? 0.8f : 1.0f;
                const float min_p = f == 3 ? 0.05f : 0.0f;
                fails += check(V, 5, 1, V + (a & 1) * 3, temps[b], top_k, top_p, min_p);
                fails += check(V, 3, 0, V, temps[b], top_k, top_p, min_p);
            }
        }
    }
    printf("sampler_ref sanitizer driver: %d failures\n", fails);
    return fails ? 1 : 0;
}
