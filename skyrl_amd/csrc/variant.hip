// Per-call kernel variants (ABI 11): the tuned defaults, the variant a *_ex call runs with, and
// the *_ex entry points. SURVEY §8(b) asks for reentrant entry points without global mutable
// state; the A/B knobs that once lived in process-wide variables set by skyrl_tune are now a
// caller-owned skyrl_variant passed to one call. While an _ex call runs, a thread-local pointer
// names its validated variant (restored when the call returns, so nested and concurrent calls
// on other threads see their own); outside an _ex call every kernel reads the defaults.
#include "variant.h"

#include <string>

namespace skyrl {
using detail::tl_knobs;

int VariantScope::enter(const skyrl_variant* v) {
    prev_ = tl_knobs;
    active_ = true;
    if (!v) {
        tl_knobs = &kDefaultKnobs;
        return SKYRL_OK;
    }
    k_ = kDefaultKnobs;
    auto take = [&](int32_t field, int& dst, auto ok, const char* name) -> int {
        if (field == SKYRL_VARIANT_DEFAULT) return SKYRL_OK;
        if (!ok(field)) return fail(SKYRL_ERR_INVALID, std::string("skyrl_variant: bad value for ") + name);
        dst = field;
        return SKYRL_OK;
    };
    auto in = [](int lo, int hi) { return [lo, hi](int x) { return x >= lo && x <= hi; }; };
    auto one_of = [](std::initializer_list<int> xs) {
        return [xs](int x) {
            for (int y : xs)
                if (x == y) return true;
            return false;
        };
    };
    int rc = SKYRL_OK;
#define SKYRL_TAKE(f, pred) \
    if (!rc) rc = take(v->f, k_.f, pred, #f)
    SKYRL_TAKE(logprob_unroll, one_of({4, 8}));
    SKYRL_TAKE(logprob_nt, in(0, 1));
    SKYRL_TAKE(train_resident, in(0, 1));
    SKYRL_TAKE(train_resident_nt, one_of({768, 1024}));
    SKYRL_TAKE(train_ntstore, in(0, 1));
    SKYRL_TAKE(train_split, in(0, 1));
    SKYRL_TAKE(train_split_shape, in(0, 5));
    SKYRL_TAKE(train_split_wait, in(0, 100000000));
    SKYRL_TAKE(grpo_slices, one_of({1, 2, 4}));
    SKYRL_TAKE(loss_units, one_of({0, 1, 2, 4}));
    SKYRL_TAKE(loss_bwd_blocks, in(1, 4096));
    SKYRL_TAKE(grpo_loss_rpb, one_of({1, 2}));
    SKYRL_TAKE(finish_mode, in(0, 4));
    SKYRL_TAKE(sampler_row, in(0, 1));
    SKYRL_TAKE(sampler_split_rows, in(1, 1024));
    SKYRL_TAKE(sampler_split_wgs, in(64, 16384));
    SKYRL_TAKE(sampler_split_nt, one_of({256, 512}));
    SKYRL_TAKE(sampler_split_gran, [](int x) { return x >= 2048 && x <= 65536 && x % 2048 == 0; });
    SKYRL_TAKE(sampler_topk_fast, in(0, 1));
    SKYRL_TAKE(sampler_topp_fast, in(0, 2));
    SKYRL_TAKE(topp_probe, [](int x) { return (x >= 0 && x <= 7) || x == 11; });
    SKYRL_TAKE(lmhead_pipe, in(-1, 14));
    SKYRL_TAKE(lmhead_group, in(0, 4095));
    SKYRL_TAKE(attn_pf, one_of({0, 4, 6, 8}));
    SKYRL_TAKE(lmhead_persist, in(0, 4));
#undef SKYRL_TAKE
    if (rc) {
        active_ = false;  // nothing installed
        return rc;
    }
    if (k_.lmhead_pipe < 0) k_.lmhead_pipe = kDefaultKnobs.lmhead_pipe;
    tl_knobs = &k_;
    return SKYRL_OK;
}

VariantScope::~VariantScope() {
    if (active_) tl_knobs = prev_;
}

}  // namespace skyrl

extern "C" void skyrl_variant_init(skyrl_variant* v) {
    if (!v) return;
    int32_t* f = reinterpret_cast<int32_t*>(v);
    for (size_t i = 0; i < sizeof(skyrl_variant) / sizeof(int32_t); ++i) f[i] = SKYRL_VARIANT_DEFAULT;
}

// ---- the *_ex entry points: the plain entry point under the call's variant ----------------------
extern "C" int skyrl_grpo_advantage_ex(const float* rewards, const float* scores_in, const void* response_mask, int mask_dtype, const int32_t* group_off, const int32_t* group_rows, int32_t num_groups, int32_t N, int32_t R, float epsilon, int32_t norm_by_std, float* advantages, float* scores_out, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_grpo_advantage(rewards, scores_in, response_mask, mask_dtype, group_off, group_rows, num_groups, N, R, epsilon, norm_by_std, advantages, scores_out, stream);
}

extern "C" int skyrl_ppo_loss_fwd_ex(const float* log_probs, const float* old_log_probs, const float* advantages, const float* loss_mask, const float* ref_log_probs, const float* entropy, const float* row_mask_sum, int32_t n, int32_t R, const skyrl_ppo_params* params, float* loss_out, float* metrics_out, float* grad_logp, float* grad_entropy, int32_t flags, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_ppo_loss_fwd(log_probs, old_log_probs, advantages, loss_mask, ref_log_probs, entropy, row_mask_sum, n, R, params, loss_out, metrics_out, grad_logp, grad_entropy, flags, workspace, stream);
}

extern "C" int skyrl_grpo_ppo_loss_fwd_ex(const float* rewards, const float* scores, const void* response_mask, int mask_dtype, int32_t num_groups, float epsilon, int32_t norm_by_std, const float* log_probs, const float* old_log_probs, const float* loss_mask, const float* ref_log_probs, const float* entropy, const float* row_mask_sum, int32_t n, int32_t R, const skyrl_ppo_params* params, float* advantages, float* loss_out, float* metrics_out, float* grad_logp, float* grad_entropy, int32_t flags, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_grpo_ppo_loss_fwd(rewards, scores, response_mask, mask_dtype, num_groups, epsilon, norm_by_std, log_probs, old_log_probs, loss_mask, ref_log_probs, entropy, row_mask_sum, n, R, params, advantages, loss_out, metrics_out, grad_logp, grad_entropy, flags, workspace, stream);
}

extern "C" int skyrl_ppo_loss_bwd_ex(const float* grad_out, int64_t numel, float* grad_logp, float* grad_entropy, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_ppo_loss_bwd(grad_out, numel, grad_logp, grad_entropy, stream);
}

extern "C" int skyrl_ppo_loss_finish_ex(const float* grad_out, float* grad_logp, float* grad_entropy, int32_t n, int32_t R, const skyrl_ppo_params* params, float* loss_out, float* metrics_out, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_ppo_loss_finish(grad_out, grad_logp, grad_entropy, n, R, params, loss_out, metrics_out, workspace, stream);
}

extern "C" int skyrl_logprob_fwd_ex(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t nb, int32_t nt, int32_t V, const int64_t* labels, int64_t lstride_b, int64_t lstride_t, float temperature, float* logp_out, float* entropy_out, float* lse_out, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_logprob_fwd(logits, dtype, stride_b, stride_t, nb, nt, V, labels, lstride_b, lstride_t, temperature, logp_out, entropy_out, lse_out, stream);
}

extern "C" int skyrl_logprob_bwd_ex(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t nb, int32_t nt, int32_t V, const int64_t* labels, int64_t lstride_b, int64_t lstride_t, float temperature, const float* lse, const float* entropy, const float* grad_logp, const float* grad_entropy, void* grad_logits, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_logprob_bwd(logits, dtype, stride_b, stride_t, nb, nt, V, labels, lstride_b, lstride_t, temperature, lse, entropy, grad_logp, grad_entropy, grad_logits, stream);
}

extern "C" int skyrl_lmhead_gemm_ex(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t M, int32_t N, int32_t K, void* out, int64_t ld_out, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_lmhead_gemm(hidden, ld_hidden, weight, ld_weight, M, N, K, out, ld_out, stream);
}

extern "C" int skyrl_lmhead_logprob_fwd_ex(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t T, int32_t V, int32_t K, const int64_t* labels, int64_t label_stride, float temperature, float* logp_out, float* entropy_out, float* lse_out, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_lmhead_logprob_fwd(hidden, ld_hidden, weight, ld_weight, T, V, K, labels, label_stride, temperature, logp_out, entropy_out, lse_out, workspace, stream);
}

extern "C" int skyrl_lmhead_sample_ex(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t M, int32_t V, int32_t K, float temperature, uint64_t seed, const int64_t* seq_ids, int64_t step, int32_t* tokens_out, float* logp_out, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_lmhead_sample(hidden, ld_hidden, weight, ld_weight, M, V, K, temperature, seed, seq_ids, step, tokens_out, logp_out, workspace, stream);
}

extern "C" int skyrl_policy_train_fwd_ex(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t n, int32_t R, int32_t V, const int64_t* labels, int64_t lstride_b, int64_t lstride_t, float temperature, const float* old_log_probs, const float* advantages, const float* loss_mask, const float* ref_log_probs, const skyrl_ppo_params* params, float* loss_out, float* metrics_out, float* logp_out, float* entropy_out, void* grad_logits, int64_t gstride_b, int64_t gstride_t, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_policy_train_fwd(logits, dtype, stride_b, stride_t, n, R, V, labels, lstride_b, lstride_t, temperature, old_log_probs, advantages, loss_mask, ref_log_probs, params, loss_out, metrics_out, logp_out, entropy_out, grad_logits, gstride_b, gstride_t, workspace, stream);
}

extern "C" int skyrl_policy_train_ragged_fwd_ex(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V, const int64_t* labels, const int32_t* token_pos, int32_t n, int32_t R, float temperature, const float* old_log_probs, const float* advantages, const float* loss_mask, const float* ref_log_probs, const skyrl_ppo_params* params, float* loss_out, float* metrics_out, float* logp_out, float* entropy_out, void* grad_logits, int64_t ld_grad, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_policy_train_ragged_fwd(logits, dtype, ld, ntok, V, labels, token_pos, n, R, temperature, old_log_probs, advantages, loss_mask, ref_log_probs, params, loss_out, metrics_out, logp_out, entropy_out, grad_logits, ld_grad, workspace, stream);
}

extern "C" int skyrl_policy_train_micro_fwd_ex(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V, const int64_t* labels, int64_t label_stride_b, int64_t label_stride_t, const int32_t* token_pos, int32_t micro, int32_t n_total, int32_t R, int32_t micro_rows, float temperature, const float* old_log_probs, const float* advantages, const float* loss_mask, const float* ref_log_probs, const skyrl_ppo_params* params, float* logp_out, float* entropy_out, void* grad_logits, int64_t ld_grad, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_policy_train_micro_fwd(logits, dtype, ld, ntok, V, labels, label_stride_b, label_stride_t, token_pos, micro, n_total, R, micro_rows, temperature, old_log_probs, advantages, loss_mask, ref_log_probs, params, logp_out, entropy_out, grad_logits, ld_grad, workspace, stream);
}

// (a query: -1 for an invalid variant, never a status code that reads as "supported")
extern "C" int skyrl_policy_train_supports_ex(int32_t V, int32_t aligned, float temperature, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (scope.enter(variant)) return -1;
    return skyrl_policy_train_supports(V, aligned, temperature);
}

extern "C" int skyrl_sample_ex(const void* logits, int dtype, int64_t ld, int32_t nseq, int32_t V, float temperature, int32_t top_k, float top_p, float min_p, uint64_t seed, const int64_t* seq_ids, int64_t step, int32_t* tokens_out, float* logp_out, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_sample(logits, dtype, ld, nseq, V, temperature, top_k, top_p, min_p, seed, seq_ids, step, tokens_out, logp_out, workspace, stream);
}

extern "C" int skyrl_paged_decode_ex(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache, const int32_t* block_tables, int64_t bt_stride, const int32_t* context_lens, int32_t nseq, int32_t nh, int32_t nkv, int32_t head_dim, float scale, int32_t part_tokens, int32_t nparts, void* out, int64_t out_stride, void* workspace, void* stream, const skyrl_variant* variant) {
    skyrl::VariantScope scope;
    if (int rc = scope.enter(variant)) return rc;
    return skyrl_paged_decode(q, q_stride, k_cache, v_cache, block_tables, bt_stride, context_lens, nseq, nh, nkv, head_dim, scale, part_tokens, nparts, out, out_stride, workspace, stream);
}
