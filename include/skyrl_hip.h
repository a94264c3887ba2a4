/*
 * skyrl_hip.h — C ABI of libskyrl_hip.so, the MI355X (gfx950) hot path of the
 * skyrl-train GRPO/PPO actor-learner loop.
 *
 * Every entry point:
 *   - takes device pointers, element counts/strides and a hipStream_t (passed as void*),
 *   - never allocates; scratch comes from the caller (see *_workspace_bytes),
 *   - is stream-ordered and never synchronises the host,
 *   - returns 0 on success or a SKYRL_ERR_* code; skyrl_last_error() returns a
 *     thread-local message describing the last failure on the calling thread.
 *
 * Reference interfaces each entry point replaces are cited as
 * path:line under /root/reference/skyrl-train/skyrl_train/ (snapshot 2026-02-27).
 * The reference has no FFI of its own (pure Python/PyTorch); the binding a
 * maintainer would add is the ctypes stub in INTEGRATION.md.
 */
#ifndef SKYRL_HIP_H
#define SKYRL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------- */
#define SKYRL_OK 0
#define SKYRL_ERR_INVALID 1   /* bad argument (shape, dtype, null pointer) */
#define SKYRL_ERR_LAUNCH 2    /* hipGetLastError() after a launch was not hipSuccess */
#define SKYRL_ERR_UNSUPPORTED 3

/* ---- dtype codes (element type of a tensor argument) -------------------- */
#define SKYRL_F32 0
#define SKYRL_BF16 1
#define SKYRL_I64 2
#define SKYRL_I32 3
#define SKYRL_U8 4   /* bool masks */

/* Thread-local text of the last error on this thread ("" if none). */
const char* skyrl_last_error(void);
/* ABI version; bumped on any signature change (2: skyrl_sample takes top_p; 3: one-launch
 * skyrl_ppo_loss_fwd writing final gradients, in-place skyrl_ppo_loss_bwd, pack emits
 * loss-mask row sums; 4: skyrl_policy_train_fwd takes grad_logits strides; 5: pack emits
 * reward row sums (GRPO scores), skyrl_grpo_advantage / skyrl_grpo_ppo_loss_fwd take them,
 * the loss forwards take flags (SKYRL_LOSS_DEFER_FOLD) and skyrl_ppo_loss_finish; 6:
 * skyrl_policy_train_ragged_fwd, the policy_train workspace holds the split-row exchange; 7:
 * skyrl_comm_* RCCL collectives; 8: the step form of the fused policy pass,
 * skyrl_policy_train_plan / _micro_fwd / _fold; 9: per-parameter AdamW,
 * skyrl_adamw_seg_plan / _seg_update / _seg_tile, skyrl_debug_occupy, skyrl_policy_train_plan_grpo;
 * 10: skyrl_adv_norm_stats / _apply; 11: skyrl_tune and skyrl_debug_occupy removed, per-call
 * kernel variants through skyrl_variant and the *_ex entry points; 12: skyrl_variant.lmhead_persist,
 * the persistent learner lm_head forward). */
int skyrl_abi_version(void);
/* ---- kernel variants, per call ---------------------------------------------------------------
 * Every entry point runs the tuned kernels. The *_ex forms (declared after each family) take a
 * caller-owned skyrl_variant as their LAST argument and run another variant of the same
 * computation for that call only: A/B measurement, and the tests that pin the alternatives
 * against each other. NULL means the tuned defaults, and so does every field left at
 * SKYRL_VARIANT_DEFAULT. The library keeps no mutable state between calls: a variant is read only
 * while its _ex call runs (a bad field value fails that call with SKYRL_ERR_INVALID before any
 * launch). Every variant gives identical results except the split-row fused training pass vs the
 * resident one (another fp32 summation order) and the timing probes topp_probe 1..4 /
 * 6 / 7 / 11 and finish_mode 2..4 (deliberately wrong values). */
#define SKYRL_VARIANT_DEFAULT INT32_MIN
typedef struct skyrl_variant {
    int32_t logprob_unroll;      /* {4, 8}: 16-B loads in flight per lane (logprob fwd / bwd) */
    int32_t logprob_nt;          /* {0, 1}: non-temporal streaming loads of the logits */
    int32_t train_resident;      /* {0, 1}: the fused training pass keeps the row in registers */
    int32_t train_resident_nt;   /* {768, 1024}: threads per register-resident row at V ~ 152K */
    int32_t train_ntstore;       /* {0, 1}: non-temporal dlogits stores */
    int32_t train_split;         /* {0, 1}: split-row fused training pass where it applies */
    int32_t train_split_shape;   /* 0 by vocabulary, 1..5: pieces x threads 8x128, 4x256, 2x512, 5x256, 6x256 */
    int32_t train_split_wait;    /* [0, 1e8] ticks a piece waits for a partner before recomputing it */
    int32_t grpo_slices;         /* {1, 2, 4}: column slices per group (contiguous-group GRPO) */
    int32_t loss_units;          /* {0 auto, 1, 2, 4}: row chunks per block of the fused PPO loss */
    int32_t loss_bwd_blocks;     /* [1, 4096]: grid of skyrl_ppo_loss_finish / _bwd */
    int32_t grpo_loss_rpb;       /* {1, 2}: row chunks per block of the GRPO + loss launch */
    int32_t finish_mode;         /* [0, 4]: 0 block tree, 1 nb first; 2..4 timing probes */
    int32_t sampler_row;         /* {0, 1}: row-mode sampler without / with progress priority */
    int32_t sampler_split_rows;  /* [1, 1024]: rows split over workgroups below this */
    int32_t sampler_split_wgs;   /* [64, 16384]: workgroups a split launch aims at */
    int32_t sampler_split_nt;    /* {256, 512}: threads per split-mode workgroup */
    int32_t sampler_split_gran;  /* multiple of 2048 in [2048, 65536]: split chunk granule (elements) */
    int32_t sampler_topk_fast;   /* {0, 1}: top_k <= 128 through the one-pass kernel */
    int32_t sampler_topp_fast;   /* {0, 1, 2}: top_p / min_p through the one-pass kernel (2: always) */
    int32_t topp_probe;          /* {0 .. 7, 11}: top_p timing probes (0 = product) */
    int32_t lmhead_pipe;         /* -1 default or 0..14: K pipeline of the lm_head MFMA GEMM */
    int32_t lmhead_group;        /* [0, 4096): M tiles per group of its tile order (0 = all) */
    int32_t attn_pf;             /* {0 default, 4, 6, 8}: K/V blocks in flight per D = 128 decode wave */
    int32_t lmhead_persist;      /* [0, 4]: learner lm_head forward on the persistent tile kernel (0: off; 1..4 copy placement) */
} skyrl_variant;
/* Fills every field with SKYRL_VARIANT_DEFAULT (a pure function of its argument). */
void skyrl_variant_init(skyrl_variant* v);

/* ---- a4: GRPO outcome advantage ----------------------------------------
 * Replaces compute_grpo_outcome_advantage (utils/ppo_utils.py:1132-1182) as
 * reached through compute_advantages_and_returns (ppo_utils.py:1190-1214).
 * score[i] = sum_t rewards[i,t]; per uid group: mean, unbiased std (singleton:
 * mean 0, std 1); adv = (score-mean)/(std+eps) (or score-mean); out = adv*mask.
 * scores_in (f32 [N], e.g. skyrl_pack_experience's reward_row_sum) replaces the reward
 * reads when given (rewards may then be NULL).
 * Groups are given in CSR form: rows of group g are group_rows[group_off[g] ..
 * group_off[g+1]) (the host maps the reference's `index` uids to groups).
 * group_off == group_rows == NULL means contiguous groups of G = N/num_groups
 * rows each (the trainer's layout, generators/utils.py:373-393); that form needs
 * G <= 16, R % 4 == 0 and 16-B aligned buffers, and skips the index loads.
 * rewards/out: f32 [N,R] row-major contiguous; mask: [N,R] of mask_dtype.   */
int skyrl_grpo_advantage(const float* rewards, const float* scores_in /* [N] or NULL */,
                         const void* response_mask, int mask_dtype,
                         const int32_t* group_off, const int32_t* group_rows, int32_t num_groups,
                         int32_t N, int32_t R, float epsilon, int32_t norm_by_std,
                         float* advantages, float* scores_out /* [N] or NULL */, void* stream);
int skyrl_grpo_advantage_ex(const float* rewards, const float* scores_in /* [N] or NULL */,
                         const void* response_mask, int mask_dtype,
                         const int32_t* group_off, const int32_t* group_rows, int32_t num_groups,
                         int32_t N, int32_t R, float epsilon, int32_t norm_by_std,
                         float* advantages, float* scores_out /* [N] or NULL */, void* stream,
        const skyrl_variant* variant);

/* ---- a4 (cont.): advantage_batch_normalize --------------------------------
 * Replaces normalize_advantages_dict (utils/ppo_utils.py:127-145) as applied after the
 * advantages when trainer.algorithm.advantage_batch_normalize is set (trainer.py:275-276,
 * fully_async_trainer.py:514-515): mean over EVERY element (unmasked), ss = sum((adv -
 * mean)^2 * mask), rstd = rsqrt(clamp(ss / sum(mask), 1e-8)), out = (adv - mean) * rstd
 * (not re-masked). Two launches so a data-parallel caller can SUM-all-reduce the sums between
 * them (one all-reduce of 5 fp64 scalars):
 *   skyrl_adv_norm_stats  sums_out f64[5] (device) = (sum adv, sum mask, sum adv*mask,
 *                         sum adv^2*mask, n); workspace: skyrl_adv_norm_workspace_bytes(),
 *                         16-B aligned, zeroed once at allocation (the kernel re-arms it).
 *   skyrl_adv_norm_apply  out f32[n] from the (reduced) sums; out may equal advantages.   */
size_t skyrl_adv_norm_workspace_bytes(void);
int skyrl_adv_norm_stats(const float* advantages, const void* response_mask, int mask_dtype, int64_t n,
                         double* sums_out, void* workspace, void* stream);
int skyrl_adv_norm_apply(const float* advantages, int64_t n, const double* sums, float* out, void* stream);

/* ---- a5: GAE + masked whitening ----------------------------------------
 * Replaces compute_gae_advantage_return (ppo_utils.py:1101-1129) and
 * masked_whiten/masked_var (ppo_utils.py:148-172). Recursion over all R
 * positions with no mask (parity trap: padded values leak into the last
 * valid delta). adv is whitened by masked mean / unbiased masked var.
 * workspace: skyrl_gae_workspace_bytes(N) bytes, 16-B aligned.
 * status (int32, device): 0 ok, 1 mask sum == 0, 2 mask sum == 1 (the two
 * ValueErrors of masked_var, ppo_utils.py:157-163).                        */
size_t skyrl_gae_workspace_bytes(int32_t N);
int skyrl_gae_advantage_return(const float* rewards, const float* values, const void* response_mask,
                               int mask_dtype, int32_t N, int32_t R, float gamma, float lambd,
                               float* advantages, float* returns, void* workspace,
                               int32_t* status, void* stream);

/* ---- a6: approximate KL -------------------------------------------------
 * Replaces compute_approx_kl (ppo_utils.py:88-124). kl_type: 0 k1, 1 abs,
 * 2 k2, 3 k3. loss_mask may be NULL. All f32 [n] contiguous.               */
int skyrl_approx_kl(const float* log_probs, const float* log_probs_base, const void* loss_mask,
                    int mask_dtype, int64_t n, int32_t kl_type, float* kl_out, void* stream);

/* ---- a6 (reward side): KL penalty on rewards -----------------------------
 * Replaces RayPPOTrainer.apply_reward_kl_penalty (trainer.py:981-1035):
 * rewards_out = rewards - kl*max(0,coef); metrics_out[0] = avg_kl
 * (mean over rows of masked_mean(kl,mask,-1)), metrics_out[1] = avg_kl_max
 * (mean over rows of max_t |kl|). loss_mask f32 [N,R].                     */
size_t skyrl_reward_kl_workspace_bytes(int32_t N);
int skyrl_reward_kl_penalty(const float* rewards, const float* action_log_probs,
                            const float* base_action_log_probs, const float* loss_mask,
                            int32_t N, int32_t R, int32_t kl_type, float kl_coef,
                            float* rewards_out, float* metrics_out /* [2] device */,
                            void* workspace, void* stream);

/* ---- a7: fused clipped policy loss + KL(ref) + entropy term --------------
 * Replaces ppo_policy_loss (ppo_utils.py:548-586) + reduce_loss (:984-1009)
 * + the loss assembly of PolicyWorkerBase._forward_backward_micro
 * (workers/worker.py:810-876: entropy masked_mean, k-type KL seq-mean then
 * batch-mean, final = pg + kl*coef - H*coef*[use_entropy_loss]).
 * Forward writes the scalar loss, the metric vector and dL/dlogp (and dL/dentropy)
 * for a unit upstream gradient; skyrl_ppo_loss_bwd rescales them for any other.
 * Gradient semantics follow torch autograd of the reference: min() ties split
 * the gradient 1/2-1/2, clamp passes gradient on the closed interval, the KL
 * term carries NO gradient (compute_approx_kl is @torch.no_grad()).         */
typedef struct skyrl_ppo_params {
    float eps_clip_low;
    float eps_clip_high;
    float clip_ratio_c;
    int32_t dual_clip;        /* policy_loss_type == "dual_clip" */
    int32_t loss_reduction;   /* 0 token_mean, 1 sequence_mean, 2 seq_mean_token_sum_norm */
    float max_seq_len;        /* used by seq_mean_token_sum_norm */
    int32_t use_kl_loss;
    int32_t kl_type;          /* 0 k1, 1 abs, 2 k2, 3 k3 */
    float kl_loss_coef;
    int32_t use_entropy_loss;
    float entropy_loss_coef;
    int32_t has_entropy;      /* entropy pointer given: policy_entropy metric */
} skyrl_ppo_params;

/* metric vector layout (f32, device) */
#define SKYRL_M_FINAL_LOSS 0
#define SKYRL_M_POLICY_LOSS 1
#define SKYRL_M_ENTROPY 2
#define SKYRL_M_KL 3
#define SKYRL_M_CLIP_RATIO 4
#define SKYRL_M_MASK_SUM 5
#define SKYRL_M_COUNT 8

size_t skyrl_ppo_loss_workspace_bytes(int32_t n, int32_t R);
/* flags of the loss forwards */
#define SKYRL_LOSS_DEFER_FOLD 1 /* leave the loss/metric fold to skyrl_ppo_loss_finish: the
                                   forward writes gradients and per-block records only, and
                                   loss_out/metrics_out are written by the finish launch */
/* ONE launch (two when row_mask_sum is NULL, plus one when a token_mean total over
 * n > 1024 rows is needed): writes the scalar loss, the metric vector and the FINAL
 * gradients for a unit upstream gradient:
 *   grad_logp[i,t]    = dL/dlogp[i,t]
 *   grad_entropy[i,t] = -entropy_loss_coef*mask/max(sum mask,1) (only when use_entropy_loss;
 *                       pass NULL otherwise).
 * row_mask_sum: f32 [n] per-row sums of loss_mask (skyrl_pack_experience emits them), or
 * NULL to have them computed here. The reduction scales depend on the mask only, so the
 * gradient is final when written. workspace (skyrl_ppo_loss_workspace_bytes) must be zeroed
 * once at allocation; the kernel leaves it re-usable.                                      */
int skyrl_ppo_loss_fwd(const float* log_probs, const float* old_log_probs, const float* advantages,
                       const float* loss_mask /* NULL = all ones */, const float* ref_log_probs,
                       const float* entropy, const float* row_mask_sum /* [n] or NULL */,
                       int32_t n, int32_t R, const skyrl_ppo_params* params,
                       float* loss_out /* [1] */, float* metrics_out /* [SKYRL_M_COUNT] */,
                       float* grad_logp /* [n,R] */, float* grad_entropy /* [n,R] or NULL */,
                       int32_t flags, void* workspace, void* stream);
int skyrl_ppo_loss_fwd_ex(const float* log_probs, const float* old_log_probs, const float* advantages,
                       const float* loss_mask /* NULL = all ones */, const float* ref_log_probs,
                       const float* entropy, const float* row_mask_sum /* [n] or NULL */,
                       int32_t n, int32_t R, const skyrl_ppo_params* params,
                       float* loss_out /* [1] */, float* metrics_out /* [SKYRL_M_COUNT] */,
                       float* grad_logp /* [n,R] */, float* grad_entropy /* [n,R] or NULL */,
                       int32_t flags, void* workspace, void* stream,
        const skyrl_variant* variant);
/* a4 + a7 for a batch that is one micro-batch: skyrl_grpo_advantage (contiguous groups of
 * G = n/num_groups rows; its contiguous-form conditions apply: G <= 16, R % 4 == 0, 16-B
 * aligned rewards/mask/advantages) followed by skyrl_ppo_loss_fwd on its advantages. ONE
 * launch when row_mask_sum is given, every buffer is 16-B aligned, n*ceil(R/1024) <= 2048 and
 * (token_mean) n <= 1024; the two launches otherwise. Outputs are bit-identical to the two calls: advantages
 * (adv*response_mask, f32 [n,R]), loss, metrics, grad_logp, grad_entropy. Replaces
 * compute_grpo_outcome_advantage (ppo_utils.py:1132-1182) + the loss of
 * PolicyWorkerBase._forward_backward_micro (workers/worker.py:810-876) when the mini-batch is
 * the whole batch. scores (f32 [n], pack's reward_row_sum, or NULL) replaces the reward-row
 * reads of the group statistics (rewards may then be NULL). advantages may be NULL on the
 * one-launch layout (not written); response_mask may then be NULL too, and every token of a
 * row uses the row's advantage, which gives the same loss and gradients whenever loss_mask is
 * 0 outside the response (the pack layout). workspace:
 * skyrl_ppo_loss_workspace_bytes(n, R), zeroed once.                                      */
int skyrl_grpo_ppo_loss_fwd(const float* rewards, const float* scores /* [n] or NULL */,
                            const void* response_mask, int mask_dtype,
                            int32_t num_groups, float epsilon, int32_t norm_by_std,
                            const float* log_probs, const float* old_log_probs,
                            const float* loss_mask /* NULL = all ones */, const float* ref_log_probs,
                            const float* entropy, const float* row_mask_sum /* [n] or NULL */,
                            int32_t n, int32_t R, const skyrl_ppo_params* params,
                            float* advantages /* [n,R] */, float* loss_out /* [1] */,
                            float* metrics_out /* [SKYRL_M_COUNT] */, float* grad_logp /* [n,R] */,
                            float* grad_entropy /* [n,R] or NULL */, int32_t flags, void* workspace,
                            void* stream);
int skyrl_grpo_ppo_loss_fwd_ex(const float* rewards, const float* scores /* [n] or NULL */,
                            const void* response_mask, int mask_dtype,
                            int32_t num_groups, float epsilon, int32_t norm_by_std,
                            const float* log_probs, const float* old_log_probs,
                            const float* loss_mask /* NULL = all ones */, const float* ref_log_probs,
                            const float* entropy, const float* row_mask_sum /* [n] or NULL */,
                            int32_t n, int32_t R, const skyrl_ppo_params* params,
                            float* advantages /* [n,R] */, float* loss_out /* [1] */,
                            float* metrics_out /* [SKYRL_M_COUNT] */, float* grad_logp /* [n,R] */,
                            float* grad_entropy /* [n,R] or NULL */, int32_t flags, void* workspace,
                            void* stream,
        const skyrl_variant* variant);
/* Autograd backward of the loss: grad_logp (and grad_entropy, if given) *= grad_out[0] in
 * place; no memory is touched when grad_out[0] == 1 (loss.backward()).                    */
int skyrl_ppo_loss_bwd(const float* grad_out /* [1] device */, int64_t numel, float* grad_logp,
                       float* grad_entropy /* or NULL */, void* stream);
int skyrl_ppo_loss_bwd_ex(const float* grad_out /* [1] device */, int64_t numel, float* grad_logp,
                       float* grad_entropy /* or NULL */, void* stream,
        const skyrl_variant* variant);
/* The backward of a forward run with SKYRL_LOSS_DEFER_FOLD (same workspace, same stream):
 * folds its per-block records into loss_out and metrics_out (bit-identical to the in-launch
 * fold; stream-ordered, no polling) and, when grad_out is given and grad_out[0] != 1,
 * rescales grad_logp (and grad_entropy) [n,R] in place, as skyrl_ppo_loss_bwd. grad_out
 * NULL: fold only. n, R and params as given to the forward. The reference reads loss and
 * metrics after backward (workers/worker.py:876-894).                                      */
int skyrl_ppo_loss_finish(const float* grad_out /* [1] device or NULL */, float* grad_logp,
                          float* grad_entropy /* or NULL */, int32_t n, int32_t R, const skyrl_ppo_params* params,
                          float* loss_out, float* metrics_out, void* workspace, void* stream);
int skyrl_ppo_loss_finish_ex(const float* grad_out /* [1] device or NULL */, float* grad_logp,
                          float* grad_entropy /* or NULL */, int32_t n, int32_t R, const skyrl_ppo_params* params,
                          float* loss_out, float* metrics_out, void* workspace, void* stream,
        const skyrl_variant* variant);

/* ---- a8: clipped value loss ---------------------------------------------
 * Replaces ppo_critic_loss (ppo_utils.py:175-193): 0.5*mean_rows(masked_mean(
 * max((clip(V,old±c)-ret)^2,(V-ret)^2), mask, -1)); value_clip<0 => no clip.
 * Forward writes loss[1], clipfrac[1] and grad_values (for g=1).            */
int skyrl_critic_loss_fwd(const float* values, const float* old_values, const float* returns,
                          const float* loss_mask, int32_t n, int32_t R, float value_clip,
                          float* loss_out, float* clipfrac_out, float* grad_values, void* workspace,
                          void* stream);
size_t skyrl_critic_loss_workspace_bytes(int32_t n, int32_t R);

/* ---- a2/a3: logprob + entropy over the vocabulary ------------------------
 * Replaces logprobs_from_logits (utils/torch_utils.py:115-177, flash-attn CE
 * semantics: fp32 LSE of the (temperature-divided) logits minus the label
 * logit) and chunked_entropy_from_logits (torch_utils.py:59-111) as used by
 * HFModelWrapper.forward (model_wrapper.py:313-363). Row r = (b,t) reads
 * logits + b*stride_b + t*stride_t (elements), V contiguous elements.
 * temperature: logits are divided by it in their own dtype first
 * (model_wrapper.py:314 divides in place in bf16).
 * Outputs (f32 [nb*nt], row-major (b,t)): logp, entropy (NULL skips), lse.  */
int skyrl_logprob_fwd(const void* logits, int dtype, int64_t stride_b, int64_t stride_t,
                      int32_t nb, int32_t nt, int32_t V, const int64_t* labels,
                      int64_t lstride_b, int64_t lstride_t, float temperature, float* logp_out,
                      float* entropy_out, float* lse_out, void* stream);
int skyrl_logprob_fwd_ex(const void* logits, int dtype, int64_t stride_b, int64_t stride_t,
                      int32_t nb, int32_t nt, int32_t V, const int64_t* labels,
                      int64_t lstride_b, int64_t lstride_t, float temperature, float* logp_out,
                      float* entropy_out, float* lse_out, void* stream,
        const skyrl_variant* variant);
/* d logits (same dtype, dense [nb,nt,V]) = (g_lp*(onehot-p) + g_ent*(-p*(logp_v+H)))/T.
 * grad_entropy may be NULL; entropy must be given if grad_entropy is.          */
int skyrl_logprob_bwd(const void* logits, int dtype, int64_t stride_b, int64_t stride_t,
                      int32_t nb, int32_t nt, int32_t V, const int64_t* labels,
                      int64_t lstride_b, int64_t lstride_t, float temperature, const float* lse,
                      const float* entropy, const float* grad_logp, const float* grad_entropy,
                      void* grad_logits, void* stream);
int skyrl_logprob_bwd_ex(const void* logits, int dtype, int64_t stride_b, int64_t stride_t,
                      int32_t nb, int32_t nt, int32_t V, const int64_t* labels,
                      int64_t lstride_b, int64_t lstride_t, float temperature, const float* lse,
                      const float* entropy, const float* grad_logp, const float* grad_entropy,
                      void* grad_logits, void* stream,
        const skyrl_variant* variant);

/* ---- §8(f)1: lm_head-fused logprob + entropy (logits never materialized) ----
 * Replaces the lm_head output -> logits.div_(T) -> logprobs_from_logits +
 * chunked_entropy_from_logits sequence of HFModelWrapper.forward
 * (model_wrapper.py:308-363; torch_utils.py:59-177). The caller cuts V into chunks
 * and, per chunk c (columns [v0, v0+vc)), runs the plain GEMM z = h @ W[v0:v0+vc]^T
 * (bf16 [T,vc], row stride ldz) into one reused buffer, then:
 *   skyrl_lmhead_chunk_fwd  merges z into the per-token state (skyrl_lmhead_state_bytes(T);
 *                           first=1 on chunk 0, which needs no initialized state); on the
 *                           chunk with last=1 writes logp/entropy/lse f32 [T] (entropy,
 *                           lse may be NULL). labels: int64, token r at labels[r*label_stride].
 *   skyrl_lmhead_chunk_bwd  dz (bf16 [T,vc], row stride lddz) = dL/dz for the chunk, from the
 *                           forward's lse/entropy and the upstream grad_logp/grad_entropy
 *                           (grad_entropy may be NULL); same formula as skyrl_logprob_bwd.
 * The caller then accumulates dh += dz @ W_chunk and dW_chunk = dz^T @ h.            */
size_t skyrl_lmhead_state_bytes(int32_t T);
int skyrl_lmhead_chunk_fwd(const void* z, int64_t ldz, int32_t T, int32_t vc, int64_t v0, const int64_t* labels,
                           int64_t label_stride, float temperature, void* state, int32_t first, int32_t last,
                           float* logp_out, float* entropy_out, float* lse_out, void* stream);
/* Vocab-parallel (tensor-parallel lm_head) variant, replacing DistributedLogprob +
 * _VocabParallelEntropy (distributed/megatron/model_utils.py:64-136, 548-578): each rank runs
 * skyrl_lmhead_chunk_fwd over its shard with v0 = global column and last=0 on every chunk, the
 * ranks all-gather their [T] states (skyrl_lmhead_state_bytes(T) each, rank order), and
 * skyrl_lmhead_state_merge folds the nstates states into logp/entropy/lse f32 [T]. The
 * backward is skyrl_lmhead_chunk_bwd on the local shard with the merged lse/entropy.      */
int skyrl_lmhead_state_merge(const void* states, int32_t nstates, int32_t T, float* logp_out, float* entropy_out,
                             float* lse_out, void* stream);
int skyrl_lmhead_chunk_bwd(const void* z, int64_t ldz, int32_t T, int32_t vc, int64_t v0, const int64_t* labels,
                           int64_t label_stride, float temperature, const float* lse, const float* entropy,
                           const float* grad_logp, const float* grad_entropy, void* dz, int64_t lddz,
                           void* stream);

/* ---- §8(f)1 decode side: lm_head GEMM with the sampler in its epilogue ----------------
 * Replaces the rollout step's logits = lm_head(hidden) + sampler sequence (vLLM
 * LogitsProcessor + Sampler behind vllm_engine.py:139-149,196-218; params
 * inference_engines/utils.py:15-42) with one MFMA GEMM whose epilogue runs skyrl_sample's
 * decision on the bf16 logits tile in LDS, so [M,V] logits never reach HBM.
 * hidden bf16 [M,K] (row stride ld_hidden), weight bf16 [V,K] (HF lm_head.weight, row stride
 * ld_weight); K % 64 == 0, strides multiples of 8 elements, operands 16-B aligned.
 *   skyrl_lmhead_gemm    out bf16 [M,N] (row stride ld_out) = hidden @ weight^T (fp32 accumulate,
 *                        round to bf16): the plain GEMM of the same kernel.
 *   skyrl_lmhead_sample  tokens_out int32 [M], logp_out f32 [M] (may be NULL) exactly as
 *                        skyrl_sample(logits = skyrl_lmhead_gemm(...), temperature, top_k=-1,
 *                        top_p=1, min_p=0, seed, seq_ids, step) decides them (tokens bit-exact;
 *                        logp = log_softmax(raw logits)[token]). No top_k/top_p/min_p here:
 *                        callers with filters use the unfused pair. Workspace:
 *                        skyrl_lmhead_sample_workspace_bytes(M, V), 16-B aligned.            */
int skyrl_lmhead_gemm(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t M,
                      int32_t N, int32_t K, void* out, int64_t ld_out, void* stream);
int skyrl_lmhead_gemm_ex(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t M,
                      int32_t N, int32_t K, void* out, int64_t ld_out, void* stream,
        const skyrl_variant* variant);
size_t skyrl_lmhead_sample_workspace_bytes(int32_t M, int32_t V);
/* Learner side (old / ref log-probs, no grad): logp/entropy/lse f32 [T] of log_softmax(bf16(h W^T) / T)
 * at labels (int64, token r at labels[r*label_stride]) with the same kernel's online-softmax
 * epilogue (no [T,V] logits in HBM), one 16-B state per (token, 256-column tile) folded by
 * skyrl_lmhead_state_merge. entropy_out / lse_out may be NULL. Workspace:
 * skyrl_lmhead_logprob_workspace_bytes(T, V), 16-B aligned.                              */
size_t skyrl_lmhead_logprob_workspace_bytes(int32_t T, int32_t V);
int skyrl_lmhead_logprob_fwd(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t T,
                             int32_t V, int32_t K, const int64_t* labels, int64_t label_stride, float temperature,
                             float* logp_out, float* entropy_out, float* lse_out, void* workspace, void* stream);
int skyrl_lmhead_logprob_fwd_ex(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t T,
                             int32_t V, int32_t K, const int64_t* labels, int64_t label_stride, float temperature,
                             float* logp_out, float* entropy_out, float* lse_out, void* workspace, void* stream,
        const skyrl_variant* variant);
int skyrl_lmhead_sample(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t M,
                        int32_t V, int32_t K, float temperature, uint64_t seed, const int64_t* seq_ids, int64_t step,
                        int32_t* tokens_out, float* logp_out, void* workspace, void* stream);
int skyrl_lmhead_sample_ex(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t M,
                        int32_t V, int32_t K, float temperature, uint64_t seed, const int64_t* seq_ids, int64_t step,
                        int32_t* tokens_out, float* logp_out, void* workspace, void* stream,
        const skyrl_variant* variant);

/* ---- a2+a3+a6+a7 fused: the policy training pass ------------------------------
 * One call per micro-batch replaces logprob fwd + fused loss fwd + loss bwd +
 * logprob bwd (same values and gradients as those four, see policy_train.hip):
 * logits bf16 [n,R,V] (row (b,t) at logits + b*stride_b + t*stride_t) -> loss_out[1],
 * metrics_out[SKYRL_M_COUNT], logp_out/entropy_out f32 [n,R], and grad_logits bf16
 * [n,R,V] (row (b,t) at grad_logits + b*gstride_b + t*gstride_t) = dL/dlogits for a unit
 * upstream gradient (rescale with skyrl_scale_bf16_by_device_scalar when the upstream
 * gradient is not 1). Any V and row alignment (GPT-2's odd 50,257 included); the
 * register-resident kernel (V <= 155,648) needs every grad_logits row to sit at the same
 * position within 16 B as its logits row (equal strides mod 8 elements and 16-B-congruent
 * bases), which the dense [n,R,V] layout gives whenever V % 8 == 0.
 * old/adv/mask/ref: f32 [n,R] contiguous. workspace: skyrl_policy_train_workspace_bytes. */
size_t skyrl_policy_train_workspace_bytes(int32_t n, int32_t R);
int skyrl_policy_train_fwd(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t n,
                           int32_t R, int32_t V, const int64_t* labels, int64_t lstride_b,
                           int64_t lstride_t, float temperature, const float* old_log_probs,
                           const float* advantages, const float* loss_mask, const float* ref_log_probs,
                           const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                           float* logp_out, float* entropy_out, void* grad_logits, int64_t gstride_b,
                           int64_t gstride_t, void* workspace,
                           void* stream);
int skyrl_policy_train_fwd_ex(const void* logits, int dtype, int64_t stride_b, int64_t stride_t, int32_t n,
                           int32_t R, int32_t V, const int64_t* labels, int64_t lstride_b,
                           int64_t lstride_t, float temperature, const float* old_log_probs,
                           const float* advantages, const float* loss_mask, const float* ref_log_probs,
                           const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                           float* logp_out, float* entropy_out, void* grad_logits, int64_t gstride_b,
                           int64_t gstride_t, void* workspace,
                           void* stream,
        const skyrl_variant* variant);
/* The same pass over a sample-packed batch (the learner's padding-free layout,
 * model_wrapper.py:272-330 with the lm_head of :308-363): ntok tokens with dense logits rows
 * (row q at logits + q*ld, bf16; V <= 155,648, or <= 114,688 when V % 8 != 0 or rows are not
 * 16-B aligned; each grad_logits row at its logits row's offset within 16 B), labels int64 [ntok], and
 * token_pos int32 [ntok]: token q's position in the padded [n,R] per-token arrays (old / adv /
 * loss_mask / ref in, logp_out / entropy_out out; positions no token maps to must have
 * loss_mask 0 and are left untouched in the outputs). loss / metrics / gradients are those of
 * skyrl_policy_train_fwd on the padded batch, for every loss reduction; grad_logits rows
 * [ntok, V] at grad_logits + q*ld_grad. Same workspace query (n, R). */
int skyrl_policy_train_ragged_fwd(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V,
                                  const int64_t* labels, const int32_t* token_pos, int32_t n, int32_t R,
                                  float temperature, const float* old_log_probs, const float* advantages,
                                  const float* loss_mask, const float* ref_log_probs,
                                  const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                                  float* logp_out, float* entropy_out, void* grad_logits, int64_t ld_grad,
                                  void* workspace, void* stream);
int skyrl_policy_train_ragged_fwd_ex(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V,
                                  const int64_t* labels, const int32_t* token_pos, int32_t n, int32_t R,
                                  float temperature, const float* old_log_probs, const float* advantages,
                                  const float* loss_mask, const float* ref_log_probs,
                                  const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                                  float* logp_out, float* entropy_out, void* grad_logits, int64_t ld_grad,
                                  void* workspace, void* stream,
        const skyrl_variant* variant);
/* Step form: one mini-batch of n_total rows in micro-batches of micro_rows (the last one may be
 * short), the loss folded once per mini-batch. The reference's micro-batch loop
 * (workers/worker.py:731-900) reads loss and metrics only after the mini-batch's backward
 * passes (optim_step, :900-925), and the loss's reduction scales depend on the loss mask only,
 * so: skyrl_policy_train_plan computes every micro-batch's scales in one launch (one wave
 * per row, the last row of each micro-batch totalling it); skyrl_policy_train_plan_grpo does
 * the same and, in the same launch, writes the mini-batch's GRPO advantages
 * (compute_grpo_outcome_advantage, utils/ppo_utils.py:1132-1182, bit-identical to
 * skyrl_grpo_advantage) from the per-row scores (skyrl_pack_experience's reward_row_sum) over
 * contiguous groups of group_size rows times the response mask (with loss_mask_row_sum, pack's
 * loss-mask row sums, it reads neither the loss mask nor hands rows over: each row's wave totals
 * its micro-batch from them; same scales for masks whose row sums are exact, e.g. 0/1);
 * skyrl_policy_train_micro_fwd is
 * the fused pass of micro-batch `micro` alone (no scales or epilogue launch);
 * skyrl_policy_train_fold folds every micro-batch's per-token records into loss_out[n_micro]
 * and metrics_out[n_micro * SKYRL_M_COUNT] in one launch (one wave per row, the last row of each
 * micro-batch folding its rows' records in row order). Per micro-batch the loss and metrics are the bits skyrl_policy_train_fwd /
 * _ragged_fwd return for it (same code and order; a position with loss mask 0 contributes
 * nothing). All per-token arrays (old / adv / loss_mask / ref, logp_out / entropy_out) are
 * the mini-batch's f32 [n_total, R]; loss_mask is required. micro_fwd, dense form
 * (token_pos NULL): ntok = rows * R, position (b, t) of the micro-batch is logits row b*R + t
 * (logits + (b*R + t)*ld), labels at labels + b*label_stride_b + t*label_stride_t; packed form:
 * token q of the launch at logits + q*ld, labels[q*label_stride_t], token_pos[q] its position
 * within the micro-batch's [rows, R]. Same V / alignment rules as skyrl_policy_train_ragged_fwd.
 * The plan must precede the micro-batch launches and the fold follow them on one stream; the
 * workspace (skyrl_policy_train_step_workspace_bytes, zeroed once) must not be shared by two
 * mini-batches in flight. At most 4096 micro-batches. */
size_t skyrl_policy_train_step_workspace_bytes(int32_t n_total, int32_t R, int32_t micro_rows);
int skyrl_policy_train_plan(const float* loss_mask, int32_t n_total, int32_t R, int32_t micro_rows,
                            const skyrl_ppo_params* params, void* workspace, void* stream);
int skyrl_policy_train_plan_grpo(const float* loss_mask, int32_t n_total, int32_t R, int32_t micro_rows,
                                 const skyrl_ppo_params* params, const float* scores, const void* response_mask,
                                 int mask_dtype, int32_t group_size, float epsilon, int32_t norm_by_std,
                                 float* advantages, const float* loss_mask_row_sum /* [n_total] or NULL */,
                                 void* workspace, void* stream);
int skyrl_policy_train_micro_fwd(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V,
                                 const int64_t* labels, int64_t label_stride_b, int64_t label_stride_t,
                                 const int32_t* token_pos, int32_t micro, int32_t n_total, int32_t R,
                                 int32_t micro_rows, float temperature, const float* old_log_probs,
                                 const float* advantages, const float* loss_mask, const float* ref_log_probs,
                                 const skyrl_ppo_params* params, float* logp_out, float* entropy_out,
                                 void* grad_logits, int64_t ld_grad, void* workspace, void* stream);
int skyrl_policy_train_micro_fwd_ex(const void* logits, int dtype, int64_t ld, int32_t ntok, int32_t V,
                                 const int64_t* labels, int64_t label_stride_b, int64_t label_stride_t,
                                 const int32_t* token_pos, int32_t micro, int32_t n_total, int32_t R,
                                 int32_t micro_rows, float temperature, const float* old_log_probs,
                                 const float* advantages, const float* loss_mask, const float* ref_log_probs,
                                 const skyrl_ppo_params* params, float* logp_out, float* entropy_out,
                                 void* grad_logits, int64_t ld_grad, void* workspace, void* stream,
        const skyrl_variant* variant);
int skyrl_policy_train_fold(const float* loss_mask, int32_t n_total, int32_t R, int32_t micro_rows,
                            const skyrl_ppo_params* params, float* loss_out, float* metrics_out,
                            void* workspace, void* stream);
/* 1 if the packed and step forms take vocabulary V (aligned: rows 16-B aligned and V % 8 == 0)
 * at this temperature, else 0: the same plan their launches make. */
int skyrl_policy_train_supports(int32_t V, int32_t aligned, float temperature);
int skyrl_policy_train_supports_ex(int32_t V, int32_t aligned, float temperature,
        const skyrl_variant* variant);
/* x[i] *= g[0] over a bf16 buffer; a no-op kernel when g[0] == 1. */
int skyrl_scale_bf16_by_device_scalar(const float* g, void* x, int64_t n, void* stream);

/* ---- a1: rollout token sampling -----------------------------------------
 * Replaces the vLLM sampler behind VLLMInferenceEngine.generate
 * (inference_engines/vllm/vllm_engine.py:196-218) with sampled-token logprob
 * extraction (vllm_engine.py:139-149) and SamplingParams defaults
 * (config/ppo_base_config.yaml:316-324). Filters on the temperature-scaled
 * logits: top_k (exactly the k largest, equal values taken in index order, as
 * skyrl-tx/tx/utils/generator.py:398-420 lax.top_k + first-k mask; <= 0 off), min_p
 * (p >= min_p * p_max), then top_p (skyrl-tx/tx/utils/generator.py:424-449:
 * in descending order keep tokens while the mass strictly before them is
 * < top_p, the top token always, ties in index order; 1.0 off, 0 keeps one); the top_p
 * masses are fixed-point 2^31 e^((x-max)/T) summed exactly, so decisions are
 * reproducible. temperature==0 => greedy (lowest index wins ties). Otherwise
 * Gumbel-max with a counter-based hash keyed by (seed, seq_ids[i], step,
 * vocab index), so the token is a pure function of its inputs (bit-exact vs
 * oracle/sampler_ref.c). logp_out = log_softmax(raw logits)[token].
 * logits row i at logits + i*ld (elements).                                  */
int skyrl_sample(const void* logits, int dtype, int64_t ld, int32_t nseq, int32_t V,
                 float temperature, int32_t top_k, float top_p, float min_p, uint64_t seed,
                 const int64_t* seq_ids, int64_t step, int32_t* tokens_out, float* logp_out,
                 void* workspace, void* stream);
int skyrl_sample_ex(const void* logits, int dtype, int64_t ld, int32_t nseq, int32_t V,
                 float temperature, int32_t top_k, float top_p, float min_p, uint64_t seed,
                 const int64_t* seq_ids, int64_t step, int32_t* tokens_out, float* logp_out,
                 void* workspace, void* stream,
        const skyrl_variant* variant);
size_t skyrl_sample_workspace_bytes(int32_t nseq, int32_t V);

/* ---- a9: experience pack --------------------------------------------------
 * Replaces convert_prompts_responses_to_batch_tensors (dataset/preprocess.py:
 * 28-132) + pad_batch (trainer.py:872-907). Ragged inputs in CSR form
 * (offsets int64 [N+1]); P/R = max prompt/response length; rows N..N+pad-1
 * are clones of rows 0..pad-1 with loss_mask 0 (pad_batch).
 * Outputs: sequences i64 [Np,P+R] (left-padded prompt | right-padded
 * response), attention_mask i64 [Np,P+R], response_mask i64 [Np,R],
 * rewards f32 [Np,R], loss_mask f32 [Np,R], rollout_logprobs f32 [Np,R]
 * (NULL when logprob_vals is NULL), loss_mask_row_sum f32 [Np] (per-row sum of
 * loss_mask, the input of skyrl_ppo_loss_fwd's reduction scales; may be NULL),
 * reward_row_sum f32 [Np] (per-row sum of rewards = the GRPO score of
 * ppo_utils.py:1156, in skyrl_grpo_advantage's summation order; may be NULL).
 * Np = N + pad.                                                               */
typedef struct skyrl_pack_inputs {
    const int64_t* prompt_tokens;   const int64_t* prompt_off;
    const int64_t* response_tokens; const int64_t* response_off;
    const float* reward_vals;       const int64_t* reward_off;
    const float* loss_mask_vals;    const int64_t* loss_mask_off;
    const float* logprob_vals;      const int64_t* logprob_off;   /* may be NULL */
} skyrl_pack_inputs;
int skyrl_pack_experience(const skyrl_pack_inputs* in, int32_t N, int32_t pad, int32_t P, int32_t R,
                          int64_t pad_token_id, int64_t* sequences, int64_t* attention_mask,
                          int64_t* response_mask, float* rewards, float* loss_mask,
                          float* rollout_logprobs, float* loss_mask_row_sum, float* reward_row_sum,
                          void* stream);

/* ---- a12: gradient scale ------------------------------------------------
 * grads *= scale over a flat fp32 bucket (optim_step's 1/n_micro scaling,
 * workers/worker.py:909-914) fused with the squared-L2 partial for clipping
 * (fsdp_utils.py:388-401): sumsq_out[0] += sum(x^2) (device, f32, atomics).  */
int skyrl_scale_and_sumsq(float* grads, int64_t n, float scale, float* sumsq_out, void* stream);

/* out[i] = g[0] * in[i] (g on device): autograd backward of a scalar loss whose
 * per-element gradient was produced by a forward kernel for unit upstream grad. */
int skyrl_scale_by_device_scalar(const float* g, const float* in, float* out, int64_t n, void* stream);

/* ---- a12/a14: optimizer step ---------------------------------------------
 * Replaces PolicyWorkerBase.optim_step (workers/worker.py:900-925) ->
 * FSDPStrategy.optimizer_step (distributed/fsdp_strategy.py:160-190): grads *=
 * 1/n_micro, clip_grad_norm_(max_norm) (fsdp_utils.py:388-401), skip on a
 * non-finite norm, torch AdamW (fsdp_strategy.py:284-296), over a flat fp32
 * parameter shard. No host sync: the step counter and the plan live on device.
 *   skyrl_sumsq        sumsq_out[0] = sum(x^2), deterministic (workspace:
 *                      skyrl_sumsq_workspace_bytes(n)). Under DP sharding the
 *                      caller all-reduces it (SUM) before the plan.
 *   skyrl_adamw_plan   grad_norm_out[0] = sqrt(sumsq)*grad_scale (the returned
 *                      grad_norm); clip coef; ++step_count unless non-finite;
 *                      plan: skyrl_adamw_plan_floats() floats.
 *   skyrl_adamw_update one pass over (param, grad, exp_avg, exp_avg_sq); when
 *                      param_bf16 != NULL also writes the bf16 copy consumed by
 *                      the rollout engine (colocated weight sync, a14). */
typedef struct skyrl_adamw_params {
    float lr, beta1, beta2, eps, weight_decay;
    float max_grad_norm; /* <= 0: no clipping (grad_norm still reported) */
    float grad_scale;    /* 1/(n_micro) x 1/(dp world if grads are SUM-reduced) */
} skyrl_adamw_params;
size_t skyrl_sumsq_workspace_bytes(int64_t n);
int skyrl_sumsq(const float* x, int64_t n, float* sumsq_out, void* workspace, void* stream);
size_t skyrl_adamw_plan_floats(void);
int skyrl_adamw_plan(const float* sumsq, const skyrl_adamw_params* hp, int32_t* step_count, float* plan,
                     float* grad_norm_out, void* stream);
int skyrl_adamw_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* param_bf16,
                       int64_t n, const float* plan, float beta1, float beta2, void* stream);
/* Per-parameter form for a module's parameters in one flat shard (torch.optim.AdamW over
 * named parameters, fsdp_strategy.py:284-296: a parameter whose .grad is None is skipped and
 * its own `step` is not advanced). touched i32[nparams]: 1 = some DP rank's backward reached
 * the parameter since the last step (the caller MAX-all-reduces it on device). No host sync.
 *   skyrl_adamw_seg_plan    as skyrl_adamw_plan, plus per parameter p: if touched[p],
 *                           ++param_step[p] and coef f32[2*nparams] = (-lr/bc1, sqrt(bc2)) of
 *                           its own count, else (0, 0). One launch of one workgroup.
 *   skyrl_adamw_seg_update  as skyrl_adamw_update; shard element e belongs to segment s with
 *                           seg_start[s] <= e < seg_start[s+1] (i64[nseg+1], seg_start[0] = 0,
 *                           seg_start[nseg] = n) of parameter seg_owner[s] (i32[nseg]);
 *                           tile_seg[t] (i32[ceil(n / skyrl_adamw_seg_tile())]) = the segment
 *                           holding element t * tile. Untouched parameters' elements (param,
 *                           moments, bf16 copy) are left as they are. When every parameter is
 *                           touched at one common count it runs skyrl_adamw_update's loop. */
int skyrl_adamw_seg_plan(const float* sumsq, const skyrl_adamw_params* hp, const int32_t* touched, int32_t nparams,
                         int32_t* param_step, float* plan, float* coef, float* grad_norm_out, void* stream);
int skyrl_adamw_seg_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* param_bf16,
                           int64_t n, const float* plan, const float* coef, const int64_t* seg_start,
                           const int32_t* seg_owner, int32_t nseg, const int32_t* tile_seg, float beta1, float beta2,
                           void* stream);
size_t skyrl_adamw_seg_tile(void);
/* y = bf16(x), round-to-nearest-even: the learner -> rollout weight copy when the
 * optimizer ran without a bf16 shadow (FSDPWeightExtractor, fsdp_worker.py:30-87). */
int skyrl_cast_bf16(const float* x, void* y, int64_t n, void* stream);

/* ---- §8(f)2: rollout decode loop (paged KV cache) ------------------------
 * Replace the attention of vLLM's decode step behind VLLMInferenceEngine.generate
 * (inference_engines/vllm/vllm_engine.py:196-218); model semantics are HF
 * Qwen2/Llama (rotate_half RoPE, GQA). One KV cache per layer:
 *   K bf16 [num_blocks, nkv, 16, head_dim], V bf16 [num_blocks, nkv, head_dim, 16];
 * slot = block * 16 + offset; head_dim in {64, 128}; nh % nkv == 0.
 *   skyrl_rope_kv_write  qkv bf16 [T, (nh+2nkv)*head_dim] (row stride qkv_stride):
 *                        rotates q into q_out bf16 [T,nh,head_dim], rotates k into the
 *                        K cache (and k_out [T,nkv,head_dim] if non-NULL), copies v into
 *                        the V cache; slot_mapping[t] < 0 skips the cache write.
 *                        cos_sin f32 [max_pos, head_dim] = cos | sin halves.
 *   skyrl_paged_decode   one query token per sequence: out[s] = softmax(scale q.K^T) V over
 *                        context_lens[s] >= 1 cached tokens listed by block_tables
 *                        i32 [nseq, bt_stride]; nh/nkv <= 16. Each sequence's context is
 *                        split over at most nparts waves per kv head, each partition at
 *                        least part_tokens (a multiple of 16) tokens, decided on device
 *                        from context_lens (so a fixed launch fits any context);
 *                        nparts > 1 needs
 *                        skyrl_paged_decode_workspace_bytes(nseq, nh, head_dim, nparts). */
int skyrl_rope_kv_write(const void* qkv, int64_t qkv_stride, int32_t T, int32_t nh, int32_t nkv, int32_t head_dim,
                        const int64_t* positions, const int64_t* slot_mapping, const float* cos_sin, void* q_out,
                        void* k_out, void* k_cache, void* v_cache, void* stream);
size_t skyrl_paged_decode_workspace_bytes(int32_t nseq, int32_t nh, int32_t head_dim, int32_t nparts);
int skyrl_paged_decode(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                       const int32_t* block_tables, int64_t bt_stride, const int32_t* context_lens, int32_t nseq,
                       int32_t nh, int32_t nkv, int32_t head_dim, float scale, int32_t part_tokens, int32_t nparts,
                       void* out, int64_t out_stride, void* workspace, void* stream);
int skyrl_paged_decode_ex(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                       const int32_t* block_tables, int64_t bt_stride, const int32_t* context_lens, int32_t nseq,
                       int32_t nh, int32_t nkv, int32_t head_dim, float scale, int32_t part_tokens, int32_t nparts,
                       void* out, int64_t out_stride, void* workspace, void* stream,
        const skyrl_variant* variant);
/* skyrl_paged_decode_balanced: the same attention with the work split by blocks instead of by
 *                        sequence: the cache blocks of all sequences (per kv head) are laid end
 *                        to end and each of `waves` waves streams an equal share, so a ragged
 *                        batch costs what a uniform one of the same total does. Three launches on
 *                        `stream` (plan: block prefix sums; attention; merge of the sequences
 *                        split across waves). nseq <= 8192; the workspace is
 *                        skyrl_paged_decode_balanced_workspace_bytes(nseq, nh, head_dim, waves). */
size_t skyrl_paged_decode_balanced_workspace_bytes(int32_t nseq, int32_t nh, int32_t head_dim, int32_t waves);
int skyrl_paged_decode_balanced(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                                const int32_t* block_tables, int64_t bt_stride, const int32_t* context_lens,
                                int32_t nseq, int32_t nh, int32_t nkv, int32_t head_dim, float scale, int32_t waves,
                                void* out, int64_t out_stride, void* workspace, void* stream);
/* Decoder-layer glue (HF Qwen2DecoderLayer/LlamaDecoderLayer), bf16 [n, H] rows:
 *   skyrl_add_rmsnorm  hidden = bf16(hidden + delta) (delta may be NULL), then
 *                      out = bf16(weight * bf16(hidden * rsqrt(mean(hidden^2) + eps)));
 *                      H % 4 == 0, H <= 8192.
 *   skyrl_silu_mul     out [n, I] = bf16(bf16(silu(gate)) * up) of gate_up [n, 2I]. */
int skyrl_add_rmsnorm(const void* delta, void* hidden, const void* weight, int32_t n, int32_t H, float eps, void* out,
                      void* stream);
int skyrl_silu_mul(const void* gate_up, int64_t n, int32_t I, void* out, void* stream);

/* ---- a12-a14 collectives over RCCL (xGMI), one communicator per process and GPU ----------
 * SURVEY §8(b)'s skyrl_comm_{init, allreduce, broadcast}, for hosts that bind this library
 * directly (the Python host reaches the same RCCL through torch.distributed, skyrl_amd/comm.py).
 * Reference call sites: all-reduce = metric reduction (distributed/strategy.py:70-95) and the DP
 * gradient mean (distributed/fsdp_strategy.py:216-226); reduce-scatter = FSDP2's fp32 gradient
 * reduce-scatter (fsdp_strategy.py:253-271); all-gather = the sharded optimizer's shards;
 * broadcast = learner -> rollout weights (weight_sync/broadcast_strategy.py:98-191).
 *   skyrl_comm_get_unique_id  rank 0 writes skyrl_comm_unique_id_bytes() bytes; the caller hands
 *                             them to every rank (any out-of-band channel)
 *   skyrl_comm_init           on the current HIP device; *comm_out is caller-owned until
 *                             skyrl_comm_destroy
 *   counts are elements of dtype (SKYRL_F32, SKYRL_BF16, SKYRL_I64, SKYRL_I32, SKYRL_U8);
 *   reduce_scatter: send holds nranks * recv_count, allgather: recv holds nranks * send_count;
 *   broadcast: send is read on root only (may be NULL elsewhere), recv written everywhere.
 * Stream-ordered on `stream`, no host synchronization, nothing allocated per call. */
#define SKYRL_COMM_SUM 0
#define SKYRL_COMM_MAX 1
#define SKYRL_COMM_MIN 2
#define SKYRL_COMM_AVG 3
size_t skyrl_comm_unique_id_bytes(void);
int skyrl_comm_get_unique_id(void* id_out);
int skyrl_comm_init(const void* unique_id, int32_t nranks, int32_t rank, void** comm_out);
int skyrl_comm_destroy(void* comm);
int skyrl_comm_size(void* comm, int32_t* nranks_out, int32_t* rank_out);
int skyrl_comm_allreduce(const void* send, void* recv, int64_t count, int dtype, int op, void* comm, void* stream);
int skyrl_comm_reduce_scatter(const void* send, void* recv, int64_t recv_count, int dtype, int op, void* comm,
                              void* stream);
int skyrl_comm_allgather(const void* send, void* recv, int64_t send_count, int dtype, void* comm, void* stream);
int skyrl_comm_broadcast(const void* send, void* recv, int64_t count, int dtype, int32_t root, void* comm,
                         void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SKYRL_HIP_H */
