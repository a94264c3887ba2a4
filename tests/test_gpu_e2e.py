"""50-step GRPO loss curve through the HIP path vs the oracle (north_star: "loss curve matching
reference to 1e-3 over 50 GRPO steps").

Every step is the reference's training step (trainer.py:1037-1085 `_execute_training_step`,
workers/worker.py:731-925): a rollout of 8 prompts x G 4 with unequal response lengths, old and
ref logprobs, GRPO advantages, then 2 update epochs x 2 mini-batches x 2 micro-batches, each
mini-batch ending in optim_step (grads x 1/n_micro, clip at max_grad_norm, AdamW). After the
first optimizer step of a step the policy is off its rollout (ratio != 1): the clip and
dual-clip branches fire, the entropy and KL terms carry weight.

The policy is a bigram table model (logits_t = W[token_{t-1}], W in R^{V x V}) so its forward
is a lookup and the comparison isolates the hot path:

  HIP path : TokenSampler rollout on the bf16 rollout weights -> skyrl_pack_experience ->
             logprob_fwd (old, ref) -> GRPO registry -> per micro-batch PolicyMicroStep (ONE
             fused pass: logprob + entropy + dual-clip PPO/KL/entropy loss + dlogits) ->
             dlogits scattered into GradReducer.grad -> ShardedAdamW.step(n_micro) (clip +
             AdamW, bf16 rollout copy written in the same pass)
  oracle   : cpu_ref pack / logprobs / GRPO / loss assembly with torch-CPU autograd (dlogits
             rounded to bf16, the reference's logits dtype), grads x 1/n_micro,
             clip_grad_norm_ + torch AdamW (fsdp_strategy.py:284-296)

The oracle starts every step from the HIP side's state (weights, Adam moments, step count) and
runs the whole step on the same trajectories itself, so each step's comparison is of the same
function on the same inputs: final_loss / policy_loss / clip_ratio / policy_kl /
policy_entropy per micro-batch and grad_norm per mini-batch agree to rel 1e-3 (abs 1e-6), and
the weights after the step to rel 1e-4 in L2. `test_loss_curve_detects_perturbations` shows
the comparison fails when the oracle's clip range, dual-clip, 1/n_micro scaling, off-policy
ratio or entropy coefficient is perturbed.
"""

import math

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import comm, ops, ppo_utils
from skyrl_amd.config import AlgorithmConfig, SamplingParams
from skyrl_amd.sampler import TokenSampler
from skyrl_amd.trainer_utils import Experience
from skyrl_amd.worker import PolicyMicroStep

pytestmark = pytest.mark.gpu

V, P, R, B, G = 256, 4, 24, 8, 4
N = B * G
EPOCHS, MINI, MICRO = 2, 2, 2  # update_epochs_per_batch, mini-batches per step, micro-batches each
STOP_MOD = 11                  # a response ends at (and includes) its first token divisible by 11
REL, ABS = 1e-3, 1e-6


def _cfg():
    return AlgorithmConfig(policy_loss_type="dual_clip", eps_clip_low=0.1, eps_clip_high=0.1, clip_ratio_c=1.05,
                           use_kl_loss=True, kl_loss_coef=0.05, use_entropy_loss=True, entropy_loss_coef=0.01,
                           loss_reduction="token_mean")


def _reward(resp, lens):  # fraction of the response's tokens divisible by 7, on its last token
    r = torch.zeros(resp.shape, dtype=torch.float32)
    for i in range(resp.shape[0]):
        k = int(lens[i])
        r[i, k - 1] = float((resp[i, :k] % 7 == 0).float().mean())
    return r


def _close(a, b):
    return abs(a - b) <= ABS + REL * abs(b)


def run_curve(dev, steps, perturb=None):
    """Runs `steps` GRPO steps; returns (list of per-step records, list of mismatches)."""
    cfg = _cfg()
    eps_hi = cfg.eps_clip_high + (0.05 if perturb == "clip" else 0.0)
    dual = perturb != "dual_clip"
    ent_coef = 0.0 if perturb == "entropy" else cfg.entropy_loss_coef
    ocfg = comm.AdamWConfig(lr=0.1, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=1.0)
    torch.manual_seed(0)
    w0 = torch.randn(V, V) * 0.5
    ref_bf = w0.to(torch.bfloat16)  # frozen reference policy
    red = comm.GradReducer(V * V, dev)
    opt = comm.ShardedAdamW(red, w0.reshape(-1).to(dev), ocfg)
    step_fn = PolicyMicroStep(cfg)
    w = torch.nn.Parameter(w0.clone())
    topt = torch.optim.AdamW([w], lr=ocfg.lr, betas=ocfg.betas, eps=ocfg.eps, weight_decay=ocfg.weight_decay)
    prompts = torch.randint(0, V, (B, P), generator=torch.Generator().manual_seed(1)).repeat_interleave(G, 0)
    uids = [str(i // G) for i in range(N)]
    records, bad = [], []
    for it in range(steps):
        wb = opt.weights_bf16[: V * V].view(V, V)
        # ---- rollout on the bf16 rollout weights; a response stops at its first STOP_MOD token
        smp = TokenSampler(N, V, R, dev, SamplingParams(), seed=it)
        last = prompts[:, -1].to(dev)
        for t in range(R):
            tok, _ = smp.step(wb[last].contiguous(), t)
            last = tok.long()
        raw = smp.tokens.t().cpu().long()
        stop = (raw % STOP_MOD == 0).float()
        lens = torch.where(stop.any(1), stop.argmax(1) + 1, torch.full((N,), R))
        resp_lists = [raw[i, : int(lens[i])].tolist() for i in range(N)]
        rew = _reward(raw, lens)
        rew_lists = [rew[i, : int(lens[i])].tolist() for i in range(N)]
        # ---- pack (HIP) vs oracle pack: bit-exact
        csr = lambda ls: (torch.tensor([x for l in ls for x in l]),  # noqa: E731
                          torch.tensor([0] + [len(l) for l in ls]).cumsum(0))
        pv, po = csr([p.tolist() for p in prompts])
        rv, ro = csr(resp_lists)
        wv, wo = csr(rew_lists)
        mv, mo = csr([[1.0] * len(l) for l in resp_lists])
        seq_d, _, rmask_d, rew_d, lmask_d, _ = ops.pack_experience(
            pv.to(dev), po, rv.to(dev), ro, wv.float().to(dev), wo, mv.float().to(dev), mo, None, None,
            N=N, P=P, R=R, pad=0, pad_token_id=0)
        seq_c, _, rm_c, rw_c, lm_c, _ = cpu_ref.pack([p.tolist() for p in prompts], resp_lists, rew_lists,
                                                     [[1.0] * len(l) for l in resp_lists], None, 0)
        rc = seq_c.shape[1] - P  # the oracle packs to the longest response; the HIP pack to R
        assert torch.equal(seq_d.cpu()[:, :P + rc], torch.from_numpy(seq_c))
        assert (seq_d.cpu()[:, P + rc:] == 0).all() and (lmask_d.cpu()[:, rc:] == 0).all()
        assert torch.equal(lmask_d.cpu()[:, :rc], torch.from_numpy(lm_c))
        pad = lambda a: torch.nn.functional.pad(torch.from_numpy(a), (0, R - rc))  # noqa: E731
        rw_c, rm_c = pad(rw_c), pad(rm_c)
        seqs = seq_d.cpu()
        mask = lmask_d.cpu()
        prev_all, lab_all = seqs[:, -R - 1:-1], seqs[:, -R:]
        # ---- old / ref logprobs and GRPO advantages (HIP) vs oracle
        old_d, _ = ops.logprobs_and_entropy(wb[prev_all.to(dev)].contiguous(), lab_all.to(dev), 1.0,
                                            compute_entropy=False)
        ref_d, _ = ops.logprobs_and_entropy(ref_bf.to(dev)[prev_all.to(dev)].contiguous(), lab_all.to(dev), 1.0,
                                            compute_entropy=False)
        adv_d, _ = ppo_utils.compute_grpo_outcome_advantage(rew_d, rmask_d, uids)
        # oracle starts the step from the HIP state (teacher forcing)
        with torch.no_grad():
            w.copy_(opt.param[: V * V].cpu().view(V, V))
        topt.state[w] = {"step": torch.tensor(float(opt.step_count.item())),
                         "exp_avg": opt.exp_avg[: V * V].cpu().view(V, V).clone(),
                         "exp_avg_sq": opt.exp_avg_sq[: V * V].cpu().view(V, V).clone()}
        with torch.no_grad():
            old_c = cpu_ref.logprobs_from_logits(w.to(torch.bfloat16)[prev_all].float(), lab_all)
            ref_c = cpu_ref.logprobs_from_logits(ref_bf[prev_all].float(), lab_all)
        adv_c = cpu_ref.grpo_advantage(rw_c, rm_c.float(), uids)
        torch.testing.assert_close(old_d.cpu(), old_c, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(adv_d.cpu(), adv_c, atol=1e-5, rtol=1e-5)
        rec = {"step": it, "micro": [], "grad_norm": [], "dual_active": 0, "mean_len": float(lens.float().mean())}
        mb = N // MINI
        for _ in range(EPOCHS):
            for m0 in range(0, N, mb):
                # -- HIP: the worker's micro-batches, then optim_step
                for s0 in range(m0, m0 + mb, mb // MICRO):
                    sl = slice(s0, s0 + mb // MICRO)
                    n = mb // MICRO
                    wbn = opt.weights_bf16[: V * V].view(V, V)
                    prev = seq_d[sl, -R - 1:-1]
                    x = torch.zeros(n, P + R, V, dtype=torch.bfloat16, device=dev)
                    x[:, -R - 1:-1] = wbn[prev]
                    x.requires_grad_(True)
                    exp = Experience(sequences=seq_d[sl], action_log_probs=old_d[sl], base_action_log_probs=ref_d[sl],
                                     values=None, returns=None, advantages=adv_d[sl], attention_mask=None,
                                     loss_mask=lmask_d[sl], action_mask=rmask_d[sl], rollout_logprobs=None,
                                     num_actions=R, info={})
                    st = step_fn(x, exp)
                    g = x.grad[:, -R - 1:-1].float().reshape(-1, V)
                    red.grad[: V * V].view(V, V).index_add_(0, prev.reshape(-1), g)
                    rec["micro"].append({"hip": {k: st[k] for k in ("final_loss", "policy_loss", "policy_kl",
                                                                     "policy_entropy", "loss_metrics/clip_ratio")}})
                gn = float(opt.step(n_micro=MICRO).item())
                # -- oracle: the same mini-batch from its own (teacher-forced) state
                wgrad = torch.zeros(V, V)
                for j, s0 in enumerate(range(m0, m0 + mb, mb // MICRO)):
                    sl = slice(s0, s0 + mb // MICRO)
                    prev, lab = prev_all[sl], lab_all[sl]
                    lg = w.detach().to(torch.bfloat16)[prev].float().requires_grad_(True)
                    lp = cpu_ref.logprobs_from_logits(lg, lab)
                    ent = cpu_ref.entropy_from_logits(lg)
                    old = cpu_ref.logprobs_from_logits(lg.detach(), lab) if perturb == "ratio" else old_c[sl]
                    loss, m = cpu_ref.policy_loss_assembly(
                        lp, old, adv_c[sl], mask[sl], ref_c[sl], ent, kl_coef=cfg.kl_loss_coef,
                        use_entropy_loss=True, ent_coef=ent_coef, eps_low=cfg.eps_clip_low, eps_high=eps_hi,
                        clip_c=cfg.clip_ratio_c, dual_clip=dual, reduction="token_mean")
                    loss.backward()
                    wgrad.index_add_(0, prev.reshape(-1), lg.grad.to(torch.bfloat16).float().reshape(-1, V))
                    with torch.no_grad():  # tokens where the dual-clip branch decides the loss
                        ratio = torch.exp(torch.clamp(lp.detach() - old, -20, 20))
                        pg1 = -torch.min(ratio * adv_c[sl], ratio.clamp(1 - cfg.eps_clip_low, 1 + eps_hi) * adv_c[sl])
                        rec["dual_active"] += int(((adv_c[sl] < 0) & (-adv_c[sl] * cfg.clip_ratio_c < pg1)
                                                   & (mask[sl] > 0)).sum())
                    k = len(rec["micro"]) - MICRO + j
                    rec["micro"][k]["oracle"] = {"final_loss": m["final_loss"], "policy_loss": m["policy_loss"],
                                                 "policy_kl": m["policy_kl"], "policy_entropy": m["policy_entropy"],
                                                 "loss_metrics/clip_ratio": m["clip_ratio"]}
                scale = 1.0 if perturb == "n_micro" else 1.0 / MICRO
                w.grad = wgrad * scale
                gn_c = float(torch.nn.utils.clip_grad_norm_([w], max_norm=ocfg.max_grad_norm))
                topt.step()
                topt.zero_grad()
                rec["grad_norm"].append((gn, gn_c))
                if not _close(gn, gn_c):
                    bad.append((it, "grad_norm", gn, gn_c))
        for mrec in rec["micro"]:
            for k, hv in mrec["hip"].items():
                if not _close(hv, mrec["oracle"][k]):
                    bad.append((it, k, hv, mrec["oracle"][k]))
        w_gpu = opt.param[: V * V].cpu().view(V, V)
        rel = float((w_gpu - w.detach()).norm() / w.detach().norm())
        rec["weight_rel_l2"] = rel
        if rel > 1e-4:
            bad.append((it, "weights", rel, 0.0))
        records.append(rec)
    return records, bad


def test_grpo_loss_curve_matches_oracle(dev):
    records, bad = run_curve(dev, 50)
    assert not bad, bad[:10]
    # the curve is not degenerate: the off-policy branches fire and the loss terms carry weight
    clip_steps = sum(any(m["hip"]["loss_metrics/clip_ratio"] > 0 for m in r["micro"]) for r in records)
    dual_steps = sum(r["dual_active"] > 0 for r in records)
    pg = [abs(m["hip"]["policy_loss"]) for r in records for m in r["micro"]]
    lens = [r["mean_len"] for r in records]
    assert clip_steps >= 25, clip_steps
    assert dual_steps >= 5, dual_steps
    assert sum(p > 1e-2 for p in pg) >= len(pg) // 4, sorted(pg)[-5:]
    assert min(lens) < R and max(lens) > 2  # unequal response lengths
    assert all(math.isfinite(m["hip"]["final_loss"]) for r in records for m in r["micro"])
    # the policy drifts from the frozen reference over the run
    assert records[-1]["micro"][-1]["hip"]["policy_kl"] > records[0]["micro"][-1]["hip"]["policy_kl"]


@pytest.mark.parametrize("perturb", ["clip", "dual_clip", "n_micro", "ratio", "entropy"])
def test_loss_curve_detects_perturbations(dev, perturb):
    """The comparison above is sensitive: perturbing one semantic of the oracle's step makes it
    fail within 4 steps."""
    _, bad = run_curve(dev, 4, perturb=perturb)
    assert bad, f"perturbation {perturb} went unnoticed"
