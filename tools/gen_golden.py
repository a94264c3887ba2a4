"""Generate golden vectors for the hot path by running the REAL reference (build container only).

Imports skyrl_train from /root/reference/skyrl-train (read-only; bytecode writing disabled)
behind a stub shim for its uninstalled infra dependencies (ray, omegaconf, loguru, jaxtyping,
torchdata, peft, flash_attn.bert_padding — none carries hot-path arithmetic; see
SURVEY.md §8(c) / Appendix A), calls the reference functions on seeded inputs and writes
small .npz fixtures (inputs + expected outputs, arrays only, no pickles) to tests/golden/.

The reference never travels to the GPU box: only the .npz data does.

    PYTHONDONTWRITEBYTECODE=1 python -B tools/gen_golden.py
"""

from __future__ import annotations

import dataclasses
import enum
import json
import importlib.machinery
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference/skyrl-train"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


# ----------------------------------------------------------------------------- shim
def install_shim():
    import torch.utils.data as tud

    if not hasattr(enum, "StrEnum"):
        class StrEnum(str, enum.Enum):
            def __str__(self):
                return str(self.value)

        enum.StrEnum = StrEnum

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        m.__spec__ = importlib.machinery.ModuleSpec(name, None)
        sys.modules[name] = m
        return m

    class _Any:
        def __init__(self, *a, **k):
            pass

        def __getitem__(self, k):
            return self

        def __call__(self, *a, **k):
            return self

        def __getattr__(self, k):
            return _Any()

    mod("jaxtyping", Float=_Any(), Integer=_Any())

    class _Log:
        def _emit(self, *a, **k):
            pass

        debug = info = warning = error = exception = critical = success = trace = log = _emit

        def opt(self, *a, **k):
            return self

        def bind(self, *a, **k):
            return self

        def remove(self, *a, **k):
            pass

        def add(self, *a, **k):
            return 0

        def level(self, *a, **k):
            return self

    mod("loguru", logger=_Log())

    class DictConfig(dict):
        pass

    class ListConfig(list):
        pass

    class OmegaConf:
        to_container = staticmethod(lambda c, resolve=True: dict(c))
        create = staticmethod(lambda x: DictConfig(x))

        @staticmethod
        def merge(*a):
            d = {}
            for x in a:
                d.update(x)
            return DictConfig(d)

    mod("omegaconf", DictConfig=DictConfig, ListConfig=ListConfig, OmegaConf=OmegaConf)
    ray = mod("ray", is_initialized=lambda: False, init=lambda *a, **k: None, shutdown=lambda *a, **k: None,
              remote=lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f)),
              get=lambda x: x, put=lambda x: x, ObjectRef=object, get_gpu_ids=lambda: [0])
    mod("ray.actor", ActorHandle=object)
    ray.util = mod("ray.util")
    mod("ray.util.placement_group", placement_group=None, PlacementGroupSchedulingStrategy=None,
        PlacementGroup=object, placement_group_table=None)
    mod("ray.util.scheduling_strategies", PlacementGroupSchedulingStrategy=None, NodeAffinitySchedulingStrategy=None)
    ray._private = mod("ray._private")
    mod("ray._private.services", get_node_ip_address=lambda: "127.0.0.1")
    mod("torchdata")
    mod("torchdata.stateful_dataloader", StatefulDataLoader=tud.DataLoader)

    class _LoraConfig:
        def __init__(self, *a, **k):
            pass

    mod("peft", LoraConfig=_LoraConfig, TaskType=_Any(), get_peft_model=lambda m, c: m)
    mod("peft.tuners")
    mod("peft.tuners.lora", LoraLayer=type("LoraLayer", (), {}))
    mod("flash_attn")
    mod("flash_attn.bert_padding", pad_input=None, unpad_input=None)
    sys.path.insert(0, REF)
    sys.path.insert(0, "/root/reference/skyrl-gym")


def save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    clean = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu()
            if v.dtype == torch.bfloat16:
                v = v.view(torch.int16).numpy().view(np.uint16)
                k = k + "__bf16"
            else:
                v = v.numpy()
        clean[k] = np.asarray(v)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **clean)
    print(f"wrote {name}.npz ({', '.join(clean)})")


# ----------------------------------------------------------------------------- cases
def gen_grpo(pu):
    g = torch.Generator().manual_seed(1234)
    cases = []
    # mixed: groups of 4, 4, 3, a singleton, a zero-variance group, pad rows
    N, R = 20, 16
    uids = ["0"] * 4 + ["1"] * 4 + ["2"] * 3 + ["solo"] + ["zv"] * 4 + ["pad0", "pad1", "0", "1"]
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    rew = torch.zeros(N, R)
    for i in range(N):
        rew[i, lens[i] - 1] = float(torch.rand((), generator=g) < 0.4)
    rew[:11] += torch.randn(11, R, generator=g) * 0.1 * mask[:11]
    rew[12:16] = 0.0
    rew[12:16, 0] = 1.0
    cases.append(("grpo_mixed", rew, mask, uids))
    # synthetic-like: 16 prompts x group 8, Bernoulli(0.3) at last token
    N, R = 128, 64
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    rew = torch.zeros(N, R)
    hit = (torch.rand(N, generator=g) < 0.3).float()
    rew[torch.arange(N), lens - 1] = hit
    uids = [str(i // 8) for i in range(N)]
    cases.append(("grpo_synth", rew, mask, uids))
    for name, rew, mask, uids in cases:
        out = {}
        for nbs in (True, False):
            adv, ret = pu.compute_grpo_outcome_advantage(
                token_level_rewards=rew.clone(), response_mask=mask, index=np.array(uids), grpo_norm_by_std=nbs)
            assert torch.equal(adv, ret)
            out[f"adv_norm{int(nbs)}"] = adv
        save(name, rewards=rew, response_mask=mask, uids=np.array(uids), **out)


def gen_advnorm(pu):
    """advantage_batch_normalize (trainer.py:275-276 -> normalize_advantages_dict,
    ppo_utils.py:127-145): the unmasked mean, the masked sum of squared deviations."""
    g = torch.Generator().manual_seed(99)
    out = {}
    # GRPO advantages of a synthetic batch (16 prompts x 8, int64 response mask)
    N, R = 128, 96
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    rew = torch.zeros(N, R)
    rew[torch.arange(N), lens - 1] = (torch.rand(N, generator=g) < 0.3).float()
    adv, _ = pu.compute_grpo_outcome_advantage(token_level_rewards=rew, response_mask=mask,
                                               index=np.array([str(i // 8) for i in range(N)]))
    d = {"advantages": adv.clone(), "response_mask": mask}
    out["grpo_in"], out["grpo_mask"], out["grpo_out"] = adv, mask, pu.normalize_advantages_dict(d)["advantages"]
    # dense float advantages with an offset (mean far from 0), f32 mask, odd width
    N, R = 37, 131
    a = torch.randn(N, R, generator=g) * 0.7 + 2.5
    m = (torch.rand(N, R, generator=g) < 0.6).float()
    d = {"advantages": a.clone(), "response_mask": m}
    out["dense_in"], out["dense_mask"], out["dense_out"] = a, m, pu.normalize_advantages_dict(d)["advantages"]
    # constant advantages: zero variance, the clamp at 1e-8 decides rstd
    a = torch.full((4, 10), 0.25)
    m = torch.ones(4, 10, dtype=torch.int64)
    d = {"advantages": a.clone(), "response_mask": m}
    out["const_in"], out["const_mask"], out["const_out"] = a, m, pu.normalize_advantages_dict(d)["advantages"]
    save("advnorm", **out)


def gen_gae(pu):
    g = torch.Generator().manual_seed(7)
    N, R = 6, 40
    lens = torch.randint(2, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.float32)
    rew = torch.randn(N, R, generator=g) * mask
    vals = torch.randn(N, R, generator=g)  # padded values are NOT zero: leak trap
    out = {}
    for tag, gamma, lambd in (("g1_l1", 1.0, 1.0), ("g099_l095", 0.99, 0.95), ("g05_l1", 0.5, 1.0)):
        adv, ret = pu.compute_gae_advantage_return(token_level_rewards=rew, values=vals, response_mask=mask,
                                                   gamma=gamma, lambd=lambd)
        out[f"adv_{tag}"] = adv
        out[f"ret_{tag}"] = ret
    save("gae", rewards=rew, values=vals, response_mask=mask, **out)
    # long rows (scan across several 256-step tiles)
    N, R = 4, 700
    lens = torch.tensor([700, 513, 256, 3])
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    rew = torch.randn(N, R, generator=g) * 0.1 * mask
    vals = torch.randn(N, R, generator=g) * 0.1
    adv, ret = pu.compute_gae_advantage_return(token_level_rewards=rew, values=vals, response_mask=mask,
                                               gamma=0.99, lambd=0.95)
    save("gae_long", rewards=rew, values=vals, response_mask=mask, adv=adv, ret=ret)


def gen_kl(pu):
    g = torch.Generator().manual_seed(11)
    lp = torch.randn(8, 33, generator=g) - 2
    base = lp + torch.randn(8, 33, generator=g) * 0.5
    base[0, :4] = lp[0, :4] + torch.tensor([25.0, -25.0, 5.0, -5.0])  # clamp branches
    mask = (torch.rand(8, 33, generator=g) < 0.8).float()
    out = {}
    for k in ("k1", "abs", "k2", "k3"):
        out[f"kl_{k}_masked"] = pu.compute_approx_kl(lp, base, loss_mask=mask, kl_estimator_type=k)
        out[f"kl_{k}"] = pu.compute_approx_kl(lp, base, loss_mask=None, kl_estimator_type=k)
    save("kl", log_probs=lp, log_probs_base=base, loss_mask=mask, **out)


def _ppo_inputs(g, n, R):
    lens = torch.randint(1, R + 1, (n,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).float()
    old = torch.randn(n, R, generator=g) * 0.5 - 2
    lp = old + torch.randn(n, R, generator=g) * 0.3
    lp[0, :3] = old[0, :3]                      # ratio == 1 exactly (min tie)
    lp[1, :2] = old[1, :2] + torch.tensor([30.0, -30.0])  # safe_exp_delta clamp
    adv = torch.randn(n, R, generator=g)
    adv[2, :2] = 0.0
    ref = lp + torch.randn(n, R, generator=g) * 0.2
    ent = torch.rand(n, R, generator=g) * 3
    return lp, old, adv, mask, ref, ent


def gen_ppo(pu, cfgmod):
    from skyrl_train.utils.torch_utils import masked_mean

    g = torch.Generator().manual_seed(99)
    n, R = 6, 37
    lp, old, adv, mask, ref, ent = _ppo_inputs(g, n, R)
    out = {}
    for lt in ("regular", "dual_clip"):
        for red in ("token_mean", "sequence_mean", "seq_mean_token_sum_norm"):
            cfg = cfgmod.AlgorithmConfig(policy_loss_type=lt, loss_reduction=red, max_seq_len=50,
                                         eps_clip_low=0.2, eps_clip_high=0.28, clip_ratio_c=3.0)
            x = lp.clone().requires_grad_(True)
            fn = pu.PolicyLossRegistry.get(lt)
            loss, m = fn(x, old, adv, cfg, loss_mask=mask)
            loss.backward()
            tag = f"{lt}_{red}"
            out[f"loss_{tag}"] = loss.detach()
            out[f"clip_{tag}"] = np.float32(m["clip_ratio"])
            out[f"grad_{tag}"] = x.grad
    # worker.py:801-876 assembly from the reference's own functions
    for use_ent in (False, True):
        cfg = cfgmod.AlgorithmConfig(policy_loss_type="regular", loss_reduction="token_mean")
        x = lp.clone().requires_grad_(True)
        e = ent.clone().requires_grad_(use_ent)
        pg, m = pu.PolicyLossRegistry.get("regular")(x, old, adv, cfg, loss_mask=mask)
        with torch.set_grad_enabled(use_ent):
            entropy = masked_mean(e, mask)
        ent_term = entropy * 0.01 if use_ent else torch.tensor(0.0)
        kl = pu.compute_approx_kl(x, ref, loss_mask=mask, kl_estimator_type="k3")
        kl = masked_mean(kl, mask, dim=-1).mean()
        final = pg + kl * 0.001 - ent_term
        final.backward()
        tag = f"asm_ent{int(use_ent)}"
        out[f"final_{tag}"] = final.detach()
        out[f"pg_{tag}"] = pg.detach()
        out[f"kl_{tag}"] = kl.detach()
        out[f"entropy_{tag}"] = entropy.detach()
        out[f"clip_{tag}"] = np.float32(m["clip_ratio"])
        out[f"grad_lp_{tag}"] = x.grad
        if use_ent:
            out[f"grad_ent_{tag}"] = e.grad
    save("ppo", log_probs=lp, old_log_probs=old, advantages=adv, loss_mask=mask, ref_log_probs=ref, entropy=ent,
         **out)


def gen_ppo_offpolicy(pu, cfgmod):
    """ppo_policy_loss with apply_off_policy_correction enabled (off_policy_correction_utils.py:7-296)."""
    g = torch.Generator().manual_seed(123)
    n, R = 8, 33
    lp, old, adv, mask, ref, ent = _ppo_inputs(g, n, R)
    rollout = old + torch.randn(n, R, generator=g) * 0.05
    rollout[3] = old[3] - 1.5        # large token ratios: tis caps, outlier / product masks fire
    rollout[4] = old[4] + 0.004      # geometric mean just inside [0.99, 1.01]
    cases = {
        "tis_token": dict(tis_ratio_type="token", token_tis_ratio_clip_high=2.0),
        "tis_seq": dict(tis_ratio_type="sequence", sequence_tis_ratio_clip_high=5.0),
        "mask_geo": dict(sequence_mask_metric="geometric", geo_mask_high=1.01, geo_mask_low=0.99),
        "mask_prod": dict(sequence_mask_metric="product", product_mask_high=2.0, product_mask_low=0.5),
        "tis_outlier": dict(tis_ratio_type="token", token_tis_ratio_clip_high=3.0,
                            outlier_token_is_threshold_low=0.2, outlier_token_is_threshold_high=4.0),
    }
    out = {}
    names = []
    for tag, kw in cases.items():
        for lt in ("regular", "dual_clip"):
            opc = cfgmod.OffPolicyCorrectionConfig(**kw)
            cfg = cfgmod.AlgorithmConfig(policy_loss_type=lt, loss_reduction="token_mean",
                                         eps_clip_low=0.2, eps_clip_high=0.28, off_policy_correction=opc)
            x = lp.clone().requires_grad_(True)
            loss, m = pu.PolicyLossRegistry.get(lt)(x, old, adv, cfg, loss_mask=mask, rollout_logprobs=rollout)
            loss.backward()
            t = f"{tag}_{lt}"
            out[f"loss_{t}"] = loss.detach()
            out[f"grad_{t}"] = x.grad
            keys = sorted(m)
            out[f"mkeys_{t}"] = np.array(keys)
            out[f"mvals_{t}"] = np.array([float(m[k]) for k in keys], dtype=np.float64)
            names.append(t)
    save("ppo_offpolicy", log_probs=lp, old_log_probs=old, advantages=adv, loss_mask=mask, rollout_logprobs=rollout,
         **out)


def gen_critic(pu, cfgmod):
    g = torch.Generator().manual_seed(5)
    n, R = 5, 29
    lens = torch.randint(1, R + 1, (n,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).float()
    old = torch.randn(n, R, generator=g)
    v = old + torch.randn(n, R, generator=g) * 0.4
    ret = torch.randn(n, R, generator=g)
    out = {}
    for tag, vc in (("clip", 0.2), ("noclip", None)):
        cfg = cfgmod.AlgorithmConfig(value_clip=vc)
        x = v.clone().requires_grad_(True)
        loss, cf = pu.ppo_critic_loss(x, old, ret, cfg, loss_mask=mask)
        loss.backward()
        out[f"loss_{tag}"] = loss.detach()
        out[f"clipfrac_{tag}"] = np.float32(cf if cf is not None else -1.0)
        out[f"grad_{tag}"] = x.grad
    save("critic", values=v, old_values=old, returns=ret, loss_mask=mask, **out)


def gen_logprob(tu):
    g = torch.Generator().manual_seed(3)
    out = {}
    # fp32 logits, V not a multiple of the vector width
    B, T, V = 3, 7, 1027
    logits = torch.randn(B, T, V, generator=g) * 3
    labels = torch.randint(0, V, (B, T), generator=g)
    for temp in (1.0, 0.7):
        x = logits.clone()
        x.div_(temp)  # model_wrapper.py:314
        x.requires_grad_(True)
        lp = tu.logprobs_from_logits(x, labels)
        ent = tu.chunked_entropy_from_logits(x, requires_grad=True)
        glp = torch.randn(B, T, generator=g)
        gent = torch.randn(B, T, generator=g)
        (lp * glp + ent * gent).sum().backward()
        tag = f"f32_t{str(temp).replace('.', '')}"
        out[f"logp_{tag}"] = lp.detach()
        out[f"ent_{tag}"] = ent.detach()
        out[f"glp_{tag}"] = glp
        out[f"gent_{tag}"] = gent
        out[f"dlogits_{tag}"] = x.grad / temp  # chain through the in-place div
    save("logprob_f32", logits=logits, labels=labels, **out)
    # bf16 logits (Qwen-like V slice): flash-CE semantics = fp32 math on the bf16 values
    out = {}
    B, T, V = 2, 5, 4096
    lb = (torch.randn(B, T, V, generator=g) * 3).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g)
    out["logp_fp32math"] = tu.logprobs_from_logits(lb.float(), labels)
    out["ent_fp32math"] = tu.chunked_entropy_from_logits(lb.float())
    out["ent_bf16math"] = tu.chunked_entropy_from_logits(lb).float()  # the reference's own dtype path
    x = lb.clone()
    x.div_(0.6)
    out["logp_t06"] = tu.logprobs_from_logits(x.float(), labels)
    save("logprob_bf16", logits=lb, labels=labels, **out)


def gen_pack(pre, trainer_mod, tb):
    g = torch.Generator().manual_seed(21)
    N = 7
    prompts = [torch.randint(3, 100, (int(torch.randint(1, 9, (1,), generator=g)),), generator=g).tolist()
               for _ in range(N)]
    responses = [torch.randint(3, 100, (int(torch.randint(1, 12, (1,), generator=g)),), generator=g).tolist()
                 for _ in range(N)]
    rewards = []
    for r in responses:
        rr = [0.0] * len(r)
        rr[-1] = float(torch.rand((), generator=g))
        rewards.append(rr)
    loss_masks = [[1] * (len(r) - 1) + [0] if len(r) > 1 else [1] for r in responses]
    logprobs = [(torch.randn(len(r), generator=g) - 1).tolist() for r in responses]
    tok = SimpleNamespace(pad_token_id=0)
    seq, att, am, rw, lm, lp = pre.convert_prompts_responses_to_batch_tensors(
        tok, prompts, responses, rewards, loss_masks, logprobs)
    # pad_batch (trainer.py:872-907) to a multiple of dp=4
    batch = tb.TrainingInputBatch({"sequences": seq, "attention_mask": att, "response_mask": am, "rewards": rw,
                                   "loss_mask": lm, "rollout_logprobs": lp})
    batch.metadata = {"uids": [str(i) for i in range(N)]}
    fake = SimpleNamespace(dispatch=SimpleNamespace(get_lcm_dp_size=lambda: 4))
    padded = trainer_mod.RayPPOTrainer.pad_batch(fake, batch)

    def ragged(lists, dtype):
        off = np.zeros(len(lists) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(x) for x in lists])
        vals = np.concatenate([np.asarray(x, dtype=dtype) for x in lists]) if off[-1] else np.zeros(0, dtype)
        return vals, off

    pv, po = ragged(prompts, np.int64)
    rv, ro = ragged(responses, np.int64)
    wv, wo = ragged(rewards, np.float32)
    mv, mo = ragged(loss_masks, np.float32)
    lv, lo = ragged(logprobs, np.float32)
    save("pack", prompt_vals=pv, prompt_off=po, response_vals=rv, response_off=ro, reward_vals=wv, reward_off=wo,
         loss_mask_vals=mv, loss_mask_off=mo, logprob_vals=lv, logprob_off=lo, pad_token_id=np.int64(0),
         sequences=seq, attention_mask=att, response_mask=am, rewards=rw, loss_mask=lm, rollout_logprobs=lp,
         pad_size=np.int64(padded.metadata["pad_size"]), p_sequences=padded["sequences"],
         p_attention_mask=padded["attention_mask"], p_response_mask=padded["response_mask"],
         p_rewards=padded["rewards"], p_loss_mask=padded["loss_mask"], p_rollout_logprobs=padded["rollout_logprobs"],
         p_uids=np.array(padded.metadata["uids"]))


def gen_reward_kl(trainer_mod, tb, cfgmod):
    g = torch.Generator().manual_seed(8)
    N, R = 9, 21
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).float()
    lp = torch.randn(N, R, generator=g) - 2
    base = lp + torch.randn(N, R, generator=g) * 0.4
    rew = torch.zeros(N, R)
    rew[torch.arange(N), lens - 1] = 1.0
    out = {}
    for kind in ("k1", "k3"):
        batch = tb.TrainingInputBatch({"loss_mask": mask, "rewards": rew.clone(), "base_action_log_probs": base,
                                       "action_log_probs": lp})
        batch.metadata = {}
        cfg = SimpleNamespace(trainer=SimpleNamespace(algorithm=cfgmod.AlgorithmConfig(kl_estimator_type=kind,
                                                                                       kl_loss_coef=0.05)))
        fake = SimpleNamespace(cfg=cfg, reward_kl_controller=None, all_metrics={})
        res = trainer_mod.RayPPOTrainer.apply_reward_kl_penalty(fake, batch)
        out[f"rewards_{kind}"] = res["rewards"]
        out[f"avg_kl_{kind}"] = np.float32(res.metadata["metrics"]["avg_kl"])
        out[f"avg_kl_max_{kind}"] = np.float32(res.metadata["metrics"]["avg_kl_max"])
    save("reward_kl", rewards=rew, loss_mask=mask, action_log_probs=lp, base_action_log_probs=base, kl_coef=0.05,
         **out)


def _metrics(out, tag, m):
    keys = sorted(m)
    out[f"mkeys_{tag}"] = np.array(keys)
    out[f"mvals_{tag}"] = np.array([float(m[k]) for k in keys], dtype=np.float64)


def gen_secondary(pu, cfgmod):
    """The secondary registry entries (ppo_utils.py:589-981 losses, :1013-1098 estimators) on the
    reference's own KAT inputs (tests/cpu/algorithms/test_losses.py:85-137, 291-402, 442-615;
    tests/cpu/utils/test_ppo_utils.py:65-129) and on seeded ragged batches, with every
    reduction and (where the loss applies it) off-policy correction. Records loss, metrics and
    dL/dlog_probs (autograd). clip_cov draws torch.randperm: the global seed is set right before
    each call (the restatement consumes the generator identically)."""
    out = {}
    null_opc = cfgmod.OffPolicyCorrectionConfig(tis_ratio_type=None, sequence_mask_metric=None,
                                                outlier_token_is_threshold_low=None,
                                                outlier_token_is_threshold_high=None)
    cases = []  # (tag, loss name, lp, old, adv, mask or None, rollout or None, cfg kwargs, seed)
    # --- the reference's KAT inputs
    adv3 = torch.tensor([[1.0, -1.0, -4.0]])
    old3 = torch.tensor([[-1.0, -1.0, -3.0]])
    lp3 = torch.tensor([[-1.69315, -1.0, -0.69741]])
    cases.append(("kat_cispo", "cispo", lp3, old3, adv3, None, None,
                  dict(cispo=cfgmod.CISPOConfig(cispo_eps_clip_low=0.2, cispo_eps_clip_high=0.2),
                       loss_reduction="token_mean", max_seq_len=4), 0))
    gadv = torch.tensor([[1.5, 2.0, 1.0, 0.8, 0.5, 0.0, 0.0, 0.0], [3.0, 1.5, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0],
                         [0.5, 0.8, 1.2, 2.5, 0.0, 0.0, 0.0, 0.0]])
    gold = torch.full((3, 8), -1.0)
    glp = torch.tensor([[0.2, -2.5, -0.3, 0.1, -1.8, -1.0, -1.0, -1.0], [0.8, -0.2, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0],
                        [-0.5, 0.3, -1.7, 0.4, -1.0, -1.0, -1.0, -1.0]])
    gmask = torch.tensor([[1.0, 1.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0], [1.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0],
                          [1.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0]])
    cases.append(("kat_gspo", "gspo", glp, gold, gadv, gmask, None,
                  dict(eps_clip_low=0.2, eps_clip_high=0.2, clip_ratio_c=3.0, loss_reduction="sequence_mean",
                       max_seq_len=4), 0))
    cadv = torch.tensor([[2.0, -1.0, 1.5, 0.8], [1.0, 0.5, -2.0, 1.2]])
    cold = torch.full((2, 4), -1.0)
    clp = torch.tensor([[-0.5, -1.5, -0.8, -1.2], [-1.3, -0.7, -1.8, -0.9]])
    cmask = torch.tensor([[1.0, 1.0, 1.0, 1.0], [1.0, 1.0, 1.0, 0.0]])
    cases.append(("kat_clip_cov", "clip_cov", clp, cold, cadv, cmask, None,
                  dict(eps_clip_low=0.2, eps_clip_high=0.2, loss_reduction="token_mean", max_seq_len=4,
                       clip_cov=cfgmod.ClipCovConfig(clip_ratio=0.5, clip_cov_lb=-5.0, clip_cov_ub=5.0)), 42))
    kadv = torch.tensor([[1.5, -0.5, 2.0, 0.8], [0.5, 1.0, -1.5, 1.2]])
    klp = torch.tensor([[-0.8, -1.2, -0.6, -1.1], [-1.1, -0.9, -1.4, -0.7]])
    cases.append(("kat_kl_cov", "kl_cov", klp, cold, kadv, cmask, None,
                  dict(loss_reduction="token_mean", max_seq_len=4,
                       kl_cov=cfgmod.KLCovConfig(kl_cov_frac=0.5, ppo_kl_coef=1.0)), 42))
    sadv = torch.tensor([[1.0, -1.0, 0.5]])
    slp = torch.tensor([[-1.5, -0.8, -1.1]])
    cases.append(("kat_sapo", "sapo", slp, torch.full((1, 3), -1.0), sadv, None, None,
                  dict(loss_reduction="sequence_mean", max_seq_len=4,
                       sapo=cfgmod.SAPOConfig(tau_pos=1.0, tau_neg=2.0)), 0))
    # --- seeded ragged batches: every reduction, off-policy correction where the loss applies it
    g = torch.Generator().manual_seed(2024)
    n, R = 6, 37
    lp, old, adv, mask, ref, ent = _ppo_inputs(g, n, R)
    rollout = old + torch.randn(n, R, generator=g) * 0.05
    rollout[3] = old[3] - 1.5
    extra = {"gspo": dict(eps_clip_low=0.2, eps_clip_high=0.28),
             "sapo": dict(sapo=cfgmod.SAPOConfig(tau_pos=1.0, tau_neg=1.05)),
             "cispo": dict(cispo=cfgmod.CISPOConfig(cispo_eps_clip_low=0.2, cispo_eps_clip_high=0.3)),
             "clip_cov": dict(eps_clip_low=0.2, eps_clip_high=0.28,
                              clip_cov=cfgmod.ClipCovConfig(clip_ratio=0.05, clip_cov_lb=-1.0, clip_cov_ub=2.0)),
             "kl_cov": dict(kl_cov=cfgmod.KLCovConfig(kl_cov_frac=0.1, ppo_kl_coef=0.5)),
             "cross_entropy": {}, "importance_sampling": {}}
    for name, kw in extra.items():
        reds = ("token_mean",) if name in ("cross_entropy", "importance_sampling") else (
            "token_mean", "sequence_mean", "seq_mean_token_sum_norm")
        for red in reds:
            cases.append((f"rand_{name}_{red}", name, lp, old, adv, mask, None,
                          dict(kw, loss_reduction=red, max_seq_len=50), 7))
        if name in ("gspo", "sapo", "cispo"):  # these apply apply_off_policy_correction
            opc = cfgmod.OffPolicyCorrectionConfig(tis_ratio_type="token", token_tis_ratio_clip_high=2.0,
                                                   sequence_mask_metric="product", product_mask_high=2.0,
                                                   product_mask_low=0.5)
            cases.append((f"rand_{name}_offpolicy", name, lp, old, adv, mask, rollout,
                          dict(kw, loss_reduction="token_mean", max_seq_len=50, off_policy_correction=opc), 7))
    tags = []
    for tag, name, x0, o, a, m, ro, kw, seed in cases:
        kw = dict(kw)
        kw.setdefault("off_policy_correction", null_opc)
        cfg = cfgmod.AlgorithmConfig(policy_loss_type=name, **kw)
        x = x0.clone().requires_grad_(True)
        torch.manual_seed(seed)
        loss, met = pu.PolicyLossRegistry.get(name)(x, o, a, cfg, loss_mask=m, rollout_logprobs=ro)
        loss.backward()
        out[f"lp_{tag}"] = x0
        out[f"old_{tag}"] = o
        out[f"adv_{tag}"] = a
        if m is not None:
            out[f"mask_{tag}"] = m
        if ro is not None:
            out[f"rollout_{tag}"] = ro
        out[f"loss_{tag}"] = loss.detach()
        out[f"grad_{tag}"] = x.grad if x.grad is not None else torch.zeros_like(x0)
        _metrics(out, tag, met)
        cfgd = {k: (dataclasses.asdict(v) if dataclasses.is_dataclass(v) else v) for k, v in kw.items()}
        cfgd["policy_loss_type"] = name
        out[f"cfg_{tag}"] = np.array(json.dumps(cfgd, sort_keys=True))
        out[f"seed_{tag}"] = np.int64(seed)
        tags.append(tag)
    # --- estimators: the KAT inputs and a seeded ragged batch
    est = []
    r3 = torch.tensor([[1.0, 2.0, 3.0]])
    est.append(("kat_rpp_g1", "reinforce++", r3, torch.tensor([[1.0, 1.0, 0.0]]), None, 1.0))
    est.append(("kat_rpp_g05", "reinforce++", r3, torch.ones(1, 3), None, 0.5))
    rl = torch.tensor([[0.0, 0.0, 6.0], [0.0, 0.0, 3.0], [0.0, 0.0, 9.0], [0.0, 0.0, 12.0], [0.0, 0.0, 1.0]])
    est.append(("kat_rloo", "rloo", rl, torch.ones_like(rl), np.array([0, 0, 1, 1, 2]), 1.0))
    g2 = torch.Generator().manual_seed(77)
    rn, rR = 12, 19
    lens = torch.randint(1, rR + 1, (rn,), generator=g2)
    rmask = (torch.arange(rR)[None, :] < lens[:, None]).float()
    rrew = torch.randn(rn, rR, generator=g2) * rmask
    ridx = np.array([str(i // 4) for i in range(rn - 1)] + ["solo"])
    est.append(("rand_rpp", "reinforce++", rrew, rmask, None, 0.97))
    est.append(("rand_rloo", "rloo", rrew, rmask, ridx, 1.0))
    etags = []
    for tag, name, rew, rm, idx, gamma in est:
        fn = pu.AdvantageEstimatorRegistry.get(name)
        a, r = fn(token_level_rewards=rew.clone(), response_mask=rm, index=idx, gamma=gamma)
        out[f"rew_{tag}"] = rew
        out[f"rmask_{tag}"] = rm
        if idx is not None:
            out[f"index_{tag}"] = np.asarray(idx).astype(str)
        out[f"gamma_{tag}"] = np.float64(gamma)
        out[f"eadv_{tag}"] = a
        out[f"eret_{tag}"] = r
        etags.append(tag)
    save("secondary", loss_tags=np.array(tags), est_tags=np.array(etags), **out)


def main():
    install_shim()
    torch.set_num_threads(4)
    from skyrl_train import config as cfgmod
    from skyrl_train import trainer as trainer_mod
    from skyrl_train import training_batch as tb
    from skyrl_train.dataset import preprocess as pre
    from skyrl_train.utils import ppo_utils as pu
    from skyrl_train.utils import torch_utils as tu

    assert not tu.FLASH_ATTN_CROSS_ENTROPY_LOSS_AVAILABLE
    jobs = {
        "grpo": lambda: gen_grpo(pu),
        "advnorm": lambda: gen_advnorm(pu),
        "gae": lambda: gen_gae(pu),
        "kl": lambda: gen_kl(pu),
        "ppo": lambda: gen_ppo(pu, cfgmod),
        "ppo_offpolicy": lambda: gen_ppo_offpolicy(pu, cfgmod),
        "critic": lambda: gen_critic(pu, cfgmod),
        "logprob": lambda: gen_logprob(tu),
        "pack": lambda: gen_pack(pre, trainer_mod, tb),
        "reward_kl": lambda: gen_reward_kl(trainer_mod, tb, cfgmod),
        "secondary": lambda: gen_secondary(pu, cfgmod),
    }
    for name in (sys.argv[1:] or list(jobs)):  # `python -B tools/gen_golden.py ppo_offpolicy` regenerates one
        jobs[name]()


if __name__ == "__main__":
    main()
