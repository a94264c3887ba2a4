"""Sample packing on the learner (skyrl_amd/packing.py; reference use_sample_packing,
model_wrapper.py:272-330): the packed [1, nnz] forward through the ROCm varlen flash attention
gives the padded forward's hidden states, logprobs and gradients (bf16 tolerance; the two runs
order their reductions differently), with and without gradient checkpointing, for Qwen2
(GQA + qkv bias) and Llama."""

import pytest
import torch

from skyrl_amd.config import AlgorithmConfig
from skyrl_amd.packing import enable_sample_packing, packed_hidden_states
from skyrl_amd.trainer import GRPOTrainer, TrainerConfig, _positions

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def model_and_batch(kind, seed=0):
    from transformers import AutoModelForCausalLM, LlamaConfig, Qwen2Config

    kw = dict(vocab_size=997, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, max_position_embeddings=512, tie_word_embeddings=(kind == "qwen2"))
    cfg = Qwen2Config(**kw) if kind == "qwen2" else LlamaConfig(**kw)
    torch.manual_seed(seed)
    m = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("bias"):
                p.add_(0.1 * torch.randn_like(p))
    g = torch.Generator().manual_seed(seed + 1)
    n, P, R = 5, 24, 40
    pl = torch.tensor([1, 24, 7, 13, 20])
    rl = torch.tensor([40, 1, 17, 33, 2])
    S = P + R
    seq = torch.randint(0, 997, (n, S), generator=g)
    col = torch.arange(S)
    att = ((col[None] >= P - pl[:, None]) & (col[None] < P + rl[:, None])).long()
    rmask = (torch.arange(R)[None] < rl[:, None]).float()
    return m, seq.to(DEV), att.to(DEV), rmask.to(DEV), R


@pytest.mark.parametrize("kind", ["qwen2", "llama"])
@pytest.mark.parametrize("ckpt", [False, True])
def test_packed_forward_matches_padded(kind, ckpt):
    m, seq, att, rmask, R = model_and_batch(kind)
    if ckpt:
        m.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
        m.config.use_cache = False
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = m.model(input_ids=seq, attention_mask=att, position_ids=_positions(att)).last_hidden_state[:, -R - 1:-1]
    (ref.float().pow(2) * rmask[..., None]).sum().backward()
    gref = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    enable_sample_packing(m)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        h = packed_hidden_states(m.model, seq, att, R)
    valid = rmask.bool()
    # the last prompt position (column 0) is always a valid token too
    valid[:, 0] = True
    err = (h.float() - ref.float())[valid].norm() / ref.float()[valid].norm()
    assert err < 1e-2, err
    (h.float().pow(2) * rmask[..., None]).sum().backward()
    for n, p in m.named_parameters():
        if n in gref:
            e = (p.grad - gref[n]).norm() / gref[n].norm().clamp_min(1e-12)
            assert e < 3e-2, (n, float(e))
    # the switched model still runs padded batches (SDPA fall-through)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        again = m.model(input_ids=seq, attention_mask=att, position_ids=_positions(att)).last_hidden_state[:, -R - 1:-1]
    assert (again.float() - ref.float())[valid].abs().max() < 0.05


def test_trainer_logprobs_packed_vs_padded():
    m, seq, att, rmask, R = model_and_batch("qwen2", seed=3)
    out = {}
    for packing in (False, True):
        tr = GRPOTrainer(TrainerConfig(use_sample_packing=packing, micro_forward_batch_size_per_gpu=2,
                                       algorithm=AlgorithmConfig(use_kl_loss=False)), m, None, None, pad_token_id=0)
        out[packing] = tr._fwd_logprobs(m, {"sequences": seq, "attention_mask": att,
                                            "response_mask": rmask.long()})
    d = (out[True] - out[False]).abs()[rmask.bool()]
    assert d.max() < 0.05 and d.mean() < 5e-3, (float(d.max()), float(d.mean()))
