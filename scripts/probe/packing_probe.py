"""Sample packing on the learner: (1) varlen flash attention (GQA, causal) vs SDPA per
sequence, fwd + bwd; (2) Qwen2.5-1.5B shape (28 layers) fwd+bwd of a 16-sequence micro-batch
with the e2e length distribution, padded vs packed."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from skyrl_amd.packing import enable_sample_packing, packed_hidden_states  # noqa: E402

DEV = torch.device("cuda:0")


def varlen_check():
    from torch.nn.attention.varlen import varlen_attn

    g = torch.Generator(device=DEV).manual_seed(0)
    lens = [37, 128, 5, 300]
    H, Hk, D = 12, 2, 128
    T = sum(lens)
    q = torch.randn(T, H, D, device=DEV, generator=g, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(T, Hk, D, device=DEV, generator=g, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(T, Hk, D, device=DEV, generator=g, dtype=torch.bfloat16, requires_grad=True)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    res = {}
    try:
        out = varlen_attn(q, k, v, cu, cu, max(lens), max(lens), is_causal=True)
        res["gqa_native"] = True
    except Exception as e:  # noqa: BLE001
        res["gqa_native"] = f"{type(e).__name__}: {str(e)[:200]}"
        out = varlen_attn(q, k.repeat_interleave(6, 1), v.repeat_interleave(6, 1), cu, cu, max(lens), max(lens),
                          is_causal=True)
    ref = []
    for a, b in zip(cu[:-1].tolist(), cu[1:].tolist()):
        ref.append(F.scaled_dot_product_attention(q[a:b].transpose(0, 1)[None], k[a:b].transpose(0, 1)[None].float().to(
            torch.bfloat16), v[a:b].transpose(0, 1)[None], is_causal=True, enable_gqa=True)[0].transpose(0, 1))
    ref = torch.cat(ref)
    res["fwd_max_err"] = float((out.float() - ref.float()).abs().max())
    go = torch.randn_like(out)
    gq, gk, gv = torch.autograd.grad(out, (q, k, v), go)
    rq, rk, rv = torch.autograd.grad(ref, (q, k, v), go)
    res["bwd_rel_err"] = [float((a.float() - b.float()).norm() / b.float().norm()) for a, b in ((gq, rq), (gk, rk), (gv, rv))]
    return res


def model_timing(packed: bool, reps=3):
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(vocab_size=151936, hidden_size=1536, intermediate_size=8960, num_hidden_layers=28,
                      num_attention_heads=12, num_key_value_heads=2, max_position_embeddings=32768,
                      rope_theta=1000000.0, rms_norm_eps=1e-6, tie_word_embeddings=True)
    torch.manual_seed(0)
    m = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    m.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
    m.config.use_cache = False
    if packed:
        enable_sample_packing(m)
    g = torch.Generator().manual_seed(1)
    n, P, R = 16, 512, 1024
    pl = torch.randint(16, 513, (n,), generator=g)
    rl = torch.randint(1, 1025, (n,), generator=g)
    S = P + R
    seq = torch.randint(0, 151936, (n, S), generator=g).to(DEV)
    col = torch.arange(S)
    att = ((col[None] >= P - pl[:, None]) & (col[None] < P + rl[:, None])).long().to(DEV)
    from skyrl_amd.trainer import _positions

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if packed:
                h = packed_hidden_states(m.model, seq, att, R)
            else:
                h = m.model(input_ids=seq, attention_mask=att, position_ids=_positions(att)).last_hidden_state[:, -R - 1:-1]
            loss = h.float().pow(2).mean()
        loss.backward()
        return h

    h = step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, h.detach(), int(att.sum())


if __name__ == "__main__":
    out = {"varlen": varlen_check()}
    print(json.dumps(out), flush=True)
    tp, hp, nnz = model_timing(True)
    print(json.dumps({"packed_s": tp, "nnz": nnz}), flush=True)
    tu, hu, _ = model_timing(False)
    out.update(packed_s=round(tp, 3), padded_s=round(tu, 3), nnz=nnz, padded_tokens=16 * 1536)
    print(json.dumps(out), flush=True)
