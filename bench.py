"""Hot-path benchmark: trained samples/sec (rollout + update) of the GRPO actor-learner loop.

Workload (BASELINE.json configs[1] shape, the metric's [batch=64, seq=1024, group=8]):
64 prompts x group 8 = 512 trajectories, response width R = 1024, prompt width P = 512,
Qwen2.5-1.5B vocabulary V = 151,936, bf16 logits. With N ranks (strong scaling, the default)
the 512 trajectories are ONE global batch and rank r runs rows [r*512/N, (r+1)*512/N), whole
prompt groups (the reference's DP chunking distributed/dispatch.py:122-141).
One step is one pass of the hot path over one synthetic batch (per rank, its rows):

  rollout   R decode steps of skyrl_sample over [512, V] logits (T=1, top_p=1, top_k=-1)
  pack      skyrl_pack_experience: ragged prompts/responses -> padded training tensors
  ref/old   skyrl_logprob_fwd over all 512x1024 response positions (2 passes)
  update    the step form of the fused policy pass (GRPOTrainer's): skyrl_policy_train_plan_grpo
            (GRPO advantages over contiguous groups from pack's reward row sums + every
            micro-batch's loss scales, one launch), per micro-batch (16 seqs)
            skyrl_policy_train_micro_fwd, ONE pass per token computing logprob + entropy + PPO/KL
            loss terms and writing dlogits (bf16), each row held in the registers of 6
            workgroups, then skyrl_policy_train_fold (every micro-batch's loss + metrics, one
            launch); metrics read once per step
  optimizer grad norm + clip + AdamW over Qwen2.5-1.5B's 1.54 B fp32 params, writing the bf16
            rollout copy (reduce-scatter / all-gather over RCCL when N > 1)

The transformer forward/backward is outside the hot path (north_star: PyTorch-ROCm owns it),
so its logits are synthetic and resident in HBM before timing (data="synthetic"). With N > 1
ranks no data-path collective is needed (the advantage / loss / logprob / sampler rows shard by
whole prompt groups); the exchanges are the DP gradient reduce-scatter, the grad-norm scalar,
the bf16 weight all-gather (the learner -> rollout sync) and one packed fp32 metric all-reduce
per step, over RCCL. Over DP ranks the weight sync is in flight (configs 3/5): the optimizer
chain runs on the comm stream under the next step's rollout and ref pass. --scaling weak gives
every rank a 512-trajectory batch of its own; --emulate-world W times one rank's share of a
W-rank job on one GPU (collectives excluded).

Every hot kernel is timed live with HIP events on its launch stream (the dominant one feeds
`roofline`). After the timed steps, the advantage + loss kernels (56 B/token)
are replayed from a HIP graph at the batch size and at 16x it (`advantage_loss`). The CPU
oracle (oracle/cpu_ref.py + oracle/sampler_ref.c, "port") is timed on a bounded sample on
rank 0 at N=1.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

P_MAX, R_MAX, PROMPTS, GROUP, VOCAB = 512, 1024, 64, 8, 151936
QWEN_1_5B_PARAMS = 1_543_714_304  # Qwen2.5-1.5B, tied embeddings
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def SAMPLER_LABEL(nrows, rollout="live"):
    """The T = 1 sampler kernel(s) the library picks (csrc/sampler.hip launch_sample: at or above
    256 rows one 512-thread workgroup per row, below it the split form of the same kernel)."""
    if rollout == "live":
        return ("skyrl_sample over the live decode batch (sample_kernel<bf16,3,512> one workgroup per row at >= 256 "
                "live rows, sample_kernel<bf16,3,256> below: rows split over workgroups, last arriver merges)")
    if nrows >= 256:
        return "skyrl_sample (sample_kernel<bf16,3,512>: T=1, one workgroup per row)"
    return ("skyrl_sample (sample_kernel<bf16,3,256>: T=1, each row over several 256-thread workgroups, last "
            "arriver merges)")
# reported beside frac, never instead of it: the guide's measured float4 copy (MI355X_MICROARCH.md,
# "6.29 TB/s measured") for read+write kernels, and the read-only grid-stride stream our probe
# measured on the box (7.0-7.1 TB/s, profiles/r03_rw_ceiling_probe2.log) for read-only kernels
CEILING_READ_GBS = 7100.0
CEILING_RW_GBS = 6290.0


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def rank_rows(n_global, world, rank):
    """SURVEY §8(e) / the reference's DP rule (distributed/dispatch.py:122-141: chunk_size =
    len(data) // dp_size, rank r takes rows [r*chunk, (r+1)*chunk)): ONE global batch split into
    contiguous row ranges of whole prompt groups. Returns (first row, rows)."""
    if n_global % world or (n_global // world) % GROUP:
        raise ValueError(f"{n_global} trajectories do not split into whole groups of {GROUP} over {world} ranks")
    rows = n_global // world
    return rank * rows, rows


def synth_inputs(dev, N, seed=1234, row0=0, rows=None):
    """SURVEY §8(d) synthetic batch of N trajectories (torch.Generator seed 1234), of which rows
    [row0, row0 + rows) are returned (a DP rank's chunk): the global batch is drawn first, so
    every rank of every world size sees the same trajectories as the N = 1 run."""
    g = torch.Generator().manual_seed(seed)
    plens = torch.randint(16, P_MAX + 1, (PROMPTS,), generator=g).repeat_interleave(GROUP)[:N]
    rlens = torch.randint(1, R_MAX + 1, (N,), generator=g)
    rlens[0] = R_MAX  # the padded width is R_MAX
    plens[0] = P_MAX
    hit = (torch.rand(N, generator=g) < 0.3).float()
    poff = torch.zeros(N + 1, dtype=torch.int64)
    poff[1:] = torch.cumsum(plens, 0)
    roff = torch.zeros(N + 1, dtype=torch.int64)
    roff[1:] = torch.cumsum(rlens, 0)
    ptok = torch.randint(0, VOCAB, (int(poff[-1]),), generator=g)
    rtok = torch.randint(0, VOCAB, (int(roff[-1]),), generator=g)
    rew = torch.zeros(int(roff[-1]))
    rew[roff[1:] - 1] = hit
    lmask = torch.ones(int(roff[-1]))
    rlp = -2 + 0.1 * torch.randn(int(roff[-1]), generator=g)
    rows = N - row0 if rows is None else rows
    a, b = row0, row0 + rows
    pa, pb, ra, rb = int(poff[a]), int(poff[b]), int(roff[a]), int(roff[b])
    uids = [str(i // GROUP) for i in range(a, b)]
    d = dict(plens=plens[a:b], rlens=rlens[a:b], poff=poff[a:b + 1] - pa, roff=roff[a:b + 1] - ra,
             ptok=ptok[pa:pb], rtok=rtok[ra:rb], rew=rew[ra:rb], lmask=lmask[ra:rb], rlp=rlp[ra:rb])
    return {k: v.to(dev) for k, v in d.items()}, uids


def fill_logits(dev, rows, V, chunk_rows=8192):
    """Resident bf16 logits [rows, V] ~ N(0, 3^2), generated on device in chunks."""
    x = torch.empty((rows, V), dtype=torch.bfloat16, device=dev)
    gen = torch.Generator(device=dev).manual_seed(42)
    for s in range(0, rows, chunk_rows):
        e = min(rows, s + chunk_rows)
        x[s:e].normal_(0.0, 3.0, generator=gen)
    return x


class KernelTimer:
    """HIP events around launches of one kernel on its launch stream (timed region only)."""

    def __init__(self):
        self.pairs = []
        self.active = False

    def wrap(self, fn):
        if not self.active:
            return fn()
        s = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        out = fn()
        b.record(s)
        self.pairs.append((a, b))
        return out

    def begin(self):
        """Open a block of back-to-back launches (one event pair per block, see end())."""
        if self.active:
            self._open = torch.cuda.Event(enable_timing=True)
            self._open.record(torch.cuda.current_stream())

    def end(self, launches):
        if self.active:
            b = torch.cuda.Event(enable_timing=True)
            b.record(torch.cuda.current_stream())
            self.pairs.append((self._open, b, launches))

    @property
    def launches(self):
        return sum(p[2] if len(p) > 2 else 1 for p in self.pairs)

    def avg_ms(self):
        if not self.pairs:
            return float("nan")
        return sum(p[0].elapsed_time(p[1]) for p in self.pairs) / self.launches


def run(args):
    from skyrl_amd import ops, ppo_utils
    from skyrl_amd.config import AlgorithmConfig

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # SKYRL_FORCE_COLLECTIVES=1 under a one-rank torchrun: the group is initialized and every
    # exchange runs as a (one-rank) RCCL collective, so the N>1 code path runs on one GPU
    dist_on = world > 1 or os.environ.get("SKYRL_FORCE_COLLECTIVES", "0") == "1"
    if dist_on:
        import datetime

        # rank 0 runs the single-GPU legs after the timed region while the others wait at the
        # final barrier: a timeout well above those legs' length
        tmo = datetime.timedelta(minutes=60)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:  # rehearsal of the N>1 path with several ranks on one GPU (RCCL refuses duplicate GPUs)
            dist.init_process_group(args.backend, timeout=tmo)
        world = dist.get_world_size()  # n_gpus is the communicator's size
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but the launcher started {world} ranks; reporting n_gpus = {world}")
    R, V, mb = R_MAX, VOCAB, args.micro_batch
    # the work split: strong scaling (default) cuts ONE global batch of 64 prompts x G 8 = 512
    # trajectories into contiguous whole-group row ranges, one per rank (the
    # reference's MeshDispatch, distributed/dispatch.py:122-141); --scaling weak gives every rank a
    # batch of its own. --emulate-world W (one process) runs rank --emulate-rank's share of a
    # W-rank strong-scaling job: its rows, its 1/W optimizer shard, no collectives.
    emulate = args.emulate_world if world == 1 else 1
    N_GLOBAL = PROMPTS * GROUP * (world if args.scaling == "weak" else 1)
    if args.scaling == "weak":
        row0, N = 0, PROMPTS * GROUP
        data, uids = synth_inputs(dev, N, seed=1234 + rank)
    else:
        part_world, part_rank = (emulate, args.emulate_rank) if emulate > 1 else (world, rank)
        row0, N = rank_rows(N_GLOBAL, part_world, part_rank)
        data, uids = synth_inputs(dev, N_GLOBAL, seed=1234, row0=row0, rows=N)
    if N % mb:
        raise ValueError(f"{N} rows per rank are not a multiple of the micro-batch {mb}")
    log(f"rank {rank}/{world}: rows [{row0}, {row0 + N}) of a {N_GLOBAL}-trajectory global batch "
        f"({args.scaling} scaling{f', emulating rank {args.emulate_rank} of {emulate}' if emulate > 1 else ''})")
    # weight-sync order: "sync" (the default at every world size): the optimizer step runs on the
    # compute stream and the next rollout waits for the weight all-gather, as the reference pauses
    # generation for the sync (fully_async_trainer.py:415-419); "inflight" (opt-in): reduce-scatter
    # + clip/AdamW + all-gather on the comm stream under the next step's rollout and ref pass, the
    # old-policy pass waiting for the new weights. The inflight overlap rewrites the rollout
    # weights during generation, so it stands for an engine with double-buffered rollout weights;
    # with synthetic logits nothing here reads them.
    inflight = args.weight_sync == "inflight"

    # a12/a14 learner state: flat fp32 gradient of the policy (written by the transformer backward,
    # outside the path: synthetic here), FSDP2-style sharded AdamW, bf16 rollout weights
    from skyrl_amd import comm

    reducer = opt = None
    n_params = -(-args.params // emulate)  # an emulated rank's shard (the real layout pads to 64 x W)
    if args.params > 0:
        reducer = comm.GradReducer(n_params, dev, bucket_bytes=args.bucket_mb << 20)
        init = torch.empty(n_params, dtype=torch.float32, device=dev).normal_(0.0, 0.02)
        opt = comm.ShardedAdamW(reducer, init, comm.AdamWConfig())
        del init
        reducer.grad.normal_(0.0, 1e-3)
        torch.cuda.synchronize()
    upd_done = None  # inflight: the comm stream's update of the previous step

    # resident logits: all N*R response positions if HBM allows, else a pool reused round-robin
    free, _ = torch.cuda.mem_get_info(dev)
    row_bytes = V * 2
    dlogits_bytes = mb * R * row_bytes
    budget = free - dlogits_bytes - (8 << 30)
    rows = N * R if args.logits_rows <= 0 else args.logits_rows
    rows = int(min(rows, max(mb * R, budget // row_bytes)))
    rows = (rows // (mb * R)) * (mb * R)
    log(f"rank {rank}/{world}: free HBM {free / 2**30:.1f} GiB, resident logits rows {rows} "
        f"({rows * row_bytes / 2**30:.1f} GiB; full batch needs {N * R})")
    logits = fill_logits(dev, rows, V)
    dlogits = torch.empty((mb, R, V), dtype=torch.bfloat16, device=dev)
    full = rows == N * R
    n_pools = rows // (mb * R)

    def lg_rows(seq0, nseq):  # [nseq, R, V] view of the logits of sequences seq0..
        blk = (seq0 // mb) % n_pools
        return logits[blk * mb * R:(blk + 1) * mb * R].view(mb, R, V)[: nseq] if not full else \
            logits[seq0 * R:(seq0 + nseq) * R].view(nseq, R, V)

    # decode slots. The rollout's decode batch holds the LIVE sequences (logits
    # [num_live_seqs, V]): a sequence leaves after its last token, as vLLM's continuous batching
    # does. Slot s holds trajectory order[s], longest response first, so decode step t samples
    # slots [0, live[t]); --rollout all keeps every sequence in the batch for all R steps (the
    # r01-r05 bench). The resident logits are indexed by slot for the rollout (synthetic values).
    roff = data["roff"]
    rl_cpu = data["rlens"].cpu()
    order = (torch.argsort(-rl_cpu, stable=True) if args.rollout == "live" else torch.arange(N)).to(dev)
    slot_of = torch.empty_like(order)
    slot_of[order] = torch.arange(N, device=dev)
    srt = torch.sort(rl_cpu, descending=True).values
    live = [int((srt > t).sum()) if args.rollout == "live" else N for t in range(R)]
    # the rollout's sampled tokens / logprobs ([R, N] per decode step, by slot) become the ragged
    # response CSR that pack consumes: token j of sequence n was sampled at decode step j - roff[n]
    tok_n = torch.repeat_interleave(torch.arange(N, device=dev), data["rlens"])
    tok_t = torch.arange(int(roff[-1]), device=dev) - roff[:-1][tok_n]
    tok_s = slot_of[tok_n]
    # sampler keys are the global trajectory ids: a trajectory's tokens do not depend on the world size
    seq_ids = (torch.arange(N, device=dev, dtype=torch.int64) + (row0 if args.scaling == "strong" else rank * N))[order]
    from skyrl_amd.config import SamplingParams
    from skyrl_amd.sampler import TokenSampler

    sampler = TokenSampler(N, V, R, dev, SamplingParams(), seed=0, seq_ids=seq_ids)
    base_ptr = logits.data_ptr()
    _, _, ng = ops.groups_from_index(uids)  # contiguous groups of GROUP rows (uid = i // GROUP)
    cfg = AlgorithmConfig()
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, has_entropy=True)
    fwd_timer = KernelTimer()
    train_timer = KernelTimer()
    sample_timer = KernelTimer()
    adam_timer = KernelTimer()
    timers = (fwd_timer, train_timer, sample_timer, adam_timer)
    lp = torch.empty((mb, R), dtype=torch.float32, device=dev)
    ent = torch.empty_like(lp)
    lse = torch.empty_like(lp)
    # the step form of the fused pass (GRPOTrainer's): one plan launch (every micro-batch's loss
    # scales), the micro-batches' passes, one fold launch (every micro-batch's loss + metrics)
    n_micro = N // mb
    step_ws = torch.zeros(ops._ffi.query("skyrl_policy_train_step_workspace_bytes", N, R, mb), dtype=torch.uint8,
                          device=dev)
    step_loss = torch.empty(n_micro, dtype=torch.float32, device=dev)
    step_met = torch.empty((n_micro, 8), dtype=torch.float32, device=dev)
    step_lp = torch.empty((N, R), dtype=torch.float32, device=dev)
    step_ent = torch.empty((N, R), dtype=torch.float32, device=dev)
    step_adv = torch.empty((N, R), dtype=torch.float32, device=dev)
    metrics_acc = torch.zeros(8, dtype=torch.float32, device=dev)
    grpo_timer, plan_timer, fold_timer = KernelTimer(), KernelTimer(), KernelTimer()
    timers = timers + (grpo_timer, plan_timer, fold_timer)

    def step(step_idx):
        nonlocal upd_done
        # ---- rollout: R decode steps over [N, V] logits (row stride R*V in the resident tensor)
        sampler.seed = step_idx
        if opt is not None and not inflight:  # generation starts on the previous step's new weights
            opt.wait_weights()
        sh = torch.cuda.current_stream(dev).cuda_stream
        for t in range(R):
            ptr, ld = (base_ptr + 2 * V * t, R * V) if full else (base_ptr + 2 * V * ((t * N) % (rows - N + 1)), V)
            if t % 64 == 0:  # event-timed in blocks of 64 back-to-back decode-step launches
                sample_timer.begin()
            sampler.step_ptr(ptr, ld, t, sh, nseq=live[t])
            if t % 64 == 63 or t == R - 1:
                sample_timer.end(t % 64 + 1)
        # ---- pack ragged rollout output into the padded training tensors
        rtok = sampler.tokens[tok_t, tok_s]
        rlp_sampled = sampler.logprobs[tok_t, tok_s]
        seqs, att, rmask, rew, lmask, rlp, lrows, scores = ops.pack_experience(
            data["ptok"], data["poff"], rtok, roff, data["rew"], roff, data["lmask"],
            roff, rlp_sampled, roff, N=N, P=P_MAX, R=R, pad=0, pad_token_id=0, return_row_sums=True)
        labels = seqs[:, P_MAX:]  # the sampled response tokens (int64 view, row stride P+R)
        # ---- ref + old policy logprobs over all response positions (no grad). The old policy is the
        #      rollout policy (on-policy, one mini-batch per step: ratio 1 as in the reference); the ref
        #      policy's logits stand in as another sequence block's, so KL-to-ref is nonzero
        ref_lp = torch.empty((N, R), dtype=torch.float32, device=dev)
        old_lp = torch.empty((N, R), dtype=torch.float32, device=dev)
        for which in ("ref", "old"):  # the ref model's pass needs no policy weights; the old pass does
            if which == "old" and inflight and opt is not None:
                if upd_done is not None:
                    torch.cuda.current_stream(dev).wait_event(upd_done)
                opt.wait_weights()
            for s in range(0, N, mb):
                lab = labels[s:s + mb]
                out, x = (ref_lp, lg_rows((s + mb) % N, mb)) if which == "ref" else (old_lp, lg_rows(s, mb))
                fwd_timer.wrap(lambda: ops._ffi.call(
                    "skyrl_logprob_fwd", ops._ptr(x), ops.BF16, x.stride(0), x.stride(1), mb, R, V, ops._ptr(lab),
                    lab.stride(0), lab.stride(1), 1.0, ops._ptr(out[s:s + mb]), None, None, ops._stream(dev)))
        # ---- GRPO advantage over the whole batch: contiguous groups of G (the rollout layout), the
        #      pack kernel's per-row reward sums as the scores
        # ---- update: per micro-batch fused policy pass (logprob/entropy fwd + PPO/KL loss +
        #      logprob bwd -> dlogits); --unfused runs the four separate kernels instead. The step
        #      plan computes GRPO (pack's reward row sums, contiguous groups of G) into `adv` in the
        #      same launch as every micro-batch's loss scales (skyrl_policy_train_plan_grpo)
        metrics_acc.zero_()
        if args.unfused:
            adv = grpo_timer.wrap(lambda: ops.grpo_advantage(rew, rmask, None, None, ng, scores=scores))
        else:
            adv = step_adv
            plan_timer.wrap(lambda: ops._ffi.call(
                "skyrl_policy_train_plan_grpo", ops._ptr(lmask), N, R, mb, ctypes.byref(params), ops._ptr(scores),
                ops._ptr(rmask), ops.I64, GROUP, 1e-6, 1, ops._ptr(adv), ops._ptr(lrows), ops._ptr(step_ws),
                ops._stream(dev)))
        for s in range(0, N, mb):
            x = lg_rows(s, mb)
            lab = labels[s:s + mb]
            if args.unfused:
                fwd_timer.wrap(lambda: ops._ffi.call(
                    "skyrl_logprob_fwd", ops._ptr(x), ops.BF16, x.stride(0), x.stride(1), mb, R, V, ops._ptr(lab),
                    lab.stride(0), lab.stride(1), 1.0, ops._ptr(lp), ops._ptr(ent), ops._ptr(lse), ops._stream(dev)))
                lpr = lp.detach().requires_grad_(True)
                loss, m = ops.ppo_loss(lpr, old_lp[s:s + mb], adv[s:s + mb], lmask[s:s + mb], params,
                                       ref_log_probs=ref_lp[s:s + mb], entropy=ent)
                (glp,) = torch.autograd.grad(loss, lpr)
                ops._ffi.call("skyrl_logprob_bwd", ops._ptr(x), ops.BF16, x.stride(0), x.stride(1), mb, R, V,
                              ops._ptr(lab), lab.stride(0), lab.stride(1), 1.0, ops._ptr(lse), ops._ptr(ent),
                              ops._ptr(glp), None, ops._ptr(dlogits), ops._stream(dev))
                metrics_acc.add_(m)
            else:
                train_timer.wrap(lambda: ops._ffi.call(
                    "skyrl_policy_train_micro_fwd", ops._ptr(x), ops.BF16, x.stride(1), mb * R, V, ops._ptr(lab),
                    lab.stride(0), lab.stride(1), None, s // mb, N, R, mb, 1.0, ops._ptr(old_lp), ops._ptr(adv),
                    ops._ptr(lmask), ops._ptr(ref_lp), ctypes.byref(params), ops._ptr(step_lp), ops._ptr(step_ent),
                    ops._ptr(dlogits), V, ops._ptr(step_ws), ops._stream(dev)))
        if not args.unfused:
            fold_timer.wrap(lambda: ops._ffi.call("skyrl_policy_train_fold", ops._ptr(lmask), N, R, mb,
                                                  ctypes.byref(params), ops._ptr(step_loss), ops._ptr(step_met),
                                                  ops._ptr(step_ws), ops._stream(dev)))
            torch.sum(step_met, 0, out=metrics_acc)
        if dist_on:
            dist.all_reduce(metrics_acc)
        # ---- optimizer step (one mini-batch per step at 64 prompts): DP gradient reduce-scatter on
        #      the comm stream, sharded clip + AdamW (one HIP pass, bf16 copy written in the same
        #      pass), then the bf16 all-gather = learner -> rollout weight sync, left in flight
        if opt is not None:
            reducer.launch()  # the comm stream waits for the compute stream's work so far
            if inflight:  # clip/AdamW + all-gather follow the reduce-scatter on the comm stream
                reducer.stream.wait_stream(torch.cuda.current_stream(dev))  # (world 1: launch() is a no-op)
                with torch.cuda.stream(reducer.stream):
                    adam_timer.wrap(lambda: opt.step(n_micro=N // mb, zero_grad=False))
                    opt.sync_weights()
                    upd_done = torch.cuda.Event()
                    upd_done.record(reducer.stream)
            else:
                adam_timer.wrap(lambda: opt.step(n_micro=N // mb, zero_grad=False))
                opt.sync_weights()
        return metrics_acc

    for w in range(args.warmup):
        t0 = time.time()
        step(w)
        torch.cuda.synchronize()
        log(f"warmup {w}: {time.time() - t0:.3f}s")
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    for tm in timers:
        tm.active = True
    t0 = time.perf_counter()
    for k in range(args.steps):
        m = step(1000 + k)
        if k == args.steps - 1 or (k % 2 == 0):
            log(f"step {k} enqueued ({time.perf_counter() - t0:.2f}s)")
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    for tm in timers:
        tm.active = False
    mvals = m.tolist()
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = N * world * args.steps / elapsed

    # per-kernel roofline: algorithmic bytes per launch / average event-timed launch duration
    rows_per_launch = mb * R
    kernels = {}
    sampled_rows = sum(live)  # per step: the live sequences of every decode step
    for name, tm, nbytes, launches_per_step, ceiling in (
        (SAMPLER_LABEL(N, args.rollout), sample_timer, sampled_rows * (V * 2 + 16) // R, R,
         CEILING_READ_GBS),
        ("skyrl_logprob_fwd (logprob_fwd_kernel<bf16>)", fwd_timer, rows_per_launch * (V * 2 + 8 + 4),
         2 * (N // mb) + (N // mb if args.unfused else 0), CEILING_READ_GBS),
        ("skyrl_policy_train_micro_fwd (policy_train_split_kernel: each row in 6 pieces of 256 threads)", train_timer,
         rows_per_launch * (V * 4 + 8 + 20 + 8), 0 if args.unfused else N // mb, CEILING_RW_GBS),
        ("skyrl_adamw_step (sumsq + plan + adamw_update_kernel<shadow>)", adam_timer,
         (reducer.layout.shard_numel * (4 + 30)) if reducer is not None else 0, 1, CEILING_RW_GBS),
    ):
        if not tm.pairs:
            continue
        ms = tm.avg_ms()
        kernels[name] = {"avg_launch_ms": round(ms, 4), "bytes_per_launch": int(nbytes),
                         "achieved_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                         "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "ms_per_step": round(ms * launches_per_step, 2), "launches_timed": tm.launches,
                         "ceiling_GBps": ceiling}
        if launches_per_step == 1:  # one launch (block) per step: each step's time, for the spread
            kernels[name]["per_step_ms"] = [round(pr[0].elapsed_time(pr[1]), 3) for pr in tm.pairs]
    dom_name = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
    # the advantage + loss launches the product issues per step outside the fused logits pass, eager
    # and event-timed inside the timed steps (GRPOTrainer: compute_advantages_and_returns' GRPO, then
    # PolicyTrainStep's plan and fold); the per-token loss terms themselves are computed inside
    # policy_train's pass (their 40 B/token are in its bytes). Algorithmic bytes: GRPO with the pack
    # scores reads the int64 response mask and writes adv (12 B/token), the plan reads the loss mask
    # (4), the fold reads the records and the mask (20).
    product = None
    if plan_timer.pairs and fold_timer.pairs:
        us = {k: round(t.avg_ms() * 1e3, 2) for k, t in (("plan_grpo_us", plan_timer), ("fold_us", fold_timer))}
        tot = sum(us.values())
        # plan + GRPO: int64 response mask 8 read, advantages 4 written (pack's loss-mask row sums and
        # reward row sums: 8 B per row); fold: records 16 + loss mask 4 read
        nbytes = N * R * (12 + 20) + N * 8
        product = dict(us, total_us=round(tot, 2), launches_per_step=2, bytes_per_step=nbytes,
                       achieved_GBps=round(nbytes / (tot * 1e-6) / 1e9, 1),
                       frac=round(nbytes / (tot * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                       note="eager, event-timed in the timed steps: exactly the launches GRPOTrainer issues per "
                            "step for GRPO + the loss outside the fused logits pass (GRPO inside the plan launch)")
    dom = kernels[dom_name]
    result = {
        "metric": "trained samples/sec (rollout+update), Qwen2.5-1.5B GRPO at 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic",
        "config": {
            "workload": "grpo_hot_path_qwen2.5-1.5b_vocab",
            "prompts": N_GLOBAL // GROUP, "group": GROUP, "global_batch": N_GLOBAL, "seq_len": R,
            "prompt_len": P_MAX, "vocab": V, "micro_batch": mb, "parallelism": f"dp{world}",
            "rows_per_rank": N, "rank0_rows": [row0, row0 + N],
            "rollout": ({"form": "live decode batch (continuous batching: a sequence leaves after its last token)",
                         "sampled_rows_per_step": sampled_rows, "decode_steps": R, "first_live": live[0],
                         "last_live": live[-1]} if args.rollout == "live" else
                        {"form": "every sequence at every decode step", "sampled_rows_per_step": sampled_rows,
                         "decode_steps": R}),
            "work_split": ("strong: one global batch of 512 trajectories, rank r takes rows [r*512/N, (r+1)*512/N) "
                           "(whole prompt groups; dispatch.py:122-141)" if args.scaling == "strong" else
                           "weak: every rank its own 512-trajectory batch"),
            "weight_sync": ("inflight: reduce-scatter + clip/AdamW + all-gather on the comm stream under the next "
                            "step's rollout and ref pass; the old-policy pass waits for the new weights (an engine "
                            "would need double-buffered rollout weights for this overlap)"
                            if inflight else "sync: optimizer on the compute stream; the next step's rollout "
                            "waits for the weight all-gather (the reference pauses generation for the sync)"),
            "logits_resident_rows": rows, "logits_full_batch_resident": full,
            "final_loss_sum_last_step": round(mvals[0], 6),
            "policy_params": args.params, "grad_bucket_mb": args.bucket_mb,
            "optimizer": "sharded AdamW (fp32 master, bf16 rollout copy), reduce-scatter + all-gather over RCCL",
            "collectives": (dist.get_backend() + (" (one-rank group, SKYRL_FORCE_COLLECTIVES)" if world == 1 else ""))
            if dist_on else "none (world size 1)",
            "launch": ("single process" if world == 1 else
                       "bench.py --gpus N -> torch.distributed.run child, one rank per GPU"
                       if os.environ.get("SKYRL_BENCH_SPAWNED") == "1" else "external torch.distributed.run"),
        },
        "roofline": {
            "kernel": dom_name,
            "bound": "hbm",
            "achieved": dom["achieved_GBps"],
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": dom["frac"],
            "traffic": pmc_traffic(dom_name, dom["bytes_per_launch"]),
            "bytes_per_launch": dom["bytes_per_launch"],
            "avg_launch_ms": dom["avg_launch_ms"],
            "measured_ceiling_GBps": dom["ceiling_GBps"],
            "frac_of_measured_ceiling": round(dom["achieved_GBps"] / dom["ceiling_GBps"], 4),
        },
        "kernels": kernels,
        "advantage_loss": None,
        "advantage_loss_product": product,
        "cpu_baseline": None,
    }
    if emulate > 1:
        result["emulated"] = {
            "world": emulate, "rank": args.emulate_rank, "optimizer_shard_params": n_params,
            "note": "one process running one rank's share of a strong-scaling job: its rows and its 1/W "
                    "optimizer shard, no reduce-scatter / all-gather / metric all-reduce (collectives excluded)",
            "projected_value_excluding_collectives": round(N_GLOBAL * args.steps / elapsed, 3)}
    legs = rank == 0  # the single-GPU legs after the timed region: rank 0 only; the others wait at the barrier
    NL = PROMPTS * GROUP  # the legs keep the headline shape (512 trajectories) at every world size
    if legs and not args.no_adv_loss_leg:
        result["advantage_loss"] = {"batch": advantage_loss_leg(dev, NL, R, variants=args.adv_loss_variants),
                                    "batch_x16": advantage_loss_leg(dev, 16 * NL, R, reps=5)}
    if legs and not args.no_attention_leg:
        result["rollout_attention"] = rollout_attention_leg(dev, NL)
    if legs and not args.no_lmhead_leg:
        result["rollout_lmhead_sample"] = lmhead_sample_leg(dev, NL)
        result["learner_lmhead_fwd"] = learner_lmhead_fwd_leg(dev)
    if legs and not args.no_filtered_leg:
        result["sampler_filtered"] = sampler_filtered_leg(dev, NL, V)
    if legs and not args.no_vocab_legs:
        result["policy_train_vocabs"] = policy_train_vocab_legs(dev, mb, R)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)
    if rank == 0 and world == 1 and not args.no_e2e:
        del logits, dlogits, reducer, opt  # the real-model leg needs the HBM the resident logits hold
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        result["end_to_end"] = end_to_end_leg()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.barrier()  # every rank leaves together (rank 0 ran the legs)
        dist.destroy_process_group()


def end_to_end_leg(timeout_s=900):
    """The same configuration with the transformer in the loop (scripts/e2e_bench.py, a child
    process): random-init Qwen2.5-1.5B policy + ref, AMDInferenceEngine rollout of 512
    trajectories (responses U[1,1024]), HF learner fwd/bwd with the HIP logprob/loss path, AdamW,
    weight sync. Informational: the headline value above is the hot path (north star)."""
    import collections
    import subprocess
    import threading

    cmd = [sys.executable, "-u", os.path.join(ROOT, "scripts", "e2e_bench.py"), "--steps", "1", "--warmup", "1"]
    tail = collections.deque(maxlen=40)  # the child's last stderr lines, kept for the JSON on failure

    def pump(stream):  # forward the child's stderr live (progress) and remember its tail
        for ln in stream:
            sys.stderr.write(ln)
            tail.append(ln.rstrip("\n"))

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    th = threading.Thread(target=pump, args=(p.stderr,), daemon=True)
    th.start()
    try:
        out, _ = p.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        p.kill()
        p.communicate()
        th.join(5)
        return {"error": f"timeout after {timeout_s}s", "stderr_tail": list(tail)}
    th.join(5)
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit {p.returncode}", "stderr_tail": list(tail)}
    return json.loads(lines[-1])


def pmc_traffic(kernel_name, algorithmic_bytes):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json,
    FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, KB -> B), or None if not profiled."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        table = json.load(f)
    for key, rec in table.get("kernels", {}).items():
        if key in kernel_name:
            return rec.get("hbm_bytes_per_launch")
    return None


def advantage_loss_leg(dev, N, R, reps=20, variants=False):
    """GRPO advantage + fused PPO/KL loss + the loss backward on [N, R]: the SURVEY §8(d)
    "advantage+loss" kernels (12 + 20 + 24 = 56 algorithmic B/token). Launched through the C
    ABI inside a captured HIP graph and replayed, so host launch cost is excluded and
    inter-kernel gaps are included. The loss-mask row sums and the GRPO scores (per-row reward
    sums) are the pack kernel's (skyrl_pack_experience emits both with the batch).

    This leg is the standalone loss kernels (graph-replayed), not the trainer's default: GRPOTrainer
    computes the loss terms inside the fused logits pass and issues GRPO + plan + fold per step,
    timed eagerly as `advantage_loss_product`; its unfused path runs GRPO once per step and
    ops.ppo_loss per micro-batch (`loss_fwd_us` + `loss_bwd_us` here).
    `total_us` is the one-launch form (ops.grpo_ppo_loss(defer_fold=True, want_advantages=False)
    and its backward): skyrl_grpo_ppo_loss_fwd with the scores and
    SKYRL_LOSS_DEFER_FOLD (GRPO, loss and gradient in one launch that leaves per-block records;
    no advantages output, so the int64 response mask is not read: the loss mask is 0 outside the
    response) + skyrl_ppo_loss_finish (the backward: folds the records into loss/metrics,
    rescales when the upstream gradient != 1). `deferred_with_adv_out_total_us` also writes the
    advantages.
    `in_launch_fold_total_us` is the r02 form (the fold spins in the forward's last block,
    then a separate backward); `two_call_total_us` GRPO, loss, backward as three launches.
    All keep the 56 B/token figure. Returns per-kernel and total microseconds."""
    from skyrl_amd import _ffi, ppo_utils
    from skyrl_amd.config import AlgorithmConfig
    from skyrl_amd.ops import _ptr

    g = torch.Generator(device=dev).manual_seed(7)
    lens = torch.randint(1, R + 1, (N,), device=dev, generator=g)
    rew = torch.zeros(N, R, device=dev)
    rew[torch.arange(N, device=dev), lens - 1] = (torch.rand(N, device=dev, generator=g) < 0.3).float()
    rmask = (torch.arange(R, device=dev)[None] < lens[:, None]).to(torch.int64)
    lmask = rmask.float()
    rows = lens.float()  # = pack's loss_mask_row_sum for this batch
    lp = -2 + 0.1 * torch.randn(N, R, device=dev, generator=g)
    old = lp + 0.05 * torch.randn(N, R, device=dev, generator=g)
    ref = lp + 0.05 * torch.randn(N, R, device=dev, generator=g)
    adv = torch.empty(N, R, device=dev)
    glp = torch.empty(N, R, device=dev)
    loss = torch.empty(1, device=dev)
    met = torch.empty(8, device=dev)
    gout = torch.ones(1, device=dev)
    ws = torch.zeros(_ffi.query("skyrl_ppo_loss_workspace_bytes", N, R), dtype=torch.uint8, device=dev)
    params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=False)
    ng = N // GROUP
    scores = rew.sum(-1)  # = pack's reward_row_sum (one nonzero per row: any summation order is exact)

    def grpo(s, sc=None):
        _ffi.call("skyrl_grpo_advantage", _ptr(rew), _ptr(sc), _ptr(rmask), _ffi.I64, None, None, ng, N, R, 1e-6, 1,
                  _ptr(adv), None, s)

    def fwd(s, with_rows=True, flags=0):
        _ffi.call("skyrl_ppo_loss_fwd", _ptr(lp), _ptr(old), _ptr(adv), _ptr(lmask), _ptr(ref), None,
                  _ptr(rows) if with_rows else None, N, R, ctypes.byref(params), _ptr(loss), _ptr(met), _ptr(glp),
                  None, flags, _ptr(ws), s)

    def bwd(s):
        _ffi.call("skyrl_ppo_loss_bwd", _ptr(gout), N * R, _ptr(glp), None, s)

    def fused(s, sc=None, flags=0, adv_out=True):  # GRPO inside the loss launch (skyrl_grpo_ppo_loss_fwd)
        _ffi.call("skyrl_grpo_ppo_loss_fwd", _ptr(rew), _ptr(sc), _ptr(rmask) if adv_out else None, _ffi.I64, ng,
                  1e-6, 1, _ptr(lp), _ptr(old), _ptr(lmask), _ptr(ref), None, _ptr(rows), N, R,
                  ctypes.byref(params), _ptr(adv) if adv_out else None, _ptr(loss), _ptr(met), _ptr(glp), None, flags,
                  _ptr(ws), s)

    one_launch = N * ((R + 1023) // 1024) <= 2048  # skyrl_grpo_ppo_loss_fwd's one-launch layout

    def fused_deferred(s):  # the product path (GRPOTrainer._loss): pack's scores, no advantages output (the
        # trainer has them; ops passes the buffers when the layout runs two launches), fold left to the backward
        fused(s, scores, _ffi.LOSS_DEFER_FOLD, adv_out=not one_launch)

    def fused_deferred_adv(s):  # the same, writing adv * response_mask as well
        fused(s, scores, _ffi.LOSS_DEFER_FOLD)

    def finish(s):  # backward of the deferred forward: fold + rescale (nothing to rescale at g == 1)
        _ffi.call("skyrl_ppo_loss_finish", _ptr(gout), _ptr(glp), None, N, R, ctypes.byref(params), _ptr(loss),
                  _ptr(met), _ptr(ws), s)

    def timed(fns):
        side = torch.cuda.Stream(dev)
        with torch.cuda.stream(side):
            h = torch.cuda.current_stream(dev).cuda_stream
            for f in fns:
                f(h)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=side):
            h = torch.cuda.current_stream(dev).cuda_stream
            for _ in range(reps):
                for f in fns:
                    f(h)
        graph.replay()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            graph.replay()
        b.record()
        b.synchronize()
        del graph
        return round(a.elapsed_time(b) * 1e3 / (5 * reps), 2)

    out = {}
    for name, fns in (("grpo_us", (grpo,)), ("loss_fwd_us", (fwd,)), ("loss_bwd_us", (bwd,)),
                      ("grpo_loss_fused_us", (fused,)), ("two_call_total_us", (grpo, fwd, bwd)),
                      ("in_launch_fold_total_us", (fused, bwd)),
                      ("grpo_loss_deferred_us", (fused_deferred,)), ("finish_us", (finish,)),
                      ("deferred_with_adv_out_total_us", (fused_deferred_adv, finish)),
                      ("total_us", (fused_deferred, finish))):
        out[name] = timed(fns)
    if variants:
        out["variants"] = {"total_without_row_sums_us": timed((grpo, lambda s: fwd(s, False), bwd)),
                           "grpo_adv_loss_no_bwd_us": timed((grpo, fwd))}
        for sl in (1, 2, 4):
            with _ffi.variant(grpo_slices=sl):
                out["variants"][f"grpo_slices{sl}_us"] = timed((grpo,))
        for u in (1, 2, 4):
            with _ffi.variant(loss_units=u):
                out["variants"][f"loss_units{u}_us"] = timed((fwd,))
    nbytes = 56 * N * R
    gbs = nbytes / (out["total_us"] * 1e-6) / 1e9
    out.update({"rows": N, "R": R, "algorithmic_bytes": nbytes, "achieved_GBps": round(gbs, 1),
                "frac": round(gbs / HBM_PEAK_GBS, 4)})
    return out


def policy_train_vocab_legs(dev, mb, R, reps=10):
    """The fused training pass (skyrl_policy_train_fwd) at every BASELINE.json vocabulary, one
    micro-batch of mb x R tokens each: GPT-2 (50,257: odd V, so the rows of a [n, S, V] model
    output are not 16-B aligned; timed on the model-wrapper slice [:, -R-1:-1] of such a
    tensor), Llama-3 (128,256), Qwen2.5-1.5B (151,936), Qwen2.5-7B (152,064). Algorithmic bytes
    per token: V*2 read + V*2 written + 36 (label, old, adv, mask, ref, logp, entropy, record)."""
    from skyrl_amd import ops, ppo_utils
    from skyrl_amd.config import AlgorithmConfig

    params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=True)
    out = {}
    for name, V in (("gpt2", 50257), ("llama3_8b", 128256), ("qwen2.5_1.5b", 151936), ("qwen2.5_7b", 152064)):
        S = R + 2 if V % 8 else R
        full = torch.empty((mb, S, V), dtype=torch.bfloat16, device=dev).normal_(0.0, 3.0)
        x = full[:, S - R - 1:S - 1] if V % 8 else full
        g = torch.Generator(device=dev).manual_seed(3)
        labels = torch.randint(0, V, (mb, R), device=dev, generator=g)
        old = -12 + torch.randn(mb, R, device=dev, generator=g)
        adv = torch.randn(mb, R, device=dev, generator=g)
        mask = torch.ones(mb, R, device=dev)
        ref = old + 0.01
        torch.cuda.synchronize(dev)
        run = lambda: ops.policy_train(x, labels, old, adv, mask, params, ref_log_probs=ref)  # noqa: E731
        run()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            run()
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / reps
        nbytes = mb * R * (4 * V + 36)
        out[name] = {"V": V, "rows_16B_aligned": V % 8 == 0, "ms_per_microbatch": round(ms, 4),
                     "bytes": nbytes, "achieved_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                     "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        del full, x
        torch.cuda.empty_cache()
    return out


def lmhead_sample_leg(dev, nseq, reps=30):
    """One rollout decode step's logits projection + sampling at the headline shape (SURVEY
    §8(f)1 decode side): hidden [nseq, 1536] (Qwen2.5-1.5B) x lm_head [151,936, 1536] bf16.
    fused   = skyrl_lmhead_sample (MFMA GEMM with the sampler in its epilogue, one merge launch)
    unfused = library GEMM (torch/hipBLASLt) writing bf16 logits + skyrl_sample reading them.
    Random operands (logits ~ N(0, 9)). The MFMA roofline is against the 2.5 PF/s dense bf16 peak."""
    from skyrl_amd import ops

    H, V = 1536, VOCAB
    g = torch.Generator(device=dev).manual_seed(5)
    w = (torch.randn(V, H, device=dev, generator=g) * (3.0 / H ** 0.5)).to(torch.bfloat16)
    h = torch.randn(nseq, H, device=dev, generator=g).to(torch.bfloat16)
    ids = torch.arange(nseq, device=dev)
    z = torch.empty(nseq, V, dtype=torch.bfloat16, device=dev)
    tok = torch.empty(nseq, dtype=torch.int32, device=dev)
    lp = torch.empty(nseq, dtype=torch.float32, device=dev)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        return round(a.elapsed_time(b) * 1e3 / reps, 2)

    out = {"rows": nseq, "hidden": H, "vocab": V}
    for name, T in (("t1", 1.0), ("greedy", 0.0)):
        out[f"fused_{name}_us"] = timed(lambda: ops.lmhead_sample(h, w, temperature=T, seed=1, seq_ids=ids, step=3,
                                                                   tokens_out=tok, logp_out=lp))

        def unfused():
            torch.matmul(h, w.T, out=z)
            ops.sample(z, temperature=T, seed=1, seq_ids=ids, step=3, tokens_out=tok, logp_out=lp)
        out[f"unfused_{name}_us"] = timed(unfused)
    out["gemm_only_us"] = timed(lambda: ops.lmhead_gemm(h, w, out=z))
    out["library_gemm_only_us"] = timed(lambda: torch.matmul(h, w.T, out=z))
    flops = 2.0 * nseq * H * V
    tf = flops / (out["fused_t1_us"] * 1e-6) / 1e12
    out["roofline"] = {"kernel": "lmhead_gemm_kernel<sample> + merge", "bound": "mfma", "achieved": round(tf, 1),
                       "peak": 2500.0, "unit": "TFLOP/s", "frac": round(tf / 2500.0, 4)}
    out["gemm_TFs"] = round(flops / (out["gemm_only_us"] * 1e-6) / 1e12, 1)
    out["logits_bytes_not_written"] = nseq * V * 2
    return out


def learner_lmhead_fwd_leg(dev, T=8192, reps=10):
    """The learner's forward-only lm_head pass (old / ref log-probs + entropy) at
    T = 8192 tokens of Qwen2.5-1.5B (hidden 1536 x lm_head [151,936, 1536] bf16):
    fused   = skyrl_lmhead_logprob_fwd (persistent MFMA GEMM with the online softmax in its
              epilogue + the label/merge launch): no logits leave the registers;
    chunked = hipBLASLt GEMM into a reused [T, 16384] bf16 buffer + the HIP chunk merge.
    Interleaved over 3 rounds, medians. The MFMA roofline is against the 2.5 PF/s dense bf16 peak."""
    import statistics

    from skyrl_amd import lmhead, ops

    H, V = 1536, VOCAB
    g = torch.Generator(device=dev).manual_seed(6)
    w = (torch.randn(V, H, device=dev, generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16)
    h = torch.randn(T, H, device=dev, generator=g).to(torch.bfloat16)
    lab = torch.randint(0, V, (T,), device=dev, generator=g)
    fns = {"fused": lambda: ops.lmhead_logprob_fwd(h, w, lab),
           "chunked": lambda: lmhead.LMHeadLogprob.apply(h, w, lab, 1.0, True, None)}
    times = {k: [] for k in fns}
    with torch.no_grad():
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        for _ in range(3):
            for k, f in fns.items():
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(reps):
                    f()
                b.record()
                b.synchronize()
                times[k].append(a.elapsed_time(b) / reps)
    out = {"tokens": T, "hidden": H, "vocab": V}
    for k, v in times.items():
        out[f"{k}_ms"] = round(statistics.median(v), 4)
    flops = 2.0 * T * H * V
    tf = flops / (out["fused_ms"] * 1e-3) / 1e12
    out["roofline"] = {"kernel": "lmhead_logprob_pkernel + lmhead_label_merge_kernel", "bound": "mfma",
                       "achieved": round(tf, 1), "peak": 2500.0, "unit": "TFLOP/s", "frac": round(tf / 2500.0, 4)}
    out["logits_bytes_not_written"] = T * V * 2
    return out


def sampler_filtered_leg(dev, nseq, V, reps=20):
    """The §8(d) filter variant of the rollout sampler (top_k = 50 with top_p = 0.9, and top_k =
    50 alone), the SkyRL-SQL recipe's top_p = 0.95 alone at T = 1 and at its T = 0.6
    (examples/text_to_sql/run_skyrl_sql.sh:59-60), and min_p = 0.05 (skyrl-tx generator.py:423-449)
    at the decode step's shape [nseq, V] bf16: the whole skyrl_sample call (with top_k the
    one-pass kernel; without it the top_p kernel, which decides most rows in one pass and hands
    the rest to a second launch that re-reads each of them in 8 pieces; rows either kernel cannot
    take run the pre-pass + MODE 2 code in the same workgroup), against the two-kernel path
    (skyrl_variant sampler_topk_fast / sampler_topp_fast 0). "one_pass" is the fast path's whole call
    (for top_p both launches). Algorithmic bytes = one read of the logits + 16 B per row (the
    left rows' re-read, ~6 % at top_p 0.95, is meant to hit the Infinity Cache)."""
    from skyrl_amd import ops

    g = torch.Generator(device=dev).manual_seed(5)
    x = (torch.randn(nseq, V, device=dev, generator=g) * 3).to(torch.bfloat16)
    ids = torch.arange(nseq, dtype=torch.int64, device=dev)
    tok = torch.empty(nseq, dtype=torch.int32, device=dev)
    lp = torch.empty(nseq, dtype=torch.float32, device=dev)
    nbytes = nseq * V * 2 + nseq * 16
    out = {"shape": [nseq, V], "dtype": "bf16", "temperature": 1.0, "bytes_per_launch": nbytes}
    for name, k, p, t, mp in (("top_k50_top_p0.9", 50, 0.9, 1.0, 0.0), ("top_k50", 50, 1.0, 1.0, 0.0),
                              ("top_p0.95", -1, 0.95, 1.0, 0.0), ("top_p0.95_T0.6", -1, 0.95, 0.6, 0.0),
                              ("min_p0.05", -1, 1.0, 1.0, 0.05), ("min_p0.05_T0.6", -1, 1.0, 0.6, 0.05)):
        res = {}
        knob = "sampler_topk_fast" if k > 0 else "sampler_topp_fast"  # the one-pass / two-pass kernels
        for fast in (1, 0):
            vscope = ops.variant(**{knob: fast})
            vscope.__enter__()
            run = lambda: ops.sample(x, temperature=t, top_k=k, top_p=p, min_p=mp, seed=3, seq_ids=ids,  # noqa: E731
                                     step=1, tokens_out=tok, logp_out=lp)
            run()
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                run()
            b.record()
            b.synchronize()
            us = a.elapsed_time(b) * 1e3 / reps
            gbs = nbytes / (us * 1e-6) / 1e9
            vscope.__exit__(None, None, None)
            res["one_pass" if fast else "two_kernel"] = {"avg_launch_us": round(us, 2), "achieved_GBps": round(gbs, 1),
                                                         "frac": round(gbs / HBM_PEAK_GBS, 4)}
        out[name] = res
    return out


def rollout_attention_leg(dev, nseq, reps=20):
    """Rollout decode attention (csrc/attention.hip paged_decode_kernel) at the
    headline shape: Qwen2.5-1.5B heads (12 q / 2 kv, D=128), one decode step of all nseq
    trajectories with ragged contexts U[17, 1536] (prompt U[16,512] + responses up to 1024).
    Algorithmic bytes = K+V of every live context token (nkv*D*2 B each, x2) + q + out, i.e.
    1024 B/token; timed per launch with HIP events on the stream the kernel runs on."""
    import math

    from skyrl_amd.inference_engines import kernels

    nh, nkv, D, BS = 12, 2, 128, 16
    g = torch.Generator(device=dev).manual_seed(11)
    ctx = torch.randint(17, 1537, (nseq,), device=dev, generator=g, dtype=torch.int32)
    nb = (ctx + BS - 1) // BS
    max_ctx = int(ctx.max())
    width = (max_ctx + BS - 1) // BS
    nblk = int(nb.sum())
    kc = torch.randn(nblk, nkv, BS, D, device=dev, generator=g).to(torch.bfloat16)
    vc = torch.randn(nblk, nkv, D, BS, device=dev, generator=g).to(torch.bfloat16)
    perm = torch.randperm(nblk, device=dev, generator=g).int()  # scattered blocks, as after churn
    bt = torch.zeros(nseq, width, dtype=torch.int32, device=dev)
    starts = torch.cumsum(nb, 0) - nb
    col = torch.arange(width, device=dev)
    live = col[None] < nb[:, None]
    bt[live] = perm[(starts[:, None] + col[None])[live]]
    q = torch.randn(nseq, nh, D, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty_like(q)
    ws = kernels.DecodeWorkspace(dev)
    nparts = kernels.choose_nparts(nseq, nkv, max_ctx)
    run = lambda: kernels.paged_decode(q, kc, vc, bt, ctx, max_ctx, 1 / math.sqrt(D), out=out,  # noqa: E731
                                       workspace=ws, nparts=nparts)
    run()
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        run()
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    tokens = int(ctx.sum())
    nbytes = tokens * nkv * D * 2 * 2 + 2 * nseq * nh * D * 2
    gbs = nbytes / (us * 1e-6) / 1e9
    return {"kernel": "paged_decode_kernel<128> (+ reduce)", "seqs": nseq, "context_tokens": tokens,
            "context_len": "U[17,1536]", "heads": f"{nh}q/{nkv}kv x {D}", "nparts": nparts,
            "avg_launch_us": round(us, 2), "bytes_per_launch": nbytes, "achieved_GBps": round(gbs, 1),
            "peak_GBps": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4),
            "frac_of_measured_read_ceiling": round(gbs / CEILING_READ_GBS, 4),
            "traffic": pmc_traffic("paged_decode_kernel", nbytes)}


def cpu_baseline(args):
    """The oracle (CPU restatement, 'port') on a bounded sample of the same workload.

    Sample: 2 trajectories' per-token work (R decode steps of the C sampler oracle over V, two
    no-grad logprob passes and one logprob fwd+bwd pass over R x V fp32 on torch-CPU) plus the
    batch-level work (GRPO, loss fwd/bwd, pack) on the full 512 x 1024 batch divided by 512.
    """
    import numpy as np

    from oracle import cpu_ref

    # the GPU box's CPU share is 16 threads (OMP_NUM_THREADS there); affinity shows the whole host
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    cores = min(cores, args.cpu_threads) if args.cpu_threads > 0 else cores
    torch.set_num_threads(cores)
    R, V, N = R_MAX, VOCAB, PROMPTS * GROUP
    n_traj = 2
    g = torch.Generator().manual_seed(0)
    logits = (torch.randn(n_traj, R, V, generator=g) * 3).to(torch.bfloat16)
    labels = torch.randint(0, V, (n_traj, R), generator=g)
    from oracle import sampler as osamp

    ids = torch.arange(n_traj, dtype=torch.int64)
    steps = args.cpu_sampler_steps
    t0 = time.perf_counter()
    for t in range(steps):  # one decode step = n_traj rows of V
        osamp.sample(logits[:, t].contiguous(), 1.0, -1, 1.0, 0.0, 0, ids, t)
    t_sample = (time.perf_counter() - t0) * (R / steps)
    tok_sample = args.cpu_logprob_tokens
    x = logits.reshape(-1, V)[:tok_sample]
    lab = labels.reshape(-1)[:tok_sample]
    t0 = time.perf_counter()
    for _ in range(2):
        cpu_ref.logprobs_from_logits(x, lab)
    xg = x.float().requires_grad_(True)
    lp = cpu_ref.logprobs_from_logits(xg, lab)
    ent = cpu_ref.entropy_from_logits(xg)
    (lp.sum() + ent.sum()).backward()
    t_lp = (time.perf_counter() - t0) * (n_traj * R / tok_sample)
    # batch-level ops on the full batch
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None] < lens[:, None]).float()
    rew = torch.zeros(N, R)
    rew[torch.arange(N), lens - 1] = (torch.rand(N, generator=g) < 0.3).float()
    uids = [str(i // GROUP) for i in range(N)]
    lpb = -2 + 0.1 * torch.randn(N, R, generator=g)
    t0 = time.perf_counter()
    adv = cpu_ref.grpo_advantage(rew, mask, uids)
    xb = lpb.clone().requires_grad_(True)
    loss, _ = cpu_ref.policy_loss_assembly(xb, lpb + 0.01, adv, mask, lpb - 0.01, torch.rand(N, R))
    loss.backward()
    prompts = [list(range(int(k))) for k in torch.randint(16, P_MAX + 1, (N,), generator=g)]
    responses = [list(range(int(k))) for k in lens]
    cpu_ref.pack(prompts, responses, [[0.0] * len(r) for r in responses], [[1.0] * len(r) for r in responses],
                 None, 0)
    t_batch = time.perf_counter() - t0
    per_traj = (t_sample + t_lp) / n_traj + t_batch / N
    return {
        "value": round(1.0 / per_traj, 4),
        "unit": "samples/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"{n_traj} trajectories x R={R}: sampler_ref.c over V={V} for {steps} decode steps "
                   f"(extrapolated to {R}), torch-CPU fp32 logprob x2 + logprob/entropy fwd+bwd on {tok_sample} "
                   f"tokens (extrapolated to {n_traj * R}); GRPO + fused-loss fwd/bwd + pack on the full "
                   f"{N}x{R} batch / {N}"),
        "seconds": round(t_sample + t_lp + t_batch, 2),
    }


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv) -> int:
    """`--gpus N` (N > 1) from a plain `python bench.py`: start N ranks, one per GPU, under
    torch.distributed.run (127.0.0.1 rendezvous) as a CHILD process and return its exit code.
    Called before anything touches the GPU; the parent never initialises HIP (no exec either).
    The reference starts one NCCL rank per GPU the same way (workers/worker.py:102-126)."""
    import subprocess

    if not args.dry_run and args.backend == "nccl":  # (gloo rehearsals share one GPU)
        n_dev = torch.cuda.device_count()  # does not initialise the GPU on this image
        if n_dev < args.gpus:
            log(f"--gpus {args.gpus} but only {n_dev} visible GPUs")
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC (the host driver's only mode)
    env.setdefault("OMP_NUM_THREADS", "1")
    env["SKYRL_BENCH_SPAWNED"] = "1"
    log(f"launching {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def dry_run(args) -> None:
    """--dry-run: report this process's rank layout and exercise the rendezvous (a gloo
    all-reduce of the ranks) without any GPU work; one JSON line per rank."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rank_sum = rank
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([rank], dtype=torch.int64)
        dist.all_reduce(t)
        rank_sum = int(t.item())
        world = dist.get_world_size()
        dist.destroy_process_group()
    if args.scaling == "strong":
        n_global = PROMPTS * GROUP
        row0, rows = rank_rows(n_global, world, rank)
    else:
        n_global, row0, rows = PROMPTS * GROUP * world, rank * PROMPTS * GROUP, PROMPTS * GROUP
    print(json.dumps({"dry_run": True, "rank": rank, "world_size": world, "local_rank": local, "gpus": args.gpus,
                      "master_addr": os.environ.get("MASTER_ADDR"), "rank_sum": rank_sum,
                      "collectives": "nccl" if world > 1 else "none (world size 1)", "scaling": args.scaling,
                      "global_batch": n_global, "rows": [row0, row0 + rows],
                      "prompt_groups": [row0 // GROUP, (row0 + rows) // GROUP]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU, RCCL); from a plain `python bench.py` N > 1 starts them itself")
    ap.add_argument("--dry-run", action="store_true", help="print the rank layout and stop before any GPU work")
    ap.add_argument("--backend", default="nccl", help="nccl (RCCL); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: one 512-trajectory batch split over the ranks (SURVEY 8(e)); weak: 512 per rank")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="(one process) run one rank's share of a W-rank strong-scaling job, collectives excluded")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--weight-sync", choices=("auto", "sync", "inflight"), default="auto",
                    help="auto = sync: the next rollout waits for the new weights; inflight: the update "
                         "overlaps the next rollout (needs double-buffered engine weights)")
    ap.add_argument("--rollout", choices=("live", "all"), default="all",
                    help="live: each decode step samples the sequences still generating (continuous batching); "
                         "all (default, the r01-r05 workload): every sequence at every one of the R steps")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--micro-batch", type=int, default=16)
    ap.add_argument("--logits-rows", type=int, default=0, help="0 = the whole batch if HBM allows")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the real-model end-to-end leg (N=1 only)")
    ap.add_argument("--no-adv-loss-leg", action="store_true", help="skip the graph-replayed advantage+loss leg")
    ap.add_argument("--adv-loss-variants", action="store_true", help="also time the A/B variants of that leg")
    ap.add_argument("--no-attention-leg", action="store_true", help="skip the rollout paged-attention leg")
    ap.add_argument("--no-lmhead-leg", action="store_true", help="skip the decode lm_head + sampler leg")
    ap.add_argument("--no-vocab-legs", action="store_true", help="skip the per-vocabulary fused training pass legs")
    ap.add_argument("--no-filtered-leg", action="store_true", help="skip the top_k / top_p sampler leg")
    ap.add_argument("--unfused", action="store_true", help="separate logprob/loss kernels instead of the fused pass")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--params", type=int, default=QWEN_1_5B_PARAMS, help="policy parameter count (0: no optimizer leg)")
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--cpu-sampler-steps", type=int, default=64)
    ap.add_argument("--cpu-logprob-tokens", type=int, default=256)
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, sys.argv[1:]))
    if args.dry_run:
        dry_run(args)
        return
    run(args)


if __name__ == "__main__":
    main()
