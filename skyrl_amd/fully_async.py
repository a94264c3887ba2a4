"""Fully-async GRPO: generation runs ahead of training under a staleness budget, and weights
are swapped into the engine in flight (pause -> update -> resume).

Restates skyrl_train/fully_async_trainer.py:
  * _AsyncStalenessManager (:79-190): never have more trajectory groups accepted-or-running than
    the trainer will consume within `max_staleness_steps` steps of the version being trained,
    nor more than `max_concurrent_generation_groups` running:
        capacity = min(max_concurrent - running,
                       (max_staleness_steps + current_step) * mini_batch - (accepted + running));
  * the loop (:300-460): generation workers acquire a slot, generate one group (single-prompt
    client calls, so an abort during pause is retried with the tokens so far), and queue it; the
    trainer takes `mini_batch` groups per step, trains, then pauses generation, updates the
    engine's weights, resumes it, and raises the version (notify_capacity_change).
Each group records the policy version it was generated under; the step metrics report the
staleness (trained version - generated version) of what was consumed.
"""

from __future__ import annotations

import asyncio
from dataclasses import dataclass
from typing import Any, Dict, Iterator, List, Optional

from .trainer import GRPOTrainer


@dataclass
class RolloutStat:
    submitted: int = 0
    accepted: int = 0
    running: int = 0


class AsyncStalenessManager:
    def __init__(self, max_concurrent_generation_groups: int, mini_batch_size: int, max_staleness_steps: int):
        self.max_concurrent_generation_groups = max_concurrent_generation_groups
        self.mini_batch_size = mini_batch_size
        self.max_staleness_steps = max_staleness_steps
        self.stat = RolloutStat()
        self._cond = asyncio.Condition()
        self.current_global_step = 1  # the version being trained

    def capacity(self) -> int:
        consumer = (self.max_staleness_steps + self.current_global_step) * self.mini_batch_size
        staleness_cap = consumer - (self.stat.accepted + self.stat.running)
        concurrency_cap = self.max_concurrent_generation_groups - self.stat.running
        return min(concurrency_cap, staleness_cap)

    async def acquire_submission_slot(self) -> None:
        async with self._cond:
            while self.capacity() <= 0:
                await self._cond.wait()
            self.stat.submitted += 1
            self.stat.running += 1

    async def on_rollout_accepted(self) -> None:
        async with self._cond:
            self.stat.accepted += 1
            self.stat.running -= 1
            self._cond.notify_all()

    async def on_rollout_rejected(self) -> None:
        async with self._cond:
            self.stat.running -= 1
            self._cond.notify_all()

    async def notify_capacity_change(self, new_global_step: int) -> None:
        async with self._cond:
            self.current_global_step = int(new_global_step)
            self._cond.notify_all()


class FullyAsyncGRPOTrainer:
    """Drives a GRPOTrainer (policy, optimizer, pack/logprob/advantage/loss path) with
    asynchronous generation through an InferenceEngineClient (pause/resume support)."""

    def __init__(self, trainer: GRPOTrainer, client, mini_batch_groups: int, max_staleness_steps: int = 4,
                 max_concurrent_generation_groups: Optional[int] = None, num_generation_workers: int = 4):
        self.trainer = trainer
        self.client = client
        self.mini_batch_groups = mini_batch_groups
        self.num_workers = num_generation_workers
        self.staleness = AsyncStalenessManager(
            max_concurrent_generation_groups or mini_batch_groups * (max_staleness_steps // 2 + 1),
            mini_batch_groups, max_staleness_steps)

    async def _generate_group(self, prompt: List[int]) -> Dict[str, Any]:
        cfg = self.trainer.cfg
        sp = dict(cfg.sampling_params)
        sp.setdefault("logprobs", 0)
        sp.setdefault("temperature", cfg.temperature)
        outs = await asyncio.gather(*[self.client.generate({"prompt_token_ids": [prompt], "sampling_params": sp})
                                      for _ in range(cfg.n_samples_per_prompt)])
        return {"prompt": prompt, "response_ids": [o["response_ids"][0] for o in outs],
                "stop_reasons": [o["stop_reasons"][0] for o in outs],
                "rollout_logprobs": [(o["response_logprobs"] or [[]])[0] for o in outs]}

    async def _worker(self, prompts: Iterator[Any], queue: asyncio.Queue):
        while True:
            await self.staleness.acquire_submission_slot()
            try:
                prompt, extra = next(prompts)
            except StopIteration:
                await self.staleness.on_rollout_rejected()
                return
            version = self.staleness.current_global_step
            group = await self._generate_group(prompt)
            group.update(extra=extra, version=version)
            await self.staleness.on_rollout_accepted()
            await queue.put(group)

    async def train(self, prompts: Iterator[Any], num_steps: int) -> List[Dict[str, float]]:
        """prompts yields (prompt_token_ids, extra); returns the metrics of every step."""
        tr = self.trainer
        queue: asyncio.Queue = asyncio.Queue()
        workers = [asyncio.create_task(self._worker(prompts, queue)) for _ in range(self.num_workers)]
        history = []
        try:
            for step in range(1, num_steps + 1):
                groups = [await queue.get() for _ in range(self.mini_batch_groups)]
                gen = {"prompt_token_ids": [], "response_ids": [], "stop_reasons": [], "rollout_logprobs": [],
                       "loss_masks": [], "rewards": []}
                for g in groups:
                    for r, s, lp in zip(g["response_ids"], g["stop_reasons"], g["rollout_logprobs"]):
                        gen["prompt_token_ids"].append(g["prompt"])
                        gen["response_ids"].append(r)
                        gen["stop_reasons"].append(s)
                        gen["rollout_logprobs"].append(lp)
                        gen["loss_masks"].append([1] * len(r))
                        gen["rewards"].append(float(tr.reward_fn(g["prompt"], r, g["extra"])))
                tr.timings = {}
                import time

                import torch

                torch.cuda.synchronize()
                tr._t = time.perf_counter()
                metrics = tr.train_on(gen)
                stale = [step - g["version"] for g in groups]
                metrics.update({"async/staleness_max": max(stale), "async/staleness_mean": sum(stale) / len(stale),
                                "async/submitted": self.staleness.stat.submitted})
                # in-flight weight update (fully_async_trainer.py:415-419)
                await self.client.pause_generation()
                await self.client.update_named_weights(tr.weight_update_request())
                await self.client.resume_generation()
                await self.staleness.notify_capacity_change(step + 1)
                history.append(metrics)
        finally:
            for w in workers:
                w.cancel()
            await asyncio.gather(*workers, return_exceptions=True)
            if self.client.generation_paused_event.is_set():
                await self.client.resume_generation()
            await self.client._run_on_all_engines("abort_generation")  # drop generation still in flight
            for _ in range(3):
                await asyncio.sleep(0)
        return history
