"""Fully-async staleness control (fully_async_trainer.py:79-190) on CPU.

capacity = min(max_concurrent - running, (max_staleness + current_step) * mini_batch -
(accepted + running)); acquire blocks at capacity 0 and wakes on accept / version change.
"""

import asyncio

from skyrl_amd.fully_async import AsyncStalenessManager


def test_capacity_formula():
    m = AsyncStalenessManager(max_concurrent_generation_groups=5, mini_batch_size=4, max_staleness_steps=2)
    assert m.capacity() == 5  # concurrency-bound: (2 + 1) * 4 = 12 > 5
    m.stat.running, m.stat.accepted = 3, 8
    assert m.capacity() == min(5 - 3, 12 - 11) == 1
    m.current_global_step = 2
    assert m.capacity() == 2


def test_acquire_blocks_until_capacity_returns():
    async def main():
        m = AsyncStalenessManager(max_concurrent_generation_groups=10, mini_batch_size=2, max_staleness_steps=0)
        # staleness 0: only the groups of the version being trained may be in flight (2)
        await m.acquire_submission_slot()
        await m.acquire_submission_slot()
        third = asyncio.create_task(m.acquire_submission_slot())
        await asyncio.sleep(0.01)
        assert not third.done()
        await m.on_rollout_accepted()
        await m.on_rollout_accepted()
        await asyncio.sleep(0.01)
        assert not third.done()  # accepted groups still count until the version moves on
        await m.notify_capacity_change(2)
        await asyncio.wait_for(third, 1.0)
        assert (m.stat.submitted, m.stat.accepted, m.stat.running) == (3, 2, 1)
        await m.on_rollout_rejected()
        assert m.stat.running == 0

    asyncio.run(main())
