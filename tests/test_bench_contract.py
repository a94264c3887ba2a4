"""bench.py's output contract, checked on CPU against the committed r01 bench line
(profiles/r01_bench.json, written by `python bench.py` on the MI355X) and bench.py's own
helpers: the driver and the judge read exactly these keys."""

import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line():
    with open(os.path.join(ROOT, "profiles", "r01_bench.json")) as f:
        return json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])


def test_bench_line_has_the_contract_keys():
    d = _line()
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["data"] == "synthetic" and "workload" in d["config"]
    # value = trajectories * steps / elapsed: consistent with ms_per_step at N = 1
    assert abs(d["value"] - d["config"]["global_batch"] / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-3
    r = d["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert abs(r["achieved"] - r["bytes_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e9) / r["achieved"] < 1e-2
    # PMC traffic within 5 % of the algorithmic bytes: no wasted re-reads in the dominant kernel
    assert r["traffic"] is not None and abs(r["traffic"] / r["bytes_per_launch"] - 1) < 0.05
    c = d["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0 and c["sample"]


def test_pmc_traffic_lookup_matches_committed_profile():
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        table = json.load(f)["kernels"]
    assert bench.pmc_traffic("skyrl_policy_train_fwd (policy_train_split_kernel: 6 pieces)", 0) == \
        table["policy_train_split_kernel"]["hbm_bytes_per_launch"]
    assert bench.pmc_traffic("paged_decode_kernel", 0) == table["paged_decode_kernel"]["hbm_bytes_per_launch"]
    assert bench.pmc_traffic("no_such_kernel", 0) is None


def _dry(gpus):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    import re  # ranks share stdout (gloo prints without newlines): pick the records out by pattern

    return [json.loads(m) for m in re.findall(r'\{"dry_run"[^{}]*\}', p.stdout)]


def test_gpus_2_spawns_two_ranks():
    """`python bench.py --gpus 2` (no launcher env) starts two ranks under torch.distributed.run
    with WORLD_SIZE=2 and a working 127.0.0.1 rendezvous; --dry-run stops before GPU work. The
    ranks split ONE 512-trajectory batch by whole prompt groups (SURVEY §8(e), strong scaling)."""
    recs = sorted(_dry(2), key=lambda r: r["rank"])
    assert [r["rank"] for r in recs] == [0, 1]
    assert {r["world_size"] for r in recs} == {2} and {r["local_rank"] for r in recs} == {0, 1}
    assert {r["rank_sum"] for r in recs} == {1}  # the gloo all-reduce across both ranks ran
    assert {r["master_addr"] for r in recs} == {"127.0.0.1"} and {r["collectives"] for r in recs} == {"nccl"}
    assert [r["rows"] for r in recs] == [[0, 256], [256, 512]]
    assert [r["prompt_groups"] for r in recs] == [[0, 32], [32, 64]]
    assert {r["global_batch"] for r in recs} == {512} and {r["scaling"] for r in recs} == {"strong"}


def test_gpus_4_row_ranges():
    recs = sorted(_dry(4), key=lambda r: r["rank"])
    assert [r["rows"] for r in recs] == [[0, 128], [128, 256], [256, 384], [384, 512]]


def test_gpus_1_stays_in_process():
    recs = _dry(1)
    assert recs == [{"dry_run": True, "rank": 0, "world_size": 1, "local_rank": 0, "gpus": 1, "master_addr": None,
                     "rank_sum": 0, "collectives": "none (world size 1)", "scaling": "strong", "global_batch": 512,
                     "rows": [0, 512], "prompt_groups": [0, 64]}]


def test_rank_rows_partition_the_global_batch():
    """The 8 ranks' inputs are the N = 1 batch cut into contiguous whole-group chunks
    (dispatch.py:122-141): concatenated, they are the global batch element for element."""
    import torch

    full, uids = bench.synth_inputs("cpu", 512)
    for world in (2, 4, 8):
        parts = [bench.synth_inputs("cpu", 512, row0=r * 512 // world, rows=512 // world) for r in range(world)]
        assert [u for _, us in parts for u in us] == uids
        for k in ("plens", "rlens", "ptok", "rtok", "rew", "lmask", "rlp"):
            assert torch.equal(torch.cat([p[k] for p, _ in parts]), full[k]), (world, k)
        for p, _ in parts:
            assert int(p["poff"][0]) == 0 and int(p["roff"][-1]) == len(p["rtok"])
            assert int(p["poff"][-1]) == len(p["ptok"])
        assert [bench.rank_rows(512, world, r) for r in range(world)] == [(r * 512 // world, 512 // world)
                                                                           for r in range(world)]
    import pytest

    with pytest.raises(ValueError):
        bench.rank_rows(512, 128, 0)  # 4 rows per rank would cut prompt groups of 8
