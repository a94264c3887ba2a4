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
