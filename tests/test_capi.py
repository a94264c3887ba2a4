"""The C-ABI library loads and exports exactly what include/skyrl_hip.h declares (no GPU needed)."""

import ctypes
import os
import re

import pytest

from skyrl_amd import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "skyrl_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(skyrl_\w+)\s*\(", src, flags=re.M)))


def test_header_parsed():
    names = header_functions()
    assert "skyrl_grpo_advantage" in names and "skyrl_logprob_fwd" in names and len(names) >= 18


def test_library_exports_every_declared_symbol():
    lib = _ffi.load()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, f"declared in skyrl_hip.h but not exported: {missing}"


def test_ffi_signatures_cover_header():
    assert sorted(_ffi.SIGNATURES) == header_functions()


def test_abi_version_and_error_path():
    lib = _ffi.load()
    assert lib.skyrl_abi_version() == 12
    # argument validation happens on the host before any launch: no GPU needed
    with pytest.raises(_ffi.SkyrlHipError, match="temperature"):
        _ffi.call("skyrl_logprob_fwd", ctypes.c_void_p(16), _ffi.BF16, 8, 8, 1, 1, 8, ctypes.c_void_p(16), 1, 1,
                  -1.0, ctypes.c_void_p(16), None, None, None)
    assert "temperature" in lib.skyrl_last_error().decode()


def test_workspace_queries():
    assert _ffi.query("skyrl_ppo_loss_workspace_bytes", 512, 1024) >= 512 * 5 * 4
    assert _ffi.query("skyrl_sample_workspace_bytes", 512, 151936) > 0
    assert _ffi.query("skyrl_gae_workspace_bytes", 512) >= 512 * 24


def test_workspace_queries_degenerate_sizes():
    """Host-only size queries must not trap (e.g. divide by zero) on empty batches."""
    for name, args in (("skyrl_sample_workspace_bytes", (0, 7)), ("skyrl_sample_workspace_bytes", (1, 1)),
                       ("skyrl_gae_workspace_bytes", (0,)), ("skyrl_ppo_loss_workspace_bytes", (0, 0)),
                       ("skyrl_reward_kl_workspace_bytes", (0,)), ("skyrl_critic_loss_workspace_bytes", (0, 0)),
                       ("skyrl_policy_train_workspace_bytes", (0, 0)), ("skyrl_sumsq_workspace_bytes", (0,))):
        assert _ffi.query(name, *args) > 0, name


def test_oracle_sampler_builds():
    path = os.path.join(ROOT, "oracle", "_build", "libsampler_ref.so")
    assert os.path.exists(path), "oracle C restatement not built (make -C oracle)"
    ctypes.CDLL(path).sampler_ref


def test_cpu_tensor_is_rejected_not_computed():
    import torch

    from skyrl_amd import ops

    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.approx_kl(torch.zeros(4), torch.zeros(4))


def test_grpo_ppo_loss_entry_validates_on_host():
    """skyrl_grpo_ppo_loss_fwd checks its layout before any launch: no GPU needed."""
    params = _ffi.PPOParams(0.2, 0.2, 3.0, 0, 0, 0.0, 1, 3, 0.001, 0, 0.0, 0)
    p = ctypes.c_void_p(16)
    args = lambda ng, mdt: (p, None, p, mdt, ng, 1e-6, 1, p, p, p, p, None, p, 512, 1024,  # noqa: E731
                            ctypes.byref(params), p, p, p, p, None, 0, p, None)
    with pytest.raises(_ffi.SkyrlHipError, match="n % num_groups"):
        _ffi.call("skyrl_grpo_ppo_loss_fwd", *args(7, _ffi.I64))
    with pytest.raises(_ffi.SkyrlHipError, match="mask dtype"):
        _ffi.call("skyrl_grpo_ppo_loss_fwd", *args(64, 99))
    with pytest.raises(_ffi.SkyrlHipError, match="params is null"):
        a = list(args(64, _ffi.I64))
        a[15] = None
        _ffi.call("skyrl_grpo_ppo_loss_fwd", *a)
    with pytest.raises(_ffi.SkyrlHipError, match="unknown flags"):
        a = list(args(64, _ffi.I64))
        a[21] = 6
        _ffi.call("skyrl_grpo_ppo_loss_fwd", *a)
    with pytest.raises(_ffi.SkyrlHipError, match="null pointer"):
        a = list(args(64, _ffi.I64))
        a[0] = None  # neither rewards nor scores
        _ffi.call("skyrl_grpo_ppo_loss_fwd", *a)


def test_ppo_loss_finish_validates_on_host():
    params = _ffi.PPOParams(0.2, 0.2, 3.0, 0, 0, 0.0, 1, 3, 0.001, 0, 0.0, 0)
    p = ctypes.c_void_p(16)
    with pytest.raises(_ffi.SkyrlHipError, match="ppo_loss_finish: null pointer"):
        _ffi.call("skyrl_ppo_loss_finish", None, None, None, 4, 4, ctypes.byref(params), p, p, None, None)
    with pytest.raises(_ffi.SkyrlHipError, match="grad_out needs grad_logp"):
        _ffi.call("skyrl_ppo_loss_finish", p, None, None, 4, 4, ctypes.byref(params), p, p, p, None)
    with pytest.raises(_ffi.SkyrlHipError, match="bad sizes"):
        _ffi.call("skyrl_ppo_loss_finish", None, None, None, 0, 4, ctypes.byref(params), p, p, p, None)


def test_comm_abi_host_checks():
    """The RCCL entry points validate on the host (no GPU, no RCCL call)."""
    assert _ffi.query("skyrl_comm_unique_id_bytes") == 128  # sizeof(ncclUniqueId)
    with pytest.raises(_ffi.SkyrlHipError, match="null pointer"):
        _ffi.call("skyrl_comm_init", None, 1, 0, ctypes.byref(ctypes.c_void_p()))
    with pytest.raises(_ffi.SkyrlHipError, match="rank must be"):
        _ffi.call("skyrl_comm_init", ctypes.c_void_p(16), 2, 2, ctypes.byref(ctypes.c_void_p()))
    with pytest.raises(_ffi.SkyrlHipError, match="null communicator"):
        _ffi.call("skyrl_comm_allreduce", ctypes.c_void_p(16), ctypes.c_void_p(16), 4, _ffi.F32, 0, None, None)
    with pytest.raises(_ffi.SkyrlHipError, match="dtype"):
        _ffi.call("skyrl_comm_broadcast", ctypes.c_void_p(16), ctypes.c_void_p(16), 4, 9, 0, ctypes.c_void_p(16), None)
    assert _ffi.call("skyrl_comm_destroy", None) == 0


def _exported_symbols():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _ffi.LIB_PATH], stdout=subprocess.PIPE, text=True, check=True)
    return sorted({ln.split()[-1] for ln in out.stdout.splitlines() if " T " in ln and ln.split()[-1].startswith("skyrl_")})


def test_no_process_state_setters_exported():
    """reentrant entry points, no global mutable state. The A/B
    knobs are a caller-owned skyrl_variant passed to one *_ex call; nothing exported stores state:
    no skyrl_tune, no test hook, and every exported C symbol is an entry point of skyrl_hip.h."""
    syms = _exported_symbols()
    assert syms == header_functions(), set(syms) ^ set(header_functions())
    assert not [s for s in syms if "tune" in s or "occupy" in s or s.startswith("skyrl_set")]
    assert all(n + "_ex" in syms for n in _ffi.EX_FORMS)


def test_variant_applies_to_its_call_only():
    """A variant changes the decision of the call it is passed to and of no other call: the
    fused-pass support query (host-only, no GPU) with the 4 x 256 split shape at V = 200,000 says
    no; the plain call before and after, and an _ex call with NULL or an all-default variant, say
    yes. A bad field fails that call alone."""
    lib = _ffi.load()
    V = 200_000
    v = _ffi.Variant(train_split_shape=2)
    d = _ffi.Variant()
    lib.skyrl_variant_init(ctypes.byref(d))
    assert all(getattr(d, f) == _ffi.VARIANT_DEFAULT for f in _ffi.VARIANT_FIELDS)
    assert lib.skyrl_policy_train_supports(V, 1, 1.0) == 1
    assert lib.skyrl_policy_train_supports_ex(V, 1, 1.0, ctypes.byref(v)) == 0
    assert lib.skyrl_policy_train_supports(V, 1, 1.0) == 1
    assert lib.skyrl_policy_train_supports_ex(V, 1, 1.0, None) == 1
    assert lib.skyrl_policy_train_supports_ex(V, 1, 1.0, ctypes.byref(d)) == 1
    bad = _ffi.Variant(sampler_split_nt=300)
    assert lib.skyrl_policy_train_supports_ex(V, 1, 1.0, ctypes.byref(bad)) == -1
    with pytest.raises(_ffi.SkyrlHipError, match="bad value for sampler_split_nt"):
        _ffi.call("skyrl_sample_ex", ctypes.c_void_p(16), _ffi.BF16, 8, 1, 8, 1.0, -1, 1.0, 0.0, 0, None, 0,
                  ctypes.c_void_p(16), None, ctypes.c_void_p(16), None, ctypes.byref(bad))
    # the host-side scope: nested scopes override fields, leaving restores the enclosing one
    with _ffi.variant(train_split_shape=2):
        assert _ffi.query("skyrl_policy_train_supports", V, 1, 1.0) == 0
        with _ffi.variant(train_split_shape=5):
            assert _ffi.query("skyrl_policy_train_supports", V, 1, 1.0) == 1
        assert _ffi.query("skyrl_policy_train_supports", V, 1, 1.0) == 0
    assert _ffi.query("skyrl_policy_train_supports", V, 1, 1.0) == 1 and _ffi.current_variant() is None
