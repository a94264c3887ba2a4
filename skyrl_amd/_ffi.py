"""ctypes binding of ``libskyrl_hip.so`` (the C ABI declared in ``include/skyrl_hip.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C skyrl_amd/csrc``).
There is no fallback: if the library is missing, or no GPU is visible, every op raises.

torch is imported first on purpose: torch ships its own ``libamdhip64.so.7``; loading it
before the extension makes the dynamic linker bind our NEEDED ``libamdhip64.so.7`` to the
same HIP runtime instance, so torch's device pointers and ``hipStream_t`` handles are valid
inside our kernels.
"""

from __future__ import annotations

import contextlib
import contextvars
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libskyrl_hip.so")

F32, BF16, I64, I32, U8 = 0, 1, 2, 3, 4
M_FINAL_LOSS, M_POLICY_LOSS, M_ENTROPY, M_KL, M_CLIP_RATIO, M_MASK_SUM = 0, 1, 2, 3, 4, 5
M_COUNT = 8
LOSS_DEFER_FOLD = 1  # SKYRL_LOSS_DEFER_FOLD


class SkyrlHipError(RuntimeError):
    """A C-ABI entry point returned a non-zero status."""


class PPOParams(ctypes.Structure):
    """Mirror of ``skyrl_ppo_params`` (include/skyrl_hip.h)."""

    _fields_ = [
        ("eps_clip_low", ctypes.c_float),
        ("eps_clip_high", ctypes.c_float),
        ("clip_ratio_c", ctypes.c_float),
        ("dual_clip", ctypes.c_int32),
        ("loss_reduction", ctypes.c_int32),
        ("max_seq_len", ctypes.c_float),
        ("use_kl_loss", ctypes.c_int32),
        ("kl_type", ctypes.c_int32),
        ("kl_loss_coef", ctypes.c_float),
        ("use_entropy_loss", ctypes.c_int32),
        ("entropy_loss_coef", ctypes.c_float),
        ("has_entropy", ctypes.c_int32),
    ]


class AdamWParams(ctypes.Structure):
    """Mirror of ``skyrl_adamw_params`` (include/skyrl_hip.h)."""

    _fields_ = [
        ("lr", ctypes.c_float),
        ("beta1", ctypes.c_float),
        ("beta2", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("weight_decay", ctypes.c_float),
        ("max_grad_norm", ctypes.c_float),
        ("grad_scale", ctypes.c_float),
    ]


class PackInputs(ctypes.Structure):
    """Mirror of ``skyrl_pack_inputs`` (include/skyrl_hip.h)."""

    _fields_ = [
        ("prompt_tokens", ctypes.c_void_p),
        ("prompt_off", ctypes.c_void_p),
        ("response_tokens", ctypes.c_void_p),
        ("response_off", ctypes.c_void_p),
        ("reward_vals", ctypes.c_void_p),
        ("reward_off", ctypes.c_void_p),
        ("loss_mask_vals", ctypes.c_void_p),
        ("loss_mask_off", ctypes.c_void_p),
        ("logprob_vals", ctypes.c_void_p),
        ("logprob_off", ctypes.c_void_p),
    ]


VARIANT_FIELDS = (
    "logprob_unroll", "logprob_nt", "train_resident", "train_resident_nt", "train_ntstore", "train_split",
    "train_split_shape", "train_split_wait", "grpo_slices", "loss_units", "loss_bwd_blocks", "grpo_loss_rpb",
    "finish_mode", "sampler_row", "sampler_split_rows", "sampler_split_wgs", "sampler_split_nt", "sampler_split_gran",
    "sampler_topk_fast", "sampler_topp_fast", "topp_probe", "lmhead_pipe",
    "lmhead_group", "attn_pf", "lmhead_persist")
VARIANT_DEFAULT = -(2 ** 31)  # SKYRL_VARIANT_DEFAULT


class Variant(ctypes.Structure):
    """Mirror of ``skyrl_variant`` (include/skyrl_hip.h): per-call kernel variant selection."""

    _fields_ = [(f, ctypes.c_int32) for f in VARIANT_FIELDS]

    def __init__(self, **kw):
        super().__init__(*([VARIANT_DEFAULT] * len(VARIANT_FIELDS)))
        for k, v in kw.items():
            if k not in VARIANT_FIELDS:
                raise KeyError(f"unknown kernel variant field {k!r}")
            setattr(self, k, int(v))


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F = ctypes.c_float
_SZ = ctypes.c_size_t
_INT = ctypes.c_int

# name -> (restype, argtypes); the complete exported surface of include/skyrl_hip.h
SIGNATURES = {
    "skyrl_last_error": (ctypes.c_char_p, []),
    "skyrl_abi_version": (_INT, []),
    "skyrl_comm_unique_id_bytes": (_SZ, []),
    "skyrl_comm_get_unique_id": (_INT, [_P]),
    "skyrl_comm_init": (_INT, [_P, _I32, _I32, ctypes.POINTER(_P)]),
    "skyrl_comm_destroy": (_INT, [_P]),
    "skyrl_comm_size": (_INT, [_P, ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    "skyrl_comm_allreduce": (_INT, [_P, _P, _I64, _INT, _INT, _P, _P]),
    "skyrl_comm_reduce_scatter": (_INT, [_P, _P, _I64, _INT, _INT, _P, _P]),
    "skyrl_comm_allgather": (_INT, [_P, _P, _I64, _INT, _P, _P]),
    "skyrl_comm_broadcast": (_INT, [_P, _P, _I64, _INT, _I32, _P, _P]),
    "skyrl_variant_init": (None, [ctypes.POINTER(Variant)]),
    "skyrl_grpo_advantage": (_INT, [_P, _P, _P, _INT, _P, _P, _I32, _I32, _I32, _F, _I32, _P, _P, _P]),
    "skyrl_adv_norm_workspace_bytes": (_SZ, []),
    "skyrl_adv_norm_stats": (_INT, [_P, _P, _INT, _I64, _P, _P, _P]),
    "skyrl_adv_norm_apply": (_INT, [_P, _I64, _P, _P, _P]),
    "skyrl_gae_workspace_bytes": (_SZ, [_I32]),
    "skyrl_gae_advantage_return": (_INT, [_P, _P, _P, _INT, _I32, _I32, _F, _F, _P, _P, _P, _P, _P]),
    "skyrl_approx_kl": (_INT, [_P, _P, _P, _INT, _I64, _I32, _P, _P]),
    "skyrl_reward_kl_workspace_bytes": (_SZ, [_I32]),
    "skyrl_reward_kl_penalty": (_INT, [_P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _P, _P, _P]),
    "skyrl_ppo_loss_workspace_bytes": (_SZ, [_I32, _I32]),
    "skyrl_ppo_loss_fwd": (
        _INT,
        [_P, _P, _P, _P, _P, _P, _P, _I32, _I32, ctypes.POINTER(PPOParams), _P, _P, _P, _P, _I32, _P, _P],
    ),
    "skyrl_grpo_ppo_loss_fwd": (
        _INT,
        [_P, _P, _P, _INT, _I32, _F, _I32, _P, _P, _P, _P, _P, _P, _I32, _I32, ctypes.POINTER(PPOParams),
         _P, _P, _P, _P, _P, _I32, _P, _P],
    ),
    "skyrl_ppo_loss_bwd": (_INT, [_P, _I64, _P, _P, _P]),
    "skyrl_ppo_loss_finish": (_INT, [_P, _P, _P, _I32, _I32, ctypes.POINTER(PPOParams), _P, _P, _P, _P]),
    "skyrl_critic_loss_workspace_bytes": (_SZ, [_I32, _I32]),
    "skyrl_critic_loss_fwd": (_INT, [_P, _P, _P, _P, _I32, _I32, _F, _P, _P, _P, _P, _P]),
    "skyrl_logprob_fwd": (_INT, [_P, _INT, _I64, _I64, _I32, _I32, _I32, _P, _I64, _I64, _F, _P, _P, _P, _P]),
    "skyrl_logprob_bwd": (
        _INT,
        [_P, _INT, _I64, _I64, _I32, _I32, _I32, _P, _I64, _I64, _F, _P, _P, _P, _P, _P, _P],
    ),
    "skyrl_lmhead_state_bytes": (_SZ, [_I32]),
    "skyrl_lmhead_chunk_fwd": (_INT, [_P, _I64, _I32, _I32, _I64, _P, _I64, _F, _P, _I32, _I32, _P, _P, _P, _P]),
    "skyrl_lmhead_chunk_bwd": (_INT, [_P, _I64, _I32, _I32, _I64, _P, _I64, _F, _P, _P, _P, _P, _P, _I64, _P]),
    "skyrl_lmhead_state_merge": (_INT, [_P, _I32, _I32, _P, _P, _P, _P]),
    "skyrl_lmhead_gemm": (_INT, [_P, _I64, _P, _I64, _I32, _I32, _I32, _P, _I64, _P]),
    "skyrl_lmhead_sample_workspace_bytes": (_SZ, [_I32, _I32]),
    "skyrl_lmhead_logprob_workspace_bytes": (_SZ, [_I32, _I32]),
    "skyrl_lmhead_logprob_fwd": (
        _INT, [_P, _I64, _P, _I64, _I32, _I32, _I32, _P, _I64, _F, _P, _P, _P, _P, _P]),
    "skyrl_lmhead_sample": (
        _INT, [_P, _I64, _P, _I64, _I32, _I32, _I32, _F, ctypes.c_uint64, _P, _I64, _P, _P, _P, _P]),
    "skyrl_policy_train_workspace_bytes": (_SZ, [_I32, _I32]),
    "skyrl_policy_train_fwd": (
        _INT,
        [_P, _INT, _I64, _I64, _I32, _I32, _I32, _P, _I64, _I64, _F, _P, _P, _P, _P, ctypes.POINTER(PPOParams), _P,
         _P, _P, _P, _P, _I64, _I64, _P, _P],
    ),
    "skyrl_policy_train_ragged_fwd": (
        _INT,
        [_P, _INT, _I64, _I32, _I32, _P, _P, _I32, _I32, _F, _P, _P, _P, _P, ctypes.POINTER(PPOParams), _P, _P, _P,
         _P, _P, _I64, _P, _P],
    ),
    "skyrl_policy_train_step_workspace_bytes": (_SZ, [_I32, _I32, _I32]),
    "skyrl_policy_train_plan": (_INT, [_P, _I32, _I32, _I32, ctypes.POINTER(PPOParams), _P, _P]),
    "skyrl_policy_train_plan_grpo": (_INT, [_P, _I32, _I32, _I32, ctypes.POINTER(PPOParams), _P, _P, _I32, _I32, _F, _I32, _P,
                                           _P, _P, _P]),
    "skyrl_policy_train_micro_fwd": (
        _INT,
        [_P, _INT, _I64, _I32, _I32, _P, _I64, _I64, _P, _I32, _I32, _I32, _I32, _F, _P, _P, _P, _P,
         ctypes.POINTER(PPOParams), _P, _P, _P, _I64, _P, _P],
    ),
    "skyrl_policy_train_fold": (_INT, [_P, _I32, _I32, _I32, ctypes.POINTER(PPOParams), _P, _P, _P, _P]),
    "skyrl_policy_train_supports": (_INT, [_I32, _I32, _F]),
    "skyrl_scale_bf16_by_device_scalar": (_INT, [_P, _P, _I64, _P]),
    "skyrl_sample_workspace_bytes": (_SZ, [_I32, _I32]),
    "skyrl_sample": (_INT, [_P, _INT, _I64, _I32, _I32, _F, _I32, _F, _F, ctypes.c_uint64, _P, _I64, _P, _P, _P, _P]),
    "skyrl_pack_experience": (
        _INT,
        [ctypes.POINTER(PackInputs), _I32, _I32, _I32, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    ),
    "skyrl_scale_and_sumsq": (_INT, [_P, _I64, _F, _P, _P]),
    "skyrl_scale_by_device_scalar": (_INT, [_P, _P, _P, _I64, _P]),
    "skyrl_sumsq_workspace_bytes": (_SZ, [_I64]),
    "skyrl_sumsq": (_INT, [_P, _I64, _P, _P, _P]),
    "skyrl_adamw_plan_floats": (_SZ, []),
    "skyrl_adamw_plan": (_INT, [_P, ctypes.POINTER(AdamWParams), _P, _P, _P, _P]),
    "skyrl_adamw_update": (_INT, [_P, _P, _P, _P, _P, _I64, _P, _F, _F, _P]),
    "skyrl_adamw_seg_plan": (_INT, [_P, ctypes.POINTER(AdamWParams), _P, _I32, _P, _P, _P, _P, _P]),
    "skyrl_adamw_seg_update": (_INT, [_P, _P, _P, _P, _P, _I64, _P, _P, _P, _P, _I32, _P, _F, _F, _P]),
    "skyrl_adamw_seg_tile": (_SZ, []),
    "skyrl_cast_bf16": (_INT, [_P, _P, _I64, _P]),
    "skyrl_rope_kv_write": (_INT, [_P, _I64, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "skyrl_paged_decode_workspace_bytes": (_SZ, [_I32, _I32, _I32, _I32]),
    "skyrl_paged_decode": (_INT, [_P, _I64, _P, _P, _P, _I64, _P, _I32, _I32, _I32, _I32, _F, _I32, _I32, _P, _I64,
                                  _P, _P]),
    "skyrl_paged_decode_balanced_workspace_bytes": (_SZ, [_I32, _I32, _I32, _I32]),
    "skyrl_paged_decode_balanced": (_INT, [_P, _I64, _P, _P, _P, _I64, _P, _I32, _I32, _I32, _I32, _F, _I32, _P, _I64,
                                           _P, _P]),
    "skyrl_add_rmsnorm": (_INT, [_P, _P, _P, _I32, _I32, _F, _P, _P]),
    "skyrl_silu_mul": (_INT, [_P, _I64, _I32, _P, _P]),
}

# entry points with a per-call variant form (name + "_ex": the same arguments, then the variant)
EX_FORMS = ("skyrl_grpo_advantage", "skyrl_ppo_loss_fwd", "skyrl_grpo_ppo_loss_fwd", "skyrl_ppo_loss_bwd",
            "skyrl_ppo_loss_finish", "skyrl_logprob_fwd", "skyrl_logprob_bwd", "skyrl_lmhead_gemm",
            "skyrl_lmhead_logprob_fwd", "skyrl_lmhead_sample", "skyrl_policy_train_fwd", "skyrl_policy_train_ragged_fwd",
            "skyrl_policy_train_micro_fwd", "skyrl_policy_train_supports", "skyrl_sample", "skyrl_paged_decode")
for _n in EX_FORMS:
    _r, _a = SIGNATURES[_n]
    SIGNATURES[_n + "_ex"] = (_r, _a + [ctypes.POINTER(Variant)])

# The host's kernel-variant selection: a context variable (per thread / task), never library
# state. ``variant(**fields)`` scopes it; ``set_default_variant`` (probes) sets it until reset.
_VARIANT: contextvars.ContextVar = contextvars.ContextVar("skyrl_variant", default=None)


def _merged(fields):
    """The enclosing variant (if any) with `fields` overridden."""
    base = _VARIANT.get()
    out = Variant(**{f: getattr(base, f) for f in VARIANT_FIELDS}) if base is not None else Variant()
    for k, v in fields.items():
        if k not in VARIANT_FIELDS:
            raise KeyError(f"unknown kernel variant field {k!r}")
        setattr(out, k, int(v))
    return out


@contextlib.contextmanager
def variant(**fields):
    """Run the enclosed calls with another variant of the kernels (skyrl_variant, A/B and tests);
    nested scopes override the enclosing one's fields."""
    tok = _VARIANT.set(_merged(fields) if fields else _VARIANT.get())
    try:
        yield
    finally:
        _VARIANT.reset(tok)


def set_default_variant(**fields) -> None:
    """Probe scripts: keep this variant for the following calls of this thread (no args: the defaults)."""
    _VARIANT.set(_merged(fields) if fields else None)


def current_variant():
    return _VARIANT.get()


_lock = threading.Lock()
_lib = None


def lib_available() -> bool:
    return os.path.exists(LIB_PATH)


def load() -> ctypes.CDLL:
    """Load the library once and bind every signature. Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"skyrl_amd HIP library not built: {LIB_PATH} is missing. "
                "Run `python -c 'import __graft_entry__ as g; g.build()'` (make -C skyrl_amd/csrc)."
            )
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def call(name: str, *args) -> int:
    """Invoke a status-returning entry point; raise SkyrlHipError on a non-zero status. Under an
    active ``variant(...)`` an entry point with an _ex form runs that form with the variant."""
    lib = load()
    v = _VARIANT.get()
    if v is not None and name in EX_FORMS:
        rc = getattr(lib, name + "_ex")(*args, ctypes.byref(v))
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.skyrl_last_error().decode(errors="replace")
        raise SkyrlHipError(f"{name} failed (status {rc}): {msg}")
    return rc


def query(name: str, *args):
    """Invoke a non-status entry point (workspace sizes, version, support queries)."""
    v = _VARIANT.get()
    if v is not None and name in EX_FORMS:
        return getattr(load(), name + "_ex")(*args, ctypes.byref(v))
    return getattr(load(), name)(*args)
