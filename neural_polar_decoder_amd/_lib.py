"""ctypes binding of libnpd.so (include/npd.h).

The product path has exactly one implementation: the HIP kernels in libnpd.so.  If the library is
missing or no GPU is visible, every compute call raises :class:`NpdError` -- there is no CPU fallback.
Host tensors given to the reference-surface methods are staged to the GPU (:func:`stage`) and the
results copied back (:func:`home`); the compute stays on the GPU.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NPD_LIB", os.path.join(_HERE, "libnpd.so"))

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_float = ctypes.c_float

# (name, restype, argtypes) -- must match include/npd.h exactly (tests check every symbol)
SIGNATURES = [
    ("npd_abi_version", c_int, []),
    ("npd_last_error", ctypes.c_char_p, []),
    ("npd_device_count", c_int, []),
    ("npd_code_create", c_int, [c_int, c_int, c_void_p, c_int, c_float, ctypes.POINTER(c_void_p)]),
    ("npd_code_destroy", c_int, [c_void_p]),
    ("npd_encode", c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    ("npd_awgn", c_int, [c_void_p, c_void_p, c_i64, c_int, c_float, c_u64, c_u32, c_u64, c_void_p]),
    ("npd_mc_generate", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_float, c_u64, c_u32, c_u64,
                                c_void_p]),
    ("npd_sc_decode", c_int, [c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    ("npd_sc_decode_mc", c_int, [c_void_p, c_void_p, c_float, c_void_p, c_u64, c_u64, c_i64, c_void_p, c_void_p]),
    ("npd_sc_decode_mc_sweep", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_u64, c_u64, c_i64, c_void_p,
                                       c_void_p]),
    ("npd_sc_mc_sweep_fused", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_u32, c_u64, c_u64, c_i64, c_void_p,
                                      c_void_p, c_void_p]),
    ("npd_sc_decode_lse", c_int, [c_void_p, c_void_p, c_float, c_int, c_void_p, c_void_p, c_i64, c_void_p]),
    ("npd_sc_decode_soft", c_int, [c_void_p, c_void_p, c_float, c_int, c_void_p, c_void_p, c_void_p, c_i64,
                                   c_void_p]),
    ("npd_sc_decode_soft_new", c_int, [c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    ("npd_scl_decode", c_int, [c_void_p, c_void_p, c_float, c_int, c_void_p, c_void_p, c_i64, c_void_p]),
    ("npd_scl_decode_mc", c_int, [c_void_p, c_void_p, c_float, c_int, c_void_p, c_u64, c_u64, c_i64, c_void_p,
                                  c_void_p]),
    ("npd_list_prune_select", c_int, [c_void_p, c_int, c_int, c_void_p]),
    ("npd_count_errors", c_int, [c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p]),
    ("npd_count_errors_cols", c_int, [c_void_p, c_void_p, c_i64, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    ("npd_count_errors_masked", c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p]),
    ("npd_gru_create", c_int, [c_int, c_int, c_int, c_int, c_void_p, c_i64, c_int, ctypes.POINTER(c_void_p)]),
    ("npd_gru_destroy", c_int, [c_void_p]),
    ("npd_gru_decode", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    ("npd_rnn_create", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_i64, c_int, ctypes.POINTER(c_void_p)]),
    ("npd_rnn_create_ex", c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_i64, c_int, c_void_p, c_void_p,
                                  c_float, c_int, c_int, c_void_p, c_i64, ctypes.POINTER(c_void_p)]),
    ("npd_gru_decode_ex", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64,
                                  c_void_p]),
    ("npd_gru_decode_count_sweep", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                           c_void_p, c_i64, c_void_p, c_void_p]),
    ("npd_ymlp_layer", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int, c_int, c_void_p]),
    ("npd_conv_create", c_int, [c_int, c_int, c_void_p, c_i64, c_int, ctypes.POINTER(c_void_p)]),
    ("npd_conv_destroy", c_int, [c_void_p]),
    ("npd_conv_workspace_bytes", c_i64, [c_void_p, c_i64]),
    ("npd_conv_forward", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    ("npd_conv_forward_ex", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
]


class NpdError(RuntimeError):
    pass


_lib = None


def load():
    """Load libnpd.so (raises NpdError if it is missing -- build it with `make lib`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NpdError(f"libnpd.so not found at {LIB_PATH}; build it with `make` or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().npd_last_error()
        raise NpdError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def require_gpu(t: torch.Tensor, name: str):
    """Device-only entry points (the Monte-Carlo extras): fail loudly for host tensors."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise NpdError(f"{name} must be a device (HIP) tensor: libnpd has no CPU path")


def check_out(t, name: str, dtype: torch.dtype, numel: int, device: torch.device | None = None, optional=False):
    """A caller-supplied output buffer the kernels write through a raw pointer: it must be a contiguous device
    tensor of ``dtype`` with at least ``numel`` elements (on ``device``), or the kernel would write past it."""
    if t is None:
        if optional:
            return
        raise ValueError(f"{name} is required")
    require_gpu(t, name)
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.numel() < numel:
        raise ValueError(f"{name} holds {t.numel()} elements, the call writes {numel}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, the call runs on {device}")


def compute_device() -> torch.device:
    """The GPU that runs a call whose inputs live on the host: torch's current HIP device."""
    if not torch.cuda.is_available():
        raise NpdError("no GPU visible: libnpd computes only on the MI355X (there is no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def stage(t, name: str, device: torch.device | None = None) -> torch.Tensor:
    """Input of a reference-surface method as a device tensor.

    The reference's eval loops hand some methods host tensors (``polar.scl_decode(noisy_code.cpu(), ...)``
    run_models.py:329, rnn_all.py:858; ``errors_ber(msg_bits.cpu(), ...)`` run_models.py:330-336).
    Those are copied to ``device`` (default: the current HIP device) and computed on the GPU; the caller
    returns results with :func:`home`.  Device tensors pass through untouched (no copy, no sync)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.is_cuda:
        return t if device is None or t.device == device else t.to(device)
    return t.to(device if device is not None else compute_device())


def home(t: torch.Tensor | None, like: torch.Tensor):
    """Return a result on the device of the caller's input ``like`` (host results of host inputs)."""
    if t is None or t.device == like.device:
        return t
    return t.to(like.device)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def f32c(t: torch.Tensor) -> torch.Tensor:
    """contiguous fp32 view/copy on the same device"""
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()
