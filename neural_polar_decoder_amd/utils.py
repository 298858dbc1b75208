"""Numerics helpers and error counters with the reference's semantics (utils.py:5-51).

``errors_ber`` / ``errors_bler`` keep the reference's signatures and return values but count on
the GPU (npd_count_errors) into device uint64 counters: no per-batch host round trip
(the reference copies to numpy in errors_bler, utils.py:41-45).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def snr_db2sigma(train_snr):
    """sigma = 10^(-snr/20) (utils.py:5-6)."""
    return 10 ** (-train_snr * 1.0 / 20)


def llr_scale(snr) -> float:
    """fl32(2 / sigma^2): the scalar torch applies in ``(2/sigma**2)*y`` (polar.py:468)."""
    sigma = snr_db2sigma(snr)
    return float(np.float32(2 / sigma ** 2))


def sigma_f32(snr) -> float:
    return float(np.float32(snr_db2sigma(snr)))


def count_errors(y_true: torch.Tensor, y_pred: torch.Tensor, counters: torch.Tensor | None = None) -> torch.Tensor:
    """Device counters [bit errors, block errors] (uint64 stored in an int64 tensor), accumulated."""
    _lib.require_gpu(y_true, "y_true")
    _lib.require_gpu(y_pred, "y_pred")
    t = _lib.f32c(y_true.reshape(y_true.shape[0], -1))
    p = _lib.f32c(y_pred.reshape(y_pred.shape[0], -1))
    if t.shape != p.shape:
        raise ValueError(f"shape mismatch {tuple(t.shape)} vs {tuple(p.shape)}")
    if counters is None:
        counters = torch.zeros(2, dtype=torch.int64, device=t.device)
    L = _lib.load()
    _lib.check(L.npd_count_errors(_lib.ptr(t), _lib.ptr(p), t.shape[0], t.shape[1], _lib.ptr(counters),
                                  _lib.stream_of(t.device)), "npd_count_errors")
    return counters


def errors_ber(y_true, y_pred, mask=None):
    """Bit error rate (utils.py:17-25): mean of round(true) != round(pred). Returns a 0-dim tensor."""
    if mask is not None and not bool(torch.all(mask == 1)):
        # masked form is only used with all-ones masks in the eval loops (run_models.py:323-341)
        y_true = y_true.reshape(y_true.shape[0], -1)
        y_pred = y_pred.reshape(y_pred.shape[0], -1)
        m = mask.reshape(mask.shape[0], -1).to(y_true.dtype)
        return (m * torch.ne(torch.round(y_true), torch.round(y_pred)).float()).sum() / m.sum()
    c = count_errors(y_true, y_pred)
    n = y_true.numel()
    return c[0].double() / n


def errors_bler(y_true, y_pred, get_pos=False):
    """Block error rate (utils.py:37-51): fraction of rows with any rounded mismatch. Returns a float."""
    if get_pos:
        t = torch.round(y_true.reshape(y_true.shape[0], -1))
        p = torch.round(y_pred.reshape(y_pred.shape[0], -1))
        bad = (t != p).any(dim=1)
        return float(bad.float().mean()), list(torch.nonzero(bad).flatten().cpu().numpy())
    c = count_errors(y_true, y_pred)
    return float(c[1].item()) / y_true.shape[0]
