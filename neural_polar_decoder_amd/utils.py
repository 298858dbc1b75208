"""Numerics helpers and error counters with the reference's semantics (utils.py:5-51).

``errors_ber`` / ``errors_bler`` keep the reference's signatures and return types (a (1,) float32
tensor on the input's device / a ``numpy.float64``) but count on the GPU (npd_count_errors) into
device uint64 counters.  Host inputs (the eval loops pass ``msg_bits.cpu()``, run_models.py:330-336)
are staged to the GPU first.
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


def count_errors(y_true: torch.Tensor, y_pred: torch.Tensor, counters: torch.Tensor | None = None,
                 cols=None) -> torch.Tensor:
    """Device counters [bit errors, block errors] (uint64 stored in an int64 tensor), accumulated.

    ``cols`` (K ints): compare y_true (B,K) with y_pred[:, cols] of a (B,W) y_pred without gathering it
    (npd_count_errors_cols).  Host inputs are staged to the GPU of ``counters`` (or the current device)."""
    dev = counters.device if counters is not None and counters.is_cuda else None
    t = _lib.stage(y_true, "y_true", dev)
    p = _lib.stage(y_pred, "y_pred", t.device)
    # explicit widths: an empty batch (B = 0) is a no-op, not an ambiguous reshape
    t = _lib.f32c(t.reshape(t.shape[0], int(np.prod(t.shape[1:], dtype=np.int64))))
    p = _lib.f32c(p.reshape(p.shape[0], int(np.prod(p.shape[1:], dtype=np.int64))))
    if counters is None:
        counters = torch.zeros(2, dtype=torch.int64, device=t.device)
    _lib.require_gpu(counters, "counters")
    L = _lib.load()
    if cols is not None:
        c = np.ascontiguousarray(np.asarray(cols, dtype=np.int64).reshape(-1), dtype=np.int32)
        if t.shape[0] != p.shape[0] or c.size != t.shape[1]:
            raise ValueError(f"shape mismatch {tuple(t.shape)} vs {tuple(p.shape)} at {c.size} columns")
        if t.shape[0] == 0:
            return counters
        _lib.check(L.npd_count_errors_cols(_lib.ptr(t), _lib.ptr(p), t.shape[0], t.shape[1], p.shape[1],
                                           c.ctypes.data_as(_lib.c_void_p), _lib.ptr(counters),
                                           _lib.stream_of(t.device)), "npd_count_errors_cols")
        return counters
    if t.shape != p.shape:
        raise ValueError(f"shape mismatch {tuple(t.shape)} vs {tuple(p.shape)}")
    if t.shape[0] == 0:
        return counters
    _lib.check(L.npd_count_errors(_lib.ptr(t), _lib.ptr(p), t.shape[0], t.shape[1], _lib.ptr(counters),
                                  _lib.stream_of(t.device)), "npd_count_errors")
    return counters


def _masked_errors(y_true, y_pred, mask):
    """(mask * (round(true) != round(pred))) as float on the GPU, per element (utils.py:20-23)."""
    t = _lib.stage(y_true, "y_true")
    p = _lib.stage(y_pred, "y_pred", t.device)
    t = t.reshape(t.shape[0], -1, 1)
    p = p.reshape(p.shape[0], -1, 1)
    m = _lib.stage(mask, "mask", t.device).reshape(mask.shape[0], -1, 1)
    return (m * torch.ne(torch.round(t), torch.round(p))).float(), m


def errors_ber(y_true, y_pred, mask=None):
    """Bit error rate (utils.py:17-25): mean of round(true) != round(pred) over the mask.

    Returns what the reference returns -- a float32 tensor of shape (1,) on ``y_true``'s device
    (``sum(sum(x)) / torch.sum(mask)``) -- so the eval loops' ``.item()`` works unchanged.  The counts are
    exact (device int64), then each is rounded once to fp32 and divided in fp32: exact-then-rounded, not an fp32
    accumulation.  Below 2^24 errors / mask elements per call both are exact and the result is the reference's
    bit for bit; above it the reference's float32 sums drop low bits as they accumulate and ours is the correctly
    rounded quotient of the true counts.  An integer mask (the loops' torch.ones(...).long()) is counted by
    npd_count_errors_masked -- sum(mask * err) / sum(mask), decided on the device with no host read of the mask
    (an all-ones mask costs the same single pass); a floating-point mask takes the reference's formula on the GPU."""
    y_true.view(y_true.shape[0], -1, 1)  # the reference's first step (utils.py:20): raises on an empty batch as there
    if mask is not None:
        t = _lib.f32c(_lib.stage(y_true, "y_true"))
        if mask.dtype.is_floating_point or mask.dtype.is_complex:
            e, m = _masked_errors(y_true, y_pred, mask)
            return _lib.home((e.sum() / torch.sum(m)).reshape(1).float(), y_true)
        p = _lib.f32c(_lib.stage(y_pred, "y_pred", t.device))
        m = _lib.stage(mask, "mask", t.device).to(torch.int64).contiguous()
        t, p = t.reshape(t.shape[0], -1), p.reshape(p.shape[0], -1)
        m = m.reshape(m.shape[0], -1)
        if t.shape != p.shape or t.shape != m.shape:
            raise ValueError(f"shape mismatch {tuple(t.shape)} / {tuple(p.shape)} / mask {tuple(m.shape)}")
        c = torch.zeros(2, dtype=torch.int64, device=t.device)
        _lib.check(_lib.load().npd_count_errors_masked(_lib.ptr(t), _lib.ptr(p), _lib.ptr(m), t.shape[0], t.shape[1],
                                                       _lib.ptr(c), _lib.stream_of(t.device)), "npd_count_errors_masked")
        return _lib.home((c[0:1].float() / c[1:2].float()), y_true)
    c = count_errors(y_true, y_pred)
    n = y_true.numel()
    res = c[0:1].float() / torch.tensor(float(n), dtype=torch.float32, device=c.device)
    return _lib.home(res, y_true)


def errors_bitwise_ber(y_true, y_pred, mask=None):
    """Per-position bit error rate (utils.py:27-35): shape (K, 1), on ``y_true``'s device."""
    if mask is None:
        mask = torch.ones(y_true.size(), device=y_true.device)
    e, m = _masked_errors(y_true, y_pred, mask)
    return _lib.home(torch.sum(e, 0) / torch.sum(m, 0), y_true)


def errors_bler(y_true, y_pred, get_pos=False):
    """Block error rate (utils.py:37-51): fraction of rows with any rounded mismatch.

    Returns ``numpy.float64`` like the reference (its loops call ``.item()`` on it, rnn_all.py:856,
    run_models.py:331); with ``get_pos`` also the list of erroneous row indices (numpy int64)."""
    B = y_true.shape[0]
    y_true.view(B, -1, 1)  # the reference's first step (utils.py:38): raises on an empty batch as there
    if get_pos:
        e, _ = _masked_errors(y_true, y_pred, torch.ones(1, dtype=torch.float32).expand(B, 1))
        bad = (e.reshape(B, -1).sum(1) > 0).cpu().numpy()
        return np.float64(int(bad.sum()) * 1.0 / B), list(np.nonzero(bad.astype(int))[0])
    c = count_errors(y_true, y_pred)
    return np.float64(int(c[1].item()) * 1.0 / B)
