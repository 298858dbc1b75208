"""PolarCode -- drop-in for the reference's ``polar.PolarCode`` hot-path surface (polar.py:64-484).

Same constructor and method signatures as the reference; every compute method runs on the MI355X
through libnpd (HIP kernels, ctypes C-ABI).  Host tensors (the eval loops pass ``noisy_code.cpu()``
to ``scl_decode``, run_models.py:329) are staged to the current GPU and results come back on the
input's device.

  PolarCode(n, K, args=None, F=None, rs=None, use_cuda=True, infty=1000.)      polar.py:66-117
  .encode_plotkin(message, scaling=None, custom_info_positions=None)            polar.py:128-148
  .encode  (alias of encode_plotkin, as rnn_all.get_code sets it, rnn_all.py:1187)
  .channel(code, snr[, noise_type, vv, radar_power, radar_prob])                polar.py:201-207
  .sc_decode_new(corrupted_codewords, snr, use_gt=None) -> (leaf_llrs, msg_hat) polar.py:465-484
  .sc_decode(noisy_code, snr) -> msg_hat   (exact-LSE SC, hard or soft)         polar.py:209-279
  .sc_decode_soft(noisy_code, snr, priors=None) -> msg_hat  (soft-output SC)     polar.py:281-358
  .sc_decode_soft_new(y, snr, priors=None) -> decoded_bits  (soft partial sums)   polar.py:485-607

MI355X extras (no reference equivalent, used by the Monte-Carlo driver and bench):
  .mc_generate(B, snr, seed, snr_index, cw_offset)   fused msg -> encode -> AWGN on device
  .sc_decode_mc(y, snr, seed, cw_offset, counters)   decode + fused error counting
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib
from .codes import info_from_frozen, polar_rs
from .utils import llr_scale, sigma_f32, snr_db2sigma


class _CodeHandle:
    """Owns one npd_code (immutable once created)."""

    def __init__(self, N: int, info: np.ndarray, pac_g: int = 0, infty: float = 1000.0):
        L = _lib.load()
        info32 = np.ascontiguousarray(np.sort(np.asarray(info, dtype=np.int64)), dtype=np.int32)
        out = ctypes.c_void_p()
        _lib.check(L.npd_code_create(int(N), int(info32.size), info32.ctypes.data_as(ctypes.c_void_p), int(pac_g),
                                     float(infty), ctypes.byref(out)), "npd_code_create")
        self.h = out
        self.N = int(N)
        self.K = int(info32.size)
        self.info = info32.astype(np.int64)

    def __del__(self):
        try:
            if self.h:
                _lib.load().npd_code_destroy(self.h)
        except Exception:
            pass


class _Philox:
    """Host-side bookkeeping for the counter-based channel RNG: (seed, running codeword offset)."""

    def __init__(self, seed=None):
        self.seed = int(torch.initial_seed() if seed is None else seed) & 0xFFFFFFFFFFFFFFFF
        self.offset = 0
        self.lock = threading.Lock()

    def take(self, n):
        with self.lock:
            o = self.offset
            self.offset += int(n)
        return o


class PolarCode:
    def __init__(self, n, K, args=None, F=None, rs=None, use_cuda=True, infty=1000.):
        assert n >= 1
        self.args = args
        self.n = n
        self.N = 2 ** n
        self.K = K
        self.infty = infty
        self.device = torch.device("cuda" if use_cuda else "cpu")
        if F is not None:
            assert len(F) == self.N - self.K
            self.frozen_positions = np.sort(np.asarray(F))
            self.unsorted_frozen_positions = np.asarray(F)
            self.info_positions = info_from_frozen(self.N, F)
            self.unsorted_info_positions = self.info_positions
        else:
            if rs is None:
                self.reliability_seq = np.arange(1023, -1, -1)
            else:
                self.reliability_seq = np.asarray(rs)
            self.rs = self.reliability_seq[self.reliability_seq < self.N]
            if rs is not None:
                assert len(self.rs) == self.N
            self.unsorted_info_positions = np.flip(self.rs[:self.K].copy())
            self.info_positions = np.sort(self.rs[:self.K].copy())
            self.unsorted_frozen_positions = self.rs[self.K:].copy()
            self.frozen_positions = np.sort(self.rs[self.K:].copy())
        self._code = None
        self._custom = {}
        self._rng = _Philox()

    # ------------------------------------------------------------------ handles
    @property
    def code(self) -> _CodeHandle:
        if self._code is None:
            self._code = _CodeHandle(self.N, self.info_positions, 0, self.infty)
        return self._code

    def _code_for(self, info_positions) -> _CodeHandle:
        if info_positions is None:
            return self.code
        key = tuple(int(i) for i in np.sort(np.asarray(info_positions)))
        h = self._custom.get(key)
        if h is None:
            h = self._custom[key] = _CodeHandle(self.N, np.asarray(key), 0, self.infty)
        return h

    def manual_seed(self, seed: int):
        """Seed the channel's Philox stream (the reference draws torch.randn on the CPU generator)."""
        self._rng = _Philox(seed)

    # ------------------------------------------------------------------ encoder (polar.py:128-148)
    def encode_plotkin(self, message, scaling=None, custom_info_positions=None):
        h = self._code_for(custom_info_positions)
        msg = _lib.f32c(_lib.stage(message, "message"))
        if msg.dim() != 2 or msg.shape[1] != h.K:
            raise ValueError(f"message must be (batch, {h.K}), got {tuple(msg.shape)}")
        x = torch.empty(msg.shape[0], self.N, dtype=torch.float32, device=msg.device)
        _lib.check(_lib.load().npd_encode(h.h, _lib.ptr(msg), _lib.ptr(x), msg.shape[0], _lib.stream_of(msg.device)),
                   "npd_encode")
        if scaling is not None:
            x = (scaling.to(x.device) * np.sqrt(self.N) * x) / torch.norm(scaling)
        return _lib.home(x, message)

    encode = encode_plotkin

    # ------------------------------------------------------------------ channel (polar.py:201-207)
    def channel(self, code, snr, noise_type="awgn", vv=None, radar_power=None, radar_prob=None, *, snr_index: int = 0):
        """y = x + sigma * N(0,1).  The extra arguments are the 6-argument call of rnn_all.py:847 /
        rnn.py:864 (which the reference's own 2-argument channel rejects); only 'awgn' is defined in
        the reference's code, so other noise types raise."""
        if noise_type not in (None, "awgn"):
            raise NotImplementedError(f"noise_type {noise_type!r}: the reference defines only the AWGN channel "
                                      "(polar.py:201-207)")
        x = _lib.f32c(_lib.stage(code, "code"))
        B, N = x.shape
        y = torch.empty_like(x)
        off = self._rng.take(B)
        _lib.check(_lib.load().npd_awgn(_lib.ptr(x), _lib.ptr(y), B, N, sigma_f32(snr), self._rng.seed, int(snr_index),
                                        off, _lib.stream_of(x.device)), "npd_awgn")
        return _lib.home(y, code)

    # ------------------------------------------------------------------ SC (polar.py:465-484)
    def sc_decode_new(self, corrupted_codewords, snr, use_gt=None):
        """Min-sum SC; returns (leaf LLRs incl. the frozen prior (B,N), msg_hat (B,K)) bit-exactly."""
        y = _aligned(_lib.f32c(_lib.stage(corrupted_codewords, "corrupted_codewords")))
        B = y.shape[0]
        leaf = torch.empty(B, self.N, dtype=torch.float32, device=y.device)
        hat = torch.empty(B, self.K, dtype=torch.float32, device=y.device)
        gt = None if use_gt is None else _lib.f32c(_lib.stage(use_gt, "use_gt", y.device))
        _lib.check(_lib.load().npd_sc_decode(self.code.h, _lib.ptr(y), llr_scale(snr), _lib.ptr(leaf), _lib.ptr(hat), None,
                                             _lib.ptr(gt), B, _lib.stream_of(y.device)), "npd_sc_decode")
        return _lib.home(leaf, corrupted_codewords), _lib.home(hat, corrupted_codewords)

    def sc_decode_msg(self, corrupted_codewords, snr):
        """msg_hat only (no leaf LLR traffic): the form the BER/BLER loops consume."""
        y = _aligned(_lib.f32c(_lib.stage(corrupted_codewords, "corrupted_codewords")))
        hat = torch.empty(y.shape[0], self.K, dtype=torch.float32, device=y.device)
        _lib.check(_lib.load().npd_sc_decode(self.code.h, _lib.ptr(y), llr_scale(snr), None, _lib.ptr(hat), None, None,
                                             y.shape[0], _lib.stream_of(y.device)), "npd_sc_decode")
        return _lib.home(hat, corrupted_codewords)

    # ------------------------------------------------------------------ SC-List (polar.py:793-876)
    def scl_decode(self, corrupted_codewords, snr, L=1, use_CRC=False, want_llrs=True):
        """SC-List decoding; returns (leaf LLRs of the chosen path (B,N), msg_hat (B,K)).

        The chosen path's leaf LLRs are recomputed by a genie SC pass with its decisions (identical
        values); ``want_llrs=False`` skips that pass and returns None in their place."""
        if use_CRC:
            raise NotImplementedError("scl_decode(use_CRC=True) depends on module globals of the reference "
                                      "(polar.py:741-763: `polar.CRC_len`); only the use_CRC=False path is built")
        y = _aligned(_lib.f32c(_lib.stage(corrupted_codewords, "corrupted_codewords")))
        B = y.shape[0]
        hat = torch.empty(B, self.K, dtype=torch.float32, device=y.device)
        uh = torch.empty(B, self.N, dtype=torch.float32, device=y.device) if want_llrs else None
        st = _lib.stream_of(y.device)
        _lib.check(_lib.load().npd_scl_decode(self.code.h, _lib.ptr(y), llr_scale(snr), int(L), _lib.ptr(hat),
                                              _lib.ptr(uh), B, st), "npd_scl_decode")
        if not want_llrs:
            return None, _lib.home(hat, corrupted_codewords)
        leaf = torch.empty(B, self.N, dtype=torch.float32, device=y.device)
        _lib.check(_lib.load().npd_sc_decode(self.code.h, _lib.ptr(y), llr_scale(snr), _lib.ptr(leaf), None, None,
                                             _lib.ptr(uh), B, st), "npd_sc_decode (genie leaf LLRs)")
        return _lib.home(leaf, corrupted_codewords), _lib.home(hat, corrupted_codewords)

    def scl_decode_mc(self, y, snr, L, seed, cw_offset, counters, msg_hat=None):
        _lib.require_gpu(y, "y")
        if y.dim() != 2 or y.shape[1] != self.N:
            raise ValueError(f"y must be (batch, {self.N}), got {tuple(y.shape)}")
        _lib.check_out(counters, "counters", torch.int64, 2, y.device)
        _lib.check_out(msg_hat, "msg_hat", torch.float32, y.shape[0] * self.K, y.device, optional=True)
        y = _aligned(_lib.f32c(y))
        _lib.check(_lib.load().npd_scl_decode_mc(self.code.h, _lib.ptr(y), llr_scale(snr), int(L), _lib.ptr(msg_hat),
                                                 int(seed), int(cw_offset), y.shape[0], _lib.ptr(counters),
                                                 _lib.stream_of(y.device)), "npd_scl_decode_mc")
        return counters

    # ------------------------------------------------------------------ exact-LSE SC (polar.py:209-279)
    def sc_decode(self, noisy_code, snr, hard_decision=None, return_bits=False):
        """PolarCode.sc_decode: SC with the exact boxplus (log_sum_avoid_zero_NaN, utils.py:295-397), no
        frozen prior; returns decoded_message = sign(decoded_bits)[:, info] (B,K).

        Decisions follow ``self.args.hard_decision`` as in the reference (sign(L) if set, else the soft
        tanh(L/2) -- argparse's default); ``hard_decision=`` overrides it.  ``return_bits=True`` also
        returns decoded_bits (B,N).  Not the min-sum ``sc_decode_new`` the eval loops call."""
        if hard_decision is None:
            hard_decision = bool(getattr(self.args, "hard_decision", False)) if self.args is not None else False
        y = _lib.f32c(_lib.stage(noisy_code, "noisy_code"))
        if y.dim() != 2 or y.shape[1] != self.N:
            raise ValueError(f"noisy_code must be (batch, {self.N}), got {tuple(y.shape)}")
        B = y.shape[0]
        hat = torch.empty(B, self.K, dtype=torch.float32, device=y.device)
        bits = torch.empty(B, self.N, dtype=torch.float32, device=y.device) if return_bits else None
        _lib.check(_lib.load().npd_sc_decode_lse(self.code.h, _lib.ptr(y), llr_scale(snr), 1 if hard_decision else 0,
                                                 _lib.ptr(hat), _lib.ptr(bits), B, _lib.stream_of(y.device)),
                   "npd_sc_decode_lse")
        hat = _lib.home(hat, noisy_code)
        return (hat, _lib.home(bits, noisy_code)) if return_bits else hat

    def sc_decode_soft(self, noisy_code, snr, priors=None, hard_decision=None, return_bits=False):
        """PolarCode.sc_decode_soft (polar.py:281-358): soft-output SC -- every node returns LLRs
        (LSE(L^_u, L^_v), L^_v), leaves clamp(L + prior, +-1000); frozen positions are not special (the
        priors carry them, as in the reference).  Returns sign(decoded_bits)[:, info] (B,K).  N <= 256."""
        if hard_decision is None:
            hard_decision = bool(getattr(self.args, "hard_decision", False)) if self.args is not None else False
        y = _aligned(_lib.f32c(_lib.stage(noisy_code, "noisy_code")))
        if y.dim() != 2 or y.shape[1] != self.N:
            raise ValueError(f"noisy_code must be (batch, {self.N}), got {tuple(y.shape)}")
        pr = self._priors(priors)
        B = y.shape[0]
        hat = torch.empty(B, self.K, dtype=torch.float32, device=y.device)
        bits = torch.empty(B, self.N, dtype=torch.float32, device=y.device) if return_bits else None
        _lib.check(_lib.load().npd_sc_decode_soft(self.code.h, _lib.ptr(y), llr_scale(snr), 1 if hard_decision else 0,
                                                  None if pr is None else pr.ctypes.data_as(ctypes.c_void_p),
                                                  _lib.ptr(hat), _lib.ptr(bits), B, _lib.stream_of(y.device)),
                   "npd_sc_decode_soft")
        hat = _lib.home(hat, noisy_code)
        return (hat, _lib.home(bits, noisy_code)) if return_bits else hat

    def _priors(self, priors):
        if priors is None:
            return None
        pr = np.ascontiguousarray(np.asarray(priors.cpu() if torch.is_tensor(priors) else priors,
                                             dtype=np.float32).reshape(-1))
        if pr.size != self.N:
            raise ValueError(f"priors must hold N = {self.N} values")
        return pr

    def sc_decode_soft_new(self, corrupted_codewords, snr, priors=None, return_u_hat=False):
        """PolarCode.sc_decode_soft_new (polar.py:592-607, with updateLLR_soft / partial_decode_soft /
        updatePartialSums_soft, polar.py:485-590): SC with LLR-valued ("soft") partial sums, leaves stored
        as clamp(L + prior, +-1000) + prior; returns decoded_bits = sign(stored leaf)[:, info] (B,K).
        priors=None means zeros, so frozen positions are decided like information positions, as in the
        reference.  ``return_u_hat=True`` also returns u_hat (B,N).  N <= 256."""
        y = _aligned(_lib.f32c(_lib.stage(corrupted_codewords, "corrupted_codewords")))
        if y.dim() != 2 or y.shape[1] != self.N:
            raise ValueError(f"corrupted_codewords must be (batch, {self.N}), got {tuple(y.shape)}")
        pr = self._priors(priors)
        B = y.shape[0]
        hat = torch.empty(B, self.K, dtype=torch.float32, device=y.device)
        u = torch.empty(B, self.N, dtype=torch.float32, device=y.device) if return_u_hat else None
        _lib.check(_lib.load().npd_sc_decode_soft_new(self.code.h, _lib.ptr(y), llr_scale(snr),
                                                      None if pr is None else pr.ctypes.data_as(ctypes.c_void_p),
                                                      _lib.ptr(hat), _lib.ptr(u), B, _lib.stream_of(y.device)),
                   "npd_sc_decode_soft_new")
        hat = _lib.home(hat, corrupted_codewords)
        return (hat, _lib.home(u, corrupted_codewords)) if return_u_hat else hat

    # ------------------------------------------------------------------ Monte-Carlo extras
    def mc_generate(self, B, snr, seed, snr_index=0, cw_offset=0, device=None, want_msg=True, want_x=False, out=None):
        device = torch.device(device or "cuda") if out is None else out.device
        if out is not None:
            _lib.check_out(out, "out", torch.float32, B * self.N, device)
        y = torch.empty(B, self.N, dtype=torch.float32, device=device) if out is None else out
        msg = torch.empty(B, self.K, dtype=torch.float32, device=device) if want_msg else None
        x = torch.empty(B, self.N, dtype=torch.float32, device=device) if want_x else None
        _lib.check(_lib.load().npd_mc_generate(self.code.h, _lib.ptr(msg), _lib.ptr(x), _lib.ptr(y), B, sigma_f32(snr),
                                               int(seed), int(snr_index), int(cw_offset), _lib.stream_of(device)),
                   "npd_mc_generate")
        return msg, x, y

    def fused_mc_supported(self) -> bool:
        """Codes whose Monte-Carlo step is faster as one fused generate + decode + count launch
        (npd_sc_mc_sweep_fused) than as npd_mc_generate + npd_sc_decode_mc_sweep: N <= 128 (measured per 2^20 words:
        N = 64 0.076 vs 0.40 ms, N = 128 0.375 vs 0.392 ms; at N = 256 the fused kernel spills and takes 2.7 ms
        against 1.3 ms, so the Monte-Carlo driver generates y there -- the C ABI still accepts every N)."""
        return 4 <= self.N <= 128

    def sc_decode_mc_sweep(self, y, snrs, seed, cw_offset, counters, msg_hat=None):
        """y (n_snr, B, N) -> counters (n_snr, 2) += errors at each SNR, one launch (npd_sc_decode_mc_sweep)."""
        _lib.require_gpu(y, "y")
        if y.dim() != 3 or y.shape[2] != self.N:
            raise ValueError(f"y must be (n_snr, B, {self.N}), got {tuple(y.shape)}")
        n, B = y.shape[0], y.shape[1]
        _lib.check_out(counters, "counters", torch.int64, 2 * n, y.device)
        _lib.check_out(msg_hat, "msg_hat", torch.float32, n * B * self.K, y.device, optional=True)
        scales = np.asarray([llr_scale(s) for s in snrs], dtype=np.float32)
        if len(scales) != n:
            raise ValueError("one SNR per y segment")
        y = _aligned(_lib.f32c(y))
        _lib.check(_lib.load().npd_sc_decode_mc_sweep(self.code.h, n, _lib.ptr(y), scales.ctypes.data_as(ctypes.c_void_p),
                                                      _lib.ptr(msg_hat), int(seed), int(cw_offset), B,
                                                      _lib.ptr(counters), _lib.stream_of(y.device)),
                   "npd_sc_decode_mc_sweep")
        return counters

    def sc_mc_sweep_fused(self, B, snrs, seed, cw_offset, counters, msg_hat=None, snr_index0=0):
        """counters (n_snr, 2) += errors of SC on B fresh codewords per SNR, generated in the decode kernel
        (npd_sc_mc_sweep_fused): identical counts to mc_generate(snr_index = snr_index0 + s) followed by
        sc_decode_mc_sweep.  Codes with fused_mc_supported(); at most 16 SNR points per call."""
        _lib.check_out(counters, "counters", torch.int64, 2 * len(snrs))
        _lib.check_out(msg_hat, "msg_hat", torch.float32, len(snrs) * int(B) * self.K, counters.device, optional=True)
        sig = np.asarray([sigma_f32(s) for s in snrs], dtype=np.float32)
        scl = np.asarray([llr_scale(s) for s in snrs], dtype=np.float32)
        _lib.check(_lib.load().npd_sc_mc_sweep_fused(self.code.h, len(sig), sig.ctypes.data_as(ctypes.c_void_p),
                                                     scl.ctypes.data_as(ctypes.c_void_p), int(snr_index0), int(seed),
                                                     int(cw_offset), int(B), _lib.ptr(msg_hat), _lib.ptr(counters),
                                                     _lib.stream_of(counters.device)), "npd_sc_mc_sweep_fused")
        return counters

    def sc_decode_mc(self, y, snr, seed, cw_offset, counters, msg_hat=None):
        _lib.require_gpu(y, "y")
        if y.dim() != 2 or y.shape[1] != self.N:
            raise ValueError(f"y must be (batch, {self.N}), got {tuple(y.shape)}")
        _lib.check_out(counters, "counters", torch.int64, 2, y.device)
        _lib.check_out(msg_hat, "msg_hat", torch.float32, y.shape[0] * self.K, y.device, optional=True)
        y = _aligned(_lib.f32c(y))
        _lib.check(_lib.load().npd_sc_decode_mc(self.code.h, _lib.ptr(y), llr_scale(snr), _lib.ptr(msg_hat), int(seed),
                                                int(cw_offset), y.shape[0], _lib.ptr(counters), _lib.stream_of(y.device)),
                   "npd_sc_decode_mc")
        return counters


def _aligned(y: torch.Tensor) -> torch.Tensor:
    """The list kernel reads 16-byte vectors: re-base an unaligned view (rare: odd row offsets)."""
    return y if y.data_ptr() % 16 == 0 else y.clone()


def reference_polar_code(N: int, K: int, args=None, infty=1000.) -> PolarCode:
    """PolarCode(n, K, args, rs=rs) with the reference's 'polar' reliability order (run_models.py:630-639)."""
    n = int(np.log2(N))
    return PolarCode(n, K, args, rs=polar_rs(N), infty=infty)


__all__ = ["PolarCode", "reference_polar_code", "snr_db2sigma"]
