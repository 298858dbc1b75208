"""PAC -- drop-in for the reference's ``pac_code.PAC`` hot-path surface (pac_code.py:94-573).

  PAC(args, N, K, g, infty=1000., rate_profile='RM')                   pac_code.py:97-119
  .rate_profiler(msg_bits, scheme='RM', custom_info_positions=None)   pac_code.py:121-174
  .pac_encode(msg_bits, scheme=None, custom_info_positions=None)      pac_code.py:220-224
  .polar_encode(u) (rate-1 Plotkin)                                   pac_code.py:210-218
  .channel(code, snr)                                                 pac_code.py:226-231
  .pac_sc_decode(y, snr, use_gt_codeword=None) -> (llr, v_hat[:,B], u_hat)   pac_code.py:534-573
  .extract(v_hat, B=None)                                             pac_code.py:528-531
All compute runs in libnpd's HIP kernels; host inputs are staged to the current GPU and results come
back on the input's device.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .codes import pac_info_positions
from .polar import _aligned, _CodeHandle, _Philox
import ctypes

from .utils import llr_scale, sigma_f32


def dec2bitarray(in_number, bit_width):
    bits = np.zeros(bit_width, "int")
    s = bin(int(in_number))[2:]
    for i, ch in enumerate(reversed(s)):
        bits[bit_width - 1 - i] = int(ch)
    return bits


class PAC:
    def __init__(self, args, N, K, g, infty=1000., rate_profile="RM"):
        self.N = N
        self.n = int(np.log2(N))
        self.K = K
        self.args = args
        self.g = int(g)
        M = int(np.floor(np.log2(g))) + 1
        self.g_array = 1 - 2 * dec2bitarray(g, M)
        self.rate_profile = rate_profile
        self.infty = infty
        w = np.array([bin(i).count("1") for i in range(N)])
        self.unsorted_info_positions = np.argsort(w)[-self.K:]
        self.B = np.sort(self.unsorted_info_positions.copy())
        self._codes = {}
        self._rate1 = None
        self._rng = _Philox()

    def _target_K(self):
        try:
            return int(self.args.target_K)
        except Exception:
            return self.N // 2

    def _set_for(self, scheme=None, custom_info_positions=None):
        if custom_info_positions is not None:
            return np.sort(np.asarray(custom_info_positions))
        if scheme is None:
            scheme = self.rate_profile
        return pac_info_positions(self.N, self.K, scheme, self._target_K())

    def _code_for(self, B) -> _CodeHandle:
        key = tuple(int(i) for i in B)
        h = self._codes.get(key)
        if h is None:
            h = self._codes[key] = _CodeHandle(self.N, np.asarray(key), self.g, self.infty)
        return h

    def manual_seed(self, seed: int):
        self._rng = _Philox(seed)

    # ------------------------------------------------------------------ encoder
    def rate_profiler(self, msg_bits, scheme="RM", custom_info_positions=None):
        B = self._set_for(scheme, custom_info_positions)
        u = torch.ones((msg_bits.shape[0], self.N), dtype=torch.float, device=msg_bits.device)
        u[:, torch.as_tensor(B, device=msg_bits.device)] = msg_bits.float()
        self.B = B
        return u

    def pac_encode(self, msg_bits, scheme=None, custom_info_positions=None):
        B = self._set_for(scheme, custom_info_positions)
        self.B = B
        h = self._code_for(B)
        msg = _lib.f32c(_lib.stage(msg_bits, "msg_bits"))
        x = torch.empty(msg.shape[0], self.N, dtype=torch.float32, device=msg.device)
        _lib.check(_lib.load().npd_encode(h.h, _lib.ptr(msg), _lib.ptr(x), msg.shape[0], _lib.stream_of(msg.device)),
                   "npd_encode")
        return _lib.home(x, msg_bits)

    encode = pac_encode

    def polar_encode(self, msg_bits):
        """Rate-1 Plotkin transform of u (B,N)."""
        if self._rate1 is None:
            self._rate1 = _CodeHandle(self.N, np.arange(self.N), 0, self.infty)
        u = _lib.f32c(_lib.stage(msg_bits, "msg_bits"))
        x = torch.empty_like(u)
        _lib.check(_lib.load().npd_encode(self._rate1.h, _lib.ptr(u), _lib.ptr(x), u.shape[0], _lib.stream_of(u.device)),
                   "npd_encode")
        return _lib.home(x, msg_bits)

    # ------------------------------------------------------------------ channel
    def channel(self, code, snr, noise_type="awgn", vv=None, radar_power=None, radar_prob=None, *, snr_index: int = 0):
        """y = x + sigma * N(0,1); the extra arguments accept rnn.py:754's 6-argument call (AWGN only)."""
        if noise_type not in (None, "awgn"):
            raise NotImplementedError(f"noise_type {noise_type!r}: the reference defines only the AWGN channel "
                                      "(pac_code.py:226-231)")
        x = _lib.f32c(_lib.stage(code, "code"))
        Bn, N = x.shape
        y = torch.empty_like(x)
        off = self._rng.take(Bn)
        _lib.check(_lib.load().npd_awgn(_lib.ptr(x), _lib.ptr(y), Bn, N, sigma_f32(snr), self._rng.seed, int(snr_index),
                                        off, _lib.stream_of(x.device)), "npd_awgn")
        return _lib.home(y, code)

    # ------------------------------------------------------------------ SC (pac_code.py:534-573)
    def pac_sc_decode(self, corrupted_codewords, snr, use_gt_codeword=None):
        y = _aligned(_lib.f32c(_lib.stage(corrupted_codewords, "corrupted_codewords")))
        Bn = y.shape[0]
        h = self._code_for(self.B)
        llr = torch.empty(Bn, self.N, dtype=torch.float32, device=y.device)
        vh = torch.empty(Bn, h.K, dtype=torch.float32, device=y.device)
        uh = torch.empty(Bn, self.N, dtype=torch.float32, device=y.device)
        gt = None if use_gt_codeword is None else _lib.f32c(_lib.stage(use_gt_codeword, "use_gt_codeword", y.device))
        _lib.check(_lib.load().npd_sc_decode(h.h, _lib.ptr(y), llr_scale(snr), _lib.ptr(llr), _lib.ptr(vh), _lib.ptr(uh),
                                             _lib.ptr(gt), Bn, _lib.stream_of(y.device)), "npd_sc_decode")
        c = corrupted_codewords
        return _lib.home(llr, c), _lib.home(vh, c), _lib.home(uh, c)

    def extract(self, v_hat, B=None):
        if B is None:
            B = self.B
        return v_hat[:, torch.as_tensor(np.asarray(B), device=v_hat.device)]

    # ------------------------------------------------------------------ Monte-Carlo extras
    def mc_generate(self, Bn, snr, seed, snr_index=0, cw_offset=0, device=None, want_msg=True, want_x=False, out=None):
        device = torch.device(device or "cuda") if out is None else out.device
        h = self._code_for(self.B)
        if out is not None:
            _lib.check_out(out, "out", torch.float32, Bn * self.N, device)
        y = torch.empty(Bn, self.N, dtype=torch.float32, device=device) if out is None else out
        msg = torch.empty(Bn, h.K, dtype=torch.float32, device=device) if want_msg else None
        x = torch.empty(Bn, self.N, dtype=torch.float32, device=device) if want_x else None
        _lib.check(_lib.load().npd_mc_generate(h.h, _lib.ptr(msg), _lib.ptr(x), _lib.ptr(y), Bn, sigma_f32(snr),
                                               int(seed), int(snr_index), int(cw_offset), _lib.stream_of(device)),
                   "npd_mc_generate")
        return msg, x, y

    def fused_mc_supported(self) -> bool:
        """The Monte-Carlo driver runs the PAC step as one fused generate + SC decode + count launch for N <= 128.
        At N = 256 the fused kernel spills (1 KB/lane) and measured 2.7 ms against 1.1 + 0.2 ms for decode +
        generate per 2^20 Polar(256,128) words, so there the driver generates y first; the C ABI
        (npd_sc_mc_sweep_fused) still fuses every N."""
        return 4 <= self.N <= 128

    def sc_mc_sweep_fused(self, Bn, snrs, seed, cw_offset, counters, msg_hat=None, snr_index0=0):
        """counters (n_snr, 2) += errors of PAC SC on Bn fresh codewords per SNR point, generated inside the
        decode kernel (npd_sc_mc_sweep_fused; y never stored): identical counts and v_hat[:, B] to
        mc_generate(snr_index = snr_index0 + s) followed by sc_decode_mc at each SNR (the configs[3] eval's
        SC baseline, rnn_all.py:730-776, without the received words' HBM round trip)."""
        h = self._code_for(self.B)
        _lib.check_out(counters, "counters", torch.int64, 2 * len(snrs))
        _lib.check_out(msg_hat, "msg_hat", torch.float32, len(snrs) * int(Bn) * h.K, counters.device, optional=True)
        sig = np.asarray([sigma_f32(s) for s in snrs], dtype=np.float32)
        scl = np.asarray([llr_scale(s) for s in snrs], dtype=np.float32)
        _lib.check(_lib.load().npd_sc_mc_sweep_fused(h.h, len(sig), sig.ctypes.data_as(ctypes.c_void_p),
                                                     scl.ctypes.data_as(ctypes.c_void_p), int(snr_index0), int(seed),
                                                     int(cw_offset), int(Bn), _lib.ptr(msg_hat), _lib.ptr(counters),
                                                     _lib.stream_of(counters.device)), "npd_sc_mc_sweep_fused")
        return counters

    def sc_decode_mc(self, y, snr, seed, cw_offset, counters, msg_hat=None):
        _lib.require_gpu(y, "y")
        if y.dim() != 2 or y.shape[1] != self.N:
            raise ValueError(f"y must be (batch, {self.N}), got {tuple(y.shape)}")
        h = self._code_for(self.B)
        _lib.check_out(counters, "counters", torch.int64, 2, y.device)
        _lib.check_out(msg_hat, "msg_hat", torch.float32, y.shape[0] * h.K, y.device, optional=True)
        y = _aligned(_lib.f32c(y))
        _lib.check(_lib.load().npd_sc_decode_mc(h.h, _lib.ptr(y), llr_scale(snr), _lib.ptr(msg_hat), int(seed),
                                                int(cw_offset), y.shape[0], _lib.ptr(counters), _lib.stream_of(y.device)),
                   "npd_sc_decode_mc")
        return counters
