"""convNet decoder -- drop-in for models.convNet (models.py:691-772).

Same modules and parameter names as the reference (so ``load_state_dict`` of a reference checkpoint
works); ``decode``/``forward`` run the whole network through libnpd's MFMA kernels
(npd_conv_forward): implicit-GEMM dilated Conv1d + GELU (+ residual) layers, FC GEMMs with fused
bias/GELU, LayerNorm + sign.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from . import _lib


class convNet(nn.Module):
    """models.convNet.  ``precision`` (keyword, not in the reference): "fp32" (default; exact fp32 FMA chains on
    v_mfma_f32_32x32x2_f32) or "fp16x3" (the conv layers with cin > 1 and the three Linear layers on v_mfma_f32_32x32x16_f16
    with hi + lo fp16 operands, three products per multiply, fp32 accumulation; layer 0, GELU, residuals and
    LayerNorm stay fp32)."""

    PRECISIONS = {"fp32": 0, "fp16x3": 3}

    def __init__(self, config, precision="fp32"):
        super().__init__()
        if precision not in self.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(self.PRECISIONS)}")
        self.precision = precision
        self.hidden_dim = config.embed_dim
        self.input_len = config.max_len
        self.output_len = config.N
        bias = not getattr(config, "dont_use_bias", False)
        self.use_bias = bias
        k, p = 7, 3
        h, e = self.hidden_dim // 2, self.hidden_dim
        self.kernel, self.padding = k, p
        self.layers1 = nn.Sequential(nn.Conv1d(1, h, k, padding=p, bias=bias), nn.GELU(),
                                     nn.Conv1d(h, h, k, padding=2 * p, dilation=2, bias=bias), nn.GELU())
        self.layers2 = nn.Sequential(nn.Conv1d(h, h, k, padding=4 * p, dilation=4, bias=bias), nn.GELU(),
                                     nn.Conv1d(h, h, k, padding=p, bias=bias), nn.GELU())
        self.layers3 = nn.Sequential(nn.Conv1d(h, h, k, padding=2 * p, dilation=2, bias=bias), nn.GELU(),
                                     nn.Conv1d(h, h, k, padding=4 * p, dilation=4, bias=bias), nn.GELU())
        self.layers4 = nn.Sequential(nn.Conv1d(h, h, k, padding=p, bias=bias), nn.GELU(),
                                     nn.Conv1d(h, h, k, padding=2 * p, dilation=2, bias=bias), nn.GELU())
        self.layers5 = nn.Sequential(nn.Conv1d(h, e, k, padding=4 * p, dilation=4, bias=bias), nn.GELU(),
                                     nn.Conv1d(e, e, k, padding=p, bias=bias), nn.GELU())
        n = self.output_len
        self.layersFin = nn.Sequential(nn.Linear(e * n, 4 * n), nn.GELU(), nn.Linear(4 * n, n), nn.GELU(),
                                       nn.Linear(n, n))
        self.layer_norm = nn.LayerNorm(n, eps=1e-6)
        self.dropout = nn.Dropout(getattr(config, "dropout", 0.0))
        self._handle = None
        self._hkey = None

    # ------------------------------------------------------------------ fused path
    def _packed(self) -> np.ndarray:
        parts = []
        convs = [self.layers1[0], self.layers1[2], self.layers2[0], self.layers2[2], self.layers3[0], self.layers3[2],
                 self.layers4[0], self.layers4[2], self.layers5[0], self.layers5[2]]
        for c in convs:
            parts.append(c.weight.detach().float().cpu().numpy().ravel())
            b = c.bias.detach().float().cpu().numpy() if c.bias is not None else np.zeros(c.out_channels, np.float32)
            parts.append(b.ravel())
        for li in (0, 2, 4):
            parts.append(self.layersFin[li].weight.detach().float().cpu().numpy().ravel())
            parts.append(self.layersFin[li].bias.detach().float().cpu().numpy().ravel())
        parts.append(self.layer_norm.weight.detach().float().cpu().numpy().ravel())
        parts.append(self.layer_norm.bias.detach().float().cpu().numpy().ravel())
        return np.ascontiguousarray(np.concatenate(parts), dtype=np.float32)

    def _get_handle(self, device):
        key = (str(device), self.precision, tuple(p._version for p in self.parameters()),
               tuple(p.data_ptr() for p in self.parameters()))
        if self._handle is None or self._hkey != key:
            W = self._packed()
            out = ctypes.c_void_p()
            L = _lib.load()
            with torch.cuda.device(device):
                _lib.check(L.npd_conv_create(int(self.output_len), int(self.hidden_dim), W.ctypes.data_as(ctypes.c_void_p),
                                             int(W.size), self.PRECISIONS[self.precision], ctypes.byref(out)),
                           "npd_conv_create")
            if self._handle is not None:
                L.npd_conv_destroy(self._handle)
            self._handle, self._hkey = out, key
        return self._handle

    def __del__(self):
        try:
            if self._handle is not None:
                _lib.load().npd_conv_destroy(self._handle)
        except Exception:
            pass

    def logits(self, noisy_enc: torch.Tensor, want_decisions=True, want_input4=False):
        if self.training:
            raise _lib.NpdError("the fused convNet path is inference-only (eval mode)")
        y = _lib.f32c(_lib.stage(noisy_enc, "noisy_enc"))
        B = y.shape[0]
        if y.shape[1] != self.output_len:
            raise ValueError("input length must equal config.N (= max_len)")
        h = self._get_handle(y.device)
        L = _lib.load()
        wsb = L.npd_conv_workspace_bytes(h, B)
        ws = torch.empty(max(int(wsb), 1), dtype=torch.uint8, device=y.device)
        lg = torch.empty(B, self.output_len, dtype=torch.float32, device=y.device)
        dec = torch.empty_like(lg) if want_decisions else None
        in4 = torch.empty(B, self.hidden_dim // 2, self.output_len, dtype=torch.float32, device=y.device) \
            if want_input4 else None
        _lib.check(L.npd_conv_forward_ex(h, _lib.ptr(y), _lib.ptr(lg), _lib.ptr(dec), _lib.ptr(in4), _lib.ptr(ws), B,
                                         _lib.stream_of(y.device)), "npd_conv_forward")
        if want_input4:
            return _lib.home(lg, noisy_enc), _lib.home(dec, noisy_enc), _lib.home(in4, noisy_enc)
        return _lib.home(lg, noisy_enc), _lib.home(dec, noisy_enc)

    def forward(self, noisy_enc, mask, trg_seq, device):
        """models.py:742-767: returns (output, decoded_msg_bits, out_mask, logits, input4), input4 being the
        (B, embed/2, N) activation after layers3 + residual, written out by the fused forward on request."""
        lg, dec, in4 = self.logits(noisy_enc, want_input4=True)
        logits = lg.unsqueeze(-1)
        out = torch.sigmoid(logits)
        return torch.cat((1 - out, out), -1), dec.unsqueeze(-1), mask, logits, in4

    def decode(self, noisy_enc, info_positions, mask, device, trg_seq=None):
        """models.py:769-772: (decoded_msg_bits (B,N,1), mask)."""
        _, dec = self.logits(noisy_enc)
        return dec.unsqueeze(-1), mask
