"""CRISP GRU decoder -- drop-in for rnn_all.RNN_Model / RNN_decoder (rnn_all.py:294-561).

``RNN_Model`` keeps the reference's constructor and parameter names (``rnn.weight_ih_l0`` ...,
``linear.weight``) so reference state dicts / checkpoints load unchanged; it is the weight container
(its ``forward`` is the reference's single-step training API, plain PyTorch).  The decode hot path,
``RNN_decoder.decode(net, False, y, ...)`` (rnn_all.py:532-547), runs the whole N-step
autoregressive loop in one fused HIP kernel (npd_gru_decode; fp32 MFMA).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from . import _lib


class RNN_Model(nn.Module):
    """Same parameters as the reference (rnn_all.py:294-385).  The fused decoder accepts nets with output_size 1,
    out_linear_depth 1, 1 or 2 layers, GRU or LSTM cells (rnn_all.py:69) at hidden 32, 64, 128, 256 or
    512 -- a bidirectional net (rnn_all.py:307) runs as the one-directional cell of hidden 2F, so its packed width 2F
    must be one of those -- with decoding_type 'y_input' -- y_depth 0 (the CRISP scripts, rnn_all.py:250-253) or
    --use_ynn's y-MLP of N outputs feeding the cell in place of y (rnn_all.py:1319-1320, :533-536) -- or 'y_h0' (the
    argparse default, rnn_all.py:73) with its y-MLP (y_linears, with or without skip; LSTM: (h, c) both start from
    it).  LSTM cells run fp32; the split precisions (fp16x3, bf16x3, bf16) cover GRUs of packed hidden <= 64, and
    y_h0 in a split precision needs the 16-codeword kernel (hidden 64, 2 layers, N % 32 == 0).  fused_supported(...,
    precision, N) mirrors these limits and npd_rnn_create's LDS bound for hidden 512 x 2 layers.  --use_layernorm nets
    (LayerNorm(F) before the output Linear, rnn_all.py:317-320, :387-398) run on the fp32 GRU kernel at hidden 32 / 64
    (npd_rnn_create_ex); so do --out_linear_depth > 1 heads (Linear(F, H), SELU, ..., Linear(H, 1) with H = y_hidden_size
    <= 128, rnn_all.py:336-343; each head layer an fp32 MFMA GEMM per decoding step)."""

    def __init__(self, rnn_type, input_size, feature_size, output_size, num_rnn_layers, y_size, y_hidden_size,
                 y_depth, activation="relu", dropout=0., skip=False, out_linear_depth=1, y_output_size=None,
                 bidirectional=False, use_layernorm=False):
        super().__init__()
        assert rnn_type in ["GRU", "LSTM"]
        self.rnn_type = rnn_type
        self.input_size = input_size
        self.feature_size = feature_size
        self.output_size = output_size
        self.num_rnn_layers = num_rnn_layers
        self.bidirectional = bidirectional
        self.y_size = y_size
        self.y_hidden_size = y_hidden_size
        self.y_depth = y_depth
        self.out_linear_depth = out_linear_depth
        self.activation = activation
        self.skip = skip
        self.rnn = getattr(nn, rnn_type)(input_size, feature_size, num_rnn_layers, bidirectional=bidirectional,
                                         batch_first=True)
        self.y_output_size = ((int(bidirectional) + 1) * num_rnn_layers * feature_size if y_output_size is None
                              else y_output_size)
        if y_hidden_size > 0 and y_depth > 0:  # rnn_all.py:323-329, same module order and names
            self.y_linears = nn.ModuleList([nn.Linear(y_size, y_hidden_size, bias=True)])
            self.y_linears.extend([nn.Linear(y_hidden_size, y_hidden_size, bias=True) for _ in range(1, y_depth - 1)])
            self.y_linears.append(nn.Linear(y_hidden_size, self.y_output_size - (y_size if skip else 0), bias=True))
        self.drop = nn.Dropout(dropout)
        self.layernorm = nn.LayerNorm(feature_size) if use_layernorm else nn.Identity()
        if out_linear_depth == 1:
            self.linear = nn.Linear((int(bidirectional) + 1) * feature_size, output_size)
        else:
            layers = [nn.Linear((int(bidirectional) + 1) * feature_size, y_hidden_size)]
            for _ in range(1, out_linear_depth - 1):
                layers += [nn.SELU(), nn.Linear(y_hidden_size, y_hidden_size)]
            layers += [nn.SELU(), nn.Linear(y_hidden_size, output_size)]
            self.linear = nn.Sequential(*layers)

    ACTS = {"linear": 0, "relu": 1, "selu": 2, "elu": 3, "tanh": 4, "sigmoid": 5}

    def act(self, inputs):
        """rnn_all.py:346-360 (an unknown name is the identity)."""
        import torch.nn.functional as Fn
        fn = {"tanh": torch.tanh, "elu": Fn.elu, "relu": Fn.relu, "selu": Fn.selu, "sigmoid": torch.sigmoid}
        return fn.get(self.activation, lambda x: x)(inputs)

    def get_h0(self, y):
        """rnn_all.py:362-375 in PyTorch, reference semantics: layer ii is followed by act iff ii != y_depth (every
        layer, the last included, for y_depth >= 2; all but the last for y_depth = 1).  The fused decoder runs this
        MLP on npd_ymlp_layer instead."""
        x = y.clone()
        for ii, layer in enumerate(self.y_linears):
            x = layer(x) if ii == self.y_depth else self.act(layer(x))
        if self.skip:
            x = torch.cat([y, x], 1)
        x = x.reshape(-1, self.feature_size, (int(self.bidirectional) + 1) * self.num_rnn_layers).permute(2, 0, 1)
        x = x.contiguous()
        return x if self.rnn_type == "GRU" else (x, x)

    def get_Fy(self, y):
        """rnn_all.py:377-383 in PyTorch (--use_ynn): the y-MLP with get_h0's activation rule, no reshape.  The fused
        decoder runs it on npd_ymlp_layer."""
        x = y.clone()
        for ii, layer in enumerate(self.y_linears):
            x = layer(x) if ii == self.y_depth else self.act(layer(x))
        return x

    def _ymlp_ok(self, out_size, allow_skip=False):
        # skip (get_h0 only, rnn_all.py:369-370): the MLP's y_output_size - y_size outputs follow y itself
        return (hasattr(self, "y_linears") and (allow_skip or not self.skip) and self.activation in self.ACTS
                and self.y_output_size == out_size)

    def forward(self, input, hidden, Fy=None):
        """Single recurrent step (rnn_all.py:387-398) -- the training-time API."""
        out, hidden = self.rnn(input, hidden)
        out = self.layernorm(self.drop(out))
        decoded = self.linear(out if Fy is None else torch.cat([Fy, out], -1))
        return decoded.view(-1, self.output_size), hidden

    def fused_supported(self, decoding_type="y_input", precision="fp32", N=None) -> bool:
        """True when npd_rnn_create / npd_gru_decode_ex accept this net for `decoding_type` at `precision` (and code
        length N when given): the same limits, checked before any handle is built."""
        fe = self.feature_size * (2 if self.bidirectional else 1)  # a bidirectional net runs as the 2F cell
        # LayerNorm head: the fp32 GRU kernel (npd_rnn_create_ex), hidden 32 / 64, unidirectional
        ln_ok = isinstance(self.layernorm, nn.Identity) or (
            isinstance(self.layernorm, nn.LayerNorm) and self.rnn_type == "GRU" and not self.bidirectional
            and fe in (32, 64) and precision == "fp32" and self.out_linear_depth == 1)
        # out_linear_depth > 1 head: the fp32 GRU kernel, packed hidden 32 / 64, head width y_hidden_size <= 128
        head_ok = self.out_linear_depth == 1 or (
            2 <= self.out_linear_depth <= 8 and self.rnn_type == "GRU" and fe in (32, 64) and precision == "fp32"
            and 1 <= self.y_hidden_size <= 128)
        common = self.output_size == 1 and head_ok and ln_ok and self.num_rnn_layers in (1, 2)
        if N is not None:
            # npd_gru_create: N a multiple of 8 in [8, 256]; the weight-streaming kernels hold both layers' states and
            # the tile's y in LDS (gru::wide_lds_bytes), so hidden 512 x 2 layers needs N <= 128
            nw = min(fe // 32, 8)
            if not (8 <= N <= 256 and N % 8 == 0):
                return False
            if fe > 64 and (self.num_rnn_layers * fe * 32 + N * 32 + nw * 32) * 4 > 160 * 1024:
                return False
        if precision != "fp32":
            # LSTM cells are fp32 only; the split kernels cover packed hidden <= 64 and need N % 16 == 0; an initial
            # state (y_h0) in a split precision runs only on the 16-codeword kernel (hidden 64, 2 layers, N % 32 == 0)
            if self.rnn_type == "LSTM" or fe > 64:
                return False
            if N is not None and N % 16:
                return False
            if decoding_type == "y_h0" and not (fe == 64 and self.num_rnn_layers == 2 and (N is None or N % 32 == 0)):
                return False
        if self.rnn_type == "LSTM":  # fp32: lstm_decode_kernel (F 32, F 64 x 1 layer), lstm_wide_kernel (the rest)
            shape = fe in (32, 64, 128, 256, 512)
            if decoding_type == "y_h0":  # (h, c) both start from get_h0's x (rnn_all.py:370-375)
                return common and shape and self._ymlp_ok(self.num_rnn_layers * fe, allow_skip=True)
            return common and shape and decoding_type == "y_input" and (self.y_depth == 0 or self._ymlp_ok(self.y_size))
        base = common and self.rnn_type == "GRU" and fe in (32, 64, 128, 256, 512)
        if decoding_type == "y_h0":
            return base and self._ymlp_ok(self.num_rnn_layers * fe, allow_skip=True)
        # y_input: y itself (y_depth 0) or --use_ynn's Fy = get_Fy(y) with N outputs (rnn_all.py:533-536)
        return base and (self.y_depth == 0 or self._ymlp_ok(self.y_size))


def pack_gru_weights(net: nn.Module, layers: int, y_cols: int = 0) -> np.ndarray:
    """Flatten the state dict in the order of include/npd.h npd_gru_create; y_cols > 0 ('y_h0'): weight_ih_l0 gets
    y_cols zero columns in front (the y_input layout with no y).

    A bidirectional net (--bidirectional: nn.GRU / nn.LSTM over the one-step sequence, rnn_all.py:307) is packed as the
    one-directional cell of hidden 2F it is on that sequence: unit dir F + f of the packed cell is unit f of direction
    dir, so per gate the forward rows come first, then the reverse ones; both directions read the same layer input
    (layer 0: [y, bit]; layer l > 0: the previous layer's [h_fwd, h_rev] = the packed state); W_hh is block-diagonal
    (each direction's recurrence sees only its own state -- the zero blocks add exact zeros); linear.weight already
    runs over [h_fwd, h_rev] (rnn_all.py:335)."""
    sd = {k: v.detach().float().cpu().numpy() for k, v in net.state_dict().items()}
    F = net.feature_size
    G = 4 if net.rnn_type == "LSTM" else 3
    parts = []
    for l in range(layers):
        for nm in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
            w = sd[f"rnn.{nm}_l{l}"]
            if net.bidirectional:
                wr = sd[f"rnn.{nm}_l{l}_reverse"]
                if nm == "weight_hh":  # block-diagonal: (G 2F, 2F)
                    z = np.zeros((G, F, F), np.float32)
                    fw = np.concatenate([w.reshape(G, F, F), z], 2)
                    rv = np.concatenate([z, wr.reshape(G, F, F)], 2)
                else:  # rows of each gate: forward then reverse
                    fw, rv = w.reshape(G, F, -1), wr.reshape(G, F, -1)
                w = np.concatenate([fw, rv], 1).reshape(2 * G * F, -1).squeeze(-1) if w.ndim == 1 else \
                    np.concatenate([fw, rv], 1).reshape(2 * G * F, -1)
            if nm == "weight_ih" and l == 0 and y_cols:
                w = np.concatenate([np.zeros((w.shape[0], y_cols), np.float32), w], 1)
            parts.append(w.ravel())
    if net.out_linear_depth == 1:
        parts.append(sd["linear.weight"].ravel())
        parts.append(sd["linear.bias"].ravel())
    else:  # the Linear(F, 1) slot of npd_gru_create's layout is unused: the head goes to npd_rnn_create_ex
        parts.append(np.zeros((2 if net.bidirectional else 1) * F + 1, np.float32))
    return np.ascontiguousarray(np.concatenate(parts), dtype=np.float32)


def pack_head_weights(net: nn.Module) -> np.ndarray:
    """The out_linear_depth > 1 head (rnn_all.py:336-343: Sequential(Linear, SELU, ..., Linear)) flattened for
    npd_rnn_create_ex: each Linear's weight then bias, in order."""
    lins = [m for m in net.linear if isinstance(m, nn.Linear)]
    return np.ascontiguousarray(np.concatenate([np.concatenate([m.weight.detach().float().cpu().numpy().ravel(),
                                                                m.bias.detach().float().cpu().numpy().ravel()])
                                                for m in lins]), dtype=np.float32)


class _GruHandle:
    def __init__(self, N, F, layers, onehot, W: np.ndarray, precision=0, cell=0, ln=None, head=None):
        L = _lib.load()
        out = ctypes.c_void_p()
        if head is not None:  # (depth, hidden, weights) of an out_linear_depth > 1 head
            d, hid, hw = head
            _lib.check(L.npd_rnn_create_ex(int(cell), int(N), int(F), int(layers), 1 if onehot else 0,
                                           W.ctypes.data_as(ctypes.c_void_p), int(W.size), int(precision), None, None,
                                           0.0, int(d), int(hid), hw.ctypes.data_as(ctypes.c_void_p), int(hw.size),
                                           ctypes.byref(out)), "npd_rnn_create_ex")
        elif ln is None:
            _lib.check(L.npd_rnn_create(int(cell), int(N), int(F), int(layers), 1 if onehot else 0,
                                        W.ctypes.data_as(ctypes.c_void_p), int(W.size), int(precision),
                                        ctypes.byref(out)), "npd_rnn_create")
        else:  # (gamma, beta, eps) of the --use_layernorm head
            g, b, eps = ln
            _lib.check(L.npd_rnn_create_ex(int(cell), int(N), int(F), int(layers), 1 if onehot else 0,
                                           W.ctypes.data_as(ctypes.c_void_p), int(W.size), int(precision),
                                           g.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p),
                                           float(eps), 1, 0, None, 0, ctypes.byref(out)), "npd_rnn_create_ex")
        self.h = out

    def __del__(self):
        try:
            if self.h:
                _lib.load().npd_gru_destroy(self.h)
        except Exception:
            pass


class RNN_decoder:
    """rnn_all.RNN_decoder (rnn_all.py:400-561): eval (``train=False``) decoding for decoding_type
    'y_input' runs fused on the GPU.

    ``precision`` (keyword, not in the reference): "fp32" (default; the reference's arithmetic),
    "fp16x3" (hi + lo fp16 split on the fp16 MFMA: three products per multiply, fp32 accumulation; F = 64 with 2
    layers and N % 32 == 0 runs the unscaled split, whose lo parts of weights / states below 2^-14 are fp16
    subnormals (absolute resolution 2^-24); other shapes scale operands by 2^8 first; held to the fp32 path's
    tolerance, tests/test_gru_gpu.py), "bf16x3" (split-bf16, ~2^-16 relative per
    product) or "bf16" (plain bf16 MFMA, fp32 accumulation).  The split paths cover hidden sizes <= 64."""

    PRECISIONS = {"fp32": 0, "bf16x3": 1, "bf16": 2, "fp16x3": 3}

    def __init__(self, decoding_type, N, info_inds, onehot=False, reverse_order=False, precision="fp32"):
        if precision not in self.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(self.PRECISIONS)}")
        self.precision = precision
        self.decoding_type = decoding_type
        self.N = N
        self.info_inds = info_inds
        self.onehot = onehot
        self.reverse_order = reverse_order
        self._cache = {}

    def _handle(self, net: RNN_Model, device):
        # re-pack when the weights change (parameter versions) or the device differs
        key = (id(net), str(device), self.precision, self.decoding_type, tuple(p._version for p in net.parameters()),
               tuple(p.data_ptr() for p in net.parameters()))
        h = self._cache.get(key)
        if h is None:
            self._cache.clear()
            W = pack_gru_weights(net, net.num_rnn_layers, self.N if self.decoding_type == "y_h0" else 0)
            ln = None
            if isinstance(net.layernorm, nn.LayerNorm):
                ln = (np.ascontiguousarray(net.layernorm.weight.detach().float().cpu().numpy()),
                      np.ascontiguousarray(net.layernorm.bias.detach().float().cpu().numpy()), net.layernorm.eps)
            head = None
            if net.out_linear_depth > 1:
                head = (net.out_linear_depth, net.y_hidden_size, pack_head_weights(net))
            with torch.cuda.device(device):
                h = _GruHandle(self.N, net.feature_size * (2 if net.bidirectional else 1), net.num_rnn_layers, self.onehot, W,
                               self.PRECISIONS[self.precision], 1 if net.rnn_type == "LSTM" else 0, ln, head)
            self._cache[key] = h
        return h

    def decode(self, net, train, y, gt=None, teacher_forcing_ratio=0., loss_inds=None, return_logits=False):
        if train:
            raise _lib.NpdError("RNN_decoder.decode(train=True) is the training path (out of scope for the fused "
                                "decoder); use the reference's PyTorch loop for training")
        if self.decoding_type not in ("y_input", "y_h0"):
            raise _lib.NpdError(f"fused decode supports decoding_type 'y_input' and 'y_h0', got {self.decoding_type!r}"
                                " ('y_h0_out' builds a (1 + depth) F y-MLP that get_h0 cannot reshape, rnn_all.py:1324)")
        if not (hasattr(net, "fused_supported") and net.fused_supported(self.decoding_type, self.precision, self.N)):
            raise _lib.NpdError("network configuration not supported by the fused GRU decoder")
        din = (self.N if self.decoding_type == "y_input" else 0) + 1 + int(self.onehot)
        if net.input_size != din:
            raise ValueError(f"net.input_size must be {'N + ' if self.decoding_type == 'y_input' else ''}1 + onehot")
        y_in = y
        y = _lib.f32c(_lib.stage(y, "y"))
        if self.decoding_type == "y_input" and net.y_depth > 0:
            y = _ymlp_forward(net, y)  # --use_ynn: Fy = net.get_Fy(y) replaces y as the GRU input (rnn_all.py:533-536)
        B = y.shape[0]
        if loss_inds is None:
            loss_inds = self.info_inds
        is_info = np.zeros(self.N, np.uint8)
        is_info[np.asarray(loss_inds, np.int64)] = 1
        h = self._handle(net, y.device)
        dec = torch.empty(B, self.N, dtype=torch.float32, device=y.device)
        logits = torch.empty(B, self.N, dtype=torch.float32, device=y.device) if return_logits else None
        g = None if gt is None else _lib.f32c(_lib.stage(gt, "gt", y.device))
        h0 = self._h0(net, y) if self.decoding_type == "y_h0" else None
        _lib.check(_lib.load().npd_gru_decode_ex(h.h, None if h0 is not None else _lib.ptr(y), _lib.ptr(h0),
                                                 is_info.ctypes.data_as(ctypes.c_void_p),
                                                 1 if self.reverse_order else 0, _lib.ptr(g), _lib.ptr(dec),
                                                 _lib.ptr(logits), B, _lib.stream_of(y.device)), "npd_gru_decode")
        dec = _lib.home(dec, y_in)
        return (dec, _lib.home(logits, y_in)) if return_logits else dec

    def decode_count_sweep(self, net, y, msg, counters, cols=None, decoded=None):
        """The eval loop's GRU half over an SNR sweep (rnn_all.py:853-880): y (n_snr, B, N) on the GPU, msg (B, K) the
        messages of the B codewords (every segment's), counters (n_snr, 2) += [bit errors, block errors] of
        decode(net, False, y[s])[:, cols] against msg (cols defaults to the information set) -- npd_gru_decode_count_sweep:
        ONE launch for the sweep on the 16-codeword split kernel (hidden 64, 2 layers, fp16x3 / bf16x3 / bf16), else a
        decode + count per segment into `decoded` (n_snr, B, N), allocated here when not given.  y_input decoding."""
        if self.decoding_type != "y_input" or net.y_depth > 0:
            raise _lib.NpdError("decode_count_sweep covers y_input decoding without the y-MLP")
        if not (hasattr(net, "fused_supported") and net.fused_supported("y_input", self.precision, self.N)):
            raise _lib.NpdError("network configuration not supported by the fused GRU decoder")
        _lib.require_gpu(y, "y")
        if y.dim() != 3 or y.shape[2] != self.N:
            raise ValueError(f"y must be (n_snr, B, {self.N}), got {tuple(y.shape)}")
        n, B = y.shape[0], y.shape[1]
        c = np.ascontiguousarray(np.asarray(self.info_inds if cols is None else cols, np.int64).reshape(-1), np.int32)
        msg = _lib.f32c(_lib.stage(msg, "msg", y.device))
        if msg.shape != (B, c.size):
            raise ValueError(f"msg must be ({B}, {c.size}), got {tuple(msg.shape)}")
        _lib.check_out(counters, "counters", torch.int64, 2 * n, y.device)
        is_info = np.zeros(self.N, np.uint8)
        is_info[np.asarray(self.info_inds, np.int64)] = 1
        h = self._handle(net, y.device)
        y = _lib.f32c(y)
        # the 16-codeword split kernel's handles (npd_gru_create: split precision, packed hidden 64, 2 layers, N % 32 == 0;
        # a bidirectional hidden-32 net is such a cell) decode and count in one launch without `decoded`
        fused = (self.precision != "fp32" and net.rnn_type == "GRU" and net.num_rnn_layers == 2 and self.N % 32 == 0
                 and net.feature_size * (2 if net.bidirectional else 1) == 64)
        if decoded is None and not fused:
            decoded = torch.empty(n, B, self.N, dtype=torch.float32, device=y.device)
        _lib.check_out(decoded, "decoded", torch.float32, n * B * self.N, y.device, optional=True)
        _lib.check(_lib.load().npd_gru_decode_count_sweep(h.h, n, _lib.ptr(y), is_info.ctypes.data_as(ctypes.c_void_p),
                                                          1 if self.reverse_order else 0, _lib.ptr(msg), int(c.size),
                                                          c.ctypes.data_as(ctypes.c_void_p), _lib.ptr(decoded), B,
                                                          _lib.ptr(counters), _lib.stream_of(y.device)),
                   "npd_gru_decode_count_sweep")
        return counters

    def _h0(self, net, y):
        """(B, F * layers) initial states: get_h0's MLP (y first when the net was built with skip, rnn_all.py:369-370),
        kept alive past the stream-ordered decode by the caller."""
        x = _ymlp_forward(net, y)
        x = torch.cat([y, x], 1).contiguous() if net.skip else x
        if net.bidirectional:  # get_h0's state (l, dir) of unit f is x[f 2L + 2l + dir]; the 2F cell wants (dir F + f) L + l
            B, F, L = x.shape[0], net.feature_size, net.num_rnn_layers
            x = x.view(B, F, L, 2).permute(0, 3, 1, 2).contiguous().view(B, 2 * F * L)
        return x


def _ymlp_forward(net: RNN_Model, y: torch.Tensor) -> torch.Tensor:
    """The y-MLP (rnn_all.py:362-383: get_h0 / get_Fy) on npd_ymlp_layer: (B, N) -> (B, y_output_size), layer ii followed
    by the activation iff ii != y_depth.  y_h0: x before get_h0's reshape (element f * layers + l = layer l's initial
    state of unit f); --use_ynn: Fy."""
    L = _lib.load()
    x = y
    step = 65535 * 64
    for ii, layer in enumerate(net.y_linears):
        act = 0 if ii == net.y_depth else RNN_Model.ACTS[net.activation]
        W = _lib.f32c(layer.weight.detach().to(y.device))
        b = _lib.f32c(layer.bias.detach().to(y.device))
        out = torch.empty(y.shape[0], W.shape[0], dtype=torch.float32, device=y.device)
        for s0 in range(0, y.shape[0], step):
            xs, os_ = x[s0:s0 + step], out[s0:s0 + step]
            _lib.check(L.npd_ymlp_layer(_lib.ptr(xs), _lib.ptr(W), _lib.ptr(b), _lib.ptr(os_), xs.shape[0],
                                        W.shape[1], W.shape[0], act, _lib.stream_of(y.device)), "npd_ymlp_layer")
        x = out
    return x


def get_onehot(actions):
    """rnn_all.py:258-260."""
    inds = (0.5 + 0.5 * actions).long()
    return torch.eye(2, device=inds.device)[inds].reshape(actions.shape[0], -1)
