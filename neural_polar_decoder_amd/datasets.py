"""Standard test sets and trained checkpoints in the reference's on-disk formats.

Standard test sets (run_models.py:797-803, rnn_all.py:1299-1305, run_models.py:1422-1446):
``./data/polar/test/test_N{N}_K{K}.p`` and ``./data/pac/test/Scheme_{rp}/test_N{N}_K{K}_g{g}.p`` are
``torch.save`` dicts ``{'msg': (B,K), 'rec': {snr: (B,N)}, 'snr': [...]}``.  ``test_standard``
(run_models.py:495-551) decodes them in full batches of ``test_batch_size`` (a trailing partial batch
is dropped) and averages per-batch BER/BLER, which equals pooled counts over the batches used.

Checkpoints (rnn_all.py:1474-1615, run_models.py:980-1049) are ``{'net'|'xformer': state_dict, 'step',
'args': argparse.Namespace}``.  They are read with ``torch.load(weights_only=True)`` -- nothing in the
file is executed; ``argparse.Namespace`` is the one non-tensor class allow-listed.
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from .codes import pac_default_g, pac_info_positions, polar_info_positions


# ------------------------------------------------------------------------------------ test sets
def polar_test_path(N: int, K: int, root: str = "./data") -> str:
    return os.path.join(root, "polar", "test", f"test_N{N}_K{K}.p")


def pac_test_path(N: int, K: int, g: int = 91, rate_profile: str = "RM", root: str = "./data") -> str:
    return os.path.join(root, "pac", "test", f"Scheme_{rate_profile}", f"test_N{N}_K{K}_g{g}.p")


def load_standard(path: str):
    """-> (msg (B,K) fp32 CPU, rec {snr: (B,N)}, snrs list)."""
    d = torch.load(path, map_location="cpu", weights_only=True)
    rec = d["rec"]
    snrs = list(d["snr"]) if "snr" in d else list(rec.keys())
    return d["msg"], rec, snrs


def make_standard(code, snrs, B: int, seed: int = 1234, device=None):
    """A standard test set in the reference's format, drawn on the GPU (Philox streams: message of
    codeword b is the same at every SNR, as in the reference's generator)."""
    device = torch.device(device or "cuda")
    msg = None
    rec = {}
    for si, snr in enumerate(snrs):
        m, _, y = code.mc_generate(B, float(snr), seed, si, 0, device=device, want_msg=msg is None)
        if msg is None:
            msg = m.cpu()
        rec[snr] = y.cpu()
    return {"msg": msg, "rec": rec, "snr": list(snrs)}


def save_standard(path: str, data: dict) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    torch.save(data, path)


def evaluate_standard(code, msg, rec, test_batch_size: int, list_size=None, gru=None, device=None):
    """test_standard (run_models.py:495-551) for the decoders of this package: SC always, SC-List when
    ``list_size`` is given (polar.py:793), the CRISP GRU when ``gru=(net, RNN_decoder)``.  Returns
    {decoder: {'ber': [...], 'bler': [...]}} over the SNRs of ``rec`` (dict order)."""
    from .utils import count_errors
    device = torch.device(device or "cuda")
    msg = msg.to(device=device, dtype=torch.float32)
    nb = msg.shape[0] // int(test_batch_size)
    used = nb * int(test_batch_size)
    if used == 0:
        raise ValueError("test set smaller than one test batch")
    K = msg.shape[1]
    info = getattr(code, "info_positions", None)
    info = torch.as_tensor(np.asarray(info if info is not None else code.B), device=device)
    names = ["SC"] + (["SCL"] if list_size else []) + (["RNN"] if gru else [])
    out = {k: {"ber": [], "bler": []} for k in names}
    for snr, y_all in rec.items():
        y = y_all[:used].to(device=device, dtype=torch.float32).contiguous()
        m = msg[:used]
        cnt = {k: torch.zeros(2, dtype=torch.int64, device=device) for k in names}
        for b in range(nb):
            sl = slice(b * test_batch_size, (b + 1) * test_batch_size)
            yb, mb = y[sl], m[sl]
            if hasattr(code, "pac_sc_decode"):
                _, hat, _ = code.pac_sc_decode(yb, float(snr))
            else:
                hat = code.sc_decode_msg(yb, float(snr))
            count_errors(mb, hat, cnt["SC"])
            if list_size:
                _, h = code.scl_decode(yb, float(snr), int(list_size), want_llrs=False)
                count_errors(mb, h, cnt["SCL"])
            if gru:
                net, dec = gru
                d = dec.decode(net, False, yb)
                count_errors(mb, d.index_select(1, info), cnt["RNN"])
        for k in names:
            be, bl = cnt[k].cpu().tolist()
            out[k]["ber"].append(be / (used * K))
            out[k]["bler"].append(bl / used)
    return out


# ------------------------------------------------------------------------------------ checkpoints
def load_checkpoint(path: str) -> dict:
    """A reference checkpoint dict, loaded without executing anything from the file."""
    with torch.serialization.safe_globals([argparse.Namespace]):
        return torch.load(path, map_location="cpu", weights_only=True)


def code_from_args(args):
    """The code of a checkpoint's args (rnn_all.py:1015-1196 get_code; run_models.py's --code)."""
    from .pac_code import PAC
    from .polar import PolarCode
    kind = str(getattr(args, "code", "Polar")).lower()
    N, K = int(args.N), int(args.K)
    tK = getattr(args, "target_K", None)
    rp = getattr(args, "rate_profile", "polar")
    if kind == "pac":
        return PAC(argparse.Namespace(target_K=tK or K), N, K, int(getattr(args, "g", pac_default_g(N))), rate_profile=rp)
    info = polar_info_positions(N, K, rp, tK)
    return PolarCode(int(np.log2(N)), K, F=np.setdiff1d(np.arange(N), info))


def rnn_from_checkpoint(ckpt, device="cuda", precision="fp32"):
    """(net, RNN_decoder, code) of a CRISP checkpoint ({'net', 'args'}, rnn_all.py:1310-1330): decoding_type y_input
    without the y-MLP (the CRISP scripts) or with --use_ynn's (rnn_all.py:1319), or y_h0 with its y-MLP
    (rnn_all.py:1316-1317), GRU or LSTM cells."""
    from .rnn import RNN_Model, RNN_decoder
    if isinstance(ckpt, str):
        ckpt = load_checkpoint(ckpt)
    a = ckpt["args"]
    dtype = getattr(a, "decoding_type", "y_input")
    if dtype not in ("y_input", "y_h0"):
        raise NotImplementedError("fused decode supports decoding_type 'y_input' (with or without --use_ynn) and 'y_h0'")
    ynn = dtype == "y_input" and bool(getattr(a, "use_ynn", False))
    onehot = bool(getattr(a, "onehot", False))
    N = int(a.N)
    din = (N if dtype == "y_input" else 0) + 1 + int(onehot)
    # the reference's constructors (rnn_all.py:1316-1320): y_h0 builds out_linear_depth 1 whatever the flag says;
    # y_input (no --use_ynn) passes y_hidden_size only for an out_linear_depth > 1 head
    old = int(getattr(a, "out_linear_depth", 1)) if dtype == "y_input" else 1
    if dtype == "y_input" and not ynn:
        yh, yd = (int(getattr(a, "y_hidden_size", 128)) if old > 1 else 0), 0
    else:  # y_h0, or y_input --use_ynn (rnn_all.py:1319: the y-MLP with y_output_size = N)
        yh, yd = int(getattr(a, "y_hidden_size", 128)), int(getattr(a, "y_depth", 3))
    net = RNN_Model(getattr(a, "rnn_type", "GRU"), din, int(a.rnn_feature_size), 1, int(a.rnn_depth), N,
                    yh, yd, getattr(a, "activation", "selu"), float(getattr(a, "dropout", 0.0)),
                    bool(getattr(a, "use_skip", False)), out_linear_depth=old, y_output_size=N if ynn else None,
                    bidirectional=bool(getattr(a, "bidirectional", False)),
                    use_layernorm=bool(getattr(a, "use_layernorm", False))).to(device)
    net.load_state_dict(ckpt["net"])
    net.eval()
    code = code_from_args(a)
    info = getattr(code, "info_positions", None)
    info = np.asarray(info if info is not None else code.B)
    dec = RNN_decoder(dtype, N, info, onehot=onehot, reverse_order=bool(getattr(a, "reverse_order", False)),
                      precision=precision)
    return net, dec, code


def convnet_from_checkpoint(ckpt, device="cuda"):
    """convNet of a run_models.py checkpoint ({'xformer', 'args'} with --model conv, run_models.py:723)."""
    from .models import convNet
    if isinstance(ckpt, str):
        ckpt = load_checkpoint(ckpt)
    a = ckpt["args"]
    if getattr(a, "model", "conv") != "conv":
        raise NotImplementedError(f"model {a.model!r}: only the convNet decoder is built")
    net = convNet(a)
    net.load_state_dict(ckpt["xformer"])
    return net.to(device).eval()


__all__ = ["polar_test_path", "pac_test_path", "load_standard", "make_standard", "save_standard",
           "evaluate_standard", "load_checkpoint", "code_from_args", "rnn_from_checkpoint", "convnet_from_checkpoint"]
