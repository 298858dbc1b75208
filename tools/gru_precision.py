#!/usr/bin/env python3
"""GRU precision study (round 4): logit error of every implementation of the CRISP decode against
a float64 restatement (oracle.gru_decode_f64), on a trained net.

    python tools/gru_precision.py [--fixture trained_crisp_64_32] [--n 65536] [--snrs 0 2 4] [--out FILE]

Implementations:
  * "reference"  -- the reference's arithmetic: RNN_decoder.decode's y_input test loop (rnn_all.py:532-547) run
                    with torch fp32 on the CPU, one nn.GRU call per step (this package's RNN_Model holds the same
                    modules as rnn_all.RNN_Model, so the ATen calls are the reference's);
  * "fp32"       -- the HIP kernel the bench times (gru_decode_kernel, v_mfma_f32_32x32x2_f32);
  * "fp16x3"     -- the split fp16 kernel (gru16p_kernel, hi + lo fp16, three products);
  * "bf16x3"     -- the split bf16 kernel (for scale).
Each implementation decodes autoregressively; its logits are compared step for step with the float64 logits of
the SAME decision path (oracle teacher-forced along it), over the information steps.  Decision flips are counted
against the float64 decoder's own autoregressive decisions.  Words: Philox AWGN words (npd_mc_generate).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model  # noqa: E402
from oracle import oracle as O  # noqa: E402

PCT = [50.0, 99.0, 99.9, 100.0]


def reference_loop(net, y, N, info):
    """rnn_all.py:532-547 (y_input, onehot, test branch) on the CPU in torch fp32 -> (decisions, logits by step)."""
    B = y.shape[0]
    isinfo = np.zeros(N, bool)
    isinfo[info] = True
    dec = torch.ones(B, N)
    lg = torch.empty(B, N)
    hidden = torch.zeros(net.num_rnn_layers, B, net.feature_size)
    eye = torch.eye(2)
    with torch.no_grad():
        for ii in range(N):
            prev = torch.ones(B) if ii == 0 else dec[:, ii - 1].sign()
            oh = eye[(0.5 + 0.5 * prev).long()].reshape(B, -1)
            out, hidden = net(torch.cat([y.unsqueeze(1), oh.view(-1, 1, 2)], 2), hidden)
            lg[:, ii] = out.squeeze()
            if isinfo[ii]:
                dec[:, ii] = out.squeeze().sign()
    return dec.numpy(), lg.numpy()


def stats(err, flips_cw, flips_bits):
    q = np.percentile(err, PCT)
    return {"p50": float(q[0]), "p99": float(q[1]), "p99.9": float(q[2]), "max": float(q[3]),
            "mean": float(err.mean()), "cw_flips": int(flips_cw), "bit_flips": int(flips_bits)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="trained_crisp_64_32")
    ap.add_argument("--n", type=int, default=1 << 16)
    ap.add_argument("--snrs", type=float, nargs="*", default=[0.0, 2.0, 4.0])
    ap.add_argument("--impls", nargs="*", default=["reference", "fp32", "fp16x3", "bf16x3"])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    d = np.load(os.path.join(ROOT, "tests", "golden", args.fixture + ".npz"))
    N, K, F, L = int(d["N"]), int(d["K"]), int(d["F"]), int(d["layers"])
    info = np.asarray(d["info"], np.int64)
    sd = {k[2:]: np.asarray(d[k]) for k in d.files if k.startswith("w.")}
    net = RNN_Model("GRU", N + 2, F, 1, L, N, 0, 0).eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gnet = RNN_Model("GRU", N + 2, F, 1, L, N, 0, 0).cuda().eval()
    gnet.load_state_dict(net.state_dict())
    code = reference_polar_code(N, K)
    assert np.array_equal(np.asarray(code.info_positions), info)
    res = {"fixture": args.fixture, "n_per_snr": args.n, "snrs": args.snrs, "impls": {}}
    errs = {k: [] for k in args.impls}
    flips = {k: [0, 0] for k in args.impls}
    for si, s in enumerate(args.snrs):
        _, _, y = code.mc_generate(args.n, s, seed=4242, snr_index=si, device="cuda", want_msg=False)
        yc = y.cpu()
        d64, _ = O.gru_decode_f64(yc.numpy(), sd, N, F, L, info)
        for impl in args.impls:
            t0 = time.time()
            if impl == "reference":
                dec, lg = reference_loop(net, yc, N, info)
            else:
                dd = RNN_decoder("y_input", N, info, onehot=True, precision=impl)
                dec, lg = dd.decode(gnet, False, y, return_logits=True)
                dec, lg = dec.cpu().numpy(), lg.cpu().numpy()
            _, l64 = O.gru_decode_f64(yc.numpy(), sd, N, F, L, info, path=dec)
            errs[impl].append(np.abs(lg[:, info].astype(np.float64) - l64[:, info]).ravel())
            diff = dec[:, info] != d64[:, info]
            flips[impl][0] += int(diff.any(1).sum())
            flips[impl][1] += int(diff.sum())
            print(f"{s:g} dB {impl:9s} max |dlogit| {errs[impl][-1].max():.3e}  cw flips {int(diff.any(1).sum())}"
                  f"  ({time.time() - t0:.1f} s)", flush=True)
    for impl in args.impls:
        res["impls"][impl] = stats(np.concatenate(errs[impl]), *flips[impl])
    res["words"] = args.n * len(args.snrs)
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
