#!/usr/bin/env python3
"""GPU stages of the conv-model curriculum behind tests/golden/trained_conv_64_22_e128.npz (test infrastructure, not
product code): run_alt.sh's own configuration -- Polar(64,22), rate profile 'polar' with the n2c curriculum, embed 128,
batch 8192, AdamW 1e-3, the dec_train_snr ramp -6 -> 0 dB -- with shortened stages (run_alt.sh: 1000 steps at K = 1..7,
5000 at K = 8..21, 150000 at K = 22).  The reference's run_models.py costs minutes per step on this container's CPUs at
embed 128 / batch 8192, so the loop is restated here on one MI355X; tests/golden/gen_trained_conv.py then evaluates the
final weights with the reference's own convNet (decisions, logits, Monte-Carlo curve).  Nothing here imports the
reference (it runs on the GPU box).

Restatement of run_models.py's training loop (run_models.py:760-1000) for --model conv, --loss MSE (defaults: no
lr scheduler, no range training, --mult 1, --clip 0.25, --dropout 0.1):
  * stage K of n2c (run_models.py:666-669): info = sort(flip(rs_N[:target_K])[:K]) -- the K least reliable positions
    of the target information set; rs_N the run_models.py:630 reliability sequence below N;
  * per step: msg = 1 - 2 (rand < 0.5) (B, K); gt = ones (B, N), gt[:, info] = msg; y = encode_plotkin(msg,
    custom_info_positions = info) + sigma(snr_K) randn;
  * convNet.forward (models.py:691-767) in training mode: the 10 dilated Conv1d + GELU layers with the three residual
    blocks, flatten, Linear-GELU-Linear-GELU-Linear, Dropout(0.1), LayerNorm(N, eps 1e-6); each Conv1d is computed as
    one (B N, 7 Cin) x (7 Cin, Cout) GEMM over the im2col of its 7 dilated taps (the same function as nn.Conv1d;
    MIOpen's conv1d measured 3x slower here);
  * loss = MSE(logits[:, info], gt[:, info]) (out_mask is all ones, run_models.py:874-876); backward;
    clip_grad_norm_(0.25); AdamW.step(); zero_grad(); a fresh AdamW per stage (each stage is one run_models.py
    invocation, --load_previous chaining the weights, run_models.py:730-740).

    python tests/golden/train_conv_gpu.py --state S.pt --out W.pt [--budget-s 1000]   (resumable, as train_crisp_gpu.py)
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from neural_polar_decoder_amd.codes import polar_rs  # noqa: E402
from neural_polar_decoder_amd.utils import snr_db2sigma  # noqa: E402

# run_alt.sh's dec_train_snr per K (n2c, target 22)
SNR_OF_K = {1: -6, 2: -6, 3: -5, 4: -5, 5: -4, 6: -4, 7: -4, 8: -4, 9: -3, 10: -3, 11: -2, 12: -2, 13: -1, 14: -1,
            15: -1, 16: -1, 17: 0, 18: 0, 19: 0, 20: 0, 21: 0, 22: 0}
CASE = dict(name="trained_conv_64_22_e128", N=64, K=22, embed=128, batch=8192, lr=1e-3, seed_init=6422128,
            curriculum=[(k, 600 if k <= 7 else 1200, SNR_OF_K[k]) for k in range(1, 22)] + [(22, 24000, 0)])

# (layer, cin, cout, dilation) of convNet's ten Conv1d in forward order (models.py:701-735); halves = embed / 2
def conv_shapes(E):
    h = E // 2
    return [("layers1.0", 1, h, 1), ("layers1.2", h, h, 2), ("layers2.0", h, h, 4), ("layers2.2", h, h, 1),
            ("layers3.0", h, h, 2), ("layers3.2", h, h, 4), ("layers4.0", h, h, 1), ("layers4.2", h, h, 2),
            ("layers5.0", h, E, 4), ("layers5.2", E, E, 1)]


class ConvNetT(nn.Module):
    """convNet's parameters under the reference's names (state dicts interchange) with a GEMM-form forward."""

    def __init__(self, E, N):
        super().__init__()
        self.E, self.N = E, N
        for name, cin, cout, dil in conv_shapes(E):
            seq, idx = name.split(".")
            if not hasattr(self, seq):
                setattr(self, seq, nn.ModuleDict())
            getattr(self, seq)[idx] = nn.Conv1d(cin, cout, 7, padding=3 * dil, dilation=dil)
        self.layersFin = nn.ModuleDict({"0": nn.Linear(E * N, 4 * N), "2": nn.Linear(4 * N, N), "4": nn.Linear(N, N)})
        self.layer_norm = nn.LayerNorm(N, eps=1e-6)

    def conv(self, x, name, dil):
        """x (B, N, Cin) -> (B, N, Cout): sum over taps t of x[:, l + dil (t - 3)] W[:, :, t]^T, zero-padded."""
        seq, idx = name.split(".")
        m = getattr(self, seq)[idx]
        p = 3 * dil
        xp = F.pad(x, (0, 0, p, p))
        # im2col: (B, N, 7 Cin) with column t Cin + ci = x[:, l + dil (t - 3), ci], against W as (7 Cin, Cout): one GEMM
        cols = torch.cat([xp[:, dil * t: dil * t + self.N, :] for t in range(7)], 2)
        return torch.addmm(m.bias, cols.reshape(-1, cols.shape[2]),
                           m.weight.permute(2, 1, 0).reshape(-1, m.weight.shape[0])).view(x.shape[0], self.N, -1)

    native = False  # True: F.conv1d on (B, C, N) (MIOpen), else the tap-GEMM form on (B, N, C)

    def forward(self, y, dropout=0.1):
        g = F.gelu
        shapes = {n: d for n, _, _, d in conv_shapes(self.E)}
        if self.native:
            def c(x_, n):
                seq, idx = n.split(".")
                m = getattr(self, seq)[idx]
                return g(F.conv1d(x_, m.weight, m.bias, padding=3 * shapes[n], dilation=shapes[n]))
            x = y.unsqueeze(1)                               # (B, 1, N)
        else:
            c = lambda x_, n: g(self.conv(x_, n, shapes[n]))  # noqa: E731
            x = y.unsqueeze(-1)                              # (B, N, 1)
        x2 = c(c(x, "layers1.0"), "layers1.2")
        x3 = c(c(x2, "layers2.0"), "layers2.2") + x2
        x4 = c(c(x3, "layers3.0"), "layers3.2") + x3
        x5 = c(c(x4, "layers4.0"), "layers4.2") + x4
        x6 = c(c(x5, "layers5.0"), "layers5.2")
        # torch.flatten of (B, C, N): c N + l
        flat = (x6 if self.native else x6.permute(0, 2, 1)).reshape(y.shape[0], -1)
        f = self.layersFin
        h = f["4"](g(f["2"](g(f["0"](flat)))))
        return self.layer_norm(F.dropout(h, dropout, self.training))

    def reference_state_dict(self):
        """Keys exactly as models.convNet's (layers1.0.weight, ..., layersFin.4.bias, layer_norm.weight / bias)."""
        return {k: v.detach().cpu().clone() for k, v in self.state_dict().items()}


def plotkin(u):
    """x = u F^{(x)n} in BPSK (polar.py:128-148), as train_crisp_gpu.plotkin."""
    B, N = u.shape
    x = u.clone()
    s = 1
    while s < N:
        v = x.view(B, N // (2 * s), 2, s)
        v[:, :, 0, :] = v[:, :, 0, :] * v[:, :, 1, :]
        s *= 2
    return x


def stage_info(N, target_K, K):
    """n2c (run_models.py:666-669 with polar.py:101-106): the K least reliable of the target's information set."""
    rs = polar_rs(N)
    return np.sort(np.flip(rs[:target_K])[:K].copy()).astype(np.int64)


@torch.no_grad()
def evaluate(net, c, dev, n=1 << 14, snrs=(0.0, 2.0, 4.0)):
    """BER / BLER of the final code (the target information set) with the training forward in eval mode."""
    net.eval()
    info = torch.as_tensor(stage_info(c["N"], c["K"], c["K"]), device=dev)
    res = []
    for s in snrs:
        msg = 1 - 2 * (torch.rand(n, c["K"], device=dev) < 0.5).float()
        u = torch.ones(n, c["N"], device=dev)
        u[:, info] = msg
        y = plotkin(u) + snr_db2sigma(s) * torch.randn(n, c["N"], device=dev)
        e = (net(y)[:, info].sign() != msg).sum(1)
        res.append((float(e.sum()) / (n * c["K"]), float((e > 0).float().mean())))
    net.train()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--state", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--budget-s", type=float, default=1000.0)
    ap.add_argument("--eval-every", type=int, default=2000)
    ap.add_argument("--probe", type=int, default=0)
    ap.add_argument("--native", action="store_true", help="F.conv1d through MIOpen instead of the tap-GEMM form")
    ap.add_argument("--amp", choices=["none", "bf16"], default="none",
                    help="bf16 autocast of the forward (training speed only; every parity claim rests on the "
                         "reference's fp32 convNet run on the resulting weights)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    c = CASE
    N, E = c["N"], c["embed"]
    torch.manual_seed(c["seed_init"])
    net = ConvNetT(E, N).to(dev)
    net.native = args.native
    st = {"stage": 0, "step": 0}
    if os.path.exists(args.state):
        st = torch.load(args.state, map_location=dev, weights_only=True)
        net.load_state_dict(st["net"])
        print(f"resume: stage {st['stage']} step {st['step']}", flush=True)
    t_start = last_save = last_print = time.time()
    stages = c["curriculum"]

    def save(opt, stage, step):
        tmp = args.state + ".tmp"
        torch.save({"stage": stage, "step": step, "net": net.state_dict(), "opt": opt.state_dict()}, tmp)
        os.replace(tmp, args.state)

    while st["stage"] < len(stages):
        si = st["stage"]
        K, steps, snr = stages[si]
        info = torch.as_tensor(stage_info(N, c["K"], K), device=dev)
        opt = torch.optim.AdamW(net.parameters(), lr=c["lr"])
        if st["step"] > 0 and "opt" in st:
            opt.load_state_dict(st["opt"])
        torch.manual_seed(c["seed_init"] * 1009 + 7919 * si + st["step"])
        sigma = snr_db2sigma(snr)
        net.train()
        t0, s0 = time.time(), st["step"]
        for step in range(st["step"], steps):
            msg = 1 - 2 * (torch.rand(c["batch"], K, device=dev) < 0.5).float()
            u = torch.ones(c["batch"], N, device=dev)
            u[:, info] = msg
            y = plotkin(u) + sigma * torch.randn(c["batch"], N, device=dev)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.amp == "bf16"):
                logits = net(y)
            loss = F.mse_loss(logits[:, info].float(), msg)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(net.parameters(), 0.25)
            opt.step()
            opt.zero_grad()
            now = time.time()
            if args.probe and step + 1 - s0 == args.probe:
                torch.cuda.synchronize()
                print(f"PROBE {c['name']}: {args.probe / (time.time() - t0):.2f} steps/s", flush=True)
                return
            if now - last_print > 30 or step == steps - 1:
                print(f"[{c['name']}] stage {si + 1}/{len(stages)} K={K} snr={snr} step {step + 1}/{steps} loss "
                      f"{loss.item():.5f} ({(step + 1 - s0) / max(now - t0, 1e-9):.1f} steps/s)", flush=True)
                last_print = now
            if step == steps - 1 or (K == c["K"] and (step + 1) % args.eval_every == 0):
                r = evaluate(net, c, dev)
                print("   eval (target code) " + " ".join(f"{s:g}dB BER {b:.4f} BLER {k:.4f}"
                                                       for s, (b, k) in zip((0, 2, 4), r)), flush=True)
            if now - t_start > args.budget_s:
                save(opt, si, step + 1)
                print(f"RESUME at stage {si} step {step + 1}", flush=True)
                return
            if now - last_save > 60:
                save(opt, si, step + 1)
                last_save = now
        st = {"stage": si + 1, "step": 0}
        save(opt, si + 1, 0)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    torch.save({"xformer": net.reference_state_dict()}, args.out)
    print(f"DONE {c['name']} -> {args.out}", flush=True)


if __name__ == "__main__":
    main()
