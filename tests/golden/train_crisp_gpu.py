#!/usr/bin/env python3
"""GPU stages of the CRISP curricula behind the trained fixtures (test infrastructure, not product code).

The reference's training loop costs 0.6-2.3 s per step on this container's 8 CPU cores at the fixture
shapes (Polar(64,32): 0.65 s, PAC(128,64): 2.3 s at batch 4096), so a run_crisp.sh-shaped curriculum --
K + 1 per stage, >= 1000 steps per stage, a long final stage -- takes days there for PAC(128,64).  This
script runs the early stages of such a curriculum on one MI355X with PyTorch-ROCm; tests/golden/gen_trained.py
then runs the LAST stage(s) with the reference's own rnn_all.py (unmodified, on the CPU, --load_path = the
weights written here) and evaluates the final net with the reference's own decoder.  Nothing here imports
the reference (it runs on the GPU box); the fixtures' parity claims rest on the reference's decoder alone.

Restatement of rnn_all.py's training loop (rnn_all.py:1386-1440) for decoding_type y_input, onehot, GRU,
teacher forcing ratio 1 (tfr_min = tfr_max = 1, run_crisp.sh:2):
  * per step: msg = 1 - 2 (rand < 0.5) (B, K); gt = ones (B, N), gt[:, info] = msg (rnn_all.py:1395-1397);
    y = channel(encode(msg), snr_train) (:1399-1400; encode: a torch restatement of encode_plotkin / pac_encode,
    held to the oracle's bit-exact encoders by tests/test_trained_gru.py; noise: sigma * randn);
  * teacher forcing (rnn_all.py:436-450): N single-step GRU calls with input [y, onehot(prev)], prev = +1
    for step 0 and gt[:, i-1] after; the same recurrence as ONE nn.GRU call over the length-N sequence;
    decoded[:, i] = Linear(h1_i) (rnn_all.py:387-398);
  * loss = MSELoss(decoded[:, info], msg) (:1409-1417); loss.backward(); clip_grad_norm_(0.25) (:1431,
    --clip default); AdamW(lr).step(); zero_grad(); StepLR(lr_decay, gamma).step() (:1343-1359, 1433-1438);
  * each curriculum stage is one rnn_all.py invocation in run_crisp.sh: fresh AdamW and StepLR, weights
    from the previous stage (--load_path, rnn_all.py:1326-1329); the first stage starts from PyTorch's
    default initialisation (RNN_Model, rnn_all.py:294-344).

Resumable (gpurun calls are limited to 20 minutes): the state (stage, step, weights, optimizer, scheduler)
is written to --state every ~60 s and when --budget-s runs out; a rerun with the same --state continues.
When every stage is done the final weights are written to --out as {'net': state_dict}.

    python tests/golden/train_crisp_gpu.py CASE --state train_state/CASE.pt --out gpurun_out/train/CASE.net.pt
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from neural_polar_decoder_amd.codes import pac_info_positions, polar_info_positions  # noqa: E402
from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model  # noqa: E402
from neural_polar_decoder_amd.utils import snr_db2sigma  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from crisp_cases import CASES  # noqa: E402


def plotkin(u):
    """x = u F^{(x)n} in BPSK (XOR as product): stage d, blocks of 2^(d+1): left <- left * right (polar.py:128-148)."""
    B, N = u.shape
    x = u.clone()
    s = 1
    while s < N:
        v = x.view(B, N // (2 * s), 2, s)
        v[:, :, 0, :] = v[:, :, 0, :] * v[:, :, 1, :]
        s *= 2
    return x


def pac_taps(g):
    """Delays j >= 1 whose generator bit is set (g_array = 1 - 2 bits(g), pac_code.py:101-103): g = 91 -> (2, 3, 5, 6),
    g = 53 (the reference's choice at N = 32, rnn_all.py:231-232) -> (1, 3, 5)."""
    bits = [int(ch) for ch in bin(g)[2:]]
    return tuple(j for j in range(1, len(bits)) if bits[j] == 1)


def pac_conv(v, taps=(2, 3, 5, 6)):
    """PAC rate-1/1 convolution (pac_code.py:193-200): u_i = v_i prod_{j in taps} v_{i-j}, v_{<0} = +1 (default g = 91)."""
    B, N = v.shape
    vp = torch.cat([torch.ones(B, max(taps), device=v.device), v], 1)
    u = v.clone()
    for j in taps:
        u = u * vp[:, max(taps) - j: max(taps) - j + N]
    return u


def make_code(c, K, device="cuda"):
    """Stage-K code of the curriculum: rnn_all.get_code(code, rate_profile, N, K) with --target_K = c['K'].
    Returns (info, encode) with encode(msg) -> x on msg's device (torch restatement of encode_plotkin /
    pac_encode, checked against the oracle's bit-exact encoders by tests/test_trained_gru.py)."""
    N = c["N"]
    if c["code"] == "Polar":
        info = polar_info_positions(N, K, c["profile"], target_K=c["K"])
    else:
        info = pac_info_positions(N, K, c["profile"], target_K=c["K"])
    it = torch.as_tensor(info, device=device)
    pac = c["code"] == "PAC"

    def enc(msg):
        u = torch.ones(msg.shape[0], N, device=msg.device)
        u[:, it] = msg
        return plotkin(pac_conv(u, pac_taps(c.get("g", 91))) if pac else u)
    return info, enc


def teacher_forced(net, y, gt):
    """decoded (B, N) of the teacher-forcing branch (rnn_all.py:436-450) as one sequence call."""
    B, N = y.shape
    prev = torch.cat([torch.ones(B, 1, device=y.device), gt[:, :-1]], 1)
    oh = torch.stack([(prev < 0).float(), (prev > 0).float()], -1)  # get_onehot: +1 -> [0, 1], -1 -> [1, 0]
    x = torch.cat([y.unsqueeze(1).expand(B, N, N), oh], 2)
    h0 = torch.zeros(net.num_rnn_layers, B, net.feature_size, device=y.device)
    out, _ = net.rnn(x, h0)
    return net.linear(out).squeeze(-1)


@torch.no_grad()
def evaluate(net, c, K, snrs, dev, n=1 << 14):
    """BER / BLER at the stage's code: the fused HIP decoder (the product's eval path) on a GPU, the
    reference's per-step loop (rnn_all.py:532-547, RNN_Model.forward) on the CPU."""
    info, enc = make_code(c, K, dev)
    it = torch.as_tensor(info, device=dev)
    net.eval()
    res = []
    for s in snrs:
        msg = 1 - 2 * (torch.rand(n, K, device=dev) < 0.5).float()
        y = enc(msg) + snr_db2sigma(s) * torch.randn(n, c["N"], device=dev)
        if dev.type == "cuda":
            d = RNN_decoder("y_input", c["N"], info, onehot=True).decode(net, False, y)[:, it]
        else:
            N = c["N"]
            isinfo = np.zeros(N, bool)
            isinfo[info] = True
            dd = torch.ones(n, N)
            hidden = torch.zeros(net.num_rnn_layers, n, net.feature_size)
            for ii in range(N):
                prev = torch.ones(n) if ii == 0 else dd[:, ii - 1].sign()
                oh = torch.stack([(prev <= 0).float(), (prev > 0).float()], 1)
                out, hidden = net(torch.cat([y.unsqueeze(1), oh.view(-1, 1, 2)], 2), hidden)
                if isinfo[ii]:
                    dd[:, ii] = out.squeeze().sign()
            d = dd[:, it]
        e = (d != msg).sum(1)
        res.append((float(e.sum()) / (n * K), float((e > 0).float().mean())))
    net.train()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case", choices=sorted(CASES))
    ap.add_argument("--state", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--budget-s", type=float, default=1000.0)
    ap.add_argument("--eval-every", type=int, default=1000)
    ap.add_argument("--miopen", action="store_true", help="nn.GRU through MIOpen (default: PyTorch's native GRU)")
    ap.add_argument("--device", default="cuda", help="cuda (MI355X) or cpu")
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--amp", choices=["none", "bf16"], default="none",
                    help="bf16 autocast of the forward (training speed only; the fixture is whatever weights result, "
                         "and every parity claim rests on the reference's fp32 decoder run on them)")
    ap.add_argument("--probe", type=int, default=0, help="time this many steps and exit (no state written)")
    ap.add_argument("--graph", action="store_true",
                    help="capture one whole training step (data, forward, backward, clip, AdamW) in a HIP graph and "
                         "replay it: the hidden-64 step is launch-bound (~600 small kernels for the 64-step GRU and its "
                         "backward); StepLR is applied by writing the tensor learning rate between replays")
    ap.add_argument("--init", default=None, help="weights ({'net': state_dict}) to start the first GPU stage from "
                                                  "(the reference-loop stages before the GPU block)")
    args = ap.parse_args()
    torch.backends.cudnn.enabled = args.miopen
    dev = torch.device(args.device)
    if args.threads:
        torch.set_num_threads(args.threads)
    c = CASES[args.case]
    stages = [(K, steps) for K, steps, who in c["curriculum"] if who == "gpu"]
    t_start = time.time()
    N, F, L = c["N"], c["F"], c["layers"]
    net = RNN_Model("GRU", N + 2, F, 1, L, N, 0, 0).to(dev)
    st = {"stage": 0, "step": 0}
    if os.path.exists(args.state):
        st = torch.load(args.state, map_location=dev, weights_only=True)
        net.load_state_dict(st["net"])
        print(f"resume {args.case}: stage {st['stage']} step {st['step']}", flush=True)
    elif args.init:
        net.load_state_dict(torch.load(args.init, map_location=dev, weights_only=True)["net"])
        print(f"init {args.case} from {args.init}", flush=True)
    else:
        torch.manual_seed(c["seed_init"])
        net = RNN_Model("GRU", N + 2, F, 1, L, N, 0, 0).to(dev)  # PyTorch default init, as RNN_Model(...)
    loss_fn = nn.MSELoss()
    last_save = time.time()
    last_print = time.time()

    def save(opt, sched, stage, step):
        tmp = args.state + ".tmp"
        os.makedirs(os.path.dirname(os.path.abspath(args.state)) or ".", exist_ok=True)
        torch.save({"stage": stage, "step": step, "net": net.state_dict(), "opt": opt.state_dict(),
                    "sched": sched.state_dict()}, tmp)
        os.replace(tmp, args.state)

    while st["stage"] < len(stages):
        si = st["stage"]
        K, steps = stages[si]
        info, enc = make_code(c, K, dev)
        info_t = torch.as_tensor(info, device=dev)
        opt = torch.optim.AdamW(net.parameters(), lr=c["lr"])
        sched = torch.optim.lr_scheduler.StepLR(opt, c["lr_decay"], c["lr_gamma"])
        if st["step"] > 0 and "opt" in st:
            opt.load_state_dict(st["opt"])
            sched.load_state_dict(st["sched"])
        torch.manual_seed(c["seed_init"] * 100003 + 1009 * si + st["step"])
        sigma = snr_db2sigma(c["snr_train"])
        net.train()
        t0, s0 = time.time(), st["step"]

        def train_step():
            msg = 1 - 2 * (torch.rand(c["batch"], K, device=dev) < 0.5).float()
            gt = torch.ones(c["batch"], N, device=dev)
            gt[:, info_t] = msg
            y = enc(msg) + sigma * torch.randn(c["batch"], N, device=dev)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.amp == "bf16"):
                decoded = teacher_forced(net, y, gt)
            loss = loss_fn(decoded[:, info_t].float(), msg)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(net.parameters(), 0.25)
            opt.step()
            opt.zero_grad(set_to_none=not args.graph)
            return loss

        graph = None
        if args.graph:
            # capturable AdamW with a tensor learning rate (the same update rule); StepLR's value is written into it
            lr_t = torch.tensor(sched.get_last_lr()[0], device=dev)
            sd = opt.state_dict()
            opt = torch.optim.AdamW(net.parameters(), lr=lr_t, capturable=True)
            if st["step"] > 0 and "opt" in st:
                sd["param_groups"][0]["lr"] = lr_t
                sd["param_groups"][0]["capturable"] = True
                opt.load_state_dict(sd)
                for p_ in opt.state.values():
                    if "step" in p_:
                        p_["step"] = p_["step"].to(dev)
                opt.param_groups[0]["lr"] = lr_t
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # warm-up outside the capture (allocations, AdamW state)
                for _ in range(3):
                    train_step()
            torch.cuda.current_stream().wait_stream(side)  # (3 extra updates per resumed slice, kept)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                g_loss = train_step()
        for step in range(st["step"], steps):
            if graph is not None:
                lr_now = c["lr"] * c["lr_gamma"] ** (step // c["lr_decay"])  # StepLR(lr_decay, gamma) before step
                lr_t.fill_(lr_now)
                graph.replay()
                loss = g_loss
                sched.step()
            else:
                loss = train_step()
                sched.step()
            now = time.time()
            if args.probe and step + 1 - s0 == args.probe:
                torch.cuda.synchronize()
                print(f"PROBE {args.case} amp={args.amp} miopen={args.miopen}: "
                      f"{args.probe / (time.time() - t0):.2f} steps/s (incl. warm-up)", flush=True)
                return
            if now - last_print > 30 or step == steps - 1:
                rate = (step + 1 - s0) / max(now - t0, 1e-9)
                print(f"[{args.case}] stage {si + 1}/{len(stages)} K={K} step {step + 1}/{steps} "
                      f"loss {loss.item():.5f} lr {sched.get_last_lr()[0]:.2e} ({rate:.1f} steps/s)", flush=True)
                last_print = now
            if (step + 1) % args.eval_every == 0 or step == steps - 1:
                r = evaluate(net, c, K, c["eval_snrs"], dev)
                print("   eval " + " ".join(f"{s:g}dB BER {b:.4f} BLER {k:.4f}" for s, (b, k) in zip(c["eval_snrs"], r)),
                      flush=True)
            if now - t_start > args.budget_s:
                save(opt, sched, si, step + 1)
                print(f"RESUME {args.case} at stage {si} step {step + 1}", flush=True)
                return
            if now - last_save > 60:
                save(opt, sched, si, step + 1)
                last_save = now
        st = {"stage": si + 1, "step": 0}
        save(opt, sched, si + 1, 0)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    torch.save({"net": {k: v.detach().cpu() for k, v in net.state_dict().items()}}, args.out)
    print(f"DONE {args.case} -> {args.out}", flush=True)


if __name__ == "__main__":
    main()
