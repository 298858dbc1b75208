"""A/B timing of the fp16x3 GRU kernel (gru16p_kernel<5>) across libnpd builds: 2^20 Polar(64,32) words at 2 dB with
the trained tests/golden/trained_crisp_64_32.npz net (the headline's GRU).  Each library runs in its own process
(NPD_LIB), alternating A B A B ..., and reports ms per 2^20 decode (HIP events, 5 launches) plus its decisions'
agreement with the fp32 kernel of the same build and the max |logit| difference on agreeing codewords.

    python tools/gru16_time.py tools/bin/libnpd_a.so tools/bin/libnpd_b.so [--rounds 2]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from neural_polar_decoder_amd import reference_polar_code
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    d = np.load(os.path.join(ROOT, "tests", "golden", "trained_crisp_64_32.npz"))
    net = RNN_Model("GRU", 66, 64, 1, 2, 64, 0, 0).cuda().eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    code = reference_polar_code(64, 32)
    _, _, y = code.mc_generate(1 << 20, 2.0, 1234, 2, 0, want_msg=False)
    out = {}
    res = {}
    for prec in ("fp32", "fp16x3"):
        dec = RNN_decoder("y_input", 64, code.info_positions, onehot=True, precision=prec)
        dd, lg = dec.decode(net, False, y, return_logits=True)
        res[prec] = (dd, lg)
        if True:
            for _ in range(2):
                dec.decode(net, False, y)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                dec.decode(net, False, y)
            e.record()
            torch.cuda.synchronize()
            out["ms" if prec == "fp16x3" else "ms_fp32"] = s.elapsed_time(e) / 5
    same = (res["fp32"][0] == res["fp16x3"][0]).all(1)
    out["cw_agree"] = same.float().mean().item()
    out["max_logit_diff"] = (res["fp32"][1][same] - res["fp16x3"][1][same]).abs().max().item()
    print("RESULT " + json.dumps(out), flush=True)


def main():
    if os.environ.get("GRU16_CHILD"):
        return child()
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, GRU16_CHILD="1", NPD_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                               timeout=300)
            line = next((l for l in p.stdout.splitlines() if l.startswith("RESULT ")), None)
            if p.returncode != 0 or line is None:
                print(f"{lib}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                return 1
            res = json.loads(line[7:])
            print(f"round {r} {os.path.basename(lib):28s} {res['ms']:8.3f} ms/2^20  cw_agree {res['cw_agree']:.6f}  "
                  f"max_logit_diff {res['max_logit_diff']:.2e}  fp32 kernel {res['ms_fp32']:.2f} ms", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
