"""PAC(128,64) SC per 2^20 codewords per SNR on cuda:0: the streaming decode (y resident, msg_hat written) and
the fused Monte-Carlo sweep (generation in the decode kernel): python tools/pac_bench.py"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import PAC, reference_polar_code  # noqa: E402


def ev(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev = "cuda:0"
    B = 1 << 20
    snrs = [0.0, 1.0, 2.0, 3.0, 4.0]
    for name, code in [("PAC(128,64)", PAC(argparse.Namespace(target_K=64), 128, 64, 91)),
                       ("Polar(128,64)", reference_polar_code(128, 64)), ("Polar(256,128)", reference_polar_code(256, 128))]:
        K = code.K
        c = torch.zeros(len(snrs), 2, dtype=torch.int64, device=dev)
        hat = torch.empty(B, K, device=dev)
        _, _, y = code.mc_generate(B, 2.0, 1, 2, 0, device=dev, want_msg=False)
        t_dec = ev(lambda: code.sc_decode_mc(y, 2.0, 1, 0, c[2], msg_hat=hat))
        t_gen = ev(lambda: code.mc_generate(B, 2.0, 1, 2, 0, device=dev, want_msg=False), 5)
        t_fused = ev(lambda: code.sc_mc_sweep_fused(B, snrs, 1, 0, c), 5) / len(snrs)
        print(f"{name}: decode {t_dec:.3f} ms + generate {t_gen:.3f} ms per 2^20 | fused sweep {t_fused:.3f} ms per "
              f"2^20 per SNR", flush=True)


if __name__ == "__main__":
    main()
