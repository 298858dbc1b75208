"""Probe: the configs[4] FC0 product (4096 codewords x K = E N = 32768 -> 4N = 1024) as library fp16 GEMMs with fp32
output (torch.mm(..., out_dtype=float32) -> hipBLASLt), the fp16x3 split written as one GEMM over a tripled K
([Xhi | Xhi | Xlo] . [Whi ; Wlo ; Whi]) or three accumulated GEMMs, against fc_split_wsp_kernel's ~1.02 ms."""
import time

import torch

dev = "cuda:0"


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for M in (4096, 8192):
    K, Nn = 32768, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    xh = torch.randn(M, 3 * K, device=dev, generator=g).half()
    wt = torch.randn(3 * K, Nn, device=dev, generator=g).half()
    w_nk = torch.randn(Nn, 3 * K, device=dev, generator=g).half()
    flop = 2.0 * M * Nn * 3 * K
    try:
        t = bench(lambda: torch.mm(xh, wt, out_dtype=torch.float32))
        print(f"M {M}: one GEMM K 3x32768 fp16 -> fp32 (B K-major): {t:.3f} ms, {flop / t / 1e9:.0f} TFLOP/s issued", flush=True)
    except Exception as e:  # noqa: BLE001
        print("out_dtype mm failed:", repr(e)[:200], flush=True)
    try:
        t = bench(lambda: torch.mm(xh, w_nk.t(), out_dtype=torch.float32))
        print(f"M {M}: one GEMM, B = W (Nout, K) row-major transposed: {t:.3f} ms, {flop / t / 1e9:.0f} TFLOP/s", flush=True)
    except Exception as e:  # noqa: BLE001
        print("out_dtype mm (t) failed:", repr(e)[:200], flush=True)
    t = bench(lambda: torch.mm(xh, w_nk.t()))
    print(f"M {M}: fp16 output (reference point): {t:.3f} ms, {flop / t / 1e9:.0f} TFLOP/s", flush=True)
    del xh, wt, w_nk
    torch.cuda.empty_cache()
