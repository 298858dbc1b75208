import sys, torch
sys.path.insert(0, '.')
from neural_polar_decoder_amd import reference_polar_code
code = reference_polar_code(64, 32)
B = 1 << 20
ys = [code.mc_generate(B, float(s), 1234, s, 0, want_msg=False)[2] for s in range(5)]
hat = torch.empty(B, 32, device='cuda')
cnt = torch.zeros(2, dtype=torch.int64, device='cuda')
def run(mode, it=20):
    for _ in range(3):
        for s, y in enumerate(ys):
            f(mode, s, y)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        for s, y in enumerate(ys):
            f(mode, s, y)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / (it * 5)
    return ms
def f(mode, s, y):
    if mode == 'count+msg': code.sc_decode_mc(y, float(s), 1234, 0, cnt, msg_hat=hat)
    elif mode == 'count': code.sc_decode_mc(y, float(s), 1234, 0, cnt)
    elif mode == 'msg': code.sc_decode_msg(y, float(s))
for mode in ['count+msg', 'count', 'msg', 'count+msg', 'count']:
    ms = run(mode)
    print(f"{mode:10s} {ms*1e3:7.1f} us  {B/ms/1e6:6.2f} Gcw/s  read-only GB/s {B*256/ms/1e6:7.0f}")
