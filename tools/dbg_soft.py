import sys, os, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from oracle import oracle as O
from neural_polar_decoder_amd import PolarCode
d = np.load("tests/golden/lse_soft_128_64.npz")
N = 128
code = PolarCode(7, 64, F=np.setdiff1d(np.arange(N), d["info"]))
for s in np.unique(d["snr"]):
    m = d["snr"] == s
    y = d["y"][m]
    h, b = code.sc_decode_soft(torch.from_numpy(y).cuda(), float(s), priors=d["prior"], hard_decision=False, return_bits=True)
    b = b.cpu().numpy()
    ob = O.sc_decode_soft(y, float(s), d["info"], False, d["prior"])[1]
    g = d["bits_soft_pr"][m]
    dn = np.isnan(b) != np.isnan(g)
    do = np.isnan(ob) != np.isnan(g)
    print("snr", s, "rows", y.shape[0], "gpu-vs-ref nan mismatches", dn.sum(), "oracle-vs-ref", do.sum())
    if dn.any():
        r, c = np.nonzero(dn)
        print(" first rows/cols", list(zip(r[:10].tolist(), c[:10].tolist())))
        print(" gpu", b[r[:5], c[:5]], "ref", g[r[:5], c[:5]], "oracle", ob[r[:5], c[:5]])
        print(" nan count gpu row", np.isnan(b[r[0]]).sum(), "ref row", np.isnan(g[r[0]]).sum())
        print(" |y| max of row", np.abs(y[r[0]]).max())
