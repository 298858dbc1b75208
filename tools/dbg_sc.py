import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from conftest import golden
from oracle import oracle as O
from neural_polar_decoder_amd import PolarCode
for N, K in [(128, 64), (256, 128)]:
    d = golden(f"sc_polar_{N}_{K}.npz")
    F = np.array(sorted(set(range(N)) - set(int(i) for i in d["info"])))
    code = PolarCode(int(np.log2(N)), K, F=F)
    for s in np.unique(d["snr"]):
        m = d["snr"] == s
        leaf, hat = code.sc_decode_new(torch.from_numpy(d["y"][m]).cuda(), float(s))
        leaf = leaf.cpu().numpy(); hat = hat.cpu().numpy()
        bad = np.argwhere(leaf != d["leaf"][m])
        print(N, s, "leaf bad", len(bad), "hat bad", (hat != d["msg_hat"][m]).sum())
        if len(bad):
            r, c = bad[0]
            print("  first", r, c, leaf[r, c], d["leaf"][m][r, c], "cols", np.unique(bad[:, 1])[:40])
