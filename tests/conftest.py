import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device; runs the product kernels")
    config.addinivalue_line("markers", "slow: longer-running test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible (run on the MI355X box: pytest -m gpu)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def weights_digest(sd):
    """sha256 over a state dict's arrays in sorted key order (tests/golden/gen_golden.py)."""
    import hashlib
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], np.float32).tobytes())
    return h.hexdigest()


def gru_state_dict(d):
    """A GRU fixture's weights: stored arrays, or (F > 64) regenerated from the stored torch seed with this
    package's RNN_Model (same parameter draws as the reference's) and checked against the stored digest."""
    if "w_seed" not in d.files:
        return {k[2:]: np.asarray(d[k]) for k in d.files if k.startswith("w.")}
    import torch
    from neural_polar_decoder_amd.rnn import RNN_Model
    N, F = int(d["N"]), int(d["F"])
    torch.manual_seed(int(d["w_seed"]))
    net = RNN_Model("GRU", N + 1 + int(d["onehot"]), F, 1, 2, N, 0, 0, "selu", 0.0, False, out_linear_depth=1)
    sd = {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}
    assert weights_digest(sd) == bytes(d["w_digest"]).decode(), "regenerated GRU weights differ from the fixture's"
    return sd


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


def conv_weights_from_seed(embed, N, seed):
    """Mirror of tests/golden/gen_golden.py::conv_weights_from_seed (documented generator):
    PCG64(seed); parameters in convNet.state_dict order ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in));
    LayerNorm weight = 1 + 0.1 U(-1,1), bias = 0.1 U(-1,1)."""
    h = embed // 2
    k = 7
    spec = [("layers1.0", h, 1), ("layers1.2", h, h), ("layers2.0", h, h), ("layers2.2", h, h),
            ("layers3.0", h, h), ("layers3.2", h, h), ("layers4.0", h, h), ("layers4.2", h, h),
            ("layers5.0", embed, h), ("layers5.2", embed, embed)]
    shapes = []
    for name, cout, cin in spec:
        shapes.append((name + ".weight", (cout, cin, k)))
        shapes.append((name + ".bias", (cout,)))
    shapes += [("layersFin.0.weight", (4 * N, embed * N)), ("layersFin.0.bias", (4 * N,)),
               ("layersFin.2.weight", (N, 4 * N)), ("layersFin.2.bias", (N,)),
               ("layersFin.4.weight", (N, N)), ("layersFin.4.bias", (N,)),
               ("layer_norm.weight", (N,)), ("layer_norm.bias", (N,))]
    wshape = dict(shapes)
    rng = np.random.default_rng(seed)
    sd = {}
    for key, shape in shapes:
        if key.startswith("layer_norm"):
            a = rng.uniform(-1, 1, size=shape)
            arr = (1.0 + 0.1 * a) if key.endswith("weight") else 0.1 * a
        else:
            ws = wshape[key.rsplit(".", 1)[0] + ".weight"]
            bnd = 1.0 / np.sqrt(int(np.prod(ws[1:])))
            arr = rng.uniform(-bnd, bnd, size=shape)
        sd[key] = arr.astype(np.float32)
    return sd


def trained_fixture(name):
    """A trained CRISP fixture (tests/golden/gen_trained.py) or a skip if it has not been generated."""
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        pytest.skip(f"{name}.npz not generated (tests/golden/gen_trained.py)")
    return np.load(path)


def trained_words(d, si):
    """The fixture's decision words at SNR index si, regenerated exactly as gen_trained.py drew them through
    the reference (torch.manual_seed(seed_dec + si); msg = 1 - 2 (rand < 0.5); y = encode(msg) + sigma *
    randn, polar.py:128-148, 201-207; PAC fixtures: pac_encode, pac_code.py:220-231) -- the encoder is the
    oracle's (bit-exact +-1) -- and checked against
    the stored sha256 of y.  Returns (msg (B,K), y (B,N)) as float32 numpy arrays."""
    import hashlib
    import torch
    from oracle import oracle as O
    N, K = int(d["N"]), int(d["K"])
    torch.manual_seed(int(d["seed_dec"]) + si)
    msg = 1.0 - 2.0 * (torch.rand(int(d["n_dec"]), K) < 0.5).float()
    pac = "pac" in d.files and int(d["pac"]) == 1
    if pac:  # pac_code.py:220-224 with the fixture's generator (g = 91; 53 at N = 32 as rnn_all.py:231-232 sets it)
        x = torch.from_numpy(O.pac_encode(msg.numpy(), N, d["info"], g=int(d["g"]) if "g" in d.files else 91))
    else:  # polar.py:128-148
        x = torch.from_numpy(O.encode_plotkin(msg.numpy(), N, d["info"]))
    sigma = 10 ** (-float(d["snr"][si]) * 1.0 / 20)
    y = x + sigma * torch.randn(x.shape, dtype=torch.float)
    yn = y.numpy()
    assert hashlib.sha256(np.ascontiguousarray(yn).tobytes()).hexdigest() == bytes(d[f"y_digest_{si}"]).decode(), \
        "regenerated fixture words differ from the reference's (torch RNG stream changed?)"
    return msg.numpy(), yn


def trained_decisions(d, si):
    """The reference's RNN_decoder.decode decisions at the information positions (+-1), (B, K)."""
    K = int(d["K"])
    bits = np.unpackbits(d[f"dec_bits_{si}"], axis=1)[:, :K]
    return np.where(bits == 1, -1.0, 1.0).astype(np.float32)


def db_offsets(snrs, bler, ref_snrs, ref_bler, min_bler=1e-4):
    """Horizontal offset (dB) of a BLER curve from a reference curve: for each point, the SNR at which the
    reference's log-BLER (linear in SNR between its grid points; the end segments extended linearly) equals
    log(bler), minus the point's SNR.  Positive = the curve needs more SNR than the reference.  Points below
    min_bler are skipped (None)."""
    rs = np.asarray(ref_snrs, float)
    lr = np.log(np.maximum(np.asarray(ref_bler, float), 1e-300))
    out = []
    for s, p in zip(snrs, bler):
        if p < min_bler or p <= 0:
            out.append(None)
            continue
        lp = np.log(p)
        j = None
        for i in range(len(rs) - 1):
            if (lr[i] - lp) * (lr[i + 1] - lp) <= 0 and lr[i] != lr[i + 1]:
                j = i
                break
        if j is None:  # outside the reference's range: the nearer end segment, extended
            j = 0 if abs(lp - lr[0]) < abs(lp - lr[-1]) else len(rs) - 2
        a, b = lr[j], lr[j + 1]
        out.append(float(rs[j] + (lp - a) / (b - a) * (rs[j + 1] - rs[j]) - s))
    return out


def assert_db_bar(snrs, bler, n, ref_bler, nr, need=2):
    """The +-0.05 dB bar on a BLER curve (north_star: within +-0.05 dB of the reference over 0-4 dB): the horizontal
    offset of our curve from the reference's is defined where the reference's BLER is in [1e-3, 0.9] and resolvable
    where the two Monte-Carlo samples pin it -- 3 sigma_dB <= 0.05, sigma_dB the binomial sigma of ln BLER of both curves
    over the reference's local slope |d ln BLER / d SNR|; there |offset| <= 0.05, elsewhere in the domain within its own
    3 sigma.  At least `need` resolvable points must exist, so the dB bar always runs.  Returns that count."""
    import numpy as np
    offs = db_offsets(snrs, bler, snrs, ref_bler, min_bler=1e-3)
    lr = np.log(np.maximum(ref_bler, 1e-300))
    checked = 0
    for i, (s, o, p, pr) in enumerate(zip(snrs, offs, bler, ref_bler)):
        if not 1e-3 <= pr <= 0.9:
            continue
        j0, j1 = max(i - 1, 0), min(i + 1, len(snrs) - 1)
        slope = abs(lr[j1] - lr[j0]) / (snrs[j1] - snrs[j0])
        sig = np.sqrt((1 - p) / (p * n) + (1 - pr) / (pr * nr)) / max(slope, 1e-9)
        assert o is not None, (s, p, pr)
        if 3 * sig <= 0.05:
            assert abs(o) <= 0.05, (s, o, pr, sig)
            checked += 1
        else:
            assert abs(o) <= 3 * sig, (s, o, pr, sig)
    assert checked >= need, f"only {checked} SNR points where the +-0.05 dB bar is defined and resolvable"
    return checked
