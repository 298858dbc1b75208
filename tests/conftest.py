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
