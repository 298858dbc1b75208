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
