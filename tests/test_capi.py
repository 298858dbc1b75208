"""CPU: the C-ABI library loads, exports exactly what include/npd.h declares, and validates
arguments without touching a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "npd.h")
LIB = os.path.join(ROOT, "neural_polar_decoder_amd", "libnpd.so")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(npd_[a-z0-9_]+)\s*\(", src)))


def test_library_exists():
    assert os.path.exists(LIB), "build libnpd.so first (make lib / __graft_entry__.build())"


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 18
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (npd_[a-z0-9_]+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    L = ctypes.CDLL(LIB)
    for s in syms:
        assert getattr(L, s) is not None


def test_python_binding_matches_header():
    from neural_polar_decoder_amd import _lib
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert bound == set(declared_symbols())


def test_abi_and_device_count_without_gpu():
    from neural_polar_decoder_amd import _lib
    L = _lib.load()
    assert L.npd_abi_version() == 1
    assert L.npd_device_count() >= 0


def test_code_create_argument_errors():
    from neural_polar_decoder_amd import _lib
    L = _lib.load()
    out = ctypes.c_void_p()
    info = np.arange(4, dtype=np.int32)
    p = info.ctypes.data_as(ctypes.c_void_p)
    assert L.npd_code_create(48, 4, p, 0, 1000.0, ctypes.byref(out)) == -1      # not a power of two
    assert b"power of two" in L.npd_last_error()
    assert L.npd_code_create(512, 4, p, 0, 1000.0, ctypes.byref(out)) == -1     # too long
    bad = np.array([3, 1], dtype=np.int32)
    assert L.npd_code_create(8, 2, bad.ctypes.data_as(ctypes.c_void_p), 0, 1000.0, ctypes.byref(out)) == -1
    assert L.npd_code_create(8, 4, p, 91, 1000.0, ctypes.byref(out)) == 0       # valid PAC handle (host only)
    assert out.value
    assert L.npd_code_destroy(out) == 0


def test_null_pointer_errors_are_reported_not_fatal():
    from neural_polar_decoder_amd import _lib
    L = _lib.load()
    assert L.npd_sc_decode(None, None, 1.0, None, None, None, None, 16, None) == -1
    assert L.npd_awgn(None, None, 16, 6, 1.0, 0, 0, 0, None) == -1             # N % 4 != 0
    assert L.npd_count_errors(None, None, 4, 4, None, None) == -1
    assert L.npd_sc_decode_lse(None, None, 1.0, 1, None, None, 16, None) == -1
    assert L.npd_sc_decode_soft(None, None, 1.0, 1, None, None, None, 16, None) == -1
    assert L.npd_sc_decode_soft_new(None, None, 1.0, None, None, None, 16, None) == -1


def test_product_path_has_no_cpu_fallback():
    """Host inputs are staged to the GPU; with no GPU visible every compute call raises."""
    import torch
    from neural_polar_decoder_amd import NpdError, errors_bler, reference_polar_code
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: host tensors are staged to it")
    code = reference_polar_code(64, 32)
    with pytest.raises(NpdError):
        code.sc_decode_new(torch.zeros(4, 64), 1.0)
    with pytest.raises(NpdError):
        code.scl_decode(torch.zeros(4, 64), 1.0, 4)
    with pytest.raises(NpdError):
        errors_bler(torch.zeros(4, 8), torch.zeros(4, 8))


def test_list_prune_select_host_utility_matches_std_nth_element(oracle):
    """npd_list_prune_select (the tie rule compiled into the SCL kernel) == std::nth_element (oracle)."""
    import ctypes
    import numpy as np
    from neural_polar_decoder_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(3)
    m = ctypes.c_uint32()
    for n in range(1, 17):
        for k in range(1, n + 1):
            for _ in range(60):
                v = (-rng.integers(0, 3, n)).astype(np.float32)
                assert L.npd_list_prune_select(v.ctypes.data_as(ctypes.c_void_p), n, k, ctypes.byref(m)) == 0
                got = {i for i in range(n) if (m.value >> i) & 1}
                assert got == set(oracle.topk_select(v, k).tolist()), (n, k, v)
    assert L.npd_list_prune_select(None, 4, 2, ctypes.byref(m)) < 0
    v = np.zeros(20, np.float32)
    assert L.npd_list_prune_select(v.ctypes.data_as(ctypes.c_void_p), 20, 2, ctypes.byref(m)) < 0


def test_every_entry_point_rejects_null_operands():
    """Every compute and create entry point, called with NULL for each pointer (handles, operands, out-handles) and
    small valid sizes, returns a negative status with a message -- checked before any HIP call, so it runs without a
    GPU; destroy(NULL) is a no-op.  Run in a child process, so a crash fails this test instead of the session."""
    script = r'''
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from neural_polar_decoder_amd import _lib
L = _lib.load()
skip = {"npd_abi_version", "npd_last_error", "npd_device_count", "npd_conv_workspace_bytes",
        "npd_code_destroy", "npd_gru_destroy", "npd_conv_destroy"}
bad = []
for name, res, argt in _lib.SIGNATURES:
    if name in skip:
        continue
    args = []
    for t in argt:
        if t in (ctypes.c_int, ctypes.c_uint):
            args.append(16)
        elif t in (ctypes.c_long, ctypes.c_ulong):
            args.append(16)
        elif t is ctypes.c_float:
            args.append(1.0)
        else:
            args.append(None)
    rc = getattr(L, name)(*args)
    if not (rc < 0 and L.npd_last_error()):
        bad.append((name, rc))
for d in ("npd_code_destroy", "npd_gru_destroy", "npd_conv_destroy"):
    if getattr(L, d)(None) != 0:
        bad.append((d, "destroy(NULL)"))
print("BAD", bad)
sys.exit(1 if bad else 0)
'''
    r = subprocess.run([os.sys.executable, "-c", script, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
