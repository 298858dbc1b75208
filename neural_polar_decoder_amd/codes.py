"""Code construction (host logic): information / frozen sets for Polar and PAC codes.

Restates the reference's rate profiles:
  * PolarCode.__init__ with ``rs`` or ``F`` (polar.py:66-117)
  * rnn_all.get_code rate profiles 'polar', 'RM', 'rev_RM', 'custom', 'sorted', 'sorted_last',
    'rev_polar', 'random' (rnn_all.py:1015-1196; run_models.py:620-660 for 'polar'/'RM')
  * PAC rate_profiler 'RM', 'rev_RM', 'sorted', 'sorted_last', 'last', 'freeze_even', 'freeze_odd'
    (pac_code.py:121-174)
The information sets are pinned against the reference by tests/golden/codes.npz.
"""
from __future__ import annotations

import numpy as np

# Reliability order (most reliable first) of the 256-length polar sequence used by the reference
# ("computed for SNR = 0"), zero-based (run_models.py:630, rnn_all.py get_code, polar.py:1173).
RELIABILITY_256 = np.array([
    255, 254, 251, 253, 247, 223, 239, 191, 127, 252, 243, 250, 249, 238, 237, 246, 245, 222, 221, 231, 215, 235, 219, 187, 207, 183, 190, 189, 175, 126, 125, 123,
    119, 248, 244, 242, 241, 159, 230, 229, 236, 234, 233, 111, 227, 220, 218, 217, 211, 214, 213, 188, 186, 95, 185, 206, 205, 182, 181, 203, 179, 199, 63, 174,
    173, 171, 124, 122, 121, 118, 158, 117, 157, 167, 240, 115, 110, 232, 155, 109, 228, 226, 216, 107, 212, 151, 225, 94, 210, 93, 204, 184, 103, 209, 202, 180,
    91, 143, 201, 178, 198, 172, 177, 62, 197, 120, 170, 87, 61, 116, 169, 195, 156, 166, 59, 114, 154, 108, 165, 79, 113, 153, 106, 55, 224, 150, 163, 105,
    92, 149, 208, 102, 90, 142, 200, 101, 47, 147, 176, 89, 141, 196, 86, 99, 60, 168, 194, 139, 85, 58, 31, 164, 193, 112, 78, 57, 152, 83, 135, 54,
    162, 77, 104, 148, 161, 53, 75, 100, 46, 146, 88, 51, 140, 98, 45, 145, 71, 84, 138, 97, 30, 43, 192, 137, 56, 82, 29, 134, 76, 39, 81, 133,
    160, 27, 52, 74, 131, 23, 50, 73, 44, 144, 70, 49, 15, 96, 69, 42, 136, 67, 41, 28, 38, 80, 26, 132, 37, 25, 35, 130, 22, 72, 21, 129,
    48, 14, 19, 68, 13, 11, 66, 40, 7, 65, 36, 24, 34, 33, 20, 128, 18, 12, 17, 10, 9, 6, 64, 5, 3, 32, 16, 8, 4, 2, 1, 0,
], dtype=np.int64)


def count_set_bits(n: int) -> int:
    return bin(int(n)).count("1")


def rm_weight(N: int) -> np.ndarray:
    return np.array([count_set_bits(i) for i in range(N)])


def polar_rs(N: int) -> np.ndarray:
    return RELIABILITY_256[RELIABILITY_256 < N].copy()


def info_from_rs(rs: np.ndarray, K: int) -> np.ndarray:
    """PolarCode(rs=...): info = sort(rs[:K]) (polar.py:92-108)."""
    return np.sort(np.asarray(rs)[:K]).astype(np.int64)


def info_from_frozen(N: int, F) -> np.ndarray:
    """PolarCode(F=...): info = complement of F (polar.py:80-87)."""
    F = set(int(f) for f in np.asarray(F).ravel())
    return np.array(sorted(set(range(N)) - F), dtype=np.int64)


def polar_info_positions(N: int, K: int, rate_profile: str = "polar", target_K: int | None = None,
                         random_seed: int = 42, info_ind: int | None = None) -> np.ndarray:
    """Sorted information positions of the reference's Polar rate profiles (rnn_all.py:1015-1196)."""
    tK = K if target_K is None else target_K
    if rate_profile == "polar":
        return info_from_rs(polar_rs(N), K)
    if rate_profile == "RM":
        Fr = np.argsort(rm_weight(N))[:-K] if K > 0 else np.arange(N)
        return info_from_frozen(N, Fr)
    if rate_profile == "rev_RM":
        wts = np.argsort(rm_weight(N))
        Fr = np.concatenate([wts[:-tK], wts[N - tK + K:]])
        return info_from_frozen(N, Fr)
    if rate_profile == "custom":
        if info_ind is None:
            raise ValueError("rate_profile 'custom' needs info_ind")
        return np.array([int(info_ind)], dtype=np.int64)
    rs = polar_rs(N)
    first = rs[:tK].copy()
    if rate_profile == "sorted":
        first.sort()
        rs[:tK] = first
    elif rate_profile == "sorted_last":
        first.sort()
        rs[:tK] = first[::-1]
    elif rate_profile == "rev_polar":
        rs[:tK] = first[::-1]
    elif rate_profile == "random":
        rs[:tK] = np.random.RandomState(seed=random_seed).permutation(first)
    else:
        raise ValueError(f"unknown polar rate profile {rate_profile!r}")
    return info_from_rs(rs, K)


def pac_info_positions(N: int, K: int, scheme: str = "RM", target_K: int | None = None) -> np.ndarray:
    """PAC rate profiler set B (pac_code.py:121-174).  'RM' uses np.argsort of the row weights exactly
    as the reference does; where K splits a weight class the tie order is numpy's (as in the
    reference run on the same host)."""
    tK = N // 2 if target_K is None else target_K
    w = rm_weight(N)
    if scheme == "RM":
        B = np.argsort(w)[-K:]
    elif scheme == "rev_RM":
        B = np.argsort(w)[-tK:][:K].copy()
    elif scheme == "sorted":
        B = np.sort(np.argsort(w)[-int(tK):])[:K]
    elif scheme == "sorted_last":
        B = np.sort(np.argsort(w)[-int(tK):])[-K:]
    elif scheme == "last":
        B = np.arange(N - 1, N - K - 1, -1)
    elif scheme == "freeze_even":
        B = np.arange(N - 1, -1, -2)
    elif scheme == "freeze_odd":
        B = np.arange(N - 2, -1, -2)
    else:
        raise ValueError(f"unsupported PAC rate profile {scheme!r} (polar/custom need data files absent from the reference)")
    return np.sort(np.asarray(B)).astype(np.int64)


def pac_default_g(N: int) -> int:
    """The PAC convolution polynomial the reference's scripts use for length N: rnn_all.py:218-235, run_models.py:197-213
    and rnn.py:224-240 overwrite --g from N (7, 13, 21, 53 at N = 4, 8, 16, 32; 91 otherwise)."""
    return {4: 7, 8: 13, 16: 21, 32: 53}.get(int(N), 91)
