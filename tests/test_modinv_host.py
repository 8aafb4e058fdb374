"""The device-shared safegcd inversion (csrc/hlc_modinv.hpp) built for the host and checked
against Python's pow(a, -1, m) -- host logic of the product, no GPU."""
import ctypes
import os
import random

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hashgraph-like-consensus_amd", "lib", "libhlc_modinv_host.so")
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _run(vals, which):
    lib = ctypes.CDLL(LIB)
    lib.hlc_modinv_host.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    a = np.zeros((len(vals), 8), np.uint32)
    for i, v in enumerate(vals):
        for k in range(8):
            a[i, k] = (v >> (32 * k)) & 0xFFFFFFFF
    out = np.zeros_like(a)
    lib.hlc_modinv_host(a.ctypes.data, which, out.ctypes.data, len(vals))
    return [sum(int(out[i, k]) << (32 * k) for k in range(8)) for i in range(len(vals))]


def test_safegcd_inverse_mod_p_and_n():
    rnd = random.Random(7)
    for which, m in ((0, P), (1, N)):
        vals = [1, 2, 3, m - 1, m - 2, 2**255 % m, m // 2, 2**128, 2**30, 2**30 - 1, 2**32 - 1]
        vals += [rnd.randrange(1, m) for _ in range(20000)]
        # adversarial-ish: long runs of ones / zeros in binary
        vals += [(2**k - 1) % m for k in range(1, 256, 5)] + [2**k % m for k in range(0, 256, 3)]
        vals = [v for v in vals if v % m]
        got = _run(vals, which)
        bad = [v for v, r in zip(vals, got) if r != pow(v, -1, m)]
        assert not bad, f"modulus {which}: {len(bad)} wrong inverses, e.g. {hex(bad[0])}"
