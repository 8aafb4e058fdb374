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


def _mont_ref(a: int, b: int) -> int:
    """What the 8 x 32 CIOS form returned (and hlc_scmul.hpp must): t = (a b + M n) / 2^256,
    M = -a b n^-1 mod 2^256, then t - n when t >= n (one conditional subtract, any a, b < 2^256)."""
    R = 1 << 256
    m = (-a * b * pow(N, -1, R)) % R
    t = (a * b + m * N) >> 256
    return t - N if t >= N else t


def test_sc_mont_mul29_matches_the_cios_form():
    """csrc/hlc_scmul.hpp sc_mont_mul29 (the recovery's products mod n since round 6) against the
    Montgomery product it replaced, bit for bit: random scalars, the edges of [0, n) and inputs
    >= n up to 2^256 - 1 (the form is defined for any 256-bit operands)."""
    lib = ctypes.CDLL(LIB)
    lib.hlc_sc_mont_mul_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    rnd = random.Random(29)
    edge = [0, 1, 2, N - 1, N - 2, N, N + 1, 2**256 - 1, 2**255, 2**232 - 1, 2**232, (N - 1) // 2,
            2**29 - 1, 2**261 % N, 2**256 % N]
    pairs = [(x, y) for x in edge for y in edge]
    pairs += [(rnd.randrange(N), rnd.randrange(N)) for _ in range(20000)]
    pairs += [(rnd.randrange(2**256), rnd.randrange(2**256)) for _ in range(5000)]
    pairs += [(rnd.randrange(N), (1 << rnd.randrange(256)) - 1) for _ in range(2000)]

    def words(vals):
        arr = np.zeros((len(vals), 8), np.uint32)
        for i, v in enumerate(vals):
            for k in range(8):
                arr[i, k] = (v >> (32 * k)) & 0xFFFFFFFF
        return arr
    a, b = words([p[0] for p in pairs]), words([p[1] for p in pairs])
    out = np.zeros_like(a)
    lib.hlc_sc_mont_mul_host(a.ctypes.data, b.ctypes.data, out.ctypes.data, len(pairs))
    got = [sum(int(out[i, k]) << (32 * k) for k in range(8)) for i in range(len(pairs))]
    bad = [(hex(x), hex(y)) for (x, y), g in zip(pairs, got) if g != _mont_ref(x, y)]
    assert not bad, f"{len(bad)} wrong products, e.g. {bad[0]}"
