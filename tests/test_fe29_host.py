"""The 29-bit unsaturated field layer (hashgraph-like-consensus_amd/csrc/hlc_fe29.hpp), compiled for
the host, against Python integers: every operation, at random values AND at the limb-magnitude
bounds of its contract, with the output bounds the next operation relies on.  CPU only.

(The arithmetic it implements is the base field of k256 0.13.4's FieldElement, the recovery
behind /root/reference/src/signing/ethereum.rs:89.)"""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hashgraph-like-consensus_amd", "lib", "libhlc_fe29_host.so")
P = 2**256 - 2**32 - 977
M = 2**29 - 1
MUL_IN = int(2**30.35)          # mul / sqr input limb bound
ADD_IN = 2**29 + 2**18          # largest limb of a normalised value
SUB_IN = int(2**30.4)           # sub / neg input limb bound


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "hashgraph-like-consensus_amd"),
                        "lib/libhlc_fe29_host.so"], check=True)
    L = ctypes.CDLL(LIB)
    L.fe29_op.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L


def val(limbs) -> int:
    return sum(int(x) << (29 * i) for i, x in enumerate(limbs))


def run(lib, op, a, b=None):
    a = np.ascontiguousarray(a, np.uint32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), np.uint32)
    out = np.zeros((a.shape[0], 9), np.uint32)
    lib.fe29_op(op, a.shape[0], a.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out


def limbs(rnd, n, hi, extreme_frac=0.3):
    out = np.zeros((n, 9), np.uint32)
    for k in range(n):
        mode = rnd.random()
        for i in range(9):
            if mode < extreme_frac:
                out[k, i] = hi - 1 - rnd.randrange(4)
            elif mode < extreme_frac + 0.1:
                out[k, i] = rnd.choice([0, 1, hi - 1])
            else:
                out[k, i] = rnd.randrange(hi)
    return out


def check_normalised(o, extra0=2**18, extra1=2**12 + 8, extra2=2**19 + 2**13, rest=8):
    """mul / sqr outputs: limbs < 2^29 except limb 2 (< 2^29 + 2^19); sub / neg / mul_small
    (one parallel carry step): limbs < 2^29 + 8, limb 0 < 2^29 + 2^18, limb 1 < 2^29 + 2^12 + 8."""
    assert (o[:, 0] < 2**29 + extra0).all() and (o[:, 1] < 2**29 + extra1).all()
    assert (o[:, 2] < 2**29 + extra2).all() and (o[:, 3:] < 2**29 + rest).all()


def test_mul_sqr_at_bounds(lib):
    rnd = random.Random(1)
    a, b = limbs(rnd, 4000, MUL_IN), limbs(rnd, 4000, MUL_IN)
    a[0] = MUL_IN - 1
    b[0] = MUL_IN - 1
    o = run(lib, 0, a, b)
    s = run(lib, 1, a)
    for k in range(a.shape[0]):
        x, y = val(a[k]), val(b[k])
        assert val(o[k]) % P == x * y % P, k
        assert val(s[k]) % P == x * x % P, k
    check_normalised(o, 1, 1, rest=0)
    check_normalised(s, 1, 1, rest=0)


def test_add_sub_neg_small(lib):
    rnd = random.Random(2)
    a, b = limbs(rnd, 3000, ADD_IN), limbs(rnd, 3000, ADD_IN)
    o = run(lib, 2, a, b)
    assert (o < MUL_IN).all()
    for k in range(a.shape[0]):
        assert val(o[k]) == val(a[k]) + val(b[k])
    a, b = limbs(rnd, 3000, SUB_IN), limbs(rnd, 3000, SUB_IN)
    d = run(lib, 3, a, b)
    n = run(lib, 4, a)
    check_normalised(d)
    check_normalised(n)
    for k in range(a.shape[0]):
        assert val(d[k]) % P == (val(a[k]) - val(b[k])) % P, k
        assert val(n[k]) % P == (-val(a[k])) % P, k
    for m in (1, 2, 3, 4):
        a = limbs(rnd, 800, int(2**29.5))
        mm = np.full((a.shape[0], 9), m, np.uint32)
        o = run(lib, 5, a, mm)
        check_normalised(o)
        for k in range(a.shape[0]):
            assert val(o[k]) % P == m * val(a[k]) % P


def test_normalize_and_zero(lib):
    rnd = random.Random(3)
    a = limbs(rnd, 3000, SUB_IN)
    extra = []
    # multiples of p and values next to them, in lazy limb layouts
    for mult in (0, 1, 2, 3, 31):
        for delta in (0, 1, -1, 977, 2**32):
            v = mult * P + delta
            if v < 0 or v >= 2**261:
                continue
            d = [(v >> (29 * i)) & M for i in range(8)] + [v >> 232]
            # move one unit of limb i+1 into limb i (lazy layout) where possible
            for i in range(8):
                if d[i + 1] > 0 and d[i] + 2**29 < SUB_IN:
                    d[i + 1] -= 1
                    d[i] += 2**29
                    break
            extra.append(d)
    a = np.concatenate([a, np.array(extra, np.uint32)])
    o = run(lib, 6, a)
    z = run(lib, 7, a)
    for k in range(a.shape[0]):
        v = val(a[k])
        assert val(o[k]) == v % P and (o[k] < 2**29).all(), k
        assert bool(z[k, 0]) == (v % P == 0), k


def test_conversions_round_trip(lib):
    rnd = random.Random(4)
    ws = [[rnd.getrandbits(32) for _ in range(8)] for _ in range(2000)]
    ws += [[0xFFFFFFFF] * 8, [0] * 8, [0xFFFFFC2F, 0xFFFFFFFE] + [0xFFFFFFFF] * 6]  # 2^256-1, 0, p
    w9 = np.zeros((len(ws), 9), np.uint32)
    w9[:, :8] = np.array(ws, np.uint32)
    f = run(lib, 8, w9)
    back = run(lib, 9, f)
    for k, w in enumerate(ws):
        x = sum(int(v) << (32 * i) for i, v in enumerate(w))
        assert val(f[k]) == x
        assert sum(int(v) << (32 * i) for i, v in enumerate(back[k, :8])) == x % P


def test_lazy_subtraction_chains(lib):
    """The lazy patterns of hlc_point29.hpp: (a - b) lazy x normalised, (a - b - c) then one carry,
    2 (a - b) with carry, and the bounds each step promises."""
    rnd = random.Random(5)
    n = 3000
    nrm = lambda: limbs(rnd, n, ADD_IN)       # normalised operands (largest limbs)
    a, b, c, e = nrm(), nrm(), nrm(), nrm()
    l1 = run(lib, 10, a, b)                    # a - b + 64p
    assert (l1 < int(2**30.59)).all()
    m = run(lib, 0, l1, e)                     # lazy x normalised
    l2 = run(lib, 10, l1, c)                   # (a - b) - c, still lazy (< 2^31.35)
    assert (l2 < int(2**31.35)).all()
    z = run(lib, 11, l2)
    d = run(lib, 5, l1, np.full((n, 9), 2, np.uint32))   # 2 (a - b), normalised
    check_normalised(z)
    check_normalised(d)
    check_normalised(m, 1, 1, rest=0)
    for k in range(n):
        va, vb, vc, ve = val(a[k]), val(b[k]), val(c[k]), val(e[k])
        assert val(l1[k]) % P == (va - vb) % P
        assert val(m[k]) % P == (va - vb) * ve % P
        assert val(z[k]) % P == (va - vb - vc) % P
        assert val(d[k]) % P == 2 * (va - vb) % P
