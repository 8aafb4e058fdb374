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


# ---- three-operand subtractions and the point formulas (hlc_point29.hpp) ----
# Largest limbs of a normalised value: mul/sqr outputs (limb 2 < 2^29 + 2^19) and carry-step
# outputs (limb 0 < 2^29 + 2^18, limb 1 < 2^29 + 2^12 + 8, others < 2^29 + 8).
NB = [2**29 + 2**18 - 1, 2**29 + 2**12 + 7, 2**29 + 2**19 - 1] + [2**29 + 7] * 6
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def to_limbs(v):
    return [(v >> (29 * i)) & M for i in range(8)] + [v >> 232]


def nrm_limbs(rnd, n, mode=None):
    """n limb vectors within the normalised bounds NB: random, all-max, or near-max."""
    out = np.zeros((n, 9), np.uint32)
    for k in range(n):
        m = rnd.random() if mode is None else mode
        for i in range(9):
            if m < 0.15:
                out[k, i] = NB[i]
            elif m < 0.4:
                out[k, i] = NB[i] - rnd.randrange(2**12)
            else:
                out[k, i] = rnd.randrange(NB[i] + 1)
    return out


@pytest.fixture()
def checked(lib):
    lib.fe29_violations.restype = ctypes.c_ulonglong
    lib.fe29_violations.argtypes = [ctypes.c_int]
    lib.gej29_op.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.fe29_violations(1)
    yield lib
    assert lib.fe29_violations(1) == 0, "magnitude-contract violation in the checked host build"


def test_sub2_sub_b2c(checked):
    rnd = random.Random(6)
    n = 3000
    a = nrm_limbs(rnd, n)
    a[: n // 3] = limbs(rnd, n // 3, int(2**30.58))        # a up to the 128p headroom
    b, c = nrm_limbs(rnd, n), nrm_limbs(rnd, n)
    bc = np.concatenate([b, c])
    o2 = run(checked, 12, a, bc)
    c3 = nrm_limbs(rnd, n)
    c3[: n // 2] = nrm_limbs(rnd, n // 2, 0.0)
    o3 = run(checked, 13, a, np.concatenate([b, c3]))
    check_normalised(o2)
    check_normalised(o3)
    for k in range(n):
        va, vb, vc, v3 = val(a[k]), val(b[k]), val(c[k]), val(c3[k])
        assert val(o2[k]) % P == (va - vb - vc) % P
        assert val(o3[k]) % P == (va - vb - 2 * v3) % P


def test_muladd_at_bounds(checked):
    """fe29_muladd (a b + c e, one reduction for both products) at the operand bounds of its use in
    the mixed addition's Y3 = R (V - X3) + 2 Y1 (-J): a normalised, b a lazy difference (< 2^30.59),
    c a lazy doubling (< 2^30.01), e normalised -- every limb at its maximum included."""
    rnd = random.Random(61)
    n = 3000
    a, e = nrm_limbs(rnd, n), nrm_limbs(rnd, n)
    b, c = limbs(rnd, n, int(2**30.59)), limbs(rnd, n, 2**30 + 2**19)
    a[0], e[0] = 2**29 + 2**18 - 1, 2**29 + 2**18 - 1
    b[0], c[0] = int(2**30.59) - 1, 2**30 + 2**19 - 1
    o = run(checked, 15, a, np.concatenate([b, c, e]))
    check_normalised(o, 1, 1, rest=0)
    for k in range(n):
        assert val(o[k]) % P == (val(a[k]) * val(b[k]) + val(c[k]) * val(e[k])) % P, k


def jac(x, y, z, inf=0):
    w = np.zeros(28, np.uint32)
    w[0:9], w[9:18], w[18:27], w[27] = x, y, z, inf
    return w


def runp(lib, op, A, B):
    A = np.ascontiguousarray(A, np.uint32)
    B = np.ascontiguousarray(B, np.uint32)
    out = np.zeros((A.shape[0], 37 if op == 3 else 28), np.uint32)
    lib.gej29_op(op, A.shape[0], A.ctypes.data, B.ctypes.data, out.ctypes.data)
    return out


def dbl_textbook(X, Y, Z):
    """dbl-2009-l as polynomials mod p."""
    A, B = X * X % P, Y * Y % P
    C = B * B % P
    D = 2 * ((X + B) ** 2 - A - C) % P
    E = 3 * A % P
    F = E * E % P
    X3 = (F - 2 * D) % P
    return X3, (E * (D - X3) - 8 * C) % P, 2 * Y * Z % P


def madd_textbook(X1, Y1, Z1, x2, y2):
    """madd-2007-bl as polynomials mod p."""
    Z1Z1 = Z1 * Z1 % P
    U2, S2 = x2 * Z1Z1 % P, y2 * Z1 * Z1Z1 % P
    H = (U2 - X1) % P
    HH = H * H % P
    I = 4 * HH % P
    J, r, V = H * I % P, 2 * (S2 - Y1) % P, X1 * I % P
    X3 = (r * r - J - 2 * V) % P
    Y3 = (r * (V - X3) - 2 * Y1 * J) % P
    Z3 = ((Z1 + H) ** 2 - Z1Z1 - HH) % P
    return X3, Y3, Z3


def test_point_formulas_at_limb_bounds(checked):
    """Doubling and mixed addition on arbitrary limb vectors at the normalised bounds (the
    formulas are polynomial maps, so any input tests the arithmetic): values mod p equal the
    textbook formulas, outputs are normalised, and no intermediate breaks the magnitude contract."""
    rnd = random.Random(7)
    n = 1500
    X, Y, Z = nrm_limbs(rnd, n), nrm_limbs(rnd, n), nrm_limbs(rnd, n)
    x2, y2 = nrm_limbs(rnd, n), nrm_limbs(rnd, n)
    A = np.array([jac(X[k], Y[k], Z[k]) for k in range(n)])
    B = np.concatenate([x2, y2], axis=1)
    d = runp(checked, 0, A, B)
    m = runp(checked, 1, A, B)
    mz = runp(checked, 3, A, B)
    for o in (d, m, mz):
        for q in range(3):
            check_normalised(o[:, 9 * q: 9 * q + 9])
    for k in range(n):
        vx, vy, vz = val(X[k]) % P, val(Y[k]) % P, val(Z[k]) % P
        assert tuple(val(d[k, 9 * q: 9 * q + 9]) % P for q in range(3)) == dbl_textbook(vx, vy, vz), k
        want = madd_textbook(vx, vy, vz, val(x2[k]) % P, val(y2[k]) % P)
        assert tuple(val(m[k, 9 * q: 9 * q + 9]) % P for q in range(3)) == want, k
        assert tuple(val(mz[k, 9 * q: 9 * q + 9]) % P for q in range(3)) == want, k
        assert val(mz[k, 28:37]) % P == 2 * ((val(x2[k]) * vz * vz - vx) % P) % P  # zr = 2H


def ec_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def ec_mul(k, pt=(GX, GY)):
    acc = None
    while k:
        if k & 1:
            acc = ec_add(acc, pt)
        pt = ec_add(pt, pt)
        k >>= 1
    return acc


def affine(o):
    if o[27]:
        return None
    z = val(o[18:27]) % P
    if z == 0:
        return "Z=0"
    zi = pow(z, -1, P)
    return val(o[0:9]) * zi * zi % P, val(o[9:18]) * zi * zi * zi % P


def test_point_ops_on_curve_and_exceptional(checked):
    """Group law on real points (random Jacobian Z), the exceptional cases of the exact addition
    (a == b: doubling, a == -b: infinity, a = infinity), and the unchecked addition's zero Z."""
    rnd = random.Random(8)
    rows_a, rows_b, want_d, want_m, kinds = [], [], [], [], []
    for k in range(120):
        p1 = ec_mul(rnd.getrandbits(40) + 1)
        kind = k % 4          # 0: generic, 1: b == a, 2: b == -a, 3: a = infinity
        p2 = ec_mul(rnd.getrandbits(40) + 1) if kind in (0, 3) else (p1 if kind == 1 else (p1[0], P - p1[1]))
        z = rnd.randrange(1, P)
        A = jac(to_limbs(p1[0] * z * z % P), to_limbs(p1[1] * z * z * z % P), to_limbs(z), 1 if kind == 3 else 0)
        rows_a.append(A)
        rows_b.append(np.concatenate([to_limbs(p2[0]), to_limbs(p2[1])]).astype(np.uint32))
        want_d.append(ec_add(p1, p1))
        want_m.append(p2 if kind == 3 else ec_add(p1, p2))
        kinds.append(kind)
    A, B = np.array(rows_a), np.array(rows_b)
    d, me, mf = runp(checked, 0, A, B), runp(checked, 2, A, B), runp(checked, 1, A, B)
    for k in range(len(kinds)):
        if kinds[k] != 3:
            assert affine(d[k]) == want_d[k]
        assert affine(me[k]) == want_m[k], (k, kinds[k])
        if kinds[k] in (1, 2):
            assert affine(mf[k]) == "Z=0"   # unchecked form: the exceptional step leaves Z = 0
        else:
            assert affine(mf[k]) == want_m[k]


def test_point_chains(checked):
    """Natural magnitudes: 40 rounds of (5 doublings, 2 additions) from random points, the shape
    of the u2 R chain, stay within the contract and match the affine group law."""
    rnd = random.Random(9)
    n = 24
    pts = [ec_mul(rnd.getrandbits(32) + 1) for _ in range(n)]
    adds = [ec_mul(rnd.getrandbits(32) + 1) for _ in range(n)]
    A = np.array([jac(to_limbs(p[0]), to_limbs(p[1]), to_limbs(1)) for p in pts])
    B = np.array([np.concatenate([to_limbs(q[0]), to_limbs(q[1])]) for q in adds], np.uint32)
    cur = list(pts)
    for _ in range(40):
        for _ in range(5):
            A = runp(checked, 0, A, B)
            cur = [ec_add(p, p) for p in cur]
        for _ in range(2):
            A = runp(checked, 1, A, B)
            cur = [ec_add(p, q) for p, q in zip(cur, adds)]
    for k in range(n):
        assert affine(A[k]) == cur[k]


def test_coz_addition(checked):
    """gej29_zaddu: (a, b) sharing one Jacobian Z -> (a + b, b) sharing Z (a.x - b.x), the
    R-table build's step (b = 2R, a = (2i-1)R)."""
    rnd = random.Random(10)
    rows_a, rows_b, want = [], [], []
    for _ in range(100):
        k = rnd.getrandbits(40) + 3
        a, b = ec_mul(2 * k - 1), ec_mul(2)
        z = rnd.randrange(1, P)
        z2, z3 = z * z % P, z * z * z % P
        rows_a.append(jac(to_limbs(a[0] * z2 % P), to_limbs(a[1] * z3 % P), to_limbs(0)))
        rows_b.append(np.concatenate([to_limbs(b[0] * z2 % P), to_limbs(b[1] * z3 % P)]).astype(np.uint32))
        want.append((ec_add(a, b), b, z))
    out = runp_coz(checked, np.array(rows_a), np.array(rows_b))
    for k, (s, b, z) in enumerate(want):
        zr = val(out[k, 18:27]) % P
        zn = z * zr % P
        zi = pow(zn, -1, P)
        assert (val(out[k, 0:9]) * zi * zi % P, val(out[k, 9:18]) * zi * zi * zi % P) == s
        assert (val(out[k, 28:37]) * zi * zi % P, val(out[k, 37:46]) * zi * zi * zi % P) == b
        for q in (0, 9, 18, 28, 37):
            check_normalised(out[k:k + 1, q:q + 9])


def runp_coz(lib, A, B):
    out = np.zeros((A.shape[0], 46), np.uint32)
    lib.gej29_op(5, A.shape[0], np.ascontiguousarray(A, np.uint32).ctypes.data,
                 np.ascontiguousarray(B, np.uint32).ctypes.data, out.ctypes.data)
    return out


def test_coz_addition_at_limb_bounds(checked):
    rnd = random.Random(11)
    n = 1500
    ax, ay, bx, by = (nrm_limbs(rnd, n) for _ in range(4))
    A = np.array([jac(ax[k], ay[k], np.zeros(9, np.uint32)) for k in range(n)])
    out = runp_coz(checked, A, np.concatenate([bx, by], axis=1))
    for q in (0, 9, 18, 28, 37):
        check_normalised(out[:, q:q + 9])
    for k in range(n):
        x1, y1, x2, y2 = val(bx[k]), val(by[k]), val(ax[k]), val(ay[k])
        zr = (x2 - x1) % P
        AA = zr * zr % P
        B, C, D = x1 * AA % P, x2 * AA % P, (y2 - y1) ** 2 % P
        E = y1 * (C - B) % P
        X3 = (D - B - C) % P
        Y3 = ((y2 - y1) * (B - X3) - E) % P
        got = [val(out[k, q:q + 9]) % P for q in (0, 9, 18, 28, 37)]
        assert got == [X3, Y3, zr, B, E], k


def test_comb_collision_parity_argument():
    """tests/crypto_items.comb_collisions_possible: with 16-bit windows (2^256 mod n odd) the
    crafted construction exists and its windows really collide; with the shipped 24-bit windows
    (11 of them: 2^264 mod n even, as the 22-bit windows of rounds 1-6) it cannot (the parity
    argument in its docstring)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import crypto_items as ci
    assert ci.COMB_W == 24 and not ci.comb_collisions_possible(24) and not ci.comb_collisions_possible(22)
    assert ci.comb_collisions_possible(16)


K64 = [0x3FFF0BC0, 0x3FFFFDFE] + [0x3FFFFFFE] * 7   # 64p's limbs: bound of a lazily negated y


def lazy_limbs(rnd, n):
    out = np.zeros((n, 9), np.uint32)
    for k in range(n):
        m = rnd.random()
        for i in range(9):
            out[k, i] = K64[i] if m < 0.2 else (K64[i] - rnd.randrange(2**12) if m < 0.4 else rnd.randrange(K64[i] + 1))
    return out


def test_cneg_lazy(checked):
    rnd = random.Random(12)
    a = nrm_limbs(rnd, 3000)
    c = np.zeros((3000, 9), np.uint32)
    c[:, 0] = [rnd.randrange(2) for _ in range(3000)]
    o = run(checked, 14, a, c)
    assert (o <= np.array(K64, np.uint32)).all()
    for k in range(3000):
        assert val(o[k]) % P == ((-val(a[k])) if c[k, 0] else val(a[k])) % P


def test_point_formulas_with_lazy_y(checked):
    """The chains add table entries whose y went through fe29_cneg_lazy (limbs up to 64p's), and
    an accumulator started from such an entry carries a lazy y into the next doublings and
    additions: doubling and both additions at those bounds."""
    rnd = random.Random(13)
    n = 1500
    X, Z, x2 = nrm_limbs(rnd, n), nrm_limbs(rnd, n), nrm_limbs(rnd, n)
    Y, y2 = lazy_limbs(rnd, n), lazy_limbs(rnd, n)
    A = np.array([jac(X[k], Y[k], Z[k]) for k in range(n)])
    B = np.concatenate([x2, y2], axis=1)
    d, m, me = runp(checked, 0, A, B), runp(checked, 1, A, B), runp(checked, 2, A, B)
    for o in (d, m):
        for q in range(3):
            check_normalised(o[:, 9 * q: 9 * q + 9])
    for k in range(n):
        vx, vy, vz = val(X[k]) % P, val(Y[k]) % P, val(Z[k]) % P
        assert tuple(val(d[k, 9 * q: 9 * q + 9]) % P for q in range(3)) == dbl_textbook(vx, vy, vz), k
        want = madd_textbook(vx, vy, vz, val(x2[k]) % P, val(y2[k]) % P)
        assert tuple(val(m[k, 9 * q: 9 * q + 9]) % P for q in range(3)) == want, k
        if want[2] % P:
            assert tuple(val(me[k, 9 * q: 9 * q + 9]) % P for q in range(3)) == want, k
    # infinity accumulator + lazy entry: the exact form copies the lazy y into the accumulator
    Ai = A.copy()
    Ai[:, 27] = 1
    mi = runp(checked, 2, Ai, B)
    assert (mi[:, 9:18] == y2).all() and (mi[:, 27] == 0).all()


def test_muladd_doubling_bounds(checked):
    """fe29_muladd at the operands of the doubling's Y3 = E (D - X3) + 4B (-2B) (hlc_point29.hpp
    gej29_double), its tightest use: E normalised, t = D - X3 a lazy difference (< 2^30.59), 4B a
    doubled doubling of a normalised B (limbs up to 4 x the normalised maxima: 2^31 + 2^21 at limb
    2), -2B normalised -- with every limb of every operand at its maximum in the first rows."""
    rnd = random.Random(62)
    n = 3000
    a, e = nrm_limbs(rnd, n), nrm_limbs(rnd, n)
    b = limbs(rnd, n, int(2**30.59))
    B = nrm_limbs(rnd, n)
    c = (4 * B.astype(np.uint64)).astype(np.uint32)  # 4B, lazy
    a[:3] = NB
    e[:3] = NB
    b[:3] = int(2**30.59) - 1
    c[:3] = [4 * x for x in NB]
    o = run(checked, 15, a, np.concatenate([b, c, e]))
    check_normalised(o, 1, 1, rest=0)
    for k in range(n):
        assert val(o[k]) % P == (val(a[k]) * val(b[k]) + val(c[k]) * val(e[k])) % P, k


def test_mul_add_sqr_add_at_bounds(checked):
    """fe29_mul_add / fe29_sqr_add (a product and the subtraction after it with one reduction: the
    doubling's X3 = E^2 + (128p - 2D), the mixed addition's H = x2 Z1^2 + (128p - X1) and X3, the co-Z
    X3 / Y3): mul / sqr operands up to their bound, the addend 128p - b - c of two normalised values
    (fe29_neg_addend) at its largest (b = c = 0) and smallest (b, c at the normalised maxima)."""
    rnd = random.Random(63)
    n = 3000
    a, b = limbs(rnd, n, MUL_IN), limbs(rnd, n, MUL_IN)
    a[:2] = MUL_IN - 1
    b[:2] = MUL_IN - 1
    sb, sc = nrm_limbs(rnd, n), nrm_limbs(rnd, n)
    sb[0] = sc[0] = 0
    sb[1] = sc[1] = NB
    f = run(checked, 18, sb, sc)
    o = run(checked, 16, a, np.concatenate([b, f]))
    q = run(checked, 17, a, f)
    check_normalised(o, 1, 1, rest=0)
    check_normalised(q, 1, 1, rest=0)
    for k in range(n):
        fv = val(f[k])
        assert fv % P == (-val(sb[k]) - val(sc[k])) % P, k
        assert val(o[k]) % P == (val(a[k]) * val(b[k]) + fv) % P, k
        assert val(q[k]) % P == (val(a[k]) ** 2 + fv) % P, k
