"""Random and adversarial (payload, prehash, signature) items for the crypto pin tests
(tests/test_openssl_pin.py on the CPU, tests/test_gpu_openssl_pin.py through the C ABI).

Every item is a message signed by EthereumConsensusSigner::sign semantics (RFC 6979, low s,
v = 27 + parity; /root/reference/src/signing/ethereum.rs:58-64, signed here by the C oracle), then
optionally mutated into one of the edge classes that /root/reference/src/signing/ethereum.rs:86-89
must reject or accept (Appendix C of SURVEY.md).  TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import List

import numpy as np

import coracle
import pyoracle as po

KINDS = ["valid", "flip_rs", "bad_v", "eip155_v", "high_s", "r_range", "s_range", "no_point", "infinity"]


@dataclass
class Item:
    priv: int
    payload: bytes
    prehash: bytes
    sig: bytes
    kind: str


def _no_point_r(rnd: random.Random) -> int:
    while True:
        r = rnd.randrange(1, po.N)
        if po.decompress(r, False) is None:
            return r


_EC = []


def _kg(k: int):
    """Affine k G (input construction only): OpenSSL when loadable, else the Python oracle."""
    try:
        import openssl_ec
        if not _EC and openssl_ec.available():
            _EC.append(openssl_ec.Secp256k1())
        if _EC:
            pub = _EC[0].pubkey(k.to_bytes(32, "big"))
            return int.from_bytes(pub[:32], "big"), int.from_bytes(pub[32:], "big")
    except OSError:
        pass
    return po.point_mul(k, po.G)


COMB_W = 24                                  # HLC_GC_W of the default build (hlc_recover.hpp)
COMB_N = (255 + COMB_W - 1) // COMB_W        # windows; the top value is 1 at 2^(W N)


def comb_collisions_possible(w: int = COMB_W) -> bool:
    """Whether any u1 can make the comb add a point equal to +- its accumulator.  Before window
    j the accumulator is 2^(W N) + L_j (mod n) with L_j odd and |L_j| < 2^(W j); it would have
    to equal +- d_j 2^(W j) (even, < 2^(W (j+1)) << n).  As integers that needs
    (2^(W N) mod n) + L_j = d_j 2^(W j): odd + odd = even only when 2^(W N) mod n is odd.  For
    W = 16 (2^256 mod n, odd) collisions are constructible (`_comb_collision_sig`); for the
    shipped W = 24 (11 windows: 2^264 mod n, even; so was W = 22 through round 6) none exists, u1 = 0 aside (k = n: unreachable, it needs
    a prehash == 0 mod n)."""
    n_win = (255 + w - 1) // w
    return pow(2, w * n_win, po.N) & 1 == 1


def _comb_recode(k: int):
    """The u1 G comb's regular recoding (hlc_recover.hpp comb_digit): COMB_N odd digits of COMB_W
    bits, least significant first, and the top value (1)."""
    ds = []
    for _ in range(COMB_N):
        d = (k & ((2 << COMB_W) - 1)) - (1 << COMB_W)
        k = (k - d) >> COMB_W
        ds.append(d)
    return ds, k


def comb_exceptional_window(k: int):
    """First comb window whose addition is exceptional (accumulator == +- the added multiple of
    G), or None.  The comb starts from 2^(W N) G and adds d_w 2^(W w) G, w = 0..N-1."""
    ds, top = _comb_recode(k)
    acc = top << (COMB_W * COMB_N)
    for w, d in enumerate(ds):
        e = d << (COMB_W * w)
        if (acc - e) % po.N == 0 or (acc + e) % po.N == 0:
            return w
        acc += e
    return None


def _comb_collision_sig(z: int, rnd: random.Random) -> bytes:
    """A crafted signature whose u1 = -z/r makes the device's u1 G comb hit an exceptional
    addition (the accumulator equals the added point: a doubling inside the chain).  The
    partial sum before window w is 2^(W N) + L_w = delta + L_w (mod n), delta = 2^(W N) mod n
    (~2^137); choosing the low digits L_w = 2^(W w) - delta and d_w = 1 makes it equal
    d_w 2^(W w).  r = -z / u1 follows (retried until r is an x-coordinate).  The result is
    whatever the exact group law gives -- the point is that every implementation must agree."""
    assert comb_collisions_possible(), "no comb collision exists for this window width"
    delta = pow(2, COMB_W * COMB_N, po.N)
    w_lo = (delta.bit_length() + COMB_W) // COMB_W
    while True:
        w = rnd.randrange(w_lo, COMB_N - 1)
        hb = 256 - COMB_W * (w + 1) - 1
        k = (1 << (COMB_W * w)) - delta + (1 << (COMB_W * w)) + ((rnd.getrandbits(hb) if hb > 0 else 0) << (COMB_W * (w + 1)))
        if not k & 1 or k >= po.N or comb_exceptional_window(k) is None:
            continue
        r = (-z * pow(k, -1, po.N)) % po.N  # u1 = k (odd: the comb's own representative)
        parity = rnd.randrange(2)
        if r == 0 or po.decompress(r, bool(parity)) is None:
            continue
        s = rnd.randrange(1, po.N // 2)
        return r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([27 + parity])


def make_items(n: int, seed: int) -> List[Item]:
    rnd = random.Random(seed)
    privs = [rnd.randrange(1, po.N) for _ in range(n)]
    pays = [bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 200))) for _ in range(n)]
    pre = np.stack([np.frombuffer(coracle.eip191_hash(p), np.uint8) for p in pays])
    keys = np.stack([np.frombuffer(d.to_bytes(32, "big"), np.uint8) for d in privs])
    sigs = coracle.sign_batch(keys, pre, threads=8)
    items = []
    for i in range(n):
        kind = KINDS[i % len(KINDS)]
        sig = bytearray(sigs[i].tobytes())
        z = int.from_bytes(pre[i].tobytes(), "big") % po.N
        if kind == "flip_rs":
            sig[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
        elif kind == "bad_v":
            sig[64] = rnd.choice([2, 3, 26, 29, 30, 34])
        elif kind == "eip155_v":  # chain-id style v >= 35: parity (v - 35) % 2
            par = sig[64] - 27
            sig[64] = 35 + 2 * rnd.randrange(0, 100) + par
        elif kind == "high_s":  # must still be accepted (alloy normalized_s)
            s = int.from_bytes(sig[32:64], "big")
            sig[32:64] = (po.N - s).to_bytes(32, "big")
            sig[64] = 55 - sig[64]
        elif kind == "r_range":
            sig[0:32] = rnd.choice([0, po.N, po.N + 1, 2**256 - 1]).to_bytes(32, "big")
        elif kind == "s_range":
            sig[32:64] = rnd.choice([0, po.N, 2**256 - 1, po.N // 2 + 1]).to_bytes(32, "big")
        elif kind == "no_point":
            sig[0:32] = _no_point_r(rnd).to_bytes(32, "big")
        elif kind == "infinity":  # R = kG, s = z / k  =>  Q = r^-1 (s R - z G) = infinity
            k = rnd.randrange(1, po.N)
            rx, ry = _kg(k)
            r = rx % po.N
            s = z * pow(k, -1, po.N) % po.N or 1
            sig = bytearray(r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([27 + (ry & 1)]))
        items.append(Item(privs[i], pays[i], pre[i].tobytes(), bytes(sig), kind))
    return items
