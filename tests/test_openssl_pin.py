"""Byte-level pin of the crypto slice against an independent implementation: OpenSSL libcrypto
(tests/openssl_ec.py).  CPU only.

The reference holds no byte-level vectors (keys are random in
/root/reference/tests/common/mod.rs:20-30), so the oracle's SHA-256 (utils.rs:37-47), its
secp256k1 recovery (ethereum.rs:86-89) and its address derivation were pinned in round 1 only by a
few published vectors and by two in-repo restatements agreeing.  Here every recovery, square root,
inversion and point multiplication is recomputed by OpenSSL:
  * recovered key: OpenSSL's u1 G + u2 R equals the oracle's, address for address, and the scheme
    error class agrees on every adversarial item;
  * ECDSA_do_verify accepts (r, normalized s) under the recovered key (k256's post-recovery
    verify, which the GPU omits as redundant);
  * Address = keccak256(X || Y)[12..] over OpenSSL-derived public keys of random private keys;
  * SHA-256 of the oracle == OpenSSL SHA256 == hashlib over every length 0..300.
"""
import hashlib
import os
import random

import numpy as np
import pytest

import coracle
import pyoracle as po
from crypto_items import KINDS, make_items

openssl_ec = pytest.importorskip("openssl_ec")
if not openssl_ec.available():  # pragma: no cover
    pytest.skip("libcrypto not loadable", allow_module_level=True)

N_ITEMS = int(os.environ.get("HLC_OPENSSL_ITEMS", "10000"))


@pytest.fixture(scope="module")
def ec():
    e = openssl_ec.Secp256k1()
    yield e
    e.close()


@pytest.fixture(scope="module")
def items():
    return make_items(N_ITEMS, 0x5EC9)


def test_sha256_matches_openssl_every_length():
    rnd = random.Random(1)
    for n in list(range(0, 301)) + [1000, 4096, 65537]:
        b = bytes(rnd.randrange(256) for _ in range(n))
        want = openssl_ec.sha256(b)
        assert want == hashlib.sha256(b).digest()
        assert coracle.sha256(b) == want, n


def test_addresses_of_openssl_pubkeys(ec):
    rnd = random.Random(2)
    privs = [1, 2, 3, po.N - 1, po.N - 2, (po.N - 1) // 2] + [rnd.randrange(1, po.N) for _ in range(2000)]
    keys = np.stack([np.frombuffer(d.to_bytes(32, "big"), np.uint8) for d in privs])
    addr = coracle.address_batch(keys, threads=8)
    for i, d in enumerate(privs):
        pub = ec.pubkey(d.to_bytes(32, "big"))
        assert coracle.keccak256(pub)[12:] == addr[i].tobytes(), hex(d)
    # the published key-1 address, through OpenSSL's point
    assert coracle.keccak256(ec.pubkey((1).to_bytes(32, "big")))[12:].hex() == \
        "7e5f4552091a69125d5dfcb7b8c2659029395bdf"


def test_recovery_matches_openssl(ec, items):
    seen = {k: set() for k in KINDS}
    mism = []
    for it in items:
        code_c, addr_c = coracle.ecrecover(it.prehash, it.sig)
        code_o, pub = ec.recover(it.prehash, it.sig)
        seen[it.kind].add(code_o)
        if code_c != code_o or (code_o == 0 and coracle.keccak256(pub)[12:] != addr_c):
            mism.append((it.kind, code_c, code_o))
            continue
        if code_o == 0:
            # k256's post-recovery verify_prehash, restated by OpenSSL: (r, normalized s) under Q
            s = int.from_bytes(it.sig[32:64], "big")
            s = po.N - s if s > po.N // 2 else s
            assert ec.ecdsa_verify(it.prehash, it.sig[:32], s.to_bytes(32, "big"), pub), it.kind
    assert not mism, f"{len(mism)} of {len(items)} differ from OpenSSL, first {mism[:5]}"
    # the valid and high-s items recover the signer; every error class is exercised
    assert seen["valid"] == {0} and seen["high_s"] == {0} and seen["eip155_v"] == {0}
    assert seen["bad_v"] == {po.SCHEME_BAD_PARITY}
    assert seen["no_point"] == {po.SCHEME_NO_POINT}
    assert seen["infinity"] == {po.SCHEME_INFINITY}
    assert po.SCHEME_SCALAR_RANGE in seen["r_range"] and po.SCHEME_SCALAR_RANGE in seen["s_range"]


def test_valid_items_recover_the_signer(ec, items):
    """The signer's own key comes back (sign -> recover round trip through OpenSSL)."""
    for it in items[:500]:
        if it.kind not in ("valid", "high_s", "eip155_v"):
            continue
        code, pub = ec.recover(it.prehash, it.sig)
        assert code == 0 and pub == ec.pubkey(it.priv.to_bytes(32, "big"))


def test_glv_baseline_matches_checker_and_openssl(ec, items):
    """The k256-class recovery the CPU baseline times (GLV + wNAF + binary-GCD inversions,
    coracle glv=True) equals the independent non-GLV checker and OpenSSL on every item, and its
    post-recovery verify (k256's verify_prehash) never fails."""
    before = coracle.verify_failures()
    for it in items[:4000]:
        code_g, addr_g = coracle.ecrecover(it.prehash, it.sig, reverify=True, glv=True)
        code_c, addr_c = coracle.ecrecover(it.prehash, it.sig, reverify=False)
        assert (code_g, addr_g) == (code_c, addr_c), it.kind
        code_o, pub = ec.recover(it.prehash, it.sig)
        assert code_g == code_o and (code_o != 0 or coracle.keccak256(pub)[12:] == addr_g), it.kind
    assert coracle.verify_failures() == before
