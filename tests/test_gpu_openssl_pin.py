"""GPU recovery pinned directly against OpenSSL libcrypto (an implementation independent of both
in-repo restatements): `hlc_eth_verify_batch` (EthereumConsensusSigner::verify,
/root/reference/src/signing/ethereum.rs:66-97) over 10k random and adversarial signatures must
return, item for item, the address OpenSSL recovers (or the same scheme error class)."""
import numpy as np
import pytest

import coracle
from crypto_items import make_items

pytestmark = pytest.mark.gpu

openssl_ec = pytest.importorskip("openssl_ec")


def test_gpu_recovery_equals_openssl(engine):
    if not openssl_ec.available():
        pytest.skip("libcrypto not loadable")
    ec = openssl_ec.Secp256k1()
    try:
        items = make_items(10_000, 0x6A1)
        owners = [coracle.keccak256(ec.pubkey(it.priv.to_bytes(32, "big")))[12:] for it in items]
        st, addr = engine.eth_verify_batch(owners, [it.payload for it in items], [it.sig for it in items])
        bad = []
        for i, it in enumerate(items):
            code, pub = ec.recover(it.prehash, it.sig)
            if code:
                want_st, want_addr = 1 + code, bytes(20)
            else:
                want_addr = coracle.keccak256(pub)[12:]
                want_st = 0 if want_addr == owners[i] else 1
            if int(st[i]) != want_st or addr[i].tobytes() != want_addr:
                bad.append((i, it.kind, int(st[i]), want_st))
        assert not bad, f"{len(bad)} GPU results differ from OpenSSL, first {bad[:5]}"
        assert {0, 1, 4, 5, 6, 7}.issubset(set(int(x) for x in np.asarray(st)))
    finally:
        ec.close()
