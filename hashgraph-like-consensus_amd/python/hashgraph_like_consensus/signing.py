"""`ConsensusSignatureScheme` (/root/reference/src/signing.rs:46-74) and the default
`EthereumConsensusSigner` (/root/reference/src/signing/ethereum.rs), GPU-backed.

`verify` is static in the reference (no instance at the call site), so it runs on the
process-global engine (`Engine.default()`); `verify_batch` is the batched extension the GPU path
exists for.  `sign` and `identity` use the engine's batch signer (RFC 6979, low-s, v = 27 + y).

The service is generic over the scheme, as the reference's is (service.rs:39-51,
tests/custom_scheme_tests.rs): a scheme with `DEVICE_SCHEME = True` (EthereumConsensusSigner) has its
verify run inside the device pipeline (hlc_validate_proposals); any other scheme's `verify_batch`
(by default a loop over its `verify`) supplies per-vote verdicts to the scheme-generic entries
(hlc_validate_proposals_verdicts, hlc_process_votes_verdicts), which run every other check on the device.
"""
from __future__ import annotations

import abc
from typing import List, Sequence, Tuple, Union

import numpy as np

from .engine import Engine
from .errors import ConsensusSchemeError, SCHEME_REASONS


class ConsensusSignatureScheme(abc.ABC):
    """signing.rs:46-74."""

    # True: the engine runs this scheme's verify inside the validation pipeline itself
    DEVICE_SCHEME = False

    @classmethod
    def verify_batch(cls, items: Sequence[Tuple[bytes, bytes, bytes]]) -> List[object]:
        """Batched `verify` over (identity, payload, signature) items: element i is True / False, or the
        ConsensusSchemeError `verify` raised (the reference's Err(Verify(..))).  The default loops over
        `verify`; a scheme with a batched implementation overrides it."""
        out: List[object] = []
        for ident, payload, sig in items:
            try:
                out.append(bool(cls.verify(ident, payload, sig)))
            except ConsensusSchemeError as e:
                out.append(e)
        return out

    @abc.abstractmethod
    def identity(self) -> bytes:
        """signing.rs:53"""

    @abc.abstractmethod
    def sign(self, payload: bytes) -> bytes:
        """signing.rs:58; raises ConsensusSchemeError('Sign', ..)."""

    @staticmethod
    @abc.abstractmethod
    def verify(identity: bytes, payload: bytes, signature: bytes) -> bool:
        """signing.rs:69-73: True / False, or raises ConsensusSchemeError('Verify', ..)."""


class EthereumConsensusSigner(ConsensusSignatureScheme):
    """ECDSA-secp256k1 scheme (ethereum.rs:23-98): identity = 20-byte address."""

    DEVICE_SCHEME = True

    def __init__(self, private_key: Union[int, bytes], engine: Engine = None):
        if isinstance(private_key, int):
            private_key = private_key.to_bytes(32, "big")
        if len(private_key) != 32:
            raise ValueError("private key must be 32 bytes")
        self._key = np.frombuffer(bytes(private_key), np.uint8).reshape(1, 32).copy()
        self._engine = engine or Engine.default()
        self._address = self._engine.address_batch(self._key)[0].tobytes()

    def identity(self) -> bytes:
        return self._address

    def sign(self, payload: bytes) -> bytes:
        return self._engine.sign_batch(self._key, [payload])[0].tobytes()

    @staticmethod
    def verify(identity: bytes, payload: bytes, signature: bytes) -> bool:
        return EthereumConsensusSigner.verify_batch([(identity, payload, signature)])[0]

    @staticmethod
    def verify_batch(items: Sequence[Tuple[bytes, bytes, bytes]], engine: Engine = None) -> List[object]:
        """One launch for many (identity, payload, signature) items.  Element i is True / False,
        or a ConsensusSchemeError instance (the reference's `Err(Verify(..))`)."""
        eng = engine or Engine.default()
        st, _ = eng.eth_verify_batch([i for i, _, _ in items], [p for _, p, _ in items], [s for _, _, s in items])
        out: List[object] = []
        for s in st:
            s = int(s)
            if s == 0:
                out.append(True)
            elif s == 1:
                out.append(False)
            else:
                out.append(ConsensusSchemeError("Verify", SCHEME_REASONS.get(s - 1, str(s - 1))))
        if len(items) == 1 and isinstance(out[0], ConsensusSchemeError):
            raise out[0]
        return out


def verdict_codes(results: Sequence[object]) -> np.ndarray:
    """verify_batch results -> the ABI's per-vote verdict bytes (HLC_VERIFY_TRUE / _FALSE / _ERR)."""
    from . import _ffi
    out = np.empty(len(results), np.uint8)
    for i, r in enumerate(results):
        if isinstance(r, ConsensusSchemeError):
            out[i] = _ffi.VERIFY_ERR
        else:
            out[i] = _ffi.VERIFY_TRUE if r else _ffi.VERIFY_FALSE
    return out


def scheme_verdicts(scheme, batch, engine: Engine) -> np.ndarray:
    """`Signer::verify` (utils.rs:150-158) of every vote of a VoteBatch under `scheme`: the payloads are
    built on the device (hlc_encode_vote_payloads: prost encoding, signature cleared), the scheme's
    verify_batch decides -> verdict bytes for the *_verdicts entries."""
    if batch.n == 0:
        return np.zeros(0, np.uint8)
    arena, off, lens = engine.encode_vote_payloads(batch)
    raw = arena.tobytes()
    items = [(batch.field(i, 0), raw[int(off[i]):int(off[i]) + int(lens[i])], batch.field(i, 4))
             for i in range(batch.n)]
    return verdict_codes(scheme.verify_batch(items))
