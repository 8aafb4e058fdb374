"""`ConsensusSignatureScheme` (/root/reference/src/signing.rs:46-74) and the default
`EthereumConsensusSigner` (/root/reference/src/signing/ethereum.rs), GPU-backed.

`verify` is static in the reference (no instance at the call site), so it runs on the
process-global engine (`Engine.default()`); `verify_batch` is the batched extension the GPU path
exists for.  `sign` and `identity` use the engine's batch signer (RFC 6979, low-s, v = 27 + y).
"""
from __future__ import annotations

import abc
from typing import List, Sequence, Tuple, Union

import numpy as np

from .engine import Engine
from .errors import ConsensusSchemeError, SCHEME_REASONS


class ConsensusSignatureScheme(abc.ABC):
    """signing.rs:46-74."""

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
