"""ctypes wrapper of oracle/libhlc_oracle.so (the C CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_int, c_long, c_size_t, c_uint8, c_uint32, c_uint64

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libhlc_oracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    u8p = POINTER(c_uint8)
    u32p = POINTER(c_uint32)
    u64p = POINTER(c_uint64)
    vp = ctypes.c_void_p
    lib.hlco_sha256.argtypes = [u8p, c_size_t, u8p]
    lib.hlco_keccak256.argtypes = [u8p, c_size_t, u8p]
    lib.hlco_eip191_hash.argtypes = [u8p, c_size_t, u8p]
    lib.hlco_ecrecover.argtypes = [u8p, u8p, u8p, c_int]
    lib.hlco_ecrecover.restype = c_int
    lib.hlco_address.argtypes = [u8p, u8p]
    lib.hlco_sign_prehash.argtypes = [u8p, u8p, u8p]
    lib.hlco_sign_batch.argtypes = [c_uint64, u8p, u8p, u8p, u8p, c_int]
    lib.hlco_verify_failures.restype = c_long
    lib.hlco_compute_vote_hashes.argtypes = [vp, u8p]
    lib.hlco_encode_vote.argtypes = [vp, c_uint64, u8p]
    lib.hlco_encode_vote.restype = c_size_t
    lib.hlco_verify_batch.argtypes = [c_uint64, u8p, u64p, u32p, u64p, u32p, u64p, u32p, u8p, u8p, c_int]
    lib.hlco_validate_proposals.argtypes = [vp, vp, c_uint64, c_uint64, vp, u8p, u8p, u8p, c_int, c_int]
    lib.hlco_validate_votes_only.argtypes = [vp, vp, c_uint64, c_uint64, c_int, c_int]
    lib.hlco_validate_votes_only.restype = c_uint64
    lib.hlco_consensus_result.argtypes = [c_uint32, c_uint32, c_uint32, c_double, c_int, c_int]
    lib.hlco_consensus_result.restype = c_int
    lib.hlco_threshold_value.argtypes = [c_uint32, c_double]
    lib.hlco_threshold_value.restype = c_uint32
    lib.hlco_check_round_limit.argtypes = [c_int, c_uint32, c_double, c_uint32, c_uint32, c_uint64]
    lib.hlco_check_round_limit.restype = c_int
    lib.hlco_update_round.argtypes = [c_int, c_uint32, c_uint64]
    lib.hlco_update_round.restype = c_uint32
    lib.hlco_stub_sign.argtypes = [u8p, c_uint32, u8p, c_size_t, u8p]
    lib.hlco_stub_sign.restype = c_int
    _lib = lib
    return lib


def _u8(a):
    return a.ctypes.data_as(POINTER(c_uint8))


def _buf(b: bytes):
    arr = np.frombuffer(b, dtype=np.uint8).copy() if len(b) else np.zeros(1, np.uint8)
    return arr


def sha256(b: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    load().hlco_sha256(_u8(_buf(b)), len(b), _u8(out))
    return out.tobytes()


def keccak256(b: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    load().hlco_keccak256(_u8(_buf(b)), len(b), _u8(out))
    return out.tobytes()


def eip191_hash(b: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    load().hlco_eip191_hash(_u8(_buf(b)), len(b), _u8(out))
    return out.tobytes()


REVERIFY, GLV, STUB = 1, 2, 4  # hlco_* flags (hlc_oracle.c)


def _flags(reverify: bool, glv: bool, scheme: str = "ethereum") -> int:
    if scheme not in ("ethereum", "stub"):
        raise ValueError(f"unknown scheme {scheme!r}")
    return (REVERIFY if reverify else 0) | (GLV if glv else 0) | (STUB if scheme == "stub" else 0)


def ecrecover(prehash: bytes, sig: bytes, reverify: bool = True, glv: bool = False):
    """glv: the k256-class recovery (GLV + wNAF + binary-GCD inversions), the timed CPU baseline;
    default: the independent non-GLV checker."""
    out = np.zeros(20, np.uint8)
    code = load().hlco_ecrecover(_u8(_buf(prehash)), _u8(_buf(sig)), _u8(out), _flags(reverify, glv))
    return code, (out.tobytes() if code == 0 else None)


def sign_batch(priv: np.ndarray, prehash: np.ndarray, threads: int = 8):
    """priv [n,32] u8 big-endian, prehash [n,32] -> sig [n,65]"""
    n = priv.shape[0]
    sig = np.zeros((n, 65), np.uint8)
    load().hlco_sign_batch(n, _u8(np.ascontiguousarray(priv)), _u8(np.ascontiguousarray(prehash)),
                           _u8(sig), None, threads)
    return sig


def address_batch(priv: np.ndarray, threads: int = 8):
    n = priv.shape[0]
    addr = np.zeros((n, 20), np.uint8)
    load().hlco_sign_batch(n, _u8(np.ascontiguousarray(priv)), None, None, _u8(addr), threads)
    return addr


def verify_failures() -> int:
    return int(load().hlco_verify_failures())


def compute_vote_hashes(batch) -> np.ndarray:
    out = np.zeros((batch.n, 32), np.uint8)
    view = batch.view()
    load().hlco_compute_vote_hashes(ctypes.byref(view), _u8(out))
    return out


def encode_vote(batch, i: int) -> bytes:
    out = np.zeros(4096, np.uint8)
    view = batch.view()
    n = load().hlco_encode_vote(ctypes.byref(view), i, _u8(out))
    return out[:n].tobytes()


def validate_proposals(batch, desc: np.ndarray, now: int, threads: int = 8, reverify: bool = False,
                       glv: bool = False, scheme: str = "ethereum"):
    """-> (results structured array, vote_status u8[n], vote_reason u8[n], recovered u8[n,20]).
    scheme "stub": the votes' scheme is tests/custom_scheme_tests.rs's StubSigner (8-byte identity,
    signature = SHA256(identity || payload)) instead of EthereumConsensusSigner."""
    from hashgraph_like_consensus import _ffi  # struct layout only
    n = batch.n
    res = np.zeros(desc.shape[0], dtype=_ffi.RESULT_DTYPE)
    vst = np.full(max(n, 1), 0xFF, np.uint8)  # votes outside every proposal: 0xFF (not evaluated)
    vrs = np.zeros(max(n, 1), np.uint8)
    rec = np.zeros((max(n, 1), 20), np.uint8)
    view = batch.view()
    load().hlco_validate_proposals(ctypes.byref(view), desc.ctypes.data, desc.shape[0], now,
                                   res.ctypes.data, _u8(vst), _u8(vrs), _u8(rec), threads,
                                   _flags(reverify, glv, scheme))
    return res, vst[:n], vrs[:n], rec[:n]


def validate_votes_only(batch, desc: np.ndarray, now: int, threads: int, reverify: bool = True,
                        glv: bool = False) -> int:
    view = batch.view()
    return int(load().hlco_validate_votes_only(ctypes.byref(view), desc.ctypes.data, desc.shape[0], now,
                                               threads, _flags(reverify, glv)))


def consensus_result(total, yes, n, t, liveness, is_timeout):
    r = load().hlco_consensus_result(total, yes, n, t, int(liveness), int(is_timeout))
    return None if r < 0 else bool(r)


def threshold_value(n, t):
    return int(load().hlco_threshold_value(n, t))


def check_round_limit(gossipsub: bool, max_rounds: int, t: float, n: int, round_: int, vote_count: int) -> bool:
    """session.rs:306-344 restated in C (any round, usize vote_count)."""
    return bool(load().hlco_check_round_limit(int(gossipsub), max_rounds, t, n, round_, vote_count))


def update_round(gossipsub: bool, round_: int, vote_count: int) -> int:
    """session.rs:351-366 restated in C (P2P saturating at u32::MAX)."""
    return int(load().hlco_update_round(int(gossipsub), round_, vote_count))


def stub_sign(identity: bytes, payload: bytes) -> bytes:
    """StubSigner::sign (tests/custom_scheme_tests.rs:42-47, 55-57): SHA256(identity || payload)."""
    out = np.zeros(32, np.uint8)
    load().hlco_stub_sign(_u8(_buf(identity)), len(identity), _u8(_buf(payload)), len(payload), _u8(out))
    return out.tobytes()
