"""Pure-Python CPU restatement of the hashgraph-like-consensus vote-validation path.

TEST INFRASTRUCTURE ONLY.  This module is the parity *checker*: only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it.  The
product path (the HIP kernels behind `include/hlc.h`) never calls into it.

Every function restates one piece of the reference (`/root/reference`, crate
`hashgraph-like-consensus` v0.6.0) or of the third-party crates it calls for this
path (not vendored in the reference; versions pinned by `/root/reference/Cargo.lock`):

  * sha2 0.10.9              -- SHA-256 (FIPS 180-4)           -> `hashlib.sha256`
  * alloy-primitives 1.6.0   -- keccak256, EIP-191 prehash, `Signature::from_raw_array`,
                                `normalize_v`, `normalized_s`, `recover_address_from_msg`
  * k256 0.13.4 / ecdsa 0.16.9 -- secp256k1 recovery (`VerifyingKey::recover_from_prehash`),
                                RFC 6979 signing with low-s normalisation (used by the
                                fixture generator only, mirrors `build_vote` -> `sign`)
  * prost 0.14.4             -- proto3 encoding of `Vote` (`consensus.proto:19-29`)

Parity pinning (the reference ships no byte-level golden vectors):
  * keccak256 pinned by published KATs and by `hashlib.sha3_256` (same permutation,
    different pad) in `tests/test_oracle_kats.py`;
  * secp256k1 / EIP-191 / RFC 6979 / ecrecover pinned by the published web3.js
    `accounts.sign` vector (key 0x4c08..2318, message "Some data") and the
    key-1 address KAT;
  * the Vote encoding is cross-checked against the `protobuf` runtime (7.35.1);
  * the tally / threshold / round-limit logic is pinned by the reference's own
    deterministic tests (`tests/threshold_tests.rs`, `tests/rfc_compliance_tests.rs:361-372`,
    `src/session.rs:427-524`).
"""
from __future__ import annotations

import hashlib
import hmac
import math
import struct
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence, Tuple

# --------------------------------------------------------------------------------------
# Status codes: mirror of `ConsensusError` (src/error.rs:11-74) restricted to the hot path.
# The numeric values are the ABI of include/hlc.h (HLC_* constants) -- keep in sync.
# --------------------------------------------------------------------------------------
OK = 0
PROPOSAL_EXPIRED = 1               # error.rs:39
VOTE_PROPOSAL_ID_MISMATCH = 2      # error.rs:41
EMPTY_VOTE_OWNER = 3               # error.rs:33
EMPTY_VOTE_HASH = 4                # error.rs:37
EMPTY_SIGNATURE = 5                # error.rs:25
INVALID_VOTE_HASH = 6              # error.rs:35
SIGNATURE_SCHEME = 7               # error.rs:72-73 (ConsensusSchemeError::Verify)
INVALID_VOTE_SIGNATURE = 8         # error.rs:23
TIMESTAMP_OLDER_THAN_CREATION = 9  # error.rs:49
VOTE_EXPIRED = 10                  # error.rs:31
RECEIVED_HASH_MISMATCH = 11        # error.rs:43
PARENT_HASH_MISMATCH = 12          # error.rs:45
DUPLICATE_VOTE = 13                # error.rs:27
MAX_ROUNDS_EXCEEDED = 14           # error.rs:65
PROPOSAL_ALREADY_EXIST = 15        # error.rs:57

STATUS_NAMES = {
    OK: "Ok", PROPOSAL_EXPIRED: "ProposalExpired", VOTE_PROPOSAL_ID_MISMATCH: "VoteProposalIdMismatch",
    EMPTY_VOTE_OWNER: "EmptyVoteOwner", EMPTY_VOTE_HASH: "EmptyVoteHash", EMPTY_SIGNATURE: "EmptySignature",
    INVALID_VOTE_HASH: "InvalidVoteHash", SIGNATURE_SCHEME: "SignatureScheme",
    INVALID_VOTE_SIGNATURE: "InvalidVoteSignature", TIMESTAMP_OLDER_THAN_CREATION: "TimestampOlderThanCreationTime",
    VOTE_EXPIRED: "VoteExpired", RECEIVED_HASH_MISMATCH: "ReceivedHashMismatch",
    PARENT_HASH_MISMATCH: "ParentHashMismatch", DUPLICATE_VOTE: "DuplicateVote",
    MAX_ROUNDS_EXCEEDED: "MaxRoundsExceeded", PROPOSAL_ALREADY_EXIST: "ProposalAlreadyExist",
}

# Sub-reasons of a scheme `Err(Verify(..))` (diagnostic only; the reference surfaces
# them as one class, `ConsensusError::SignatureScheme(_)`).
SCHEME_NONE = 0
SCHEME_SIG_LEN = 1        # ethereum.rs:71-76
SCHEME_ID_LEN = 2         # ethereum.rs:77-82
SCHEME_BAD_PARITY = 3     # alloy normalize_v -> SignatureError::InvalidParity (ethereum.rs:86-87)
SCHEME_SCALAR_RANGE = 4   # r or s == 0 or >= n (k256 Signature::from_scalars, via to_k256)
SCHEME_NO_POINT = 5       # x = r has no curve point (AffinePoint::decompress is None)
SCHEME_INFINITY = 6       # recovered Q is the identity (VerifyingKey::from_affine)

# Transition codes (types.rs:29-34)
STILL_ACTIVE = 0
REACHED_NO = 1
REACHED_YES = 2

# --------------------------------------------------------------------------------------
# Keccak-256 (alloy-primitives `keccak256`; original Keccak padding 0x01 .. 0x80)
# --------------------------------------------------------------------------------------
_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61],
        [28, 55, 25, 21, 56], [27, 20, 39, 8, 14]]  # _ROT[x][y]
_M64 = (1 << 64) - 1


def _rol(v: int, n: int) -> int:
    return ((v << n) | (v >> (64 - n))) & _M64 if n else v


def keccak_f1600(a: List[int]) -> None:
    """In-place keccak-f[1600] on 25 lanes, a[x + 5*y] (FIPS 202 §3.2)."""
    for rnd in range(24):
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
        for i in range(25):
            a[i] ^= d[i % 5]
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = _rol(a[x + 5 * y], _ROT[x][y])
        for y in range(5):
            row = b[5 * y:5 * y + 5]
            for x in range(5):
                a[x + 5 * y] = row[x] ^ ((~row[(x + 1) % 5]) & row[(x + 2) % 5])
        a[0] ^= _RC[rnd]


def _keccak(data: bytes, pad: int, rate: int = 136, out_len: int = 32) -> bytes:
    state = [0] * 25
    msg = bytearray(data)
    msg.append(pad)
    while len(msg) % rate:
        msg.append(0)
    msg[-1] |= 0x80
    for off in range(0, len(msg), rate):
        for i in range(rate // 8):
            state[i] ^= int.from_bytes(msg[off + 8 * i: off + 8 * i + 8], "little")
        keccak_f1600(state)
    out = b"".join(state[i].to_bytes(8, "little") for i in range(rate // 8))
    return out[:out_len]


def keccak256(data: bytes) -> bytes:
    """alloy_primitives::keccak256 (legacy Keccak, pad 0x01)."""
    return _keccak(data, 0x01)


def sha3_256_via_keccak(data: bytes) -> bytes:
    """FIPS-202 SHA3-256 (pad 0x06) on the same permutation: lets tests pin keccak_f1600
    against `hashlib.sha3_256`."""
    return _keccak(data, 0x06)


def eip191_message(payload: bytes) -> bytes:
    """alloy_primitives::eip191_message: "\\x19Ethereum Signed Message:\\n" ‖ len ‖ payload."""
    return b"\x19Ethereum Signed Message:\n" + str(len(payload)).encode() + payload


def eip191_hash_message(payload: bytes) -> bytes:
    """alloy_primitives::eip191_hash_message (reached at src/signing/ethereum.rs:89)."""
    return keccak256(eip191_message(payload))


# --------------------------------------------------------------------------------------
# secp256k1 (k256 0.13.4 semantics)
# --------------------------------------------------------------------------------------
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)
INF = None


def _inv(a: int, m: int) -> int:
    return pow(a, m - 2, m)


def point_add(p1, p2):
    """Affine group law with all exceptional cases (identity, doubling, inverse)."""
    if p1 is INF:
        return p2
    if p2 is INF:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return INF
        lam = 3 * x1 * x1 * _inv(2 * y1, P) % P
    else:
        lam = (y2 - y1) * _inv(x2 - x1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    y3 = (lam * (x1 - x3) - y1) % P
    return (x3, y3)


def point_mul(k: int, pt):
    k %= N
    acc = INF
    addend = pt
    while k:
        if k & 1:
            acc = point_add(acc, addend)
        addend = point_add(addend, addend)
        k >>= 1
    return acc


def pubkey_to_address(pt) -> bytes:
    """alloy `Address::from_public_key`: keccak256(X ‖ Y)[12..32]."""
    x, y = pt
    return keccak256(x.to_bytes(32, "big") + y.to_bytes(32, "big"))[12:]


def privkey_to_address(d: int) -> bytes:
    return pubkey_to_address(point_mul(d, G))


def decompress(x: int, y_odd: bool):
    """k256 `AffinePoint::decompress`: None if x >= p or x^3+7 is a non-residue."""
    if x >= P:
        return None
    alpha = (pow(x, 3, P) + 7) % P
    beta = pow(alpha, (P + 1) // 4, P)
    if beta * beta % P != alpha:
        return None
    y = beta if (beta & 1) == int(y_odd) else (P - beta) % P
    return (x, y)


def normalize_v(v: int) -> Optional[bool]:
    """alloy_primitives::normalize_v: 0/27 -> even, 1/28 -> odd, >=35 -> EIP-155 parity."""
    if v in (0, 27):
        return False
    if v in (1, 28):
        return True
    if v >= 35:
        return ((v - 35) % 2) != 0
    return None


def ecrecover(prehash: bytes, sig65: bytes) -> Tuple[int, Optional[bytes]]:
    """`Signature::from_raw_array(sig).recover_address_from_prehash(prehash)` (alloy 1.6 +
    k256 0.13).  Returns (scheme_subcode, address-or-None).

    Steps: parse v (normalize_v) -> normalized_s (s > n/2 => s = n - s, parity flipped)
    -> to_k256 (r, s in [1, n-1]) -> z = prehash mod n -> R = decompress(r, parity)
    -> Q = r^-1 (s R - z G) -> identity rejected -> keccak(Q)[12..].
    The post-recovery `verify_prehash` inside k256 always succeeds for a recovered key
    (it re-derives R), so it is not restated here.
    """
    parity = normalize_v(sig65[64])
    if parity is None:
        return SCHEME_BAD_PARITY, None
    r = int.from_bytes(sig65[0:32], "big")
    s = int.from_bytes(sig65[32:64], "big")
    if s > (N >> 1):                       # normalized_s
        s = (N - s) % (1 << 256)           # wrapping U256 sub; s >= n lands >= n below
        parity = not parity
    if r == 0 or r >= N or s == 0 or s >= N:
        return SCHEME_SCALAR_RANGE, None
    z = int.from_bytes(prehash, "big") % N
    R = decompress(r, parity)
    if R is None:
        return SCHEME_NO_POINT, None
    rinv = _inv(r, N)
    u1 = (-z * rinv) % N
    u2 = (s * rinv) % N
    Q = point_add(point_mul(u1, G), point_mul(u2, R))
    if Q is INF:
        return SCHEME_INFINITY, None
    return SCHEME_NONE, pubkey_to_address(Q)


def _rfc6979_k(d: int, h1: bytes) -> int:
    """RFC 6979 §3.2 with HMAC-SHA256 (rfc6979 0.4 crate, used by k256 signing)."""
    x = d.to_bytes(32, "big")
    h = (int.from_bytes(h1, "big") % N).to_bytes(32, "big")
    V = b"\x01" * 32
    K = b"\x00" * 32
    K = hmac.new(K, V + b"\x00" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    K = hmac.new(K, V + b"\x01" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    while True:
        V = hmac.new(K, V, hashlib.sha256).digest()
        k = int.from_bytes(V, "big")
        if 1 <= k < N:
            return k
        K = hmac.new(K, V + b"\x00", hashlib.sha256).digest()
        V = hmac.new(K, V, hashlib.sha256).digest()


def sign_prehash(d: int, prehash: bytes) -> bytes:
    """k256 `sign_prehash_recoverable` (RFC 6979, low-s normalised) + alloy `as_bytes()`
    (r ‖ s ‖ 27+parity).  Mirrors `EthereumConsensusSigner::sign` (ethereum.rs:58-64)."""
    z = int.from_bytes(prehash, "big") % N
    k = _rfc6979_k(d, prehash)
    R = point_mul(k, G)
    r = R[0] % N
    y_odd = R[1] & 1
    s = _inv(k, N) * (z + r * d) % N
    if s > N >> 1:
        s = N - s
        y_odd ^= 1
    return r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([27 + y_odd])


def sign_message(d: int, payload: bytes) -> bytes:
    return sign_prehash(d, eip191_hash_message(payload))


# --------------------------------------------------------------------------------------
# Wire types (consensus.proto:5-29) and prost encoding
# --------------------------------------------------------------------------------------
@dataclass
class Vote:
    vote_id: int = 0
    vote_owner: bytes = b""
    proposal_id: int = 0
    timestamp: int = 0
    vote: bool = False
    parent_hash: bytes = b""
    received_hash: bytes = b""
    vote_hash: bytes = b""
    signature: bytes = b""


@dataclass
class Proposal:
    name: str = ""
    payload: bytes = b""
    proposal_id: int = 0
    proposal_owner: bytes = b""
    votes: List[Vote] = field(default_factory=list)
    expected_voters_count: int = 0
    round: int = 1
    timestamp: int = 0
    expiration_timestamp: int = 0
    liveness_criteria_yes: bool = False


def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def encode_vote(v: Vote) -> bytes:
    """prost `Message::encode_to_vec` for `Vote` (proto3: defaults omitted, fields in tag
    order 20..28, 2-byte keys since tags >= 16)."""
    out = bytearray()
    if v.vote_id:
        out += _varint((20 << 3) | 0) + _varint(v.vote_id)
    if v.vote_owner:
        out += _varint((21 << 3) | 2) + _varint(len(v.vote_owner)) + v.vote_owner
    if v.proposal_id:
        out += _varint((22 << 3) | 0) + _varint(v.proposal_id)
    if v.timestamp:
        out += _varint((23 << 3) | 0) + _varint(v.timestamp)
    if v.vote:
        out += _varint((24 << 3) | 0) + b"\x01"
    if v.parent_hash:
        out += _varint((25 << 3) | 2) + _varint(len(v.parent_hash)) + v.parent_hash
    if v.received_hash:
        out += _varint((26 << 3) | 2) + _varint(len(v.received_hash)) + v.received_hash
    if v.vote_hash:
        out += _varint((27 << 3) | 2) + _varint(len(v.vote_hash)) + v.vote_hash
    if v.signature:
        out += _varint((28 << 3) | 2) + _varint(len(v.signature)) + v.signature
    return bytes(out)


def signed_payload(v: Vote) -> bytes:
    """utils.rs:150-152: clone, clear signature, encode."""
    return encode_vote(replace(v, signature=b""))


def compute_vote_hash(v: Vote) -> bytes:
    """utils.rs:37-47."""
    h = hashlib.sha256()
    h.update(struct.pack("<I", v.vote_id))
    h.update(v.vote_owner)
    h.update(struct.pack("<I", v.proposal_id))
    h.update(struct.pack("<Q", v.timestamp))
    h.update(bytes([1 if v.vote else 0]))
    h.update(v.parent_hash)
    h.update(v.received_hash)
    return h.digest()


# --------------------------------------------------------------------------------------
# Signature scheme (signing.rs:46-74, signing/ethereum.rs:66-97)
# --------------------------------------------------------------------------------------
def ethereum_verify(identity: bytes, payload: bytes, signature: bytes) -> Tuple[int, Optional[bool], Optional[bytes]]:
    """EthereumConsensusSigner::verify -> (scheme_subcode, Ok(bool) or None on Err, recovered)."""
    if len(signature) != 65:
        return SCHEME_SIG_LEN, None, None
    if len(identity) != 20:
        return SCHEME_ID_LEN, None, None
    code, addr = ecrecover(eip191_hash_message(payload), signature)
    if code:
        return code, None, None
    return SCHEME_NONE, addr == identity, addr


SCHEME_PLUGIN = 7  # HLC_SCHEME_PLUGIN: Err(Verify) from a scheme other than EthereumConsensusSigner


def stub_verify(identity: bytes, payload: bytes, signature: bytes) -> Tuple[int, Optional[bool], Optional[bytes]]:
    """StubSigner::verify of /root/reference/tests/custom_scheme_tests.rs:61-73 (the reference's proof that
    ConsensusService is generic over the scheme, service.rs:39-51): Err(Verify) unless the identity is
    8 bytes, else Ok(signature == SHA256(identity || payload))."""
    if len(identity) != 8:
        return SCHEME_PLUGIN, None, None
    return SCHEME_NONE, signature == stub_sign(identity, payload), None


def stub_sign(identity: bytes, payload: bytes) -> bytes:
    """StubSigner::sign / expected_signature (custom_scheme_tests.rs:42-47, 55-57)."""
    return hashlib.sha256(identity + payload).digest()


def validate_vote(v: Vote, expiration: int, creation: int, now: int, scheme=ethereum_verify) -> Tuple[int, int]:
    """utils.rs:127-171 -> (status, scheme_subcode).  `scheme` is `Signer::verify` (signing.rs:69-73):
    ethereum_verify (the default EthereumConsensusSigner) or stub_verify."""
    if not v.vote_owner:
        return EMPTY_VOTE_OWNER, 0
    if not v.vote_hash:
        return EMPTY_VOTE_HASH, 0
    if not v.signature:
        return EMPTY_SIGNATURE, 0
    if v.vote_hash != compute_vote_hash(v):
        return INVALID_VOTE_HASH, 0
    sub, ok, _ = scheme(v.vote_owner, signed_payload(v), v.signature)
    if ok is None:
        return SIGNATURE_SCHEME, sub
    if not ok:
        return INVALID_VOTE_SIGNATURE, 0
    if v.timestamp < creation:
        return TIMESTAMP_OLDER_THAN_CREATION, 0
    if v.timestamp > expiration or now > expiration:
        return VOTE_EXPIRED, 0
    return OK, 0


def vote_status_in_proposal(p: Proposal, v: Vote, now: int, scheme=ethereum_verify) -> Tuple[int, int]:
    """Per-vote body of validate_proposal's loop (utils.rs:112-117)."""
    if v.proposal_id != p.proposal_id:
        return VOTE_PROPOSAL_ID_MISMATCH, 0
    return validate_vote(v, p.expiration_timestamp, p.timestamp, now, scheme)


def validate_vote_chain(votes: Sequence[Vote]) -> Tuple[int, int]:
    """utils.rs:175-215 -> (status, failing index or -1).  HashMap insert => last wins."""
    if len(votes) <= 1:
        return OK, -1
    index: Dict[bytes, Tuple[bytes, int, int]] = {}
    for i, v in enumerate(votes):
        index[v.vote_hash] = (v.vote_owner, v.timestamp, i)
    for i, v in enumerate(votes):
        if i > 0 and v.received_hash:
            prev = votes[i - 1]
            if v.received_hash != prev.vote_hash or prev.timestamp > v.timestamp:
                return RECEIVED_HASH_MISMATCH, i
        if v.parent_hash:
            hit = index.get(v.parent_hash)
            if hit is None:
                return PARENT_HASH_MISMATCH, i
            owner, ts, pidx = hit
            if not (owner == v.vote_owner and ts <= v.timestamp and pidx < i):
                return PARENT_HASH_MISMATCH, i
    return OK, -1


# --------------------------------------------------------------------------------------
# Tally, thresholds and round limits (utils.rs:227-313, session.rs:120-128, 306-387)
# --------------------------------------------------------------------------------------
_F64_EPS = 2.220446049250313e-16
_U32 = 0xFFFFFFFF


def _f64_to_u32_sat(x: float) -> int:
    """Rust `f64 as u32` (saturating, NaN -> 0)."""
    if x != x:
        return 0
    if x <= 0:
        return 0
    if x >= 4294967295.0:
        return _U32
    return int(x)


def calculate_threshold_based_value(n: int, t: float) -> int:
    """utils.rs:307-313.  (2n).div_ceil(3) in u32 (release-mode wrap of 2*n)."""
    if abs(t - (2.0 / 3.0)) < _F64_EPS:
        two_n = (2 * n) & _U32
        return (two_n + 2) // 3
    return _f64_to_u32_sat(math.ceil(float(n) * t))


def calculate_required_votes(n: int, t: float) -> int:
    """utils.rs:292-299."""
    return n if n <= 2 else calculate_threshold_based_value(n, t)


def has_sufficient_votes(total: int, n: int, t: float) -> bool:
    """utils.rs:360-367."""
    return total >= calculate_required_votes(n, t)


def calculate_consensus_result(total: int, yes: int, n: int, t: float, liveness: bool,
                               is_timeout: bool) -> Optional[bool]:
    """utils.rs:227-286 on (total, yes) counts of the owner->vote map."""
    no = max(total - yes, 0)
    silent = max(n - total, 0)
    if n <= 2:
        if total < n:
            return None
        return yes == n
    req = calculate_required_votes(n, t)
    eff = n if is_timeout else total
    if eff < req:
        return None
    req_choice = calculate_threshold_based_value(n, t)
    yes_w = yes + (silent if liveness else 0)
    no_w = no + (0 if liveness else silent)
    if yes_w >= req_choice and yes_w > no_w:
        return True
    if no_w >= req_choice and no_w > yes_w:
        return False
    if total == n and yes_w == no_w:
        return liveness
    return None


# Session states (session.rs:157-164) as the ABI numbers them (HLC_SESSION_*)
SESSION_ACTIVE, SESSION_REACHED_NO, SESSION_REACHED_YES, SESSION_FAILED = 0, 1, 2, 3
INSUFFICIENT_VOTES_AT_TIMEOUT = 16  # error.rs:64


def handle_consensus_timeout(state: int, total: int, yes: int, n: int, t: float,
                             liveness: bool) -> Tuple[int, int]:
    """service.rs:323-373 on one session -> (new state, status): an earlier ConsensusReached
    stands; otherwise the timeout tally decides ConsensusReached(r) or Failed + error."""
    if state in (SESSION_REACHED_NO, SESSION_REACHED_YES):
        return state, OK
    r = calculate_consensus_result(total, yes, n, t, liveness, True)
    if r is None:
        return SESSION_FAILED, INSUFFICIENT_VOTES_AT_TIMEOUT
    return (SESSION_REACHED_YES if r else SESSION_REACHED_NO), OK


@dataclass
class ConsensusConfig:
    """session.rs:27-44 (timeout omitted: not on the validation path)."""
    consensus_threshold: float = 2.0 / 3.0
    max_rounds: int = 2
    use_gossipsub_rounds: bool = True
    liveness_criteria: bool = True

    @staticmethod
    def gossipsub() -> "ConsensusConfig":
        return ConsensusConfig(2.0 / 3.0, 2, True, True)      # session.rs:52-58

    @staticmethod
    def p2p() -> "ConsensusConfig":
        return ConsensusConfig(2.0 / 3.0, 0, False, True)

    def max_round_limit(self, n: int) -> int:
        """session.rs:120-128."""
        if self.use_gossipsub_rounds:
            return self.max_rounds
        if self.max_rounds == 0:
            return calculate_threshold_based_value(n, self.consensus_threshold)
        return self.max_rounds


def check_round_limit(cfg: ConsensusConfig, n: int, round_: int, vote_count: int) -> bool:
    """session.rs:306-344 -> True if within limit.  vote_count is a usize: it is compared with n
    before any u32 arithmetic (session.rs:308), so a count past u32::MAX fails there (the
    reference's own test, session.rs:644-672); the P2P projection is
    round.saturating_sub(1).saturating_add(vote_count as u32) in u32 (session.rs:330-331)."""
    if vote_count > n:
        return False
    if cfg.use_gossipsub_rounds:
        projected = 2 if (round_ == 2 or (round_ == 1 and vote_count > 0)) else round_
    else:
        projected = min(max(round_ - 1, 0) + (vote_count & _U32), _U32)
    return projected <= cfg.max_round_limit(n)


def update_round(cfg: ConsensusConfig, round_: int, vote_count: int) -> int:
    """session.rs:351-366: Gossipsub moves 1 -> 2 on any votes; P2P adds the count with
    saturation at u32::MAX (session.rs:364; the reference's test at session.rs:674-699)."""
    if cfg.use_gossipsub_rounds:
        return 2 if (round_ == 1 and vote_count > 0) else round_
    return min(round_ + (vote_count & _U32), _U32)


@dataclass
class ProposalOutcome:
    status: int = OK
    bad_index: int = -1          # index of the failing vote (per-vote / chain errors)
    yes: int = 0
    total: int = 0
    transition: int = STILL_ACTIVE
    round: int = 1


def from_proposal(p: Proposal, cfg: ConsensusConfig, now: int,
                  vote_status: Optional[List[Tuple[int, int]]] = None, scheme=ethereum_verify) -> ProposalOutcome:
    """ConsensusSession::from_proposal (session.rs:198-221) -> validate_proposal
    (utils.rs:106-120) then initialize_with_votes (session.rs:253-298) on a clean copy
    (round reset to 1).  The second validation pass (session.rs:284-287) re-runs the same
    deterministic checks on unchanged inputs and cannot change the outcome, so it is not
    repeated here."""
    out = ProposalOutcome()
    if now >= p.expiration_timestamp:                               # utils.rs:110, 320-328
        out.status = PROPOSAL_EXPIRED
        return out
    for i, v in enumerate(p.votes):                                 # utils.rs:112-117
        st = vote_status[i] if vote_status is not None else vote_status_in_proposal(p, v, now, scheme)
        if st[0] != OK:
            out.status, out.bad_index = st[0], i
            return out
    st, idx = validate_vote_chain(p.votes)                          # utils.rs:118
    if st != OK:
        out.status, out.bad_index = st, idx
        return out
    votes = p.votes
    if not votes:                                                   # session.rs:266-268
        return out
    seen = set()
    for i, v in enumerate(votes):                                   # session.rs:270-275
        if v.vote_owner in seen:
            out.status, out.bad_index = DUPLICATE_VOTE, i
            return out
        seen.add(v.vote_owner)
    n = p.expected_voters_count
    if len(votes) > n:                                              # session.rs:279-282
        out.status = MAX_ROUNDS_EXCEEDED
        return out
    if not check_round_limit(cfg, n, 1, len(votes)):                # session.rs:289
        out.status = MAX_ROUNDS_EXCEEDED
        return out
    out.round = update_round(cfg, 1, len(votes))                    # session.rs:290, 351-366
    out.total = len(votes)
    out.yes = sum(1 for v in votes if v.vote)
    res = calculate_consensus_result(out.total, out.yes, n, cfg.consensus_threshold,
                                     p.liveness_criteria_yes, False)    # session.rs:372-387
    out.transition = STILL_ACTIVE if res is None else (REACHED_YES if res else REACHED_NO)
    return out


# --------------------------------------------------------------------------------------
# build_vote (utils.rs:55-98) with explicit vote_id, for fixture generation
# --------------------------------------------------------------------------------------
def build_vote(p: Proposal, choice: bool, priv: int, now: int, vote_id: int,
               owner: Optional[bytes] = None) -> Vote:
    owner = owner if owner is not None else privkey_to_address(priv)
    parent, received = b"", b""
    if p.votes:
        received = p.votes[-1].vote_hash
        for v in reversed(p.votes):
            if v.vote_owner == owner:
                parent = v.vote_hash
                break
    v = Vote(vote_id=vote_id, vote_owner=owner, proposal_id=p.proposal_id, timestamp=now,
             vote=choice, parent_hash=parent, received_hash=received)
    v.vote_hash = compute_vote_hash(v)
    v.signature = sign_message(priv, encode_vote(v))
    return v


def resign(v: Vote, priv: int, rehash: bool = True) -> None:
    """tests/vote_validation_tests.rs:29-40 `resign_vote`."""
    if rehash:
        v.vote_hash = compute_vote_hash(v)
    v.signature = b""
    v.signature = sign_message(priv, encode_vote(v))
