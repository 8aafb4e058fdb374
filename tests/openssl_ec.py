"""ctypes binding of the system OpenSSL libcrypto (secp256k1 + SHA-256): an INDEPENDENT
implementation used only by tests to pin the byte-level crypto slice.

TEST INFRASTRUCTURE ONLY.  Nothing here is shipped or measured.  What it restates on top of
OpenSSL's arithmetic is only the alloy/k256 *semantics* of
`Signature::from_raw_array(sig).recover_address_from_msg(payload)` (called at
/root/reference/src/signing/ethereum.rs:86-89): normalize_v, normalized_s, the r/s range check,
R = decompress(r, parity), Q = r^-1 (s R - z G), Q != infinity.  Every field / group / scalar
operation (square root, point multiplication, modular inversion) is OpenSSL's own, so agreement
with the oracle and the GPU pins those byte for byte against a second code base.
"""
from __future__ import annotations

import ctypes
import ctypes.util
from ctypes import POINTER, c_char_p, c_int, c_size_t, c_void_p

NID_SECP256K1 = 714
POINT_CONVERSION_UNCOMPRESSED = 4

_lib = None


def available() -> bool:
    try:
        load()
        return True
    except OSError:
        return False


def load():
    global _lib
    if _lib is not None:
        return _lib
    name = ctypes.util.find_library("crypto")
    if not name:
        raise OSError("libcrypto not found")
    L = ctypes.CDLL(name)
    vp = c_void_p
    sig = {
        "SHA256": ([c_char_p, c_size_t, c_char_p], vp),
        "BN_CTX_new": ([], vp), "BN_CTX_free": ([vp], None),
        "BN_new": ([], vp), "BN_free": ([vp], None),
        "BN_bin2bn": ([c_char_p, c_int, vp], vp),
        "BN_bn2binpad": ([vp, c_char_p, c_int], c_int),
        "BN_is_zero": ([vp], c_int),
        "BN_mod_inverse": ([vp, vp, vp, vp], vp),
        "BN_mod_mul": ([vp, vp, vp, vp, vp], c_int),
        "BN_mod_sub": ([vp, vp, vp, vp, vp], c_int),
        "BN_nnmod": ([vp, vp, vp, vp], c_int),
        "EC_GROUP_new_by_curve_name": ([c_int], vp), "EC_GROUP_free": ([vp], None),
        "EC_GROUP_get0_order": ([vp], vp),
        "EC_POINT_new": ([vp], vp), "EC_POINT_free": ([vp], None),
        "EC_POINT_set_compressed_coordinates": ([vp, vp, vp, c_int, vp], c_int),
        "EC_POINT_mul": ([vp, vp, vp, vp, vp, vp], c_int),
        "EC_POINT_is_at_infinity": ([vp, vp], c_int),
        "EC_POINT_point2oct": ([vp, vp, c_int, c_char_p, c_size_t, vp], c_size_t),
        "EC_KEY_new_by_curve_name": ([c_int], vp), "EC_KEY_free": ([vp], None),
        "EC_KEY_set_public_key": ([vp, vp], c_int),
        "ECDSA_SIG_new": ([], vp), "ECDSA_SIG_free": ([vp], None),
        "ECDSA_SIG_set0": ([vp, vp, vp], c_int),
        "ECDSA_do_verify": ([c_char_p, c_int, vp, vp], c_int),
    }
    for fn, (args, res) in sig.items():
        f = getattr(L, fn)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def sha256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    load().SHA256(data, len(data), out)
    return out.raw


class Secp256k1:
    """One BN_CTX + group; not thread-safe (tests use one per thread)."""

    def __init__(self):
        L = self.L = load()
        self.ctx = L.BN_CTX_new()
        self.group = L.EC_GROUP_new_by_curve_name(NID_SECP256K1)
        if not self.ctx or not self.group:
            raise OSError("OpenSSL secp256k1 unavailable")
        self.order = L.EC_GROUP_get0_order(self.group)

    def close(self):
        self.L.EC_GROUP_free(self.group)
        self.L.BN_CTX_free(self.ctx)

    def _bn(self, b: bytes):
        return self.L.BN_bin2bn(b, len(b), None)

    def _point_bytes(self, pt) -> bytes:
        buf = ctypes.create_string_buffer(65)
        n = self.L.EC_POINT_point2oct(self.group, pt, POINT_CONVERSION_UNCOMPRESSED, buf, 65, self.ctx)
        assert n == 65
        return buf.raw[1:]  # X || Y, 64 bytes big-endian

    def pubkey(self, priv32: bytes) -> bytes:
        """d G as X || Y (OpenSSL EC_POINT_mul)."""
        L = self.L
        d = self._bn(priv32)
        q = L.EC_POINT_new(self.group)
        try:
            assert L.EC_POINT_mul(self.group, q, d, None, None, self.ctx) == 1
            return self._point_bytes(q)
        finally:
            L.EC_POINT_free(q)
            L.BN_free(d)

    def recover(self, prehash: bytes, sig65: bytes):
        """(scheme_subcode, X||Y or None) with the alloy/k256 recovery semantics (see module doc);
        subcodes as pyoracle.SCHEME_*: 3 parity, 4 scalar range, 5 no point, 6 infinity."""
        L = self.L
        v = sig65[64]
        if v in (0, 27):
            parity = 0
        elif v in (1, 28):
            parity = 1
        elif v >= 35:
            parity = (v - 35) & 1
        else:
            return 3, None
        N = int.from_bytes(bytes.fromhex(
            "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141"), "big")
        r_i = int.from_bytes(sig65[:32], "big")
        s_i = int.from_bytes(sig65[32:64], "big")
        if s_i > (N >> 1):  # alloy normalized_s (wrapping U256 subtraction)
            s_i = (N - s_i) % (1 << 256)
            parity ^= 1
        if r_i == 0 or r_i >= N or s_i == 0 or s_i >= N:
            return 4, None
        r = self._bn(sig65[:32])
        s = self._bn(s_i.to_bytes(32, "big"))
        z = self._bn(prehash)
        R = L.EC_POINT_new(self.group)
        Q = L.EC_POINT_new(self.group)
        rinv, u1, u2, zn = L.BN_new(), L.BN_new(), L.BN_new(), L.BN_new()
        try:
            # R = decompress(x = r, parity): OpenSSL's own square root
            if L.EC_POINT_set_compressed_coordinates(self.group, R, r, parity, self.ctx) != 1:
                return 5, None
            assert L.BN_mod_inverse(rinv, r, self.order, self.ctx)
            assert L.BN_nnmod(zn, z, self.order, self.ctx) == 1
            zero = L.BN_new()
            try:
                assert L.BN_mod_sub(u1, zero, zn, self.order, self.ctx) == 1        # -z
            finally:
                L.BN_free(zero)
            assert L.BN_mod_mul(u1, u1, rinv, self.order, self.ctx) == 1           # -z / r
            assert L.BN_mod_mul(u2, s, rinv, self.order, self.ctx) == 1            # s / r
            assert L.EC_POINT_mul(self.group, Q, u1, R, u2, self.ctx) == 1        # u1 G + u2 R
            if L.EC_POINT_is_at_infinity(self.group, Q):
                return 6, None
            return 0, self._point_bytes(Q)
        finally:
            for b in (r, s, z, rinv, u1, u2, zn):
                L.BN_free(b)
            L.EC_POINT_free(R)
            L.EC_POINT_free(Q)

    def ecdsa_verify(self, prehash: bytes, r32: bytes, s32: bytes, pub64: bytes) -> bool:
        """OpenSSL ECDSA_do_verify of (r, s) over the 32-byte prehash under the public key."""
        L = self.L
        key = L.EC_KEY_new_by_curve_name(NID_SECP256K1)
        pt = L.EC_POINT_new(self.group)
        sig = L.ECDSA_SIG_new()
        try:
            x = self._bn(pub64[:32])
            y = self._bn(pub64[32:])
            # uncompressed octets -> point via oct2point would need one more binding: use mul-free
            # affine set through the compressed form + parity of y
            ok = L.EC_POINT_set_compressed_coordinates(self.group, pt, x, pub64[63] & 1, self.ctx)
            L.BN_free(x)
            L.BN_free(y)
            if ok != 1 or self._point_bytes(pt) != pub64:
                return False
            assert L.EC_KEY_set_public_key(key, pt) == 1
            assert L.ECDSA_SIG_set0(sig, self._bn(r32), self._bn(s32)) == 1  # sig owns r, s
            return L.ECDSA_do_verify(prehash, 32, sig, key) == 1
        finally:
            L.ECDSA_SIG_free(sig)
            L.EC_POINT_free(pt)
            L.EC_KEY_free(key)
