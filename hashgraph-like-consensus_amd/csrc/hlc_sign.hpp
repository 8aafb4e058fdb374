// hlc_sign.hpp -- the signing side of EthereumConsensusSigner (signing/ethereum.rs:54-64) on the
// device: fixed-base k G by an 8-bit comb, RFC 6979 nonces (HMAC-SHA256), low-s normalisation and
// alloy's r || s || 27+parity layout.  Used by the batch signer (hlc_recover.hip k_sign, k_address)
// and the synthetic workload generator (hlc_synth.hip).  Not on the validation hot path.
#pragma once
#include "hlc_hash.hpp"
#include "hlc_point.hpp"

namespace hlc {

HLC_DEV uint32_t load_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
HLC_DEV uint32_t load_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
// 32 big-endian bytes -> limbs
HLC_DEV void fe_load_be(fe& r, const uint8_t* p) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[7 - i] = load_be32(p + 4 * i);
}
HLC_DEV void fe_store_be(uint8_t* p, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t w = a.v[7 - i];
    p[4 * i] = (uint8_t)(w >> 24);
    p[4 * i + 1] = (uint8_t)(w >> 16);
    p[4 * i + 2] = (uint8_t)(w >> 8);
    p[4 * i + 3] = (uint8_t)w;
  }
}
// digest stored as 8 memory-order words -> big-endian integer limbs
HLC_DEV void fe_from_digest(fe& r, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[7 - i] = bswap32(w[i]);
}

// k*P for small k by plain double-and-add from the generator (table construction only)
static __device__ void scalar_mul_g(gej& acc, const fe& k) {
  ge g;
  ge_generator(g);
  gej_set_inf(acc);
  for (int bit = 255; bit >= 0; --bit) {
    gej_double(acc, acc);
    if ((k.v[bit >> 5] >> (bit & 31)) & 1u) gej_add_ge(acc, acc, g);
  }
}

// k*G via the 8-bit comb (k < n)
static __device__ void fixed_base_mul(gej& acc, const fe& k, const uint32_t* fb) {
  gej_set_inf(acc);
  for (int w = 0; w < 32; ++w) {
    uint32_t j = (k.v[w >> 2] >> (8 * (w & 3))) & 0xFFu;
    if (j) {
      ge g;
      load_ge_global(g, fb + (size_t)(w * 256 + j) * 16);
      gej_add_ge(acc, acc, g);
    }
  }
}

// ---- HMAC-SHA256 over short byte strings held in private memory (RFC 6979) ----
static __device__ void sha256_bytes(const uint8_t* pre64, const uint8_t* msg, int len, uint32_t h[8]) {
  // hashes pre64 (64 bytes, may be null) || msg (len bytes)
  sha256_init(h);
  uint32_t w[16];
  int total = (pre64 ? 64 : 0) + len;
  if (pre64) {
    for (int k = 0; k < 16; ++k) w[k] = ((uint32_t)pre64[4 * k] << 24) | ((uint32_t)pre64[4 * k + 1] << 16) |
                                        ((uint32_t)pre64[4 * k + 2] << 8) | pre64[4 * k + 3];
    sha256_compress(h, w);
  }
  // remaining message with padding
  int nblk = (len + 9 + 63) / 64;
  for (int b = 0; b < nblk; ++b) {
    uint32_t ww[16];
    for (int k = 0; k < 16; ++k) {
      uint32_t x = 0;
      for (int t = 0; t < 4; ++t) {
        int pos = b * 64 + 4 * k + t;
        uint8_t byte;
        if (pos < len) byte = msg[pos];
        else if (pos == len) byte = 0x80;
        else byte = 0;
        x = (x << 8) | byte;
      }
      ww[k] = x;
    }
    if (b == nblk - 1) {
      uint64_t bits = (uint64_t)total * 8;
      ww[14] = (uint32_t)(bits >> 32);
      ww[15] = (uint32_t)bits;
    }
    sha256_compress(h, ww);
  }
}

static __device__ void hmac_sha256(const uint8_t key[32], const uint8_t* msg, int len, uint8_t out[32]) {
  uint8_t pad[64];
  uint32_t ih[8], oh[8];
  for (int k = 0; k < 64; ++k) pad[k] = (k < 32 ? key[k] : 0) ^ 0x36;
  sha256_bytes(pad, msg, len, ih);
  uint8_t inner[32];
  for (int k = 0; k < 8; ++k) {
    inner[4 * k] = (uint8_t)(ih[k] >> 24);
    inner[4 * k + 1] = (uint8_t)(ih[k] >> 16);
    inner[4 * k + 2] = (uint8_t)(ih[k] >> 8);
    inner[4 * k + 3] = (uint8_t)ih[k];
  }
  for (int k = 0; k < 64; ++k) pad[k] = (k < 32 ? key[k] : 0) ^ 0x5c;
  sha256_bytes(pad, inner, 32, oh);
  for (int k = 0; k < 8; ++k) {
    out[4 * k] = (uint8_t)(oh[k] >> 24);
    out[4 * k + 1] = (uint8_t)(oh[k] >> 16);
    out[4 * k + 2] = (uint8_t)(oh[k] >> 8);
    out[4 * k + 3] = (uint8_t)oh[k];
  }
}

// EthereumConsensusSigner::sign (signing/ethereum.rs:58-64) given the EIP-191 prehash:
// k256 sign_prehash_recoverable = RFC 6979 (HMAC-SHA256) nonce, low-s normalisation,
// alloy as_bytes() = r || s || (27 + y_parity).
static __device__ void sign_prehash(const fe& d, const uint32_t* z_digest, const uint32_t* fb, uint8_t* o) {
  fe zr, z;
  fe_from_digest(zr, z_digest);
  sc_reduce(z, zr);
  uint8_t x[32], h1[32];
  fe_store_be(x, d);
  fe_store_be(h1, z);
  uint8_t V[32], K[32], buf[97];
  for (int k = 0; k < 32; ++k) {
    V[k] = 1;
    K[k] = 0;
  }
  for (int step = 0; step < 2; ++step) {
    for (int k = 0; k < 32; ++k) buf[k] = V[k];
    buf[32] = (uint8_t)step;
    for (int k = 0; k < 32; ++k) {
      buf[33 + k] = x[k];
      buf[65 + k] = h1[k];
    }
    hmac_sha256(K, buf, 97, K);
    hmac_sha256(K, V, 32, V);
  }
  fe k;
  for (;;) {
    hmac_sha256(K, V, 32, V);
    fe_load_be(k, V);
    if (!fe_is_zero(k) && !sc_is_ge_n(k)) break;
    for (int q = 0; q < 32; ++q) buf[q] = V[q];
    buf[32] = 0;
    hmac_sha256(K, buf, 33, K);
    hmac_sha256(K, V, 32, V);
  }
  gej Rj;
  fixed_base_mul(Rj, k, fb);
  fe rx, ry, r;
  gej_to_affine(rx, ry, Rj);
  uint32_t y_odd = ry.v[0] & 1u;
  sc_reduce(r, rx);
  // s = k^-1 (z + r d) mod n
  fe r2c, km, kinv, rR, rd, t, s;
  sc_r2(r2c);
  sc_mont_mul(km, k, r2c);
  fe kinv_plain;
  sc_inv(kinv_plain, k);
  sc_mont_mul(kinv, kinv_plain, r2c);  // k^-1 * R
  sc_mont_mul(rR, r, r2c);
  sc_mont_mul(rd, rR, d);
  sc_add(t, z, rd);
  sc_mont_mul(s, kinv, t);
  fe h;
#pragma unroll
  for (int q = 0; q < 8; ++q) h.v[q] = nhalf_limb(q);
  if (u256_lt(h, s)) {
    sc_neg(s, s);
    y_odd ^= 1u;
  }
  fe_store_be(o, r);
  fe_store_be(o + 32, s);
  o[64] = (uint8_t)(27 + y_odd);
}

}  // namespace hlc
