// hlc_hash.hpp -- register-resident keccak-f[1600] and SHA-256 compression for gfx950.
//
// keccak256 replaces alloy-primitives' keccak256 (EIP-191 prehash + pubkey->address inside
// recover_address_from_msg, /root/reference/src/signing/ethereum.rs:89); SHA-256 replaces
// sha2 0.10.9 in compute_vote_hash (/root/reference/src/utils.rs:37-47).
// Both keep their whole state in VGPRs (25 x u64 / 8 x u32 + a 16-word schedule ring);
// every array index is a compile-time constant after unrolling, so nothing spills to scratch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef HLC_DEV
#define HLC_DEV __device__ __forceinline__
#endif

namespace hlc {

__constant__ static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

// 64-bit rotate on the two 32-bit halves: two v_alignbit_b32 (the compiler's own lowering of the
// shift-or form costs two 64-bit shifts and two ORs per rotation); n is a compile-time constant
HLC_DEV uint64_t rol64(uint64_t x, int n) {
  if (n == 0) return x;
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n >= 32) {
    const uint32_t t = lo;
    lo = hi;
    hi = t;
    n -= 32;
    if (n == 0) return ((uint64_t)hi << 32) | lo;
  }
  const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - n);
  const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - n);
  return ((uint64_t)nhi << 32) | nlo;
}

// gfx950 three-input bitwise ops (v_bitop3_b32, truth table indexed by a*4 + b*2 + c) on the two
// halves of a 64-bit lane: a ^ b ^ c (0x96) and keccak's chi a ^ (~b & c) (0xD2), one instruction
// per half where the shift-free lowering took two
HLC_DEV uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
  return ((uint64_t)hi << 32) | lo;
}
HLC_DEV uint64_t chi64(uint64_t a, uint64_t b, uint64_t c) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xD2);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xD2);
  return ((uint64_t)hi << 32) | lo;
}

// In-place keccak-f[1600]; a[x + 5y].
HLC_DEV void keccak_f1600(uint64_t a[25]) {
  for (int round = 0; round < 24; ++round) {
    uint64_t c0 = xor3_64(xor3_64(a[0], a[5], a[10]), a[15], a[20]);
    uint64_t c1 = xor3_64(xor3_64(a[1], a[6], a[11]), a[16], a[21]);
    uint64_t c2 = xor3_64(xor3_64(a[2], a[7], a[12]), a[17], a[22]);
    uint64_t c3 = xor3_64(xor3_64(a[3], a[8], a[13]), a[18], a[23]);
    uint64_t c4 = xor3_64(xor3_64(a[4], a[9], a[14]), a[19], a[24]);
    uint64_t d0 = c4 ^ rol64(c1, 1), d1 = c0 ^ rol64(c2, 1), d2 = c1 ^ rol64(c3, 1);
    uint64_t d3 = c2 ^ rol64(c4, 1), d4 = c3 ^ rol64(c0, 1);
    // theta + rho + pi into b[]
    uint64_t b[25];
    b[0] = a[0] ^ d0;
    b[10] = rol64(a[1] ^ d1, 1);
    b[20] = rol64(a[2] ^ d2, 62);
    b[5] = rol64(a[3] ^ d3, 28);
    b[15] = rol64(a[4] ^ d4, 27);
    b[16] = rol64(a[5] ^ d0, 36);
    b[1] = rol64(a[6] ^ d1, 44);
    b[11] = rol64(a[7] ^ d2, 6);
    b[21] = rol64(a[8] ^ d3, 55);
    b[6] = rol64(a[9] ^ d4, 20);
    b[7] = rol64(a[10] ^ d0, 3);
    b[17] = rol64(a[11] ^ d1, 10);
    b[2] = rol64(a[12] ^ d2, 43);
    b[12] = rol64(a[13] ^ d3, 25);
    b[22] = rol64(a[14] ^ d4, 39);
    b[23] = rol64(a[15] ^ d0, 41);
    b[8] = rol64(a[16] ^ d1, 45);
    b[18] = rol64(a[17] ^ d2, 15);
    b[3] = rol64(a[18] ^ d3, 21);
    b[13] = rol64(a[19] ^ d4, 8);
    b[14] = rol64(a[20] ^ d0, 18);
    b[24] = rol64(a[21] ^ d1, 2);
    b[9] = rol64(a[22] ^ d2, 61);
    b[19] = rol64(a[23] ^ d3, 56);
    b[4] = rol64(a[24] ^ d4, 14);
    // chi + iota
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      uint64_t b0 = b[y], b1 = b[y + 1], b2 = b[y + 2], b3 = b[y + 3], b4 = b[y + 4];
      a[y] = chi64(b0, b1, b2);
      a[y + 1] = chi64(b1, b2, b3);
      a[y + 2] = chi64(b2, b3, b4);
      a[y + 3] = chi64(b3, b4, b0);
      a[y + 4] = chi64(b4, b0, b1);
    }
    a[0] ^= KECCAK_RC[round];
  }
}

__constant__ static const uint32_t SHA256_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

HLC_DEV uint32_t ror32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
HLC_DEV uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

HLC_DEV void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

// One compression over 16 big-endian-decoded message words (w is consumed).
HLC_DEV void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int r = 0; r < 64; r += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (r > 0) {
        uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
        uint32_t s0 = xor3_32(ror32(w15, 7), ror32(w15, 18), w15 >> 3);
        uint32_t s1 = xor3_32(ror32(w2, 17), ror32(w2, 19), w2 >> 10);
        w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
      }
      uint32_t S1 = xor3_32(ror32(e, 6), ror32(e, 11), ror32(e, 25));
      uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);    // e ? f : g
      uint32_t t1 = hh + S1 + ch + SHA256_K[r + j] + w[j];
      uint32_t S0 = xor3_32(ror32(a, 2), ror32(a, 13), ror32(a, 22));
      uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);    // majority
      uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

HLC_DEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

}  // namespace hlc
