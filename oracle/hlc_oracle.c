/*
 * hlc_oracle.c -- C CPU restatement of the hashgraph-like-consensus vote-validation path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the timed CPU
 * baseline ("kind": "port").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it.  The product (libhlc.so, HIP) never links it.
 *
 * It is an independent restatement of the same semantics as oracle/pyoracle.py, with a
 * deliberately different algorithm from the GPU kernels (4x64-bit limbs, 4-bit fixed
 * windows, no GLV, per-item Fermat inversions) so that agreement is evidence rather than
 * shared bugs.  A second, k256-class recovery (GLV + wNAF + binary-GCD inversions, flag
 * HLCO_GLV) is the timed CPU baseline; it must agree with the checker item for item.  Reference call sites restated (paths under /root/reference):
 *   compute_vote_hash        src/utils.rs:37-47          (sha2 0.10.9)
 *   validate_vote            src/utils.rs:127-171
 *   Vote encode_to_vec       src/utils.rs:150-152        (prost 0.14.4, consensus.proto:19-29)
 *   EthereumConsensusSigner::verify  src/signing/ethereum.rs:66-97
 *     -> alloy-primitives 1.6.0 from_raw_array / normalize_v / normalized_s /
 *        eip191_hash_message / recover_address_from_msg
 *     -> k256 0.13.4 VerifyingKey::recover_from_prehash (recover, then verify_prehash)
 *   validate_vote_chain      src/utils.rs:175-215
 *   validate_proposal        src/utils.rs:106-120
 *   initialize_with_votes    src/session.rs:253-298, check_round_limit 306-344
 *   calculate_consensus_result / thresholds  src/utils.rs:227-313
 *   EthereumConsensusSigner::sign  src/signing/ethereum.rs:58-64 (RFC 6979, low-s, v=27+y)
 * Parity pinning: see oracle/pyoracle.py header and tests/test_oracle_kats.py.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/hlc.h"

/* hlco_ecrecover / validate flags: also run k256's post-recovery verify_prehash; use the
 * k256-class GLV path instead of the independent non-GLV checker */
#define HLCO_REVERIFY 1
#define HLCO_GLV 2
/* the scheme is tests/custom_scheme_tests.rs's StubSigner (:33-74) instead of EthereumConsensusSigner:
 * an 8-byte identity, signature = SHA256(identity || payload) -- ConsensusService is generic over the
 * scheme (src/service.rs:39-51, src/signing.rs:46-74) */
#define HLCO_STUB 4

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;
typedef unsigned __int128 u128;

/* ================================ SHA-256 ===================================== */
static const u32 K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

typedef struct {
  u32 h[8];
  u8 buf[64];
  u64 len;
} sha256_ctx;

#define ROR32(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(u32 h[8], const u8* p) {
  u32 w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = ((u32)p[4 * i] << 24) | ((u32)p[4 * i + 1] << 16) | ((u32)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    u32 s0 = ROR32(w[i - 15], 7) ^ ROR32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    u32 s1 = ROR32(w[i - 2], 17) ^ ROR32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    u32 S1 = ROR32(e, 6) ^ ROR32(e, 11) ^ ROR32(e, 25);
    u32 ch = (e & f) ^ (~e & g);
    u32 t1 = hh + S1 + ch + K256[i] + w[i];
    u32 S0 = ROR32(a, 2) ^ ROR32(a, 13) ^ ROR32(a, 22);
    u32 mj = (a & b) ^ (a & c) ^ (b & c);
    u32 t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha256_init(sha256_ctx* c) {
  static const u32 iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                            0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c->h, iv, sizeof iv);
  c->len = 0;
}

static void sha256_update(sha256_ctx* c, const u8* p, size_t n) {
  size_t fill = (size_t)(c->len & 63);
  c->len += n;
  if (fill) {
    size_t take = 64 - fill < n ? 64 - fill : n;
    memcpy(c->buf + fill, p, take);
    p += take; n -= take; fill += take;
    if (fill < 64) return;
    sha256_block(c->h, c->buf);
  }
  while (n >= 64) { sha256_block(c->h, p); p += 64; n -= 64; }
  if (n) memcpy(c->buf, p, n);
}

static void sha256_final(sha256_ctx* c, u8 out[32]) {
  u64 bits = c->len * 8;
  u8 pad = 0x80, z = 0;
  sha256_update(c, &pad, 1);
  while ((c->len & 63) != 56) sha256_update(c, &z, 1);
  u8 lb[8];
  for (int i = 0; i < 8; ++i) lb[i] = (u8)(bits >> (56 - 8 * i));
  sha256_update(c, lb, 8);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (u8)(c->h[i] >> 24); out[4 * i + 1] = (u8)(c->h[i] >> 16);
    out[4 * i + 2] = (u8)(c->h[i] >> 8); out[4 * i + 3] = (u8)c->h[i];
  }
}

void hlco_sha256(const u8* p, size_t n, u8 out[32]) {
  sha256_ctx c;
  sha256_init(&c);
  sha256_update(&c, p, n);
  sha256_final(&c, out);
}

static void hmac_sha256(const u8* key, size_t klen, const u8* msg, size_t mlen, u8 out[32]) {
  u8 k[64] = {0}, ip[64], op[64], ih[32];
  if (klen > 64) hlco_sha256(key, klen, k); else memcpy(k, key, klen);
  for (int i = 0; i < 64; ++i) { ip[i] = k[i] ^ 0x36; op[i] = k[i] ^ 0x5c; }
  sha256_ctx c;
  sha256_init(&c); sha256_update(&c, ip, 64); sha256_update(&c, msg, mlen); sha256_final(&c, ih);
  sha256_init(&c); sha256_update(&c, op, 64); sha256_update(&c, ih, 32); sha256_final(&c, out);
}

/* ================================ Keccak-256 =================================== */
static const u64 KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

#define ROL64(x, n) ((n) ? (((x) << (n)) | ((x) >> (64 - (n)))) : (x))

static void keccakf(u64 a[25]) {
  for (int r = 0; r < 24; ++r) {
    u64 c[5], d[5], b[25];
    for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ ROL64(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) a[i] ^= d[i % 5];
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = ROL64(a[x + 5 * y], KROT[x + 5 * y]);
    for (int y = 0; y < 5; ++y)
      for (int x = 0; x < 5; ++x)
        a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= KRC[r];
  }
}

typedef struct {
  u64 s[25];
  size_t pos; /* bytes absorbed in current block */
} keccak_ctx;

static void keccak_init(keccak_ctx* k) { memset(k, 0, sizeof *k); }

static void keccak_update(keccak_ctx* k, const u8* p, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    k->s[k->pos >> 3] ^= (u64)p[i] << (8 * (k->pos & 7));
    if (++k->pos == 136) { keccakf(k->s); k->pos = 0; }
  }
}

static void keccak_final(keccak_ctx* k, u8 out[32]) {
  k->s[k->pos >> 3] ^= (u64)0x01 << (8 * (k->pos & 7));
  k->s[135 >> 3] ^= (u64)0x80 << (8 * (135 & 7));
  keccakf(k->s);
  for (int i = 0; i < 32; ++i) out[i] = (u8)(k->s[i >> 3] >> (8 * (i & 7)));
}

void hlco_keccak256(const u8* p, size_t n, u8 out[32]) {
  keccak_ctx k;
  keccak_init(&k);
  keccak_update(&k, p, n);
  keccak_final(&k, out);
}

/* ======================== 256-bit helpers (4 x 64, little endian) ================ */
typedef struct { u64 v[4]; } u256;

static const u256 FP = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 FN = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 FN_HALF = {{0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL, 0x7FFFFFFFFFFFFFFFULL}};
/* 2^256 - n */
static const u64 NC[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL};

static u256 u256_from_be(const u8* b) {
  u256 r;
  for (int i = 0; i < 4; ++i) {
    u64 w = 0;
    for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
    r.v[i] = w;
  }
  return r;
}

static void u256_to_be(const u256* a, u8* b) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (u8)(a->v[i] >> (56 - 8 * j));
}

static int u256_cmp(const u256* a, const u256* b) {
  for (int i = 3; i >= 0; --i) {
    if (a->v[i] < b->v[i]) return -1;
    if (a->v[i] > b->v[i]) return 1;
  }
  return 0;
}

static int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }

static u64 u256_add(u256* r, const u256* a, const u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (u64)c; c >>= 64; }
  return (u64)c;
}

static u64 u256_sub(u256* r, const u256* a, const u256* b) {
  u64 borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 t = (u128)a->v[i] - b->v[i] - borrow;
    r->v[i] = (u64)t;
    borrow = (u64)(t >> 64) & 1;
  }
  return borrow;
}

static void mul256(u64 w[8], const u256* a, const u256* b) {
  memset(w, 0, 8 * sizeof(u64));
  for (int i = 0; i < 4; ++i) {
    u64 carry = 0;
    for (int j = 0; j < 4; ++j) {
      u128 t = (u128)a->v[i] * b->v[j] + w[i + j] + carry;
      w[i + j] = (u64)t;
      carry = (u64)(t >> 64);
    }
    w[i + 4] = carry;
  }
}

/* ================================ Field mod p ================================== */
typedef u256 fe;

static void fe_reduce512(fe* r, const u64 w[8]) {
  /* 2^256 == 0x1000003D1 (mod p) */
  const u64 C = 0x1000003D1ULL;
  u128 c = 0;
  u64 t[5];
  for (int i = 0; i < 4; ++i) { c += (u128)w[4 + i] * C + w[i]; t[i] = (u64)c; c >>= 64; }
  t[4] = (u64)c;
  c = (u128)t[4] * C + t[0]; t[0] = (u64)c; c >>= 64;
  for (int i = 1; i < 4; ++i) { c += t[i]; t[i] = (u64)c; c >>= 64; }
  if (c) { /* one more wrap: add C */
    u128 d = (u128)t[0] + C; t[0] = (u64)d; d >>= 64;
    for (int i = 1; i < 4 && d; ++i) { d += t[i]; t[i] = (u64)d; d >>= 64; }
  }
  memcpy(r->v, t, 32);
  if (u256_cmp(r, &FP) >= 0) u256_sub(r, r, &FP);
}

static void fe_mul(fe* r, const fe* a, const fe* b) { u64 w[8]; mul256(w, a, b); fe_reduce512(r, w); }
static void fe_sqr(fe* r, const fe* a) { fe_mul(r, a, a); }
static void fe_add(fe* r, const fe* a, const fe* b) {
  u64 c = u256_add(r, a, b);
  if (c || u256_cmp(r, &FP) >= 0) u256_sub(r, r, &FP);
}
static void fe_sub(fe* r, const fe* a, const fe* b) {
  if (u256_sub(r, a, b)) u256_add(r, r, &FP);
}
static void fe_neg(fe* r, const fe* a) {
  if (u256_is_zero(a)) { *r = *a; return; }
  u256_sub(r, &FP, a);
}
static void fe_set_u32(fe* r, u32 v) { memset(r, 0, sizeof *r); r->v[0] = v; }
static void fe_sqr_n(fe* r, const fe* a, int n) { *r = *a; for (int i = 0; i < n; ++i) fe_sqr(r, r); }

/* Shared prefix of the libsecp256k1-style addition chains for p-2 and (p+1)/4. */
static void fe_chain223(const fe* a, fe* x2, fe* x3, fe* x22, fe* x223) {
  fe t, x6, x9, x11, x44, x88, x176, x220;
  fe_sqr(&t, a); fe_mul(x2, &t, a);
  fe_sqr(&t, x2); fe_mul(x3, &t, a);
  fe_sqr_n(&t, x3, 3); fe_mul(&x6, &t, x3);
  fe_sqr_n(&t, &x6, 3); fe_mul(&x9, &t, x3);
  fe_sqr_n(&t, &x9, 2); fe_mul(&x11, &t, x2);
  fe_sqr_n(&t, &x11, 11); fe_mul(x22, &t, &x11);
  fe_sqr_n(&t, x22, 22); fe_mul(&x44, &t, x22);
  fe_sqr_n(&t, &x44, 44); fe_mul(&x88, &t, &x44);
  fe_sqr_n(&t, &x88, 88); fe_mul(&x176, &t, &x88);
  fe_sqr_n(&t, &x176, 44); fe_mul(&x220, &t, &x44);
  fe_sqr_n(&t, &x220, 3); fe_mul(x223, &t, x3);
}

static void fe_inv(fe* r, const fe* a) {
  fe x2, x3, x22, x223, t;
  fe_chain223(a, &x2, &x3, &x22, &x223);
  fe_sqr_n(&t, &x223, 23); fe_mul(&t, &t, &x22);
  fe_sqr_n(&t, &t, 5); fe_mul(&t, &t, a);
  fe_sqr_n(&t, &t, 3); fe_mul(&t, &t, &x2);
  fe_sqr_n(&t, &t, 2); fe_mul(r, &t, a);
}

/* returns 1 if a is a square; r = sqrt(a) */
static int fe_sqrt(fe* r, const fe* a) {
  fe x2, x3, x22, x223, t, chk;
  fe_chain223(a, &x2, &x3, &x22, &x223);
  fe_sqr_n(&t, &x223, 23); fe_mul(&t, &t, &x22);
  fe_sqr_n(&t, &t, 6); fe_mul(&t, &t, &x2);
  fe_sqr_n(r, &t, 2);
  fe_sqr(&chk, r);
  return u256_cmp(&chk, a) == 0;
}

/* ================================ Scalar mod n ================================= */
typedef u256 sc;

static void sc_reduce512(sc* r, const u64 w[8]) {
  /* fold hi * (2^256 - n) into lo, twice, then conditional subtracts */
  u64 t[8];
  memcpy(t, w, sizeof t);
  for (int round = 0; round < 3; ++round) {
    u64 hi[4] = {t[4], t[5], t[6], t[7]};
    if ((hi[0] | hi[1] | hi[2] | hi[3]) == 0) break;
    u64 acc[8] = {t[0], t[1], t[2], t[3], 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
      u64 carry = 0;
      for (int j = 0; j < 3; ++j) {
        u128 x = (u128)hi[i] * NC[j] + acc[i + j] + carry;
        acc[i + j] = (u64)x;
        carry = (u64)(x >> 64);
      }
      for (int k = i + 3; k < 8 && carry; ++k) {
        u128 x = (u128)acc[k] + carry;
        acc[k] = (u64)x;
        carry = (u64)(x >> 64);
      }
    }
    memcpy(t, acc, sizeof t);
  }
  memcpy(r->v, t, 32);
  while (u256_cmp(r, &FN) >= 0) u256_sub(r, r, &FN);
}

static void sc_mul(sc* r, const sc* a, const sc* b) { u64 w[8]; mul256(w, a, b); sc_reduce512(r, w); }
static void sc_add(sc* r, const sc* a, const sc* b) {
  u64 c = u256_add(r, a, b);
  if (c || u256_cmp(r, &FN) >= 0) u256_sub(r, r, &FN);
}
static void sc_neg(sc* r, const sc* a) {
  if (u256_is_zero(a)) { *r = *a; return; }
  u256_sub(r, &FN, a);
}
static void sc_inv(sc* r, const sc* a) {
  /* a^(n-2), 4-bit fixed window */
  sc tab[16];
  memset(&tab[0], 0, sizeof tab[0]); tab[0].v[0] = 1;
  for (int i = 1; i < 16; ++i) sc_mul(&tab[i], &tab[i - 1], a);
  u256 e = FN; e.v[0] -= 2;
  sc acc = tab[0];
  for (int i = 63; i >= 0; --i) {
    for (int k = 0; k < 4; ++k) sc_mul(&acc, &acc, &acc);
    int d = (int)((e.v[i >> 4] >> (4 * (i & 15))) & 15);
    if (d) sc_mul(&acc, &acc, &tab[d]);
  }
  *r = acc;
}
static void sc_reduce_be32(sc* r, const u8* b) {
  *r = u256_from_be(b);
  while (u256_cmp(r, &FN) >= 0) u256_sub(r, r, &FN);
}

/* ================================ Group law ==================================== */
typedef struct { fe x, y, z; int inf; } gej;
typedef struct { fe x, y; int inf; } ge;

static const fe GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const fe GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};

static void gej_set_ge(gej* r, const ge* a) {
  r->x = a->x; r->y = a->y; fe_set_u32(&r->z, 1); r->inf = a->inf;
}

static void gej_double(gej* r, const gej* a) {
  if (a->inf || u256_is_zero(&a->y)) { r->inf = 1; return; }
  fe A, B, C, D, E, F, t, x3, y3, z3;
  fe_sqr(&A, &a->x);
  fe_sqr(&B, &a->y);
  fe_sqr(&C, &B);
  fe_add(&t, &a->x, &B); fe_sqr(&t, &t); fe_sub(&t, &t, &A); fe_sub(&t, &t, &C); fe_add(&D, &t, &t);
  fe_add(&E, &A, &A); fe_add(&E, &E, &A);
  fe_sqr(&F, &E);
  fe_add(&t, &D, &D); fe_sub(&x3, &F, &t);
  fe_sub(&t, &D, &x3); fe_mul(&y3, &E, &t);
  fe_add(&t, &C, &C); fe_add(&t, &t, &t); fe_add(&t, &t, &t); fe_sub(&y3, &y3, &t);
  fe_mul(&z3, &a->y, &a->z); fe_add(&z3, &z3, &z3);
  r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}

static void gej_add_ge(gej* r, const gej* a, const ge* b) {
  if (b->inf) { *r = *a; return; }
  if (a->inf) { gej_set_ge(r, b); return; }
  fe z1z1, u2, s2, h, rr, hh, hhh, v, t, x3, y3, z3;
  fe_sqr(&z1z1, &a->z);
  fe_mul(&u2, &b->x, &z1z1);
  fe_mul(&s2, &b->y, &a->z); fe_mul(&s2, &s2, &z1z1);
  fe_sub(&h, &u2, &a->x);
  fe_sub(&rr, &s2, &a->y);
  if (u256_is_zero(&h)) {
    if (u256_is_zero(&rr)) { gej_double(r, a); return; }
    r->inf = 1; return;
  }
  fe_sqr(&hh, &h); fe_mul(&hhh, &h, &hh); fe_mul(&v, &a->x, &hh);
  fe_sqr(&x3, &rr); fe_sub(&x3, &x3, &hhh); fe_add(&t, &v, &v); fe_sub(&x3, &x3, &t);
  fe_sub(&t, &v, &x3); fe_mul(&y3, &rr, &t); fe_mul(&t, &a->y, &hhh); fe_sub(&y3, &y3, &t);
  fe_mul(&z3, &a->z, &h);
  r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}

static void gej_add(gej* r, const gej* a, const gej* b) {
  if (b->inf) { *r = *a; return; }
  if (a->inf) { *r = *b; return; }
  fe z1z1, z2z2, u1, u2, s1, s2, h, rr, hh, hhh, v, t, x3, y3, z3;
  fe_sqr(&z1z1, &a->z); fe_sqr(&z2z2, &b->z);
  fe_mul(&u1, &a->x, &z2z2); fe_mul(&u2, &b->x, &z1z1);
  fe_mul(&s1, &a->y, &b->z); fe_mul(&s1, &s1, &z2z2);
  fe_mul(&s2, &b->y, &a->z); fe_mul(&s2, &s2, &z1z1);
  fe_sub(&h, &u2, &u1); fe_sub(&rr, &s2, &s1);
  if (u256_is_zero(&h)) {
    if (u256_is_zero(&rr)) { gej_double(r, a); return; }
    r->inf = 1; return;
  }
  fe_sqr(&hh, &h); fe_mul(&hhh, &h, &hh); fe_mul(&v, &u1, &hh);
  fe_sqr(&x3, &rr); fe_sub(&x3, &x3, &hhh); fe_add(&t, &v, &v); fe_sub(&x3, &x3, &t);
  fe_sub(&t, &v, &x3); fe_mul(&y3, &rr, &t); fe_mul(&t, &s1, &hhh); fe_sub(&y3, &y3, &t);
  fe_mul(&z3, &a->z, &b->z); fe_mul(&z3, &z3, &h);
  r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}

static void gej_to_ge(ge* r, const gej* a) {
  if (a->inf) { r->inf = 1; return; }
  fe zi, zi2, zi3;
  fe_inv(&zi, &a->z); fe_sqr(&zi2, &zi); fe_mul(&zi3, &zi2, &zi);
  fe_mul(&r->x, &a->x, &zi2); fe_mul(&r->y, &a->y, &zi3); r->inf = 0;
}

/* G table: k*G for k = 0..15 (affine), built once. */
static ge GTAB[16];
static pthread_once_t gtab_once = PTHREAD_ONCE_INIT;
static void build_gtab(void) {
  ge g = {GX, GY, 0};
  gej acc;
  GTAB[0].inf = 1;
  GTAB[1] = g;
  gej_set_ge(&acc, &g);
  for (int i = 2; i < 16; ++i) { gej_add_ge(&acc, &acc, &g); gej_to_ge(&GTAB[i], &acc); }
}

static int scalar_nibble(const sc* k, int i) { return (int)((k->v[i >> 4] >> (4 * (i & 15))) & 15); }

/* r = a*G + b*P (Shamir's trick, 4-bit fixed windows) */
static void ecmult(gej* r, const sc* a, const ge* P, const sc* b) {
  pthread_once(&gtab_once, build_gtab);
  gej ptab[16];
  ptab[0].inf = 1;
  gej_set_ge(&ptab[1], P);
  for (int i = 2; i < 16; ++i) gej_add_ge(&ptab[i], &ptab[i - 1], P);
  gej acc; acc.inf = 1;
  for (int i = 63; i >= 0; --i) {
    if (!acc.inf) for (int k = 0; k < 4; ++k) gej_double(&acc, &acc);
    int da = scalar_nibble(a, i), db = scalar_nibble(b, i);
    if (da) gej_add_ge(&acc, &acc, &GTAB[da]);
    if (db) gej_add(&acc, &acc, &ptab[db]);
  }
  *r = acc;
}

/* ============== k256-class scalar multiplication (the timed CPU baseline) ==============
 * The recovery algorithm class of k256 0.13.4 (/root/reference/Cargo.lock; reached at
 * src/signing/ethereum.rs:89 through alloy's recover_address_from_msg), written the faster
 * libsecp256k1 way so that the CPU baseline is conservative:
 *   - GLV endomorphism: every scalar k = k1 + k2 lambda with |k1|, |k2| < 2^128 (k256 lincomb's
 *     decompose_scalar), so the doubling chain is 129 steps, not 256;
 *   - variable-time wNAF digits: width 5 for the per-signature point R (odd multiples 1..15 R and
 *     lambda R, made affine with ONE field inversion by Montgomery's trick), width 8 for G (64 odd
 *     multiples of G and lambda G, affine, built once);
 *   - binary extended-Euclid inversions mod p and mod n (k256 uses Fermat chains);
 *   - Jacobian doublings 2M+5S and mixed additions 8M+3S (k256's complete projective formulas cost
 *     more per operation).
 * The non-GLV path above (ecmult) stays the independent checker; the two must agree on every
 * item (tests/test_openssl_pin.py). */
static const sc GLV_LAMBDA = {{0xDF02967C1B23BD72ULL, 0x122E22EA20816678ULL, 0xA5261C028812645AULL, 0x5363AD4CC05C30E0ULL}};
static const fe GLV_BETA = {{0xC1396C28719501EEULL, 0x9CF0497512F58995ULL, 0x6E64479EAC3434E9ULL, 0x7AE96A2B657C0710ULL}};
static const sc GLV_MINUS_B1 = {{0x6F547FA90ABFE4C3ULL, 0xE4437ED6010E8828ULL, 0, 0}};
static const sc GLV_MINUS_B2 = {{0xD765CDA83DB1562CULL, 0x8A280AC50774346DULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 GLV_G1 = {{0xE893209A45DBB031ULL, 0x3DAA8A1471E8CA7FULL, 0xE86C90E49284EB15ULL, 0x3086D221A7D46BCDULL}};
static const u256 GLV_G2 = {{0x1571B4AE8AC47F71ULL, 0x221208AC9DF506C6ULL, 0x6F547FA90ABFE4C4ULL, 0xE4437ED6010E8828ULL}};

/* round(k g / 2^384) */
static u256 mul_shift_384(const u256* k, const u256* g) {
  u64 w[8];
  mul256(w, k, g);
  u256 r = {{w[6], w[7], 0, 0}};
  if (w[5] >> 63) {
    u256 one = {{1, 0, 0, 0}};
    u256_add(&r, &r, &one);
  }
  return r;
}

/* k = k1 + k2 lambda (mod n): magnitudes < 2^129 and signs (libsecp256k1 scalar_split_lambda) */
static void glv_split(const sc* k, sc* k1, int* neg1, sc* k2, int* neg2) {
  u256 c1 = mul_shift_384(k, &GLV_G1), c2 = mul_shift_384(k, &GLV_G2);
  sc t1, t2, r2, r1;
  sc_mul(&t1, &c1, &GLV_MINUS_B1);
  sc_mul(&t2, &c2, &GLV_MINUS_B2);
  sc_add(&r2, &t1, &t2);
  sc_mul(&t1, &r2, &GLV_LAMBDA);
  sc_neg(&t1, &t1);
  sc_add(&r1, k, &t1);
  *neg1 = u256_cmp(&r1, &FN_HALF) > 0;
  *neg2 = u256_cmp(&r2, &FN_HALF) > 0;
  if (*neg1) sc_neg(&r1, &r1);
  if (*neg2) sc_neg(&r2, &r2);
  *k1 = r1;
  *k2 = r2;
}

/* width-w NAF of k (< 2^130): digits[i] odd in (-2^(w-1), 2^(w-1)) or 0; returns the length */
static int wnaf(int* d, const u256* k, int w) {
  u256 x = *k;
  int len = 0;
  memset(d, 0, 132 * sizeof(int));
  while (!u256_is_zero(&x)) {
    int digit = 0;
    if (x.v[0] & 1) {
      digit = (int)(x.v[0] & ((1u << w) - 1));
      if (digit >= (1 << (w - 1))) digit -= (1 << w);
      u256 dv = {{(u64)(digit < 0 ? -digit : digit), 0, 0, 0}};
      if (digit < 0) u256_add(&x, &x, &dv); else u256_sub(&x, &x, &dv);
    }
    d[len++] = digit;
    for (int i = 0; i < 3; ++i) x.v[i] = (x.v[i] >> 1) | (x.v[i + 1] << 63);
    x.v[3] >>= 1;
  }
  return len;
}

/* a^-1 mod m (m odd, 0 < a < m) by the binary extended Euclidean algorithm (variable time) */
static void modinv_binary(u256* r, const u256* a, const u256* m) {
  u256 u = *a, v = *m, x1 = {{1, 0, 0, 0}}, x2 = {{0, 0, 0, 0}};
  const u256 one = {{1, 0, 0, 0}};
  while (u256_cmp(&u, &one) != 0 && u256_cmp(&v, &one) != 0) {
    while (!(u.v[0] & 1)) {
      for (int i = 0; i < 3; ++i) u.v[i] = (u.v[i] >> 1) | (u.v[i + 1] << 63);
      u.v[3] >>= 1;
      u64 c = 0;
      if (x1.v[0] & 1) c = u256_add(&x1, &x1, m);
      for (int i = 0; i < 3; ++i) x1.v[i] = (x1.v[i] >> 1) | (x1.v[i + 1] << 63);
      x1.v[3] = (x1.v[3] >> 1) | (c << 63);
    }
    while (!(v.v[0] & 1)) {
      for (int i = 0; i < 3; ++i) v.v[i] = (v.v[i] >> 1) | (v.v[i + 1] << 63);
      v.v[3] >>= 1;
      u64 c = 0;
      if (x2.v[0] & 1) c = u256_add(&x2, &x2, m);
      for (int i = 0; i < 3; ++i) x2.v[i] = (x2.v[i] >> 1) | (x2.v[i + 1] << 63);
      x2.v[3] = (x2.v[3] >> 1) | (c << 63);
    }
    if (u256_cmp(&u, &v) >= 0) {
      u256_sub(&u, &u, &v);
      if (u256_sub(&x1, &x1, &x2)) u256_add(&x1, &x1, m);
    } else {
      u256_sub(&v, &v, &u);
      if (u256_sub(&x2, &x2, &x1)) u256_add(&x2, &x2, m);
    }
  }
  *r = u256_cmp(&u, &one) == 0 ? x1 : x2;
}

static void gej_to_ge_bin(ge* r, const gej* a) {
  if (a->inf) { r->inf = 1; return; }
  fe zi, zi2, zi3;
  modinv_binary(&zi, &a->z, &FP);
  fe_sqr(&zi2, &zi); fe_mul(&zi3, &zi2, &zi);
  fe_mul(&r->x, &a->x, &zi2); fe_mul(&r->y, &a->y, &zi3); r->inf = 0;
}

/* odd multiples (2i+1) P, i < n, made affine with one inversion (Montgomery's trick) */
static void odd_multiples_affine(ge* out, const ge* P, int n) {
  gej pj[64], d;
  gej_set_ge(&pj[0], P);
  gej_double(&d, &pj[0]);
  ge d_aff;
  gej_to_ge_bin(&d_aff, &d);
  for (int i = 1; i < n; ++i) gej_add_ge(&pj[i], &pj[i - 1], &d_aff);
  fe pre[64], inv, t;
  pre[0] = pj[0].z;
  for (int i = 1; i < n; ++i) fe_mul(&pre[i], &pre[i - 1], &pj[i].z);
  modinv_binary(&inv, &pre[n - 1], &FP);
  for (int i = n - 1; i >= 0; --i) {
    fe zi, zi2, zi3;
    if (i) { fe_mul(&zi, &inv, &pre[i - 1]); fe_mul(&inv, &inv, &pj[i].z); } else zi = inv;
    fe_sqr(&zi2, &zi); fe_mul(&zi3, &zi2, &zi);
    fe_mul(&out[i].x, &pj[i].x, &zi2); fe_mul(&out[i].y, &pj[i].y, &zi3); out[i].inf = 0;
    (void)t;
  }
}

#define GLV_WG 8
static ge GTAB_GLV[1 << (GLV_WG - 2)], GTAB_GLV_L[1 << (GLV_WG - 2)];
static pthread_once_t gtab_glv_once = PTHREAD_ONCE_INIT;
static void build_gtab_glv(void) {
  ge g = {GX, GY, 0};
  odd_multiples_affine(GTAB_GLV, &g, 1 << (GLV_WG - 2));
  for (int i = 0; i < (1 << (GLV_WG - 2)); ++i) {
    fe_mul(&GTAB_GLV_L[i].x, &GTAB_GLV[i].x, &GLV_BETA);
    GTAB_GLV_L[i].y = GTAB_GLV[i].y;
    GTAB_GLV_L[i].inf = 0;
  }
}

static void add_digit(gej* acc, const ge* tab, int d, int neg) {
  if (!d) return;
  ge e = tab[((d < 0 ? -d : d) - 1) >> 1];
  if ((d < 0) != (neg != 0)) fe_neg(&e.y, &e.y);
  gej_add_ge(acc, acc, &e);
}

/* r = a G + b P, GLV + wNAF (see above) */
static void ecmult_glv(gej* r, const sc* a, const ge* P, const sc* b) {
  pthread_once(&gtab_glv_once, build_gtab_glv);
  sc a1, a2, b1, b2;
  int na1, na2, nb1, nb2;
  glv_split(a, &a1, &na1, &a2, &na2);
  glv_split(b, &b1, &nb1, &b2, &nb2);
  int da1[132], da2[132], db1[132], db2[132];
  int la1 = wnaf(da1, &a1, GLV_WG), la2 = wnaf(da2, &a2, GLV_WG);
  int lb1 = wnaf(db1, &b1, 5), lb2 = wnaf(db2, &b2, 5);
  ge pt[8], ptl[8];
  odd_multiples_affine(pt, P, 8);
  for (int i = 0; i < 8; ++i) { fe_mul(&ptl[i].x, &pt[i].x, &GLV_BETA); ptl[i].y = pt[i].y; ptl[i].inf = 0; }
  int len = la1;
  if (la2 > len) len = la2;
  if (lb1 > len) len = lb1;
  if (lb2 > len) len = lb2;
  gej acc;
  acc.inf = 1;
  for (int i = len - 1; i >= 0; --i) {
    if (!acc.inf) gej_double(&acc, &acc);
    add_digit(&acc, pt, db1[i], nb1);
    add_digit(&acc, ptl, db2[i], nb2);
    add_digit(&acc, GTAB_GLV, da1[i], na1);
    add_digit(&acc, GTAB_GLV_L, da2[i], na2);
  }
  *r = acc;
}

/* ================================ ECDSA ======================================== */
static void ge_to_address(const ge* q, u8 addr[20]) {
  u8 buf[64], h[32];
  u256_to_be(&q->x, buf);
  u256_to_be(&q->y, buf + 32);
  hlco_keccak256(buf, 64, h);
  memcpy(addr, h + 12, 20);
}

static long g_verify_failures = 0; /* post-recovery verify must never fail */

long hlco_verify_failures(void) { return g_verify_failures; }

/* alloy Signature::from_raw_array + recover_address_from_prehash (see pyoracle.ecrecover).
 * Returns HLC_SCHEME_* (0 = success, addr filled).  flags & HLCO_REVERIFY also runs k256's
 * post-recovery verify_prehash, as upstream does (timed CPU baseline). */
int hlco_ecrecover(const u8 prehash[32], const u8 sig[65], u8 addr[20], int flags) {
  const int reverify = flags & HLCO_REVERIFY, glv = flags & HLCO_GLV;
  u8 v = sig[64];
  int parity;
  if (v == 0 || v == 27) parity = 0;
  else if (v == 1 || v == 28) parity = 1;
  else if (v >= 35) parity = ((v - 35) % 2) != 0;
  else return HLC_SCHEME_BAD_PARITY;
  sc r = u256_from_be(sig), s = u256_from_be(sig + 32);
  if (u256_cmp(&s, &FN_HALF) > 0) { /* normalized_s (wrapping U256 sub) */
    u256_sub(&s, &FN, &s);
    parity ^= 1;
  }
  if (u256_is_zero(&r) || u256_cmp(&r, &FN) >= 0 || u256_is_zero(&s) || u256_cmp(&s, &FN) >= 0)
    return HLC_SCHEME_SCALAR_RANGE;
  sc z;
  sc_reduce_be32(&z, prehash);
  /* decompress R (x = r < n < p) */
  fe x = r, x3, y2, y;
  fe seven; fe_set_u32(&seven, 7);
  fe_sqr(&x3, &x); fe_mul(&x3, &x3, &x); fe_add(&y2, &x3, &seven);
  if (!fe_sqrt(&y, &y2)) return HLC_SCHEME_NO_POINT;
  if ((int)(y.v[0] & 1) != parity) fe_neg(&y, &y);
  ge R = {x, y, 0};
  sc rinv, u1, u2;
  if (glv) modinv_binary(&rinv, &r, &FN); else sc_inv(&rinv, &r);
  sc_mul(&u1, &z, &rinv); sc_neg(&u1, &u1);
  sc_mul(&u2, &s, &rinv);
  gej Qj;
  if (glv) ecmult_glv(&Qj, &u1, &R, &u2); else ecmult(&Qj, &u1, &R, &u2);
  if (Qj.inf) return HLC_SCHEME_INFINITY;
  ge Q;
  if (glv) gej_to_ge_bin(&Q, &Qj); else gej_to_ge(&Q, &Qj);
  if (reverify) {
    /* k256 verify_prehash: x(z/s G + r/s Q) mod n == r (low-s signature) */
    sc sinv, v1, v2;
    if (glv) modinv_binary(&sinv, &s, &FN); else sc_inv(&sinv, &s);
    sc_mul(&v1, &z, &sinv);
    sc_mul(&v2, &r, &sinv);
    gej Pj; ge Pa;
    if (glv) ecmult_glv(&Pj, &v1, &Q, &v2); else ecmult(&Pj, &v1, &Q, &v2);
    int ok = 0;
    if (!Pj.inf) {
      if (glv) gej_to_ge_bin(&Pa, &Pj); else gej_to_ge(&Pa, &Pj);
      sc xr = Pa.x;
      while (u256_cmp(&xr, &FN) >= 0) u256_sub(&xr, &xr, &FN);
      ok = u256_cmp(&xr, &r) == 0;
    }
    if (!ok) __atomic_fetch_add(&g_verify_failures, 1, __ATOMIC_RELAXED);
  }
  ge_to_address(&Q, addr);
  return HLC_SCHEME_NONE;
}

void hlco_address(const u8 priv[32], u8 addr[20]) {
  sc d = u256_from_be(priv), zero;
  memset(&zero, 0, sizeof zero);
  ge dummy = {GX, GY, 0};
  gej Pj; ge P;
  ecmult(&Pj, &d, &dummy, &zero);
  gej_to_ge(&P, &Pj);
  ge_to_address(&P, addr);
}

/* RFC 6979 (HMAC-SHA256) + k256 low-s normalisation + alloy v = 27 + y_parity */
void hlco_sign_prehash(const u8 priv[32], const u8 prehash[32], u8 sig[65]) {
  sc d = u256_from_be(priv), z;
  sc_reduce_be32(&z, prehash);
  u8 h1[32];
  u256_to_be(&z, h1);
  u8 V[32], K[32], buf[32 + 1 + 32 + 32];
  memset(V, 1, 32);
  memset(K, 0, 32);
  memcpy(buf, V, 32); buf[32] = 0; memcpy(buf + 33, priv, 32); memcpy(buf + 65, h1, 32);
  hmac_sha256(K, 32, buf, 97, K);
  hmac_sha256(K, 32, V, 32, V);
  memcpy(buf, V, 32); buf[32] = 1;
  hmac_sha256(K, 32, buf, 97, K);
  hmac_sha256(K, 32, V, 32, V);
  sc k;
  for (;;) {
    hmac_sha256(K, 32, V, 32, V);
    k = u256_from_be(V);
    if (!u256_is_zero(&k) && u256_cmp(&k, &FN) < 0) break;
    memcpy(buf, V, 32); buf[32] = 0;
    hmac_sha256(K, 32, buf, 33, K);
    hmac_sha256(K, 32, V, 32, V);
  }
  sc zero;
  memset(&zero, 0, sizeof zero);
  ge dummy = {GX, GY, 0};
  gej Rj; ge R;
  ecmult(&Rj, &k, &dummy, &zero);
  gej_to_ge(&R, &Rj);
  sc r = R.x;
  int y_odd = (int)(R.y.v[0] & 1);
  while (u256_cmp(&r, &FN) >= 0) u256_sub(&r, &r, &FN);
  sc kinv, s, t;
  sc_inv(&kinv, &k);
  sc_mul(&t, &r, &d);
  sc_add(&t, &t, &z);
  sc_mul(&s, &kinv, &t);
  if (u256_cmp(&s, &FN_HALF) > 0) { sc_neg(&s, &s); y_odd ^= 1; }
  u256_to_be(&r, sig);
  u256_to_be(&s, sig + 32);
  sig[64] = (u8)(27 + y_odd);
}

/* ========================= Vote encoding + hashing ============================= */
static size_t put_varint(u8* o, u64 v) {
  size_t n = 0;
  do { u8 b = v & 0x7F; v >>= 7; o[n++] = v ? (b | 0x80) : b; } while (v);
  return n;
}
static size_t varint_len(u64 v) { size_t n = 1; while (v >= 0x80) { v >>= 7; ++n; } return n; }

typedef struct {
  u32 vote_id, proposal_id;
  u64 timestamp;
  u8 vote;
  const u8* f[HLC_NFIELDS];
  u32 flen[HLC_NFIELDS];
} vview;

static void vote_view(const hlc_votes* vs, u64 i, vview* v) {
  v->vote_id = vs->vote_id[i];
  v->proposal_id = vs->proposal_id[i];
  v->timestamp = vs->timestamp[i];
  v->vote = vs->vote[i] ? 1 : 0;
  for (int k = 0; k < HLC_NFIELDS; ++k) {
    v->flen[k] = vs->field_len[i * HLC_NFIELDS + k];
    v->f[k] = vs->bytes + vs->field_off[i * HLC_NFIELDS + k];
  }
}

/* prost encode_to_vec of Vote with signature cleared (utils.rs:150-152) */
static size_t encoded_len(const vview* v) {
  size_t n = 0;
  if (v->vote_id) n += 2 + varint_len(v->vote_id);
  if (v->flen[HLC_F_OWNER]) n += 2 + varint_len(v->flen[HLC_F_OWNER]) + v->flen[HLC_F_OWNER];
  if (v->proposal_id) n += 2 + varint_len(v->proposal_id);
  if (v->timestamp) n += 2 + varint_len(v->timestamp);
  if (v->vote) n += 3;
  for (int k = HLC_F_PARENT; k <= HLC_F_VOTE_HASH; ++k)
    if (v->flen[k]) n += 2 + varint_len(v->flen[k]) + v->flen[k];
  return n;
}

static size_t encode_vote(const vview* v, u8* o) {
  size_t n = 0;
  if (v->vote_id) { o[n++] = 0xA0; o[n++] = 0x01; n += put_varint(o + n, v->vote_id); }
  if (v->flen[HLC_F_OWNER]) {
    o[n++] = 0xAA; o[n++] = 0x01; n += put_varint(o + n, v->flen[HLC_F_OWNER]);
    memcpy(o + n, v->f[HLC_F_OWNER], v->flen[HLC_F_OWNER]); n += v->flen[HLC_F_OWNER];
  }
  if (v->proposal_id) { o[n++] = 0xB0; o[n++] = 0x01; n += put_varint(o + n, v->proposal_id); }
  if (v->timestamp) { o[n++] = 0xB8; o[n++] = 0x01; n += put_varint(o + n, v->timestamp); }
  if (v->vote) { o[n++] = 0xC0; o[n++] = 0x01; o[n++] = 0x01; }
  static const u8 keys[HLC_NFIELDS] = {0xAA, 0xCA, 0xD2, 0xDA, 0xE2};
  for (int k = HLC_F_PARENT; k <= HLC_F_VOTE_HASH; ++k) {
    if (!v->flen[k]) continue;
    o[n++] = keys[k]; o[n++] = 0x01; n += put_varint(o + n, v->flen[k]);
    memcpy(o + n, v->f[k], v->flen[k]); n += v->flen[k];
  }
  return n;
}

static void vote_hash(const vview* v, u8 out[32]) {
  sha256_ctx c;
  u8 b[8];
  sha256_init(&c);
  for (int i = 0; i < 4; ++i) b[i] = (u8)(v->vote_id >> (8 * i));
  sha256_update(&c, b, 4);
  sha256_update(&c, v->f[HLC_F_OWNER], v->flen[HLC_F_OWNER]);
  for (int i = 0; i < 4; ++i) b[i] = (u8)(v->proposal_id >> (8 * i));
  sha256_update(&c, b, 4);
  for (int i = 0; i < 8; ++i) b[i] = (u8)(v->timestamp >> (8 * i));
  sha256_update(&c, b, 8);
  b[0] = v->vote;
  sha256_update(&c, b, 1);
  sha256_update(&c, v->f[HLC_F_PARENT], v->flen[HLC_F_PARENT]);
  sha256_update(&c, v->f[HLC_F_RECEIVED], v->flen[HLC_F_RECEIVED]);
  sha256_final(&c, out);
}

static void eip191_hash(const u8* payload, size_t n, u8 out[32]) {
  static const char pre[] = "\x19" "Ethereum Signed Message:\n";
  char digits[24];
  int nd = 0;
  size_t t = n;
  do { digits[nd++] = (char)('0' + t % 10); t /= 10; } while (t);
  char lenstr[24];
  for (int i = 0; i < nd; ++i) lenstr[i] = digits[nd - 1 - i];
  keccak_ctx k;
  keccak_init(&k);
  keccak_update(&k, (const u8*)pre, 26);
  keccak_update(&k, (const u8*)lenstr, (size_t)nd);
  keccak_update(&k, payload, n);
  keccak_final(&k, out);
}

void hlco_eip191_hash(const u8* payload, size_t n, u8 out[32]) { eip191_hash(payload, n, out); }

int hlco_compute_vote_hashes(const hlc_votes* vs, u8* out) {
  for (u64 i = 0; i < vs->n; ++i) {
    vview v;
    vote_view(vs, i, &v);
    vote_hash(&v, out + 32 * i);
  }
  return 0;
}

size_t hlco_encode_vote(const hlc_votes* vs, u64 i, u8* out) {
  vview v;
  vote_view(vs, i, &v);
  return encode_vote(&v, out);
}

/* EthereumConsensusSigner::verify (ethereum.rs:66-97) -> HLC_VERIFY_* / 1+HLC_SCHEME_* */
static int eth_verify(const u8* id, u32 idlen, const u8* payload, size_t plen, const u8* sig,
                      u32 siglen, u8 addr[20], int flags) {
  if (siglen != 65) return 1 + HLC_SCHEME_SIG_LEN;
  if (idlen != 20) return 1 + HLC_SCHEME_ID_LEN;
  u8 h[32];
  eip191_hash(payload, plen, h);
  int sub = hlco_ecrecover(h, sig, addr, flags);
  if (sub) return 1 + sub;
  return memcmp(addr, id, 20) == 0 ? HLC_VERIFY_TRUE : HLC_VERIFY_FALSE;
}

int hlco_verify_batch(u64 n, const u8* bytes, const u64* id_off, const u32* id_len,
                      const u64* p_off, const u32* p_len, const u64* s_off, const u32* s_len,
                      u8* out_status, u8* out_addr, int flags) {
  for (u64 i = 0; i < n; ++i) {
    u8 addr[20] = {0};
    out_status[i] = (u8)eth_verify(bytes + id_off[i], id_len[i], bytes + p_off[i], p_len[i],
                                   bytes + s_off[i], s_len[i], addr, flags);
    if (out_addr) memcpy(out_addr + 20 * i, addr, 20);
  }
  return 0;
}

/* StubSigner::verify (tests/custom_scheme_tests.rs:61-73): Err(Verify) unless the identity is 8 bytes,
 * else Ok(signature == SHA256(identity || payload)) -> HLC_VERIFY_* / 1 + HLC_SCHEME_PLUGIN */
static int stub_verify(const u8* id, u32 idlen, const u8* payload, size_t plen, const u8* sig, u32 siglen) {
  if (idlen != 8) return 1 + HLC_SCHEME_PLUGIN;
  sha256_ctx c;
  u8 h[32];
  sha256_init(&c);
  sha256_update(&c, id, idlen);
  sha256_update(&c, payload, plen);
  sha256_final(&c, h);
  return (siglen == 32 && memcmp(sig, h, 32) == 0) ? HLC_VERIFY_TRUE : HLC_VERIFY_FALSE;
}

int hlco_stub_sign(const u8* id, u32 idlen, const u8* payload, size_t plen, u8 out[32]) {
  sha256_ctx c;
  sha256_init(&c);
  sha256_update(&c, id, idlen);
  sha256_update(&c, payload, plen);
  sha256_final(&c, out);
  return 0;
}

/* validate_vote (utils.rs:127-171) preceded by the proposal_id check (utils.rs:113-115) */
static void validate_one(const hlc_votes* vs, u64 i, const hlc_proposal* p, u64 now, u8* st,
                         u8* reason, u8 addr[20], int flags) {
  vview v;
  vote_view(vs, i, &v);
  *reason = 0;
  memset(addr, 0, 20);
  if (v.proposal_id != p->proposal_id) { *st = HLC_VOTE_PROPOSAL_ID_MISMATCH; return; }
  if (!v.flen[HLC_F_OWNER]) { *st = HLC_EMPTY_VOTE_OWNER; return; }
  if (!v.flen[HLC_F_VOTE_HASH]) { *st = HLC_EMPTY_VOTE_HASH; return; }
  if (!v.flen[HLC_F_SIGNATURE]) { *st = HLC_EMPTY_SIGNATURE; return; }
  u8 h[32];
  vote_hash(&v, h);
  if (v.flen[HLC_F_VOTE_HASH] != 32 || memcmp(h, v.f[HLC_F_VOTE_HASH], 32) != 0) {
    *st = HLC_INVALID_VOTE_HASH; return;
  }
  size_t elen = encoded_len(&v);
  u8 stackbuf[512];
  u8* enc = elen <= sizeof stackbuf ? stackbuf : (u8*)malloc(elen);
  encode_vote(&v, enc);
  int vr = (flags & HLCO_STUB)
               ? stub_verify(v.f[HLC_F_OWNER], v.flen[HLC_F_OWNER], enc, elen, v.f[HLC_F_SIGNATURE],
                             v.flen[HLC_F_SIGNATURE])
               : eth_verify(v.f[HLC_F_OWNER], v.flen[HLC_F_OWNER], enc, elen, v.f[HLC_F_SIGNATURE],
                            v.flen[HLC_F_SIGNATURE], addr, flags);
  if (enc != stackbuf) free(enc);
  if (vr >= 2) { *st = HLC_SIGNATURE_SCHEME; *reason = (u8)(vr - 1); return; }
  if (vr == HLC_VERIFY_FALSE) { *st = HLC_INVALID_VOTE_SIGNATURE; return; }
  if (v.timestamp < p->timestamp) { *st = HLC_TIMESTAMP_OLDER_THAN_CREATION; return; }
  if (v.timestamp > p->expiration_timestamp || now > p->expiration_timestamp) {
    *st = HLC_VOTE_EXPIRED; return;
  }
  *st = HLC_OK;
}

/* --- chain check (utils.rs:175-215): open-addressing map vote_hash -> last index --- */
static u64 fnv(const u8* p, u32 n) {
  u64 h = 1469598103934665603ULL;
  for (u32 i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
  return h;
}

static int bytes_eq(const u8* a, u32 al, const u8* b, u32 bl) {
  return al == bl && (al == 0 || memcmp(a, b, al) == 0);
}

/* returns status, *bad = index within proposal */
static int chain_check(const hlc_votes* vs, const hlc_proposal* p, u32* bad) {
  u32 n = p->vote_count;
  if (n <= 1) return HLC_OK;
  u64 cap = 16;
  while (cap < 2ull * n) cap <<= 1;
  int64_t* tab = (int64_t*)malloc(cap * sizeof(int64_t));
  for (u64 i = 0; i < cap; ++i) tab[i] = -1;
#define FOFF(j, k) (vs->field_off[(p->vote_begin + (j)) * HLC_NFIELDS + (k)])
#define FLEN(j, k) (vs->field_len[(p->vote_begin + (j)) * HLC_NFIELDS + (k)])
#define FPTR(j, k) (vs->bytes + FOFF(j, k))
  for (u32 j = 0; j < n; ++j) {
    u64 h = fnv(FPTR(j, HLC_F_VOTE_HASH), FLEN(j, HLC_F_VOTE_HASH)) & (cap - 1);
    for (;;) {
      if (tab[h] < 0) { tab[h] = j; break; }
      u32 o = (u32)tab[h];
      if (bytes_eq(FPTR(o, HLC_F_VOTE_HASH), FLEN(o, HLC_F_VOTE_HASH), FPTR(j, HLC_F_VOTE_HASH),
                   FLEN(j, HLC_F_VOTE_HASH))) { tab[h] = j; break; } /* last wins */
      h = (h + 1) & (cap - 1);
    }
  }
  int st = HLC_OK;
  for (u32 j = 0; j < n && st == HLC_OK; ++j) {
    u64 vj = p->vote_begin + j;
    if (j > 0 && FLEN(j, HLC_F_RECEIVED)) {
      if (!bytes_eq(FPTR(j, HLC_F_RECEIVED), FLEN(j, HLC_F_RECEIVED), FPTR(j - 1, HLC_F_VOTE_HASH),
                    FLEN(j - 1, HLC_F_VOTE_HASH)) ||
          vs->timestamp[vj - 1] > vs->timestamp[vj]) {
        st = HLC_RECEIVED_HASH_MISMATCH; *bad = j; break;
      }
    }
    if (FLEN(j, HLC_F_PARENT)) {
      u64 h = fnv(FPTR(j, HLC_F_PARENT), FLEN(j, HLC_F_PARENT)) & (cap - 1);
      int64_t hit = -1;
      for (;;) {
        if (tab[h] < 0) break;
        u32 o = (u32)tab[h];
        if (bytes_eq(FPTR(o, HLC_F_VOTE_HASH), FLEN(o, HLC_F_VOTE_HASH), FPTR(j, HLC_F_PARENT),
                     FLEN(j, HLC_F_PARENT))) { hit = o; break; }
        h = (h + 1) & (cap - 1);
      }
      if (hit < 0 ||
          !(bytes_eq(FPTR(hit, HLC_F_OWNER), FLEN(hit, HLC_F_OWNER), FPTR(j, HLC_F_OWNER),
                     FLEN(j, HLC_F_OWNER)) &&
            vs->timestamp[p->vote_begin + hit] <= vs->timestamp[vj] && (u32)hit < j)) {
        st = HLC_PARENT_HASH_MISMATCH; *bad = j; break;
      }
    }
  }
  free(tab);
  return st;
}

static int dup_check(const hlc_votes* vs, const hlc_proposal* p, u32* bad) {
  u32 n = p->vote_count;
  u64 cap = 16;
  while (cap < 2ull * n) cap <<= 1;
  int64_t* tab = (int64_t*)malloc(cap * sizeof(int64_t));
  for (u64 i = 0; i < cap; ++i) tab[i] = -1;
  int st = HLC_OK;
  for (u32 j = 0; j < n && st == HLC_OK; ++j) {
    u64 h = fnv(FPTR(j, HLC_F_OWNER), FLEN(j, HLC_F_OWNER)) & (cap - 1);
    for (;;) {
      if (tab[h] < 0) { tab[h] = j; break; }
      u32 o = (u32)tab[h];
      if (bytes_eq(FPTR(o, HLC_F_OWNER), FLEN(o, HLC_F_OWNER), FPTR(j, HLC_F_OWNER), FLEN(j, HLC_F_OWNER))) {
        st = HLC_DUPLICATE_VOTE; *bad = j; break;
      }
      h = (h + 1) & (cap - 1);
    }
  }
  free(tab);
  return st;
#undef FOFF
#undef FLEN
#undef FPTR
}

/* utils.rs:307-313 (u32 wrap of 2n as in a release build; f64 -> u32 saturating cast) */
static u32 threshold_value(u32 n, double t) {
  if (fabs(t - 2.0 / 3.0) < 2.220446049250313e-16) {
    u32 two_n = 2u * n;
    return two_n / 3u + (two_n % 3u != 0);
  }
  double x = ceil((double)n * t);
  if (!(x > 0)) return 0;
  if (x >= 4294967295.0) return 0xFFFFFFFFu;
  return (u32)x;
}

/* utils.rs:227-286 -> -1 None, 0 false, 1 true */
int hlco_consensus_result(u32 total, u32 yes, u32 n, double t, int liveness, int is_timeout) {
  u32 no = total > yes ? total - yes : 0;
  u32 silent = n > total ? n - total : 0;
  if (n <= 2) {
    if (total < n) return -1;
    return yes == n;
  }
  u32 req = threshold_value(n, t);
  u32 eff = is_timeout ? n : total;
  if (eff < req) return -1;
  u32 yw = yes + (liveness ? silent : 0), nw = no + (liveness ? 0 : silent);
  if (yw >= req && yw > nw) return 1;
  if (nw >= req && nw > yw) return 0;
  if (total == n && yw == nw) return liveness ? 1 : 0;
  return -1;
}

u32 hlco_threshold_value(u32 n, double t) { return threshold_value(n, t); }

/* ConsensusConfig::max_round_limit (session.rs:120-128) */
static u32 max_round_limit(int gossipsub, u32 max_rounds, double t, u32 n) {
  if (gossipsub) return max_rounds;
  return max_rounds ? max_rounds : threshold_value(n, t);
}

/* check_round_limit (session.rs:306-344) for any round and a usize vote_count: 1 = within the
 * limit, 0 = MaxRoundsExceeded.  vote_count is compared with n (u32) before any u32 arithmetic
 * (session.rs:308); the P2P projection saturates in u32 (session.rs:330-331). */
int hlco_check_round_limit(int gossipsub, u32 max_rounds, double t, u32 n, u32 round, u64 vote_count) {
  if (vote_count > (u64)n) return 0;
  u32 projected;
  if (gossipsub) {
    projected = (round == 2 || (round == 1 && vote_count > 0)) ? 2u : round;
  } else {
    const u32 cur = round ? round - 1u : 0u;
    const u64 sum = (u64)cur + (u32)vote_count;
    projected = sum > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)sum;
  }
  return projected <= max_round_limit(gossipsub, max_rounds, t, n);
}

/* update_round (session.rs:351-366): Gossipsub 1 -> 2 on any votes; P2P saturating_add */
u32 hlco_update_round(int gossipsub, u32 round, u64 vote_count) {
  if (gossipsub) return (round == 1 && vote_count > 0) ? 2u : round;
  const u64 sum = (u64)round + (u32)vote_count;
  return sum > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)sum;
}

static void finish_proposal(const hlc_votes* vs, const hlc_proposal* p, u64 now, const u8* vst,
                            const u8* vreason, hlc_result* res) {
  memset(res, 0, sizeof *res);
  res->bad_index = 0xFFFFFFFFu;
  if (now >= p->expiration_timestamp) { res->status = HLC_PROPOSAL_EXPIRED; return; }
  for (u32 j = 0; j < p->vote_count; ++j) {
    u64 i = p->vote_begin + j;
    if (vst[i] != HLC_OK) {
      res->status = vst[i]; res->scheme_reason = vreason[i]; res->bad_index = j; return;
    }
  }
  u32 bad = 0;
  int st = chain_check(vs, p, &bad);
  if (st) { res->status = (u8)st; res->bad_index = bad; return; }
  u32 n = p->vote_count;
  if (n == 0) return; /* StillActive (session.rs:266-268) */
  st = dup_check(vs, p, &bad);
  if (st) { res->status = (u8)st; res->bad_index = bad; return; }
  u32 ev = p->expected_voters_count;
  if (n > ev) { res->status = HLC_MAX_ROUNDS_EXCEEDED; return; }
  /* check_round_limit at round 1 (session.rs:289, 306-344) */
  if (!hlco_check_round_limit(p->use_gossipsub_rounds, p->max_rounds, p->consensus_threshold, ev, 1u, n)) {
    res->status = HLC_MAX_ROUNDS_EXCEEDED;
    return;
  }
  u32 yes = 0;
  for (u32 j = 0; j < n; ++j) yes += vs->vote[p->vote_begin + j] ? 1 : 0;
  res->yes = yes;
  res->total = n;
  int r = hlco_consensus_result(n, yes, ev, p->consensus_threshold, p->liveness_criteria_yes, 0);
  res->transition = r < 0 ? HLC_STILL_ACTIVE : (r ? HLC_REACHED_YES : HLC_REACHED_NO);
}

typedef struct {
  const hlc_votes* vs;
  const hlc_proposal* ps;
  u64 p0, p1, now;
  u8 *vst, *vreason, *rec;
  hlc_result* res;
  int flags;
} job;

static void* worker(void* arg) {
  job* jb = (job*)arg;
  for (u64 pi = jb->p0; pi < jb->p1; ++pi) {
    const hlc_proposal* p = &jb->ps[pi];
    for (u32 j = 0; j < p->vote_count; ++j) {
      u64 i = p->vote_begin + j;
      u8 addr[20];
      validate_one(jb->vs, i, p, jb->now, &jb->vst[i], &jb->vreason[i], addr, jb->flags);
      if (jb->rec) memcpy(jb->rec + 20 * i, addr, 20);
    }
    if (jb->res) finish_proposal(jb->vs, p, jb->now, jb->vst, jb->vreason, &jb->res[pi]);
  }
  return NULL;
}

/* Same contract as hlc_validate_proposals (include/hlc.h); vote_status / vote_reason are
 * required here.  threads <= 1 runs inline.  flags: HLCO_REVERIFY (also run k256's verify_prehash),
 * HLCO_GLV (the k256-class recovery instead of the non-GLV checker). */
int hlco_validate_proposals(const hlc_votes* vs, const hlc_proposal* ps, u64 np, u64 now,
                            hlc_result* res, u8* vst, u8* vreason, u8* rec, int threads,
                            int flags) {
  if (threads < 1) threads = 1;
  if ((u64)threads > np) threads = np ? (int)np : 1;
  /* balance by vote count */
  u64 total = 0;
  for (u64 i = 0; i < np; ++i) total += ps[i].vote_count;
  job* jobs = (job*)calloc((size_t)threads, sizeof(job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  u64 pi = 0;
  for (int t = 0; t < threads; ++t) {
    u64 target = total * (u64)(t + 1) / (u64)threads, acc = 0;
    jobs[t] = (job){vs, ps, pi, pi, now, vst, vreason, rec, res, flags};
    if (t == threads - 1) jobs[t].p1 = np;
    else {
      u64 done = 0;
      for (u64 k = 0; k < pi; ++k) done += ps[k].vote_count;
      acc = done;
      u64 e = pi;
      while (e < np && acc < target) acc += ps[e++].vote_count;
      jobs[t].p1 = e;
    }
    pi = jobs[t].p1;
  }
  if (threads == 1) worker(&jobs[0]);
  else {
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  }
  free(jobs);
  free(th);
  return 0;
}

/* validate_vote-only timing loop for the CPU baseline: votes [v0, v1) against proposal p */
typedef struct { const hlc_votes* vs; const hlc_proposal* ps; u64 p0, p1, now; int flags; u64 ok; } vjob;
static void* vworker(void* arg) {
  vjob* jb = (vjob*)arg;
  for (u64 pi = jb->p0; pi < jb->p1; ++pi) {
    const hlc_proposal* p = &jb->ps[pi];
    for (u32 j = 0; j < p->vote_count; ++j) {
      u8 st, rs, addr[20];
      validate_one(jb->vs, p->vote_begin + j, p, jb->now, &st, &rs, addr, jb->flags);
      jb->ok += st == HLC_OK;
    }
  }
  return NULL;
}

/* Times nothing itself: runs validate_vote over every vote of proposals [0, np) on
 * `threads` threads (static split by proposal) and returns how many were OK. */
u64 hlco_validate_votes_only(const hlc_votes* vs, const hlc_proposal* ps, u64 np, u64 now,
                             int threads, int flags) {
  if (threads < 1) threads = 1;
  vjob* jobs = (vjob*)calloc((size_t)threads, sizeof(vjob));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t)
    jobs[t] = (vjob){vs, ps, np * (u64)t / (u64)threads, np * (u64)(t + 1) / (u64)threads, now, flags, 0};
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, vworker, &jobs[t]);
  u64 ok = 0;
  for (int t = 0; t < threads; ++t) { pthread_join(th[t], NULL); ok += jobs[t].ok; }
  free(jobs);
  free(th);
  return ok;
}

/* batch signing helpers for fixture generation (multithreaded) */
typedef struct { u64 i0, i1; const u8* priv; const u8* prehash; u8* sig; u8* addr; } sjob;
static void* sworker(void* arg) {
  sjob* j = (sjob*)arg;
  for (u64 i = j->i0; i < j->i1; ++i) {
    if (j->sig) hlco_sign_prehash(j->priv + 32 * i, j->prehash + 32 * i, j->sig + 65 * i);
    if (j->addr) hlco_address(j->priv + 32 * i, j->addr + 20 * i);
  }
  return NULL;
}

int hlco_sign_batch(u64 n, const u8* priv, const u8* prehash, u8* sig, u8* addr, int threads) {
  if (threads < 1) threads = 1;
  sjob* jobs = (sjob*)calloc((size_t)threads, sizeof(sjob));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t)
    jobs[t] = (sjob){n * (u64)t / (u64)threads, n * (u64)(t + 1) / (u64)threads, priv, prehash, sig, addr};
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, sworker, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
  return 0;
}
