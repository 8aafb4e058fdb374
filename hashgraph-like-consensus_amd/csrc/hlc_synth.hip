// hlc_synth.hip -- the synthetic signed-vote workload of SURVEY.md §8d, generated on the device.
//
// Same bytes as the Python generator (python/hashgraph_like_consensus/synth.py, whose docstring
// freezes the spec; tests/test_gpu_synth.py pins the two against each other): each vote is built
// like the reference's `build_vote` (/root/reference/src/utils.rs:55-98) -- received_hash = the
// previous vote's hash, empty parent, vote hash = compute_vote_hash (utils.rs:37-47) -- and signed
// like `EthereumConsensusSigner::sign` (signing/ethereum.rs:58-64).  Config 4 (100M votes over 8
// GPUs) needs 12.5M signed votes per rank; generating them on the GPU takes seconds instead of the
// minutes a host generator needs, and nothing crosses PCIe.
//
// Three kernels (a vote's hash needs the previous vote's hash, so the chain is one lane per
// proposal; keys/addresses and signatures are one lane per vote):
//   k_synth_keys  : priv = SHA256(seed_le8 || i_le8) mod n, owner = address(priv G), ids, choice,
//                   timestamp, field offsets/lengths, owner bytes into the arena;
//   k_synth_chain : sequential vote hashes per proposal -> vote_hash and received_hash bytes;
//   k_synth_sign  : prost encoding -> EIP-191 keccak -> RFC 6979 signature into the arena.
#include "hlc_kernels.h"
#include "hlc_recover.hpp"
#include "hlc_sign.hpp"

namespace hlc {

namespace {

constexpr uint64_t T0 = 1760000000ull;
constexpr uint64_t EXPIRATION = T0 + 3600;
constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ull;
constexpr uint64_t C2 = 0xD1B54A32D192ED03ull;
constexpr int TPB = 128;

// per-vote arena record: owner(20) | received(0/32) | vote_hash(32) | signature(65)
__host__ __device__ inline uint64_t rec_base(uint64_t p, uint64_t j, uint64_t V) {
  return p * (149ull * V - 32ull) + (j ? 149ull * j - 32ull : 0ull);
}

HLC_DEV uint64_t mix(uint64_t seed, uint64_t domain, uint64_t idx) {
  uint64_t z = seed * GOLDEN + domain * C2 + idx;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// SHA256(seed_le8 || gidx_le8) mod n, 0 -> 1 (synth.privkeys)
HLC_DEV void synth_priv(fe& d, uint64_t seed, uint64_t gidx) {
  uint32_t w[16];
  w[0] = bswap32((uint32_t)seed);
  w[1] = bswap32((uint32_t)(seed >> 32));
  w[2] = bswap32((uint32_t)gidx);
  w[3] = bswap32((uint32_t)(gidx >> 32));
  w[4] = 0x80000000u;
#pragma unroll
  for (int k = 5; k < 15; ++k) w[k] = 0;
  w[15] = 128;
  uint32_t h[8];
  sha256_init(h);
  sha256_compress(h, w);
  fe x;
#pragma unroll
  for (int k = 0; k < 8; ++k) x.v[7 - k] = h[k];
  sc_reduce(d, x);
  if (fe_is_zero(d)) fe_set(d, 1);
}

struct SynthArgs {
  uint64_t seed, start, P;
  uint32_t V;
  uint8_t* bytes;
  uint32_t* vote_id;
  uint32_t* proposal_id;
  uint64_t* timestamp;
  uint8_t* vote;
  uint64_t* field_off;
  uint32_t* field_len;
  uint8_t* priv_out;
};

__global__ void k_synth_keys(SynthArgs a, const uint32_t* fb) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.P * a.V) return;
  const uint64_t p = i / a.V, j = i % a.V;
  const uint64_t gidx = a.start * a.V + i;
  fe d;
  synth_priv(d, a.seed, gidx);
  if (a.priv_out) fe_store_be(a.priv_out + 32 * i, d);
  gej q;
  fixed_base_mul(q, d, fb);
  fe x, y;
  gej_to_affine(x, y, q);
  uint32_t addr[5];
  pubkey_address(x, y, addr);
  const uint64_t base = rec_base(p, j, a.V);
  const uint32_t rl = j ? 32u : 0u;
  uint8_t* o = a.bytes + base;
#pragma unroll
  for (int k = 0; k < 20; ++k) o[k] = (uint8_t)(addr[k >> 2] >> (8 * (k & 3)));
  a.vote_id[i] = (uint32_t)mix(a.seed, 2, gidx) | 0x80000000u;
  a.proposal_id[i] = (uint32_t)mix(a.seed, 1, a.start + p) | 0x80000000u;
  a.timestamp[i] = T0 + 1 + j / 1024;
  a.vote[i] = (uint8_t)(mix(a.seed, 3, gidx) & 1u);
  uint64_t* fo = a.field_off + i * HLC_NFIELDS;
  uint32_t* fl = a.field_len + i * HLC_NFIELDS;
  fo[HLC_F_OWNER] = base;
  fo[HLC_F_PARENT] = base + 20;
  fo[HLC_F_RECEIVED] = base + 20;
  fo[HLC_F_VOTE_HASH] = base + 20 + rl;
  fo[HLC_F_SIGNATURE] = base + 20 + rl + 32;
  fl[HLC_F_OWNER] = 20;
  fl[HLC_F_PARENT] = 0;
  fl[HLC_F_RECEIVED] = rl;
  fl[HLC_F_VOTE_HASH] = 32;
  fl[HLC_F_SIGNATURE] = 65;
}

// compute_vote_hash (utils.rs:37-47) along each proposal's chain.  The chain is sequential (each
// vote's received_hash is the previous vote's hash), so one lane walks a proposal; the SHA-256
// message words are assembled in registers from the fixed layout vote_id(4 LE) | owner(20) |
// proposal_id(4 LE) | timestamp(8 LE) | vote(1) | received(0/32), no byte buffer.
__global__ void k_synth_chain(SynthArgs a, hlc_proposal* props, uint32_t expected, int gossipsub) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.P) return;
  uint32_t prev[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // previous vote hash, big-endian words
  for (uint64_t j = 0; j < a.V; ++j) {
    const uint64_t i = p * a.V + j;
    const uint64_t base = rec_base(p, j, a.V);
    uint8_t* o = a.bytes + base;
    const uint32_t vid = a.vote_id[i], pid = a.proposal_id[i];
    const uint64_t ts = a.timestamp[i];
    const uint32_t vote = a.vote[i];
    uint32_t w[16];
    w[0] = bswap32(vid);
#pragma unroll
    for (int k = 0; k < 5; ++k)
      w[1 + k] = (uint32_t)o[4 * k] << 24 | (uint32_t)o[4 * k + 1] << 16 | (uint32_t)o[4 * k + 2] << 8 |
                 (uint32_t)o[4 * k + 3];
    w[6] = bswap32(pid);
    w[7] = bswap32((uint32_t)ts);
    w[8] = bswap32((uint32_t)(ts >> 32));
    uint32_t h[8];
    sha256_init(h);
    if (j == 0) {  // 37 bytes: one block
      w[9] = vote << 24 | 0x00800000u;
#pragma unroll
      for (int k = 10; k < 15; ++k) w[k] = 0;
      w[15] = 37u * 8u;
      sha256_compress(h, w);
    } else {       // 69 bytes: received = prev (bytes 37..68), two blocks
      w[9] = vote << 24 | prev[0] >> 8;
#pragma unroll
      for (int k = 1; k < 7; ++k) w[9 + k] = prev[k - 1] << 24 | prev[k] >> 8;
      uint32_t w2[16];
      w2[0] = prev[6] << 24 | prev[7] >> 8;
      w2[1] = prev[7] << 24 | 0x00800000u;
#pragma unroll
      for (int k = 2; k < 15; ++k) w2[k] = 0;
      w2[15] = 69u * 8u;
      sha256_compress(h, w);
      sha256_compress(h, w2);
#pragma unroll
      for (int k = 0; k < 32; ++k) o[20 + k] = (uint8_t)(prev[k >> 2] >> (24 - 8 * (k & 3)));  // received_hash
    }
    uint8_t* vh = o + 20 + (j ? 32 : 0);
#pragma unroll
    for (int k = 0; k < 32; ++k) vh[k] = (uint8_t)(h[k >> 2] >> (24 - 8 * (k & 3)));
#pragma unroll
    for (int k = 0; k < 8; ++k) prev[k] = h[k];
  }
  hlc_proposal d;
  d.vote_begin = p * a.V;
  d.vote_count = a.V;
  d.proposal_id = (uint32_t)mix(a.seed, 1, a.start + p) | 0x80000000u;
  d.timestamp = T0;
  d.expiration_timestamp = EXPIRATION;
  d.expected_voters_count = expected;
  d.max_rounds = gossipsub ? 2u : 0u;
  d.consensus_threshold = 2.0 / 3.0;
  d.use_gossipsub_rounds = gossipsub ? 1 : 0;
  d.liveness_criteria_yes = 1;
  for (int k = 0; k < 6; ++k) d._pad[k] = 0;
  props[p] = d;
}

struct ByteSink {
  uint8_t* o;
  int pos;
  HLC_DEV void put(uint8_t b) { o[pos++] = b; }
  HLC_DEV void varint(uint64_t x) {
    do {
      const uint8_t b = x & 0x7F;
      x >>= 7;
      put(x ? (uint8_t)(b | 0x80) : b);
    } while (x);
  }
  HLC_DEV void bytes(const uint8_t* s, int n) {
    for (int k = 0; k < n; ++k) put(s[k]);
  }
};

HLC_DEV int varint_bytes(uint64_t x) {
  int n = 1;
  while (x >= 0x80) {
    x >>= 7;
    ++n;
  }
  return n;
}

// EthereumConsensusSigner::sign over the prost encoding of the vote with the signature cleared
// (utils.rs:94: the signature is empty when build_vote signs)
__global__ void k_synth_sign(SynthArgs a, const uint32_t* fb) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.P * a.V) return;
  const uint64_t p = i / a.V, j = i % a.V;
  const uint64_t base = rec_base(p, j, a.V);
  const uint8_t* o = a.bytes + base;
  const uint32_t vid = a.vote_id[i], pid = a.proposal_id[i];
  const uint64_t ts = a.timestamp[i];
  const uint8_t ch = a.vote[i];
  const int rl = j ? 32 : 0;
  const int enc = 2 + varint_bytes(vid) + 23 + 2 + varint_bytes(pid) + 2 + varint_bytes(ts) + (ch ? 3 : 0) +
                  (rl ? 35 : 0) + 35;
  uint8_t m[272];
  ByteSink s{m, 0};
  const char prefix[] = "\x19" "Ethereum Signed Message:\n";
  for (int k = 0; k < 26; ++k) s.put((uint8_t)prefix[k]);
  if (enc >= 100) s.put((uint8_t)('0' + enc / 100));
  if (enc >= 10) s.put((uint8_t)('0' + (enc / 10) % 10));
  s.put((uint8_t)('0' + enc % 10));
  s.put(0xA0); s.put(0x01); s.varint(vid);
  s.put(0xAA); s.put(0x01); s.put(20); s.bytes(o, 20);
  s.put(0xB0); s.put(0x01); s.varint(pid);
  s.put(0xB8); s.put(0x01); s.varint(ts);
  if (ch) { s.put(0xC0); s.put(0x01); s.put(0x01); }
  if (rl) { s.put(0xD2); s.put(0x01); s.put(32); s.bytes(o + 20, 32); }
  s.put(0xDA); s.put(0x01); s.put(32); s.bytes(o + 20 + rl, 32);
  const int len = s.pos;
  const int blocks = len / 136 + 1;
  s.put(0x01);
  while (s.pos < 136 * blocks) s.put(0);
  m[136 * blocks - 1] |= 0x80;
  uint64_t st[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) st[k] = 0;
  for (int b = 0; b < blocks; ++b) {
    for (int k = 0; k < 17; ++k) {
      uint64_t w = 0;
      for (int q = 0; q < 8; ++q) w |= (uint64_t)m[136 * b + 8 * k + q] << (8 * q);
      st[k] ^= w;
    }
    keccak_f1600(st);
  }
  uint32_t z[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    z[2 * q] = (uint32_t)st[q];
    z[2 * q + 1] = (uint32_t)(st[q] >> 32);
  }
  fe d;
  synth_priv(d, a.seed, a.start * a.V + i);
  sign_prehash(d, z, fb, a.bytes + base + 20 + rl + 32);
}

// ---- SURVEY.md §8d config 5 on the device: 1/3 Byzantine votes with outcomes known by construction ----
// Applied in place to a batch made by k_synth_* with the same (seed, start, P, V); product code only,
// so bench.py can time the Byzantine mix without the oracle.  Mutation choice (all from `mix`, so
// the host can recompute it: hashgraph_like_consensus/byzantine.py):
//   proposal mode  = mix(seed, 9, global proposal) & 7: 0-3 any kind, 4-5 chain kinds + high-s,
//                    6 high-s and a duplicate last voter, 7 high-s only;
//   vote mutated   iff mix(seed, 7, gidx) % 3 == 0, kind from mix(seed, 8, gidx).
// Kinds (include/hlc.h HLC_BYZ_*) and the validate_vote outcome each is built to have:
//   WRONG_KEY    re-signed by another key                     InvalidVoteSignature
//   FLIP_S       lowest bit of s flipped                       InvalidVoteSignature
//   BAD_V        v = 29                                        SignatureScheme (parity)
//   HIGH_S       s -> n - s, v -> 55 - v                       Ok (alloy normalises it back)
//   NO_POINT     r = 2^255 + 0x303c (x^3 + 7 a non-residue)    SignatureScheme (no point)
//   INFINITY     signed with key 0: s = z / k, R = k G         SignatureScheme (Q = infinity)
//   TAMPER_HASH  one vote_hash bit flipped                     InvalidVoteHash
//   SIG_LEN      signature length 64                           SignatureScheme (length)
//   EMPTY_*      owner / vote_hash / signature length 0        EmptyVoteOwner / Hash / Signature
//   WRONG_PID    proposal_id ^= 1                              VoteProposalIdMismatch
//   TS_OLD       timestamp T0 - 10, re-hashed + re-signed      TimestampOlderThanCreationTime
//   BAD_RECEIVED received_hash byte flipped, re-hashed+signed  Ok per vote; chain: ReceivedHashMismatch
//   TS_REGRESS   timestamp below the predecessor's, re-signed  Ok per vote; chain: ReceivedHashMismatch
//   PARENT_OTHER parent_hash = the previous (other) voter's    Ok per vote; chain: ParentHashMismatch
//   DUPLICATE    owner = the previous vote's owner, re-signed  Ok per vote; DuplicateVote
//                by that owner's key
// A re-hashed vote keeps its successor's received_hash stale (the Byzantine voter re-signs only its
// own vote), so the successor's chain link breaks too.
constexpr uint64_t BYZ_WRONG_SALT = 0x57524F4E474B4559ull;
constexpr uint64_t KEY_NONE = 0, KEY_OWN = 1, KEY_WRONG = 2, KEY_ZERO = 3;

HLC_DEV uint32_t fl_get(const SynthArgs& a, uint64_t i, int f) { return a.field_len[i * HLC_NFIELDS + f]; }
HLC_DEV const uint8_t* fp_get(const SynthArgs& a, uint64_t i, int f) {
  return a.bytes + a.field_off[i * HLC_NFIELDS + f];
}

// compute_vote_hash (utils.rs:37-47) of vote i as it now stands (any field lengths <= 32 / 20 B)
HLC_DEV void byz_rehash(const SynthArgs& a, uint64_t i) {
  uint8_t m[128];
  int L = 0;
  auto le = [&](uint64_t x, int nb) {
    for (int k = 0; k < nb; ++k) m[L++] = (uint8_t)(x >> (8 * k));
  };
  auto cp = [&](int f) {
    const uint32_t n = fl_get(a, i, f);
    const uint8_t* q = fp_get(a, i, f);
    for (uint32_t k = 0; k < n; ++k) m[L++] = q[k];
  };
  le(a.vote_id[i], 4);
  cp(HLC_F_OWNER);
  le(a.proposal_id[i], 4);
  le(a.timestamp[i], 8);
  m[L++] = a.vote[i] ? 1 : 0;
  cp(HLC_F_PARENT);
  cp(HLC_F_RECEIVED);
  const int total = L, nb = (total + 9 + 63) / 64;
  m[L++] = 0x80;
  while (L < 64 * nb - 8) m[L++] = 0;
  for (int k = 7; k >= 0; --k) m[L++] = (uint8_t)(((uint64_t)total * 8) >> (8 * k));
  uint32_t h[8];
  sha256_init(h);
  for (int b = 0; b < nb; ++b) {
    uint32_t w[16];
    for (int k = 0; k < 16; ++k) w[k] = load_be32(m + 64 * b + 4 * k);
    sha256_compress(h, w);
  }
  uint8_t* o = a.bytes + a.field_off[i * HLC_NFIELDS + HLC_F_VOTE_HASH];
  for (int k = 0; k < 32; ++k) o[k] = (uint8_t)(h[k >> 2] >> (24 - 8 * (k & 3)));
}

// EIP-191 keccak of the prost encoding of vote i with the signature cleared (utils.rs:150-152)
HLC_DEV void byz_prehash(const SynthArgs& a, uint64_t i, uint32_t z[8]) {
  uint8_t pay[160];
  ByteSink s{pay, 0};
  auto bytes_field = [&](uint8_t key, int f) {
    const uint32_t n = fl_get(a, i, f);
    if (!n) return;
    s.put(key); s.put(0x01); s.put((uint8_t)n); s.bytes(fp_get(a, i, f), (int)n);
  };
  if (a.vote_id[i]) { s.put(0xA0); s.put(0x01); s.varint(a.vote_id[i]); }
  bytes_field(0xAA, HLC_F_OWNER);
  if (a.proposal_id[i]) { s.put(0xB0); s.put(0x01); s.varint(a.proposal_id[i]); }
  if (a.timestamp[i]) { s.put(0xB8); s.put(0x01); s.varint(a.timestamp[i]); }
  if (a.vote[i]) { s.put(0xC0); s.put(0x01); s.put(0x01); }
  bytes_field(0xCA, HLC_F_PARENT);
  bytes_field(0xD2, HLC_F_RECEIVED);
  bytes_field(0xDA, HLC_F_VOTE_HASH);
  const int enc = s.pos;
  uint8_t m[272];
  ByteSink e{m, 0};
  const char prefix[] = "\x19" "Ethereum Signed Message:\n";
  for (int k = 0; k < 26; ++k) e.put((uint8_t)prefix[k]);
  if (enc >= 100) e.put((uint8_t)('0' + enc / 100));
  if (enc >= 10) e.put((uint8_t)('0' + (enc / 10) % 10));
  e.put((uint8_t)('0' + enc % 10));
  e.bytes(pay, enc);
  const int len = e.pos, blocks = len / 136 + 1;
  e.put(0x01);
  while (e.pos < 136 * blocks) e.put(0);
  m[136 * blocks - 1] |= 0x80;
  uint64_t st[25];
  for (int k = 0; k < 25; ++k) st[k] = 0;
  for (int b = 0; b < blocks; ++b) {
    for (int k = 0; k < 17; ++k) {
      uint64_t w = 0;
      for (int q = 0; q < 8; ++q) w |= (uint64_t)m[136 * b + 8 * k + q] << (8 * q);
      st[k] ^= w;
    }
    keccak_f1600(st);
  }
  for (int q = 0; q < 4; ++q) {
    z[2 * q] = (uint32_t)st[q];
    z[2 * q + 1] = (uint32_t)(st[q] >> 32);
  }
}

HLC_DEV int byz_pick(uint64_t seed, uint64_t gidx, int mode, uint64_t j) {
  if (mix(seed, 7, gidx) % 3 != 0) return HLC_BYZ_NONE;
  const uint64_t h = mix(seed, 8, gidx);
  if (mode <= 3) {
    int k = 1 + (int)(h % 17);
    if (j == 0 && k >= HLC_BYZ_BAD_RECEIVED) k = 1 + (int)(h % 13);  // chain kinds need a predecessor
    return k;
  }
  if (mode <= 5) {
    const int ch[5] = {HLC_BYZ_HIGH_S, HLC_BYZ_BAD_RECEIVED, HLC_BYZ_TS_REGRESS, HLC_BYZ_PARENT_OTHER,
                       HLC_BYZ_DUPLICATE};
    const int k = ch[h % 5];
    return j == 0 ? HLC_BYZ_HIGH_S : k;
  }
  return HLC_BYZ_HIGH_S;
}

// one lane per proposal, votes in order (a vote's parent / owner may point at its predecessor's
// bytes, re-hashed first); signing is deferred to k_byz_sign through key[].
__global__ void k_byz_mutate(SynthArgs a, uint8_t* kind_out, uint64_t* key) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.P) return;
  const int mode = (int)(mix(a.seed, 9, a.start + p) & 7u);
  uint64_t prev_src = 0;  // key index of the predecessor's owner
  for (uint64_t j = 0; j < a.V; ++j) {
    const uint64_t i = p * a.V + j, gidx = a.start * a.V + i;
    int kind = byz_pick(a.seed, gidx, mode, j);
    if (mode == 6 && j + 1 == a.V && j > 0) kind = HLC_BYZ_DUPLICATE;
    uint64_t* fo = a.field_off + i * HLC_NFIELDS;
    uint32_t* fl = a.field_len + i * HLC_NFIELDS;
    uint8_t* sig = a.bytes + fo[HLC_F_SIGNATURE];
    uint64_t k = KEY_NONE << 62, src = gidx;
    bool rehash = false;
    switch (kind) {
      case HLC_BYZ_WRONG_KEY: k = (KEY_WRONG << 62) | gidx; break;
      case HLC_BYZ_FLIP_S: sig[63] ^= 1u; break;
      case HLC_BYZ_BAD_V: sig[64] = 29; break;
      case HLC_BYZ_HIGH_S: {
        fe sv, n;
        fe_load_be(sv, sig + 32);
        for (int q = 0; q < 8; ++q) n.v[q] = n_limb(q);
        uint32_t bw = 0;
        for (int q = 0; q < 8; ++q) sv.v[q] = sub_cc(n.v[q], sv.v[q], bw);
        fe_store_be(sig + 32, sv);
        sig[64] = (uint8_t)(55 - sig[64]);
        break;
      }
      case HLC_BYZ_NO_POINT:
        for (int q = 0; q < 32; ++q) sig[q] = 0;
        sig[0] = 0x80; sig[30] = 0x30; sig[31] = 0x3C;
        break;
      case HLC_BYZ_INFINITY: k = KEY_ZERO << 62; break;
      case HLC_BYZ_TAMPER_HASH: a.bytes[fo[HLC_F_VOTE_HASH] + 5] ^= 0x10; break;
      case HLC_BYZ_SIG_LEN: fl[HLC_F_SIGNATURE] = 64; break;
      case HLC_BYZ_EMPTY_OWNER: fl[HLC_F_OWNER] = 0; break;
      case HLC_BYZ_EMPTY_HASH: fl[HLC_F_VOTE_HASH] = 0; break;
      case HLC_BYZ_EMPTY_SIG: fl[HLC_F_SIGNATURE] = 0; break;
      case HLC_BYZ_WRONG_PID: a.proposal_id[i] ^= 1u; break;
      case HLC_BYZ_TS_OLD: a.timestamp[i] = T0 - 10; rehash = true; break;
      case HLC_BYZ_BAD_RECEIVED: a.bytes[fo[HLC_F_RECEIVED]] ^= 0xFFu; rehash = true; break;
      case HLC_BYZ_TS_REGRESS: a.timestamp[i] = T0 + (j - 1) / 1024; rehash = true; break;  // predecessor's ts - 1
      case HLC_BYZ_PARENT_OTHER:
        fo[HLC_F_PARENT] = a.field_off[(i - 1) * HLC_NFIELDS + HLC_F_VOTE_HASH];
        fl[HLC_F_PARENT] = 32;
        rehash = true;
        break;
      case HLC_BYZ_DUPLICATE:
        fo[HLC_F_OWNER] = a.field_off[(i - 1) * HLC_NFIELDS + HLC_F_OWNER];
        src = prev_src;
        rehash = true;
        break;
      default: break;
    }
    if (rehash) {
      byz_rehash(a, i);
      k = (KEY_OWN << 62) | src;
    }
    kind_out[i] = (uint8_t)kind;
    key[i] = k;
    prev_src = src;
  }
}

// one lane per vote: the deferred signatures (the prost payload of the vote as mutated)
__global__ void k_byz_sign(SynthArgs a, const uint64_t* key, const uint32_t* fb) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.P * a.V) return;
  const uint64_t k = key[i], how = k >> 62, idx = k & ((1ull << 62) - 1);
  if (how == KEY_NONE) return;
  uint32_t z[8];
  byz_prehash(a, i, z);
  fe d;
  if (how == KEY_OWN) synth_priv(d, a.seed, idx);
  else if (how == KEY_WRONG) synth_priv(d, a.seed ^ BYZ_WRONG_SALT, idx);
  else fe_set(d, 0);  // Q = infinity: s = z / k for R = k G
  sign_prehash(d, z, fb, a.bytes + a.field_off[i * HLC_NFIELDS + HLC_F_SIGNATURE]);
}

}  // namespace

uint64_t synth_arena_bytes(uint64_t P, uint64_t V) { return V ? rec_base(P, 0, V) : 0; }

void launch_synth(uint64_t seed, uint64_t start, uint64_t P, uint32_t V, uint32_t expected, int gossipsub,
                  const hlc_votes* out, hlc_proposal* props, uint8_t* priv_out, const uint32_t* fb, hipStream_t s) {
  SynthArgs a;
  a.seed = seed;
  a.start = start;
  a.P = P;
  a.V = V;
  a.bytes = const_cast<uint8_t*>(out->bytes);
  a.vote_id = const_cast<uint32_t*>(out->vote_id);
  a.proposal_id = const_cast<uint32_t*>(out->proposal_id);
  a.timestamp = const_cast<uint64_t*>(out->timestamp);
  a.vote = const_cast<uint8_t*>(out->vote);
  a.field_off = const_cast<uint64_t*>(out->field_off);
  a.field_len = const_cast<uint32_t*>(out->field_len);
  a.priv_out = priv_out;
  const uint64_t n = P * V;
  if (!n) return;
  hipLaunchKernelGGL(k_synth_keys, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, s, a, fb);
  hipLaunchKernelGGL(k_synth_chain, dim3((unsigned)((P + 63) / 64)), dim3(64), 0, s, a, props, expected, gossipsub);
  hipLaunchKernelGGL(k_synth_sign, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, s, a, fb);
}

void launch_synth_byzantine(uint64_t seed, uint64_t start, uint64_t P, uint32_t V, const hlc_votes* v,
                            uint8_t* kind_out, uint64_t* key_work, const uint32_t* fb, hipStream_t s) {
  SynthArgs a;
  a.seed = seed;
  a.start = start;
  a.P = P;
  a.V = V;
  a.bytes = const_cast<uint8_t*>(v->bytes);
  a.vote_id = const_cast<uint32_t*>(v->vote_id);
  a.proposal_id = const_cast<uint32_t*>(v->proposal_id);
  a.timestamp = const_cast<uint64_t*>(v->timestamp);
  a.vote = const_cast<uint8_t*>(v->vote);
  a.field_off = const_cast<uint64_t*>(v->field_off);
  a.field_len = const_cast<uint32_t*>(v->field_len);
  a.priv_out = nullptr;
  const uint64_t n = P * V;
  if (!n) return;
  hipLaunchKernelGGL(k_byz_mutate, dim3((unsigned)((P + 63) / 64)), dim3(64), 0, s, a, kind_out, key_work);
  hipLaunchKernelGGL(k_byz_sign, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, s, a, key_work, fb);
}

}  // namespace hlc
