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

}  // namespace hlc
