// hlc_prehash.hip -- byte-level stages of the validate-many path (one lane per vote):
//   * proposal assignment, message sizing, message materialisation (SHA-256 input of
//     compute_vote_hash, utils.rs:37-47; EIP-191 framing of the prost-encoded Vote with the
//     signature cleared, utils.rs:150-152 + alloy eip191_hash_message),
//   * SHA-256 / keccak-256 over the materialised, padded messages,
//   * per-vote status assembly (validate_proposal loop body, utils.rs:112-117, 127-171),
//   * chain-link (utils.rs:175-215) and duplicate-owner (session.rs:270-275) hash tables,
//   * per-proposal reduction and the initialize_with_votes tail (session.rs:253-298).
// All integer/byte work: HBM/L2-bound and tiny next to recovery.
#include <hipcub/hipcub.hpp>

#include "hlc_hash.hpp"
#include "hlc_tally.hpp"
#include "hlc_kernels.h"

namespace hlc {

namespace {

constexpr int TPB = 256;
constexpr uint32_t SMALL_CAP = 512;  // proposals up to this many votes: k_chain_small
constexpr int SMALL_TPB = 64;        // one wave per proposal

__device__ __forceinline__ uint32_t flen(const hlc_votes& v, uint64_t i, int f) {
  return v.field_len[i * HLC_NFIELDS + f];
}
__device__ __forceinline__ const uint8_t* fptr(const hlc_votes& v, uint64_t i, int f) {
  return v.bytes + v.field_off[i * HLC_NFIELDS + f];
}

__device__ __forceinline__ uint32_t varint_len(uint64_t x) {
  uint32_t n = 1;
  while (x >= 0x80) {
    x >>= 7;
    ++n;
  }
  return n;
}
__device__ __forceinline__ uint32_t dec_digits(uint64_t x) {
  uint32_t n = 1;
  while (x >= 10) {
    x /= 10;
    ++n;
  }
  return n;
}

// prost encoded length of Vote with signature cleared (consensus.proto:19-29)
__device__ uint64_t vote_enc_len(const hlc_votes& v, uint64_t i) {
  uint64_t n = 0;
  uint32_t id = v.vote_id[i], pid = v.proposal_id[i];
  uint64_t ts = v.timestamp[i];
  if (id) n += 2 + varint_len(id);
  uint32_t lo = flen(v, i, HLC_F_OWNER);
  if (lo) n += 2 + varint_len(lo) + lo;
  if (pid) n += 2 + varint_len(pid);
  if (ts) n += 2 + varint_len(ts);
  if (v.vote[i]) n += 3;
  for (int f = HLC_F_PARENT; f <= HLC_F_VOTE_HASH; ++f) {
    uint32_t l = flen(v, i, f);
    if (l) n += 2 + varint_len(l) + l;
  }
  return n;
}

// Block (p, y) of a (proposals x G) grid writes every G-th span of proposal p's vote range: G > 1
// when the batch's proposals are large on average (config 3: one proposal of 1M votes).
// A large proposal also raises FLAG_LARGE_PARENTS when any of its votes has a parent_hash: only
// then does k_tables build the vote_hash table the parent lookups need.
__global__ void k_assign_props(const hlc_proposal* props, const uint32_t* field_len, uint32_t* vote_prop,
                               uint32_t* flags) {
  const uint32_t p = blockIdx.x;
  const hlc_proposal d = props[p];
  const bool large = d.vote_count > SMALL_CAP;
  if (threadIdx.x == 0 && blockIdx.y == 0 && large) atomicOr(flags, FLAG_LARGE_PROPOSAL);
  const uint64_t step = (uint64_t)blockDim.x * gridDim.y;
  bool parent = false;
  for (uint64_t j = (uint64_t)blockIdx.y * blockDim.x + threadIdx.x; j < d.vote_count; j += step) {
    vote_prop[d.vote_begin + j] = p;
    if (large) parent |= field_len[(d.vote_begin + j) * HLC_NFIELDS + HLC_F_PARENT] != 0;
  }
  if (large && __ballot(parent) && (threadIdx.x & 63) == 0) atomicOr(flags, FLAG_LARGE_PARENTS);
}

__global__ void k_msg_sizes(hlc_votes v, uint64_t n, const uint64_t* pay_off, const uint32_t* pay_len,
                            int mode, uint64_t* sha_sz, uint64_t* kec_sz) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t klen;
  if (mode == MSG_VOTE) {
    uint64_t sl = 17ull + flen(v, i, HLC_F_OWNER) + flen(v, i, HLC_F_PARENT) + flen(v, i, HLC_F_RECEIVED);
    sha_sz[i] = ((sl + 8) / 64 + 1) * 64;
    uint64_t el = vote_enc_len(v, i);
    klen = 26 + dec_digits(el) + el;
  } else {
    uint64_t pl = pay_len[i];
    klen = 26 + dec_digits(pl) + pl;
    if (sha_sz) sha_sz[i] = 0;
  }
  kec_sz[i] = (klen / 136 + 1) * 136;
}

struct Cursor {
  uint8_t* o;
  uint64_t pos;
  __device__ void put(uint8_t b) { o[pos++] = b; }
  __device__ void put_varint(uint64_t x) {
    do {
      uint8_t b = x & 0x7F;
      x >>= 7;
      put(x ? (b | 0x80) : b);
    } while (x);
  }
  __device__ void put_bytes(const uint8_t* p, uint32_t n) {
    for (uint32_t k = 0; k < n; ++k) put(p[k]);
  }
  __device__ void put_le(uint64_t x, int nbytes) {
    for (int k = 0; k < nbytes; ++k) put((uint8_t)(x >> (8 * k)));
  }
  __device__ void put_decimal(uint64_t x) {
    uint8_t d[20];
    int nd = 0;
    do {
      d[nd++] = (uint8_t)('0' + x % 10);
      x /= 10;
    } while (x);
    while (nd) put(d[--nd]);
  }
};

__device__ void put_eip191_prefix(Cursor& c) {
  const char pre[] = "\x19" "Ethereum Signed Message:\n";
  for (int k = 0; k < 26; ++k) c.put((uint8_t)pre[k]);
}

__global__ void k_build_msgs(hlc_votes v, uint64_t n, const uint8_t* bytes, const uint64_t* pay_off,
                             const uint32_t* pay_len, int mode, const uint64_t* sha_off,
                             const uint64_t* sha_sz, uint8_t* sha_buf, const uint64_t* kec_off,
                             const uint64_t* kec_sz, uint8_t* kec_buf) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (mode == MSG_VOTE) {
    // SHA-256 input of compute_vote_hash (utils.rs:39-45) + FIPS 180-4 padding
    Cursor c{sha_buf + sha_off[i], 0};
    c.put_le(v.vote_id[i], 4);
    c.put_bytes(fptr(v, i, HLC_F_OWNER), flen(v, i, HLC_F_OWNER));
    c.put_le(v.proposal_id[i], 4);
    c.put_le(v.timestamp[i], 8);
    c.put(v.vote[i] ? 1 : 0);
    c.put_bytes(fptr(v, i, HLC_F_PARENT), flen(v, i, HLC_F_PARENT));
    c.put_bytes(fptr(v, i, HLC_F_RECEIVED), flen(v, i, HLC_F_RECEIVED));
    uint64_t len = c.pos, sz = sha_sz[i];
    c.put(0x80);
    while (c.pos < sz - 8) c.put(0);
    uint64_t bits = len * 8;
    for (int k = 7; k >= 0; --k) c.put((uint8_t)(bits >> (8 * k)));
  }
  // EIP-191 message: "\x19Ethereum Signed Message:\n" || decimal(len) || payload, keccak pad
  Cursor c{kec_buf + kec_off[i], 0};
  put_eip191_prefix(c);
  if (mode == MSG_VOTE) {
    c.put_decimal(vote_enc_len(v, i));
    uint32_t id = v.vote_id[i], pid = v.proposal_id[i];
    uint64_t ts = v.timestamp[i];
    if (id) { c.put(0xA0); c.put(0x01); c.put_varint(id); }
    uint32_t lo = flen(v, i, HLC_F_OWNER);
    if (lo) { c.put(0xAA); c.put(0x01); c.put_varint(lo); c.put_bytes(fptr(v, i, HLC_F_OWNER), lo); }
    if (pid) { c.put(0xB0); c.put(0x01); c.put_varint(pid); }
    if (ts) { c.put(0xB8); c.put(0x01); c.put_varint(ts); }
    if (v.vote[i]) { c.put(0xC0); c.put(0x01); c.put(0x01); }
    const uint8_t keys[3] = {0xCA, 0xD2, 0xDA};
    for (int f = HLC_F_PARENT; f <= HLC_F_VOTE_HASH; ++f) {
      uint32_t l = flen(v, i, f);
      if (l) { c.put(keys[f - HLC_F_PARENT]); c.put(0x01); c.put_varint(l); c.put_bytes(fptr(v, i, f), l); }
    }
  } else {
    uint32_t pl = pay_len[i];
    c.put_decimal(pl);
    c.put_bytes(bytes + pay_off[i], pl);
  }
  uint64_t sz = kec_sz[i];
  c.put(0x01);
  while (c.pos < sz) c.put(0);
  c.o[sz - 1] |= 0x80;
}

__global__ void k_sha_blocks(uint64_t n, const uint64_t* off, const uint64_t* sz, const uint8_t* buf,
                             uint32_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h[8];
  sha256_init(h);
  const uint32_t* m = reinterpret_cast<const uint32_t*>(buf + off[i]);
  uint64_t nb = sz[i] / 64;
  for (uint64_t b = 0; b < nb; ++b) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = bswap32(m[b * 16 + k]);
    sha256_compress(h, w);
  }
  // digest as memory-order words (bytes 4k..4k+3 little-endian in word k)
#pragma unroll
  for (int k = 0; k < 8; ++k) out[i * 8 + k] = bswap32(h[k]);
}

__global__ void k_keccak_blocks(uint64_t n, const uint64_t* off, const uint64_t* sz, const uint8_t* buf,
                                uint32_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t st[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) st[k] = 0;
  const uint64_t* m = reinterpret_cast<const uint64_t*>(buf + off[i]);
  uint64_t nb = sz[i] / 136;
  for (uint64_t b = 0; b < nb; ++b) {
#pragma unroll
    for (int k = 0; k < 17; ++k) st[k] ^= m[b * 17 + k];
    keccak_f1600(st);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    out[i * 8 + 2 * k] = (uint32_t)st[k];
    out[i * 8 + 2 * k + 1] = (uint32_t)(st[k] >> 32);
  }
}

// validate_vote checks that precede Signer::verify (utils.rs:133-148) and the scheme's
// length checks (signing/ethereum.rs:71-82), after the proposal_id match (utils.rs:113-115).
__global__ void k_pre_status(hlc_votes v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                             const uint32_t* sha, uint8_t* pre, uint8_t* pre_reason) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (pre[i] != PRE_GENERAL) return;  // decided by k_prehash_fused
  uint8_t st, rs = 0;
  uint32_t p = vote_prop ? vote_prop[i] : 0;
  if (vote_prop && p == NO_PROP) {
    st = PRE_SKIP;
  } else if (v.proposal_id[i] != props[p].proposal_id) {
    st = HLC_VOTE_PROPOSAL_ID_MISMATCH;
  } else if (flen(v, i, HLC_F_OWNER) == 0) {
    st = HLC_EMPTY_VOTE_OWNER;
  } else if (flen(v, i, HLC_F_VOTE_HASH) == 0) {
    st = HLC_EMPTY_VOTE_HASH;
  } else if (flen(v, i, HLC_F_SIGNATURE) == 0) {
    st = HLC_EMPTY_SIGNATURE;
  } else {
    bool eq = flen(v, i, HLC_F_VOTE_HASH) == 32;
    if (eq) {
      const uint8_t* h = fptr(v, i, HLC_F_VOTE_HASH);
      for (int k = 0; k < 32 && eq; ++k) eq = h[k] == (uint8_t)(sha[i * 8 + k / 4] >> (8 * (k & 3)));
    }
    if (!eq) {
      st = HLC_INVALID_VOTE_HASH;
    } else if (flen(v, i, HLC_F_SIGNATURE) != 65) {
      st = HLC_SIGNATURE_SCHEME;
      rs = HLC_SCHEME_SIG_LEN;
    } else if (flen(v, i, HLC_F_OWNER) != 20) {
      st = HLC_SIGNATURE_SCHEME;
      rs = HLC_SCHEME_ID_LEN;
    } else {
      st = PRE_PENDING;
    }
  }
  pre[i] = st;
  pre_reason[i] = rs;
}

// validate_vote tail (utils.rs:154-168): scheme result, then timestamps
// With red != nullptr also the first failing vote per proposal (red[4p + 0], the local index): the
// chain / duplicate / tally kernels then need no vote statuses and run beside the recovery.
__global__ void k_vote_status(VoteStatusArgs a, uint64_t n, const uint8_t* pre, const uint8_t* verify) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t st = pre[i];
  vote_status_one(a, i, st, st == PRE_PENDING ? verify[i] : 0);
}

// ---------------- chain / duplicate tables ----------------
// The N-byte field at any byte address as N/4 little-endian words: 4-byte-aligned dword loads
// (only dwords that hold a byte of the field, so nothing past the field's last dword is read)
// joined by funnel shifts -- N/4 + 1 loads instead of N byte loads.
template <int N>
__device__ __forceinline__ void load_words(const uint8_t* p, uint32_t w[N / 4]) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t sh = (uint32_t)(a & 3u) * 8u;
  uint32_t r[N / 4 + 1];
#pragma unroll
  for (int k = 0; k < N / 4; ++k) r[k] = b[k];
  r[N / 4] = sh ? b[N / 4] : 0u;
#pragma unroll
  for (int k = 0; k < N / 4; ++k) w[k] = __builtin_amdgcn_alignbit(r[k + 1], r[k], sh);
}

__device__ __forceinline__ uint32_t key_fin(uint32_t h) {
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

template <int N>
__device__ __forceinline__ uint32_t key_hash_w(uint32_t p, const uint32_t w[N / 4]) {
  uint32_t h = 2166136261u ^ (p * 0x9E3779B1u) ^ (uint32_t)N;
#pragma unroll
  for (int k = 0; k < N / 4; ++k) h = __builtin_amdgcn_alignbit(h, h, 19) ^ (w[k] * 16777619u);
  return key_fin(h);
}

// hash of (proposal, field bytes): word-wise for the canonical lengths (address 20, hash 32), byte-
// wise otherwise.  A key's length picks the form, so equal keys always hash alike.
__device__ __forceinline__ uint32_t key_hash(uint32_t p, const uint8_t* b, uint32_t len) {
  if (len == 32) {
    uint32_t w[8];
    load_words<32>(b, w);
    return key_hash_w<32>(p, w);
  }
  if (len == 20) {
    uint32_t w[5];
    load_words<20>(b, w);
    return key_hash_w<20>(p, w);
  }
  uint32_t h = 2166136261u ^ (p * 0x9E3779B1u);
  for (uint32_t k = 0; k < len; ++k) h = (h ^ b[k]) * 16777619u;
  return key_fin(h);
}

template <int N>
__device__ __forceinline__ bool words_eq(const uint8_t* a, const uint8_t* b) {
  uint32_t x[N / 4], y[N / 4], d = 0;
  load_words<N>(a, x);
  load_words<N>(b, y);
#pragma unroll
  for (int k = 0; k < N / 4; ++k) d |= x[k] ^ y[k];
  return d == 0;
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
  if (al != bl) return false;
  if (al == 32) return words_eq<32>(a, b);
  if (al == 20) return words_eq<20>(a, b);
  for (uint32_t k = 0; k < al; ++k)
    if (a[k] != b[k]) return false;
  return true;
}

// Returns EMPTY_SLOT when the key was new, else the slot's index before this insert's max / min.
template <bool LAST_WINS>
__device__ uint32_t table_insert(uint32_t* tab, uint32_t mask, const hlc_votes& v, const uint32_t* vote_prop,
                                 uint32_t idx, int f) {
  const uint32_t p = vote_prop[idx];
  const uint8_t* kb = fptr(v, idx, f);
  const uint32_t kl = flen(v, idx, f);
  uint32_t h = key_hash(p, kb, kl) & mask;
  for (;;) {
    uint32_t cur = atomicCAS(&tab[h], EMPTY_SLOT, idx);
    if (cur == EMPTY_SLOT) return EMPTY_SLOT;
    if (vote_prop[cur] == p && bytes_eq(fptr(v, cur, f), flen(v, cur, f), kb, kl))
      return LAST_WINS ? atomicMax(&tab[h], idx) : atomicMin(&tab[h], idx);
    h = (h + 1) & mask;
  }
}

__global__ void k_tables(hlc_votes v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                         uint32_t* chain_tab, uint32_t* dup_tab, uint32_t mask, uint32_t* red, const uint32_t* flags) {
  if (flags && !(*flags & FLAG_LARGE_PROPOSAL)) return;  // every proposal is small: k_chain_small
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t p = vote_prop[i];
  if (p == NO_PROP || props[p].vote_count <= SMALL_CAP) return;  // small: k_chain_small
  // HashMap<vote_hash, (owner, ts, idx)>: last index wins (utils.rs:180-183); built only when a
  // large proposal's vote has a parent_hash to look up
  if (props[p].vote_count > 1 && (!flags || (*flags & FLAG_LARGE_PARENTS)))
    (void)table_insert<true>(chain_tab, mask, v, vote_prop, (uint32_t)i, HLC_F_VOTE_HASH);
  // seen_owners HashSet (session.rs:270-275): the DuplicateVote error sits at the first index whose
  // owner appeared earlier = the smallest second-smallest index over the owner groups.  Every insert
  // into an existing group reports max(its index, the group's minimum so far); the smallest report
  // is that index (the group's second member reports it, or, when it came first, the group's first
  // member does as it lowers the minimum to itself).
  const uint32_t prev = table_insert<false>(dup_tab, mask, v, vote_prop, (uint32_t)i, HLC_F_OWNER);
  if (prev != EMPTY_SLOT) atomicMin(&red[4 * p + 2], max((uint32_t)i, prev) - (uint32_t)props[p].vote_begin);
}

__device__ __forceinline__ uint32_t table_find(const uint32_t* tab, uint32_t mask, const hlc_votes& v,
                                               const uint32_t* vote_prop, uint32_t p, const uint8_t* kb,
                                               uint32_t kl, int f) {
  uint32_t h = key_hash(p, kb, kl) & mask;
  for (;;) {
    uint32_t cur = tab[h];
    if (cur == EMPTY_SLOT) return EMPTY_SLOT;
    if (vote_prop[cur] == p && bytes_eq(fptr(v, cur, f), flen(v, cur, f), kb, kl)) return cur;
    h = (h + 1) & mask;
  }
}

// red layout per proposal: [0] first bad vote (local idx), [1] first chain error, [2] first dup, [3] yes
constexpr int CHAIN_TPB = 1024;
__global__ void __launch_bounds__(CHAIN_TPB) k_chain_check(hlc_votes v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                              const uint8_t* status, const uint32_t* chain_tab, const uint32_t* dup_tab,
                              uint32_t mask, uint8_t* chain_code, uint32_t* red, const uint32_t* flags) {
  if (flags && !(*flags & FLAG_LARGE_PROPOSAL)) return;  // every proposal is small: k_chain_small
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t p = i < n ? vote_prop[i] : NO_PROP;
  if (p != NO_PROP && props[p].vote_count <= SMALL_CAP) p = NO_PROP;  // small: k_chain_small
  bool yes = false;
  if (p != NO_PROP) {
    const hlc_proposal d = props[p];
    const uint32_t j = (uint32_t)(i - d.vote_begin);
    uint8_t cc = HLC_OK;
    if (d.vote_count > 1) {
      // received link (utils.rs:188-198)
      if (j > 0 && flen(v, i, HLC_F_RECEIVED) != 0) {
        if (!bytes_eq(fptr(v, i, HLC_F_RECEIVED), flen(v, i, HLC_F_RECEIVED), fptr(v, i - 1, HLC_F_VOTE_HASH),
                      flen(v, i - 1, HLC_F_VOTE_HASH)) ||
            v.timestamp[i - 1] > v.timestamp[i])
          cc = HLC_RECEIVED_HASH_MISMATCH;
      }
      // parent link (utils.rs:202-211)
      if (cc == HLC_OK && flen(v, i, HLC_F_PARENT) != 0) {
        uint32_t hit = table_find(chain_tab, mask, v, vote_prop, p, fptr(v, i, HLC_F_PARENT),
                                  flen(v, i, HLC_F_PARENT), HLC_F_VOTE_HASH);
        if (hit == EMPTY_SLOT ||
            !(bytes_eq(fptr(v, hit, HLC_F_OWNER), flen(v, hit, HLC_F_OWNER), fptr(v, i, HLC_F_OWNER),
                       flen(v, i, HLC_F_OWNER)) &&
              v.timestamp[hit] <= v.timestamp[i] && hit < i))
          cc = HLC_PARENT_HASH_MISMATCH;
      }
    }
    chain_code[i] = cc;
    if (cc != HLC_OK) atomicMin(&red[4 * p + 1], j);  // (first failing vote: k_vote_status)
    yes = v.vote[i] != 0;  // (duplicates were reported by k_tables)
  }
  // YES count of large proposals: one atomic per BLOCK when the whole block shares a proposal
  // (config 3: one proposal of 1M votes -- same-address atomics serialise at the L2, so one per
  // wave cost ~0.6 ms), one per wave when the wave does, else one per YES vote
  __shared__ uint32_t s_p[CHAIN_TPB / 64], s_y[CHAIN_TPB / 64];
  const uint32_t p0 = __builtin_amdgcn_readfirstlane(p);
  const bool wave_same = __ballot(p == p0) == ~0ull;
  const uint32_t wy = (uint32_t)__popcll(__ballot(yes));
  const unsigned wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_p[wv] = wave_same ? p0 : NO_PROP;
    s_y[wv] = wy;
  }
  __syncthreads();
  bool block_same = true;
#pragma unroll
  for (int k = 0; k < CHAIN_TPB / 64; ++k) block_same &= s_p[k] == s_p[0];
  if (block_same) {
    if (threadIdx.x == 0 && s_p[0] != NO_PROP) {
      uint32_t t = 0;
#pragma unroll
      for (int k = 0; k < CHAIN_TPB / 64; ++k) t += s_y[k];
      if (t) atomicAdd(&red[4 * s_p[0] + 3], t);
    }
  } else if (wave_same) {
    if (p0 != NO_PROP && (threadIdx.x & 63) == 0 && wy) atomicAdd(&red[4 * p0 + 3], wy);
  } else if (yes) {
    atomicAdd(&red[4 * p + 3], 1u);
  }
}

// ---------------- small proposals: one wave per proposal, no global tables ----------------
// validate_vote_chain (utils.rs:175-215), seen_owners (session.rs:270-275) and the YES count of a
// proposal with at most SMALL_CAP votes.  32-bit FNV keys of every owner and vote_hash sit in
// LDS; every key hit is confirmed byte for byte, so collisions cannot change an outcome.  The
// parent lookup scans from the last vote down (the reference's HashMap keeps the LAST index of a
// vote_hash), the duplicate scan from the first vote up (the first repeat is the error).
// cheap key of a byte field: length + first and last 4 bytes (all loads independent); a key
// match is always confirmed with bytes_eq_fast, so any key function is correct
__device__ __forceinline__ uint32_t key32(const uint8_t* b, uint32_t len) {
  uint32_t h = len * 0x9E3779B1u;
  if (len >= 4) {
    const uint32_t f = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    const uint8_t* e = b + len - 4;
    const uint32_t l = (uint32_t)e[0] | ((uint32_t)e[1] << 8) | ((uint32_t)e[2] << 16) | ((uint32_t)e[3] << 24);
    h ^= f ^ __builtin_amdgcn_alignbit(l, l, 13);
  } else {
    for (uint32_t k = 0; k < len; ++k) h ^= (uint32_t)b[k] << (8 * k);
  }
  return h;
}

template <int N>
__device__ __forceinline__ bool eq_n(const uint8_t* a, const uint8_t* b) {
  uint32_t d = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) d |= (uint32_t)(a[k] ^ b[k]);  // every load issued before any test
  return d == 0;
}

// bytes_eq with unrolled fast paths for the canonical field lengths (address 20, hash 32)
__device__ __forceinline__ bool bytes_eq_fast(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
  if (al != bl) return false;
  if (al == 32) return eq_n<32>(a, b);
  if (al == 20) return eq_n<20>(a, b);
  return bytes_eq(a, al, b, bl);
}

__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, off));
  return x;
}

__global__ void __launch_bounds__(SMALL_TPB) k_chain_small(hlc_votes v, const hlc_proposal* props,
                                                           uint8_t* chain_code, uint32_t* red) {
  __shared__ uint32_t h_own[SMALL_CAP], h_vh[SMALL_CAP];
  const uint32_t p = blockIdx.x;
  const hlc_proposal d = props[p];
  const uint32_t nv = d.vote_count;
  if (nv > SMALL_CAP) return;  // large proposals: global tables (k_tables / k_chain_check)
  const uint64_t b0 = d.vote_begin;
  for (uint32_t j = threadIdx.x; j < nv; j += SMALL_TPB) {
    const uint64_t i = b0 + j;
    h_own[j] = key32(fptr(v, i, HLC_F_OWNER), flen(v, i, HLC_F_OWNER));
    h_vh[j] = key32(fptr(v, i, HLC_F_VOTE_HASH), flen(v, i, HLC_F_VOTE_HASH));
  }
  __syncthreads();
  const uint32_t none = 0xFFFFFFFFu;
  uint32_t chain = none, dup = none, yes = 0;
  for (uint32_t j = threadIdx.x; j < nv; j += SMALL_TPB) {
    const uint64_t i = b0 + j;
    uint8_t cc = HLC_OK;
    if (nv > 1) {
      // received link (utils.rs:188-198)
      if (j > 0 && flen(v, i, HLC_F_RECEIVED) != 0) {
        if (!bytes_eq_fast(fptr(v, i, HLC_F_RECEIVED), flen(v, i, HLC_F_RECEIVED), fptr(v, i - 1, HLC_F_VOTE_HASH),
                      flen(v, i - 1, HLC_F_VOTE_HASH)) ||
            v.timestamp[i - 1] > v.timestamp[i])
          cc = HLC_RECEIVED_HASH_MISMATCH;
      }
      // parent link (utils.rs:202-211): the last vote whose vote_hash equals parent_hash
      const uint32_t lp = flen(v, i, HLC_F_PARENT);
      if (cc == HLC_OK && lp != 0) {
        const uint8_t* pb = fptr(v, i, HLC_F_PARENT);
        const uint32_t hp = key32(pb, lp);
        uint32_t hit = none;
        for (uint32_t k = nv; k-- > 0;) {
          if (h_vh[k] == hp &&
              bytes_eq_fast(fptr(v, b0 + k, HLC_F_VOTE_HASH), flen(v, b0 + k, HLC_F_VOTE_HASH), pb, lp)) {
            hit = k;
            break;
          }
        }
        if (hit == none ||
            !(bytes_eq_fast(fptr(v, b0 + hit, HLC_F_OWNER), flen(v, b0 + hit, HLC_F_OWNER), fptr(v, i, HLC_F_OWNER),
                       flen(v, i, HLC_F_OWNER)) &&
              v.timestamp[b0 + hit] <= v.timestamp[i] && hit < j))
          cc = HLC_PARENT_HASH_MISMATCH;
      }
    }
    chain_code[i] = cc;
    if (cc != HLC_OK) chain = min(chain, j);
    // seen_owners: an earlier vote with the same owner makes this one the duplicate
    const uint32_t ho = h_own[j];
    for (uint32_t k = 0; k < j; ++k) {
      if (h_own[k] == ho && bytes_eq_fast(fptr(v, b0 + k, HLC_F_OWNER), flen(v, b0 + k, HLC_F_OWNER),
                                     fptr(v, i, HLC_F_OWNER), flen(v, i, HLC_F_OWNER))) {
        dup = min(dup, j);
        break;
      }
    }
    yes += v.vote[i] != 0;
  }
  chain = wave_min(chain);
  dup = wave_min(dup);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) yes += (uint32_t)__shfl_xor((int)yes, off);
  if (threadIdx.x == 0) {
    red[4 * p + 1] = chain;  // (red[4p + 0], the first failing vote: k_vote_status)
    red[4 * p + 2] = dup;
    red[4 * p + 3] = yes;
  }
}

// from_proposal outcome (SURVEY.md Appendix B order)
__global__ void k_finalize(const hlc_proposal* props, uint64_t np, uint64_t now, const uint8_t* status,
                           const uint8_t* reason, const uint8_t* chain_code, const uint32_t* red,
                           hlc_result* out) {
  uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= np) return;
  const hlc_proposal d = props[p];
  hlc_result r;
  r.status = HLC_OK;
  r.transition = HLC_STILL_ACTIVE;
  r.scheme_reason = 0;
  r._pad = 0;
  r.bad_index = 0xFFFFFFFFu;
  r.yes = 0;
  r.total = 0;
  const uint32_t fb = red[4 * p], fc = red[4 * p + 1], fd = red[4 * p + 2];
  if (now >= d.expiration_timestamp) {  // utils.rs:110
    r.status = HLC_PROPOSAL_EXPIRED;
  } else if (fb != 0xFFFFFFFFu) {  // first failing vote, utils.rs:112-117
    r.status = status[d.vote_begin + fb];
    r.scheme_reason = reason[d.vote_begin + fb];
    r.bad_index = fb;
  } else if (fc != 0xFFFFFFFFu) {  // chain, utils.rs:118
    r.status = chain_code[d.vote_begin + fc];
    r.bad_index = fc;
  } else if (d.vote_count == 0) {  // session.rs:266-268
  } else if (fd != 0xFFFFFFFFu) {  // session.rs:270-275
    r.status = HLC_DUPLICATE_VOTE;
    r.bad_index = fd;
  } else if (d.vote_count > d.expected_voters_count) {  // session.rs:279-282
    r.status = HLC_MAX_ROUNDS_EXCEEDED;
  } else {
    // check_round_limit at round 1 (session.rs:306-344, 120-128)
    uint32_t projected = d.use_gossipsub_rounds ? 2u : d.vote_count;
    uint32_t limit = d.use_gossipsub_rounds
                         ? d.max_rounds
                         : (d.max_rounds ? d.max_rounds : threshold_value(d.expected_voters_count, d.consensus_threshold));
    if (projected > limit) {
      r.status = HLC_MAX_ROUNDS_EXCEEDED;
    } else {
      r.total = d.vote_count;
      r.yes = red[4 * p + 3];
      int c = consensus_result(r.total, r.yes, d.expected_voters_count, d.consensus_threshold,
                               d.liveness_criteria_yes != 0);  // session.rs:372-387
      r.transition = c < 0 ? HLC_STILL_ACTIVE : (c ? HLC_REACHED_YES : HLC_REACHED_NO);
    }
  }
  out[p] = r;
}

// handle_consensus_timeout (service.rs:323-373) per session
__global__ void k_timeout(uint64_t n, const hlc_session_tally* ss, uint8_t* out_state, uint8_t* out_status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const hlc_session_tally t = ss[i];
  uint8_t st = HLC_OK, state;
  if (t.state == HLC_SESSION_REACHED_NO || t.state == HLC_SESSION_REACHED_YES) {
    state = t.state;  // service.rs:331-333: an earlier result stands
  } else {
    const int r = consensus_result(t.total, t.yes, t.expected_voters_count, t.consensus_threshold,
                                   t.liveness_criteria_yes != 0, true);
    if (r < 0) {
      state = HLC_SESSION_FAILED;  // service.rs:344-346, 362-371
      st = HLC_INSUFFICIENT_VOTES_AT_TIMEOUT;
    } else {
      state = r ? HLC_SESSION_REACHED_YES : HLC_SESSION_REACHED_NO;
    }
  }
  out_state[i] = state;
  out_status[i] = st;
}

// ---------------- fused fast path: one kernel for the whole byte stage ----------------
// Per lane, the SHA-256 input of compute_vote_hash and then the EIP-191 message of the
// prost-encoded vote are materialised in a private LDS window (FBUF bytes, enough for every
// canonical vote and for fields up to ~80 B) and hashed straight from it: no global scratch, no
// size scan, no host round trip.  Votes whose messages do not fit are flagged PRE_GENERAL and
// handled by the general pipeline above (same semantics, global-memory staging).
constexpr int FUSED_TPB = 128;
constexpr int FBUF = 280;  // bytes per lane; 70 words: conflict-free ds_read_b32/b64 across lanes

struct LdsCursor {
  uint8_t* o;
  uint32_t pos;
  __device__ void put(uint8_t b) { o[pos++] = b; }
  __device__ void put_varint(uint64_t x) {
    do {
      uint8_t b = x & 0x7F;
      x >>= 7;
      put(x ? (b | 0x80) : b);
    } while (x);
  }
  __device__ void put_bytes(const uint8_t* p, uint32_t n) {
    for (uint32_t k = 0; k < n; ++k) put(p[k]);
  }
  __device__ void put_le(uint64_t x, int nbytes) {
    for (int k = 0; k < nbytes; ++k) put((uint8_t)(x >> (8 * k)));
  }
};

// ETH == false (a caller-side scheme's verdicts, hlc_validate_proposals_verdicts): the scheme's own checks
// (ethereum.rs:71-82) and the EIP-191 keccak are not this engine's: a vote whose hash matches is PRE_PENDING
template <bool ETH>
__global__ void __launch_bounds__(FUSED_TPB) k_prehash_fused(hlc_votes v, uint64_t n, const uint32_t* vote_prop,
                                                             const hlc_proposal* props, uint32_t* kec_dig,
                                                             uint8_t* pre, uint8_t* pre_reason, uint32_t* general) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[FUSED_TPB * FBUF];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* lb = lds + threadIdx.x * FBUF;
  const uint32_t p = vote_prop[i];
  uint8_t st = PRE_PENDING, rs = 0;
  const uint32_t lo = flen(v, i, HLC_F_OWNER), lp = flen(v, i, HLC_F_PARENT), lr = flen(v, i, HLC_F_RECEIVED);
  const uint32_t lh = flen(v, i, HLC_F_VOTE_HASH), ls = flen(v, i, HLC_F_SIGNATURE);
  if (p == NO_PROP) {
    st = PRE_SKIP;
  } else if (v.proposal_id[i] != props[p].proposal_id) {
    st = HLC_VOTE_PROPOSAL_ID_MISMATCH;
  } else if (lo == 0) {
    st = HLC_EMPTY_VOTE_OWNER;
  } else if (lh == 0) {
    st = HLC_EMPTY_VOTE_HASH;
  } else if (ls == 0) {
    st = HLC_EMPTY_SIGNATURE;
  } else {
    const uint64_t sha_len = 17ull + lo + lp + lr;
    const uint64_t sha_sz = ((sha_len + 8) / 64 + 1) * 64;
    const uint64_t el = vote_enc_len(v, i);
    const uint64_t kec_len = 26 + dec_digits(el) + el;
    const uint64_t kec_sz = (kec_len / 136 + 1) * 136;
    if (sha_sz > FBUF || (ETH && kec_sz > FBUF)) {
      pre[i] = PRE_GENERAL;
      pre_reason[i] = 0;
      atomicOr(general, FLAG_GENERAL_PATH);
      return;
    }
    // SHA-256 input (utils.rs:39-45) + padding, then compress from LDS
    LdsCursor c{lb, 0};
    c.put_le(v.vote_id[i], 4);
    c.put_bytes(fptr(v, i, HLC_F_OWNER), lo);
    c.put_le(v.proposal_id[i], 4);
    c.put_le(v.timestamp[i], 8);
    c.put(v.vote[i] ? 1 : 0);
    c.put_bytes(fptr(v, i, HLC_F_PARENT), lp);
    c.put_bytes(fptr(v, i, HLC_F_RECEIVED), lr);
    c.put(0x80);
    while (c.pos < sha_sz - 8) c.put(0);
    {
      const uint64_t bits = sha_len * 8;
      for (int k = 7; k >= 0; --k) c.put((uint8_t)(bits >> (8 * k)));
    }
    uint32_t h[8];
    sha256_init(h);
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lb);
    for (uint32_t b = 0; b < (uint32_t)(sha_sz / 64); ++b) {
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap32(lw[b * 16 + k]);
      sha256_compress(h, w);
    }
    bool eq = lh == 32;
    if (eq) {
      const uint8_t* hb = fptr(v, i, HLC_F_VOTE_HASH);
      uint32_t diff = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t want = (uint32_t)hb[4 * k] << 24 | (uint32_t)hb[4 * k + 1] << 16 |
                              (uint32_t)hb[4 * k + 2] << 8 | (uint32_t)hb[4 * k + 3];
        diff |= want ^ h[k];
      }
      eq = diff == 0;
    }
    if (!eq) {
      st = HLC_INVALID_VOTE_HASH;
    } else if (!ETH) {
      // the caller's scheme decides the signature step (st stays PRE_PENDING)
    } else if (ls != 65) {
      st = HLC_SIGNATURE_SCHEME;
      rs = HLC_SCHEME_SIG_LEN;
    } else if (lo != 20) {
      st = HLC_SIGNATURE_SCHEME;
      rs = HLC_SCHEME_ID_LEN;
    } else {
      // EIP-191 message of the prost encoding with the signature cleared (utils.rs:150-152)
      LdsCursor k{lb, 0};
      const char prefix[] = "\x19" "Ethereum Signed Message:\n";
      for (int q = 0; q < 26; ++q) k.put((uint8_t)prefix[q]);
      {
        uint8_t d[20];
        int nd = 0;
        uint64_t x = el;
        do {
          d[nd++] = (uint8_t)('0' + x % 10);
          x /= 10;
        } while (x);
        while (nd) k.put(d[--nd]);
      }
      const uint32_t id = v.vote_id[i], pid = v.proposal_id[i];
      const uint64_t ts = v.timestamp[i];
      if (id) { k.put(0xA0); k.put(0x01); k.put_varint(id); }
      k.put(0xAA); k.put(0x01); k.put_varint(lo); k.put_bytes(fptr(v, i, HLC_F_OWNER), lo);
      if (pid) { k.put(0xB0); k.put(0x01); k.put_varint(pid); }
      if (ts) { k.put(0xB8); k.put(0x01); k.put_varint(ts); }
      if (v.vote[i]) { k.put(0xC0); k.put(0x01); k.put(0x01); }
      if (lp) { k.put(0xCA); k.put(0x01); k.put_varint(lp); k.put_bytes(fptr(v, i, HLC_F_PARENT), lp); }
      if (lr) { k.put(0xD2); k.put(0x01); k.put_varint(lr); k.put_bytes(fptr(v, i, HLC_F_RECEIVED), lr); }
      k.put(0xDA); k.put(0x01); k.put_varint(lh); k.put_bytes(fptr(v, i, HLC_F_VOTE_HASH), lh);
      k.put(0x01);
      while (k.pos < kec_sz) k.put(0);
      lb[kec_sz - 1] |= 0x80;
      uint64_t sk[25];
#pragma unroll
      for (int q = 0; q < 25; ++q) sk[q] = 0;
      const uint64_t* l8 = reinterpret_cast<const uint64_t*>(lb);
      for (uint32_t b = 0; b < (uint32_t)(kec_sz / 136); ++b) {
#pragma unroll
        for (int q = 0; q < 17; ++q) sk[q] ^= l8[b * 17 + q];
        keccak_f1600(sk);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        kec_dig[i * 8 + 2 * q] = (uint32_t)sk[q];
        kec_dig[i * 8 + 2 * q + 1] = (uint32_t)(sk[q] >> 32);
      }
    }
  }
  pre[i] = st;
  pre_reason[i] = rs;
}

// ---------------- general path without host round trips ----------------
// Votes whose messages exceed the fused kernel's LDS window (PRE_GENERAL: long or non-canonical
// fields) are hashed by streaming their bytes straight from the arena: each message is a short
// list of segments (inline key / varint / integer bytes, or a field in the arena), read byte by
// byte into the SHA-256 / keccak blocks with the padding generated on the fly.  No staging
// buffer, no size scan, no host synchronisation: the kernel is always enqueued and exits at once
// unless k_prehash_fused raised FLAG_GENERAL_PATH.  One lane per vote; rare and not on the fast
// path, so it favours simplicity over speed.
struct Seg {
  const uint8_t* p;  // arena bytes, or nullptr: the inline bytes
  uint32_t len;
  uint8_t inl[12];
};

struct SegStream {
  static constexpr int MAXSEG = 24;
  Seg seg[MAXSEG];
  int nseg = 0;
  uint64_t total = 0;
  int cur = 0;
  uint32_t off = 0;
  __device__ void add_inline(const uint8_t* b, int n) {
    Seg& g = seg[nseg++];
    g.p = nullptr;
    g.len = (uint32_t)n;
    for (int k = 0; k < n; ++k) g.inl[k] = b[k];
    total += (uint64_t)n;
  }
  __device__ void add_bytes(const uint8_t* p, uint32_t n) {
    if (!n) return;
    Seg& g = seg[nseg++];
    g.p = p;
    g.len = n;
    total += n;
  }
  __device__ void add_le(uint64_t x, int n) {
    uint8_t b[8];
    for (int k = 0; k < n; ++k) b[k] = (uint8_t)(x >> (8 * k));
    add_inline(b, n);
  }
  // key (2 bytes) + varint(x)
  __device__ void add_key_varint(uint8_t k0, uint64_t x) {
    uint8_t b[12];
    int n = 0;
    b[n++] = k0;
    b[n++] = 0x01;
    do {
      const uint8_t c = x & 0x7F;
      x >>= 7;
      b[n++] = x ? (uint8_t)(c | 0x80) : c;
    } while (x);
    add_inline(b, n);
  }
  __device__ void add_decimal(uint64_t x) {
    uint8_t d[20], b[12];
    int nd = 0;
    do {
      d[nd++] = (uint8_t)('0' + x % 10);
      x /= 10;
    } while (x);
    int n = 0;
    while (nd && n < 12) b[n++] = d[--nd];
    add_inline(b, n);
    if (nd) {  // > 12 digits (never for real lengths): second piece
      int m = 0;
      while (nd) b[m++] = d[--nd];
      add_inline(b, m);
    }
  }
  __device__ void rewind() {
    cur = 0;
    off = 0;
  }
  // next message byte (caller tracks the position against total)
  __device__ uint8_t next() {
    while (cur < nseg && off >= seg[cur].len) {
      ++cur;
      off = 0;
    }
    const Seg& g = seg[cur];
    const uint8_t b = g.p ? g.p[off] : g.inl[off];
    ++off;
    return b;
  }
};

__global__ void k_prehash_stream(hlc_votes v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                                 const uint32_t* flags, uint32_t* kec_dig, uint8_t* pre, uint8_t* pre_reason,
                                 bool eth) {
  if (!(*flags & FLAG_GENERAL_PATH)) return;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (pre[i] != PRE_GENERAL) continue;  // decided by k_prehash_fused
    // k_prehash_fused only defers votes that passed the proposal_id match and the empty checks
    const uint32_t lo = flen(v, i, HLC_F_OWNER), lp = flen(v, i, HLC_F_PARENT), lr = flen(v, i, HLC_F_RECEIVED);
    const uint32_t lh = flen(v, i, HLC_F_VOTE_HASH), ls = flen(v, i, HLC_F_SIGNATURE);
    const uint32_t id = v.vote_id[i], pid = v.proposal_id[i];
    const uint64_t ts = v.timestamp[i];
    uint8_t st = PRE_PENDING, rs = 0;
    // SHA-256 of compute_vote_hash's input (utils.rs:39-45)
    SegStream m;
    m.add_le(id, 4);
    m.add_bytes(fptr(v, i, HLC_F_OWNER), lo);
    m.add_le(pid, 4);
    m.add_le(ts, 8);
    m.add_le(v.vote[i] ? 1 : 0, 1);
    m.add_bytes(fptr(v, i, HLC_F_PARENT), lp);
    m.add_bytes(fptr(v, i, HLC_F_RECEIVED), lr);
    uint32_t h[8];
    sha256_init(h);
    {
      const uint64_t L = m.total, nb = (L + 9 + 63) / 64;
      uint64_t pos = 0;
      for (uint64_t b = 0; b < nb; ++b) {
        uint32_t w[16];
        for (int k = 0; k < 16; ++k) {
          uint32_t x = 0;
          for (int q = 0; q < 4; ++q, ++pos) {
            uint8_t c;
            if (pos < L) c = m.next();
            else if (pos == L) c = 0x80;
            else if (pos >= nb * 64 - 8) c = (uint8_t)((L * 8) >> (8 * (nb * 64 - 1 - pos)));
            else c = 0;
            x = (x << 8) | c;
          }
          w[k] = x;
        }
        sha256_compress(h, w);
      }
    }
    bool eq = lh == 32;
    if (eq) {
      const uint8_t* hb = fptr(v, i, HLC_F_VOTE_HASH);
      uint32_t diff = 0;
      for (int k = 0; k < 8; ++k) {
        const uint32_t want = (uint32_t)hb[4 * k] << 24 | (uint32_t)hb[4 * k + 1] << 16 |
                              (uint32_t)hb[4 * k + 2] << 8 | (uint32_t)hb[4 * k + 3];
        diff |= want ^ h[k];
      }
      eq = diff == 0;
    }
    if (!eq) {
      st = HLC_INVALID_VOTE_HASH;
    } else if (!eth) {
      // the caller's scheme decides the signature step (st stays PRE_PENDING)
    } else if (ls != 65) {
      st = HLC_SIGNATURE_SCHEME;
      rs = HLC_SCHEME_SIG_LEN;
    } else if (lo != 20) {
      st = HLC_SIGNATURE_SCHEME;
      rs = HLC_SCHEME_ID_LEN;
    } else {
      // keccak256 of the EIP-191 message of the prost encoding, signature cleared (utils.rs:150-152)
      SegStream k;
      const uint8_t pfx[12] = {0x19, 'E', 't', 'h', 'e', 'r', 'e', 'u', 'm', ' ', 'S', 'i'};
      const uint8_t pfx2[12] = {'g', 'n', 'e', 'd', ' ', 'M', 'e', 's', 's', 'a', 'g', 'e'};
      const uint8_t pfx3[2] = {':', '\n'};
      k.add_inline(pfx, 12);
      k.add_inline(pfx2, 12);
      k.add_inline(pfx3, 2);
      k.add_decimal(vote_enc_len(v, i));
      if (id) k.add_key_varint(0xA0, id);
      k.add_key_varint(0xAA, lo);
      k.add_bytes(fptr(v, i, HLC_F_OWNER), lo);
      if (pid) k.add_key_varint(0xB0, pid);
      if (ts) k.add_key_varint(0xB8, ts);
      if (v.vote[i]) k.add_key_varint(0xC0, 1);
      if (lp) { k.add_key_varint(0xCA, lp); k.add_bytes(fptr(v, i, HLC_F_PARENT), lp); }
      if (lr) { k.add_key_varint(0xD2, lr); k.add_bytes(fptr(v, i, HLC_F_RECEIVED), lr); }
      k.add_key_varint(0xDA, lh);
      k.add_bytes(fptr(v, i, HLC_F_VOTE_HASH), lh);
      uint64_t sk[25];
      for (int q = 0; q < 25; ++q) sk[q] = 0;
      const uint64_t L = k.total, nb = L / 136 + 1;
      uint64_t pos = 0;
      for (uint64_t b = 0; b < nb; ++b) {
        for (int q = 0; q < 17; ++q) {
          uint64_t w = 0;
          for (int t = 0; t < 8; ++t, ++pos) {
            uint8_t c;
            if (pos < L) c = k.next();
            else c = (pos == L ? 0x01 : 0) | (pos == nb * 136 - 1 ? 0x80 : 0);
            w |= (uint64_t)c << (8 * t);
          }
          sk[q] ^= w;
        }
        keccak_f1600(sk);
      }
      for (int q = 0; q < 4; ++q) {
        kec_dig[i * 8 + 2 * q] = (uint32_t)sk[q];
        kec_dig[i * 8 + 2 * q + 1] = (uint32_t)(sk[q] >> 32);
      }
    }
    pre[i] = st;
    pre_reason[i] = rs;
  }
}

// per-proposal reduction records: first bad / chain / duplicate = none, YES = 0
// (flag != nullptr: the call's flag word is cleared too, before k_assign_props raises its bits;
// vote_prop != nullptr: its nv entries are set to NO_PROP, the map k_assign_props then fills)
__global__ void k_red_init(uint32_t* red, uint64_t np, uint32_t* flag, uint32_t* vote_prop, uint64_t nv,
                           unsigned long long* zero2) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (flag && p == 0) *flag = 0;
  if (zero2 && p < 2) zero2[p] = 0;
  if (vote_prop && p < nv) vote_prop[p] = NO_PROP;
  if (p < np) reinterpret_cast<uint4*>(red)[p] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u);
}

// clears a table when the device flag word has `bit` set (the large-proposal chain tables)
__global__ void k_clear_if(const uint32_t* flags, uint32_t bit, uint32_t* tab, uint64_t words) {
  if (flags && !(*flags & bit)) return;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < words; k += stride) tab[k] = EMPTY_SLOT;
}

// hlc_eth_verify_batch's byte stage over host-staged items, one lane per item: the length checks
// of EthereumConsensusSigner::verify (signing/ethereum.rs:71-82: the signature's length first, then
// the identity's) and, for the items that pass, keccak256 of the EIP-191 message of the payload
// (alloy eip191_hash_message, reached through recover_address_from_msg at ethereum.rs:89):
// "\x19Ethereum Signed Message:\n" || decimal(len) || payload, absorbed straight from the arena
// (rate 136, pad 0x01 .. 0x80) -- no message buffer, no size scan, no host round trip.
__constant__ uint8_t EIP191_PREFIX[26] = {0x19, 'E', 't', 'h', 'e', 'r', 'e', 'u', 'm', ' ', 'S', 'i', 'g',
                                          'n',  'e', 'd', ' ', 'M', 'e', 's', 's', 'a', 'g', 'e', ':', '\n'};

__global__ void k_verify_prehash(uint64_t n, const uint8_t* bytes, const uint64_t* pay_off, const uint32_t* pay_len,
                                 const uint32_t* sig_len, const uint32_t* id_len, uint32_t* kec_dig, uint8_t* pre,
                                 uint8_t* verify_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (sig_len[i] != 65) {
    pre[i] = 0;
    verify_out[i] = 1 + HLC_SCHEME_SIG_LEN;
    return;
  }
  if (id_len[i] != 20) {
    pre[i] = 0;
    verify_out[i] = 1 + HLC_SCHEME_ID_LEN;
    return;
  }
  pre[i] = PRE_PENDING;
  const uint32_t len = pay_len[i];
  const uint8_t* p = bytes + pay_off[i];
  // decimal digits of len, most significant first
  uint32_t nd = 1;
  for (uint32_t x = len; x >= 10; x /= 10) ++nd;
  const uint64_t H = 26 + nd, L = H + len, nb = L / 136 + 1;
  uint64_t sk[25];
#pragma unroll
  for (int q = 0; q < 25; ++q) sk[q] = 0;
  uint64_t pos = 0;
  for (uint64_t b = 0; b < nb; ++b) {
#pragma unroll 1
    for (int q = 0; q < 17; ++q) {
      uint64_t w = 0;
      if (pos >= H && pos + 8 <= L) {  // eight payload bytes
        const uint8_t* s8 = p + (pos - H);
#pragma unroll
        for (int t = 0; t < 8; ++t) w |= (uint64_t)s8[t] << (8 * t);
        pos += 8;
      } else {
#pragma unroll 1
        for (int t = 0; t < 8; ++t, ++pos) {
          uint32_t c;
          if (pos < 26) {
            c = EIP191_PREFIX[pos];
          } else if (pos < H) {
            uint32_t x = len;
            for (uint64_t k = pos - 26 + 1; k < nd; ++k) x /= 10;
            c = '0' + x % 10;
          } else if (pos < L) {
            c = p[pos - H];
          } else {
            c = (pos == L ? 0x01u : 0u) | (pos == nb * 136 - 1 ? 0x80u : 0u);
          }
          w |= (uint64_t)c << (8 * t);
        }
      }
      sk[q] ^= w;
    }
    keccak_f1600(sk);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    kec_dig[i * 8 + 2 * q] = (uint32_t)sk[q];
    kec_dig[i * 8 + 2 * q + 1] = (uint32_t)(sk[q] >> 32);
  }
}

// The payload `Signer::verify` gets for a vote (utils.rs:150-152): the prost encoding of the Vote with
// its signature cleared (consensus.proto:19-29), for a caller-side scheme (hlc_encode_vote_payloads).
// One lane per vote; sizes first, the bytes at the scanned offsets after.
__global__ void k_payload_sizes(hlc_votes v, uint64_t n, uint64_t* sz64, uint32_t* sz32) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t e = vote_enc_len(v, i);
  sz64[i] = e;
  sz32[i] = (uint32_t)e;
}

__global__ void k_encode_payloads(hlc_votes v, uint64_t n, const uint64_t* off, uint8_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Cursor c{out + off[i], 0};
  const uint32_t id = v.vote_id[i], pid = v.proposal_id[i];
  const uint64_t ts = v.timestamp[i];
  if (id) { c.put(0xA0); c.put(0x01); c.put_varint(id); }
  const uint32_t lo = flen(v, i, HLC_F_OWNER);
  if (lo) { c.put(0xAA); c.put(0x01); c.put_varint(lo); c.put_bytes(fptr(v, i, HLC_F_OWNER), lo); }
  if (pid) { c.put(0xB0); c.put(0x01); c.put_varint(pid); }
  if (ts) { c.put(0xB8); c.put(0x01); c.put_varint(ts); }
  if (v.vote[i]) { c.put(0xC0); c.put(0x01); c.put(0x01); }
  const uint8_t keys[3] = {0xCA, 0xD2, 0xDA};
  for (int f = HLC_F_PARENT; f <= HLC_F_VOTE_HASH; ++f) {
    const uint32_t l = flen(v, i, f);
    if (l) { c.put(keys[f - HLC_F_PARENT]); c.put(0x01); c.put_varint(l); c.put_bytes(fptr(v, i, f), l); }
  }
}

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

}  // namespace

void launch_verify_prehash(uint64_t n, const uint8_t* bytes, const uint64_t* pay_off, const uint32_t* pay_len,
                           const uint32_t* sig_len, const uint32_t* id_len, uint32_t* kec_dig, uint8_t* pre,
                           uint8_t* verify_out, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_verify_prehash, dim3(blocks_for(n)), dim3(TPB), 0, s, n, bytes, pay_off, pay_len, sig_len,
                       id_len, kec_dig, pre, verify_out);
}

hipError_t launch_exclusive_scan(const uint64_t* in, uint64_t* out, uint64_t n, void* temp, size_t& temp_bytes,
                                 hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, s);
}

void launch_prehash_fused(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                          uint32_t* kec_dig, uint8_t* pre, uint8_t* pre_reason, uint32_t* general, hipStream_t s,
                          bool eth) {
  if (!n) return;
  const dim3 grid((unsigned)((n + FUSED_TPB - 1) / FUSED_TPB));
  if (eth)
    hipLaunchKernelGGL(k_prehash_fused<true>, grid, dim3(FUSED_TPB), 0, s, *v, n, vote_prop, props, kec_dig, pre,
                       pre_reason, general);
  else
    hipLaunchKernelGGL(k_prehash_fused<false>, grid, dim3(FUSED_TPB), 0, s, *v, n, vote_prop, props, kec_dig, pre,
                       pre_reason, general);
}

void launch_payload_sizes(const hlc_votes* v, uint64_t n, uint64_t* sz64, uint32_t* sz32, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_payload_sizes, dim3(blocks_for(n)), dim3(TPB), 0, s, *v, n, sz64, sz32);
}

void launch_encode_payloads(const hlc_votes* v, uint64_t n, const uint64_t* off, uint8_t* out, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_encode_payloads, dim3(blocks_for(n)), dim3(TPB), 0, s, *v, n, off, out);
}


hipError_t launch_assign_props(const hlc_proposal* props, uint64_t np, const uint32_t* field_len, uint32_t* vote_prop,
                               uint64_t nv, uint32_t* flags, hipStream_t s, const KEv* ev, bool map_cleared) {
  if (nv && !map_cleared) {
    const hipError_t e = hipMemsetAsync(vote_prop, 0xFF, nv * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
  }
  // a second grid dimension when proposals are large on average (each block then covers ~4k votes)
  const uint64_t g = np ? std::min<uint64_t>(std::max<uint64_t>((nv / np + 4095) / 4096, 1), 1024) : 1;
  if (np)
    launch_k(ev, k_assign_props, dim3((unsigned)np, (unsigned)g), dim3(TPB), 0, s, props, field_len, vote_prop, flags);
  else
    record_kev(ev, s);
  return hipSuccess;
}

void launch_msg_sizes(const hlc_votes* v, uint64_t n, const uint64_t* pay_off, const uint32_t* pay_len,
                      int mode, uint64_t* sha_sz, uint64_t* kec_sz, hipStream_t s) {
  if (!n) return;
  hlc_votes vv = v ? *v : hlc_votes{};
  hipLaunchKernelGGL(k_msg_sizes, dim3(blocks_for(n)), dim3(TPB), 0, s, vv, n, pay_off, pay_len, mode, sha_sz,
                     kec_sz);
}

void launch_build_msgs(const hlc_votes* v, uint64_t n, const uint8_t* bytes, const uint64_t* pay_off,
                       const uint32_t* pay_len, int mode, const uint64_t* sha_off, const uint64_t* sha_sz,
                       uint8_t* sha_buf, const uint64_t* kec_off, const uint64_t* kec_sz, uint8_t* kec_buf,
                       hipStream_t s) {
  if (!n) return;
  hlc_votes vv = v ? *v : hlc_votes{};
  hipLaunchKernelGGL(k_build_msgs, dim3(blocks_for(n)), dim3(TPB), 0, s, vv, n, bytes, pay_off, pay_len, mode,
                     sha_off, sha_sz, sha_buf, kec_off, kec_sz, kec_buf);
}

void launch_sha_blocks(uint64_t n, const uint64_t* off, const uint64_t* sz, const uint8_t* buf, uint32_t* out,
                       hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_sha_blocks, dim3(blocks_for(n)), dim3(TPB), 0, s, n, off, sz, buf, out);
}

void launch_keccak_blocks(uint64_t n, const uint64_t* off, const uint64_t* sz, const uint8_t* buf, uint32_t* out,
                          hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_keccak_blocks, dim3(blocks_for(n)), dim3(TPB), 0, s, n, off, sz, buf, out);
}

void launch_pre_status(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                       const uint32_t* sha_digest, uint8_t* pre, uint8_t* pre_reason, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_pre_status, dim3(blocks_for(n)), dim3(TPB), 0, s, *v, n, vote_prop, props, sha_digest,
                       pre, pre_reason);
}

void launch_vote_status(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                        uint64_t now, const uint8_t* pre, const uint8_t* pre_reason, const uint8_t* verify,
                        uint8_t* status, uint8_t* reason, uint32_t* red, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_vote_status, dim3(blocks_for(n)), dim3(TPB), 0, s,
                       VoteStatusArgs{*v, vote_prop, props, now, pre_reason, status, reason, red}, n, pre, verify);
}

void launch_red_init(uint32_t* red, uint64_t np, hipStream_t s, uint32_t* flag, const KEv* ev, uint32_t* vote_prop,
                     uint64_t nv, unsigned long long* zero2) {
  if (!vote_prop) nv = 0;
  const uint64_t m = std::max(std::max(np, nv), zero2 ? (uint64_t)2 : 0);
  if (m) {
    launch_k(ev, k_red_init, dim3((unsigned)((m + TPB - 1) / TPB)), dim3(TPB), 0, s, red, np, flag, vote_prop, nv,
             zero2);
  } else {
    record_kev(ev, s);
    if (flag) (void)hipMemsetAsync(flag, 0, sizeof(uint32_t), s);
  }
}

void launch_tables(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                   uint32_t* chain_tab, uint32_t* dup_tab, uint32_t mask, uint32_t* red, uint64_t np,
                   const uint32_t* flags, hipStream_t s, const KEv* ev) {
  (void)np;  // (red is initialised by launch_red_init before the vote stage)
  if (!n) return record_kev(ev, s);
  const uint64_t words = (uint64_t)mask + 1;
  const unsigned cb = (unsigned)std::min<uint64_t>((words + TPB - 1) / TPB, 4096);
  const KEv first = kev_start(ev), last = kev_stop(ev);
  launch_k(&first, k_clear_if, dim3(cb), dim3(TPB), 0, s, flags, FLAG_LARGE_PARENTS, chain_tab, words);
  hipLaunchKernelGGL(k_clear_if, dim3(cb), dim3(TPB), 0, s, flags, FLAG_LARGE_PROPOSAL, dup_tab, words);
  launch_k(&last, k_tables, dim3(blocks_for(n)), dim3(TPB), 0, s, *v, n, vote_prop, props, chain_tab, dup_tab, mask,
           red, flags);
}

void launch_prehash_stream(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                           const uint32_t* flags, uint32_t* kec_dig, uint8_t* pre, uint8_t* pre_reason,
                           hipStream_t s, bool eth) {
  if (!n) return;
  // one block per CU at most: the grid exits at once unless k_prehash_fused deferred a vote (rare),
  // and a small grid keeps the queued no-op from occupying the dispatcher behind k_rec_main
  const unsigned blocks = (unsigned)std::min<uint64_t>(blocks_for(n), 256);
  hipLaunchKernelGGL(k_prehash_stream, dim3(blocks), dim3(TPB), 0, s, *v, n, vote_prop, props, flags, kec_dig, pre,
                     pre_reason, eth);
}

void launch_chain_check(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                        const uint8_t* status, const uint32_t* chain_tab, const uint32_t* dup_tab, uint32_t mask,
                        uint8_t* chain_code, uint32_t* red, uint64_t np, const uint32_t* flags, hipStream_t s,
                        const KEv* ev) {
  if (!np || !n) return record_kev(ev, s);  // (red initialised by launch_red_init)
  launch_k(ev, k_chain_check, dim3((unsigned)((n + CHAIN_TPB - 1) / CHAIN_TPB)), dim3(CHAIN_TPB), 0, s, *v, n,
                       vote_prop, props, status,
                       chain_tab, dup_tab, mask, chain_code, red, flags);
}

void launch_timeout(uint64_t n, const hlc_session_tally* ss, uint8_t* out_state, uint8_t* out_status,
                    hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_timeout, dim3(blocks_for(n)), dim3(TPB), 0, s, n, ss, out_state, out_status);
}

void launch_chain_small(const hlc_votes* v, const hlc_proposal* props, uint64_t np, uint8_t* chain_code,
                        uint32_t* red, hipStream_t s, const KEv* ev) {
  if (np)
    launch_k(ev, k_chain_small, dim3((unsigned)np), dim3(SMALL_TPB), 0, s, *v, props, chain_code, red);
  else
    record_kev(ev, s);
}

namespace {
// Outcome counters of a call (the verified / rejected-by-code counters a sharded run
// all-reduces): bins[0..31] = votes by status byte, bins[32..63] = proposals by result status.
// Per block an LDS histogram (one LDS atomic per item), then one global atomic per non-zero bin:
// an all-OK batch costs ~1 global atomic per block, not one per vote on the same address.
constexpr int HIST_BINS = 32;
__global__ void k_outcome_hist(const uint8_t* vst, uint64_t n, const hlc_result* res, uint64_t np,
                               unsigned long long* bins) {
  __shared__ unsigned int h[2 * HIST_BINS];
  if (threadIdx.x < 2 * HIST_BINS) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    atomicAdd(&h[min((unsigned)vst[i], (unsigned)HIST_BINS - 1)], 1u);
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < np; p += stride)
    atomicAdd(&h[HIST_BINS + min((unsigned)res[p].status, (unsigned)HIST_BINS - 1)], 1u);
  __syncthreads();
  if (threadIdx.x < 2 * HIST_BINS && h[threadIdx.x]) atomicAdd(&bins[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}
}  // namespace

void launch_outcome_hist(const uint8_t* vote_status, uint64_t n, const hlc_result* res, uint64_t np,
                         unsigned long long* bins, hipStream_t s) {
  const uint64_t m = std::max(n, np);
  const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((m + 4 * TPB - 1) / (4 * TPB), 1024));
  hipLaunchKernelGGL(k_outcome_hist, dim3(blocks), dim3(TPB), 0, s, vote_status, n, res, np, bins);
}

void launch_finalize(const hlc_proposal* props, uint64_t np, uint64_t now, const uint8_t* status,
                     const uint8_t* reason, const uint8_t* chain_code, const uint32_t* red, hlc_result* out,
                     hipStream_t s, const KEv* ev) {
  if (np)
    launch_k(ev, k_finalize, dim3(blocks_for(np)), dim3(TPB), 0, s, props, np, now, status, reason, chain_code, red,
             out);
  else
    record_kev(ev, s);
}

}  // namespace hlc
