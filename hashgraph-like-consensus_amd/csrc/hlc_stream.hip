// hlc_stream.hip -- the streaming vote path: many independent
// `ConsensusService::process_incoming_vote` calls (service.rs:286-305) micro-batched across
// sessions.  Per-vote validation (validate_vote, utils.rs:127-171) runs through the same
// prehash / recovery / status kernels as validate-many; this file holds the session side:
//   k_sessions_to_props  session -> hlc_proposal (the scalars validate_vote reads)
//   radix sort of (session, vote index), stable -> each session's votes in delivery order
//   k_owner_insert, k_vote_owner_insert, k_dup_flags
//                        one global (session, owner) hash table with the minimum delivery
//                        position per key -> every vote's duplicate flag, in parallel
//   k_apply_votes        one lane per session walks its votes in order: add_vote
//                        (session.rs:225-249) with check_round_limit / update_round /
//                        check_consensus (session.rs:306-387) -- register-only, no probes
// Integer work on a few bytes per vote; the sequential part is per session only.
#include <hipcub/hipcub.hpp>

#include "hlc_kernels.h"
#include "hlc_tally.hpp"

namespace hlc {

namespace {

constexpr int TPB = 256;
constexpr uint32_t EMPTY = 0xFFFFFFFFu;

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// (session, owner) key hash: word-wise for 20-byte addresses (EthereumConsensusSigner identities),
// byte-wise for any other identity length (a caller-side scheme, hlc_process_votes_verdicts)
__device__ __forceinline__ uint32_t owner_hash(uint32_t session, const uint8_t* owner, uint32_t len) {
  uint32_t h = 0x9E3779B9u ^ session * 0x85EBCA6Bu;
  if (len == 20) {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      h ^= ld_le32(owner + 4 * k) * 0xCC9E2D51u;
      h = (h << 13) | (h >> 19);
      h = h * 5u + 0xE6546B64u;
    }
  } else {
    h ^= len * 0x27D4EB2Fu;
    for (uint32_t k = 0; k < len; ++k) {
      h ^= (uint32_t)owner[k] * 0xCC9E2D51u;
      h = (h << 13) | (h >> 19);
      h = h * 5u + 0xE6546B64u;
    }
  }
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h;
}

struct OwnerKeys {
  const uint8_t* owners;          // existing owners: 20 B rows, or an arena indexed by owner_off / owner_len
  const uint64_t* owner_off;      // nullptr: 20-byte rows
  const uint32_t* owner_len;
  const uint32_t* owner_session;  // their sessions
  uint64_t n_owners;
  const uint8_t* bytes;           // vote arena
  const uint64_t* field_off;      // [n][HLC_NFIELDS]
  const uint32_t* field_len;      // [n][HLC_NFIELDS]
  const uint32_t* vote_session;   // [n]
};

__device__ __forceinline__ void existing_owner(const OwnerKeys& k, uint64_t r, const uint8_t*& owner, uint32_t& len) {
  if (k.owner_off) {
    owner = k.owners + k.owner_off[r];
    len = k.owner_len[r];
  } else {
    owner = k.owners + 20ull * r;
    len = 20;
  }
}

__device__ __forceinline__ void key_of(const OwnerKeys& k, uint32_t ref, uint32_t& session, const uint8_t*& owner,
                                       uint32_t& len) {
  if (ref < k.n_owners) {
    session = k.owner_session[ref];
    existing_owner(k, ref, owner, len);
  } else {
    const uint64_t v = ref - k.n_owners;
    session = k.vote_session[v];
    owner = k.bytes + k.field_off[v * HLC_NFIELDS + HLC_F_OWNER];
    len = k.field_len[v * HLC_NFIELDS + HLC_F_OWNER];
  }
}

__device__ __forceinline__ bool same_owner(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
  if (al != bl) return false;
  uint32_t d = 0;
  if (al == 20) {
#pragma unroll
    for (int k = 0; k < 20; ++k) d |= (uint32_t)(a[k] ^ b[k]);
  } else {
    for (uint32_t k = 0; k < al; ++k) d |= (uint32_t)(a[k] ^ b[k]);
  }
  return d == 0;
}

// Slot of key (session, owner), claiming an empty one with `ref` when the key is absent.
// Slots are never deleted, so every lane re-finds a key another lane inserted.
__device__ uint32_t key_slot(uint32_t* tab, uint32_t mask, const OwnerKeys& k, uint32_t session,
                             const uint8_t* owner, uint32_t len, uint32_t ref) {
  uint32_t slot = owner_hash(session, owner, len) & mask;
  for (;;) {
    uint32_t cur = __hip_atomic_load(tab + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == EMPTY) {
      cur = atomicCAS(tab + slot, EMPTY, ref);
      if (cur == EMPTY) return slot;
    }
    uint32_t s2, l2;
    const uint8_t* o2;
    key_of(k, cur, s2, o2, l2);
    if (s2 == session && same_owner(o2, l2, owner, len)) return slot;
    slot = (slot + 1) & mask;
  }
}

__global__ void __launch_bounds__(TPB) k_sessions_to_props(const hlc_session* __restrict__ ss, uint64_t m,
                                                           hlc_proposal* __restrict__ props) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= m) return;
  const hlc_session x = ss[s];
  hlc_proposal p;
  p.vote_begin = 0;
  p.vote_count = 0;
  p.proposal_id = x.proposal_id;
  p.timestamp = x.timestamp;
  p.expiration_timestamp = x.expiration_timestamp;
  p.expected_voters_count = x.expected_voters_count;
  p.max_rounds = x.max_rounds;
  p.consensus_threshold = x.consensus_threshold;
  p.use_gossipsub_rounds = x.use_gossipsub_rounds;
  p.liveness_criteria_yes = x.liveness_criteria_yes;
  for (int k = 0; k < 6; ++k) p._pad[k] = 0;
  props[s] = p;
}

__global__ void __launch_bounds__(TPB) k_iota(uint32_t* __restrict__ v, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

// segment [seg_begin[s], seg_end[s]) of each session in the sorted order (pre-zeroed)
__global__ void __launch_bounds__(TPB) k_segments(const uint32_t* __restrict__ key, uint64_t n,
                                                  uint32_t* __restrict__ seg_begin, uint32_t* __restrict__ seg_end) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t s = key[j];
  if (s == NO_PROP) return;
  if (j == 0 || key[j - 1] != s) seg_begin[s] = (uint32_t)j;
  if (j + 1 == n || key[j + 1] != s) seg_end[s] = (uint32_t)(j + 1);
}

// Duplicate test without the sequential replay (session.rs:236-238).  Within one session's
// delivery order, once a validated vote is refused for any reason but DuplicateVote (decided,
// Failed, expired, round limit), no later vote is inserted.  So a vote that reaches the
// duplicate test is a duplicate iff its owner is in the existing map or an EARLIER validated
// vote of the session has the same owner.  minv[slot] = min over (existing owner -> 0,
// validated vote i -> i + 1); vote i is a duplicate iff minv < i + 1.
__global__ void __launch_bounds__(TPB) k_owner_insert(uint32_t* tab, uint32_t* minv, uint32_t mask, OwnerKeys k) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= k.n_owners) return;
  const uint8_t* owner;
  uint32_t len;
  existing_owner(k, r, owner, len);
  const uint32_t slot = key_slot(tab, mask, k, k.owner_session[r], owner, len, (uint32_t)r);
  atomicMin(minv + slot, 0u);
}

__global__ void __launch_bounds__(TPB) k_vote_owner_insert(uint64_t n, const uint8_t* __restrict__ st,
                                                           uint32_t* tab, uint32_t* minv, uint32_t mask, OwnerKeys k,
                                                           uint32_t* __restrict__ slot_of) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || st[i] != HLC_OK) return;  // only votes that passed validate_vote reach add_vote
  const uint8_t* owner = k.bytes + k.field_off[i * HLC_NFIELDS + HLC_F_OWNER];
  const uint32_t len = k.field_len[i * HLC_NFIELDS + HLC_F_OWNER];
  const uint32_t slot = key_slot(tab, mask, k, k.vote_session[i], owner, len, (uint32_t)(k.n_owners + i));
  atomicMin(minv + slot, (uint32_t)(i + 1));
  slot_of[i] = slot;
}

__global__ void __launch_bounds__(TPB) k_dup_flags(uint64_t n, const uint8_t* __restrict__ st,
                                                   const uint32_t* __restrict__ minv,
                                                   const uint32_t* __restrict__ slot_of, uint8_t* __restrict__ dup) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dup[i] = st[i] == HLC_OK && minv[slot_of[i]] < (uint32_t)(i + 1);
}

// per vote: SessionNotFound or the validate_vote status (the session side may override OK)
__global__ void __launch_bounds__(TPB) k_stream_init(uint64_t n, const uint32_t* __restrict__ vote_session,
                                                     const uint8_t* __restrict__ vstatus, uint8_t* __restrict__ st,
                                                     uint8_t* __restrict__ tr, uint8_t* __restrict__ ins) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st[i] = vote_session[i] == NO_PROP ? (uint8_t)HLC_SESSION_NOT_FOUND : vstatus[i];
  tr[i] = HLC_STILL_ACTIVE;
  ins[i] = 0;
}

// ConsensusSession::add_vote for every validated vote of session s, in delivery order.
constexpr int APPLY_TPB = 64;  // one wave per block: 10k sessions spread over 157 CUs

__global__ void __launch_bounds__(APPLY_TPB) k_apply_votes(hlc_session* __restrict__ ss, uint64_t m,
                                                           const uint32_t* __restrict__ seg_begin,
                                                           const uint32_t* __restrict__ seg_end,
                                                           const uint32_t* __restrict__ order, const uint8_t* vote,
                                                           uint64_t now, const uint8_t* __restrict__ dup,
                                                           uint8_t* __restrict__ st, uint8_t* __restrict__ tr,
                                                           uint8_t* __restrict__ ins) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= m) return;
  const uint32_t b = seg_begin[s], e = seg_end[s];
  if (b >= e) return;
  hlc_session x = ss[s];
  for (uint32_t j = b; j < e; ++j) {
    const uint32_t i = order[j];
    if (st[i] != HLC_OK) continue;  // validate_vote failed: the session is not touched
    uint8_t code = HLC_OK, trans = HLC_STILL_ACTIVE;
    if (x.state == HLC_SESSION_REACHED_NO || x.state == HLC_SESSION_REACHED_YES) {
      trans = x.state == HLC_SESSION_REACHED_YES ? HLC_REACHED_YES : HLC_REACHED_NO;  // session.rs:247
    } else if (x.state != HLC_SESSION_ACTIVE) {
      code = HLC_SESSION_NOT_ACTIVE;  // session.rs:248
    } else if (now >= x.expiration_timestamp) {
      code = HLC_PROPOSAL_EXPIRED;  // session.rs:232, utils.rs:320-328
    } else {
      // check_round_limit(1), session.rs:306-344
      uint32_t projected;
      if (x.use_gossipsub_rounds) {
        projected = (x.round == 2 || x.round == 1) ? 2u : x.round;
      } else {
        const uint32_t cur = x.round ? x.round - 1 : 0;
        projected = cur == 0xFFFFFFFFu ? cur : cur + 1;
      }
      const uint32_t limit =
          x.use_gossipsub_rounds ? x.max_rounds
                                 : (x.max_rounds ? x.max_rounds : threshold_value(x.expected_voters_count,
                                                                                  x.consensus_threshold));
      if (1u > x.expected_voters_count || projected > limit) {
        x.state = HLC_SESSION_FAILED;
        code = HLC_MAX_ROUNDS_EXCEEDED;
      } else {
        if (dup[i]) {
          code = HLC_DUPLICATE_VOTE;  // session.rs:236-238
        } else {
          ins[i] = 1;
          x.total += 1;
          x.yes += vote[i] ? 1u : 0u;
          if (x.use_gossipsub_rounds) {  // update_round(1), session.rs:350-366
            if (x.round == 1) x.round = 2;
          } else if (x.round != 0xFFFFFFFFu) {
            x.round += 1;
          }
          const int c = consensus_result(x.total, x.yes, x.expected_voters_count, x.consensus_threshold,
                                         x.liveness_criteria_yes != 0);  // check_consensus, session.rs:372-387
          x.state = c < 0 ? HLC_SESSION_ACTIVE : (c ? HLC_SESSION_REACHED_YES : HLC_SESSION_REACHED_NO);
          trans = c < 0 ? HLC_STILL_ACTIVE : (c ? HLC_REACHED_YES : HLC_REACHED_NO);
        }
      }
    }
    st[i] = code;
    tr[i] = trans;
  }
  ss[s] = x;
}

}  // namespace

void launch_sessions_to_props(const hlc_session* ss, uint64_t m, hlc_proposal* props, hipStream_t s) {
  if (!m) return;
  hipLaunchKernelGGL(k_sessions_to_props, dim3(blocks_for(m)), dim3(TPB), 0, s, ss, m, props);
}

hipError_t launch_sort_by_session(const uint32_t* vote_session, uint64_t n, uint32_t* keys_out, uint32_t* iota,
                                  uint32_t* order, void* temp, size_t& temp_bytes, hipStream_t s) {
  if (!temp)
    return hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, vote_session, keys_out, iota, order, (int)n, 0, 32,
                                              s);
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_iota, dim3(blocks_for(n)), dim3(TPB), 0, s, iota, n);
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, vote_session, keys_out, iota, order, (int)n, 0, 32, s);
}

void launch_segments(const uint32_t* keys, uint64_t n, uint32_t* seg_begin, uint32_t* seg_end, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_segments, dim3(blocks_for(n)), dim3(TPB), 0, s, keys, n, seg_begin, seg_end);
}

static OwnerKeys owner_keys(const uint8_t* owners, const uint32_t* owner_session, uint64_t n_owners,
                            const hlc_votes* v, const uint32_t* vote_session, const uint64_t* owner_off,
                            const uint32_t* owner_len) {
  OwnerKeys k;
  k.owners = owners;
  k.owner_off = owner_off;
  k.owner_len = owner_len;
  k.field_len = v->field_len;
  k.owner_session = owner_session;
  k.n_owners = n_owners;
  k.bytes = v->bytes;
  k.field_off = v->field_off;
  k.vote_session = vote_session;
  return k;
}

void launch_dup_flags(uint32_t* tab, uint32_t* minv, uint32_t mask, const uint8_t* owners,
                      const uint32_t* owner_session, uint64_t n_owners, const hlc_votes* v, const uint32_t* vote_session,
                      const uint8_t* st, uint32_t* slot_of, uint8_t* dup, hipStream_t s, const uint64_t* owner_off,
                      const uint32_t* owner_len) {
  const OwnerKeys k = owner_keys(owners, owner_session, n_owners, v, vote_session, owner_off, owner_len);
  if (n_owners) hipLaunchKernelGGL(k_owner_insert, dim3(blocks_for(n_owners)), dim3(TPB), 0, s, tab, minv, mask, k);
  const uint64_t n = v->n;
  if (!n) return;
  hipLaunchKernelGGL(k_vote_owner_insert, dim3(blocks_for(n)), dim3(TPB), 0, s, n, st, tab, minv, mask, k, slot_of);
  hipLaunchKernelGGL(k_dup_flags, dim3(blocks_for(n)), dim3(TPB), 0, s, n, st, minv, slot_of, dup);
}

void launch_stream_init(uint64_t n, const uint32_t* vote_session, const uint8_t* vstatus, uint8_t* st, uint8_t* tr,
                        uint8_t* ins, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_stream_init, dim3(blocks_for(n)), dim3(TPB), 0, s, n, vote_session, vstatus, st, tr, ins);
}

void launch_apply_votes(hlc_session* ss, uint64_t m, const uint32_t* seg_begin, const uint32_t* seg_end,
                        const uint32_t* order, const hlc_votes* v, uint64_t now, const uint8_t* dup, uint8_t* st,
                        uint8_t* tr, uint8_t* ins, hipStream_t s) {
  if (!m) return;
  hipLaunchKernelGGL(k_apply_votes, dim3((unsigned)((m + APPLY_TPB - 1) / APPLY_TPB)), dim3(APPLY_TPB), 0, s, ss, m,
                     seg_begin, seg_end, order, v->vote, now, dup, st, tr, ins);
}

}  // namespace hlc
