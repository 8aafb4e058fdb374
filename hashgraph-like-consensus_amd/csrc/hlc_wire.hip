// hlc_wire.hip -- device decoder for gossip-format Proposal messages.
//
// The reference hands prost-decoded `Proposal`s (consensus.proto:5-29) to
// `ConsensusService::process_incoming_proposal` (service.rs:263-279); decoding is prost 0.14's
// `Message::decode` (restated in oracle/wire_oracle.py).  This file performs that decode on the
// GPU so raw wire bytes go straight to the validate-many pipeline, with bit-identical outcomes:
//   k_wire_walk   (one lane per message)  top-level fields of the Proposal: scalars, name
//                                          (UTF-8 checked), payload, owner, and the extents of
//                                          every `votes` record (the first 128 kept per message)
//   hipcub scan of the per-message vote counts -> vote_begin; k_wire_place moves the records
//                                          the walker kept (<= 128 per message) into place
//   k_wire_votes  (one lane per vote)      decodes one Vote record into the hlc_votes SoA;
//                                          bytes fields are (offset, length) into the wire
//                                          buffer itself -- no copy
//   k_wire_final  (one lane per message)   first error in stream order, hlc_proposal records
// All integer/byte work, latency-bound on dependent varint reads.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <utility>

#ifndef WIRE_WALK_LDS_DEFAULT
#define WIRE_WALK_LDS_DEFAULT 0  // the lane walker: 7.0 vs 7.35 ms for the device-resident config-2 wire step
#endif

#include "hlc_kernels.h"

namespace hlc {

namespace {

constexpr int TPB = 256;
constexpr int RECURSION_LIMIT = 100;  // prost DecodeContext default

// Issue priority of the decode kernels' waves (s_setprio).  The wire host entry (hlc_api.cpp
// validate_wire_host) decodes range k+1 while range k's k_rec_main grid holds the SIMDs: at the default
// priority the walker's dependent reads got a third of the issue slots or less, and one range's walk took
// up to 1.5 ms instead of ~0.1 ms, holding back that range's recovery.  The decode is a small amount of
// work that gates everything after it, so its waves go first.  (Alone on the device -- the
// device-resident wire entry -- the priority changes nothing.)
#ifndef HLC_WIRE_PRIO
#define HLC_WIRE_PRIO 3
#endif
__device__ __forceinline__ void wire_prio() {
#if HLC_WIRE_PRIO
  __builtin_amdgcn_s_setprio(HLC_WIRE_PRIO);
#endif
}
constexpr int GROUP_STACK = RECURSION_LIMIT + 1;

enum : int { WT_VARINT = 0, WT_I64 = 1, WT_LEN = 2, WT_SGROUP = 3, WT_EGROUP = 4, WT_I32 = 5 };

// Byte sources the parser reads through: global memory, or an LDS window [wlo, whi) of it with
// global fallback outside the window (fields may run past a window or a vote record).
struct GSrc {
  const uint8_t* g;
  __device__ __forceinline__ uint32_t operator[](uint64_t pos) const { return g[pos]; }
};
// the staged window as an LDS (address space 3) pointer: ds_read_u8, not a flat load that goes the
// long way round through the vector memory pipeline and waits on both counters
typedef const __attribute__((address_space(3))) uint8_t* lds_bytes;
struct WinSrc {
  const uint8_t* g;
  lds_bytes lds;
  uint64_t wlo, wlen;
  __device__ __forceinline__ uint32_t operator[](uint64_t pos) const {
    const uint64_t d = pos - wlo;
    return d < wlen ? (uint32_t)lds[(uint32_t)d] : (uint32_t)g[pos];
  }
};

// Global memory through a 16-byte register cache: a varint or key that lies in one aligned
// 16-byte granule costs one load instead of one per byte.  (An aligned granule holding a valid
// byte never crosses a page, so the granule load cannot fault past the end of the buffer.)
struct CachedSrc {
  const uint8_t* g;
  mutable uint64_t lo = ~0ull;
  mutable uint4 c;
  __device__ __forceinline__ uint32_t operator[](uint64_t pos) const {
    const uint64_t a = pos & ~15ull;
    if (a != lo) {
      c = *reinterpret_cast<const uint4*>(g + a);
      lo = a;
    }
    const uint32_t k = (uint32_t)(pos & 15);
    const uint32_t w = k < 8 ? (k < 4 ? c.x : c.y) : (k < 12 ? c.z : c.w);
    return (w >> (8 * (k & 3))) & 0xFFu;
  }
};

// prost decode_varint: <= 10 bytes, the 10th must be < 2; out of bytes = invalid varint.
template <class Src>
__device__ __forceinline__ int rd_varint(const Src& b, uint64_t& pos, uint64_t end, uint64_t& v) {
  v = 0;
  uint64_t avail = end - pos;
  int lim = avail < 10 ? (int)avail : 10;
  for (int c = 0; c < lim; ++c) {
    uint32_t byte = b[pos + c];
    v |= (uint64_t)(byte & 0x7F) << (7 * c);
    if (byte < 0x80) {
      if (c == 9 && byte >= 2) return HLC_WIRE_INVALID_VARINT;
      pos += c + 1;
      return HLC_WIRE_OK;
    }
  }
  return HLC_WIRE_INVALID_VARINT;
}

// prost decode_key
template <class Src>
__device__ __forceinline__ int rd_key(const Src& b, uint64_t& pos, uint64_t end, uint32_t& tag, int& wt) {
  uint64_t k;
  int e = rd_varint(b, pos, end, k);
  if (e) return e;
  if (k > 0xFFFFFFFFull) return HLC_WIRE_INVALID_KEY;
  wt = (int)(k & 7);
  if (wt > 5) return HLC_WIRE_INVALID_WIRE_TYPE;
  tag = (uint32_t)(k >> 3);
  if (tag < 1) return HLC_WIRE_INVALID_TAG;
  return HLC_WIRE_OK;
}

// length-delimited value: (offset, length) of the payload, "buffer underflow" past the end
template <class Src>
__device__ __forceinline__ int rd_len(const Src& b, uint64_t& pos, uint64_t end, uint64_t& off, uint32_t& len) {
  uint64_t n;
  int e = rd_varint(b, pos, end, n);
  if (e) return e;
  if (n > end - pos) return HLC_WIRE_BUFFER_UNDERFLOW;
  off = pos;
  len = (uint32_t)n;  // < end - pos <= message length (u32)
  pos += n;
  return HLC_WIRE_OK;
}

// prost skip_field for a non-group unknown field (the recursion budget is checked by the caller)
template <class Src>
__device__ __forceinline__ int skip_scalar(const Src& b, uint64_t& pos, uint64_t end, int wt) {
  if (wt == WT_VARINT) {
    uint64_t v;
    return rd_varint(b, pos, end, v);
  }
  if (wt == WT_LEN) {
    uint64_t off;
    uint32_t len;
    return rd_len(b, pos, end, off, len);
  }
  const uint64_t n = wt == WT_I64 ? 8 : 4;
  if (n > end - pos) return HLC_WIRE_BUFFER_UNDERFLOW;
  pos += n;
  return HLC_WIRE_OK;
}

// prost skip_field for an unknown field, `budget` = DecodeContext recursion budget (every call
// checks it; nested fields are skipped with ctx.enter_recursion()).  Groups are skipped
// iteratively with an explicit stack of open group tags (private memory, touched only by
// messages that carry groups).
__device__ __noinline__ int skip_field(const uint8_t* __restrict__ g, uint64_t& pos, uint64_t end, int wt,
                                       uint32_t tag, int budget) {
  const GSrc b{g};  // unknown fields are rare: read them from global memory
  if (budget == 0) return HLC_WIRE_RECURSION_LIMIT;
  if (wt == WT_EGROUP) return HLC_WIRE_UNEXPECTED_END_GROUP;
  if (wt != WT_SGROUP) return skip_scalar(b, pos, end, wt);
  uint32_t stack[GROUP_STACK];
  int depth = 0;
  stack[0] = tag;
  for (;;) {
    uint32_t itag;
    int iwt;
    int e = rd_key(b, pos, end, itag, iwt);
    if (e) return e;
    if (iwt == WT_EGROUP) {
      if (itag != stack[depth]) return HLC_WIRE_UNEXPECTED_END_GROUP;
      if (depth == 0) return HLC_WIRE_OK;
      --depth;
      continue;
    }
    if (budget - 1 - depth == 0) return HLC_WIRE_RECURSION_LIMIT;  // the nested call's check
    if (iwt == WT_SGROUP) {
      stack[++depth] = itag;
      continue;
    }
    if ((e = skip_scalar(b, pos, end, iwt))) return e;
  }
}

// Rust str::from_utf8 (well-formed UTF-8: no overlongs, surrogates or > U+10FFFF)
__device__ __noinline__ bool utf8_ok(const uint8_t* __restrict__ p, uint32_t n) {
  uint32_t i = 0;
  while (i < n) {
    uint32_t c = p[i];
    if (c < 0x80) {
      ++i;
      continue;
    }
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) {
      need = 1;
    } else if (c >= 0xE0 && c <= 0xEF) {
      need = 2;
      if (c == 0xE0) lo = 0xA0;
      if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      need = 3;
      if (c == 0xF0) lo = 0x90;
      if (c == 0xF4) hi = 0x8F;
    } else {
      return false;
    }
    if (n - i - 1 < need) return false;
    uint32_t c1 = p[i + 1];
    if (c1 < lo || c1 > hi) return false;
    for (uint32_t k = 2; k <= need; ++k) {
      uint32_t ck = p[i + k];
      if (ck < 0x80 || ck > 0xBF) return false;
    }
    i += need + 1;
  }
  return true;
}

struct WalkOut {
  uint32_t proposal_id, expected_voters, round;
  uint64_t timestamp, expiration;
  uint8_t liveness;
  uint64_t name_off, payload_off, owner_off;
  uint32_t name_len, payload_len, owner_len;
};

constexpr uint32_t SLAB = 128;  // vote records a walker keeps per message before the vote count is known
// Messages longer than this are not walked by one lane (about 1 us per field) but by the parallel
// boundary-discovery path below.  Its next[] array encodes offsets below HUGE_ERR and its scans
// count items in an int, so messages of 2^31 - 2 bytes or more stay with the (slow, exact) walker.
constexpr uint32_t HUGE_MSG = 1u << 20;
constexpr uint32_t HUGE_MAX = 0x7FFFFFFEu;
constexpr uint32_t HUGE_ERR = 0xFFFFFF00u;
constexpr uint32_t HUGE_UNRES = 0xFFu;  // internal marker, never reported (not a prost error code)
constexpr int HUGE_RESUME_PASSES = 4;     // parallel re-marking passes past long top-level groups
constexpr uint64_t HUGE_GROUP_SCAN = 256;
__host__ __device__ __forceinline__ bool is_huge(uint32_t len) { return len > HUGE_MSG && len < HUGE_MAX; }

// Loads wire[wlo, whi) (wlo 16-byte aligned) into LDS with the calling block's threads.  Each thread
// issues LW_BATCH 16-byte loads before its first LDS write, so a window costs one or two memory round
// trips instead of one per granule (a load followed by its LDS write in one loop iteration waits for
// the load every time: 12 serial misses for a 12 KB message window on a 64-lane block).
#ifndef HLC_WIN_BATCH
#define HLC_WIN_BATCH 12  // A/B knob: 1 = one granule per round trip (the round-5 loader's behaviour)
#endif
constexpr int LW_BATCH = HLC_WIN_BATCH;
__device__ __forceinline__ void load_window(uint8_t* lds, const uint8_t* __restrict__ wire, uint64_t wlo,
                                            uint64_t whi, bool aligned) {
  const uint64_t n = whi - wlo;
  const uint64_t full = aligned ? n / 16 : 0;  // granules loaded whole
  const uint64_t step = blockDim.x;
  const uint8_t* src = wire + wlo;  // uniform base, 32-bit per-lane offsets (windows are < 4 GB)
  for (uint64_t c0 = threadIdx.x; c0 < full; c0 += step * LW_BATCH) {
    uint4 r[LW_BATCH];
    // unpredicated loads (a granule past the window reloads the window's last one)
#pragma unroll
    for (int j = 0; j < LW_BATCH; ++j) {
      const uint32_t c = (uint32_t)std::min<uint64_t>(c0 + j * step, full - 1);
      r[j] = *reinterpret_cast<const uint4*>(src + c * 16u);
    }
    // (unpredicated stores too: a clamped granule is written again with the same bytes.  A store under
    // a branch lets the compiler sink its load into the branch, one wait per load again.)
#pragma unroll
    for (int j = 0; j < LW_BATCH; ++j) {
      const uint64_t c = std::min<uint64_t>(c0 + j * step, full - 1);
      *reinterpret_cast<uint4*>(lds + c * 16) = r[j];
    }
  }
  for (uint64_t k = full * 16 + threadIdx.x; k < n; k += step) lds[k] = wire[wlo + k];  // the ragged tail
}

// One field of the Proposal at `pos` (prost Proposal::merge_field, consensus.proto:5-16).
template <class Src>
__device__ __forceinline__ int walk_field(const Src& src, const uint8_t* __restrict__ wire, uint64_t& pos,
                                          uint64_t base, uint64_t end, WalkOut& o, uint32_t& nv,
                                          uint64_t* __restrict__ rec_off, uint32_t* __restrict__ rec_len,
                                          uint32_t rec_cap) {
  uint32_t tag;
  int wt, err;
  if ((err = rd_key(src, pos, end, tag, wt))) return err;
  uint64_t v = 0, off = 0;
  uint32_t len = 0;
  if (tag >= 10 && tag <= 19) {
    const bool is_len = tag == 10 || tag == 11 || tag == 13 || tag == 14;
    if (wt != (is_len ? WT_LEN : WT_VARINT)) return HLC_WIRE_WIRE_TYPE_MISMATCH;
    if ((err = is_len ? rd_len(src, pos, end, off, len) : rd_varint(src, pos, end, v))) return err;
  }
  switch (tag) {
    case 10:
      o.name_off = off - base;
      o.name_len = len;
      return utf8_ok(wire + off, len) ? HLC_WIRE_OK : HLC_WIRE_INVALID_UTF8;
    case 11: o.payload_off = off - base; o.payload_len = len; return HLC_WIRE_OK;
    case 12: o.proposal_id = (uint32_t)v; return HLC_WIRE_OK;
    case 13: o.owner_off = off - base; o.owner_len = len; return HLC_WIRE_OK;
    case 14:
      if (nv < rec_cap) {
        rec_off[nv] = off;
        rec_len[nv] = len;
      }
      ++nv;
      return HLC_WIRE_OK;
    case 15: o.expected_voters = (uint32_t)v; return HLC_WIRE_OK;
    case 16: o.round = (uint32_t)v; return HLC_WIRE_OK;
    case 17: o.timestamp = v; return HLC_WIRE_OK;
    case 18: o.expiration = v; return HLC_WIRE_OK;
    case 19: o.liveness = v != 0; return HLC_WIRE_OK;
    default: return skip_field(wire, pos, end, wt, tag, RECURSION_LIMIT);
  }
}

// Per-message outputs of a completed top-level walk (shared by the serial walker and the
// parallel huge-message path).
__device__ __forceinline__ void emit_message(uint64_t m, const WalkOut& o, uint32_t nv, int err,
                                             uint64_t* __restrict__ vote_count, hlc_wire_proposal* __restrict__ wout,
                                             hlc_proposal* __restrict__ pout, const hlc_scope_config* scope,
                                             uint64_t n_scope) {
  vote_count[m] = nv;
  hlc_wire_proposal w;
  w.name_off = o.name_off;  // relative to the message; 0 when the field is absent
  w.payload_off = o.payload_off;
  w.owner_off = o.owner_off;
  w.name_len = o.name_len;
  w.payload_len = o.payload_len;
  w.owner_len = o.owner_len;
  w.round = o.round;
  w.decode_status = (uint8_t)err;  // k_wire_final folds in the votes' errors
  w.bad_vote = 0xFFFFFFFFu;
  for (int k = 0; k < 3; ++k) w._pad[k] = 0;
  wout[m] = w;
  const hlc_scope_config sc = scope[n_scope == 1 ? 0 : m];
  hlc_proposal p;
  p.vote_begin = 0;
  p.vote_count = nv;
  p.proposal_id = o.proposal_id;
  p.timestamp = o.timestamp;
  p.expiration_timestamp = o.expiration;
  p.expected_voters_count = o.expected_voters;
  p.max_rounds = sc.max_rounds;
  p.consensus_threshold = sc.consensus_threshold;
  p.use_gossipsub_rounds = sc.use_gossipsub_rounds;
  p.liveness_criteria_yes = o.liveness;
  for (int k = 0; k < 6; ++k) p._pad[k] = 0;
  pout[m] = p;
}

// Top-level walk of message m, one lane per message.  The walk is a chain of dependent reads
// (key, length, skip) -- about one cache miss per field -- so lanes are kept independent: a wave
// walks 64 messages at once.  (A wave-per-message walker parsing out of an LDS window measured
// 2x slower: the parse is issue-bound when one lane of 64 does it.)
// mode 0 (every message): writes wout[m], pout[m] (vote_begin later), vote_count[m] and the first
//   SLAB vote records to slab[m * SLAB + k]; sets *big when a message has more records.
// mode 1 (only messages with > SLAB records): writes every record at vote_begin[m] + k.
constexpr int WALK_TPB = 64;  // one wave per block: 10k messages = 157 waves spread over 157 CUs, not 40

__global__ void __launch_bounds__(WALK_TPB) k_wire_walk(int mode, const uint8_t* __restrict__ wire, int aligned,
                                                   const uint64_t* __restrict__ msg_off,
                                                   const uint32_t* __restrict__ msg_len, uint64_t nm,
                                                   uint64_t* __restrict__ vote_count,
                                                   const uint64_t* __restrict__ vote_begin,
                                                   hlc_wire_proposal* __restrict__ wout,
                                                   hlc_proposal* __restrict__ pout, const hlc_scope_config* scope,
                                                   uint64_t n_scope, uint64_t* __restrict__ slab_off,
                                                   uint32_t* __restrict__ slab_len, uint32_t* __restrict__ big,
                                                   uint64_t* __restrict__ vrec_off, uint32_t* __restrict__ vrec_len,
                                                   uint32_t* __restrict__ vrec_msg, uint64_t* __restrict__ huge,
                                                   uint32_t* __restrict__ first_bad) {
  wire_prio();
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  if (mode == 0 && first_bad) first_bad[m] = 0xFFFFFFFFu;  // (k_wire_votes*' atomicMin target)
  if (is_huge(msg_len[m])) {  // decoded by the parallel boundary-discovery path instead
    if (mode == 0) {
      vote_count[m] = 0;  // until launch_huge_decode
      const uint64_t i = atomicAdd((unsigned long long*)huge, 1ull);
      huge[1 + 2 * i] = m;
      huge[2 + 2 * i] = msg_len[m];
    }
    return;
  }
  if (mode == 1 && vote_count[m] <= SLAB) return;
  const uint64_t base = msg_off[m];
  const uint64_t end = base + msg_len[m];
  uint64_t* rec_off;
  uint32_t* rec_len;
  uint32_t rec_cap;
  if (mode == 0) {
    rec_off = slab_off + m * SLAB;
    rec_len = slab_len + m * SLAB;
    rec_cap = SLAB;
  } else {
    rec_off = vrec_off + vote_begin[m];
    rec_len = vrec_len + vote_begin[m];
    rec_cap = 0xFFFFFFFFu;
  }
  WalkOut o = {};
  uint32_t nv = 0;
  int err = HLC_WIRE_OK;
  uint64_t pos = base;
  if (aligned) {
    const CachedSrc src{wire};
    while (pos < end)
      if ((err = walk_field(src, wire, pos, base, end, o, nv, rec_off, rec_len, rec_cap))) break;
  } else {
    const GSrc src{wire};
    while (pos < end)
      if ((err = walk_field(src, wire, pos, base, end, o, nv, rec_off, rec_len, rec_cap))) break;
  }
  if (mode == 1) {
    for (uint32_t k = 0; k < nv; ++k) vrec_msg[vote_begin[m] + k] = (uint32_t)m;
    return;
  }
  if (nv > SLAB) atomicOr(big, 1u);
  emit_message(m, o, nv, err, vote_count, wout, pout, scope, n_scope);
}

// Mode-0 walk with the messages staged in LDS first: one wave per LW_MPW messages.  The wave's 64 lanes
// copy each message's first LW_WIN bytes into LDS with 16-byte loads (coalesced, all misses in flight at
// once), then lane j parses message j out of LDS (WinSrc: bytes past the window from global memory,
// e.g. the tail of a message longer than the window; the name's UTF-8 check and unknown fields read
// global memory as in k_wire_walk).  The lane-per-message walker above pays one dependent miss per
// field (~70 per config-2 message); here a field costs a few LDS reads.  That matters most when the
// walk shares the device with k_rec_main (the wire host entry decodes range k+1 while range k
// recovers): there the lane walker's misses wait behind the recovery's table traffic.  Same outputs
// as k_wire_walk mode 0, message for message.
constexpr int LW_MPW = 4;           // messages per wave
constexpr uint32_t LW_WIN = 12288;  // LDS bytes per message (a config-2 message is ~11.9 KB)

__global__ void __launch_bounds__(64) k_wire_walk_lds(const uint8_t* __restrict__ wire, int aligned,
                                                      const uint64_t* __restrict__ msg_off,
                                                      const uint32_t* __restrict__ msg_len, uint64_t nm,
                                                      uint64_t* __restrict__ vote_count,
                                                      hlc_wire_proposal* __restrict__ wout,
                                                      hlc_proposal* __restrict__ pout, const hlc_scope_config* scope,
                                                      uint64_t n_scope, uint64_t* __restrict__ slab_off,
                                                      uint32_t* __restrict__ slab_len, uint32_t* __restrict__ big,
                                                      uint64_t* __restrict__ huge, uint32_t* __restrict__ first_bad) {
  wire_prio();
  __shared__ __attribute__((aligned(16))) uint8_t win[LW_MPW * LW_WIN];
  const uint64_t m0 = (uint64_t)blockIdx.x * LW_MPW;
  uint64_t my_lo = 0, my_len = 0;
#pragma unroll 1
  for (int j = 0; j < LW_MPW; ++j) {
    const uint64_t m = m0 + j;
    if (m >= nm) break;
    const uint32_t len = msg_len[m];
    if (!len || is_huge(len)) continue;
    const uint64_t lo = msg_off[m] & ~15ull;
    const uint64_t hi = std::min<uint64_t>(msg_off[m] + len, lo + LW_WIN);
    load_window(win + (size_t)j * LW_WIN, wire, lo, hi, aligned != 0);
    if ((int)threadIdx.x == j) {
      my_lo = lo;
      my_len = hi - lo;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x >= LW_MPW) return;
  const uint64_t m = m0 + threadIdx.x;
  if (m >= nm) return;
  if (first_bad) first_bad[m] = 0xFFFFFFFFu;
  if (is_huge(msg_len[m])) {  // decoded by the parallel boundary-discovery path instead
    vote_count[m] = 0;
    const uint64_t i = atomicAdd((unsigned long long*)huge, 1ull);
    huge[1 + 2 * i] = m;
    huge[2 + 2 * i] = msg_len[m];
    return;
  }
  const uint64_t base = msg_off[m];
  const uint64_t end = base + msg_len[m];
  WalkOut o = {};
  uint32_t nv = 0;
  int err = HLC_WIRE_OK;
  uint64_t pos = base;
  const WinSrc src{wire, (lds_bytes)(win + (size_t)threadIdx.x * LW_WIN), my_lo, my_len};
  while (pos < end)
    if ((err = walk_field(src, wire, pos, base, end, o, nv, slab_off + m * SLAB, slab_len + m * SLAB, SLAB))) break;
  if (nv > SLAB) atomicOr(big, 1u);
  emit_message(m, o, nv, err, vote_count, wout, pout, scope, n_scope);
}

// ---- Huge messages: parallel record-boundary discovery --------------------------------------
// One lane walking a 180 MB gossip message costs about 1 us per field however the bytes are
// staged (dependent reads, branchy 64-bit arithmetic).  Instead every byte offset p of the message
// is parsed as a candidate top-level field start: next[p] = offset just past that field, or
// HUGE_ERR | error code.  The fields of the message are the chain 0 -> next[0] -> ... ; pointer
// jumping marks it in log2(len) rounds: round k, with J = next^(2^k), marks J[p] for every marked
// p (steps [2^k, 2^(k+1)) from the start) and squares J.  The marked offsets are then parsed in
// parallel; stream order is the byte offset itself (first error = smallest marked offset whose
// parse fails, scalar fields = largest marked offset of their tag, vote records ranked by a scan).

// The candidate top-level field at offset p: the offset just past it, or HUGE_ERR | error code.
// bounded: a group is scanned at most HUGE_GROUP_SCAN bytes (HUGE_UNRES beyond), since a group
// started at a byte inside a record can run on through every later record -- quadratic over all
// offsets.  Unbounded (the tail walk below), it is exactly walk_field's structure check.
__device__ __forceinline__ uint32_t huge_parse(const uint8_t* __restrict__ wire, uint64_t base, uint32_t len,
                                               uint64_t p, bool bounded) {
  const GSrc src{wire};
  const uint64_t end = base + len;
  uint64_t pos = base + p;
  uint32_t tag;
  int wt;
  int err = rd_key(src, pos, end, tag, wt);
  if (!err) {
    if (tag >= 10 && tag <= 19) {  // the same checks as walk_field, without the side effects
      const bool is_len = tag == 10 || tag == 11 || tag == 13 || tag == 14;
      if (wt != (is_len ? WT_LEN : WT_VARINT)) {
        err = HLC_WIRE_WIRE_TYPE_MISMATCH;
      } else if (is_len) {
        uint64_t off;
        uint32_t l;
        err = rd_len(src, pos, end, off, l);
      } else {
        uint64_t v;
        err = rd_varint(src, pos, end, v);
      }
    } else {
      const uint64_t lim = bounded && wt == WT_SGROUP && end - pos > HUGE_GROUP_SCAN ? pos + HUGE_GROUP_SCAN : end;
      err = skip_field(wire, pos, lim, wt, tag, RECURSION_LIMIT);
      if (err && lim < end) err = HUGE_UNRES;
    }
  }
  return err ? (HUGE_ERR | (uint32_t)err) : (uint32_t)(pos - base);
}

// next[p] for p in [0, len]; next[len] = len (the chain's regular end).
__global__ void __launch_bounds__(TPB) k_huge_next(const uint8_t* __restrict__ wire, uint64_t base, uint32_t len,
                                                   uint32_t* __restrict__ next) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= len; p += (uint64_t)gridDim.x * blockDim.x)
    next[p] = p == len ? len : huge_parse(wire, base, len, p, true);
}

// The first unresolved offset on the chain (st[11], 0xFFFFFFFF if none).  The chain stops there
// (its next[] is an error code), so no offset after it is marked.
__global__ void __launch_bounds__(TPB) k_huge_unres(uint32_t len, const uint32_t* __restrict__ next,
                                                    const uint8_t* __restrict__ mark, uint32_t* st) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < len; p += (uint64_t)gridDim.x * blockDim.x)
    if (mark[p] && next[p] == (HUGE_ERR | HUGE_UNRES)) atomicMin(st + 11, (uint32_t)p);
}

// One lane resolves the first unresolved offset on the chain (st[11]) with an unbounded group skip
// and patches next[] there, so that a fresh set of pointer-jumping rounds continues the chain in
// parallel past the long group; st[12] = 1 when it did (the rounds of this pass run), else 0.
__global__ void k_huge_resolve(const uint8_t* __restrict__ wire, uint64_t base, uint32_t len,
                               uint32_t* __restrict__ next, uint32_t* st) {
  if (threadIdx.x || blockIdx.x) return;
  const uint32_t p = st[11];
  st[12] = 0;
  if (p == 0xFFFFFFFFu) return;
  const uint32_t q = huge_parse(wire, base, len, p, false);
  next[p] = q;
  st[12] = q < HUGE_ERR ? 1u : 0u;
}

// J = next for a resumed pass (only when k_huge_resolve patched an offset)
__global__ void __launch_bounds__(TPB) k_huge_copy_if(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                      uint32_t len, const uint32_t* st) {
  if (!st[12]) return;
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= len; p += (uint64_t)gridDim.x * blockDim.x)
    dst[p] = src[p];
}

// After the bounded resumed passes, one lane walks whatever is left of the top-level fields from
// the first still-unresolved offset with unbounded group skips, writing their next[] entries and
// marks: linear in the rest of the message, with no host round trip (a no-op when st[11] is unset).
__global__ void k_huge_tail(const uint8_t* __restrict__ wire, uint64_t base, uint32_t len, uint32_t* __restrict__ next,
                            uint8_t* __restrict__ mark, const uint32_t* st) {
  if (threadIdx.x || blockIdx.x) return;
  uint32_t p = st[11];
  if (p == 0xFFFFFFFFu) return;
  while (p < len) {
    const uint32_t q = huge_parse(wire, base, len, p, false);
    next[p] = q;
    mark[p] = 1;
    if (q >= HUGE_ERR) break;
    p = q;
  }
}

// One pointer-jumping round: marks J[p] for marked p, J1 = J o J.  Concurrent marks within a round
// only ever add offsets reachable from the start, so the byte stores need no ordering.
__global__ void __launch_bounds__(TPB) k_huge_round(const uint32_t* __restrict__ J, uint32_t* __restrict__ J1,
                                                    uint8_t* mark, uint32_t len, const uint32_t* active) {
  if (active && !*active) return;  // a resumed pass that has nothing to resume
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= len; p += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = J[p];
    if (j < len) {
      if (mark[p]) mark[j] = 1;
      J1[p] = J[j];
    } else {
      J1[p] = j;
    }
  }
}

// First error in stream order: the smallest marked offset whose field fails (structure, or the
// name's UTF-8 check).  st[0] = that offset (0xFFFFFFFF if none).
__global__ void __launch_bounds__(TPB) k_huge_first_error(const uint8_t* __restrict__ wire, uint64_t base,
                                                          uint32_t len, const uint32_t* __restrict__ next,
                                                          const uint8_t* __restrict__ mark, uint32_t* st) {
  const GSrc src{wire};
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < len; p += (uint64_t)gridDim.x * blockDim.x) {
    if (!mark[p]) continue;
    if (next[p] >= HUGE_ERR) {
      atomicMin(st, (uint32_t)p);
      continue;
    }
    uint64_t pos = base + p, off;
    uint32_t tag, l;
    int wt;
    (void)rd_key(src, pos, base + len, tag, wt);  // parsed cleanly by k_huge_next
    if (tag == 10 && !rd_len(src, pos, base + len, off, l) && !utf8_ok(wire + off, l)) atomicMin(st, (uint32_t)p);
  }
}

// Marked fields at or before the first error that parsed: scalars record their last offset (+1)
// in st[1 + tag - 10]; vote records get flag 1 for the rank scan.  (A name failing UTF-8 is at the
// error offset and is still assigned, as the serial walker does.)
__global__ void __launch_bounds__(TPB) k_huge_fields(const uint8_t* __restrict__ wire, uint64_t base, uint32_t len,
                                                     const uint32_t* __restrict__ next,
                                                     const uint8_t* __restrict__ mark, uint32_t* st,
                                                     uint32_t* __restrict__ flag) {
  const GSrc src{wire};
  const uint32_t e = st[0];
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= len; p += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t f = 0;
    if (p < len && mark[p] && next[p] < HUGE_ERR && p <= e) {
      uint64_t pos = base + p;
      uint32_t tag;
      int wt;
      (void)rd_key(src, pos, base + len, tag, wt);  // parsed cleanly by k_huge_next
      if (tag == 14) {
        f = 1;
      } else if (tag >= 10 && tag <= 19) {
        atomicMax(st + 1 + (tag - 10), (uint32_t)p + 1);
      }
    }
    flag[p] = f;
  }
}

// Vote records in stream order: rank = exclusive scan of the flags.
__global__ void __launch_bounds__(TPB) k_huge_records(const uint8_t* __restrict__ wire, uint64_t base, uint32_t len,
                                                      const uint32_t* __restrict__ flag,
                                                      const uint32_t* __restrict__ rank, uint64_t* __restrict__ hoff,
                                                      uint32_t* __restrict__ hlen) {
  const GSrc src{wire};
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < len; p += (uint64_t)gridDim.x * blockDim.x) {
    if (!flag[p]) continue;
    uint64_t pos = base + p, off;
    uint32_t tag, l;
    int wt;
    (void)rd_key(src, pos, base + len, tag, wt);
    (void)rd_len(src, pos, base + len, off, l);
    hoff[rank[p]] = off;
    hlen[rank[p]] = l;
  }
}

// One lane: the winning scalar fields are re-parsed with walk_field, then the same outputs as the
// serial walker.
__global__ void k_huge_emit(const uint8_t* __restrict__ wire, uint64_t m, uint64_t base, uint32_t len,
                            const uint32_t* __restrict__ next, const uint32_t* st, const uint32_t* __restrict__ rank,
                            uint64_t* __restrict__ vote_count, hlc_wire_proposal* __restrict__ wout,
                            hlc_proposal* __restrict__ pout, const hlc_scope_config* scope, uint64_t n_scope) {
  if (threadIdx.x || blockIdx.x) return;
  const GSrc src{wire};
  WalkOut o = {};
  uint32_t dummy = 0;
  for (int t = 0; t < 10; ++t) {
    if (t == 4 || !st[1 + t]) continue;
    uint64_t pos = base + st[1 + t] - 1;
    (void)walk_field(src, wire, pos, base, base + len, o, dummy, nullptr, nullptr, 0);
  }
  const uint32_t e = st[0];
  int err = HLC_WIRE_OK;
  if (e != 0xFFFFFFFFu) err = next[e] >= HUGE_ERR ? (int)(next[e] & 0xFFu) : HLC_WIRE_INVALID_UTF8;
  emit_message(m, o, (uint32_t)rank[len], err, vote_count, wout, pout, scope, n_scope);
}

// After the vote_begin scan: the huge message's records into place.
__global__ void __launch_bounds__(TPB) k_huge_place(uint64_t m, const uint64_t* __restrict__ vote_count,
                                                    const uint64_t* __restrict__ vote_begin,
                                                    const uint64_t* __restrict__ hoff, const uint32_t* __restrict__ hlen,
                                                    uint64_t* __restrict__ vrec_off, uint32_t* __restrict__ vrec_len,
                                                    uint32_t* __restrict__ vrec_msg) {
  const uint64_t n = vote_count[m], b = vote_begin[m];
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    vrec_off[b + k] = hoff[k];
    vrec_len[b + k] = hlen[k];
    vrec_msg[b + k] = (uint32_t)m;
  }
}

// Streams the wire bytes once (16-byte loads, grid-stride) so the walker's dependent reads --
// one cache miss per field -- hit the Infinity Cache instead of HBM.
__global__ void __launch_bounds__(TPB) k_wire_touch(const uint8_t* __restrict__ wire, uint64_t len,
                                                    uint32_t* __restrict__ sink) {
  wire_prio();
  uint32_t acc = 0;
  const uint64_t n16 = len / 16;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n16; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = reinterpret_cast<const uint4*>(wire)[c];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u && len == 1) *sink = acc;  // never true: keeps the loads
}

// Slab records -> their final place (one lane per (message, record < SLAB)); vb_base + vote_begin into pout.
__global__ void __launch_bounds__(TPB) k_wire_place(uint64_t nm, const uint64_t* __restrict__ vote_count,
                                                    const uint64_t* __restrict__ vote_begin,
                                                    const uint64_t* __restrict__ slab_off,
                                                    const uint32_t* __restrict__ slab_len,
                                                    hlc_proposal* __restrict__ pout, uint64_t* __restrict__ vrec_off,
                                                    uint32_t* __restrict__ vrec_len, uint32_t* __restrict__ vrec_msg,
                                                    uint64_t vb_base, uint32_t* __restrict__ first_bad) {
  wire_prio();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t m = t / SLAB, k = t % SLAB;
  if (m >= nm) return;
  const uint64_t vb = vote_begin[m];
  if (k == 0) {
    pout[m].vote_begin = vb_base + vb;
    if (first_bad) first_bad[m] = 0xFFFFFFFFu;  // (k_wire_votes' atomicMin target, reset here)
  }
  const uint64_t nv = vote_count[m];
  if (nv > SLAB || k >= nv) return;  // > SLAB: k_wire_walk mode 1 writes them all
  vrec_off[vb + k] = slab_off[t];
  vrec_len[vb + k] = slab_len[t];
  vrec_msg[vb + k] = (uint32_t)m;
}

constexpr int VOTE_WIN = 48 * 1024;  // LDS staging of a block's vote records

// The block's record span [s_lo, s_hi) staged into LDS (a contiguous span of at most VOTE_WIN bytes;
// scattered records are read from global memory).  Every thread calls it (it has barriers).
__device__ __forceinline__ WinSrc stage_records(uint8_t* win, unsigned long long& s_lo, unsigned long long& s_hi,
                                                const uint8_t* __restrict__ wire, int aligned, bool have,
                                                uint64_t pos, uint64_t vend) {
  if (threadIdx.x == 0) {
    s_lo = ~0ull;
    s_hi = 0;
  }
  __syncthreads();
  if (have) {
    atomicMin(&s_lo, (unsigned long long)pos);
    atomicMax(&s_hi, (unsigned long long)vend);
  }
  __syncthreads();
  const uint64_t wlo = s_lo & ~15ull;
  uint64_t wlen = s_hi > wlo ? s_hi - wlo : 0;
  if (wlen > VOTE_WIN) wlen = 0;
  if (wlen) load_window(win, wire, wlo, wlo + wlen, aligned != 0);
  __syncthreads();
  return WinSrc{wire, (lds_bytes)win, wlo, wlen};
}

// One Vote record (prost message::merge -> merge_loop, consensus.proto:19-29): fields are read from the
// enclosing message (bounded by its end `end`) and the loop must stop exactly at the record's end `vend`
// ("delimited length exceeded").  Vote i of the SoA gets the decoded fields; returns the prost error.
__device__ __forceinline__ int decode_vote(const WinSrc& src, const uint8_t* __restrict__ wire, uint64_t pos,
                                           uint64_t vend, uint64_t end, uint64_t i, uint32_t* vote_id,
                                           uint32_t* proposal_id, uint64_t* timestamp, uint8_t* vote,
                                           uint64_t* field_off, uint32_t* field_len) {
  uint32_t vid = 0, pid = 0;
  uint64_t ts = 0;
  uint8_t vt = 0;
  uint64_t foff[HLC_NFIELDS] = {0, 0, 0, 0, 0};
  uint32_t flen[HLC_NFIELDS] = {0, 0, 0, 0, 0};
  int err = HLC_WIRE_OK;
  while (pos < vend) {
    uint32_t tag;
    int wt;
    if ((err = rd_key(src, pos, end, tag, wt))) break;
    if (tag >= 20 && tag <= 28) {
      const bool is_len = tag == 21 || tag >= 25;
      if (wt != (is_len ? WT_LEN : WT_VARINT)) {
        err = HLC_WIRE_WIRE_TYPE_MISMATCH;
        break;
      }
      if (is_len) {
        const int f = tag == 21 ? HLC_F_OWNER : (int)(tag - 25) + HLC_F_PARENT;
        if ((err = rd_len(src, pos, end, foff[f], flen[f]))) break;
      } else {
        uint64_t v;
        if ((err = rd_varint(src, pos, end, v))) break;
        if (tag == 20) vid = (uint32_t)v;
        else if (tag == 22) pid = (uint32_t)v;
        else if (tag == 23) ts = v;
        else vt = v != 0;
      }
    } else if ((err = skip_field(wire, pos, end, wt, tag, RECURSION_LIMIT - 1))) {
      break;
    }
  }
  if (!err && pos != vend) err = HLC_WIRE_DELIMITED_EXCEEDED;
  vote_id[i] = vid;
  proposal_id[i] = pid;
  timestamp[i] = ts;
  vote[i] = vt;
#pragma unroll
  for (int f = 0; f < HLC_NFIELDS; ++f) {
    field_off[i * HLC_NFIELDS + f] = foff[f];
    field_len[i * HLC_NFIELDS + f] = flen[f];
  }
  return err;
}

// One Vote record per lane, records in place (vrec_*).  The block's records -- contiguous in the wire
// for the usual layout -- are staged in LDS first; reads outside the staged span go to global.
__global__ void __launch_bounds__(TPB) k_wire_votes(const uint8_t* __restrict__ wire, int aligned,
                                                    const uint64_t* __restrict__ msg_off,
                                                    const uint32_t* __restrict__ msg_len, uint64_t nv,
                                                    const uint64_t* __restrict__ vrec_off,
                                                    const uint32_t* __restrict__ vrec_len,
                                                    const uint32_t* __restrict__ vrec_msg,
                                                    const uint64_t* __restrict__ vote_begin, uint32_t* vote_id,
                                                    uint32_t* proposal_id, uint64_t* timestamp, uint8_t* vote,
                                                    uint64_t* field_off, uint32_t* field_len,
                                                    uint8_t* __restrict__ vote_err, uint32_t* __restrict__ first_bad) {
  wire_prio();
  __shared__ __attribute__((aligned(16))) uint8_t win[VOTE_WIN];
  __shared__ unsigned long long s_lo, s_hi;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool have = i < nv;
  const uint64_t pos = have ? vrec_off[i] : 0, vend = have ? pos + vrec_len[i] : 0;
  const WinSrc src = stage_records(win, s_lo, s_hi, wire, aligned, have, pos, vend);
  if (!have) return;
  const uint32_t m = vrec_msg[i];
  const int err = decode_vote(src, wire, pos, vend, msg_off[m] + msg_len[m], i, vote_id, proposal_id, timestamp, vote,
                              field_off, field_len);
  vote_err[i] = (uint8_t)err;
  if (err) atomicMin(first_bad + m, (uint32_t)(i - vote_begin[m]));
}

// k_wire_place and k_wire_votes in one kernel, for a message range whose messages all have at most SLAB
// vote records (the walker kept every record in its slab): one lane per (message, slab slot), records
// read straight from the slab, vote i = vote_begin[m] + slot.  The wire host entry's per-range decode,
// where every kernel on the chain to the range's recovery waits its turn behind the running grids.
// first_bad[m] was reset by the walker.
__global__ void __launch_bounds__(TPB) k_wire_votes_slab(const uint8_t* __restrict__ wire, int aligned,
                                                         const uint64_t* __restrict__ msg_off,
                                                         const uint32_t* __restrict__ msg_len, uint64_t nm,
                                                         const uint64_t* __restrict__ vote_count,
                                                         const uint64_t* __restrict__ vote_begin,
                                                         const uint64_t* __restrict__ slab_off,
                                                         const uint32_t* __restrict__ slab_len,
                                                         hlc_proposal* __restrict__ pout, uint64_t vb_base,
                                                         uint32_t* vote_id, uint32_t* proposal_id, uint64_t* timestamp,
                                                         uint8_t* vote, uint64_t* field_off, uint32_t* field_len,
                                                         uint8_t* __restrict__ vote_err,
                                                         uint32_t* __restrict__ first_bad) {
  wire_prio();
  __shared__ __attribute__((aligned(16))) uint8_t win[VOTE_WIN];
  __shared__ unsigned long long s_lo, s_hi;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t m = t / SLAB, k = t % SLAB;
  const bool inm = m < nm;
  const bool have = inm && k < vote_count[m];
  if (inm && k == 0) pout[m].vote_begin = vb_base + vote_begin[m];
  const uint64_t pos = have ? slab_off[t] : 0, vend = have ? pos + slab_len[t] : 0;
  const WinSrc src = stage_records(win, s_lo, s_hi, wire, aligned, have, pos, vend);
  if (!have) return;
  const uint64_t i = vote_begin[m] + k;
  const int err = decode_vote(src, wire, pos, vend, msg_off[m] + msg_len[m], i, vote_id, proposal_id, timestamp, vote,
                              field_off, field_len);
  vote_err[i] = (uint8_t)err;
  if (err) atomicMin(first_bad + m, (uint32_t)k);
}

// First error in stream order: a failing vote record precedes every later top-level error.
// Messages that fail keep vote_count 0 in their hlc_proposal (validation skips their votes).
__global__ void __launch_bounds__(TPB) k_wire_final(uint64_t nm, const uint64_t* __restrict__ vote_begin,
                                                    const uint8_t* __restrict__ vote_err,
                                                    const uint32_t* __restrict__ first_bad,
                                                    hlc_wire_proposal* __restrict__ wout,
                                                    hlc_proposal* __restrict__ pout) {
  wire_prio();
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const uint32_t fb = first_bad[m];
  uint8_t st = wout[m].decode_status;
  if (fb != 0xFFFFFFFFu) {
    st = vote_err[vote_begin[m] + fb];
    wout[m].bad_vote = fb;
  }
  wout[m].decode_status = st;
  if (st != HLC_WIRE_OK) pout[m].vote_count = 0;
}

// validate-many results of messages that failed to decode
__global__ void __launch_bounds__(TPB) k_wire_results(uint64_t nm, const hlc_wire_proposal* __restrict__ wout,
                                                      hlc_result* __restrict__ res) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const hlc_wire_proposal w = wout[m];
  if (w.decode_status == HLC_WIRE_OK) return;
  hlc_result r;
  r.status = HLC_PROPOSAL_DECODE_ERROR;
  r.transition = HLC_STILL_ACTIVE;
  r.scheme_reason = w.decode_status;
  r._pad = 0;
  r.bad_index = w.bad_vote;
  r.yes = 0;
  r.total = 0;
  res[m] = r;
}

// The wire host entry's per-range scan + read-back, one block: vote_begin = the exclusive scan of the
// range's vote counts; out[0] = the range's vote total, out[1] = 1 when a message has more records than
// the walker's slab (its second walk is needed).  `out` is page-locked host memory mapped for the
// device, written with system-scope stores: the host reads it once the event behind this kernel has
// fired -- one kernel instead of a flag memset, a two-kernel library scan and a device-to-host copy,
// each of which waits its turn behind the recovery grids when the device is busy.
constexpr int RS_TPB = 1024;
__global__ void __launch_bounds__(RS_TPB) k_wire_range_scan(const uint64_t* __restrict__ vote_count,
                                                            uint64_t* __restrict__ vote_begin, uint64_t nm,
                                                            uint64_t* out) {
  wire_prio();
  __shared__ uint64_t part[RS_TPB];
  __shared__ uint64_t carry_s;
  __shared__ uint32_t big_s;
  if (threadIdx.x == 0) {
    carry_s = 0;
    big_s = 0;
  }
  __syncthreads();
  for (uint64_t b0 = 0; b0 < nm; b0 += RS_TPB) {
    const uint64_t m = b0 + threadIdx.x;
    const uint64_t v = m < nm ? vote_count[m] : 0;
    if (v > SLAB) big_s = 1;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < RS_TPB; d <<= 1) {  // inclusive Hillis-Steele scan of the block's counts
      const uint64_t x = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += x;
      __syncthreads();
    }
    const uint64_t c = carry_s;
    if (m < nm) vote_begin[m] = c + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == RS_TPB - 1) carry_s = c + part[RS_TPB - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(out, carry_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out + 1, (uint64_t)big_s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

}  // namespace

static int is_aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// the mode-0 walker (HLC_OPT_WIRE_WALK: 1 = k_wire_walk_lds, 0 = k_wire_walk, -1 = the default below)
static bool walk_lds(int walk) { return walk < 0 ? WIRE_WALK_LDS_DEFAULT : walk != 0; }

void launch_wire_walk(int mode, const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nm,
                      uint64_t* vote_count, const uint64_t* vote_begin, hlc_wire_proposal* wout, hlc_proposal* pout,
                      const hlc_scope_config* scope, uint64_t n_scope, uint64_t* slab_off, uint32_t* slab_len,
                      uint32_t* big, uint64_t* vrec_off, uint32_t* vrec_len, uint32_t* vrec_msg, uint64_t* huge,
                      hipStream_t s, uint32_t* first_bad, int walk) {
  if (!nm) return;
  if (mode == 0 && walk_lds(walk)) {
    hipLaunchKernelGGL(k_wire_walk_lds, dim3((unsigned)((nm + LW_MPW - 1) / LW_MPW)), dim3(64), 0, s, wire,
                       is_aligned16(wire), msg_off, msg_len, nm, vote_count, wout, pout, scope, n_scope, slab_off,
                       slab_len, big, huge, first_bad);
    return;
  }
  hipLaunchKernelGGL(k_wire_walk, dim3((unsigned)((nm + WALK_TPB - 1) / WALK_TPB)), dim3(WALK_TPB), 0, s, mode, wire, is_aligned16(wire), msg_off,
                     msg_len, nm,
                     vote_count, vote_begin, wout, pout, scope, n_scope, slab_off, slab_len, big, vrec_off,
                     vrec_len, vrec_msg, huge, first_bad);
}

uint64_t wire_huge_threshold() { return HUGE_MSG; }

int launch_huge_decode(const uint8_t* wire, uint64_t m, uint64_t base, uint32_t len, uint32_t* next, uint32_t* jump,
                       uint32_t* save, uint8_t* mark, uint32_t* st, uint32_t* flag, uint32_t* rank, void* scan_tmp,
                       size_t scan_bytes, uint64_t* hoff, uint32_t* hlen, uint64_t* vote_count,
                       hlc_wire_proposal* wout, hlc_proposal* pout, const hlc_scope_config* scope, uint64_t n_scope,
                       hipStream_t s) {
#define HUGE_CHK(x)                     \
  do {                                  \
    if ((x) != hipSuccess) return -1;   \
  } while (0)
  const unsigned g = (unsigned)std::min<uint64_t>(((uint64_t)len + TPB) / TPB, 8192);
  HUGE_CHK(hipMemsetAsync(mark, 0, (size_t)len + 1, s));
  HUGE_CHK(hipMemsetAsync(mark, 1, 1, s));
  hipLaunchKernelGGL(k_huge_next, dim3(g), dim3(TPB), 0, s, wire, base, len, next);
  HUGE_CHK(hipMemcpyAsync(save, next, ((size_t)len + 1) * 4, hipMemcpyDeviceToDevice, s));  // the rounds consume it
  auto rounds = [&](const uint32_t* active) {
    uint32_t* a = next;
    uint32_t* b = jump;
    for (uint64_t reach = 1; reach <= len; reach <<= 1) {  // after the round, steps < 2 * reach are marked
      hipLaunchKernelGGL(k_huge_round, dim3(g), dim3(TPB), 0, s, a, b, mark, len, active);
      std::swap(a, b);
    }
  };
  rounds(nullptr);
  // A top-level group longer than the bounded skip stops the chain.  Up to HUGE_RESUME_PASSES times:
  // one lane resolves the first such offset, and a fresh set of rounds (skipped on the device when
  // there was nothing to resolve) resumes the parallel marking past it -- a long group at the head
  // of a message no longer hands the rest of it to one lane.  Then one lane finishes whatever is
  // left (linear).
  for (int pass = 0; pass < HUGE_RESUME_PASSES; ++pass) {
    HUGE_CHK(hipMemsetAsync(st + 11, 0xFF, 4, s));
    hipLaunchKernelGGL(k_huge_unres, dim3(g), dim3(TPB), 0, s, len, save, mark, st);
    hipLaunchKernelGGL(k_huge_resolve, dim3(1), dim3(64), 0, s, wire, base, len, save, st);
    hipLaunchKernelGGL(k_huge_copy_if, dim3(g), dim3(TPB), 0, s, save, next, len, st);
    rounds(st + 12);
  }
  HUGE_CHK(hipMemsetAsync(st + 11, 0xFF, 4, s));
  hipLaunchKernelGGL(k_huge_unres, dim3(g), dim3(TPB), 0, s, len, save, mark, st);
  hipLaunchKernelGGL(k_huge_tail, dim3(1), dim3(64), 0, s, wire, base, len, save, mark, st);
  HUGE_CHK(hipMemsetAsync(st, 0, 11 * 4, s));  // st[11] is the unresolved slot
  HUGE_CHK(hipMemsetAsync(st, 0xFF, 4, s));
  hipLaunchKernelGGL(k_huge_first_error, dim3(g), dim3(TPB), 0, s, wire, base, len, save, mark, st);
  hipLaunchKernelGGL(k_huge_fields, dim3(g), dim3(TPB), 0, s, wire, base, len, save, mark, st, flag);
  HUGE_CHK(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, flag, rank, (int)(len + 1), s));
  hipLaunchKernelGGL(k_huge_records, dim3(g), dim3(TPB), 0, s, wire, base, len, flag, rank, hoff, hlen);
  hipLaunchKernelGGL(k_huge_emit, dim3(1), dim3(64), 0, s, wire, m, base, len, save, st, rank, vote_count, wout, pout,
                     scope, n_scope);
  HUGE_CHK(hipGetLastError());
#undef HUGE_CHK
  return 0;
}

size_t huge_scan_bytes(uint32_t len) {
  size_t tb = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)(len + 1));
  return tb;
}

void launch_huge_place(uint64_t m, const uint64_t* vote_count, const uint64_t* vote_begin, const uint64_t* hoff,
                       const uint32_t* hlen, uint64_t* vrec_off, uint32_t* vrec_len, uint32_t* vrec_msg,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_huge_place, dim3(2048), dim3(TPB), 0, s, m, vote_count, vote_begin, hoff, hlen, vrec_off,
                     vrec_len, vrec_msg);
}

void launch_wire_place(uint64_t nm, const uint64_t* vote_count, const uint64_t* vote_begin, const uint64_t* slab_off,
                       const uint32_t* slab_len, hlc_proposal* pout, uint64_t* vrec_off, uint32_t* vrec_len,
                       uint32_t* vrec_msg, hipStream_t s, uint64_t vb_base, uint32_t* first_bad) {
  if (!nm) return;
  hipLaunchKernelGGL(k_wire_place, dim3(blocks_for(nm * SLAB)), dim3(TPB), 0, s, nm, vote_count, vote_begin, slab_off,
                     slab_len, pout, vrec_off, vrec_len, vrec_msg, vb_base, first_bad);
}

uint64_t wire_slab() { return SLAB; }

void launch_wire_range_scan(const uint64_t* vote_count, uint64_t* vote_begin, uint64_t nm, uint64_t* out_mapped,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_wire_range_scan, dim3(1), dim3(RS_TPB), 0, s, vote_count, vote_begin, nm, out_mapped);
}

void launch_wire_touch(const uint8_t* wire, uint64_t len, uint32_t* sink, hipStream_t s) {
  if (len < 16 || !is_aligned16(wire)) return;
  hipLaunchKernelGGL(k_wire_touch, dim3(2048), dim3(TPB), 0, s, wire, len, sink);
}

void launch_wire_votes(const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nv,
                       const uint64_t* vrec_off, const uint32_t* vrec_len, const uint32_t* vrec_msg,
                       const uint64_t* vote_begin, const hlc_votes* out, uint8_t* vote_err, uint32_t* first_bad,
                       hipStream_t s) {
  if (!nv) return;
  hipLaunchKernelGGL(k_wire_votes, dim3(blocks_for(nv)), dim3(TPB), 0, s, wire, is_aligned16(wire), msg_off, msg_len,
                     nv, vrec_off, vrec_len, vrec_msg, vote_begin, const_cast<uint32_t*>(out->vote_id),
                     const_cast<uint32_t*>(out->proposal_id), const_cast<uint64_t*>(out->timestamp),
                     const_cast<uint8_t*>(out->vote), const_cast<uint64_t*>(out->field_off),
                     const_cast<uint32_t*>(out->field_len), vote_err, first_bad);
}

void launch_wire_votes_slab(const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nm,
                            const uint64_t* vote_count, const uint64_t* vote_begin, const uint64_t* slab_off,
                            const uint32_t* slab_len, hlc_proposal* pout, uint64_t vb_base, const hlc_votes* out,
                            uint8_t* vote_err, uint32_t* first_bad, hipStream_t s) {
  if (!nm) return;
  hipLaunchKernelGGL(k_wire_votes_slab, dim3(blocks_for(nm * SLAB)), dim3(TPB), 0, s, wire, is_aligned16(wire), msg_off,
                     msg_len, nm, vote_count, vote_begin, slab_off, slab_len, pout, vb_base,
                     const_cast<uint32_t*>(out->vote_id), const_cast<uint32_t*>(out->proposal_id),
                     const_cast<uint64_t*>(out->timestamp), const_cast<uint8_t*>(out->vote),
                     const_cast<uint64_t*>(out->field_off), const_cast<uint32_t*>(out->field_len), vote_err, first_bad);
}

void launch_wire_final(uint64_t nm, const uint64_t* vote_begin, const uint8_t* vote_err, const uint32_t* first_bad,
                       hlc_wire_proposal* wout, hlc_proposal* pout, hipStream_t s) {
  if (!nm) return;
  hipLaunchKernelGGL(k_wire_final, dim3(blocks_for(nm)), dim3(TPB), 0, s, nm, vote_begin, vote_err, first_bad,
                     wout, pout);
}

void launch_wire_results(uint64_t nm, const hlc_wire_proposal* wout, hlc_result* res, hipStream_t s) {
  if (!nm) return;
  hipLaunchKernelGGL(k_wire_results, dim3(blocks_for(nm)), dim3(TPB), 0, s, nm, wout, res);
}

}  // namespace hlc
