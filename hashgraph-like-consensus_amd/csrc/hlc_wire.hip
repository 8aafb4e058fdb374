// hlc_wire.hip -- device decoder for gossip-format Proposal messages.
//
// The reference hands prost-decoded `Proposal`s (consensus.proto:5-29) to
// `ConsensusService::process_incoming_proposal` (service.rs:263-279); decoding is prost 0.14's
// `Message::decode` (restated in oracle/wire_oracle.py).  This file performs that decode on the
// GPU so raw wire bytes go straight to the validate-many pipeline, with bit-identical outcomes:
//   k_wire_walk   (one lane per message)  top-level fields of the Proposal: scalars, name
//                                          (UTF-8 checked), payload, owner, and the extents of
//                                          every `votes` record; pass 0 counts, pass 1 writes
//   hipcub scan of the per-message vote counts -> vote_begin
//   k_wire_votes  (one lane per vote)      decodes one Vote record into the hlc_votes SoA;
//                                          bytes fields are (offset, length) into the wire
//                                          buffer itself -- no copy
//   k_wire_final  (one lane per message)   first error in stream order, hlc_proposal records
// All integer/byte work, latency-bound on dependent varint reads.
#include <hipcub/hipcub.hpp>

#include "hlc_kernels.h"

namespace hlc {

namespace {

constexpr int TPB = 256;
constexpr int RECURSION_LIMIT = 100;  // prost DecodeContext default
constexpr int GROUP_STACK = RECURSION_LIMIT + 1;

enum : int { WT_VARINT = 0, WT_I64 = 1, WT_LEN = 2, WT_SGROUP = 3, WT_EGROUP = 4, WT_I32 = 5 };

// prost decode_varint: <= 10 bytes, the 10th must be < 2; out of bytes = invalid varint.
__device__ __forceinline__ int rd_varint(const uint8_t* __restrict__ b, uint64_t& pos, uint64_t end,
                                         uint64_t& v) {
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
__device__ __forceinline__ int rd_key(const uint8_t* __restrict__ b, uint64_t& pos, uint64_t end, uint32_t& tag,
                                      int& wt) {
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
__device__ __forceinline__ int rd_len(const uint8_t* __restrict__ b, uint64_t& pos, uint64_t end, uint64_t& off,
                                      uint32_t& len) {
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
__device__ __forceinline__ int skip_scalar(const uint8_t* __restrict__ b, uint64_t& pos, uint64_t end, int wt) {
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
__device__ __noinline__ int skip_field(const uint8_t* __restrict__ b, uint64_t& pos, uint64_t end, int wt,
                                       uint32_t tag, int budget) {
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
__device__ bool utf8_ok(const uint8_t* __restrict__ p, uint32_t n) {
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

// Top-level walk of message m (prost Proposal::merge_field, generated from consensus.proto:5-16).
// Pass 0: counts the votes records (vote_count[m]).
// Pass 1: writes each vote record's (content offset, content length, message) at vote_begin[m] + k,
// the message's hlc_wire_proposal (walker error) and its hlc_proposal.
__global__ void __launch_bounds__(TPB) k_wire_walk(int pass, const uint8_t* __restrict__ wire,
                                                   const uint64_t* __restrict__ msg_off,
                                                   const uint32_t* __restrict__ msg_len, uint64_t nm,
                                                   uint64_t* __restrict__ vote_count,
                                                   const uint64_t* __restrict__ vote_begin,
                                                   hlc_wire_proposal* __restrict__ wout,
                                                   hlc_proposal* __restrict__ pout, const hlc_scope_config* scope,
                                                   uint64_t n_scope, uint64_t* __restrict__ vrec_off,
                                                   uint32_t* __restrict__ vrec_len, uint32_t* __restrict__ vrec_msg) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const uint64_t base = msg_off[m];
  uint64_t pos = base;
  const uint64_t end = base + msg_len[m];
  WalkOut o = {};
  uint64_t nv = 0;
  uint64_t vb = pass ? vote_begin[m] : 0;
  int err = HLC_WIRE_OK;
  while (pos < end) {
    uint32_t tag;
    int wt;
    if ((err = rd_key(wire, pos, end, tag, wt))) break;
    uint64_t v = 0, off = 0;
    uint32_t len = 0;
    if (tag >= 10 && tag <= 19) {
      const bool is_len = tag == 10 || tag == 11 || tag == 13 || tag == 14;
      if (wt != (is_len ? WT_LEN : WT_VARINT)) {
        err = HLC_WIRE_WIRE_TYPE_MISMATCH;
        break;
      }
      if (is_len) {
        if ((err = rd_len(wire, pos, end, off, len))) break;
      } else {
        if ((err = rd_varint(wire, pos, end, v))) break;
      }
    }
    switch (tag) {
      case 10:
        if (!utf8_ok(wire + off, len)) err = HLC_WIRE_INVALID_UTF8;
        o.name_off = off - base;
        o.name_len = len;
        break;
      case 11: o.payload_off = off - base; o.payload_len = len; break;
      case 12: o.proposal_id = (uint32_t)v; break;
      case 13: o.owner_off = off - base; o.owner_len = len; break;
      case 14:
        if (pass) {
          vrec_off[vb + nv] = off;
          vrec_len[vb + nv] = len;
          vrec_msg[vb + nv] = (uint32_t)m;
        }
        ++nv;
        break;
      case 15: o.expected_voters = (uint32_t)v; break;
      case 16: o.round = (uint32_t)v; break;
      case 17: o.timestamp = v; break;
      case 18: o.expiration = v; break;
      case 19: o.liveness = v != 0; break;
      default: err = skip_field(wire, pos, end, wt, tag, RECURSION_LIMIT); break;
    }
    if (err) break;
  }
  if (!pass) {
    vote_count[m] = nv;
    return;
  }
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
  p.vote_begin = vb;
  p.vote_count = (uint32_t)nv;
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

// One Vote record (prost message::merge -> merge_loop, consensus.proto:19-29): fields are read
// from the enclosing message (bounded by its end), and the loop must stop exactly at the
// record's end ("delimited length exceeded").
__global__ void __launch_bounds__(TPB) k_wire_votes(const uint8_t* __restrict__ wire,
                                                    const uint64_t* __restrict__ msg_off,
                                                    const uint32_t* __restrict__ msg_len, uint64_t nv,
                                                    const uint64_t* __restrict__ vrec_off,
                                                    const uint32_t* __restrict__ vrec_len,
                                                    const uint32_t* __restrict__ vrec_msg,
                                                    const uint64_t* __restrict__ vote_begin, uint32_t* vote_id,
                                                    uint32_t* proposal_id, uint64_t* timestamp, uint8_t* vote,
                                                    uint64_t* field_off, uint32_t* field_len,
                                                    uint8_t* __restrict__ vote_err, uint32_t* __restrict__ first_bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nv) return;
  const uint32_t m = vrec_msg[i];
  const uint64_t end = msg_off[m] + msg_len[m];
  uint64_t pos = vrec_off[i];
  const uint64_t vend = pos + vrec_len[i];
  uint32_t vid = 0, pid = 0;
  uint64_t ts = 0;
  uint8_t vt = 0;
  uint64_t foff[HLC_NFIELDS] = {0, 0, 0, 0, 0};
  uint32_t flen[HLC_NFIELDS] = {0, 0, 0, 0, 0};
  int err = HLC_WIRE_OK;
  while (pos < vend) {
    uint32_t tag;
    int wt;
    if ((err = rd_key(wire, pos, end, tag, wt))) break;
    if (tag >= 20 && tag <= 28) {
      const bool is_len = tag == 21 || tag >= 25;
      if (wt != (is_len ? WT_LEN : WT_VARINT)) {
        err = HLC_WIRE_WIRE_TYPE_MISMATCH;
        break;
      }
      if (is_len) {
        const int f = tag == 21 ? HLC_F_OWNER : (int)(tag - 25) + HLC_F_PARENT;
        if ((err = rd_len(wire, pos, end, foff[f], flen[f]))) break;
      } else {
        uint64_t v;
        if ((err = rd_varint(wire, pos, end, v))) break;
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
  vote_err[i] = (uint8_t)err;
  if (err) atomicMin(first_bad + m, (uint32_t)(i - vote_begin[m]));
}

// First error in stream order: a failing vote record precedes every later top-level error.
// Messages that fail keep vote_count 0 in their hlc_proposal (validation skips their votes).
__global__ void __launch_bounds__(TPB) k_wire_final(uint64_t nm, const uint64_t* __restrict__ vote_begin,
                                                    const uint8_t* __restrict__ vote_err,
                                                    const uint32_t* __restrict__ first_bad,
                                                    hlc_wire_proposal* __restrict__ wout,
                                                    hlc_proposal* __restrict__ pout) {
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

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

}  // namespace

void launch_wire_walk(int pass, const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nm,
                      uint64_t* vote_count, const uint64_t* vote_begin, hlc_wire_proposal* wout,
                      hlc_proposal* pout, const hlc_scope_config* scope, uint64_t n_scope, uint64_t* vrec_off,
                      uint32_t* vrec_len, uint32_t* vrec_msg, hipStream_t s) {
  if (!nm) return;
  hipLaunchKernelGGL(k_wire_walk, dim3(blocks_for(nm)), dim3(TPB), 0, s, pass, wire, msg_off, msg_len, nm,
                     vote_count, vote_begin, wout, pout, scope, n_scope, vrec_off, vrec_len, vrec_msg);
}

void launch_wire_votes(const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nv,
                       const uint64_t* vrec_off, const uint32_t* vrec_len, const uint32_t* vrec_msg,
                       const uint64_t* vote_begin, const hlc_votes* out, uint8_t* vote_err, uint32_t* first_bad,
                       hipStream_t s) {
  if (!nv) return;
  hipLaunchKernelGGL(k_wire_votes, dim3(blocks_for(nv)), dim3(TPB), 0, s, wire, msg_off, msg_len, nv, vrec_off,
                     vrec_len, vrec_msg, vote_begin, const_cast<uint32_t*>(out->vote_id),
                     const_cast<uint32_t*>(out->proposal_id), const_cast<uint64_t*>(out->timestamp),
                     const_cast<uint8_t*>(out->vote), const_cast<uint64_t*>(out->field_off),
                     const_cast<uint32_t*>(out->field_len), vote_err, first_bad);
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
