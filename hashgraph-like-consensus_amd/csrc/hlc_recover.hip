// hlc_recover.hip -- the VALU-bound kernels: batch ecrecover (the hot path),
// table construction, and the signing side (address derivation, RFC 6979 signing).
#include "hlc_kernels.h"
#include "hlc_recover.hpp"
#include "hlc_sign.hpp"

namespace hlc {

namespace {

#ifndef HLC_REC_TPB
#define HLC_REC_TPB 256
#endif
constexpr int REC_TPB = HLC_REC_TPB;  // k_rec_main block size
#ifndef HLC_REC_MIN_WAVES
// __launch_bounds__ minimum waves per SIMD for k_rec_main: a ceiling on the registers the allocator
// may take (512 / waves, in steps of 8).  At 2 the allocator takes 174 VGPRs (no spills) and the
// kernel RUNS at 2 waves per SIMD; a floor of 3 fits 168 VGPRs with two 8-byte spills outside the
// chains.  Round 3 (one-reduction sums of products, bitop3 hashes): 2 waves beat 3 by 2.0% on one
// box (profiles/r03/ab_occupancy_r03.txt) -- 131k lanes' R tables (239 MB) fit the 256 MB Infinity
// Cache, 197k lanes' (358 MB) do not.  In round 2, before those changes, 3 beat a grid capped at 2
// by 5-6% (profiles/r02_ab_main_waves_split.txt).  The grid is sized from the occupancy API
// (recover_grid_lanes), so it follows whatever the build reaches.
#define HLC_REC_MIN_WAVES 2
#endif

// ---- prep: parse + batched r^-1 + scalars (REC_BATCH votes per lane, one safegcd) ----
// Lane t owns votes t + k * L (k < REC_BATCH): a wave reads 64 consecutive votes per k.
// Forward: acc_k = mont(acc_{k-1}, r_k) = (prod r) R^-k over the lane's valid votes, each acc_{k-1}
// kept in `pfx`; one inversion cur = acc^-1; backward: r_k^-1 = mont(acc_{k-1}, cur),
// cur = mont(cur, r_k).  The stage reads the signatures (and, in validate-many, the checks that
// precede the signature in validate_vote) while the prehash kernels run on the launch stream
// (hlc_api.cpp vote_stage).  It decides every vote that needs no recovery -- no 65-byte signature, a
// v / r / s the scheme rejects, or (skip != nullptr) a vote the pre-checks reject whatever its
// signature -- writing its k_rec_main state byte, and appends the others to the work list that
// k_rec_main's waves take their votes from (in runs of up to 64 consecutive votes).
constexpr int PREP_TPB = 64;
#ifndef HLC_PREP_PRIO
#define HLC_PREP_PRIO 2  // k_rec_prep's wave issue priority (s_setprio; 0 = the default, 0)
#endif
constexpr uint32_t PREP_SKIP = 0xFFu;  // record flags bits 8-15: no 65-byte signature, not parsed
// k_rec_main -> k_rec_comb, one byte per vote: u2 R finite / at infinity / nothing to recover, or
// 1 + the scheme code (prep's v / r / s checks, or no point R)
constexpr uint8_t MST_OK = 0x00, MST_INF = 0xFE, MST_SKIP = 0xFF;

// Vote i's signature: bytes + sig_off[i * off_stride], or (sig_off == nullptr) the dense array the
// host-buffer entry uploads ahead of the other inputs, 65 bytes per vote at bytes + 65 i.
HLC_DEV const uint8_t* sig_at(const uint8_t* bytes, const uint64_t* sig_off, size_t off_stride, uint64_t i) {
  return sig_off ? bytes + sig_off[i * off_stride] : bytes + 65 * i;
}

HLC_DEV bool prep_sig(const uint8_t* bytes, const uint64_t* sig_off, size_t off_stride, const uint32_t* sig_len,
                      size_t len_stride, uint64_t i, fe& r, fe& s, int& parity, int& code) {
  if (sig_len[i * len_stride] != 65u) return false;  // rejected by the pre-checks (length)
  const uint8_t* sig = sig_at(bytes, sig_off, off_stride, i);
  fe_load_be(r, sig);
  fe_load_be(s, sig + 32);
  code = rec_parse(s, r, sig[64], parity);
  return true;
}

// The checks validate_proposal / validate_vote make before the signature (utils.rs:113-115 proposal_id
// match, 133-140 empty owner / vote_hash; the empty signature is a length skip already), and votes no
// proposal covers: such a vote's status never depends on its recovery (k_prehash_fused decides it
// from the same fields), so k_rec_main does not run its u2 R chain.
#ifndef HLC_PRE_SKIP
#define HLC_PRE_SKIP 1  // 0: A/B arm without the skip (every parsed signature runs the chain)
#endif
HLC_DEV bool pre_rejected(const RecSkip& k, uint64_t i) {
  if (!HLC_PRE_SKIP || !k.vote_prop) return false;
  const uint32_t p = k.vote_prop[i];
  if (p == NO_PROP) return true;
  if (k.proposal_id[i] != k.props[p].proposal_id) return true;
  const uint32_t* fl = k.field_len + i * HLC_NFIELDS;
  return fl[HLC_F_OWNER] == 0 || fl[HLC_F_VOTE_HASH] == 0;
}

#ifndef HLC_PREP_LOADS
#define HLC_PREP_LOADS 0  // A/B knob: k_rec_prep's per-vote loads in three round trips (see prep_vote); 2: also
                          // the backward pass's reload in two
#endif
// The forward pass's per-vote inputs in three memory round trips: every word that depends only on i
// (vote_prop, proposal_id, the owner / vote_hash lengths, the signature's length and offset) is
// issued before any is used, then the covering proposal's id, then the signature bytes (read only
// for a vote the checks pass).  pre_rejected + prep_sig waited on each load in turn (seven round
// trips per vote, eight votes per lane, at ~1.2 waves/SIMD: the PMC pass shows k_rec_prep's waves
// waiting on memory 43% of their cycles).  Same outcome as !pre_rejected && prep_sig.
HLC_DEV bool prep_vote(const RecSkip& k, const uint8_t* bytes, const uint64_t* sig_off, size_t off_stride,
                       const uint32_t* sig_len, size_t len_stride, uint64_t i, fe& r, fe& s, int& parity, int& code) {
  const bool skip = HLC_PRE_SKIP && k.vote_prop;
  const uint32_t slen = sig_len[i * len_stride];
  const uint64_t soff = sig_off ? sig_off[i * off_stride] : 65 * i;
  uint32_t p = 0, vpid = 0, flo = 1, flh = 1;
  if (skip) {
    const uint32_t* fl = k.field_len + i * HLC_NFIELDS;
    p = k.vote_prop[i];
    vpid = k.proposal_id[i];
    flo = fl[HLC_F_OWNER];
    flh = fl[HLC_F_VOTE_HASH];
  }
  if (skip && (p == NO_PROP || flo == 0 || flh == 0 || vpid != k.props[p].proposal_id)) return false;
  if (slen != 65u) return false;
  const uint8_t* sig = bytes + soff;  // read only for a vote the checks pass, as prep_sig
  fe_load_be(r, sig);
  fe_load_be(s, sig + 32);
  code = rec_parse(s, r, sig[64], parity);
  return true;
}

// n votes; records rec / mst of vote i at rec + i (stride `st` words between a record's rows), mst[i].
__global__ void __launch_bounds__(PREP_TPB) k_rec_prep(uint64_t n, uint64_t st, uint64_t L, const uint8_t* bytes,
                                                       const uint64_t* sig_off, size_t off_stride,
                                                       const uint32_t* sig_len, size_t len_stride, uint32_t* rec,
                                                       uint32_t* pfx, uint8_t* mst, uint32_t* list,
                                                       unsigned long long* list_len, RecSkip sk) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  // a few long dependent chains per lane at low occupancy: when it shares the SIMDs with a k_rec_main
  // grid (host-buffer ranges: the next range's prep beside this range's main), the arbiter serves its
  // waves first -- measured without this, a 196k-vote prep took 1.18 ms beside a main vs 0.25 alone
#if HLC_PREP_PRIO
  __builtin_amdgcn_s_setprio(HLC_PREP_PRIO);
#endif
  fe acc;
  fe_set(acc, 1);
  uint32_t active = 0;  // bit k: vote t + k L goes to k_rec_main
#pragma unroll 1
  for (int k = 0; k < REC_BATCH; ++k) {
    const uint64_t i = t + (uint64_t)k * L;
    if (i >= n) break;
    fe r, s;
    int parity, code;
#if HLC_PREP_LOADS
    if (!prep_vote(sk, bytes, sig_off, off_stride, sig_len, len_stride, i, r, s, parity, code)) {
#else
    if (pre_rejected(sk, i) || !prep_sig(bytes, sig_off, off_stride, sig_len, len_stride, i, r, s, parity, code)) {
#endif
      rec[(size_t)REC_FLAGS * st + i] = PREP_SKIP << 8;
      mst[i] = MST_SKIP;
      continue;
    }
    if (code != SCHEME_NONE) {
      rec[(size_t)REC_FLAGS * st + i] = (uint32_t)code << 8;
      mst[i] = (uint8_t)(1 + code);
      continue;
    }
    active |= 1u << k;
    store_fe_ws(acc, pfx + (size_t)k * 8 * L + t, L);
    sc_mont_mul(acc, acc, r);
  }
  fe cur;
  sc_inv(cur, acc);
#pragma unroll 1
  for (int k = REC_BATCH - 1; k >= 0; --k) {
    const uint64_t i = t + (uint64_t)k * L;
    if (i >= n || !((active >> k) & 1u)) continue;
    fe r, s, prev, rinv;
    int parity, code;
#if HLC_PREP_LOADS >= 2
    // an active vote's signature is 65 bytes (the forward pass checked): its offset and the prefix
    // product in one round trip, then the bytes
    const uint64_t soff = sig_off ? sig_off[i * off_stride] : 65 * i;
    load_fe_ws(prev, pfx + (size_t)k * 8 * L + t, L);
    const uint8_t* sig = bytes + soff;
    fe_load_be(r, sig);
    fe_load_be(s, sig + 32);
    code = rec_parse(s, r, sig[64], parity);
#else
    prep_sig(bytes, sig_off, off_stride, sig_len, len_stride, i, r, s, parity, code);
    load_fe_ws(prev, pfx + (size_t)k * 8 * L + t, L);
#endif
    sc_mont_mul(rinv, prev, cur);  // r_k^-1
    sc_mont_mul(cur, cur, r);      // acc_{k-1}^-1
    rec_prep_scalars(s, rinv, parity, rec + i, st);
  }
  // the work list: per k, the wave's active votes (64 consecutive indices) in one run, one atomic
  const unsigned lane = threadIdx.x & 63u;
#pragma unroll 1
  for (int k = 0; k < REC_BATCH; ++k) {
    const bool a = (active >> k) & 1u;
    const unsigned long long bal = __ballot(a);
    if (!bal) continue;
    const unsigned leader = (unsigned)__ffsll((long long)bal) - 1u;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(list_len, (unsigned long long)__popcll(bal));
    base = __shfl(base, (int)leader);
    if (a) list[base + __popcll(bal & ((1ull << lane) - 1ull))] = (uint32_t)(t + (uint64_t)k * L);
  }
}

// ---- main: decompress + u2 R, one vote per lane at a time (persistent grid) ----
// Needs only the prep stage's records and the signatures, not the prehash: it runs beside the
// prehash kernels (hlc_api.cpp vote_stage), on the votes k_rec_prep listed -- every parsed 65-byte
// signature whose vote the checks before the signature do not reject (validate-many passes them;
// the vote-hash check needs the prehash, so a vote it rejects is still recovered and k_rec_comb
// discards it).  Records: row stride `st` (the call's vote count; a host-buffer range's pointers
// start at its first vote).
// Work is handed out dynamically, 64 listed votes per wave per grab (one atomic by lane 0).
// The SIMD's arbiter favours its oldest wave, so with a static vote-per-lane stride the oldest of
// the 3 resident waves finishes its share long before the youngest, which then runs alone at
// lone-wave efficiency (measured with per-wave clock stamps: 4-vote blocks done at 3.5 ms, the last
// 3-vote blocks at 7.0 ms of one launch); grabbing keeps every wave busy until the work runs out.
// clk != nullptr (hlc_ctx_set_clock_probe; never on a timed call): each wave stamps its core-clock ticks
// (s_memtime) and constant 100 MHz ticks (s_memrealtime) at its start and end into clk[4w .. 4w + 3] --
// the shader clock the chain ran at (MI355X_MICROARCH.md, DVFS give-back item 6).  The start stamps go
// to memory at once, so nothing but the pointer stays live across the loop.
__global__ void __launch_bounds__(REC_TPB, HLC_REC_MIN_WAVES) k_rec_main(uint64_t st, const uint8_t* bytes,
                                                                     const uint64_t* sig_off, size_t off_stride,
                                                                     uint32_t* scratch, uint64_t lanes,
                                                                     const uint32_t* rec, uint32_t* q, uint8_t* mst,
                                                                     int force_exact, unsigned long long* ctr,
                                                                     const uint32_t* list,
                                                                     const unsigned long long* list_len,
                                                                     unsigned long long* clk) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t* ws = scratch + tid;
  rtab29 tab;
  tab.g = scratch + (size_t)IL_WORDS * lanes + (size_t)tid * RTAB_WORDS;
  const unsigned lane = threadIdx.x & 63u;
  if (clk && lane == 0) {  // (vector stores from one lane)
    clk[4 * (tid >> 6)] = __builtin_amdgcn_s_memtime();
    clk[4 * (tid >> 6) + 1] = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long nl = *list_len;  // votes k_rec_prep listed
  for (;;) {
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(ctr, 64ull);
    base = __shfl(base, 0);
    if (base >= nl) break;
    if (base + lane >= nl) continue;  // the next grab is past the list's end: the wave leaves together
    const uint64_t i = list[base + lane];
    fe r, qx, qy, qz;
    bool inf = false;
    fe_load_be(r, sig_at(bytes, sig_off, off_stride, i));
    const int code = rec_u2r29(r, rec + i, st, qx, qy, qz, inf, ws, lanes, tab, force_exact != 0);
    if (code != SCHEME_NONE) {
      mst[i] = (uint8_t)(1 + code);
      continue;
    }
    mst[i] = inf ? MST_INF : MST_OK;
    store_fe_ws(qx, q + i, st);
    store_fe_ws(qy, q + (size_t)8 * st + i, st);
    store_fe_ws(qz, q + (size_t)16 * st + i, st);
  }
  if (clk && lane == 0) {
    clk[4 * (tid >> 6) + 2] = __builtin_amdgcn_s_memtime();
    clk[4 * (tid >> 6) + 3] = __builtin_amdgcn_s_memrealtime();
  }
}

#ifndef HLC_COMB_MIN_WAVES
// launch-bounds floor.  With u2 R read back only after the comb chain (rec_comb29) the kernel takes
// 142 VGPRs and runs at 3 waves per SIMD with no spills (it held 200 at 2 waves while u2 R stayed live)
#define HLC_COMB_MIN_WAVES 2
#endif
// ---- comb: after the prehash, one lane per vote at full occupancy: u1 = -z / r, u1 G by the comb
// (12 mixed additions from the HBM table), Q = u2 R + u1 G.  Votes the pre-checks rejected keep
// their state untouched, as before the split. ----
__global__ void __launch_bounds__(256, HLC_COMB_MIN_WAVES) k_rec_comb(uint64_t n, uint64_t st, const uint8_t* pre,
                                                  const uint32_t* z_digest, const uint32_t* gcomb, uint8_t* state,
                                                  const uint32_t* rec, uint32_t* q, const uint8_t* mst,
                                                  int force_exact) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (pre && pre[i] != PRE_PENDING)) return;
  const uint8_t m = mst[i];
  if (m == MST_SKIP) return;
  if (m != MST_OK && m != MST_INF) {
    state[i] = m;
    return;
  }
  fe z, u1, qx, qy, qz;
  bool neg_g;
  fe_from_digest(z, z_digest + 8 * i);
  rec_u1(z, rec + i, st, u1, neg_g);
  const int code = rec_comb29(u1, neg_g, m == MST_INF, q + i, st, qx, qy, qz, gcomb, force_exact != 0);
  state[i] = code != SCHEME_NONE ? (uint8_t)(1 + code) : REC_PENDING;
  if (code != SCHEME_NONE) return;
  store_fe_ws(qx, q + i, st);
  store_fe_ws(qy, q + (size_t)8 * st + i, st);
  store_fe_ws(qz, q + (size_t)16 * st + i, st);
}

// ---- the comb alone (HLC_OPT_EARLY_COMB): enqueued after the prehash and the prep stage, beside
// k_rec_main, whose persistent grid holds every register until its tail, so these waves take the
// slots its waves leave.  Every vote k_rec_prep listed (prep code 0) whose prehash checks passed:
// u1 = -z / r and u1 G, stored with its infinity flag for k_rec_add. ----
__global__ void __launch_bounds__(256, HLC_COMB_MIN_WAVES) k_rec_ucomb(uint64_t n, uint64_t st, const uint8_t* pre,
                                                   const uint32_t* z_digest, const uint32_t* gcomb,
                                                   const uint32_t* rec, uint32_t* g, int force_exact) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (pre && pre[i] != PRE_PENDING)) return;
  if (((rec[(size_t)REC_FLAGS * st + i] >> 8) & 0xFFu) != 0u) return;  // not listed (skipped / scheme error)
  fe z, u1, gx, gy, gz;
  bool neg_g;
  fe_from_digest(z, z_digest + 8 * i);
  rec_u1(z, rec + i, st, u1, neg_g);
  const uint32_t inf = rec_ucomb29(u1, neg_g, gx, gy, gz, gcomb, force_exact != 0);
  store_fe_ws(gx, g + i, st);
  store_fe_ws(gy, g + (size_t)8 * st + i, st);
  store_fe_ws(gz, g + (size_t)16 * st + i, st);
  g[(size_t)24 * st + i] = inf;
}

// ---- after k_rec_main and k_rec_ucomb: Q = u2 R + u1 G, the same states as k_rec_comb ----
// (Measured and not kept, round 6: k_rec_ucomb forming Q itself for the votes whose u2 R k_rec_main had
// published -- a release of the vote's mst byte after its stores, an acquire in the comb -- left k_rec_add
// 7 us of work but ran the step 1.4% slower, 103.6 vs 105.1 M votes/s; the comb starts after k_rec_main's
// last wave anyway, behind k_chain_small on the launch stream (profiles/r06g/ab_uadd.txt, uadd_timeline.txt).)
__global__ void __launch_bounds__(256) k_rec_add(uint64_t n, uint64_t st, const uint8_t* pre, uint8_t* state,
                                                 uint32_t* q, const uint32_t* g, const uint8_t* mst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (pre && pre[i] != PRE_PENDING)) return;
  const uint8_t m = mst[i];
  if (m == MST_SKIP) return;
  if (m != MST_OK && m != MST_INF) {
    state[i] = m;
    return;
  }
  fe qx, qy, qz;
  const int code = rec_add29(m == MST_INF, q + i, g + i, st, qx, qy, qz);
  state[i] = code != SCHEME_NONE ? (uint8_t)(1 + code) : REC_PENDING;
  if (code != SCHEME_NONE) return;
  store_fe_ws(qx, q + i, st);
  store_fe_ws(qy, q + (size_t)8 * st + i, st);
  store_fe_ws(qz, q + (size_t)16 * st + i, st);
}

#ifndef HLC_FIN_BATCH
#define HLC_FIN_BATCH REC_BATCH
#endif
constexpr int FIN_BATCH = HLC_FIN_BATCH;  // votes per lane (one inversion) in k_rec_final
#ifndef HLC_FIN_LOADS
#define HLC_FIN_LOADS 0  // A/B knob: k_rec_final's loads issued ahead of their use (see k_rec_final)
#endif
// ---- final: batched Z^-1 (one safegcd per FIN_BATCH votes) and affine Q, then (k_rec_addr, one
// lane per vote at full occupancy) keccak of X || Y and the owner compare.  Split in two because
// the eight keccak-f of a lane's batch made k_rec_final one long dependent chain per lane at ~1.2
// waves/SIMD (latency-bound); the address stage runs 8x as many waves. ----
__global__ void __launch_bounds__(PREP_TPB) k_rec_final(uint64_t n, uint64_t st, uint64_t L, const uint8_t* pre,
                                                        uint8_t* state, uint32_t* q, uint32_t* pfx) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  fe acc;
  fe_set(acc, 1);
#if HLC_FIN_LOADS
  // every vote's state and Z issued before any is used (one memory round trip for the forward pass,
  // was two per vote at ~1.2 waves/SIMD); the Zs stay in registers for the backward pass
  uint32_t pend = 0;
  fe zs[FIN_BATCH];
#pragma unroll
  for (int k = 0; k < FIN_BATCH; ++k) {
    const uint64_t i = t + (uint64_t)k * L;
    if (i >= n) break;
    const bool p = (!pre || pre[i] == PRE_PENDING) && state[i] == REC_PENDING;
    pend |= (uint32_t)p << k;
    load_fe_ws(zs[k], q + (size_t)16 * st + i, st);
  }
#pragma unroll
  for (int k = 0; k < FIN_BATCH; ++k) {
    if (!((pend >> k) & 1u)) continue;
    store_fe_ws(acc, pfx + (size_t)k * 8 * L + t, L);
    fe_mul(acc, acc, zs[k]);
  }
#else
#pragma unroll 1
  for (int k = 0; k < FIN_BATCH; ++k) {
    const uint64_t i = t + (uint64_t)k * L;
    if (i >= n) break;
    if ((pre && pre[i] != PRE_PENDING) || state[i] != REC_PENDING) continue;
    fe z;
    load_fe_ws(z, q + (size_t)16 * st + i, st);
    store_fe_ws(acc, pfx + (size_t)k * 8 * L + t, L);
    fe_mul(acc, acc, z);
  }
#endif
  fe cur;
  fe_inv(cur, acc);
#if HLC_FIN_LOADS
#pragma unroll
  for (int k = FIN_BATCH - 1; k >= 0; --k) {
    if (!((pend >> k) & 1u)) continue;
    const uint64_t i = t + (uint64_t)k * L;
    fe x, y, z = zs[k], prev, zi, zi2, zi3;
    load_fe_ws(x, q + i, st);
    load_fe_ws(y, q + (size_t)8 * st + i, st);
    load_fe_ws(prev, pfx + (size_t)k * 8 * L + t, L);
#else
#pragma unroll 1
  for (int k = FIN_BATCH - 1; k >= 0; --k) {
    const uint64_t i = t + (uint64_t)k * L;
    if (i >= n || (pre && pre[i] != PRE_PENDING) || state[i] != REC_PENDING) continue;
    fe x, y, z, prev, zi, zi2, zi3;
    load_fe_ws(x, q + i, st);
    load_fe_ws(y, q + (size_t)8 * st + i, st);
    load_fe_ws(z, q + (size_t)16 * st + i, st);
    load_fe_ws(prev, pfx + (size_t)k * 8 * L + t, L);
#endif
    fe_mul(zi, prev, cur);  // Z_k^-1
    fe_mul(cur, cur, z);
    fe_sqr(zi2, zi);
    fe_mul(zi3, zi2, zi);
    fe_mul(x, x, zi2);
    fe_mul(y, y, zi3);
    fe_normalize(x, x);
    fe_normalize(y, y);
    store_fe_ws(x, q + i, st);  // affine X, Y over the Jacobian ones (k_rec_addr reads them)
    store_fe_ws(y, q + (size_t)8 * st + i, st);
  }
}

// STATUS: also the vote's validate_vote tail (vote_status_one) for every vote of the call, recovered or not
// (k_vote_status's work, without its launch after this one)
template <bool STATUS>
__global__ void __launch_bounds__(256) k_rec_addr(uint64_t n, uint64_t st, const uint8_t* pre, const uint8_t* bytes,
                                                  const uint64_t* id_off, size_t off_stride, uint8_t* state,
                                                  const uint32_t* q, uint8_t* addr_out, VoteStatusArgs sa) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t ps = pre ? pre[i] : PRE_PENDING;
  if (ps != PRE_PENDING) {
    if (STATUS) vote_status_one(sa, i, ps, 0);
    return;
  }
  const uint8_t s0 = state[i];
  if (s0 != REC_PENDING) {
    if (STATUS) vote_status_one(sa, i, ps, s0);
    return;
  }
  fe x, y;
  load_fe_ws(x, q + i, st);
  load_fe_ws(y, q + (size_t)8 * st + i, st);
  uint32_t addr[5];
  pubkey_address(x, y, addr);
  const uint8_t* id = bytes + id_off[i * off_stride];
  uint32_t diff = 0;
#pragma unroll
  for (int w = 0; w < 5; ++w) diff |= addr[w] ^ load_le32(id + 4 * w);
  const uint8_t vr = diff == 0 ? HLC_VERIFY_TRUE : HLC_VERIFY_FALSE;
  state[i] = vr;
  if (STATUS) vote_status_one(sa, i, ps, vr);
  if (addr_out) {
#pragma unroll
    for (int w = 0; w < 5; ++w) {
      addr_out[20 * i + 4 * w] = (uint8_t)addr[w];
      addr_out[20 * i + 4 * w + 1] = (uint8_t)(addr[w] >> 8);
      addr_out[20 * i + 4 * w + 2] = (uint8_t)(addr[w] >> 16);
      addr_out[20 * i + 4 * w + 3] = (uint8_t)(addr[w] >> 24);
    }
  }
}

// fixed-base comb for signing: T[w][j] = j * 2^(8w) * G, affine; j = 0 unused
__global__ void k_build_fbtab(uint32_t* fb) {
  const int w = blockIdx.x, j = threadIdx.x;
  if (j == 0) {
    for (int k = 0; k < 16; ++k) fb[(w * 256) * 16 + k] = 0;
    return;
  }
  fe k;
  fe_set(k, 0);
  const int bit = 8 * w;
  k.v[bit >> 5] = (uint32_t)j << (bit & 31);
  if ((bit & 31) > 24 && (bit >> 5) < 7) k.v[(bit >> 5) + 1] = (uint32_t)j >> (32 - (bit & 31));
  gej p;
  scalar_mul_g(p, k);
  fe x, y;
  gej_to_affine(x, y, p);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    fb[(w * 256 + j) * 16 + q] = x.v[q];
    fb[(w * 256 + j) * 16 + 8 + q] = y.v[q];
  }
}

// The u1 G comb of the recovery (hlc_recover.hpp): T[w][j] = (2j+1) 2^(W w) G, affine, and the
// constant top point 2^(W windows) G.  One thread per entry, from the signing comb fbtab.  A scalar
// that reaches past 2^256 (the top window, the top point) is reduced mod n first:
// 2^bit mod n by modular doublings, then m * that by two Montgomery products.
__global__ void k_build_gcomb(uint32_t* gcomb, const uint32_t* fb) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = (uint64_t)GC_WINDOWS * GC_ENTRIES + 1;
  if (e >= total) return;
  uint32_t m;
  int bit;
  if (e == total - 1) {
    m = 1u;
    bit = GC_W * GC_WINDOWS;
  } else {
    m = 2u * (uint32_t)(e % GC_ENTRIES) + 1u;  // < 2^W
    bit = GC_W * (int)(e / GC_ENTRIES);
  }
  fe k;
  fe_set(k, 0);
  if (bit + GC_W <= 256) {
    k.v[bit >> 5] = m << (bit & 31);
    if ((bit & 31) + GC_W > 32 && (bit >> 5) < 7) k.v[(bit >> 5) + 1] = m >> (32 - (bit & 31));
  } else {
    fe s, r2, mm;
    fe_set(s, 1);
    for (int i = 0; i < bit; ++i) sc_add(s, s, s);  // 2^bit mod n
    sc_r2(r2);
    fe_set(mm, m);
    sc_mont_mul(mm, mm, r2);  // m R
    sc_mont_mul(k, mm, s);    // m 2^bit mod n
  }
  gej p;
  fixed_base_mul(p, k, fb);
  fe x, y;
  gej_to_affine(x, y, p);
  uint32_t* o = gcomb + (e == total - 1 ? GC_TOP_OFF : e * 16);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    o[q] = x.v[q];
    o[8 + q] = y.v[q];
  }
}

__global__ void k_address(uint64_t n, const uint8_t* priv, const uint32_t* fb, uint8_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe d;
  fe_load_be(d, priv + 32 * i);
  gej p;
  fixed_base_mul(p, d, fb);
  uint32_t addr[5] = {0, 0, 0, 0, 0};
  if (!p.inf) {
    fe x, y;
    gej_to_affine(x, y, p);
    pubkey_address(x, y, addr);
  }
  for (int k = 0; k < 20; ++k) out[20 * i + k] = (uint8_t)(addr[k >> 2] >> (8 * (k & 3)));
}

// EthereumConsensusSigner::sign (signing/ethereum.rs:58-64) given the EIP-191 prehash (hlc_sign.hpp).
__global__ void k_sign(uint64_t n, const uint8_t* priv, const uint32_t* z_digest, const uint32_t* fb,
                       uint8_t* sig_out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe d;
  fe_load_be(d, priv + 32 * i);
  sign_prehash(d, z_digest + 8 * i, fb, sig_out + 65 * i);
}

inline unsigned blocks_for(uint64_t n, int tpb) { return (unsigned)((n + tpb - 1) / tpb); }

}  // namespace

uint64_t recover_scratch_words() { return SCRATCH_WORDS; }

namespace {
constexpr int G_WORDS = 25;  // k_rec_ucomb -> k_rec_add: Jacobian u1 G (24 words) + its infinity flag
uint64_t core_work_words(uint64_t n) {
  const uint64_t L = (n + REC_BATCH - 1) / REC_BATCH, Lf = (n + FIN_BATCH - 1) / FIN_BATCH;
  return n * (uint64_t)(REC_WORDS + Q_WORDS + 1) + std::max(L * REC_BATCH, Lf * FIN_BATCH) * 8 + (n + 3) / 4 + 64;
}
}  // namespace

uint64_t recover_work_words(uint64_t n) { return core_work_words(n) + (uint64_t)G_WORDS * n; }

uint64_t recover_grid_lanes() {
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_rec_main, REC_TPB, 0) != hipSuccess || per_cu < 1)
    per_cu = 2;
  return (uint64_t)cus * (uint64_t)per_cu * REC_TPB;
}

uint64_t recover_range_words(uint64_t m) { return m + (m + REC_BATCH) * 8 + 16; }

namespace {
struct RecBufs {
  uint32_t *rec, *q, *pfx, *list, *g;
  uint8_t* mst;
  unsigned long long* ctr;  // [0] k_rec_main's grab counter, [1] the work list's length
  uint64_t L;
};
RecBufs rec_bufs(uint64_t n, uint32_t* work) {
  RecBufs b;
  b.rec = work;
  b.q = b.rec + n * (uint64_t)REC_WORDS;
  b.list = b.q + n * (uint64_t)Q_WORDS;
  b.pfx = b.list + n;
  b.L = (n + REC_BATCH - 1) / REC_BATCH;
  const uint64_t Lf = (n + FIN_BATCH - 1) / FIN_BATCH;
  b.mst = reinterpret_cast<uint8_t*>(b.pfx + std::max(b.L * REC_BATCH, Lf * FIN_BATCH) * 8);  // n bytes
  // the two counters: 8-byte aligned inside the 64-word tail of recover_work_words(n)
  b.ctr = reinterpret_cast<unsigned long long*>((reinterpret_cast<uintptr_t>(b.mst + n) + 7) & ~uintptr_t(7));
  b.g = work + core_work_words(n);  // G_WORDS rows of n words
  return b;
}
// The front half's buffers for items [v0, v0 + m) of a call of n items: the per-vote records in the
// call's `work` (row stride n), the work list, prefix products and counters in `range_work` (or, for
// the whole call, in `work` too).
struct FrontBufs {
  RecBufs b;  // rec / q / mst at item v0
  uint64_t st;
};
FrontBufs front_bufs(uint64_t n, uint64_t v0, uint64_t m, uint32_t* work, uint32_t* range_work,
                     const RecRange* range) {
  FrontBufs f{rec_bufs(n, work), n};
  f.b.rec += v0;
  f.b.q += v0;
  f.b.mst += v0;
  // votes per prep lane: REC_BATCH, or fewer for a range that must start soon (more lanes, shorter
  // dependent chains; k_rec_prep's loops stop at the first vote index >= m)
  const uint64_t per = range && range->batch > 0 && range->batch < REC_BATCH ? (uint64_t)range->batch : REC_BATCH;
  f.b.L = (m + per - 1) / per;
  if (range_work) {
    f.b.list = range_work;
    f.b.pfx = range_work + m;  // (m + REC_BATCH) * 8 words >= per * L * 8
    f.b.ctr = reinterpret_cast<unsigned long long*>(
        (reinterpret_cast<uintptr_t>(f.b.pfx + (m + REC_BATCH) * 8) + 7) & ~uintptr_t(7));
  }
  return f;
}
}  // namespace

unsigned long long* recover_counters(uint64_t n, uint32_t* work) { return rec_bufs(n, work).ctr; }

void launch_recover_prep(uint64_t n, const uint8_t* bytes, const uint64_t* sig_off, size_t off_stride,
                         const uint32_t* sig_len, size_t len_stride, uint32_t* work, hipStream_t s, const RecSkip* skip,
                         const RecRange* range, const KEv* ev, bool ctr_cleared) {
  const uint64_t m = range ? range->m : n;
  if (!m) return record_kev(ev, s);
  const FrontBufs f = front_bufs(n, range ? range->v0 : 0, m, work, range ? range->work : nullptr, range);
  const unsigned pb = (unsigned)((f.b.L + PREP_TPB - 1) / PREP_TPB);
  if (!ctr_cleared || range)
    (void)hipMemsetAsync(f.b.ctr, 0, 2 * sizeof(unsigned long long), s);  // grab counter, list length
  const RecSkip none{nullptr, nullptr, nullptr, nullptr};
  launch_k(ev, k_rec_prep, dim3(pb), dim3(PREP_TPB), 0, s, m, f.st, f.b.L, bytes, sig_off, off_stride, sig_len,
           len_stride, f.b.rec, f.b.pfx, f.b.mst, f.b.list, f.b.ctr + 1, skip ? *skip : none);
}

void launch_recover_main(uint64_t n, const uint8_t* bytes, const uint64_t* sig_off, size_t off_stride,
                         uint32_t* scratch, uint64_t scratch_lanes, uint32_t* work, hipStream_t s, int force_exact,
                         const RecRange* range, unsigned long long* clk, uint64_t* clk_waves, const KEv* ev) {
  const uint64_t m = range ? range->m : n;
  if (!m) return record_kev(ev, s);
  const FrontBufs f = front_bufs(n, range ? range->v0 : 0, m, work, range ? range->work : nullptr, range);
  uint64_t blocks = scratch_lanes / REC_TPB;
  uint64_t need = (m + REC_TPB - 1) / REC_TPB;
  if (blocks > need) blocks = need;
  if (blocks == 0) blocks = 1;  // a capped grid (HLC_OPT_WIRE_FRONT_CAP below one block) still runs
  if (clk_waves) *clk_waves = blocks * (REC_TPB / 64);
  launch_k(ev, k_rec_main, dim3((unsigned)blocks), dim3(REC_TPB), 0, s, f.st, bytes, sig_off, off_stride, scratch,
           (uint64_t)blocks * REC_TPB, f.b.rec, f.b.q, f.b.mst, force_exact, f.b.ctr, f.b.list, f.b.ctr + 1, clk);
}

void launch_recover_ucomb(uint64_t n, const uint8_t* pre, const uint32_t* z_digest, const uint32_t* gcomb,
                          uint32_t* work, hipStream_t s, int force_exact, uint64_t stride) {
  if (!n) return;
  const uint64_t st = stride ? stride : n;  // the records' row stride, as launch_recover_finish
  const RecBufs b = rec_bufs(st, work);
  hipLaunchKernelGGL(k_rec_ucomb, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, st, pre, z_digest, gcomb,
                     b.rec, b.g, force_exact);
}

void launch_recover_finish(uint64_t n, const uint8_t* pre, const uint32_t* z_digest, const uint8_t* bytes,
                           const uint64_t* id_off, size_t off_stride, const uint32_t* gcomb, uint32_t* work,
                           uint8_t* verify_out, uint8_t* addr_out, hipStream_t s, int force_exact, uint64_t stride,
                           bool early_comb, const KEv* ev, const VoteStatusArgs* sa) {
  if (!n) return record_kev(ev, s);
  const uint64_t st = stride ? stride : n;  // the records' row stride (>= n)
  const RecBufs b = rec_bufs(st, work);
  const uint64_t Lf = (n + FIN_BATCH - 1) / FIN_BATCH;
  const unsigned fb = (unsigned)((Lf + PREP_TPB - 1) / PREP_TPB);
  const unsigned vb = (unsigned)((n + 255) / 256);
  const KEv first = kev_start(ev), last = kev_stop(ev);
  if (early_comb)  // u1 G is in b.g already (launch_recover_ucomb, same stride)
    launch_k(&first, k_rec_add, dim3(vb), dim3(256), 0, s, n, st, pre, verify_out, b.q, b.g, b.mst);
  else
    launch_k(&first, k_rec_comb, dim3(vb), dim3(256), 0, s, n, st, pre, z_digest, gcomb, verify_out, b.rec, b.q, b.mst,
             force_exact);
  hipLaunchKernelGGL(k_rec_final, dim3(fb), dim3(PREP_TPB), 0, s, n, st, Lf, pre, verify_out, b.q, b.pfx);
  if (sa)
    launch_k(&last, k_rec_addr<true>, dim3(vb), dim3(256), 0, s, n, st, pre, bytes, id_off, off_stride, verify_out, b.q,
             addr_out, *sa);
  else
    launch_k(&last, k_rec_addr<false>, dim3(vb), dim3(256), 0, s, n, st, pre, bytes, id_off, off_stride, verify_out,
             b.q, addr_out, VoteStatusArgs{});
}


void launch_build_gcomb(uint32_t* gcomb, const uint32_t* fbtab, hipStream_t s) {
  const uint64_t total = (uint64_t)GC_WINDOWS * GC_ENTRIES + 1;
  hipLaunchKernelGGL(k_build_gcomb, dim3(blocks_for(total, 128)), dim3(128), 0, s, gcomb, fbtab);
}

size_t gcomb_words() { return GCOMB_WORDS; }

void launch_build_fbtab(uint32_t* fbtab, hipStream_t s) {
  hipLaunchKernelGGL(k_build_fbtab, dim3(32), dim3(256), 0, s, fbtab);
}

void launch_address(uint64_t n, const uint8_t* priv, const uint32_t* fbtab, uint8_t* addr, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_address, dim3(blocks_for(n, 128)), dim3(128), 0, s, n, priv, fbtab, addr);
}

void launch_sign(uint64_t n, const uint8_t* priv, const uint32_t* z_digest, const uint32_t* fbtab, uint8_t* sig,
                 hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_sign, dim3(blocks_for(n, 128)), dim3(128), 0, s, n, priv, z_digest, fbtab, sig);
}

}  // namespace hlc
