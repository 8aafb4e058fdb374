// hlc_kernels.h -- host-side launchers of the HIP kernels (internal to libhlc.so).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/hlc.h"

namespace hlc {

constexpr uint32_t NO_PROP = 0xFFFFFFFFu;
constexpr uint32_t EMPTY_SLOT = 0xFFFFFFFFu;
// pre_status values beyond the public HLC_* codes
constexpr uint8_t PRE_PENDING = 0xFE;  // needs signature recovery
constexpr uint8_t PRE_SKIP = 0xFF;     // vote not covered by any proposal
constexpr uint8_t PRE_GENERAL = 0xFD;  // too long for the fused LDS path: general pipeline decides

// The validate_vote tail of one vote (utils.rs:154-168): its pre-status st, the scheme result vr (the
// verify byte: HLC_VERIFY_TRUE / FALSE or 1 + SCHEME) when st is PRE_PENDING, then the timestamps; with
// red != nullptr also the proposal's first failing vote (red[4p + 0], the local index), so that the chain /
// duplicate / tally kernels need no vote statuses.  k_vote_status runs it over a call's votes; k_rec_addr
// runs it right after a vote's address compare when the finish is given these arguments (one kernel
// boundary less on the call's critical path).
struct VoteStatusArgs {
  hlc_votes v;
  const uint32_t* vote_prop;
  const hlc_proposal* props;
  uint64_t now;
  const uint8_t* pre_reason;
  uint8_t* status;
  uint8_t* reason;
  uint32_t* red;
};
__device__ inline void vote_status_one(const VoteStatusArgs& a, uint64_t i, uint8_t st, uint8_t vr) {
  uint8_t rs = a.pre_reason[i];
  if (st == PRE_PENDING) {
    const hlc_proposal& p = a.props[a.vote_prop[i]];
    const uint64_t ts = a.v.timestamp[i];
    if (vr >= 2) {
      st = HLC_SIGNATURE_SCHEME;
      rs = min(vr - 1, HLC_SCHEME_PLUGIN);  // (a caller's verdict above HLC_VERIFY_ERR reads as it)
    } else if (vr == HLC_VERIFY_FALSE) {
      st = HLC_INVALID_VOTE_SIGNATURE;
    } else if (ts < p.timestamp) {
      st = HLC_TIMESTAMP_OLDER_THAN_CREATION;
    } else if (ts > p.expiration_timestamp || a.now > p.expiration_timestamp) {
      st = HLC_VOTE_EXPIRED;
    } else {
      st = HLC_OK;
    }
  }
  a.status[i] = st;
  a.reason[i] = rs;
  if (a.red && st != HLC_OK) {
    const uint32_t p = a.vote_prop[i];
    if (p != NO_PROP) atomicMin(&a.red[4 * p + 0], (uint32_t)(i - a.props[p].vote_begin));
  }
}

// message-building modes
enum MsgMode { MSG_VOTE = 0, MSG_PAYLOAD = 1 };

struct Workspace;  // defined in hlc_api.cpp

// Events bound to a kernel's own dispatch (hipExtLaunchKernelGGL): `start` takes the kernel's start,
// `stop` its completion, with no marker packet in the queue (a hipEventRecord between two kernels of
// one stream leaves the queue idle for ~6 us; tools/ext_event_probe.hip).  A `stop`
// event may also be what another stream waits on.  A launcher that launches nothing records the
// events on its stream instead, so every bracket stays valid.
struct KEv {
  hipEvent_t start = nullptr, stop = nullptr;
};
template <typename F, typename... A>
inline void launch_k(const KEv* ev, F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, A... args) {
  if (ev && (ev->start || ev->stop))
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, ev->start, ev->stop, 0u, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, shmem, s, args...);
}
inline void record_kev(const KEv* ev, hipStream_t s) {
  if (!ev) return;
  if (ev->start) (void)hipEventRecord(ev->start, s);
  if (ev->stop) (void)hipEventRecord(ev->stop, s);
}
// the start half / the stop half of a pair (for launchers that run several kernels)
inline KEv kev_start(const KEv* ev) { return KEv{ev ? ev->start : nullptr, nullptr}; }
inline KEv kev_stop(const KEv* ev) { return KEv{nullptr, ev ? ev->stop : nullptr}; }

// ---- prehash stage ----
// call flags (one device word, cleared by the caller): set by the kernels, read once per call
constexpr uint32_t FLAG_GENERAL_PATH = 1u;     // some vote exceeds the fused prehash LDS window
constexpr uint32_t FLAG_LARGE_PROPOSAL = 2u;   // some proposal has > 512 votes (global chain tables)
constexpr uint32_t FLAG_LARGE_PARENTS = 4u;    // some vote of such a proposal has a parent_hash (the chain table is needed)
hipError_t launch_assign_props(const hlc_proposal* props, uint64_t np, const uint32_t* field_len, uint32_t* vote_prop,
                               uint64_t nv, uint32_t* flags, hipStream_t s,
                               const KEv* ev = nullptr,  // ev: bound to k_assign_props
                               bool map_cleared = false);  // vote_prop already NO_PROP (launch_red_init)
void launch_msg_sizes(const hlc_votes* v, uint64_t n, const uint64_t* pay_off, const uint32_t* pay_len,
                      int mode, uint64_t* sha_sz, uint64_t* kec_sz, hipStream_t s);
void launch_build_msgs(const hlc_votes* v, uint64_t n, const uint8_t* bytes, const uint64_t* pay_off,
                       const uint32_t* pay_len, int mode, const uint64_t* sha_off, const uint64_t* sha_sz,
                       uint8_t* sha_buf, const uint64_t* kec_off, const uint64_t* kec_sz, uint8_t* kec_buf,
                       hipStream_t s);
void launch_sha_blocks(uint64_t n, const uint64_t* off, const uint64_t* sz, const uint8_t* buf,
                       uint32_t* out_digest_words, hipStream_t s);
void launch_keccak_blocks(uint64_t n, const uint64_t* off, const uint64_t* sz, const uint8_t* buf,
                          uint32_t* out_digest_words, hipStream_t s);
// exclusive prefix sum of u64 sizes (hipcub); temp == nullptr queries temp_bytes
hipError_t launch_exclusive_scan(const uint64_t* in, uint64_t* out, uint64_t n, void* temp, size_t& temp_bytes,
                           hipStream_t s);
// hlc_eth_verify_batch over host-staged items: the length checks (ethereum.rs:71-82) and the
// EIP-191 keccak of each payload streamed from the arena (dense per-item arrays, stride 1)
void launch_verify_prehash(uint64_t n, const uint8_t* bytes, const uint64_t* pay_off, const uint32_t* pay_len,
                           const uint32_t* sig_len, const uint32_t* id_len, uint32_t* kec_dig, uint8_t* pre,
                           uint8_t* verify_out, hipStream_t s);
// fused byte stage (sizes + SHA-256 compare + EIP-191 keccak + pre-status) for votes whose
// messages fit the per-lane LDS window; others get PRE_GENERAL and *general is set non-zero
// eth == false (a caller-side scheme, the *_verdicts entries): no Ethereum length checks and no EIP-191
// keccak -- every vote that passes the vote-hash compare becomes PRE_PENDING for the caller's verdict
void launch_prehash_fused(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                          uint32_t* kec_dig, uint8_t* pre, uint8_t* pre_reason, uint32_t* general, hipStream_t s,
                          bool eth = true);
// general path without host round trips: streams the PRE_GENERAL votes' messages from the arena
// (SHA-256 compare + EIP-191 keccak + pre-status); exits at once unless *flags has FLAG_GENERAL_PATH
void launch_prehash_stream(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                           const uint32_t* flags, uint32_t* kec_dig, uint8_t* pre, uint8_t* pre_reason,
                           hipStream_t s, bool eth = true);
// the scheme payload of every vote (utils.rs:150-152: prost encoding, signature cleared): sizes (u64 for
// the scan and u32 for the caller), then the bytes at the scanned offsets
void launch_payload_sizes(const hlc_votes* v, uint64_t n, uint64_t* sz64, uint32_t* sz32, hipStream_t s);
void launch_encode_payloads(const hlc_votes* v, uint64_t n, const uint64_t* off, uint8_t* out, hipStream_t s);
// general-path pre-status: decides only the votes marked PRE_GENERAL
void launch_pre_status(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                       const uint32_t* sha_digest, uint8_t* pre, uint8_t* pre_reason, hipStream_t s);

// ---- recovery ----
// items: i in [0, n) with pre[i] == PRE_PENDING; signature bytes / identity bytes read from
// bytes + sig_off[i*stride_f] etc.  verify_out[i]: HLC_VERIFY_TRUE/FALSE or 1+SCHEME.
// kernels (hlc_recover.hip): k_rec_prep, k_rec_main, k_rec_comb, k_rec_final, k_rec_addr; `work` holds
// recover_work_words(n) words of per-vote records for the call
// in three parts: the prep stage reads only the signatures (65-byte ones by sig_len; sig_off == nullptr:
// a dense array, 65 B per item at bytes + 65 i) and
// the main stage (u2 R) only the prep records, so a caller may enqueue both on a second stream
// concurrently with the prehash kernels; the finish (k_rec_comb: u1 G + the addition; k_rec_final;
// k_rec_addr) once both are done
// validate-many's checks before the signature (skip != nullptr in launch_recover_prep): votes that
// fail them are not recovered (their status does not depend on it)
struct RecSkip {
  const uint32_t* vote_prop;   // proposal index per vote (NO_PROP: not covered)
  const hlc_proposal* props;
  const uint32_t* proposal_id; // per vote
  const uint32_t* field_len;   // hlc_votes.field_len
};
// range != nullptr: the front half over items [v0, v0 + m) only (bytes / sig_off / sig_len already
// at item v0), records in the call's `work` (sized for all n items, so that one finish covers every
// range); the range's work list, prefix products and counters in range->work
// (recover_range_words(m)), so ranges may run on different streams at once.
struct RecRange {
  uint64_t v0, m;
  uint32_t* work;
  int batch;  // votes per k_rec_prep lane (one inversion each): 0 = the default (8)
};
void launch_recover_prep(uint64_t n, const uint8_t* bytes, const uint64_t* sig_off, size_t off_stride,
                         const uint32_t* sig_len, size_t len_stride, uint32_t* work, hipStream_t s,
                         const RecSkip* skip = nullptr, const RecRange* range = nullptr,
                         const KEv* ev = nullptr,  // ev: bound to k_rec_prep
                         bool ctr_cleared = false);  // (whole call) recover_counters already zero
// the whole call's two work counters (grab counter, list length) inside `work`, which a launcher before
// the prep stage may clear (launch_red_init) so that the prep stage needs no memset of its own
unsigned long long* recover_counters(uint64_t n, uint32_t* work);
void launch_recover_main(uint64_t n, const uint8_t* bytes, const uint64_t* sig_off, size_t off_stride,
                         uint32_t* scratch, uint64_t scratch_lanes, uint32_t* work, hipStream_t s, int force_exact = 0,
                         const RecRange* range = nullptr, unsigned long long* clk = nullptr,
                         uint64_t* clk_waves = nullptr, const KEv* ev = nullptr);  // ev: bound to k_rec_main
void launch_recover_finish(uint64_t n, const uint8_t* pre, const uint32_t* z_digest, const uint8_t* bytes,
                           const uint64_t* id_off, size_t off_stride, const uint32_t* gtab, uint32_t* work,
                           uint8_t* verify_out, uint8_t* addr_out, hipStream_t s, int force_exact = 0,
                           uint64_t stride = 0,  // stride: the records' row stride (0 = n; the fronts' n)
                           bool early_comb = false,  // u1 G from launch_recover_ucomb: k_rec_add, not k_rec_comb
                           const KEv* ev = nullptr,  // ev: start at the first kernel, stop at k_rec_addr
                           const VoteStatusArgs* sa = nullptr);  // sa: k_rec_addr also writes the vote statuses
// u1 G alone (k_rec_ucomb) over a whole call's records (row stride n), once the prehash (pre, z_digest)
// and the prep stage are done; launch_recover_finish(..., early_comb = true) adds u2 R after k_rec_main.
void launch_recover_ucomb(uint64_t n, const uint8_t* pre, const uint32_t* z_digest, const uint32_t* gtab,
                          uint32_t* work, hipStream_t s, int force_exact = 0, uint64_t stride = 0);
uint64_t recover_grid_lanes();
uint64_t recover_scratch_words();  // per-lane workspace words of k_rec_main
uint64_t recover_work_words(uint64_t n);
uint64_t recover_range_words(uint64_t m);  // RecRange::work words for m items
void launch_build_gcomb(uint32_t* gcomb, const uint32_t* fbtab, hipStream_t s);  // needs fbtab
size_t gcomb_words();

// ---- validation tail ----
void launch_vote_status(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                        uint64_t now, const uint8_t* pre, const uint8_t* pre_reason, const uint8_t* verify,
                        uint8_t* status, uint8_t* reason, uint32_t* red, hipStream_t s);
// per-proposal reduction records: first failing vote / chain error / duplicate = none, YES = 0
// flag != nullptr: also clears the call's flag word; vote_prop != nullptr: also sets its nv entries to
// NO_PROP for launch_assign_props(..., map_cleared = true) -- one launch instead of two memsets and a kernel
void launch_red_init(uint32_t* red, uint64_t np, hipStream_t s, uint32_t* flag = nullptr, const KEv* ev = nullptr,
                     uint32_t* vote_prop = nullptr, uint64_t nv = 0,
                     unsigned long long* zero2 = nullptr);  // zero2: two words cleared too
// large-proposal chain / duplicate tables: always enqueued, skipped on the device unless the call's
// flag word has FLAG_LARGE_PROPOSAL (flags == nullptr: always run)
// (the duplicate test reports into `red` from k_tables)
void launch_tables(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                   uint32_t* chain_tab, uint32_t* dup_tab, uint32_t mask, uint32_t* red, uint64_t np,
                   const uint32_t* flags, hipStream_t s,
                   const KEv* ev = nullptr);  // ev: start at the first kernel, stop at k_tables
void launch_chain_check(const hlc_votes* v, uint64_t n, const uint32_t* vote_prop, const hlc_proposal* props,
                        const uint8_t* status, const uint32_t* chain_tab, const uint32_t* dup_tab,
                        uint32_t mask, uint8_t* chain_code, uint32_t* red, uint64_t np, const uint32_t* flags,
                        hipStream_t s, const KEv* ev = nullptr);
// batched handle_consensus_timeout: new state + status per session
void launch_timeout(uint64_t n, const hlc_session_tally* ss, uint8_t* out_state, uint8_t* out_status, hipStream_t s);
// proposals with <= 512 votes: chain / duplicate / YES count in LDS, one wave per proposal
// (writes chain_code and red[4p+1..3] for those; the global-table kernels skip them).  Needs no vote
// statuses: vote_stage enqueues it on the launch stream after the prehash kernels, beside k_rec_main
// (which runs on the context's second stream), after launch_red_init.
void launch_chain_small(const hlc_votes* v, const hlc_proposal* props, uint64_t np, uint8_t* chain_code,
                        uint32_t* red, hipStream_t s, const KEv* ev = nullptr);
// outcome counters: bins[0..31] += votes by status, bins[32..63] += proposals by status
void launch_outcome_hist(const uint8_t* vote_status, uint64_t n, const hlc_result* res, uint64_t np,
                         unsigned long long* bins, hipStream_t s);
void launch_finalize(const hlc_proposal* props, uint64_t np, uint64_t now, const uint8_t* status,
                     const uint8_t* reason, const uint8_t* chain_code, const uint32_t* red,
                     hlc_result* out, hipStream_t s, const KEv* ev = nullptr);

// ---- wire decode (hlc_wire.hip) ----
// mode 0: vote_count[m], wout[m], pout[m], first wire_slab() records per message in slab_*, *big |= 1 when
// a message has more; mode 1 (after the scan, only when *big): every record of those messages in place
void launch_wire_walk(int mode, const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nm,
                      uint64_t* vote_count, const uint64_t* vote_begin, hlc_wire_proposal* wout, hlc_proposal* pout,
                      const hlc_scope_config* scope, uint64_t n_scope, uint64_t* slab_off, uint32_t* slab_len,
                      uint32_t* big, uint64_t* vrec_off, uint32_t* vrec_len, uint32_t* vrec_msg, uint64_t* huge,
                      hipStream_t s, uint32_t* first_bad = nullptr,  // mode 0: first_bad[m] = ~0 when given
                      int walk = -1);  // HLC_OPT_WIRE_WALK: -1 the build's default walker, 0 per lane, 1 LDS
// Messages longer than wire_huge_threshold() are skipped by the walker (mode 0 appends (m, len) to
// huge[1..], count in huge[0]) and decoded by launch_huge_decode: parallel field-boundary discovery
// (next[] per byte offset + pointer jumping), records into hoff/hlen in stream order, then
// launch_huge_place moves them to vote_begin[m] after the scan.
uint64_t wire_huge_threshold();
size_t huge_scan_bytes(uint32_t len);
// returns 0, or -1 when a HIP call failed (the caller reports HLC_EDEVICE)
int launch_huge_decode(const uint8_t* wire, uint64_t m, uint64_t base, uint32_t len, uint32_t* next, uint32_t* jump,
                       uint32_t* save, uint8_t* mark, uint32_t* st, uint32_t* flag, uint32_t* rank, void* scan_tmp,
                       size_t scan_bytes, uint64_t* hoff, uint32_t* hlen, uint64_t* vote_count,
                       hlc_wire_proposal* wout, hlc_proposal* pout, const hlc_scope_config* scope, uint64_t n_scope,
                       hipStream_t s);
void launch_huge_place(uint64_t m, const uint64_t* vote_count, const uint64_t* vote_begin, const uint64_t* hoff,
                       const uint32_t* hlen, uint64_t* vrec_off, uint32_t* vrec_len, uint32_t* vrec_msg,
                       hipStream_t s);
// (vb_base: added to vote_begin in pout[m].vote_begin -- a message range decoded on its own, with
// vote_begin relative to its first vote; first_bad != nullptr: first_bad[m] reset to ~0 for k_wire_votes)
void launch_wire_place(uint64_t nm, const uint64_t* vote_count, const uint64_t* vote_begin, const uint64_t* slab_off,
                       const uint32_t* slab_len, hlc_proposal* pout, uint64_t* vrec_off, uint32_t* vrec_len,
                       uint32_t* vrec_msg, hipStream_t s, uint64_t vb_base = 0, uint32_t* first_bad = nullptr);
uint64_t wire_slab();
// one block: vote_begin = exclusive scan of vote_count[0, nm); out_mapped (page-locked host memory, its
// device pointer): [0] = the total, [1] = 1 if some count exceeds wire_slab()
void launch_wire_range_scan(const uint64_t* vote_count, uint64_t* vote_begin, uint64_t nm, uint64_t* out_mapped,
                            hipStream_t s);
void launch_wire_touch(const uint8_t* wire, uint64_t len, uint32_t* sink, hipStream_t s);
// decodes vote records into `out` (device SoA); first_bad[m] (pre-set to ~0) = first failing record
void launch_wire_votes(const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nv,
                       const uint64_t* vrec_off, const uint32_t* vrec_len, const uint32_t* vrec_msg,
                       const uint64_t* vote_begin, const hlc_votes* out, uint8_t* vote_err, uint32_t* first_bad,
                       hipStream_t s);
// k_wire_place + k_wire_votes in one kernel for messages of at most wire_slab() records (records read from
// the walker's slab; first_bad reset by the walker); `out` at the range's first vote
void launch_wire_votes_slab(const uint8_t* wire, const uint64_t* msg_off, const uint32_t* msg_len, uint64_t nm,
                            const uint64_t* vote_count, const uint64_t* vote_begin, const uint64_t* slab_off,
                            const uint32_t* slab_len, hlc_proposal* pout, uint64_t vb_base, const hlc_votes* out,
                            uint8_t* vote_err, uint32_t* first_bad, hipStream_t s);
void launch_wire_final(uint64_t nm, const uint64_t* vote_begin, const uint8_t* vote_err, const uint32_t* first_bad,
                       hlc_wire_proposal* wout, hlc_proposal* pout, hipStream_t s);
void launch_wire_results(uint64_t nm, const hlc_wire_proposal* wout, hlc_result* res, hipStream_t s);

// ---- streaming votes (hlc_stream.hip) ----
void launch_sessions_to_props(const hlc_session* ss, uint64_t m, hlc_proposal* props, hipStream_t s);
// stable sort of vote indices by session; temp == nullptr queries temp_bytes
hipError_t launch_sort_by_session(const uint32_t* vote_session, uint64_t n, uint32_t* keys_out, uint32_t* iota,
                            uint32_t* order, void* temp, size_t& temp_bytes, hipStream_t s);
void launch_segments(const uint32_t* keys, uint64_t n, uint32_t* seg_begin, uint32_t* seg_end, hipStream_t s);
// duplicate flags: tab (pre-set to ~0), minv (pre-set to ~0) sized mask + 1; slot_of[n], dup[n].
// Existing owner k: owner_off == nullptr -> owners[20 k .. + 20] (hlc_process_votes); else
// owners[owner_off[k] .. + owner_len[k]] (any identity length, hlc_process_votes_verdicts)
void launch_dup_flags(uint32_t* tab, uint32_t* minv, uint32_t mask, const uint8_t* owners,
                      const uint32_t* owner_session, uint64_t n_owners, const hlc_votes* v, const uint32_t* vote_session,
                      const uint8_t* st, uint32_t* slot_of, uint8_t* dup, hipStream_t s,
                      const uint64_t* owner_off = nullptr, const uint32_t* owner_len = nullptr);
void launch_stream_init(uint64_t n, const uint32_t* vote_session, const uint8_t* vstatus, uint8_t* st, uint8_t* tr,
                        uint8_t* ins, hipStream_t s);
void launch_apply_votes(hlc_session* ss, uint64_t m, const uint32_t* seg_begin, const uint32_t* seg_end,
                        const uint32_t* order, const hlc_votes* v, uint64_t now, const uint8_t* dup, uint8_t* st,
                        uint8_t* tr, uint8_t* ins, hipStream_t s);

// ---- signing ----
void launch_build_fbtab(uint32_t* fbtab, hipStream_t s);
void launch_address(uint64_t n, const uint8_t* priv, const uint32_t* fbtab, uint8_t* addr, hipStream_t s);
void launch_sign(uint64_t n, const uint8_t* priv, const uint32_t* z_digest, const uint32_t* fbtab,
                 uint8_t* sig, hipStream_t s);

// ---- synthetic workload (hlc_synth.hip) ----
uint64_t synth_arena_bytes(uint64_t n_proposals, uint64_t votes_per_proposal);
void launch_synth(uint64_t seed, uint64_t start, uint64_t n_proposals, uint32_t votes_per_proposal, uint32_t expected,
                  int gossipsub, const hlc_votes* out, hlc_proposal* props, uint8_t* priv_out, const uint32_t* fbtab,
                  hipStream_t s);
// config 5 on the device (hlc_synth.hip k_byz_*): mutates a launch_synth batch in place; kind_out[n]
// (HLC_BYZ_*), key_work u64[n] scratch
void launch_synth_byzantine(uint64_t seed, uint64_t start, uint64_t n_proposals, uint32_t votes_per_proposal,
                            const hlc_votes* votes, uint8_t* kind_out, uint64_t* key_work, const uint32_t* fbtab,
                            hipStream_t s);

constexpr size_t FBTAB_WORDS = 32 * 256 * 16;   // fixed-base comb: 32 windows x 256 affine points

}  // namespace hlc
