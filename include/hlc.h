/*
 * hlc.h — C ABI of the MI355X batch vote-validation engine (libhlc.so).
 *
 * Drop-in boundary for the hot path of vacp2p/hashgraph-like-consensus v0.6.0
 * (`ConsensusService::process_incoming_proposal`, /root/reference/src/service.rs:263-279).
 * Every entry point cites the reference interface it replaces.  No torch / HIP types
 * appear in the signatures: plain pointers, sizes and an opaque context.
 *
 * Ownership: the caller owns every buffer it passes; the library owns the device
 * workspace inside `hlc_ctx`; no pointer is retained after a call returns.
 * Threading: a context serialises its calls with an internal mutex (the reference's
 * service is `Send + Sync`, CHANGELOG.md 0.5.0); use one context per thread for
 * concurrency.  Host-buffer entry points are blocking (mirror the sync Rust API).
 * Return value: 0 on success, negative HLC_E* on API / device failure.  Item-level
 * outcomes (reject codes) are only ever reported through the output arrays.
 */
#ifndef HLC_H
#define HLC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HLC_ABI_VERSION 1

/* ---- API return codes -------------------------------------------------------- */
#define HLC_SUCCESS 0
#define HLC_EINVAL (-1)   /* bad argument (NULL pointer, out-of-range offsets, ...) */
#define HLC_EDEVICE (-2)  /* HIP runtime / kernel failure */
#define HLC_ENOMEM (-3)   /* device allocation failed */
#define HLC_ENODEV (-4)   /* no usable gfx950 device */
#define HLC_ERANGE (-5)   /* an output capacity is too small (the required size is reported) */

/* ---- Item status codes: the hot-path subset of `ConsensusError`
 *      (/root/reference/src/error.rs:11-74).  Values are ABI. ------------------- */
#define HLC_OK 0
#define HLC_PROPOSAL_EXPIRED 1                 /* error.rs:39 */
#define HLC_VOTE_PROPOSAL_ID_MISMATCH 2        /* error.rs:41 */
#define HLC_EMPTY_VOTE_OWNER 3                 /* error.rs:33 */
#define HLC_EMPTY_VOTE_HASH 4                  /* error.rs:37 */
#define HLC_EMPTY_SIGNATURE 5                  /* error.rs:25 */
#define HLC_INVALID_VOTE_HASH 6                /* error.rs:35 */
#define HLC_SIGNATURE_SCHEME 7                 /* error.rs:72-73, ConsensusSchemeError::Verify */
#define HLC_INVALID_VOTE_SIGNATURE 8           /* error.rs:23 */
#define HLC_TIMESTAMP_OLDER_THAN_CREATION 9    /* error.rs:49 */
#define HLC_VOTE_EXPIRED 10                    /* error.rs:31 */
#define HLC_RECEIVED_HASH_MISMATCH 11          /* error.rs:43 */
#define HLC_PARENT_HASH_MISMATCH 12            /* error.rs:45 */
#define HLC_DUPLICATE_VOTE 13                  /* error.rs:27 */
#define HLC_MAX_ROUNDS_EXCEEDED 14             /* error.rs:65 */
#define HLC_PROPOSAL_ALREADY_EXIST 15          /* error.rs:57 (host-side, storage) */
#define HLC_INSUFFICIENT_VOTES_AT_TIMEOUT 16   /* error.rs:64 (handle_consensus_timeout) */
#define HLC_PROPOSAL_DECODE_ERROR 17           /* wire bytes are not a Proposal (prost DecodeError,
                                                  raised by the embedder before service.rs:263) */
#define HLC_SESSION_NOT_ACTIVE 18              /* error.rs:54 (add_vote on a Failed session) */
#define HLC_SESSION_NOT_FOUND 19               /* error.rs:56 (no session for the vote's proposal) */

/* Sub-reason of HLC_SIGNATURE_SCHEME (the reference's Verify(String) message class). */
#define HLC_SCHEME_NONE 0
#define HLC_SCHEME_SIG_LEN 1        /* signing/ethereum.rs:71-76 */
#define HLC_SCHEME_ID_LEN 2         /* signing/ethereum.rs:77-82 */
#define HLC_SCHEME_BAD_PARITY 3     /* alloy Signature::from_raw_array / normalize_v (ethereum.rs:86) */
#define HLC_SCHEME_SCALAR_RANGE 4   /* r or s zero or >= n (k256 from_scalars via to_k256) */
#define HLC_SCHEME_NO_POINT 5       /* R = decompress(r) does not exist */
#define HLC_SCHEME_INFINITY 6       /* recovered key is the identity */
#define HLC_SCHEME_PLUGIN 7         /* Err(Verify) returned by a caller-side scheme (the *_verdicts entries) */

/* Outcome of `ConsensusSignatureScheme::verify` (signing.rs:60-73) per item. */
#define HLC_VERIFY_TRUE 0           /* Ok(true)  */
#define HLC_VERIFY_FALSE 1          /* Ok(false) */
/* values >= 2: Err(ConsensusSchemeError::Verify), value - 1 == HLC_SCHEME_* reason */
#define HLC_VERIFY_ERR (1 + HLC_SCHEME_PLUGIN) /* a caller-side scheme's Err(Verify) */

/* SessionTransition (types.rs:29-34) */
#define HLC_STILL_ACTIVE 0
#define HLC_REACHED_NO 1
#define HLC_REACHED_YES 2

/* ---- Vote batch (struct-of-arrays view of `Vec<Vote>`, consensus.proto:19-29) ---- */
#define HLC_F_OWNER 0
#define HLC_F_PARENT 1
#define HLC_F_RECEIVED 2
#define HLC_F_VOTE_HASH 3
#define HLC_F_SIGNATURE 4
#define HLC_NFIELDS 5

typedef struct hlc_votes {
  uint64_t n;                 /* number of votes */
  const uint32_t* vote_id;    /* [n]  Vote.vote_id      (tag 20) */
  const uint32_t* proposal_id;/* [n]  Vote.proposal_id  (tag 22) */
  const uint64_t* timestamp;  /* [n]  Vote.timestamp    (tag 23) */
  const uint8_t* vote;        /* [n]  Vote.vote (0/1)   (tag 24) */
  const uint8_t* bytes;       /* arena holding every bytes field */
  uint64_t bytes_len;
  const uint64_t* field_off;  /* [n][HLC_NFIELDS] offset of owner/parent/received/vote_hash/signature */
  const uint32_t* field_len;  /* [n][HLC_NFIELDS] length (0 = empty bytes) */
} hlc_votes;

/* One proposal = a contiguous run of votes plus the scalars `resolve_config`
 * (service.rs:444-484) and the Proposal message (consensus.proto:5-16) contribute. */
typedef struct hlc_proposal {
  uint64_t vote_begin;            /* index of the proposal's first vote in hlc_votes */
  uint32_t vote_count;
  uint32_t proposal_id;           /* Proposal.proposal_id */
  uint64_t timestamp;             /* Proposal.timestamp (creation time) */
  uint64_t expiration_timestamp;  /* Proposal.expiration_timestamp */
  uint32_t expected_voters_count; /* Proposal.expected_voters_count */
  uint32_t max_rounds;            /* ConsensusConfig.max_rounds (P2P: 0 = ceil(2n/3)) */
  double consensus_threshold;     /* ConsensusConfig.consensus_threshold */
  uint8_t use_gossipsub_rounds;   /* ConsensusConfig.use_gossipsub_rounds */
  uint8_t liveness_criteria_yes;  /* Proposal.liveness_criteria_yes */
  uint8_t _pad[6];
} hlc_proposal; /* 56 bytes */

/* Per-proposal result of `ConsensusSession::from_proposal` (session.rs:198-221). */
typedef struct hlc_result {
  uint8_t status;        /* HLC_OK or the first error (SURVEY.md Appendix B order) */
  uint8_t transition;    /* HLC_STILL_ACTIVE / HLC_REACHED_NO / HLC_REACHED_YES (status == OK) */
  uint8_t scheme_reason; /* HLC_SCHEME_* when status == HLC_SIGNATURE_SCHEME */
  uint8_t _pad;
  uint32_t bad_index;    /* index (within the proposal) of the failing vote, or 0xFFFFFFFF */
  uint32_t yes;          /* YES votes in the owner->vote map (status == OK) */
  uint32_t total;        /* votes in the owner->vote map (status == OK) */
} hlc_result; /* 16 bytes */

/* Session state (session.rs:157-164) for the timeout tally. */
#define HLC_SESSION_ACTIVE 0
#define HLC_SESSION_REACHED_NO 1
#define HLC_SESSION_REACHED_YES 2
#define HLC_SESSION_FAILED 3

/* One session as `handle_consensus_timeout` (service.rs:323-373) sees it: the counts of its
 * owner->vote map (session.rs:167-178), its state, and the scalars of its config / proposal. */
typedef struct hlc_session_tally {
  uint32_t total;                 /* votes in the session (distinct owners) */
  uint32_t yes;                   /* YES votes among them */
  uint32_t expected_voters_count; /* Proposal.expected_voters_count */
  uint8_t state;                  /* HLC_SESSION_* */
  uint8_t liveness_criteria_yes;  /* Proposal.liveness_criteria_yes */
  uint8_t _pad[2];
  double consensus_threshold;     /* ConsensusConfig.consensus_threshold */
} hlc_session_tally; /* 24 bytes */

/* ---- Wire format (consensus.proto:5-29) ------------------------
 * prost 0.14 `DecodeError` classes, reported per message by the device decoder. */
#define HLC_WIRE_OK 0
#define HLC_WIRE_INVALID_VARINT 1       /* > 10 bytes, 10th byte >= 2, or out of bytes */
#define HLC_WIRE_INVALID_KEY 2          /* key > u32::MAX */
#define HLC_WIRE_INVALID_WIRE_TYPE 3    /* wire type 6 or 7 */
#define HLC_WIRE_INVALID_TAG 4          /* field number 0 */
#define HLC_WIRE_WIRE_TYPE_MISMATCH 5   /* known field with the wrong wire type */
#define HLC_WIRE_BUFFER_UNDERFLOW 6     /* length / fixed-width value past the end */
#define HLC_WIRE_DELIMITED_EXCEEDED 7   /* a Vote's fields run past the Vote's length */
#define HLC_WIRE_INVALID_UTF8 8         /* Proposal.name is not UTF-8 */
#define HLC_WIRE_UNEXPECTED_END_GROUP 9 /* end-group key without its start group */
#define HLC_WIRE_RECURSION_LIMIT 10     /* groups nested past prost's recursion limit (100) */

/* The `resolve_config` inputs (service.rs:444-484) that come from the scope, not the message:
 * the scope's ConsensusConfig (or ConsensusConfig::gossipsub() when it has none). */
typedef struct hlc_scope_config {
  double consensus_threshold;     /* ConsensusConfig.consensus_threshold */
  uint32_t max_rounds;            /* ConsensusConfig.max_rounds */
  uint8_t use_gossipsub_rounds;   /* ConsensusConfig.use_gossipsub_rounds */
  uint8_t _pad[3];
} hlc_scope_config; /* 16 bytes */

/* Decoded Proposal fields that validation does not consume, plus the decode outcome.
 * Offsets are relative to the start of the message. */
typedef struct hlc_wire_proposal {
  uint64_t name_off, payload_off, owner_off; /* Proposal.name / payload / proposal_owner */
  uint32_t name_len, payload_len, owner_len;
  uint32_t round;          /* Proposal.round (tag 16) as sent; from_proposal resets it to 1 */
  uint32_t bad_vote;       /* index of the failing `votes` record, or 0xFFFFFFFF */
  uint8_t decode_status;   /* HLC_WIRE_*: the first error prost meets in stream order */
  uint8_t _pad[3];
} hlc_wire_proposal; /* 48 bytes */

/* One live session as `process_incoming_vote` (service.rs:286-305) reads and mutates it
 * (session.rs:167-190): proposal scalars, resolved config, state, round and tally.  In/out. */
typedef struct hlc_session {
  uint64_t timestamp;             /* Proposal.timestamp (creation time, validate_vote) */
  uint64_t expiration_timestamp;  /* Proposal.expiration_timestamp */
  uint32_t proposal_id;           /* Proposal.proposal_id (votes must carry it) */
  uint32_t expected_voters_count; /* Proposal.expected_voters_count */
  uint32_t round;                 /* Proposal.round of the session (in/out) */
  uint32_t total;                 /* votes in the owner->vote map (in/out) */
  uint32_t yes;                   /* YES votes among them (in/out) */
  uint32_t max_rounds;            /* ConsensusConfig.max_rounds */
  double consensus_threshold;     /* ConsensusConfig.consensus_threshold */
  uint8_t state;                  /* HLC_SESSION_* (in/out) */
  uint8_t use_gossipsub_rounds;   /* ConsensusConfig.use_gossipsub_rounds */
  uint8_t liveness_criteria_yes;  /* Proposal.liveness_criteria_yes */
  uint8_t _pad[5];
} hlc_session; /* 56 bytes */

typedef struct hlc_ctx hlc_ctx;

/* ---- Context -------------------------------------------------------------------- */
/* Creates a context on HIP device `device` (process-global lazily-initialised device
 * state is what the static `Signer::verify` of signing.rs:69 needs).  The fixed-base tables -- the
 * u1 G comb of the recovery, 11 x 2^23 affine points = 5.9 GB of HBM, and the 512 KiB signing
 * comb -- are read-only, so there is one pair per device per process: the first context on a device
 * allocates and builds them (~0.1-0.25 s), later contexts on it share them (~1 ms), and the last one
 * destroyed frees them; HLC_ENOMEM (with hlc_last_error) when they do not fit.  The recovery's per-lane workspace (~205 MB: one R table of 16 x 64 B plus the
 * z-ratios per lane of the persistent grid) and the per-vote workspace (~0.5 KB per vote of the
 * largest batch) are allocated on first use (or hlc_ctx_reserve).
 * The host-buffer entries (hlc_validate_proposals, hlc_eth_verify_batch) add on their first call:
 * a second per-lane recovery workspace (~205 MB; their recovery ranges alternate over two streams),
 * each recovery range's work list and prefix products (~0.15 KB per vote), page-locked staging of the
 * inputs (the call's input bytes + 69 B per vote of dense signatures) and of the outputs, and a
 * device copy of each; all are kept for later calls of the same or smaller size. */
int hlc_ctx_create(int device, hlc_ctx** out);
void hlc_ctx_destroy(hlc_ctx* ctx);
/* Pre-sizes the device-resident validate-many workspace (hlc_validate_proposals_device up to these
 * sizes then allocates nothing; the host-buffer entries still add what hlc_ctx_create lists).  The
 * wire-decode and streaming paths grow their own workspace on first use and keep it for later
 * calls of the same or smaller size. */
int hlc_ctx_reserve(hlc_ctx* ctx, uint64_t max_votes, uint64_t max_proposals, uint64_t max_bytes);
const char* hlc_last_error(void);
int hlc_abi_version(void);

/* Page-locked host memory (hipHostMalloc): input arrays a caller builds in it (the SoA arrays,
 * the byte arena, the proposals; identities / payloads / signatures of hlc_eth_verify_batch) are
 * DMA'd to the device straight from there by the host-buffer entries, with no staging copy (any
 * array may be page-locked or not; the library checks each one per call).  hlc_host_free releases
 * it.  Not tied to a context. */
int hlc_host_alloc(uint64_t bytes, void** out);
void hlc_host_free(void* p);

/* ---- Context options ------------------------------------------------------------------------
 * The host-buffer entries' tunables, per context.  hlc_ctx_create reads each one's default from the
 * environment variable named beside it, once; no library call reads the environment after that (an
 * embedder's threads may setenv at any time), and hlc_ctx_set_option changes a context's value. */
#define HLC_OPT_HOST_THREADS 1     /* staging threads incl. the caller, 1..64 (HLC_HOST_THREADS; default
                                      hlc_host_threads()) */
#define HLC_OPT_POOL_BIND 2        /* the staging workers' CPUs: HLC_POOL_BIND_* (HLC_POOL_BIND) */
#define HLC_OPT_NT_COPY 3          /* 1: non-temporal staging copies on AVX2 CPUs (HLC_NT_COPY; default 1) */
#define HLC_OPT_SPLIT_VOTES 4      /* votes of the first recovery range of hlc_validate_proposals /
                                      hlc_eth_verify_batch, later ranges doubling; 0: one range; -1:
                                      the default (HLC_SPLIT_VOTES, a list "a,b,..."; 98304,196608) */
#define HLC_OPT_HOST_TRACE 5       /* 0 off; 1 phase trace on stderr and in hlc_ctx_last_host_trace; 2 the
                                      latter only (HLC_HOST_TRACE; default 0) */
#define HLC_OPT_FIRST_BATCH 6      /* votes per prep lane of the first recovery range (HLC_FIRST_BATCH; 1) */
#define HLC_OPT_REST_PIECES 7      /* pieces the non-signature inputs are staged in, 1..64 (HLC_REST_PIECES; 3) */
#define HLC_OPT_WIRE_SPLIT_BYTES 8 /* bytes of the first message range of hlc_validate_wire_proposals,
                                      later ranges doubling; 0: one range; -1: the default
                                      (HLC_WIRE_SPLIT_BYTES, a list; 8, 16, 24, 32 MiB) */
#define HLC_OPT_WIRE_FRONT_CAP 9   /* waves per recovery grid of every message range but the last; 0: full
                                      grids (HLC_WIRE_FRONT_CAP; default 1536) */
#define HLC_OPT_WIRE_CHUNK 10      /* bytes per wire staging piece, at least 4096 (a smaller value reads as
                                      4096; HLC_WIRE_CHUNK; 4 MiB) */
#define HLC_OPT_REC_FORCE_EXACT 11 /* 1: every vote through the recovery's checked chains (tests; 0) */
#define HLC_OPT_SERIAL_STAGES 12   /* 1: the recovery's prep + main after the prehash on one stream
                                      (isolated kernel traces; HLC_SERIAL_STAGES; 0) */
#define HLC_OPT_WIRE_PIPELINE 13   /* 0: the unpipelined wire host entry (A/B arm; HLC_WIRE_PIPELINE; 1) */
#define HLC_OPT_WIRE_WALK 14       /* -1 the build's wire walker, 0 one lane per message, 1 the LDS walker
                                      (HLC_WIRE_WALK = "lane" / "lds") */
#define HLC_OPT_SPLIT_VOTES_APPEND 15      /* appends a range size to HLC_OPT_SPLIT_VOTES' list ("a,b,...") */
#define HLC_OPT_WIRE_SPLIT_BYTES_APPEND 16 /* appends a range size to HLC_OPT_WIRE_SPLIT_BYTES' list */
#define HLC_OPT_EARLY_COMB 17      /* bits: 1 device-resident calls, 2 host-buffer calls run the u1 G comb in
                                      the u2 R stage's tail (k_rec_ucomb + k_rec_add); clear: after it
                                      (k_rec_comb) (HLC_EARLY_COMB; 1) */
#define HLC_POOL_BIND_NONE 0       /* workers run on any CPU of the process's affinity mask (default since
                                      round 6: DESIGN.md §5, profiles/r06/numa_ab_*.txt) */
#define HLC_POOL_BIND_GPU 1        /* the CPUs of the GPU's NUMA node (the round-5 default) */
#define HLC_POOL_BIND_SOURCE 2     /* the CPUs of the NUMA node the call's input arena lives on, per call */
int hlc_ctx_set_option(hlc_ctx* ctx, int option, int64_t value);  /* HLC_EINVAL: unknown / out of range */
int hlc_ctx_get_option(hlc_ctx* ctx, int option, int64_t* value);  /* list options: their first entry */

/* Host threads (including the caller's) a new context stages host-buffer copies with by default:
 * HLC_HOST_THREADS when set, else min(16, hardware threads, the process's CPU share = the cgroup CPU
 * quota (or the hardware threads) / LOCAL_WORLD_SIZE, the ranks on the node). */
int hlc_host_threads(void);

/* With HLC_OPT_HOST_TRACE 1 or 2: the last host-buffer call's phase times on this context as JSON --
 * {"host": {phase: ms}, "device": {event: ms}, "facts": {...}}, ms from the call's start; "" after a
 * call made without tracing.  A copy taken under the context's lock, valid on the calling thread until
 * its next hlc_ctx_last_host_trace. */
const char* hlc_ctx_last_host_trace(hlc_ctx* ctx);

/* ---- Measurement hooks (bench.py roofline): HIP events on the launch stream ------ */
/* enable = HLC_TIMING_ALL (1, or any value but 0 and 2): every validate-many call times the signature
 * recovery (k_rec_prep's start on the context's second stream .. k_rec_addr's end on the launch stream),
 * the chain/tally kernels and the whole call; HLC_TIMING_RECOVERY (2): the recovery bracket alone.  The
 * events are bound to the kernels' own dispatches (hipExtLaunchKernelGGL), not recorded between them:
 * each bound kernel still costs the queue a few microseconds, so the recovery-only mode is the one a
 * throughput measurement runs under (bench.py). */
#define HLC_TIMING_ALL 1
#define HLC_TIMING_RECOVERY 2
int hlc_ctx_set_kernel_timing(hlc_ctx* ctx, int enable);
/* Waits for the recorded events, returns the summed device time (ms) and launch count of
 * the recovery and of whole validate-many calls since the previous take, then resets them. */
int hlc_ctx_take_kernel_time(hlc_ctx* ctx, double* recover_ms, uint64_t* recover_launches,
                             double* call_ms, uint64_t* calls);
/* The same for the chain-check + duplicate + tally kernels of each validate-many call
 * (validate_vote_chain, initialize_with_votes and the tally: utils.rs:175-286, session.rs:253-298). */
int hlc_ctx_take_chain_time(hlc_ctx* ctx, double* chain_ms, uint64_t* launches);
/* enable != 0: k_rec_main of every later validate-many call on device buffers (hlc_validate_proposals_device)
 * stamps each wave's core-clock and 100 MHz reference ticks over its life (s_memtime / s_memrealtime; one
 * store per wave at its end).  Diagnostic: bench.py turns it on for calls after its timed steps only. */
int hlc_ctx_set_clock_probe(hlc_ctx* ctx, int enable);
/* The shader clock (GHz) the stamped waves of the last such launch ran at: median, minimum and maximum over
 * the waves, and how many waves stamped.  HLC_EINVAL when no launch was stamped. */
int hlc_ctx_clock_probe(hlc_ctx* ctx, double* median_ghz, double* min_ghz, double* max_ghz, uint64_t* waves);

/* ---- Hot-path entry points (host buffers, blocking) ----------------------------- */

/* Replaces `utils::compute_vote_hash` (utils.rs:37-47) over a batch: out[n][32]. */
int hlc_compute_vote_hashes(hlc_ctx* ctx, const hlc_votes* votes, uint8_t* out_hash32);

/* Replaces `EthereumConsensusSigner::verify` (signing/ethereum.rs:66-97), the static
 * `ConsensusSignatureScheme::verify` of signing.rs:69-73, over a batch of n items.
 * Item i: identity = bytes[id_off[i] .. +id_len[i]], payload likewise, signature likewise.
 * out_status[i] = HLC_VERIFY_TRUE / HLC_VERIFY_FALSE / 1 + HLC_SCHEME_* (Err).
 * out_addr (optional, n*20) receives the recovered address when one exists.  At most 2^32 - 16
 * items per call; an item whose (offset, length) leaves the arena returns HLC_EINVAL with the
 * outputs untouched. */
int hlc_eth_verify_batch(hlc_ctx* ctx, uint64_t n, const uint8_t* bytes, uint64_t bytes_len,
                         const uint64_t* id_off, const uint32_t* id_len,
                         const uint64_t* payload_off, const uint32_t* payload_len,
                         const uint64_t* sig_off, const uint32_t* sig_len,
                         uint8_t* out_status, uint8_t* out_addr);

/* Validate-many: `ConsensusSession::from_proposal` (session.rs:198-221) for every
 * proposal, i.e. validate_proposal (utils.rs:106-120) + initialize_with_votes
 * (session.rs:253-298), as called by process_incoming_proposal (service.rs:273-274).
 * out_results[p]: per-proposal outcome.  out_vote_status[v] (optional): the per-vote
 * status of validate_proposal's loop body for that vote alone (proposal_id match, then
 * validate_vote, utils.rs:112-117, 127-171), with no short-circuit across votes; votes that no
 * proposal's [vote_begin, vote_begin + vote_count) range covers are not evaluated (status 0xFF).
 * Proposal ranges must not overlap.
 * out_vote_reason (optional): HLC_SCHEME_* per vote.  out_recovered (optional, n*20):
 * recovered signer address per vote (zeros when none). */
int hlc_validate_proposals(hlc_ctx* ctx, const hlc_votes* votes, const hlc_proposal* proposals,
                           uint64_t n_proposals, uint64_t now, hlc_result* out_results,
                           uint8_t* out_vote_status, uint8_t* out_vote_reason,
                           uint8_t* out_recovered);

/* Outcome counters of a validate-many call (what a proposal-sharded run
 * all-reduces): out_counts[s] = votes whose status byte is s, out_counts[32 + s] = proposals whose
 * result status is s (s < 32; a larger byte is counted in bin 31).  Device pointers, enqueued on
 * `stream` (NULL: the context's stream) after zeroing out_counts[0..63]; no host synchronisation. */
int hlc_outcome_counts_device(hlc_ctx* ctx, const uint8_t* vote_status, uint64_t n_votes,
                              const hlc_result* results, uint64_t n_proposals, uint64_t* out_counts,
                              void* stream);

/* Same, but every pointer (inside `votes`, `proposals`, and the outputs) is DEVICE memory
 * of the context's device, and the work is enqueued on `stream` (a hipStream_t, or NULL for
 * the context's stream) without host synchronisation.  Used when inputs are already
 * resident in HBM (bench.py).  The recovery's signature-only stage runs on a second stream the
 * context owns, forked from and joined back into `stream` by events.  A context's workspace
 * serves one call at a time: successive calls on one context must be ordered (the same stream,
 * or the caller's own synchronisation between streams).  Every field's (offset, length) must lie
 * inside votes->bytes[0, bytes_len): the device entry reads them without a host-side check (the
 * host-buffer entry checks every one and returns HLC_EINVAL; the device decoders and generators
 * only produce in-arena fields). */
int hlc_validate_proposals_device(hlc_ctx* ctx, const hlc_votes* votes,
                                  const hlc_proposal* proposals, uint64_t n_proposals,
                                  uint64_t now, hlc_result* out_results,
                                  uint8_t* out_vote_status, uint8_t* out_vote_reason,
                                  uint8_t* out_recovered, void* stream);

/* ---- Scheme-generic validate-many (any `ConsensusSignatureScheme`) --------------------------
 * `ConsensusService<Scope, Storage, Event, Signer>` is generic over the signature scheme
 * (service.rs:39-51, signing.rs:46-74); the reference's tests/custom_scheme_tests.rs runs it with a
 * non-Ethereum StubSigner.  These entries are hlc_validate_proposals with the scheme step of
 * validate_vote (utils.rs:150-158: `Signer::verify(vote_owner, encode(vote, signature cleared),
 * signature)`) supplied by the caller: verdicts[v] is that call's outcome for vote v --
 * HLC_VERIFY_TRUE, HLC_VERIFY_FALSE, or Err(Verify) as HLC_VERIFY_ERR (any value 2..HLC_VERIFY_ERR is
 * an Err whose value - 1 is reported back as the HLC_SCHEME_* reason, so hlc_eth_verify_batch's
 * statuses can be passed straight in).  Everything else runs on the device as in
 * hlc_validate_proposals: the proposal_id match, the empty-field checks and the SHA-256 vote-hash
 * recompute (which precede the scheme step, so a verdict is read only for votes that reach it),
 * the timestamp checks, validate_vote_chain, the duplicate-owner and count checks, the round limit
 * and the tally, with the first-error precedence of SURVEY.md Appendix B.  No Ethereum assumption
 * is made: identities and signatures may have any length, and no secp256k1 recovery runs.
 * Host buffers, blocking; verdicts has votes->n entries (HLC_EINVAL for a value above HLC_VERIFY_ERR). */
int hlc_validate_proposals_verdicts(hlc_ctx* ctx, const hlc_votes* votes, const hlc_proposal* proposals,
                                    uint64_t n_proposals, uint64_t now, const uint8_t* verdicts,
                                    hlc_result* out_results, uint8_t* out_vote_status, uint8_t* out_vote_reason);

/* Same with every pointer in DEVICE memory, enqueued on `stream` (NULL: the context's stream) without
 * host synchronisation.  A verdict above HLC_VERIFY_ERR is read as HLC_VERIFY_ERR. */
int hlc_validate_proposals_verdicts_device(hlc_ctx* ctx, const hlc_votes* votes, const hlc_proposal* proposals,
                                           uint64_t n_proposals, uint64_t now, const uint8_t* verdicts,
                                           hlc_result* out_results, uint8_t* out_vote_status,
                                           uint8_t* out_vote_reason, void* stream);

/* The payload a scheme verifies for each vote (utils.rs:150-152): the prost encoding of the Vote with
 * its signature cleared (consensus.proto:19-29: tags 20-27, proto3 defaults omitted), built on the
 * device.  out_off[n] / out_len[n] receive every payload's place in out_bytes and *out_total the bytes
 * they need; out_bytes (capacity `cap`) may be NULL to query the size.  When cap < *out_total nothing
 * is written to out_bytes and HLC_ERANGE is returned (out_off / out_len are still written). */
int hlc_encode_vote_payloads(hlc_ctx* ctx, const hlc_votes* votes, uint64_t* out_off, uint32_t* out_len,
                             uint8_t* out_bytes, uint64_t cap, uint64_t* out_total);

/* Batched `ConsensusService::handle_consensus_timeout` (service.rs:323-373)
 * over n sessions: a session already in ConsensusReached(r) keeps it; otherwise
 * calculate_consensus_result(..., is_timeout = true) (utils.rs:227-286) decides
 * ConsensusReached(r) or Failed.  out_state[i] = the new HLC_SESSION_* state;
 * out_status[i] = HLC_OK (Ok(result)) or HLC_INSUFFICIENT_VOTES_AT_TIMEOUT (Err). */
int hlc_consensus_timeout_batch(hlc_ctx* ctx, uint64_t n, const hlc_session_tally* sessions,
                                uint8_t* out_state, uint8_t* out_status);

/* ---- Signing side (generator / embedders simulating many peers) -- */

/* EthereumConsensusSigner::identity (ethereum.rs:54-56) for n private keys: out[n][20]. */
int hlc_eth_address_batch(hlc_ctx* ctx, uint64_t n, const uint8_t* priv32, uint8_t* out_addr20);

/* EthereumConsensusSigner::sign (ethereum.rs:58-64): EIP-191 prehash + RFC 6979 +
 * low-s + v in {27,28}, over n payloads; out_sig[n][65].  Keys must be in [1, n-1]. */
int hlc_eth_sign_batch(hlc_ctx* ctx, uint64_t n, const uint8_t* priv32, const uint8_t* bytes,
                       uint64_t bytes_len, const uint64_t* payload_off,
                       const uint32_t* payload_len, uint8_t* out_sig65);

/* Synthetic signed-vote workload of SURVEY.md §8d, generated on the device (the same bytes as
 * python/hashgraph_like_consensus/synth.py): n_proposals chains of votes_per_proposal distinct
 * voters each, every vote built like `build_vote` (utils.rs:55-98) and signed like
 * EthereumConsensusSigner::sign (ethereum.rs:58-64), for global proposals
 * [start_proposal, start_proposal + n_proposals) of the seed -- rank r of a sharded run generates
 * only its own shard.  Every pointer is DEVICE memory: out_votes->n must be
 * n_proposals * votes_per_proposal, out_votes->bytes must hold hlc_synth_arena_bytes() bytes;
 * out_proposals[n_proposals]; out_priv (optional, n * 32) receives the signer keys.
 * Enqueued on `stream` (NULL: the context's stream) without host synchronisation. */
uint64_t hlc_synth_arena_bytes(uint64_t n_proposals, uint32_t votes_per_proposal);
int hlc_synth_votes_device(hlc_ctx* ctx, uint64_t seed, uint64_t start_proposal, uint64_t n_proposals,
                           uint32_t votes_per_proposal, uint32_t expected_voters, int gossipsub,
                           const hlc_votes* out_votes, hlc_proposal* out_proposals, uint8_t* out_priv,
                           void* stream);

/* SURVEY.md §8d config 5 on the device: turns a batch made by hlc_synth_votes_device with the
 * same (seed, start_proposal, n_proposals, votes_per_proposal) into the 1/3-Byzantine mix, in
 * place, by product code only (re-hashing and re-signing on the device), and reports each vote's
 * mutation kind in out_kind[n] (HLC_BYZ_*).  Every kind is built to have one validate_vote /
 * from_proposal outcome (hlc_synth.hip; the host-side expectation is
 * python/hashgraph_like_consensus/byzantine.py).  Device pointers, enqueued on `stream`. */
#define HLC_BYZ_NONE 0
#define HLC_BYZ_WRONG_KEY 1     /* InvalidVoteSignature */
#define HLC_BYZ_FLIP_S 2        /* InvalidVoteSignature */
#define HLC_BYZ_BAD_V 3         /* SignatureScheme, parity */
#define HLC_BYZ_HIGH_S 4        /* Ok: alloy normalises a high s */
#define HLC_BYZ_NO_POINT 5      /* SignatureScheme, no point */
#define HLC_BYZ_INFINITY 6      /* SignatureScheme, Q = infinity */
#define HLC_BYZ_TAMPER_HASH 7   /* InvalidVoteHash */
#define HLC_BYZ_SIG_LEN 8       /* SignatureScheme, length */
#define HLC_BYZ_EMPTY_OWNER 9   /* EmptyVoteOwner */
#define HLC_BYZ_EMPTY_HASH 10   /* EmptyVoteHash */
#define HLC_BYZ_EMPTY_SIG 11    /* EmptySignature */
#define HLC_BYZ_WRONG_PID 12    /* VoteProposalIdMismatch */
#define HLC_BYZ_TS_OLD 13       /* TimestampOlderThanCreationTime */
#define HLC_BYZ_BAD_RECEIVED 14 /* per-vote Ok; chain ReceivedHashMismatch */
#define HLC_BYZ_TS_REGRESS 15   /* per-vote Ok; chain ReceivedHashMismatch */
#define HLC_BYZ_PARENT_OTHER 16 /* per-vote Ok; chain ParentHashMismatch */
#define HLC_BYZ_DUPLICATE 17    /* per-vote Ok; DuplicateVote */
int hlc_synth_byzantine_device(hlc_ctx* ctx, uint64_t seed, uint64_t start_proposal, uint64_t n_proposals,
                               uint32_t votes_per_proposal, const hlc_votes* votes, uint8_t* out_kind,
                               void* stream);

/* ---- Streaming votes ---------------------------------------------- */

/* `ConsensusService::process_incoming_vote` (service.rs:286-305) for n votes delivered in
 * array order, micro-batched across sessions.  vote_session[i] = index into sessions[] of the
 * session the embedder's storage returns for (scope, vote.proposal_id), or 0xFFFFFFFF when
 * there is none (HLC_SESSION_NOT_FOUND); a session whose proposal_id differs from the vote's is
 * a caller mapping error, reported as HLC_VOTE_PROPOSAL_ID_MISMATCH.
 * Each vote gets exactly the outcome of the reference's
 * sequential calls: validate_vote against the session's proposal (utils.rs:127-171, the same
 * kernels as validate-many), then ConsensusSession::add_vote (session.rs:225-249): a session
 * already in ConsensusReached(r) returns it without inserting, Failed -> SessionNotActive,
 * expiry -> ProposalExpired, check_round_limit(1) -> MaxRoundsExceeded (and Failed),
 * owner already in the map (existing owners or an earlier vote of this batch) -> DuplicateVote,
 * else insert, update_round(1), check_consensus.  sessions[] is updated in place.
 * Existing owner maps: owners[k*20 .. +20] belongs to sessions[owner_session[k]] (20-byte
 * addresses, the only identities EthereumConsensusSigner admits).
 * Per vote: out_status = HLC_OK or the error; out_transition = HLC_STILL_ACTIVE /
 * HLC_REACHED_NO / HLC_REACHED_YES when OK; out_inserted = 1 when the vote entered the map
 * (the caller appends it to the session's proposal.votes); out_reason (optional) = HLC_SCHEME_*. */
int hlc_process_votes(hlc_ctx* ctx, const hlc_votes* votes, const uint32_t* vote_session,
                      hlc_session* sessions, uint64_t n_sessions, const uint8_t* owners,
                      const uint32_t* owner_session, uint64_t n_owners, uint64_t now,
                      uint8_t* out_status, uint8_t* out_transition, uint8_t* out_inserted,
                      uint8_t* out_reason);

/* Same with every pointer (inside `votes`, vote_session, sessions, owners, owner_session and the
 * outputs) in DEVICE memory, enqueued on `stream` (NULL: the context's stream); sessions are
 * updated in place on the device.  vote_session entries must be < n_sessions or 0xFFFFFFFF
 * (not re-checked on the host). */
int hlc_process_votes_device(hlc_ctx* ctx, const hlc_votes* votes, const uint32_t* vote_session,
                             hlc_session* sessions, uint64_t n_sessions, const uint8_t* owners,
                             const uint32_t* owner_session, uint64_t n_owners, uint64_t now,
                             uint8_t* out_status, uint8_t* out_transition, uint8_t* out_inserted,
                             uint8_t* out_reason, void* stream);

/* Scheme-generic form of hlc_process_votes (any `ConsensusSignatureScheme`, service.rs:39-51): the
 * scheme step of validate_vote is the caller's, verdicts[n] exactly as for
 * hlc_validate_proposals_verdicts, and the existing owner maps hold identities of any length: owner k
 * is owner_bytes[owner_off[k] .. + owner_len[k]] (inside [0, owner_bytes_len)) of session
 * owner_session[k].  Host buffers, blocking; the outcomes are those of hlc_process_votes. */
int hlc_process_votes_verdicts(hlc_ctx* ctx, const hlc_votes* votes, const uint32_t* vote_session,
                               hlc_session* sessions, uint64_t n_sessions, const uint8_t* owner_bytes,
                               uint64_t owner_bytes_len, const uint64_t* owner_off, const uint32_t* owner_len,
                               const uint32_t* owner_session, uint64_t n_owners, uint64_t now,
                               const uint8_t* verdicts, uint8_t* out_status, uint8_t* out_transition,
                               uint8_t* out_inserted, uint8_t* out_reason);

/* ---- Wire decode -------------------------------------------------- */

/* prost `Proposal::decode` (consensus.proto:5-29) on the device for n_msgs messages, message i =
 * wire[msg_off[i] .. + msg_len[i]] (messages may share or overlap bytes).  scope has n_scope
 * entries: 1 (shared by every message) or n_msgs.
 * out_props[i]: the message's hlc_proposal (vote_begin / vote_count into the decoded votes,
 * scalars from the message and scope[i]); vote_count = 0 when decoding failed.
 * out_wire[i] (optional): decode status and the remaining fields.
 * Decoded votes: *inout_n_votes is the capacity of the vote arrays on entry and the number of
 * decoded vote records on return; field_off values index `wire` itself.  When the capacity is
 * too small nothing is written to the vote arrays and HLC_ERANGE is returned (out_props and
 * out_wire are still written).  Vote arrays may all be NULL to query the count. */
int hlc_decode_proposals(hlc_ctx* ctx, const uint8_t* wire, uint64_t wire_len, const uint64_t* msg_off,
                         const uint32_t* msg_len, uint64_t n_msgs, const hlc_scope_config* scope,
                         uint64_t n_scope, hlc_proposal* out_props, hlc_wire_proposal* out_wire,
                         uint64_t* inout_n_votes, uint32_t* vote_id, uint32_t* proposal_id,
                         uint64_t* timestamp, uint8_t* vote, uint64_t* field_off, uint32_t* field_len);

/* `process_incoming_proposal` (service.rs:263-279) from wire bytes: device decode, then the
 * validate-many pipeline of hlc_validate_proposals on the decoded proposals, with no host
 * round trip of the votes.  out_results[i].status = HLC_PROPOSAL_DECODE_ERROR (scheme_reason =
 * HLC_WIRE_* reason, bad_index = failing vote record or 0xFFFFFFFF) when message i does not
 * decode, else the from_proposal outcome.  out_wire (optional) as in hlc_decode_proposals;
 * out_n_votes (optional) receives the number of decoded vote records. */
int hlc_validate_wire_proposals(hlc_ctx* ctx, const uint8_t* wire, uint64_t wire_len,
                                const uint64_t* msg_off, const uint32_t* msg_len, uint64_t n_msgs,
                                const hlc_scope_config* scope, uint64_t n_scope, uint64_t now,
                                hlc_result* out_results, hlc_wire_proposal* out_wire,
                                uint64_t* out_n_votes);

/* Same with every pointer in DEVICE memory, enqueued on `stream` (NULL: the context's stream).
 * One host synchronisation reads the decoded vote count (to size the workspace). */
int hlc_validate_wire_proposals_device(hlc_ctx* ctx, const uint8_t* wire, uint64_t wire_len,
                                       const uint64_t* msg_off, const uint32_t* msg_len,
                                       uint64_t n_msgs, const hlc_scope_config* scope,
                                       uint64_t n_scope, uint64_t now, hlc_result* out_results,
                                       hlc_wire_proposal* out_wire, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HLC_H */
