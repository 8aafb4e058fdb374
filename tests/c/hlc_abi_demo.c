/*
 * hlc_abi_demo.c -- the drop-in boundary driven from plain C11, as a non-Python embedder (the
 * Rust `hlc-sys` crate of INTEGRATION.md, a cgo / JNI stub) would drive it: include/hlc.h and
 * libhlc.so only, no HIP or torch headers.
 *
 * It signs N payloads with N keys (hlc_eth_sign_batch, EthereumConsensusSigner::sign), derives the
 * identities (hlc_eth_address_batch, ::identity), packs [identity | payload | signature] per item
 * into one arena and verifies the batch (hlc_eth_verify_batch, ConsensusSignatureScheme::verify of
 * signing.rs:69-73): every honest item Ok(true) with its own address; then items broken the ways
 * ethereum.rs:66-97 distinguishes (wrong identity, tampered payload, 64-byte signature, 19-byte
 * identity, bad v) give Ok(false) or Err(reason); an item outside the arena returns HLC_EINVAL with
 * the outputs untouched.  Then a non-Ethereum scheme of its own through the scheme-generic entries
 * (hlc_compute_vote_hashes, hlc_encode_vote_payloads, hlc_validate_proposals_verdicts: generic_scheme
 * below).  Exit status 0 when every check holds (tests/test_gpu_c_abi.py runs it).
 *
 * Build (gcc, from the repository root; __graft_entry__.build() does this):
 *   gcc -O2 -std=c11 -Wall -Iinclude tests/c/hlc_abi_demo.c -Lhashgraph-like-consensus_amd/lib -lhlc \
 *       -Wl,-rpath,'$ORIGIN/../../hashgraph-like-consensus_amd/lib' -o tests/c/hlc_abi_demo
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hlc.h"

#define N 1000
#define FAIL(...)                     \
  do {                                \
    fprintf(stderr, __VA_ARGS__);     \
    fprintf(stderr, "\n");            \
    return 1;                         \
  } while (0)
#define API(call)                                                                  \
  do {                                                                             \
    int rc_ = (call);                                                              \
    if (rc_ != HLC_SUCCESS) FAIL("%s -> %d (%s)", #call, rc_, hlc_last_error());   \
  } while (0)

static uint64_t rng = 0x484C4341424931ull;
static uint32_t next32(void) {  // xorshift64*
  rng ^= rng >> 12;
  rng ^= rng << 25;
  rng ^= rng >> 27;
  return (uint32_t)((rng * 0x2545F4914F6CDD1Dull) >> 32);
}

// ---- a non-Ethereum scheme, as an embedder's own ConsensusSignatureScheme would be (the reference's
// tests/custom_scheme_tests.rs StubSigner has the same shape: 8-byte identities, a keyless "signature"
// over identity || payload).  Here: FNV-1a-64 of identity || payload, 8 bytes.  verify: Err unless the
// identity is 8 bytes, else Ok(signature == toy_sign(identity, payload)).
static void toy_sign(const uint8_t* id, uint32_t idl, const uint8_t* p, uint32_t pl, uint8_t out[8]) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t k = 0; k < idl; ++k) h = (h ^ id[k]) * 1099511628211ull;
  for (uint32_t k = 0; k < pl; ++k) h = (h ^ p[k]) * 1099511628211ull;
  for (int k = 0; k < 8; ++k) out[k] = (uint8_t)(h >> (8 * k));
}
static uint8_t toy_verify(const uint8_t* id, uint32_t idl, const uint8_t* p, uint32_t pl, const uint8_t* sig,
                          uint32_t sl) {
  if (idl != 8) return HLC_VERIFY_ERR;
  uint8_t want[8];
  toy_sign(id, idl, p, pl, want);
  return (sl == 8 && !memcmp(sig, want, 8)) ? HLC_VERIFY_TRUE : HLC_VERIFY_FALSE;
}

// from_proposal::<ToyScheme> for P proposals of V chained votes through hlc_validate_proposals_verdicts:
// the votes' hashes come from the device (hlc_compute_vote_hashes, one position at a time, since each
// vote's received_hash is the previous vote's hash), the payloads from hlc_encode_vote_payloads, the
// verdicts from toy_verify on the host.  All Ok -> ConsensusReached(true); then a forged signature is
// InvalidVoteSignature and a 7-byte identity the scheme's Err (SignatureScheme, HLC_SCHEME_PLUGIN).
#define P 4
#define V 3
static int generic_scheme(hlc_ctx* ctx) {
  enum { SLOT = 8 + 32 + 32 + 8 };  // owner | received | vote_hash | signature
  static uint8_t arena[P * V * SLOT];
  static uint32_t vid[P * V], pid[P * V];
  static uint64_t ts[P * V], foff[P * V * HLC_NFIELDS];
  static uint8_t vote[P * V];
  static uint32_t flen[P * V * HLC_NFIELDS];
  const uint64_t T0 = 1760000000ull;
  for (int p = 0; p < P; ++p)
    for (int j = 0; j < V; ++j) {
      const int i = p * V + j;
      vid[i] = next32() | 1u;
      pid[i] = 7000u + (uint32_t)p;
      ts[i] = T0 + 1 + (uint64_t)j;
      vote[i] = 1;
      uint8_t* slot = arena + (size_t)SLOT * i;
      for (int k = 0; k < 8; ++k) slot[k] = (uint8_t)(0x10 * p + j + 1);
      foff[i * HLC_NFIELDS + HLC_F_OWNER] = (uint64_t)SLOT * i;
      flen[i * HLC_NFIELDS + HLC_F_OWNER] = (p == 3 && j == 1) ? 7 : 8;  // proposal 3: one 7-byte identity
      foff[i * HLC_NFIELDS + HLC_F_PARENT] = 0;
      flen[i * HLC_NFIELDS + HLC_F_PARENT] = 0;
      foff[i * HLC_NFIELDS + HLC_F_RECEIVED] = (uint64_t)SLOT * i + 8;
      flen[i * HLC_NFIELDS + HLC_F_RECEIVED] = j ? 32 : 0;
      foff[i * HLC_NFIELDS + HLC_F_VOTE_HASH] = (uint64_t)SLOT * i + 40;
      flen[i * HLC_NFIELDS + HLC_F_VOTE_HASH] = 32;
      foff[i * HLC_NFIELDS + HLC_F_SIGNATURE] = (uint64_t)SLOT * i + 72;
      flen[i * HLC_NFIELDS + HLC_F_SIGNATURE] = 8;
    }
  hlc_votes all = {P * V, vid, pid, ts, vote, arena, sizeof arena, foff, flen};
  static uint8_t h[P * V * 32];
  for (int j = 0; j < V; ++j) {  // build_vote (utils.rs:55-98): received = the previous vote's hash
    API(hlc_compute_vote_hashes(ctx, &all, h));
    for (int p = 0; p < P; ++p) {
      const int i = p * V + j;
      memcpy(arena + foff[i * HLC_NFIELDS + HLC_F_VOTE_HASH], h + 32 * i, 32);
      if (j + 1 < V) memcpy(arena + foff[(i + 1) * HLC_NFIELDS + HLC_F_RECEIVED], h + 32 * i, 32);
    }
  }
  static uint64_t poff[P * V];
  static uint32_t plen[P * V];
  static uint8_t pay[P * V * 256];
  uint64_t ptotal = 0;
  API(hlc_encode_vote_payloads(ctx, &all, poff, plen, pay, sizeof pay, &ptotal));
  for (int i = 0; i < P * V; ++i)  // every voter signs its payload
    toy_sign(arena + foff[i * HLC_NFIELDS + HLC_F_OWNER], flen[i * HLC_NFIELDS + HLC_F_OWNER], pay + poff[i], plen[i],
             arena + foff[i * HLC_NFIELDS + HLC_F_SIGNATURE]);
  arena[foff[(1 * V + 2) * HLC_NFIELDS + HLC_F_SIGNATURE]] ^= 0xFF;  // proposal 1, vote 2: forged
  static uint8_t verdict[P * V];
  for (int i = 0; i < P * V; ++i)
    verdict[i] = toy_verify(arena + foff[i * HLC_NFIELDS + HLC_F_OWNER], flen[i * HLC_NFIELDS + HLC_F_OWNER],
                            pay + poff[i], plen[i], arena + foff[i * HLC_NFIELDS + HLC_F_SIGNATURE],
                            flen[i * HLC_NFIELDS + HLC_F_SIGNATURE]);
  hlc_proposal props[P];
  memset(props, 0, sizeof props);
  for (int p = 0; p < P; ++p) {
    props[p].vote_begin = (uint64_t)p * V;
    props[p].vote_count = V;
    props[p].proposal_id = 7000u + (uint32_t)p;
    props[p].timestamp = T0;
    props[p].expiration_timestamp = T0 + 3600;
    props[p].expected_voters_count = V;
    props[p].max_rounds = 2;
    props[p].consensus_threshold = 2.0 / 3.0;
    props[p].use_gossipsub_rounds = 1;
    props[p].liveness_criteria_yes = 1;
  }
  hlc_result res[P];
  uint8_t vst[P * V], vrs[P * V];
  API(hlc_validate_proposals_verdicts(ctx, &all, props, P, T0 + 1800, verdict, res, vst, vrs));
  const uint8_t want_status[P] = {HLC_OK, HLC_INVALID_VOTE_SIGNATURE, HLC_OK, HLC_SIGNATURE_SCHEME};
  for (int p = 0; p < P; ++p) {
    if (res[p].status != want_status[p]) FAIL("toy scheme: proposal %d status %d, want %d", p, res[p].status, want_status[p]);
    if (res[p].status == HLC_OK && (res[p].transition != HLC_REACHED_YES || res[p].yes != V || res[p].total != V))
      FAIL("toy scheme: proposal %d did not reach consensus YES", p);
  }
  if (res[1].bad_index != 2 || res[3].bad_index != 1 || res[3].scheme_reason != HLC_SCHEME_PLUGIN)
    FAIL("toy scheme: first-error index / reason wrong");
  if (vst[V + 2] != HLC_INVALID_VOTE_SIGNATURE || vst[3 * V + 1] != HLC_SIGNATURE_SCHEME || vrs[3 * V + 1] != HLC_SCHEME_PLUGIN)
    FAIL("toy scheme: per-vote statuses wrong");
  // the same batch under EthereumConsensusSigner rejects every vote: 8-byte signatures, 8-byte identities
  API(hlc_validate_proposals(ctx, &all, props, P, T0 + 1800, res, vst, vrs, NULL));
  if (res[0].status != HLC_SIGNATURE_SCHEME || res[0].scheme_reason != HLC_SCHEME_SIG_LEN)
    FAIL("Ethereum scheme accepted a toy-scheme vote");
  return 0;
}


int main(void) {
  if (hlc_abi_version() != HLC_ABI_VERSION) FAIL("ABI version %d, header %d", hlc_abi_version(), HLC_ABI_VERSION);
  hlc_ctx* ctx = NULL;
  API(hlc_ctx_create(0, &ctx));

  static uint8_t priv[N * 32], addr[N * 20], sig[N * 65];
  static uint64_t poff[N];
  static uint32_t plen[N];
  uint64_t ptotal = 0;
  for (int i = 0; i < N; ++i) {
    priv[32 * i] = 0x11;  // below the group order
    for (int k = 1; k < 32; ++k) priv[32 * i + k] = (uint8_t)next32();
    plen[i] = 100 + next32() % 51;  // 100..150 bytes: a prost-encoded vote's size
    poff[i] = ptotal;
    ptotal += plen[i];
  }
  uint8_t* payloads = malloc(ptotal);
  for (uint64_t b = 0; b < ptotal; ++b) payloads[b] = (uint8_t)next32();
  API(hlc_eth_address_batch(ctx, N, priv, addr));
  API(hlc_eth_sign_batch(ctx, N, priv, payloads, ptotal, poff, plen, sig));

  // one arena: [identity 20 | payload | signature 65] per item, with (offset, length) arrays
  const uint64_t total = ptotal + (uint64_t)N * (20 + 65);
  uint8_t* arena = malloc(total);
  static uint64_t id_off[N], pay_off[N], sig_off[N];
  static uint32_t id_len[N], pay_len[N], sig_len[N];
  uint64_t pos = 0;
  for (int i = 0; i < N; ++i) {
    id_off[i] = pos;
    id_len[i] = 20;
    memcpy(arena + pos, addr + 20 * i, 20);
    pos += 20;
    pay_off[i] = pos;
    pay_len[i] = plen[i];
    memcpy(arena + pos, payloads + poff[i], plen[i]);
    pos += plen[i];
    sig_off[i] = pos;
    sig_len[i] = 65;
    memcpy(arena + pos, sig + 65 * i, 65);
    pos += 65;
  }

  static uint8_t st[N], rec[N * 20];
  API(hlc_eth_verify_batch(ctx, N, arena, total, id_off, id_len, pay_off, pay_len, sig_off, sig_len, st, rec));
  for (int i = 0; i < N; ++i) {
    if (st[i] != HLC_VERIFY_TRUE) FAIL("honest item %d: status %d", i, st[i]);
    if (memcmp(rec + 20 * i, addr + 20 * i, 20)) FAIL("honest item %d: recovered another address", i);
  }

  // the item-level outcomes ethereum.rs:66-97 distinguishes
  arena[id_off[1]] ^= 0x01;                 // another identity: Ok(false)
  arena[pay_off[2] + 7] ^= 0x80;            // tampered payload: Ok(false)
  sig_len[3] = 64;                          // ethereum.rs:71-76
  id_len[4] = 19;                           // ethereum.rs:77-82
  arena[sig_off[5] + 64] = 30;              // v outside {0, 1, 27, 28, >= 35}
  API(hlc_eth_verify_batch(ctx, N, arena, total, id_off, id_len, pay_off, pay_len, sig_off, sig_len, st, rec));
  const uint8_t want[6] = {HLC_VERIFY_TRUE, HLC_VERIFY_FALSE, HLC_VERIFY_FALSE, 1 + HLC_SCHEME_SIG_LEN,
                           1 + HLC_SCHEME_ID_LEN, 1 + HLC_SCHEME_BAD_PARITY};
  for (int i = 0; i < 6; ++i)
    if (st[i] != want[i]) FAIL("item %d: status %d, want %d", i, st[i], want[i]);
  for (int i = 6; i < N; ++i)
    if (st[i] != HLC_VERIFY_TRUE) FAIL("untouched item %d: status %d", i, st[i]);

  // an item outside the arena: HLC_EINVAL, outputs untouched
  memset(st, 0xAB, sizeof st);
  pay_off[N - 1] = total + 1;
  if (hlc_eth_verify_batch(ctx, N, arena, total, id_off, id_len, pay_off, pay_len, sig_off, sig_len, st, rec) !=
      HLC_EINVAL)
    FAIL("out-of-arena payload not rejected");
  for (int i = 0; i < N; ++i)
    if (st[i] != 0xAB) FAIL("outputs written on HLC_EINVAL (item %d)", i);

  if (generic_scheme(ctx)) return 1;

  hlc_ctx_destroy(ctx);
  free(arena);
  free(payloads);
  printf("hlc_abi_demo ok: %d items signed, verified Ok(true); 5 broken items classified; arena bounds enforced; "
         "a non-Ethereum scheme's verdicts validated %d proposals\n", N, P);
  return 0;
}
