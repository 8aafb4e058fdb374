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
 * the outputs untouched.  Exit status 0 when every check holds (tests/test_gpu_c_abi.py runs it).
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

  hlc_ctx_destroy(ctx);
  free(arena);
  free(payloads);
  printf("hlc_abi_demo ok: %d items signed, verified Ok(true); 5 broken items classified; arena bounds enforced\n", N);
  return 0;
}
