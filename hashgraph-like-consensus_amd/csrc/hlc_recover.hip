// hlc_recover.hip -- the VALU-bound kernels: batch ecrecover (the hot path),
// table construction, and the signing side (address derivation, RFC 6979 signing).
#include "hlc_kernels.h"
#include "hlc_recover.hpp"

namespace hlc {

namespace {

constexpr int REC_TPB = 256;
#ifndef HLC_REC_WAVES
#define HLC_REC_WAVES 4  // waves per SIMD the register allocator must admit for k_recover
#endif

__device__ __forceinline__ uint32_t load_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
__device__ __forceinline__ uint32_t load_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
// 32 big-endian bytes -> limbs
__device__ __forceinline__ void fe_load_be(fe& r, const uint8_t* p) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[7 - i] = load_be32(p + 4 * i);
}
__device__ __forceinline__ void fe_store_be(uint8_t* p, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t w = a.v[7 - i];
    p[4 * i] = (uint8_t)(w >> 24);
    p[4 * i + 1] = (uint8_t)(w >> 16);
    p[4 * i + 2] = (uint8_t)(w >> 8);
    p[4 * i + 3] = (uint8_t)w;
  }
}
// digest stored as 8 memory-order words -> big-endian integer limbs
__device__ __forceinline__ void fe_from_digest(fe& r, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[7 - i] = bswap32(w[i]);
}

__global__ void __launch_bounds__(REC_TPB, HLC_REC_WAVES) k_recover(uint64_t n, const uint8_t* pre, const uint32_t* z_digest,
                                                     const uint8_t* bytes, const uint64_t* sig_off,
                                                     const uint64_t* id_off, size_t off_stride,
                                                     const uint32_t* gcomb, uint32_t* scratch, uint64_t lanes,
                                                     uint8_t* verify_out, uint8_t* addr_out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t* ws = scratch + tid;
  uint32_t* tab = scratch + (size_t)IL_WORDS * lanes + (size_t)tid * RTAB_WORDS;
  for (uint64_t i = tid; i < n; i += lanes) {
    if (pre && pre[i] != PRE_PENDING) continue;
    const uint8_t* sig = bytes + sig_off[i * off_stride];
    fe r, s, z;
    fe_load_be(r, sig);
    fe_load_be(s, sig + 32);
    fe_from_digest(z, z_digest + 8 * i);
    uint32_t addr[5];
    int code = ecrecover_lane(z, r, s, sig[64], addr, gcomb, ws, lanes, tab);
    uint8_t vr;
    if (code != SCHEME_NONE) {
      vr = (uint8_t)(1 + code);
#pragma unroll
      for (int k = 0; k < 5; ++k) addr[k] = 0;
    } else {
      const uint8_t* id = bytes + id_off[i * off_stride];
      uint32_t diff = 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) diff |= addr[k] ^ load_le32(id + 4 * k);
      vr = diff == 0 ? HLC_VERIFY_TRUE : HLC_VERIFY_FALSE;
    }
    verify_out[i] = vr;
    if (addr_out) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        addr_out[20 * i + 4 * k] = (uint8_t)addr[k];
        addr_out[20 * i + 4 * k + 1] = (uint8_t)(addr[k] >> 8);
        addr_out[20 * i + 4 * k + 2] = (uint8_t)(addr[k] >> 16);
        addr_out[20 * i + 4 * k + 3] = (uint8_t)(addr[k] >> 24);
      }
    }
  }
}

// k*P for small k by plain double-and-add from the generator (table construction only)
__device__ void scalar_mul_g(gej& acc, const fe& k) {
  ge g;
  ge_generator(g);
  gej_set_inf(acc);
  for (int bit = 255; bit >= 0; --bit) {
    gej_double(acc, acc);
    if ((k.v[bit >> 5] >> (bit & 31)) & 1u) gej_add_ge(acc, acc, g);
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

// k*G via the 8-bit comb (k < n)
__device__ void fixed_base_mul(gej& acc, const fe& k, const uint32_t* fb) {
  gej_set_inf(acc);
  for (int w = 0; w < 32; ++w) {
    uint32_t j = (k.v[w >> 2] >> (8 * (w & 3))) & 0xFFu;
    if (j) {
      ge g;
      load_ge_global(g, fb + (size_t)(w * 256 + j) * 16);
      gej_add_ge(acc, acc, g);
    }
  }
}

// The u1 G comb of the recovery (hlc_recover.hpp): T[w][j] = (2j+1) 2^(16w) G, affine, and the
// constant top point 2^256 G.  One thread per entry, from the signing comb fbtab.
__global__ void k_build_gcomb(uint32_t* gcomb, const uint32_t* fb) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = (uint64_t)GC_WINDOWS * GC_ENTRIES + 1;
  if (e >= total) return;
  fe k;
  fe_set(k, 0);
  if (e == total - 1) {
    // 2^256 mod n = 2^256 - n
    uint32_t bw = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) k.v[q] = sub_cc(0u, n_limb(q), bw);
  } else {
    const int w = (int)(e / GC_ENTRIES), j = (int)(e % GC_ENTRIES);
    const uint32_t m = 2u * (uint32_t)j + 1u;  // < 2^16
    const int bit = GC_W * w;
    k.v[bit >> 5] = m << (bit & 31);
    if ((bit & 31) > 16 && (bit >> 5) < 7) k.v[(bit >> 5) + 1] = m >> (32 - (bit & 31));
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

// ---- HMAC-SHA256 over short byte strings held in private memory (RFC 6979) ----
__device__ void sha256_bytes(const uint8_t* pre64, const uint8_t* msg, int len, uint32_t h[8]) {
  // hashes pre64 (64 bytes, may be null) || msg (len bytes)
  sha256_init(h);
  uint32_t w[16];
  int total = (pre64 ? 64 : 0) + len;
  if (pre64) {
    for (int k = 0; k < 16; ++k) w[k] = ((uint32_t)pre64[4 * k] << 24) | ((uint32_t)pre64[4 * k + 1] << 16) |
                                        ((uint32_t)pre64[4 * k + 2] << 8) | pre64[4 * k + 3];
    sha256_compress(h, w);
  }
  // remaining message with padding
  int nblk = (len + 9 + 63) / 64;
  for (int b = 0; b < nblk; ++b) {
    uint32_t ww[16];
    for (int k = 0; k < 16; ++k) {
      uint32_t x = 0;
      for (int t = 0; t < 4; ++t) {
        int pos = b * 64 + 4 * k + t;
        uint8_t byte;
        if (pos < len) byte = msg[pos];
        else if (pos == len) byte = 0x80;
        else byte = 0;
        x = (x << 8) | byte;
      }
      ww[k] = x;
    }
    if (b == nblk - 1) {
      uint64_t bits = (uint64_t)total * 8;
      ww[14] = (uint32_t)(bits >> 32);
      ww[15] = (uint32_t)bits;
    }
    sha256_compress(h, ww);
  }
}

__device__ void hmac_sha256(const uint8_t key[32], const uint8_t* msg, int len, uint8_t out[32]) {
  uint8_t pad[64];
  uint32_t ih[8], oh[8];
  for (int k = 0; k < 64; ++k) pad[k] = (k < 32 ? key[k] : 0) ^ 0x36;
  sha256_bytes(pad, msg, len, ih);
  uint8_t inner[32];
  for (int k = 0; k < 8; ++k) {
    inner[4 * k] = (uint8_t)(ih[k] >> 24);
    inner[4 * k + 1] = (uint8_t)(ih[k] >> 16);
    inner[4 * k + 2] = (uint8_t)(ih[k] >> 8);
    inner[4 * k + 3] = (uint8_t)ih[k];
  }
  for (int k = 0; k < 64; ++k) pad[k] = (k < 32 ? key[k] : 0) ^ 0x5c;
  sha256_bytes(pad, inner, 32, oh);
  for (int k = 0; k < 8; ++k) {
    out[4 * k] = (uint8_t)(oh[k] >> 24);
    out[4 * k + 1] = (uint8_t)(oh[k] >> 16);
    out[4 * k + 2] = (uint8_t)(oh[k] >> 8);
    out[4 * k + 3] = (uint8_t)oh[k];
  }
}

// EthereumConsensusSigner::sign (signing/ethereum.rs:58-64) given the EIP-191 prehash:
// k256 sign_prehash_recoverable = RFC 6979 (HMAC-SHA256) nonce, low-s normalisation,
// alloy as_bytes() = r || s || (27 + y_parity).
__global__ void k_sign(uint64_t n, const uint8_t* priv, const uint32_t* z_digest, const uint32_t* fb,
                       uint8_t* sig_out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe d, zr, z;
  fe_load_be(d, priv + 32 * i);
  fe_from_digest(zr, z_digest + 8 * i);
  sc_reduce(z, zr);
  uint8_t x[32], h1[32];
  fe_store_be(x, d);
  fe_store_be(h1, z);
  uint8_t V[32], K[32], buf[97];
  for (int k = 0; k < 32; ++k) {
    V[k] = 1;
    K[k] = 0;
  }
  for (int step = 0; step < 2; ++step) {
    for (int k = 0; k < 32; ++k) buf[k] = V[k];
    buf[32] = (uint8_t)step;
    for (int k = 0; k < 32; ++k) {
      buf[33 + k] = x[k];
      buf[65 + k] = h1[k];
    }
    hmac_sha256(K, buf, 97, K);
    hmac_sha256(K, V, 32, V);
  }
  fe k;
  for (;;) {
    hmac_sha256(K, V, 32, V);
    fe_load_be(k, V);
    if (!fe_is_zero(k) && !sc_is_ge_n(k)) break;
    for (int q = 0; q < 32; ++q) buf[q] = V[q];
    buf[32] = 0;
    hmac_sha256(K, buf, 33, K);
    hmac_sha256(K, V, 32, V);
  }
  gej Rj;
  fixed_base_mul(Rj, k, fb);
  fe rx, ry, r;
  gej_to_affine(rx, ry, Rj);
  uint32_t y_odd = ry.v[0] & 1u;
  sc_reduce(r, rx);
  // s = k^-1 (z + r d) mod n
  fe r2c, km, kinv, rR, rd, t, s;
  sc_r2(r2c);
  sc_mont_mul(km, k, r2c);
  fe kinv_plain;
  sc_inv(kinv_plain, k);
  sc_mont_mul(kinv, kinv_plain, r2c);  // k^-1 * R
  sc_mont_mul(rR, r, r2c);
  sc_mont_mul(rd, rR, d);
  sc_add(t, z, rd);
  sc_mont_mul(s, kinv, t);
  fe h;
#pragma unroll
  for (int q = 0; q < 8; ++q) h.v[q] = nhalf_limb(q);
  if (u256_lt(h, s)) {
    sc_neg(s, s);
    y_odd ^= 1u;
  }
  uint8_t* o = sig_out + 65 * i;
  fe_store_be(o, r);
  fe_store_be(o + 32, s);
  o[64] = (uint8_t)(27 + y_odd);
}

inline unsigned blocks_for(uint64_t n, int tpb) { return (unsigned)((n + tpb - 1) / tpb); }

}  // namespace

uint64_t recover_scratch_words() { return SCRATCH_WORDS; }

uint64_t recover_grid_lanes() {
  int dev = 0, cus = 256, per_cu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_recover, REC_TPB, 0) != hipSuccess || per_cu < 1)
    per_cu = 2;
  return (uint64_t)cus * (uint64_t)per_cu * REC_TPB;
}

void launch_recover(uint64_t n, const uint8_t* pre, const uint32_t* z_digest, const uint8_t* bytes,
                    const uint64_t* sig_off, const uint64_t* id_off, size_t off_stride, const uint32_t* gcomb,
                    uint32_t* scratch, uint64_t scratch_lanes, uint8_t* verify_out, uint8_t* addr_out,
                    hipStream_t s) {
  if (!n) return;
  uint64_t blocks = scratch_lanes / REC_TPB;
  uint64_t need = (n + REC_TPB - 1) / REC_TPB;
  if (blocks > need) blocks = need;
  hipLaunchKernelGGL(k_recover, dim3((unsigned)blocks), dim3(REC_TPB), 0, s, n, pre, z_digest, bytes, sig_off,
                     id_off, off_stride, gcomb, scratch, (uint64_t)blocks * REC_TPB, verify_out, addr_out);
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
