#!/usr/bin/env python3
"""Generate hashgraph-like-consensus_amd/csrc/hlc_field_asm.hpp: hand-scheduled gfx950 field
multiplication and squaring mod p = 2^256 - 2^32 - 977, one inline-asm block each, plus the plain
512-bit product the scalar code uses.

Why asm: the compiler's lowering of a product scan with carry-out (v_mad_u64_u32 sdst) keeps
re-pairing 64-bit registers (~100 v_mov per product) and pads every carry read with s_nop.

Schedule
  * Product scanning: column k = sum_{i+j=k} a_i b_j is accumulated in a 96-bit (lo, hi, W)
    triple -- (lo, hi) is the current pair P of v[0:1] / v[2:3], W the high half of the other
    pair Q.  At the end of the column t_k = P.lo, and `v_mov Q.lo, P.hi` turns Q into the next
    column's accumulator (hi, W): one v_mov per column.
  * Carry-outs rotate over three SGPR pairs and are folded into W two MADs later, so every carry
    is read >= 2 instructions after it is written (the VALU-writes-SGPR -> VALU-reads-SGPR
    spacing the compiler keeps on gfx950); a checker inserts s_nop only where a short column
    leaves no filler.
  * The reduction (2^256 == K = 2^32 + 977) is interleaved with the scan: when column 8+i is
    complete its limb H_i is still in the accumulator; (ml_i, mh_i) = H_i * 977 and three carry
    chains add ml_i, mh_{i-1} and H_{i-1} into limb i of the low half.  The reduction's ops fill
    the scan's carry slots and the high limbs never leave the accumulator registers.  The top
    e < 2^33 is folded once more (e*K into limbs 0..2); the carry out of limb 2 (c3 <= 2, almost
    always 0) is returned for a rare C++ fix-up.
  * Squaring scans the 28 off-diagonal products the same way; each finished column is doubled
    (v_alignbit) and its diagonal square added on one more carry chain, and the limbs feed the
    same interleaved reduction.
Outputs are in [0, 2^256) (lazy: congruent mod p; hlc_field.hpp).

Run:  python tools/gen_field_asm.py > hashgraph-like-consensus_amd/csrc/hlc_field_asm.hpp
"""
import sys

PAIRS = [("v0", "v1"), ("v2", "v3")]
MP = [("v4", "v5"), ("v6", "v7")]          # H_i * 977 products (alternating)
DP = ("v8", "v9")                          # diagonal square a_i^2 (squaring)
T = "v10"                                  # doubled column (squaring)
TH = ["v11", "v12"]                        # high limbs H_i (squaring)
NCARRY = 3


def vp(p):
    return f"v[{p[0][1:]}:{p[1][1:]}]"


class Emitter:
    def __init__(self):
        self.ins = []  # (text, sgpr_written, sgpr_read)

    def emit(self, text, writes=None, reads=None):
        # a VALU read of an SGPR written by a VALU needs >= 2 instructions in between
        if reads is not None:
            for back in range(1, 3):
                if len(self.ins) < back:
                    break
                if self.ins[-back][1] == reads:
                    self.ins.append((f"s_nop {2 - back}", None, None))
                    break
        self.ins.append((text, writes, reads))

    def text(self):
        return [t for t, _, _ in self.ins]


def add(em, dst, src0, src1, chain, start):
    """dst = src0 + src1 (+ carry of `chain`), carry out into `chain`."""
    if start:
        em.emit(f"v_add_co_u32_e64 {dst}, {chain}, {src0}, {src1}", writes=chain)
    else:
        em.emit(f"v_addc_co_u32_e64 {dst}, {chain}, {src0}, {src1}, {chain}", writes=chain, reads=chain)


def scan(em, columns, a, b, first_zero, col_end, last_w_zero=True):
    """Product scan over `columns` [(k, [(i, j), ...])]; col_end(k, P, Q, last) runs at each
    column end after W is complete and before the transition."""
    cur = 0
    ctr = 0
    for ci, (k, prods) in enumerate(columns):
        P, Q = PAIRS[cur], PAIRS[1 - cur]
        W = Q[1]
        is_first = ci == 0 and first_zero
        is_last = ci == len(columns) - 1
        pending = []
        w_init = False
        for idx, (i, j) in enumerate(prods):
            c = f"%[c{ctr % NCARRY}]"
            ctr += 1
            addend = "0" if (is_first and idx == 0) else vp(P)
            em.emit(f"v_mad_u64_u32 {vp(P)}, {c}, {a(i)}, {b(j)}, {addend}", writes=c)
            if is_first and idx == 0:
                continue  # adding 0 never carries
            pending.append(c)
            if len(pending) > 2:
                cc = pending.pop(0)
                if not (is_last and last_w_zero):
                    em.emit(f"v_addc_co_u32_e64 {W}, {cc}, 0, {W if w_init else '0'}, {cc}", writes=cc, reads=cc)
                    w_init = True
        if not (is_last and last_w_zero):
            for cc in pending:
                em.emit(f"v_addc_co_u32_e64 {W}, {cc}, 0, {W if w_init else '0'}, {cc}", writes=cc, reads=cc)
                w_init = True
            if not w_init:
                em.emit(f"v_mov_b32 {W}, 0")
        col_end(k, P, Q, is_last)
        if is_last:
            return
        em.emit(f"v_mov_b32 {Q[0]}, {P[1]}")
        cur = 1 - cur


def red_step(em, i, H, Hm1):
    """Fold the high limb H_i (and H_{i-1}) into low limb r_i: the three reduction chains."""
    m = MP[i % 2]
    em.emit(f"v_mad_u64_u32 {vp(m)}, vcc, {H}, %[k977], 0")
    r = f"%[r{i}]"
    if i >= 1:
        add(em, r, r, Hm1, "%[cC]", i == 1)              # + H_{i-1} * 2^32
        add(em, r, r, MP[(i - 1) % 2][1], "%[cB]", i == 1)  # + hi(H_{i-1} * 977)
    add(em, r, r, m[0], "%[cA]", i == 0)                  # + lo(H_i * 977)


def red_tail(em, H7, tmp):
    """e = mh_7 + H_7 + carries (< 2^33) folded into limbs 0..2; c3 = carry out of limb 2."""
    e_lo, e_hi = tmp
    mh7 = MP[1][1]
    em.emit(f"v_addc_co_u32_e64 {e_lo}, %[cA], {mh7}, 0, %[cA]", writes="%[cA]", reads="%[cA]")
    em.emit(f"v_addc_co_u32_e64 {e_lo}, %[cB], {e_lo}, 0, %[cB]", writes="%[cB]", reads="%[cB]")
    em.emit(f"v_addc_co_u32_e64 {e_lo}, %[cC], {e_lo}, {H7}, %[cC]", writes="%[cC]", reads="%[cC]")
    em.emit(f"v_addc_co_u32_e64 {e_hi}, %[cC], 0, 0, %[cC]", writes="%[cC]", reads="%[cC]")
    # e*K = e_lo*977 + (e_hi*977 + e_lo) 2^32 + e_hi 2^64
    f = MP[0]
    em.emit(f"v_mad_u64_u32 {vp(f)}, vcc, {e_lo}, %[k977], 0")
    em.emit(f"v_mad_u32_u24 {f[1]}, {e_hi}, %[k977], {f[1]}")
    add(em, "%[r1]", "%[r1]", e_lo, "%[c1]", True)          # chain E: + e_lo
    add(em, "%[r0]", "%[r0]", f[0], "%[c0]", True)          # chain D: + f_lo
    add(em, "%[r2]", "%[r2]", e_hi, "%[c1]", False)         # E: + e_hi
    add(em, "%[r1]", "%[r1]", f[1], "%[c0]", False)         # D: + g
    em.emit("v_addc_co_u32_e64 %[c3], %[c1], 0, 0, %[c1]", writes="%[c1]", reads="%[c1]")
    add(em, "%[r2]", "%[r2]", "0", "%[c0]", False)          # D: limb 2
    em.emit("v_addc_co_u32_e64 %[c3], %[c0], %[c3], 0, %[c0]", writes="%[c0]", reads="%[c0]")


def gen_mul_fused():
    em = Emitter()
    cols = [(k, [(i, k - i) for i in range(max(0, k - 7), min(k, 7) + 1)]) for k in range(15)]

    def col_end(k, P, Q, last):
        if k < 8:
            em.emit(f"v_mov_b32 %[r{k}], {P[0]}")
            return
        red_step(em, k - 8, P[0], Q[0])
        if last:  # k == 14: P = (H_6, H_7)
            red_step(em, 7, P[1], P[0])
            red_tail(em, P[1], Q)

    scan(em, cols, lambda i: f"%[a{i}]", lambda j: f"%[b{j}]", True, col_end)
    return em.text()


def gen_sqr_fused():
    em = Emitter()
    cols = [(k, [(i, k - i) for i in range(max(0, k - 7), 8) if i < k - i]) for k in range(1, 14)]
    em.emit(f"v_mad_u64_u32 {vp(DP)}, vcc, %[a0], %[a0], 0")
    em.emit(f"v_mov_b32 %[r0], {DP[0]}")

    def limb(k, y):
        """t_k = y + (k even: lo(a_{k/2}^2), k odd: hi(a_{(k-1)/2}^2)) on chain D; then reduce."""
        if k % 2 == 0:
            em.emit(f"v_mad_u64_u32 {vp(DP)}, vcc, %[a{k // 2}], %[a{k // 2}], 0")
            src = DP[0]
        else:
            src = DP[1]
        dst = f"%[r{k}]" if k < 8 else TH[(k - 8) % 2]
        add(em, dst, y, src, "%[cD]", k == 1)
        if k >= 8:
            red_step(em, k - 8, dst, TH[(k - 9) % 2])

    def col_end(k, P, Q, last):
        if k == 1:
            em.emit(f"v_lshlrev_b32 {T}, 1, {P[0]}")
        else:
            em.emit(f"v_alignbit_b32 {T}, {P[0]}, {Q[0]}, 31")
        limb(k, T)
        if last:  # k == 13: x_14 = P.hi, x_15 = 0
            em.emit(f"v_alignbit_b32 {T}, {P[1]}, {P[0]}, 31")
            limb(14, T)
            em.emit(f"v_lshrrev_b32 {T}, 31, {P[1]}")
            limb(15, T)
            red_tail(em, TH[1], PAIRS[0])

    scan(em, cols, lambda i: f"%[a{i}]", lambda j: f"%[a{j}]", True, col_end)
    return em.text()


def gen_mul512():
    """Plain 512-bit product (scalar code: GLV rounding)."""
    em = Emitter()
    cols = [(k, [(i, k - i) for i in range(max(0, k - 7), min(k, 7) + 1)]) for k in range(15)]

    def col_end(k, P, Q, last):
        em.emit(f"v_mov_b32 %[t{k}], {P[0]}")
        if last:
            em.emit(f"v_mov_b32 %[t{k + 1}], {P[1]}")

    scan(em, cols, lambda i: f"%[a{i}]", lambda j: f"%[b{j}]", True, col_end)
    return em.text()


def asm_block(lines):
    return "\n".join(f'      "{l}\\n"' for l in lines)


def main():
    mul = gen_mul_fused()
    sqr = gen_sqr_fused()
    m512 = gen_mul512()
    o = sys.stdout
    o.write("// GENERATED by tools/gen_field_asm.py -- do not edit.  Hand-scheduled gfx950 field\n")
    o.write("// multiplication / squaring mod p (see the generator's docstring for the schedule and the\n")
    o.write("// hazard rule it keeps).  Outputs are lazy: in [0, 2^256), congruent mod p, plus c3, the\n")
    o.write("// carry out of limb 2 (<= 2, almost always 0) that hlc_field.hpp folds in.\n")
    o.write("#pragma once\n#include <stdint.h>\n\nnamespace hlc {\n\n")
    r_out = ", ".join(f'[r{k}] "=&v"(r[{k}])' for k in range(8))
    sg = lambda names: ", ".join(f'[{n}] "=&s"({n})' for n in names)
    ins_a = ", ".join(f'[a{i}] "v"(a[{i}])' for i in range(8))
    ins_b = ", ".join(f'[b{i}] "v"(b[{i}])' for i in range(8))
    o.write(f"// r = a * b mod p (lazy), {len(mul)} instructions\n")
    o.write("__device__ __forceinline__ void fe_mul_asm(uint32_t r[8], uint32_t& c3, const uint32_t a[8],\n"
            "                                           const uint32_t b[8]) {\n")
    o.write("  uint64_t c0, c1, c2, cA, cB, cC;\n  asm volatile(\n")
    o.write(asm_block(mul) + "\n")
    o.write(f"      : {r_out}, [c3] \"=&v\"(c3), {sg(['c0', 'c1', 'c2', 'cA', 'cB', 'cC'])}\n")
    o.write(f"      : {ins_a}, {ins_b}, [k977] \"s\"(977u)\n")
    o.write('      : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "vcc");\n}\n\n')
    o.write(f"// r = a^2 mod p (lazy), {len(sqr)} instructions\n")
    o.write("__device__ __forceinline__ void fe_sqr_asm(uint32_t r[8], uint32_t& c3, const uint32_t a[8]) {\n")
    o.write("  uint64_t c0, c1, c2, cA, cB, cC, cD;\n  asm volatile(\n")
    o.write(asm_block(sqr) + "\n")
    o.write(f"      : {r_out}, [c3] \"=&v\"(c3), {sg(['c0', 'c1', 'c2', 'cA', 'cB', 'cC', 'cD'])}\n")
    o.write(f"      : {ins_a}, [k977] \"s\"(977u)\n")
    o.write('      : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "vcc");\n}\n\n')
    t_out = ", ".join(f'[t{k}] "=&v"(t[{k}])' for k in range(16))
    o.write(f"// t[0..15] = a * b  (256 x 256 -> 512 bits), {len(m512)} instructions\n")
    o.write("__device__ __forceinline__ void mul512_asm(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {\n")
    o.write("  uint64_t c0, c1, c2;\n  asm volatile(\n")
    o.write(asm_block(m512) + "\n")
    o.write(f"      : {t_out}, {sg(['c0', 'c1', 'c2'])}\n")
    o.write(f"      : {ins_a}, {ins_b}\n")
    o.write('      : "v0", "v1", "v2", "v3");\n}\n\n')
    o.write("}  // namespace hlc\n")


if __name__ == "__main__":
    main()
