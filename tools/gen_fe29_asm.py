#!/usr/bin/env python3
"""Generate hashgraph-like-consensus_amd/csrc/hlc_fe29_asm.hpp: gfx950 inline-asm multiplication and
squaring for the 9 x 29-bit unsaturated field layer (hlc_fe29.hpp holds the C++ reference of the same
schedule, used on the host and by the CPU tests).

Why asm: left to itself the compiler re-associates the column sums into independent partial
products and joins them with 64-bit adds (v_lshl_add_u64), and turns the 256 * H folds into
64-bit shift + add pairs -- about 245 instructions against the ~140 of the intended schedule.

Schedule (every instruction VOP3 unless noted; measured issue costs in profiles/r02_ubench_isa.txt):
  * high columns 9..16: one 64-bit accumulator, every product a v_mad_u64_u32 whose 64-bit addend
    is the running column (no carry instruction: nine 58-bit products fit in 64 bits); the column
    ends with v_and_b32 (VOP2) -> H_k and v_lshrrev_b64 29 -> the next column's start value;
  * low columns 0..8 the same, each also receiving 31264 H_{j+9} and 256 H_{j+8} (2^261 = 2^37 +
    31264 mod p) as two more v_mad_u64_u32, and 256 H_17 folded once more into columns 0 and 1;
  * the carry out of column 8 (< 2^35) folds into limbs 0..2 (mad / mad24 / mad-by-1 adds).
Squaring uses doubled operands (2 a_i, computed by the compiler before the block) for the cross
products.  Only the three 64-bit accumulators are fixed registers (v[0:5]); H and the doubled
operands are compiler-allocated operands.

Run:  python tools/gen_fe29_asm.py > hashgraph-like-consensus_amd/csrc/hlc_fe29_asm.hpp
"""
import sys


class Em:
    def __init__(self):
        self.ins = []

    def __call__(self, s):
        self.ins.append(s)


def column(em, prods, acc, first_zero, sd):
    for idx, (x, y) in enumerate(prods):
        addend = "0" if (first_zero and idx == 0) else acc
        em(f"v_mad_u64_u32 {acc}, {sd}, {x}, {y}, {addend}")


def gen(square, tag="", base=0, dual=False, plus=False):
    """One product's instruction list.  tag prefixes the operand names, base the fixed registers
    (v[base .. base+5]) so that two independent products can be interleaved (gen_dual).
    dual: a*b + c*e in one column schedule (both products accumulate into the same 64-bit columns,
    one split / fold / carry pass for the sum).
    plus: a*b + f for a nine-limb f (limbs < 2^32, e.g. 128p - c): f_j enters low column j as one
    more v_mad_u64_u32 by the inline constant 1, so a product and a following subtraction share
    one reduction (no separate carry pass)."""
    em = Em()
    A = lambda i: f"%[{tag}a{i}]"
    B = (lambda i: f"%[{tag}a{i}]") if square else (lambda i: f"%[{tag}b{i}]")
    D = lambda i: f"%[{tag}d{i}]"    # doubled limbs (squaring), computed by the compiler before the asm
    H = lambda k: f"%[{tag}h{k}]"    # H_{9+k}, k = 0..7 (compiler-allocated); H_17 stays in acc1.lo
    R = lambda j: f"%[{tag}r{j}]"
    C = lambda i: f"%[{tag}c{i}]"    # dual: the second product's operands
    E = lambda i: f"%[{tag}e{i}]"
    F = lambda j: f"%[{tag}f{j}]"    # addend limbs
    v = lambda k: f"v{base + k}"
    acc1, acc2, tt = f"v[{base}:{base + 1}]", f"v[{base + 2}:{base + 3}]", f"v[{base + 4}:{base + 5}]"
    sd = f"%[{tag}sd]"

    def prods(k, lo, hi):
        out = []
        for i in range(lo, hi + 1):
            j = k - i
            if j < 0 or j > 8:
                continue
            if square:
                if i < j:
                    out.append((D(i), A(j)))
                elif i == j:
                    out.append((A(i), A(i)))
            else:
                out.append((A(i), B(j)))
                if dual:
                    out.append((C(i), E(j)))
        return out

    # The high columns (9..16) and the low columns (0..8) are two independent mad chains until the
    # low column's fold needs H: they are interleaved product by product (two chains in flight
    # per wave instead of one).  Step t: high column 9+t (t <= 7) and low column t, then H_{9+t},
    # then column t's fold (31264 H_{9+t} or, for t = 8, 31264 H_17; 256 H_{8+t}).  256 H_17 (at
    # 2^261) is folded at the end together with the carry out of column 8.
    for t in range(9):
        hp = prods(9 + t, 1 + t, 8) if t <= 7 else []
        lp = prods(t, 0, t)
        seq = []
        for q in range(max(len(hp), len(lp))):
            if q < len(hp):
                seq.append(("h", q, hp[q]))
            if q < len(lp):
                seq.append(("l", q, lp[q]))
        for kind, q, (x, y) in seq:
            if kind == "h":
                addend = "0" if (t == 0 and q == 0) else acc1
                em(f"v_mad_u64_u32 {acc1}, {sd}, {x}, {y}, {addend}")
            else:
                addend = "0" if (t == 0 and q == 0) else acc2
                em(f"v_mad_u64_u32 {acc2}, {sd}, {x}, {y}, {addend}")
        if plus:
            em(f"v_mad_u64_u32 {acc2}, {sd}, {F(t)}, 1, {acc2}")
        if t <= 7:
            em(f"v_and_b32 {H(t)}, 0x1fffffff, {v(0)}")
            em(f"v_lshrrev_b64 {acc1}, 29, {acc1}")   # after t = 7: H_17 in v0
        em(f"v_mad_u64_u32 {acc2}, {sd}, {H(t) if t < 8 else v(0)}, %[kfl], {acc2}")
        if t >= 1:
            em(f"v_mad_u64_u32 {acc2}, {sd}, {H(t - 1)}, %[kfh], {acc2}")
        em(f"v_and_b32 {R(t)}, 0x1fffffff, {v(2)}")
        em(f"v_lshrrev_b64 {acc2}, 29, {acc2}")
    # end: c = acc2 (< 2^35, carry out of column 8) and 256 H_17 sit at 2^261 -> limbs 0, 1:
    # limb 0 += 31264 c + 256*31264 H_17, limb 1 += 256 c + 65536 H_17, then settle limbs 0..2
    em(f"v_mad_u64_u32 {tt}, {sd}, {v(2)}, %[kfl], 0")
    em(f"v_mad_u32_u24 {v(5)}, {v(3)}, %[kfl], {v(5)}")
    em(f"v_mad_u64_u32 {tt}, {sd}, {v(0)}, %[kf00], {tt}")
    em(f"v_mad_u64_u32 {tt}, {sd}, {R(0)}, 1, {tt}")
    em(f"v_and_b32 {R(0)}, 0x1fffffff, {v(4)}")
    em(f"v_lshrrev_b64 {tt}, 29, {tt}")
    em(f"v_mad_u64_u32 {tt}, {sd}, {v(2)}, %[kfh], {tt}")
    em(f"v_mad_u32_u24 {v(5)}, {v(3)}, %[kfh], {v(5)}")
    em(f"v_mad_u64_u32 {tt}, {sd}, {v(0)}, %[kf01], {tt}")
    em(f"v_mad_u64_u32 {tt}, {sd}, {R(1)}, 1, {tt}")
    em(f"v_and_b32 {R(1)}, 0x1fffffff, {v(4)}")
    em(f"v_lshrrev_b64 {tt}, 29, {tt}")
    em(f"v_add_u32 {R(2)}, {R(2)}, {v(4)}")
    return em.ins


def block(lines):
    return "\n".join(f'      "{l}\\n"' for l in lines)


HEAD = '''// GENERATED by tools/gen_fe29_asm.py -- do not edit.  gfx950 inline-asm schedules of
// fe29_mul / fe29_sqr (hlc_fe29.hpp is the C++ reference of the same arithmetic; the docstring of
// the generator explains the schedule).  Same contract: inputs limbs < 2^30.35, output normalised.
#pragma once
#include <stdint.h>

namespace hlc {

'''


def emit(name, square, lines, b_sgpr=False):
    o = []
    sig = "uint32_t r[9], const uint32_t a[9]" + ("" if square else ", const uint32_t b[9]")
    o.append(f"// {len(lines)} instructions\n__device__ __forceinline__ void {name}({sig}) {{\n")
    o.append("  uint64_t sd;\n  uint32_t h[8];\n")
    if square:
        o.append("  uint32_t d[8];\n#pragma unroll\n  for (int i = 0; i < 8; ++i) d[i] = a[i] << 1;\n")
    o.append("  asm volatile(\n")
    o.append(block(lines) + "\n")
    outs = [f'[r{j}] "=&v"(r[{j}])' for j in range(9)] + [f'[h{k}] "=&v"(h[{k}])' for k in range(8)]
    outs += ['[sd] "=&s"(sd)']
    ins = [f'[a{i}] "v"(a[{i}])' for i in range(9)]
    if not square:
        ins += [f'[b{i}] "{"s" if b_sgpr else "v"}"(b[{i}])' for i in range(9)]
    else:
        ins += [f'[d{i}] "v"(d[{i}])' for i in range(8)]
    ins += ['[kfl] "s"(31264u)', '[kfh] "s"(256u)', '[kf00] "s"(256u * 31264u)', '[kf01] "s"(65536u)']
    clob = ", ".join(f'"v{i}"' for i in range(6))
    o.append("      : " + ", ".join(outs) + "\n")
    o.append("      : " + ", ".join(ins) + "\n")
    o.append("      : " + clob + ");\n}\n\n")
    return "".join(o)


def emit_dual(name, sq1, sq2):
    """Two independent products (x = a*b or a^2, y = c*d or c^2) in one block, instructions
    interleaved one by one: two dependency chains in flight per wave."""
    l1 = gen(sq1, "p", 0)
    l2 = gen(sq2, "q", 6)
    lines = []
    for k in range(max(len(l1), len(l2))):
        if k < len(l1):
            lines.append(l1[k])
        if k < len(l2):
            lines.append(l2[k])
    o = []
    args = ["uint32_t x[9]", "const uint32_t a[9]"] + ([] if sq1 else ["const uint32_t b[9]"])
    args += ["uint32_t y[9]", "const uint32_t c[9]"] + ([] if sq2 else ["const uint32_t d[9]"])
    o.append(f"// {len(lines)} instructions\n__device__ __forceinline__ void {name}({', '.join(args)}) {{\n")
    o.append("  uint64_t psd, qsd;\n  uint32_t ph[8], qh[8];\n")
    for tag, sq, src in (("p", sq1, "a"), ("q", sq2, "c")):
        if sq:
            o.append(f"  uint32_t {tag}d[8];\n#pragma unroll\n  for (int i = 0; i < 8; ++i) {tag}d[i] = {src}[i] << 1;\n")
    o.append("  asm volatile(\n")
    o.append(block(lines) + "\n")
    outs = [f'[pr{j}] "=&v"(x[{j}])' for j in range(9)] + [f'[qr{j}] "=&v"(y[{j}])' for j in range(9)]
    outs += [f'[ph{k}] "=&v"(ph[{k}])' for k in range(8)] + [f'[qh{k}] "=&v"(qh[{k}])' for k in range(8)]
    outs += ['[psd] "=&s"(psd)', '[qsd] "=&s"(qsd)']
    ins = [f'[pa{i}] "v"(a[{i}])' for i in range(9)]
    ins += [f'[pb{i}] "v"(b[{i}])' for i in range(9)] if not sq1 else [f'[pd{i}] "v"(pd[{i}])' for i in range(8)]
    ins += [f'[qa{i}] "v"(c[{i}])' for i in range(9)]
    ins += [f'[qb{i}] "v"(d[{i}])' for i in range(9)] if not sq2 else [f'[qd{i}] "v"(qd[{i}])' for i in range(8)]
    ins += ['[kfl] "s"(31264u)', '[kfh] "s"(256u)', '[kf00] "s"(256u * 31264u)', '[kf01] "s"(65536u)']
    clob = ", ".join(f'"v{i}"' for i in range(12))
    o.append("      : " + ", ".join(outs) + "\n")
    o.append("      : " + ", ".join(ins) + "\n")
    o.append("      : " + clob + ");\n}\n\n")
    return "".join(o)


def emit_muladd(name):
    """r = a b + c e (mod p): one column schedule for the sum of two products (hlc_fe29.hpp
    fe29_muladd_ref is the same arithmetic)."""
    lines = gen(False, dual=True)
    o = [f"// {len(lines)} instructions\n__device__ __forceinline__ void {name}(uint32_t r[9], const uint32_t a[9], "
         "const uint32_t b[9], const uint32_t c[9], const uint32_t e[9]) {\n"]
    o.append("  uint64_t sd;\n  uint32_t h[8];\n")
    o.append("  asm volatile(\n")
    o.append(block(lines) + "\n")
    outs = [f'[r{j}] "=&v"(r[{j}])' for j in range(9)] + [f'[h{k}] "=&v"(h[{k}])' for k in range(8)]
    outs += ['[sd] "=&s"(sd)']
    ins = [f'[{x}{i}] "v"({x}[{i}])' for x in "abce" for i in range(9)]
    ins += ['[kfl] "s"(31264u)', '[kfh] "s"(256u)', '[kf00] "s"(256u * 31264u)', '[kf01] "s"(65536u)']
    clob = ", ".join(f'"v{i}"' for i in range(6))
    o.append("      : " + ", ".join(outs) + "\n")
    o.append("      : " + ", ".join(ins) + "\n")
    o.append("      : " + clob + ");\n}\n\n")
    return "".join(o)


def emit_addend(name, square):
    """r = a b + f or a^2 + f (mod p) for an addend f of nine limbs < 2^32 (hlc_fe29.hpp
    fe29_mul_add_ref / fe29_sqr_add_ref are the same arithmetic)."""
    lines = gen(square, plus=True)
    sig = "uint32_t r[9], const uint32_t a[9]" + ("" if square else ", const uint32_t b[9]") + ", const uint32_t f[9]"
    o = [f"// {len(lines)} instructions\n__device__ __forceinline__ void {name}({sig}) {{\n"]
    o.append("  uint64_t sd;\n  uint32_t h[8];\n")
    if square:
        o.append("  uint32_t d[8];\n#pragma unroll\n  for (int i = 0; i < 8; ++i) d[i] = a[i] << 1;\n")
    o.append("  asm volatile(\n")
    o.append(block(lines) + "\n")
    outs = [f'[r{j}] "=&v"(r[{j}])' for j in range(9)] + [f'[h{k}] "=&v"(h[{k}])' for k in range(8)]
    outs += ['[sd] "=&s"(sd)']
    ins = [f'[a{i}] "v"(a[{i}])' for i in range(9)]
    ins += [f'[d{i}] "v"(d[{i}])' for i in range(8)] if square else [f'[b{i}] "v"(b[{i}])' for i in range(9)]
    ins += [f'[f{i}] "v"(f[{i}])' for i in range(9)]
    ins += ['[kfl] "s"(31264u)', '[kfh] "s"(256u)', '[kf00] "s"(256u * 31264u)', '[kf01] "s"(65536u)']
    clob = ", ".join(f'"v{i}"' for i in range(6))
    o.append("      : " + ", ".join(outs) + "\n")
    o.append("      : " + ", ".join(ins) + "\n")
    o.append("      : " + clob + ");\n}\n\n")
    return "".join(o)


def main():
    mul = gen(False)
    sqr = gen(True)
    text = (HEAD + emit("fe29_mul_asm", False, mul) + emit("fe29_sqr_asm", True, sqr)
            + "// b wave-uniform, held in SGPRs (constants such as beta): saves nine VGPRs at the call site\n"
            + emit("fe29_mul_sb_asm", False, mul, b_sgpr=True)
            + "// two independent products interleaved (x = a b, y = c d / x = a^2, y = c^2 / x = a b, y = c^2)\n"
            + emit_dual("fe29_mul2_asm", False, False) + emit_dual("fe29_sqr2_asm", True, True)
            + emit_dual("fe29_mulsqr_asm", False, True)
            + "// sum of two products with one reduction (r = a b + c e)\n" + emit_muladd("fe29_muladd_asm")
            + "// a product / square plus a nine-limb addend with one reduction (r = a b + f, r = a^2 + f)\n"
            + emit_addend("fe29_mul_add_asm", False) + emit_addend("fe29_sqr_add_asm", True)
            + "}  // namespace hlc\n")
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
