#!/usr/bin/env python3
"""Algorithmic work per vote of the recovery kernel (k_recover), counted from the algorithm's
field-operation structure (hlc_recover.hpp), not from the ISA.

Two figures:
  * SURVEY.md §8(d) frozen canonical work: 2,480 modmul x 136 limb products (8x32 Montgomery
    CIOS) = 3.4e5 32x32->64 limb products per vote -- the unit bench.py's roofline uses;
  * the implemented algorithm's own count (GLV + regular 5-bit windows for u2 R, 16-bit comb for
    u1 G, pseudo-Mersenne reduction): M field multiplications (64 products + 8 for the fold)
    and S squarings (36 + 8), plus the two safegcd inversions.

Run: python tools/work_model.py
"""

M_PRODUCTS = 64 + 8     # 8x8 product scan + H*977 fold
S_PRODUCTS = 36 + 8     # 28 off-diagonal + 8 diagonal + fold
INV_PRODUCTS = 20 * 96  # safegcd: 20 batches of 30 divsteps; matrix update 4 x 2 x 9 products + fold


def implemented():
    M = S = 0
    # decompress R: x^3 (1S + 1M), sqrt chain 254S + 13M (incl. the r^2 == a check)
    S += 1 + 254
    M += 1 + 13
    # scalars: r^-1 (safegcd), 3 Montgomery products, GLV split of u2 (2 x 256x256 + 3 Montgomery)
    M += 3 + 2 + 3
    # R table: 2R (2M + 5S), C^2 C^3 (1S + 1M), phi(R) (2M), 15 x madd_zr (8M + 3S),
    # common-Z walk 15 x (4M + 1S), zg (1M)
    M += 2 + 1 + 2 + 15 * 8 + 15 * 4 + 1
    S += 5 + 1 + 15 * 3 + 15
    # main loop: 125 doublings (2M + 5S), 52 mixed additions (7M + 4S), 26 beta products,
    # 2 skew corrections (+1 beta)
    M += 125 * 2 + 52 * 7 + 26 + 2 * 7 + 1
    S += 125 * 5 + 52 * 4 + 2 * 4
    # back to the real frame (1M), comb: 16 mixed additions, final Jacobian add (11M + 5S)
    M += 1 + 16 * 7 + 11
    S += 16 * 4 + 5
    # to affine: Z^-1 (safegcd), Z^-2, Z^-3, X, Y (1S + 3M)
    M += 3
    S += 1
    return M, S


def implemented_limb_products() -> int:
    M, S = implemented()
    return M * M_PRODUCTS + S * S_PRODUCTS + 2 * INV_PRODUCTS


def main():
    M, S = implemented()
    print(f"implemented algorithm: {M} M + {S} S + 2 inversions = {implemented_limb_products():,} "
          f"limb products / vote")
    print(f"SURVEY §8(d) canonical: 2,480 modmul x 136 = {2480 * 136:,} limb products / vote")


if __name__ == "__main__":
    main()
