#!/usr/bin/env python3
"""Generate lodestar_amd/csrc/bls_consts.h: BLS12-381 constants in the
device representation (12 x u32 little-endian limbs, Montgomery form with
R = 2^384).

Self-contained build tool (it does not import oracle/): the curve definition
(p, r, generators, xi = 1 + i, RFC 9380 SSWU + 3-isogeny constants) is stated
below and every derived value (Montgomery forms, Frobenius and psi
coefficients, SSWU helpers) is computed here.  tests/test_constants.py checks
the emitted header against the oracle.  Re-run: python tools/gen_constants.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_PARAM = -0xD201000000010000  # BLS parameter u (negative)

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (
    0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
    0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
)
G2_Y = (
    0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
    0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
)
G1 = (G1_X, G1_Y)
G2 = (G2_X, G2_Y)

B1 = 4
B2 = (4, 4)  # 4 * (1 + i)


# --------------------------------------------------------------------------
# Fp
# --------------------------------------------------------------------------


def fp_inv(a: int) -> int:
    return pow(a % P, P - 2, P)


# --------------------------------------------------------------------------
# Fp2 = Fp[i] / (i^2 + 1), elements as (c0, c1)
# --------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, s: int):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = fp_inv(a[0] * a[0] + a[1] * a[1])
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_pow(a, e: int):
    r = F2_ONE
    b = a
    while e > 0:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a) -> bool:
    return a[0] % P == 0 and a[1] % P == 0


def f2_eq(a, b) -> bool:
    return (a[0] - b[0]) % P == 0 and (a[1] - b[1]) % P == 0


# E2': y^2 = x^3 + A' x + B'
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)  # Z = -(2 + i)


def _k(a, b=0):
    return (a % P, b % P)


# RFC 9380 Appendix E.3: 3-isogeny E2' -> E2 constants
ISO_XNUM = [
    _k(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
       0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    _k(0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    _k(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
       0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    _k(0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO_XDEN = [
    _k(0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
    _k(0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
    _k(1, 0),
]
ISO_YNUM = [
    _k(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
       0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    _k(0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    _k(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
       0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    _k(0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO_YDEN = [
    _k(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
       0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
    _k(0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
    _k(0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
    _k(1, 0),
]



_XI = (1, 1)
PSI_CX = f2_inv(f2_pow(_XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(_XI, (P - 1) // 2))

NLIMB = 12
RM = 1 << 384


def limbs(v):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(NLIMB)]


def mont(v):
    return (v % P) * RM % P


def fp_lit(v, montgomery=True):
    vv = mont(v) if montgomery else v
    return "{{" + ", ".join("0x%08xu" % l for l in limbs(vv)) + "}}"


def fp2_lit(c):
    return "{" + fp_lit(c[0]) + ", " + fp_lit(c[1]) + "}"


out = []
w = out.append
w("// GENERATED by tools/gen_constants.py from the curve definition -- do not edit.")
w("// Representation: Fp = 12 x u32 little-endian limbs, Montgomery R = 2^384.")
w("#pragma once")
w('#include "bls_types.h"')
w("")
w("namespace bgv {")
w("")
w("// modulus p (plain), -p^-1 mod 2^32, R^2 mod p (plain), 1 in Montgomery form")
w("BGV_CONST fp_t P_MOD = " + fp_lit(P, False) + ";")
w("BGV_CONST uint32_t P_INV32 = 0x%08xu;" % ((-pow(P, -1, 1 << 32)) % (1 << 32)))
w("BGV_CONST fp_t R2_MOD = " + fp_lit(RM * RM % P, False) + ";")
w("BGV_CONST fp_t FP_ONE = " + fp_lit(1) + ";")
w("")
w("// exponents (plain integers, 12 x u32) for Fermat inverse / sqrt / Legendre")
w("BGV_CONST fp_t EXP_P_MINUS_2 = " + fp_lit(P - 2, False) + ";")
w("BGV_CONST fp_t EXP_P_PLUS_1_DIV_4 = " + fp_lit((P + 1) // 4, False) + ";")


def pow_plan(e, wbits=4):
    """4-bit sliding-window plan of a fixed exponent, MSB first: the first
    window's odd value selects the start, then each step squares `shift`
    times and multiplies by a^(2 idx + 1) (idx 0xFF: squarings only)."""
    b = bin(e)[2:]
    i, first, pend, steps = 0, None, 0, []
    while i < len(b):
        if b[i] == "0":
            pend += 1
            i += 1
            continue
        j = min(i + wbits, len(b))
        while b[j - 1] == "0":
            j -= 1
        v = int(b[i:j], 2)
        if first is None:
            first = (v - 1) // 2
        else:
            steps.append((pend + (j - i), (v - 1) // 2))
        pend = 0
        i = j
    if pend:
        steps.append((pend, 0xFF))
    acc = 2 * first + 1  # check the plan reproduces e
    for sh, ix in steps:
        acc <<= sh
        if ix != 0xFF:
            acc += 2 * ix + 1
    assert acc == e
    return first, steps


for _name, _e in (("SQRT", (P + 1) // 4), ("SQRT_TAIL", (P - 3) // 4)):
    _first, _steps = pow_plan(_e)
    w("// sliding-window plan of %s (fp.h fp_pow_plan): %d steps, %d products" % (
        "(p+1)/4" if _name == "SQRT" else "(p-3)/4", len(_steps), sum(1 for _s in _steps if _s[1] != 0xFF)))
    w("constexpr uint32_t POWP_%s_N = %d, POWP_%s_FIRST = %d;" % (_name, len(_steps), _name, _first))
    w("BGV_CONST uint8_t POWP_%s_SHIFT[%d] = {%s};" % (_name, len(_steps), ", ".join(str(a) for a, _ in _steps)))
    w("BGV_CONST uint8_t POWP_%s_IDX[%d] = {%s};" % (_name, len(_steps), ", ".join(str(b_) for _, b_ in _steps)))
w("BGV_CONST fp_t EXP_P_MINUS_3_DIV_4 = " + fp_lit((P - 3) // 4, False) + ";")
w("BGV_CONST fp_t EXP_P_MINUS_1_DIV_2 = " + fp_lit((P - 1) // 2, False) + ";")
w("// (p - 1) / 2 plain, for the lexicographic sign of a coordinate")
w("BGV_CONST fp_t P_HALF = " + fp_lit((P - 1) // 2, False) + ";")
w("")
w("// |x| of the BLS parameter x = -0xd201000000010000")
w("BGV_CONST uint64_t BLS_X_ABS = 0x%016xull;" % (-X_PARAM))
w("constexpr uint64_t BLS_X_ABS_C = 0x%016xull;  // compile-time copy (curve.h x-chain runs)" % (-X_PARAM))
w("")
w("// E1: y^2 = x^3 + 4 ; E2: y^2 = x^3 + 4(1+i)")
w("BGV_CONST fp_t B1_MONT = " + fp_lit(4) + ";")
w("BGV_CONST fp2_t B2_MONT = " + fp2_lit((4, 4)) + ";")
w("BGV_CONST fp2_t B2_X3_MONT = " + fp2_lit((12, 12)) + ";  // 3 b'")
w("BGV_CONST fp_t G1_X_MONT = " + fp_lit(G1_X) + ";")
w("BGV_CONST fp_t G1_Y_MONT = " + fp_lit(G1_Y) + ";")
w("BGV_CONST fp_t G1_NEG_Y_MONT = " + fp_lit(-G1_Y) + ";")
w("BGV_CONST fp2_t G2_X_MONT = " + fp2_lit(G2_X) + ";")
w("BGV_CONST fp2_t G2_Y_MONT = " + fp2_lit(G2_Y) + ";")
w("")
w("// psi(x, y) = (conj(x) * PSI_CX, conj(y) * PSI_CY); psi^2(x, y) = (x * PSI2_CX, y * PSI2_CY)")
w("BGV_CONST fp2_t PSI_CX = " + fp2_lit(PSI_CX) + ";")
w("BGV_CONST fp2_t PSI_CY = " + fp2_lit(PSI_CY) + ";")
psi2x = f2_mul(f2_conj(PSI_CX), PSI_CX)
psi2y = f2_mul(f2_conj(PSI_CY), PSI_CY)
assert psi2x[1] == 0 and psi2y[1] == 0
w("BGV_CONST fp_t PSI2_CX = " + fp_lit(psi2x[0]) + ";")
w("BGV_CONST fp_t PSI2_CY = " + fp_lit(psi2y[0]) + ";")
w("")
w("// Frobenius on the tower: coefficient at w^i of pi^k(f) = conj^k(c_i) * FROB_G[k-1][i-1],")
w("// FROB_G[k-1][i-1] = xi^(i (p^k - 1) / 6), xi = 1 + i, k = 1..3, i = 1..5")
w("BGV_CONST fp2_t FROB_G[3][5] = {")
for k in (1, 2, 3):
    row = []
    for i in range(1, 6):
        row.append(fp2_lit(f2_pow((1, 1), i * (P**k - 1) // 6)))
    w("  {" + ", ".join(row) + "},")
w("};")
w("")
w("// RFC 9380 G2 suite: SSWU on E2': y^2 = x^3 + A x + B, Z = -(2 + i)")
A, Bc, Z = SSWU_A, SSWU_B, SSWU_Z
w("BGV_CONST fp2_t SSWU_A = " + fp2_lit(A) + ";")
w("BGV_CONST fp2_t SSWU_B = " + fp2_lit(Bc) + ";")
w("BGV_CONST fp2_t SSWU_Z = " + fp2_lit(Z) + ";")
w("BGV_CONST fp2_t SSWU_MINUS_B_OVER_A = " + fp2_lit(f2_mul(f2_neg(Bc), f2_inv(A))) + ";")
w("BGV_CONST fp2_t SSWU_B_OVER_ZA = " + fp2_lit(f2_mul(Bc, f2_inv(f2_mul(Z, A)))) + ";")
w("// sqrt(-norm(Z)^3) in Fp: gx2 = Z^3 u^6 gx1, so when norm(gx1) is a non-square with")
w("// d = norm(gx1)^((p+1)/4) (d^2 = -norm(gx1)), sqrt(norm(gx2)) = this * norm(u)^3 * d")
_nz3 = (-pow((Z[0] * Z[0] + Z[1] * Z[1]) % P, 3, P)) % P
_c = pow(_nz3, (P + 1) // 4, P)
assert _c * _c % P == _nz3
w("BGV_CONST fp_t SSWU_SQRT_NEG_NZ3 = " + fp_lit(_c) + ";")
w("// 3-isogeny E2' -> E2 (RFC 9380 appendix E.3), lowest degree first")
w("BGV_CONST fp2_t ISO_XNUM[4] = {" + ", ".join(fp2_lit(c) for c in ISO_XNUM) + "};")
w("BGV_CONST fp2_t ISO_XDEN[3] = {" + ", ".join(fp2_lit(c) for c in ISO_XDEN) + "};")
w("BGV_CONST fp2_t ISO_YNUM[4] = {" + ", ".join(fp2_lit(c) for c in ISO_YNUM) + "};")
w("BGV_CONST fp2_t ISO_YDEN[4] = {" + ", ".join(fp2_lit(c) for c in ISO_YDEN) + "};")
w("")
w("// hash_to_field: 64-byte big-endian e = hi 2^256 + lo ; mont(e) = mont_mul(hi, H2F_K) + mont_mul(lo, R2)")
w("BGV_CONST fp_t H2F_K = " + fp_lit((1 << 256) * RM * RM % P, False) + ";")
w("// 1/2 in Montgomery form (Fp2 sqrt)")
w("BGV_CONST fp_t FP_HALF = " + fp_lit(pow(2, -1, P)) + ";")
w("// R^3 mod p (plain): Montgomery fix-up after a binary-GCD inverse of a Montgomery value")
w("BGV_CONST fp_t R3_MOD = " + fp_lit(RM ** 3 % P, False) + ";")
w("// p as 13 signed 30-bit limbs and p^-1 mod 2^30 (divstep inversion, fp.h)")
w("BGV_CONST int32_t P_S30[13] = {" + ", ".join("0x%08x" % ((P >> (30 * i)) & (2**30 - 1)) for i in range(13)) + "};")
w("BGV_CONST uint32_t P_INV30 = 0x%08xu;" % pow(P, -1, 2**30))
w("")
w("}  // namespace bgv")

dst = os.path.join(ROOT, "lodestar_amd", "csrc", "bls_consts.h")
with open(dst, "w") as f:
    f.write("\n".join(out) + "\n")
print("wrote", dst)
