"""The device arithmetic headers (lodestar_amd/csrc/*.h), compiled for the
HOST by tests/native/hostcheck.cpp, against the from-spec oracle.  This pins
every algebraic layer the HIP kernels are built from (field tower, curve
formulas, decompression, subgroup test, hash_to_G2 stages, Miller loop steps,
final exponentiation) on the CPU; tests/test_gpu_*.py then check that the
kernels built from the same headers agree on the GPU."""
import ctypes
import random

import pytest

from oracle import bls12_381 as B
from tests import hostcheck as H

lib = H.load()
rnd = random.Random(0xB15)


def rfp():
    return rnd.randrange(B.P)


def rfp2():
    return (rfp(), rfp())


def rf12():
    return tuple(tuple(rfp2() for _ in range(3)) for _ in range(2))


def test_fp_ops():
    for _ in range(200):
        a, b = rfp(), rfp()
        o = H.buf(48)
        lib.hc_fp_mul(H.fp_b(a), H.fp_b(b), o)
        assert H.b_fp(o.raw) == a * b % B.P
        lib.hc_fp_add(H.fp_b(a), H.fp_b(b), o)
        assert H.b_fp(o.raw) == (a + b) % B.P
        lib.hc_fp_sub(H.fp_b(a), H.fp_b(b), o)
        assert H.b_fp(o.raw) == (a - b) % B.P
    # divstep inversion: edge values (Montgomery images 1, 2, p-1 included) and random values
    rinv = pow(2**384, -1, B.P)
    edge = [1, 2, 3, B.P - 1, B.P - 2, (B.P - 1) // 2, rinv, 2 * rinv % B.P, (B.P - 1) * rinv % B.P, 2**380 % B.P]
    for a in edge + [rfp() for _ in range(400)]:
        o = H.buf(48)
        lib.hc_fp_inv(H.fp_b(a), o)
        assert H.b_fp(o.raw) * a % B.P == 1, hex(a)
    o = H.buf(48)
    lib.hc_fp_inv(H.fp_b(0), o)
    assert H.b_fp(o.raw) == 0
    # edge values
    for a, b in [(B.P - 1, B.P - 1), (0, B.P - 1), (1, 1)]:
        o = H.buf(48)
        lib.hc_fp_mul(H.fp_b(a), H.fp_b(b), o)
        assert H.b_fp(o.raw) == a * b % B.P


def test_fp2_ops():
    for _ in range(50):
        a, b = rfp2(), rfp2()
        o = H.buf(96)
        lib.hc_fp2_mul(H.fp2_b(a), H.fp2_b(b), o)
        assert H.b_fp2(o.raw) == B.f2_mul(a, b)
        lib.hc_fp2_sqr(H.fp2_b(a), o)
        assert H.b_fp2(o.raw) == B.f2_sqr(a)
        lib.hc_fp2_inv(H.fp2_b(a), o)
        assert B.f2_eq(B.f2_mul(H.b_fp2(o.raw), a), B.F2_ONE)
        assert lib.hc_fp2_sgn0(H.fp2_b(a)) == B.f2_sgn0(a)
    assert lib.hc_lazy_mul_canonical(ctypes.c_uint64(12345), 20000) == 0
    # the sum-of-products Fp2 product (the device's Fp2 leaf): against the oracle,
    # and bit-identical to Karatsuba on canonical and lazy (< 2p) operands
    for _ in range(50):
        a, b = rfp2(), rfp2()
        o = H.buf(96)
        lib.hc_fp2_mul_sop(H.fp2_b(a), H.fp2_b(b), o)
        assert H.b_fp2(o.raw) == B.f2_mul(a, b)
    assert lib.hc_sop_lazy_check(ctypes.c_uint64(777), 20000) == 0
    # lazy Karatsuba sums (fp_add_lazy, < 2p): Montgomery images at p-1, p-2 make them largest
    rinv = pow(2**384, -1, B.P)
    hi = [(B.P - k) * rinv % B.P for k in (1, 2, 3)] + [B.P - 1, 1, 0, (B.P - 1) // 2 * rinv % B.P]
    for x0 in hi:
        for x1 in hi:
            a, b = (x0, x1), (x1, hi[0])
            o = H.buf(96)
            lib.hc_fp2_mul(H.fp2_b(a), H.fp2_b(b), o)
            assert H.b_fp2(o.raw) == B.f2_mul(a, b)
            lib.hc_fp2_sqr(H.fp2_b(a), o)
            assert H.b_fp2(o.raw) == B.f2_sqr(a)
    for _ in range(40):
        a = rfp2()
        sq = B.f2_is_square(a)
        assert bool(lib.hc_fp2_is_square(H.fp2_b(a))) == sq
        o = H.buf(96)
        ok = lib.hc_fp2_sqrt(H.fp2_b(a), o)
        assert bool(ok) == sq
        if sq:
            assert B.f2_eq(B.f2_sqr(H.b_fp2(o.raw)), a)
    # a1 == 0 branch: squares and non-squares of Fp embedded in Fp2
    for a0 in [4, 5, B.P - 4, rfp(), rfp()]:
        o = H.buf(96)
        assert lib.hc_fp2_sqrt(H.fp2_b((a0, 0)), o) == 1
        assert B.f2_eq(B.f2_sqr(H.b_fp2(o.raw)), (a0, 0))
        # the exact root: a0^((p+1)/4), or (-a0)^((p+1)/4) i for a non-residue
        e = (B.P + 1) // 4
        s = pow(a0, e, B.P)
        want = (s, 0) if s * s % B.P == a0 % B.P else (0, pow(-a0 % B.P, e, B.P))
        assert H.b_fp2(o.raw) == want


def test_fp12_ops():
    for _ in range(5):
        a, b = rf12(), rf12()
        o = H.buf(576)
        lib.hc_fp12_mul(H.tower_b(a), H.tower_b(b), o)
        assert B.f12_eq(B.tower_to_f12(H.b_tower(o.raw)), B.f12_mul(B.tower_to_f12(a), B.tower_to_f12(b)))
        lib.hc_fp12_sqr(H.tower_b(a), o)
        assert B.f12_eq(B.tower_to_f12(H.b_tower(o.raw)), B.f12_mul(B.tower_to_f12(a), B.tower_to_f12(a)))
        lib.hc_fp12_inv(H.tower_b(a), o)
        assert B.f12_eq(B.f12_mul(B.tower_to_f12(H.b_tower(o.raw)), B.tower_to_f12(a)), B.F12_ONE)
        for k in (1, 2, 3):
            lib.hc_fp12_frob(H.tower_b(a), k, o)
            assert B.f12_eq(B.tower_to_f12(H.b_tower(o.raw)), B.f12_pow(B.tower_to_f12(a), B.P**k))
        # sparse line multiplication
        l0, l1, l2 = rfp2(), rfp2(), rfp2()
        lib.hc_fp12_mul_line(H.tower_b(a), H.fp2_b(l0), H.fp2_b(l1), H.fp2_b(l2), o)
        line = ((l0, l1, (0, 0)), ((0, 0), l2, (0, 0)))
        assert B.f12_eq(B.tower_to_f12(H.b_tower(o.raw)), B.f12_mul(B.tower_to_f12(a), B.tower_to_f12(line)))


def test_cyclotomic_and_final_exp():
    a = rf12()
    o = H.buf(576)
    lib.hc_fp12_final_exp(H.tower_b(a), o)
    got = B.tower_to_f12(H.b_tower(o.raw))
    want = B.final_exponentiation(B.tower_to_f12(a))
    # the device hard part computes the fixed cube of the canonical value
    assert B.f12_eq(got, B.f12_pow(want, 3))
    # cyclotomic squaring on an element of the cyclotomic subgroup
    lib.hc_fp12_cyc_sqr(o.raw, o)
    assert B.f12_eq(B.tower_to_f12(H.b_tower(o.raw)), B.f12_mul(got, got))


def test_g2_decompress_and_subgroup():
    for k in [1, 2, 12345, rnd.randrange(B.R)]:
        pt = B.E2.mul(B.G2, k)
        enc = B.g2_compress(pt)
        o = H.buf(192)
        inf = H.ctypes.c_int()
        assert lib.hc_g2_decompress(enc, o, H.ctypes.byref(inf)) == 0
        assert B.E2.eq(H.b_g2(o.raw), pt)
        assert lib.hc_g2_in_subgroup(o.raw) == 1
        # uncompressed
        assert lib.hc_g2_deserialize(B.g2_serialize(pt), o, H.ctypes.byref(inf)) == 0
        assert B.E2.eq(H.b_g2(o.raw), pt)
    # on-curve points outside G2 (no cofactor clearing)
    n_checked = 0
    while n_checked < 3:
        x = rfp2()
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2))
        if y is None:
            continue
        pt = (x, y)
        assert not B.g2_in_subgroup(pt)
        assert lib.hc_g2_in_subgroup(H.g2_b(pt)) == 0
        n_checked += 1


def test_decompress_error_codes():
    inf = H.ctypes.c_int()
    o = H.buf(192)
    good = bytearray(B.g2_compress(B.G2))
    cases = []
    cases.append((bytes([good[0] & 0x7F]) + bytes(good[1:]), B.BLST_BAD_ENCODING))  # no compression bit
    cases.append((bytes([0xC0]) + bytes(95), 0))  # infinity
    cases.append((bytes([0xE0]) + bytes(95), B.BLST_BAD_ENCODING))  # infinity + sign
    cases.append((bytes([0xC0]) + bytes(94) + b"\x01", B.BLST_BAD_ENCODING))
    xp = bytearray(B.P.to_bytes(48, "big"))
    xp[0] |= 0x80
    cases.append((bytes(xp) + bytes(48), B.BLST_BAD_ENCODING))  # x1 = p
    for enc, code in cases:
        assert lib.hc_g2_decompress(enc, o, H.ctypes.byref(inf)) == code
        if code == 0:
            ref_code, _ = B.g2_decompress(enc)
            assert ref_code == 0
    # not on curve: search x with x^3 + b' non-square
    while True:
        x = rfp2()
        if not B.f2_is_square(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2)):
            break
    enc = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    enc[0] |= 0x80
    assert lib.hc_g2_decompress(bytes(enc), o, H.ctypes.byref(inf)) == B.BLST_POINT_NOT_ON_CURVE
    assert B.g2_decompress(bytes(enc))[0] == B.BLST_POINT_NOT_ON_CURVE


def test_point_arith():
    P = B.E2.mul(B.G2, 77)
    Q = B.E2.mul(B.G2, 1234567)
    o = H.buf(192)
    lib.hc_g2_add(H.g2_b(P), H.g2_b(Q), o)
    assert B.E2.eq(H.b_g2(o.raw), B.E2.add(P, Q))
    lib.hc_g2_add(H.g2_b(P), H.g2_b(P), o)
    assert B.E2.eq(H.b_g2(o.raw), B.E2.dbl(P))
    assert lib.hc_g2_add(H.g2_b(P), H.g2_b(B.E2.neg(P)), o) == 0
    k = 0xF00DFACE12345679
    lib.hc_g2_mul_u64(H.g2_b(P), k, o)
    assert B.E2.eq(H.b_g2(o.raw), B.E2.mul(P, k))
    o1 = H.buf(96)
    G = B.E1.mul(B.G1, 99)
    lib.hc_g1_mul_u64(H.g1_b(G), k, o1)
    assert B.E1.eq(H.b_g1(o1.raw), B.E1.mul(G, k))
    # fixed-window variant used by the kernels for the random batch scalars
    for kk in (1, 2, 15, 16, 0x10, 0xF000000000000000, k, 2**64 - 1, 0x8000000000000001):
        lib.hc_g2_mul_u64_w4(H.g2_b(P), kk, o)
        assert B.E2.eq(H.b_g2(o.raw), B.E2.mul(P, kk)), hex(kk)
        lib.hc_g1_mul_u64_w4(H.g1_b(G), kk, o1)
        assert B.E1.eq(H.b_g1(o1.raw), B.E1.mul(G, kk)), hex(kk)
    pts = [B.E1.mul(B.G1, i + 3) for i in range(5)]
    blob = b"".join(H.g1_b(p) for p in pts)
    lib.hc_g1_sum(blob, 5, o1)
    assert B.E1.eq(H.b_g1(o1.raw), B.E1.mul(B.G1, sum(i + 3 for i in range(5))))


def test_hash_to_g2_stages():
    msg = bytes(range(32))
    o = H.buf(256)
    lib.hc_expand_message(msg, o)
    assert o.raw == B.expand_message_xmd(msg, B.DST_POP, 256)
    o = H.buf(192)
    lib.hc_hash_to_field(msg, o)
    u0, u1 = B.hash_to_field_fp2(msg, 2, B.DST_POP)
    assert H.b_fp2(o.raw[:96]) == u0 and H.b_fp2(o.raw[96:]) == u1
    for u in [u0, u1, B.F2_ZERO, (1, 0)] + [rfp2() for _ in range(12)]:
        lib.hc_sswu(H.fp2_b(u), o)
        q = B.map_to_curve_sswu(u)
        assert B.E2.eq(H.b_g2(o.raw), q)
        lib.hc_iso_map(H.g2_b(q), o)
        assert B.E2.eq(H.b_g2(o.raw), B.iso_map_g2(q))
    st = {}
    B.hash_to_g2(msg, B.DST_POP, st)
    lib.hc_clear_cofactor(H.g2_b(st["r"]), o)
    assert B.E2.eq(H.b_g2(o.raw), st["h"])
    lib.hc_hash_to_g2(msg, o)
    assert B.E2.eq(H.b_g2(o.raw), st["h"])


def test_miller_steps_and_pairing():
    P = B.E1.mul(B.G1, 5)
    Q = B.E2.mul(B.G2, 7)
    # doubling step: point part must equal 2Q (homogeneous projective)
    T = H.fp2_b(Q[0]) + H.fp2_b(Q[1]) + H.fp2_b((1, 0))
    to, line = H.buf(288), H.buf(288)
    lib.hc_miller_dbl_step(T, H.g1_b(P), to, line)
    X, Y, Z = (H.b_fp2(to.raw[96 * i : 96 * i + 96]) for i in range(3))
    zi = B.f2_inv(Z)
    assert B.E2.eq((B.f2_mul(X, zi), B.f2_mul(Y, zi)), B.E2.dbl(Q))
    R2 = B.E2.mul(B.G2, 11)
    lib.hc_miller_add_step(T, H.g2_b(R2), H.g1_b(P), to, line)
    X, Y, Z = (H.b_fp2(to.raw[96 * i : 96 * i + 96]) for i in range(3))
    zi = B.f2_inv(Z)
    assert B.E2.eq((B.f2_mul(X, zi), B.f2_mul(Y, zi)), B.E2.add(Q, R2))
    # full Miller loop + device final exp == oracle pairing^3
    o = H.buf(576)
    lib.hc_miller_loop(H.g1_b(P), H.g2_b(Q), o)
    fe = H.buf(576)
    lib.hc_fp12_final_exp(o.raw, fe)
    got = B.tower_to_f12(H.b_tower(fe.raw))
    want = B.pairing(P, Q)
    assert B.f12_eq(got, B.f12_pow(want, 3))


def test_miller_loop2_equals_product_of_single_loops():
    """the 2-pair shared-accumulator loop used by k_miller is bit-identical to
    the product of two single Miller loops (same tower element, no FE)"""
    P1, Q1 = B.E1.mul(B.G1, 5), B.E2.mul(B.G2, 9)
    P2, Q2 = B.E1.mul(B.G1, 123), B.E2.mul(B.G2, 77)
    o1, o2, o12, prod = H.buf(576), H.buf(576), H.buf(576), H.buf(576)
    lib.hc_miller_loop(H.g1_b(P1), H.g2_b(Q1), o1)
    lib.hc_miller_loop(H.g1_b(P2), H.g2_b(Q2), o2)
    lib.hc_fp12_mul(o1.raw, o2.raw, prod)
    lib.hc_miller_loop2(H.g1_b(P1), H.g2_b(Q1), H.g1_b(P2), H.g2_b(Q2), o12)
    assert o12.raw == prod.raw


def test_chacha20_block_rfc8439():
    """rng.h block function (the device batch-scalar generator) on the
    RFC 8439 section 2.3.2 test vector."""
    key = (ctypes.c_uint32 * 8)(*[int.from_bytes(bytes(range(4 * i, 4 * i + 4)), "little") for i in range(8)])
    nonce = (ctypes.c_uint32 * 3)(0x09000000, 0x4A000000, 0x00000000)
    out = (ctypes.c_uint32 * 16)()
    lib.hc_chacha20_block(key, 1, nonce, out)
    assert list(out) == [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
                         0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2]


def test_hash_to_g2_split_equals_single_lane():
    """latency mode (k_hash_map + k_hash_clear) computes the same H(m)"""
    for k in range(8):
        msg = bytes((k * 37 + i) & 0xFF for i in range(32))
        assert lib.hc_hash_to_g2_split_eq(msg) == 1
