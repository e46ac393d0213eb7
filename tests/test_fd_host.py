"""The signed-digit field of the latency kernels (lodestar_amd/csrc/fd.h) and
their cooperative G2 formulas (coop_g2_fd.h, run one lane at a time on the
host through gd_host), compiled for the HOST with every fd bound asserted
(-DBGV_FD_CHECK: digit and value bounds before each product, int32 digits
after each digit-wise operation; a violation aborts the library call), against
the from-spec oracle.  tests/test_gpu_parity.py then checks the HIP kernels
built from the same formulas against the one-lane kernels on the GPU."""
import os
import random
import subprocess

import pytest

from oracle import bls12_381 as B
from tests import hostcheck as H

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "fdcheck.cpp")
LIB = os.path.join(HERE, "native", "libfdcheck.so")
CSRC = os.path.join(os.path.dirname(HERE), "lodestar_amd", "csrc")


def _load():
    import ctypes

    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if not os.path.exists(LIB) or any(os.path.getmtime(d) > os.path.getmtime(LIB) for d in deps):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-DBGV_FD_CHECK", "-o", LIB, SRC])
    lib = ctypes.CDLL(LIB)
    lib.fdc_mul_u64_w4.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    return lib


lib = _load()
rnd = random.Random(0xFD)


def rfp():
    return rnd.randrange(B.P)


def test_fd_field_ops():
    edge = [0, 1, 2, B.P - 1, B.P - 2, (B.P - 1) // 2, 2**380 % B.P, 2**381 % B.P]
    vals = edge + [rfp() for _ in range(300)]
    o = H.buf(48)
    for i, a in enumerate(vals):
        b = vals[(i * 7 + 3) % len(vals)]
        lib.fdc_mul(H.fp_b(a), H.fp_b(b), o)
        assert H.b_fp(o.raw) == a * b % B.P
        lib.fdc_sqr(H.fp_b(a), o)
        assert H.b_fp(o.raw) == a * a % B.P
        c = vals[(i * 13 + 5) % len(vals)]
        assert lib.fdc_expr(H.fp_b(a), H.fp_b(b), H.fp_b(c), o) == 1
        want = ((a + b) * (a - 3 * c) - 2 * (b - c) ** 2) * pow(2, -1, B.P) % B.P
        assert H.b_fp(o.raw) == want
        assert lib.fdc_is_zero(H.fp_b(a)) == (a == 0)


def _g2(k):
    return B.E2.mul(B.G2, k)


def _off_subgroup(seed):
    """a point of E2 outside G2 (SSWU + isogeny output, before clearing)"""
    u = (seed * 0x9E3779B97F4A7C15 % B.P, (seed * 0xC2B2AE3D27D4EB4F + 7) % B.P)
    return B.iso_map_g2(B.map_to_curve_sswu(u))


def test_fd_g2_dbl_add_and_exceptional_cases():
    o = H.buf(192)
    for k1, k2 in [(77, 1234567), (5, 9), (2**64 - 59, 3), (1, 2)]:
        P, Q = _g2(k1), _g2(k2)
        assert lib.fdc_g2_add(H.g2_b(P), H.g2_b(Q), o) == 1
        assert B.E2.eq(H.b_g2(o.raw), B.E2.add(P, Q))
        assert lib.fdc_g2_dbl(H.g2_b(P), o) == 1
        assert B.E2.eq(H.b_g2(o.raw), B.E2.dbl(P))
        assert lib.fdc_g2_add_jac(H.g2_b(P), H.g2_b(Q), o) == 1
        assert B.E2.eq(H.b_g2(o.raw), B.E2.add(B.E2.dbl(P), Q))
    P = _g2(4242)
    assert lib.fdc_g2_add(H.g2_b(P), H.g2_b(P), o) == 1  # P == Q: the doubling branch
    assert B.E2.eq(H.b_g2(o.raw), B.E2.dbl(P))
    assert lib.fdc_g2_add(H.g2_b(P), H.g2_b(B.E2.neg(P)), o) == 0  # P == -Q: infinity
    # [2]P + (-[2]P) through a Jacobian (z != 1) operand
    assert lib.fdc_g2_add_jac(H.g2_b(P), H.g2_b(B.E2.neg(B.E2.dbl(P))), o) == 0


@pytest.mark.parametrize("seed", range(6))
def test_fd_g2_clear_cofactor_and_subgroup(seed):
    Pt = _off_subgroup(seed + 1)
    assert not B.g2_in_subgroup(Pt)
    o = H.buf(192)
    assert lib.fdc_clear_cofactor(H.g2_b(Pt), o) == 1
    assert B.E2.eq(H.b_g2(o.raw), B.clear_cofactor_g2(Pt))
    assert lib.fdc_in_subgroup(H.g2_b(Pt)) == 0
    assert lib.fdc_in_subgroup(H.g2_b(H.b_g2(o.raw))) == 1
    lib.fdc_mul_abs_x(H.g2_b(Pt), o)
    assert B.E2.eq(H.b_g2(o.raw), B.E2.mul(Pt, 0xD201000000010000))


def test_fd_g2_mul_u64_w4():
    P = _g2(31337)
    o = H.buf(192)
    for k in (1, 2, 15, 16, 0x10, 0xF000000000000000, 0xF00DFACE12345679, 2**64 - 1, 0x8000000000000001,
              rnd.getrandbits(64), rnd.getrandbits(64)):
        assert lib.fdc_mul_u64_w4(H.g2_b(P), k, o) == 1
        assert B.E2.eq(H.b_g2(o.raw), B.E2.mul(P, k)), hex(k)
    assert lib.fdc_mul_u64_w4(H.g2_b(P), 0, o) == 0
