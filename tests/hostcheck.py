"""ctypes view of tests/native/libhostcheck.so (device headers compiled for
the host) plus encoders between the oracle's Python values and the harness'
byte layout.  TEST ONLY."""
import ctypes
import os
import subprocess

from oracle import bls12_381 as B

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "hostcheck.cpp")
DEFS = [d for d in os.environ.get("BGV_HOST_DEFS", "").split() if d]  # e.g. "-DBGV_FPMUL28=1"
LIB = os.path.join(HERE, "native", "libhostcheck%s.so" % ("_" + "_".join(x.strip("-D").replace("=", "") for x in DEFS) if DEFS else ""))
CSRC = os.path.join(os.path.dirname(HERE), "lodestar_amd", "csrc")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return any(os.path.getmtime(d) > t for d in deps)


def load():
    if _stale():
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC"] + DEFS + ["-o", LIB, SRC])
    lib = ctypes.CDLL(LIB)
    lib.hc_g2_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.hc_g1_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.hc_g2_mul_u64_w4.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.hc_g1_mul_u64_w4.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    return lib


def fp_b(v):
    return (v % B.P).to_bytes(48, "big")


def b_fp(b):
    return int.from_bytes(b, "big")


def fp2_b(c):
    return fp_b(c[0]) + fp_b(c[1])


def b_fp2(b):
    return (b_fp(b[:48]), b_fp(b[48:96]))


def g2_b(pt):
    return fp2_b(pt[0]) + fp2_b(pt[1])


def b_g2(b):
    return (b_fp2(b[:96]), b_fp2(b[96:192]))


def g1_b(pt):
    return fp_b(pt[0]) + fp_b(pt[1])


def b_g1(b):
    return (b_fp(b[:48]), b_fp(b[48:96]))


def tower_b(t):
    """tower tuple ((c00,c01,c02),(c10,c11,c12)) -> 576 bytes ordered by w^k"""
    (a0, a1, a2), (b0, b1, b2) = t
    return b"".join(fp2_b(c) for c in (a0, b0, a1, b1, a2, b2))


def b_tower(b):
    cs = [b_fp2(b[96 * k : 96 * k + 96]) for k in range(6)]
    return ((cs[0], cs[2], cs[4]), (cs[1], cs[3], cs[5]))


def buf(n):
    return ctypes.create_string_buffer(n)
