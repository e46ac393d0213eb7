"""From-spec BLS12-381 oracle (pure Python big integers).

TEST INFRASTRUCTURE ONLY.  Nothing under ``lodestar_amd/`` may import this
module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker.

What it restates
----------------
The arithmetic the reference delegates to the third-party, un-vendored
``@chainsafe/bls@7.1.1`` -> ``@chainsafe/blst@0.2.8`` -> supranational
``blst`` (``yarn.lock:483-498``; call sites
``packages/beacon-node/src/chain/bls/maybeBatch.ts:18-25,36-37``,
``chain/bls/utils.ts:11``).  Those libraries are NOT in /root/reference, so
this is a restatement of the public specifications they implement:

* BLS12-381 curve constants and the ZCash point serialization
  (flags 0x80 compressed / 0x40 infinity / 0x20 lexicographic sign,
  big-endian, Fp2 written c1 || c0);
* RFC 9380 ``expand_message_xmd`` (SHA-256), ``hash_to_field``,
  simplified SWU on the 3-isogenous curve E2', the 3-isogeny map and
  ``clear_cofactor`` by h_eff, suite ``BLS12381G2_XMD:SHA-256_SSWU_RO_``;
* IETF BLS signatures, proof-of-possession ciphersuite
  DST = ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`` (the Ethereum
  consensus ciphersuite), minimal-pubkey-size (pk in G1, sig in G2);
* the optimal-ate pairing (Miller loop over |x|, x = -0xd201000000010000,
  then the final exponentiation by (p^12 - 1) / r);
* random-linear-combination batch verification with injectable scalars
  (blst ``Pairing::mul_n_aggregate`` + ``finalverify``).

Pinning (see tests/test_oracle_kat.py):
* ``packages/state-transition/test-cache/interop-pubkeys.json`` — 100
  compressed pubkeys sk_i * G1 for ``interopSecretKey(i)``
  (``packages/state-transition/src/util/interop.ts:19-23``);
* ``packages/beacon-node/test/e2e/interop/genesisState.test.ts:50-55`` —
  deposit #0 signature (hash_to_G2 with the POP DST + G2 mult + compression);
* bilinearity / non-degeneracy self-checks of the pairing.

The Fp12 used by the pairing here is the flat representation
Fp[w] / (w^12 - 2 w^6 + 2) (w^6 = 1 + i), deliberately different from the
Fp2/Fp6/Fp12 tower the HIP kernels use, so agreement is not an artefact of
shared structure.
"""
from __future__ import annotations

import hashlib

# --------------------------------------------------------------------------
# Curve constants
# --------------------------------------------------------------------------
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

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# RFC 9380 section 8.8.2: effective cofactor for G2
H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551

# --------------------------------------------------------------------------
# Fp
# --------------------------------------------------------------------------


def fp_inv(a: int) -> int:
    return pow(a % P, P - 2, P)


def fp_sqrt(a: int):
    """Square root in Fp (p = 3 mod 4); None if a is a non-residue."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_sgn0(a: int) -> int:
    return a % P & 1


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


def f2_is_square(a) -> bool:
    # a is a square in Fp2 iff its norm is a square in Fp
    n = (a[0] * a[0] + a[1] * a[1]) % P
    return n == 0 or pow(n, (P - 1) // 2, P) == 1


def f2_sqrt(a):
    """Any square root of a in Fp2, or None.  The caller fixes the sign."""
    if f2_is_zero(a):
        return F2_ZERO
    # p^2 = 9 mod 16; candidate = a^((p^2 + 7) / 16) times a 8th root of unity
    c = f2_pow(a, (P * P + 7) // 16)
    # eighth roots of unity in Fp2: (1+i)^k / sqrt(2)^k ... just try the four
    # square roots of unity times {1, sqrt(i)}: brute force over candidates.
    for root in _ROOTS_OF_UNITY_8:
        y = f2_mul(c, root)
        if f2_eq(f2_sqr(y), a):
            return y
    return None


def _eighth_roots():
    # all x with x^8 = 1 in Fp2
    roots = []
    # generator of the 8-torsion: g = z^((p^2-1)/8) for a non-residue z
    z = (1, 1)
    while f2_is_square(z):
        z = (z[0] + 1, z[1])
    g = f2_pow(z, (P * P - 1) // 8)
    x = F2_ONE
    for _ in range(8):
        roots.append(x)
        x = f2_mul(x, g)
    return roots


_ROOTS_OF_UNITY_8 = _eighth_roots()


def f2_sgn0(a) -> int:
    """RFC 9380 sgn0 for Fp2 (section 4.1)."""
    sign_0 = a[0] % 2
    zero_0 = a[0] == 0
    sign_1 = a[1] % 2
    return sign_0 | (zero_0 & sign_1)


def f2_lex_largest(a) -> bool:
    """ZCash serialization 'sign' flag for Fp2: compare c1 first, then c0."""
    half = (P - 1) // 2
    if a[1] != 0:
        return a[1] > half
    return a[0] > half


def fp_lex_largest(a: int) -> bool:
    return a > (P - 1) // 2


# --------------------------------------------------------------------------
# Generic short-Weierstrass y^2 = x^3 + a x + b, affine, None = infinity.
# A field "ops" record lets G1 (Fp) and G2 (Fp2) share the formulas.
# --------------------------------------------------------------------------


class _FpOps:
    zero = 0
    one = 1

    @staticmethod
    def add(a, b):
        return (a + b) % P

    @staticmethod
    def sub(a, b):
        return (a - b) % P

    @staticmethod
    def mul(a, b):
        return a * b % P

    @staticmethod
    def neg(a):
        return (-a) % P

    @staticmethod
    def inv(a):
        return fp_inv(a)

    @staticmethod
    def muls(a, s):
        return a * s % P

    @staticmethod
    def eq(a, b):
        return (a - b) % P == 0

    @staticmethod
    def is_zero(a):
        return a % P == 0


class _Fp2Ops:
    zero = F2_ZERO
    one = F2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    neg = staticmethod(f2_neg)
    inv = staticmethod(f2_inv)
    muls = staticmethod(f2_muls)
    eq = staticmethod(f2_eq)
    is_zero = staticmethod(f2_is_zero)


class Curve:
    def __init__(self, F, a, b):
        self.F, self.a, self.b = F, a, b

    def on_curve(self, Pt) -> bool:
        if Pt is None:
            return True
        F = self.F
        x, y = Pt
        lhs = F.mul(y, y)
        rhs = F.add(F.add(F.mul(F.mul(x, x), x), F.mul(self.a, x)), self.b)
        return F.eq(lhs, rhs)

    def neg(self, Pt):
        if Pt is None:
            return None
        return (Pt[0], self.F.neg(Pt[1]))

    def add(self, A, B):
        F = self.F
        if A is None:
            return B
        if B is None:
            return A
        x1, y1 = A
        x2, y2 = B
        if F.eq(x1, x2):
            if F.eq(y1, y2) and not F.is_zero(y1):
                return self.dbl(A)
            return None
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
        x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
        y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
        return (x3, y3)

    def dbl(self, A):
        F = self.F
        if A is None:
            return None
        x1, y1 = A
        if F.is_zero(y1):
            return None
        num = F.add(F.muls(F.mul(x1, x1), 3), self.a)
        lam = F.mul(num, F.inv(F.muls(y1, 2)))
        x3 = F.sub(F.mul(lam, lam), F.muls(x1, 2))
        y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
        return (x3, y3)

    def mul(self, Pt, k: int):
        if k < 0:
            return self.mul(self.neg(Pt), -k)
        acc = None
        addend = Pt
        while k:
            if k & 1:
                acc = self.add(acc, addend)
            addend = self.dbl(addend)
            k >>= 1
        return acc

    def eq(self, A, B) -> bool:
        if A is None or B is None:
            return A is None and B is None
        return self.F.eq(A[0], B[0]) and self.F.eq(A[1], B[1])


E1 = Curve(_FpOps, 0, B1)
E2 = Curve(_Fp2Ops, F2_ZERO, B2)

# --------------------------------------------------------------------------
# Frobenius endomorphism psi on E2 (untwist-Frobenius-twist)
# psi(x, y) = (conj(x) * c_x, conj(y) * c_y),
# c_x = 1 / (1+i)^((p-1)/3), c_y = 1 / (1+i)^((p-1)/2)
# --------------------------------------------------------------------------
_XI = (1, 1)
PSI_CX = f2_inv(f2_pow(_XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(_XI, (P - 1) // 2))


def psi(Pt):
    if Pt is None:
        return None
    x, y = Pt
    return (f2_mul(f2_conj(x), PSI_CX), f2_mul(f2_conj(y), PSI_CY))


def g1_in_subgroup(Pt) -> bool:
    return E1.on_curve(Pt) and E1.mul(Pt, R) is None


def g2_in_subgroup(Pt) -> bool:
    """Definitional subgroup check [r]P == O."""
    return E2.on_curve(Pt) and E2.mul(Pt, R) is None


# --------------------------------------------------------------------------
# ZCash serialization
# --------------------------------------------------------------------------
# blst error codes (supranational/blst bindings/blst.h BLST_ERROR enum order)
BLST_SUCCESS = 0
BLST_BAD_ENCODING = 1
BLST_POINT_NOT_ON_CURVE = 2
BLST_POINT_NOT_IN_GROUP = 3
BLST_AGGR_TYPE_MISMATCH = 4
BLST_VERIFY_FAIL = 5
BLST_PK_IS_INFINITY = 6
BLST_BAD_SCALAR = 7
# @chainsafe/blst extension: wrong byte length (multithread.test.ts:97)
BLST_INVALID_SIZE = 8

ERROR_NAMES = {
    BLST_BAD_ENCODING: "BLST_BAD_ENCODING",
    BLST_POINT_NOT_ON_CURVE: "BLST_POINT_NOT_ON_CURVE",
    BLST_POINT_NOT_IN_GROUP: "BLST_POINT_NOT_IN_GROUP",
    BLST_AGGR_TYPE_MISMATCH: "BLST_AGGR_TYPE_MISMATCH",
    BLST_VERIFY_FAIL: "BLST_VERIFY_FAIL",
    BLST_PK_IS_INFINITY: "BLST_PK_IS_INFINITY",
    BLST_BAD_SCALAR: "BLST_BAD_SCALAR",
    BLST_INVALID_SIZE: "BLST_INVALID_SIZE",
}


class BlstError(Exception):
    def __init__(self, code: int):
        self.code = code
        super().__init__(f"BLST_ERROR: {ERROR_NAMES[code]}")


def _be(b: bytes) -> int:
    return int.from_bytes(b, "big")


def _tobe(v: int, n: int = 48) -> bytes:
    return v.to_bytes(n, "big")


def g1_compress(Pt) -> bytes:
    if Pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = Pt
    out = bytearray(_tobe(x))
    out[0] |= 0x80
    if fp_lex_largest(y):
        out[0] |= 0x20
    return bytes(out)


def g1_serialize(Pt) -> bytes:
    """96-byte uncompressed (the pool's PointFormat.uncompressed)."""
    if Pt is None:
        return bytes([0x40]) + bytes(95)
    return _tobe(Pt[0]) + _tobe(Pt[1])


def g1_decompress(b: bytes):
    """Returns (code, point).  Mirrors blst POINTonE1_Uncompress_Z semantics."""
    if len(b) != 48:
        return BLST_INVALID_SIZE, None
    b0 = b[0]
    if not b0 & 0x80:
        return BLST_BAD_ENCODING, None
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return BLST_SUCCESS, None
        return BLST_BAD_ENCODING, None
    x = _be(bytes([b0 & 0x1F]) + b[1:])
    if x >= P:
        return BLST_BAD_ENCODING, None
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        return BLST_POINT_NOT_ON_CURVE, None
    if fp_lex_largest(y) != bool(b0 & 0x20):
        y = (-y) % P
    return BLST_SUCCESS, (x, y)


def g2_compress(Pt) -> bytes:
    if Pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = Pt
    out = bytearray(_tobe(x[1]) + _tobe(x[0]))
    out[0] |= 0x80
    if f2_lex_largest(y):
        out[0] |= 0x20
    return bytes(out)


def g2_serialize(Pt) -> bytes:
    if Pt is None:
        return bytes([0x40]) + bytes(191)
    x, y = Pt
    return _tobe(x[1]) + _tobe(x[0]) + _tobe(y[1]) + _tobe(y[0])


def g2_decompress(b: bytes):
    """96-byte compressed G2 -> (code, point).  blst POINTonE2_Uncompress_Z."""
    b0 = b[0]
    if not b0 & 0x80:
        return BLST_BAD_ENCODING, None
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:96]):
            return BLST_SUCCESS, None
        return BLST_BAD_ENCODING, None
    x1 = _be(bytes([b0 & 0x1F]) + b[1:48])
    x0 = _be(b[48:96])
    if x1 >= P or x0 >= P:
        return BLST_BAD_ENCODING, None
    x = (x0, x1)
    rhs = f2_add(f2_mul(f2_sqr(x), x), B2)
    y = f2_sqrt(rhs)
    if y is None:
        return BLST_POINT_NOT_ON_CURVE, None
    if f2_lex_largest(y) != bool(b0 & 0x20):
        y = f2_neg(y)
    return BLST_SUCCESS, (x, y)


def g2_deserialize(b: bytes):
    """192-byte uncompressed G2 -> (code, point).  blst POINTonE2_Deserialize_Z
    as @chainsafe/blst reaches it through P2_Affine(bytes, len): a 192-byte
    input must not carry the compression flag (len != (in[0] & 0x80 ? 96 :
    192) is BAD_ENCODING), the infinity flag needs every other bit zero, and
    the sign flag (0x20) on an uncompressed encoding is BAD_ENCODING."""
    b0 = b[0]
    if b0 & 0x80:
        return BLST_BAD_ENCODING, None
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:192]):
            return BLST_SUCCESS, None
        return BLST_BAD_ENCODING, None
    if b0 & 0x20:
        return BLST_BAD_ENCODING, None
    x1 = _be(bytes([b0 & 0x1F]) + b[1:48])
    x0 = _be(b[48:96])
    y1 = _be(b[96:144])
    y0 = _be(b[144:192])
    if max(x1, x0, y1, y0) >= P:
        return BLST_BAD_ENCODING, None
    pt = ((x0, x1), (y0, y1))
    if not E2.on_curve(pt):
        return BLST_POINT_NOT_ON_CURVE, None
    return BLST_SUCCESS, pt


def signature_from_bytes(b: bytes, validate: bool = True):
    """``bls.Signature.fromBytes(bytes, CoordType.affine, validate)``
    (maybeBatch.ts:23,36).  Raises BlstError like the reference throws."""
    if len(b) == 96:
        code, pt = g2_decompress(b)
    elif len(b) == 192:
        code, pt = g2_deserialize(b)
    else:
        code, pt = BLST_INVALID_SIZE, None
    if code != BLST_SUCCESS:
        raise BlstError(code)
    if validate and pt is not None and not g2_in_subgroup(pt):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


# --------------------------------------------------------------------------
# RFC 9380 hash_to_curve for G2
# --------------------------------------------------------------------------


def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in_bytes, s_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(s_in_bytes)
    l_i_b_str = len_in_bytes.to_bytes(2, "big")
    msg_prime = z_pad + msg + l_i_b_str + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    b1 = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = [b1]
    for i in range(2, ell + 1):
        prev = out[-1]
        out.append(hashlib.sha256(bytes(x ^ y for x, y in zip(b0, prev)) + bytes([i]) + dst_prime).digest())
    return b"".join(out)[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(_be(ub[off : off + L]) % P)
        out.append((e[0], e[1]))
    return out


# E2': y^2 = x^3 + A' x + B'
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)  # Z = -(2 + i)
E2_ISO = Curve(_Fp2Ops, SSWU_A, SSWU_B)


def map_to_curve_sswu(u):
    """RFC 9380 section 6.6.2 (straight-line description)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    z_u2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(z_u2), z_u2)  # Z^2 u^4 + Z u^2
    tv1 = F2_ZERO if f2_is_zero(den) else f2_inv(den)
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, tv1))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(z_u2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


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


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(Pt):
    if Pt is None:
        return None
    x, y = Pt
    xd = _poly(ISO_XDEN, x)
    yd = _poly(ISO_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    xn = f2_mul(_poly(ISO_XNUM, x), f2_inv(xd))
    yn = f2_mul(y, f2_mul(_poly(ISO_YNUM, x), f2_inv(yd)))
    return (xn, yn)


def clear_cofactor_g2(Pt):
    return E2.mul(Pt, H_EFF_G2)


def clear_cofactor_g2_psi(Pt):
    """Budroni-Pintore form: [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P).
    Equal to [h_eff]P (checked in tests)."""
    x = X_PARAM
    t1 = E2.mul(Pt, x * x - x - 1)
    t2 = E2.mul(psi(Pt), x - 1)
    t3 = psi(psi(E2.dbl(Pt)))
    return E2.add(E2.add(t1, t2), t3)


def hash_to_g2(msg: bytes, dst: bytes = DST_POP, stages: dict | None = None):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0p = map_to_curve_sswu(u0)
    q1p = map_to_curve_sswu(u1)
    q0 = iso_map_g2(q0p)
    q1 = iso_map_g2(q1p)
    r = E2.add(q0, q1)
    out = clear_cofactor_g2(r)
    if stages is not None:
        stages.update(u0=u0, u1=u1, q0=q0, q1=q1, r=r, h=out)
    return out


# --------------------------------------------------------------------------
# Fp12 = Fp[w] / (w^12 - 2 w^6 + 2), flat coefficient lists
# --------------------------------------------------------------------------


def f12(coeffs):
    c = [0] * 12
    for i, v in enumerate(coeffs):
        c[i] = v % P
    return tuple(c)


F12_ONE = f12([1])


def f12_mul(a, b):
    t = [0] * 23
    for i in range(12):
        ai = a[i]
        if ai == 0:
            continue
        for j in range(12):
            t[i + j] += ai * b[j]
    for k in range(22, 11, -1):
        c = t[k]
        if c:
            t[k - 6] += 2 * c
            t[k - 12] -= 2 * c
    return tuple(v % P for v in t[:12])


def f12_pow(a, e: int):
    r = F12_ONE
    b = a
    while e > 0:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_mul(b, b)
        e >>= 1
    return r


def f12_eq(a, b) -> bool:
    return all((x - y) % P == 0 for x, y in zip(a, b))


def f12_from_f2_at(c, k: int):
    """Embed Fp2 element c = c0 + c1 i at position w^k, with i = w^6 - 1."""
    out = [0] * 12
    out[k % 12] += c[0] - c[1]
    # c1 * w^6 * w^k
    kk = k + 6
    if kk < 12:
        out[kk] += c[1]
    else:  # w^12 = 2 w^6 - 2
        out[kk - 6] += 2 * c[1]
        out[kk - 12] -= 2 * c[1]
    return out


def _f12_sum(*lists):
    acc = [0] * 12
    for l in lists:
        for i, v in enumerate(l):
            acc[i] += v
    return f12(acc)


def f2_to_f12(c):
    return f12(f12_from_f2_at(c, 0))


def tower_to_f12(t):
    """Map a tower element ((c00, c01, c02), (c10, c11, c12)) of
    Fp12 = Fp6[w]/(w^2 - v), Fp6 = Fp2[v]/(v^3 - (1+i)) into this flat
    representation (v = w^2).  Used to compare with the HIP/C++ tower."""
    (a0, a1, a2), (b0, b1, b2) = t
    return _f12_sum(
        f12_from_f2_at(a0, 0), f12_from_f2_at(a1, 2), f12_from_f2_at(a2, 4),
        f12_from_f2_at(b0, 1), f12_from_f2_at(b1, 3), f12_from_f2_at(b2, 5),
    )


def _line_eval(lam, xt, yt, Pp):
    """Line of slope lam (computed on the twist) through T=(xt,yt) on the
    twist, untwisted by (x, y) -> (x / w^2, y / w^3), evaluated at P in G1 and
    multiplied by w^3 (an element of Fp4, killed by the final exponentiation):
        l * w^3 = y_P w^3 - lam x_P w^2 + (lam x_T - y_T)."""
    xp, yp = Pp
    c0 = f2_sub(f2_mul(lam, xt), yt)
    c2 = f2_neg(f2_muls(lam, xp))
    out = f12_from_f2_at(c0, 0)
    tmp = f12_from_f2_at(c2, 2)
    out = [a + b for a, b in zip(out, tmp)]
    out[3] += yp
    return f12(out)


def _vertical_eval(xt, Pp):
    """Vertical line x - x_T (untwisted, times w^2): x_P w^2 - x_T."""
    out = f12_from_f2_at(f2_neg(xt), 0)
    out[2] += Pp[0]
    return f12(out)


def miller_loop(Pp, Qq):
    """f_{|x|, Q}(P): affine double-and-add on the twist (T in E2 over Fp2),
    each line untwisted and evaluated at P into the flat Fp12.  Vertical lines
    are omitted (they lie in Fp6 and die in the final exponentiation).  The
    sign of x is applied in ``pairing``."""
    if Pp is None or Qq is None:
        return F12_ONE
    T = Qq
    f = F12_ONE
    n = -X_PARAM
    for bit in bin(n)[3:]:
        # doubling step
        xt, yt = T
        lam = f2_mul(f2_muls(f2_sqr(xt), 3), f2_inv(f2_muls(yt, 2)))
        f = f12_mul(f12_mul(f, f), _line_eval(lam, xt, yt, Pp))
        T = E2.dbl(T)
        if bit == "1":
            xt, yt = T
            xq, yq = Qq
            if f2_eq(xt, xq):
                # T == +-Q never happens for |x| < r with Q of order r
                raise AssertionError("degenerate Miller step")
            lam = f2_mul(f2_sub(yq, yt), f2_inv(f2_sub(xq, xt)))
            f = f12_mul(f, _line_eval(lam, xt, yt, Pp))
            T = E2.add(T, Qq)
    return f


FINAL_EXP = (P**12 - 1) // R


def final_exponentiation(f):
    return f12_pow(f, FINAL_EXP)


def pairing(Pp, Qq):
    """e(P, Q) with the sign of x handled: e = FE(f_{|x|})^-1 = FE(f)^(p^6)."""
    f = miller_loop(Pp, Qq)
    e = final_exponentiation(f)
    # x < 0: the optimal-ate value is FE(1/f) = FE(f)^-1 = FE(f)^(r-1)
    return f12_pow(e, R - 1) if X_PARAM < 0 else e


def multi_pairing_is_one(pairs) -> bool:
    """Prod e(P_i, Q_i) == 1 with ONE final exponentiation (the sign of x does
    not matter for an equality with 1)."""
    f = F12_ONE
    for Pp, Qq in pairs:
        f = f12_mul(f, miller_loop(Pp, Qq))
    return f12_eq(final_exponentiation(f), F12_ONE)


# --------------------------------------------------------------------------
# BLS signatures (IETF, POP ciphersuite)
# --------------------------------------------------------------------------


def sk_to_pk(sk: int):
    return E1.mul(G1, sk % R)


def sign(sk: int, msg: bytes, dst: bytes = DST_POP):
    return E2.mul(hash_to_g2(msg, dst), sk % R)


def core_verify(pk, msg: bytes, sig, dst: bytes = DST_POP) -> bool:
    """e(pk, H(m)) == e(G1, sig)  <=>  e(-G1, sig) * e(pk, H(m)) == 1."""
    h = hash_to_g2(msg, dst)
    return multi_pairing_is_one([(E1.neg(G1), sig), (pk, h)])


def aggregate_pubkeys(pks):
    """``bls.PublicKey.aggregate`` (chain/bls/utils.ts:11); throws on empty."""
    if len(pks) == 0:
        raise ValueError("EMPTY_AGGREGATE_ARRAY")
    acc = None
    for pk in pks:
        acc = E1.add(acc, pk)
    return acc


def batch_verify(sets, scalars) -> bool:
    """blst verifyMultipleAggregateSignatures with injected 64-bit scalars.
    sets: list of (pk_point, msg, sig_point); all already parsed/validated.
    Raises BlstError(PK_IS_INFINITY) like Pairing.mul_n_aggregate."""
    pairs = []
    s_acc = None
    for (pk, msg, sig), r in zip(sets, scalars):
        if pk is None:
            raise BlstError(BLST_PK_IS_INFINITY)
        pairs.append((E1.mul(pk, r), hash_to_g2(msg)))
        s_acc = E2.add(s_acc, E2.mul(sig, r))
    pairs.append((E1.neg(G1), s_acc))
    return multi_pairing_is_one(pairs)


# --------------------------------------------------------------------------
# Interop keys (packages/state-transition/src/util/interop.ts:19-23)
# --------------------------------------------------------------------------


def interop_secret_key(index: int) -> int:
    d = hashlib.sha256(index.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R


# --------------------------------------------------------------------------
# Job semantics of the reference pool (maybeBatch.ts:16-38)
# --------------------------------------------------------------------------


def verify_job(sets, scalars=None):
    """``verifySignatureSetsMaybeBatch`` for one job.

    sets: list of (pk_point_or_None, msg32, sig_bytes); pk already aggregated.
    Every signature is parsed + subgroup-checked first (``sets.map(fromBytes)``,
    maybeBatch.ts:20-24), raising BlstError on the first failure in set
    order.  n >= 2: random-scalar batch verify (``scalars`` injected);
    n == 1: core verify; n == 0: ValueError("Empty signature set").
    Returns the boolean verdict."""
    if len(sets) == 0:
        raise ValueError("Empty signature set")
    parsed = [(pk, msg, signature_from_bytes(sig, True)) for pk, msg, sig in sets]
    for pk, _, _ in parsed:
        if pk is None:
            raise BlstError(BLST_PK_IS_INFINITY)
    if len(parsed) >= 2:
        return batch_verify(parsed, scalars if scalars is not None else [1 + i for i in range(len(parsed))])
    pk, msg, sig = parsed[0]
    return core_verify(pk, msg, sig)
