"""ctypes binding of the C ABI in include/bgv.h (lodestar_amd/libbgv.so).

This is the Python counterpart of the N-API addon described in
INTEGRATION.md: plain pointers and sizes cross the boundary, nothing else.
There is no CPU fallback: if the gfx950 library is missing or no HIP device
is visible, every entry point raises ``BgvNativeError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BGV_LIB", os.path.join(HERE, "libbgv.so"))

# include/bgv.h enums
BGV_OK = 0
BGV_E_INVALID_ARG = -1
BGV_E_HIP = -2
BGV_E_NO_DEVICE = -3
BGV_E_TABLE_RANGE = -4
BGV_E_EMPTY_SET = -5
BGV_E_BAD_PUBKEY = -6
BGV_E_STATE = -7
ABI_VERSION = 4

SET_CODE_NAMES = {
    0: "BLST_SUCCESS",
    1: "BLST_BAD_ENCODING",
    2: "BLST_POINT_NOT_ON_CURVE",
    3: "BLST_POINT_NOT_IN_GROUP",
    4: "BLST_AGGR_TYPE_MISMATCH",
    5: "BLST_VERIFY_FAIL",
    6: "BLST_PK_IS_INFINITY",
    7: "BLST_BAD_SCALAR",
    8: "BLST_INVALID_SIZE",
    9: "BGV_INDEX_RANGE",
    10: "EMPTY_SIGNATURE_SET",
}

PK_COMPRESSED_48 = 0
PK_UNCOMPRESSED_96 = 1
N_STAGES = 16

EXPORTS = [
    "bgv_abi_version", "bgv_build_id", "bgv_set_code_name", "bgv_stage_name", "bgv_last_error", "bgv_open", "bgv_open_cfg",
    "bgv_cfg_default", "bgv_close",
    "bgv_pubkeys_set", "bgv_pubkeys_count", "bgv_pubkeys_get", "bgv_pubkeys_validate", "bgv_verify", "bgv_last_stats",
    "bgv_partial", "bgv_partial_finish", "bgv_combine_final", "bgv_debug_stages", "bgv_gen_keys", "bgv_gen_sign", "bgv_bench_fpmul",
    "bgv_bench_mad", "bgv_debug_fp_ops", "bgv_debug_g2_decode",
]
FP_OPS_N = 13


class BgvNativeError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"bgv status {status}: {msg}")
        self.status = status


class BgvBatch(ctypes.Structure):
    _fields_ = [
        ("n_sets", ctypes.c_uint32),
        ("n_jobs", ctypes.c_uint32),
        ("job_offsets", ctypes.c_void_p),
        ("pk_offsets", ctypes.c_void_p),
        ("pk_indices", ctypes.c_void_p),
        ("raw_pks", ctypes.c_void_p),
        ("n_raw", ctypes.c_uint32),
        ("msgs", ctypes.c_void_p),
        ("sigs", ctypes.c_void_p),
        ("sig_len", ctypes.c_void_p),
        ("scalars", ctypes.c_void_p),
        ("on_device", ctypes.c_uint32),
    ]


class BgvStats(ctypes.Structure):
    _fields_ = [
        ("stage_ms", ctypes.c_float * N_STAGES),
        ("total_ms", ctypes.c_float),
        ("batch_retries", ctypes.c_uint32),
        ("batch_sigs_success", ctypes.c_uint32),
        ("n_sets", ctypes.c_uint32),
        ("n_jobs", ctypes.c_uint32),
        ("pubkeys_aggregated", ctypes.c_uint64),
        ("split", ctypes.c_uint32),
        ("miller_lanes", ctypes.c_uint32),
        ("pairs_per_item", ctypes.c_uint32),
        ("msm", ctypes.c_uint32),
        ("lines", ctypes.c_uint32),
        ("defer_from", ctypes.c_uint32),
        ("clear_lanes", ctypes.c_uint32),
        ("miller_kv", ctypes.c_uint32),
    ]
    LAYOUT = ("split", "miller_lanes", "pairs_per_item", "msm", "lines", "defer_from", "clear_lanes", "miller_kv")

    def as_dict(self, lib=None):
        names = [lib.stage_name(i) for i in range(N_STAGES)] if lib else [str(i) for i in range(N_STAGES)]
        return {
            "stage_ms": dict(zip(names, [float(x) for x in self.stage_ms])),
            "total_ms": float(self.total_ms),
            "batch_retries": int(self.batch_retries),
            "batch_sigs_success": int(self.batch_sigs_success),
            "n_sets": int(self.n_sets),
            "n_jobs": int(self.n_jobs),
            "pubkeys_aggregated": int(self.pubkeys_aggregated),
            "layout": self.layout(),
        }

    def layout(self) -> dict:
        """the pipeline variant the last batch ran with (prepare() in bgv_api.hip)"""
        return {k: int(getattr(self, k)) for k in self.LAYOUT}


class BgvCfg(ctypes.Structure):
    """bgv_cfg (include/bgv.h): pipeline overrides for tests and A/B tools.
    Production contexts use the defaults (every field "auto")."""
    _fields_ = [("struct_size", ctypes.c_uint32)] + [
        (k, ctypes.c_int32) for k in
        ("split", "miller", "job_lanes", "msm", "pairs", "prefold", "lines", "defer_pct", "timing", "clear_lanes",
         "miller_kv", "cu_split")]
    AUTO = {"split": -1, "miller": -1, "job_lanes": 0, "msm": -1, "pairs": 0, "prefold": -1, "lines": -1,
            "defer_pct": -1, "timing": -1, "clear_lanes": -1, "miller_kv": -1, "cu_split": 0}

    @classmethod
    def make(cls, **over) -> "BgvCfg":
        bad = set(over) - set(cls.AUTO)
        if bad:
            raise ValueError(f"unknown bgv_cfg fields {sorted(bad)}")
        c = cls(struct_size=ctypes.sizeof(cls), **{**cls.AUTO, **over})
        return c


class BgvDebug(ctypes.Structure):
    """bgv_debug (include/bgv.h): host buffers for bgv_debug_stages."""
    _fields_ = [(k, ctypes.c_void_p) for k in
                ("sig_aff", "h_aff", "pk_agg", "rpk_aff", "s_aff", "pair_fe", "job_fe", "batch_fe")]


_lib = None
_lib_lock = threading.Lock()

ROOT = os.path.dirname(HERE)


def source_files(root: str = ROOT) -> list[str]:
    """The sources libbgv.so is compiled from, relative to the repo root."""
    csrc = os.path.join(root, "lodestar_amd", "csrc")
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".h", ".hip")))
    return [os.path.join("lodestar_amd", "csrc", f) for f in names] + [os.path.join("include", "bgv.h")]


def source_hash(root: str = ROOT) -> str:
    """SHA-256 over (path, content) of source_files(): the id tools/build.py
    compiles into the library (bgv_build_id) and load_library checks."""
    import hashlib

    h = hashlib.sha256()
    for rel in source_files(root):
        with open(os.path.join(root, rel), "rb") as f:
            data = f.read()
        h.update(rel.replace(os.sep, "/").encode() + b"\0" + len(data).to_bytes(8, "little") + data)
    return h.hexdigest()


def check_build_id(lib_id: str, root: str = ROOT) -> None:
    """A library compiled from other sources than the tree beside it is
    refused (variant builds carry the id plus '+' and their defines).  An
    install that ships the library without its csrc tree has nothing to
    compare against: the check is skipped with a warning."""
    try:
        want = source_hash(root)
    except OSError as e:
        import warnings
        warnings.warn(f"libbgv.so build id not checked: sources not readable ({e})", RuntimeWarning, stacklevel=2)
        return
    if lib_id != want and not lib_id.startswith(want + "+"):
        raise BgvNativeError(BGV_E_INVALID_ARG,
                             f"libbgv.so was built from other sources (id {lib_id[:16]}, tree {want[:16]}): "
                             "rebuild with __graft_entry__.build()")


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libbgv.so (no compute). Raises BgvNativeError when absent or when
    it was not compiled from the sources in this tree."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise BgvNativeError(BGV_E_NO_DEVICE, f"{path} not built (run __graft_entry__.build())")
        # One HIP runtime per process: torch ships its own libamdhip64 with the
        # same soname as /opt/rocm's.  Loaded first, torch's copy satisfies
        # libbgv's dependency; loaded after libbgv, torch brings a second
        # runtime that cannot open the GPU ("No HIP GPUs are available").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        try:
            lib = ctypes.CDLL(path)
            build_id_fn = lib.bgv_build_id
        except (OSError, AttributeError) as e:
            raise BgvNativeError(BGV_E_INVALID_ARG, f"{path}: not a loadable libbgv.so of this ABI ({e}): rebuild") from e
        build_id_fn.argtypes = []
        build_id_fn.restype = ctypes.c_char_p
        check_build_id(build_id_fn().decode())
        P = ctypes.c_void_p
        u32, i32, u64 = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64
        sig = {
            "bgv_abi_version": ([], ctypes.c_int),
            "bgv_set_code_name": ([ctypes.c_int], ctypes.c_char_p),
            "bgv_stage_name": ([ctypes.c_int], ctypes.c_char_p),
            "bgv_last_error": ([], ctypes.c_char_p),
            "bgv_open": ([ctypes.c_int, ctypes.POINTER(P)], ctypes.c_int),
            "bgv_open_cfg": ([ctypes.c_int, ctypes.POINTER(BgvCfg), ctypes.POINTER(P)], ctypes.c_int),
            "bgv_cfg_default": ([ctypes.POINTER(BgvCfg)], None),
            "bgv_close": ([P], ctypes.c_int),
            "bgv_pubkeys_set": ([P, u32, u32, P, u32], ctypes.c_int),
            "bgv_pubkeys_count": ([P, ctypes.POINTER(u32)], ctypes.c_int),
            "bgv_pubkeys_get": ([P, u32, u32, P], ctypes.c_int),
            "bgv_pubkeys_validate": ([P, P, u32, P], ctypes.c_int),
            "bgv_verify": ([P, ctypes.POINTER(BgvBatch), P, P, ctypes.POINTER(BgvStats)], ctypes.c_int),
            "bgv_partial": ([P, ctypes.POINTER(BgvBatch), P, P, P, ctypes.POINTER(i32)], ctypes.c_int),
            "bgv_partial_finish": ([P, P, ctypes.POINTER(BgvStats)], ctypes.c_int),
            "bgv_last_stats": ([P, ctypes.POINTER(BgvStats)], ctypes.c_int),
            "bgv_debug_stages": ([P, ctypes.POINTER(BgvBatch), P, P, ctypes.POINTER(BgvDebug)], ctypes.c_int),
            "bgv_combine_final": ([P, P, u32, ctypes.POINTER(i32)], ctypes.c_int),
            "bgv_gen_keys": ([P, u32, u32, u64], ctypes.c_int),
            "bgv_gen_sign": ([P, ctypes.POINTER(BgvBatch), P], ctypes.c_int),
            "bgv_bench_fpmul": ([P, u32, u32, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "bgv_bench_mad": ([P, u32, u32, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "bgv_debug_fp_ops": ([P, P, u32, P], ctypes.c_int),
            "bgv_debug_g2_decode": ([P, P, P, u32, P, P], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.bgv_abi_version() != ABI_VERSION:
            raise BgvNativeError(BGV_E_INVALID_ARG, f"{path}: ABI {lib.bgv_abi_version()}, expected {ABI_VERSION} (rebuild)")
        _lib = lib
        return lib


def _ptr(a) -> int | None:
    """address of a numpy array / torch tensor / None"""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())  # torch tensor (device-resident)


def _sync_producers(*objs) -> None:
    """Device-resident inputs must be complete before the library reads them
    (include/bgv.h, bgv_batch.on_device): the library runs on its own streams,
    which do not wait for the stream that produced a torch tensor.  Wait for
    the current torch stream of every device a tensor argument lives on (a
    tensor filled by torch.full / torch.zeros / a copy is otherwise still being
    written when the library's kernels read it, or -- for an output buffer --
    overwrites what they wrote)."""
    seen = set()
    for o in objs:
        vals = o.values() if isinstance(o, dict) else (o,)
        for a in vals:
            if a is None or isinstance(a, (np.ndarray, bytes, bytearray, int, float, str)):
                continue
            dev = getattr(a, "device", None)
            if dev is None or getattr(dev, "type", "") != "cuda":
                continue
            key = getattr(dev, "index", None)
            if key in seen:
                continue
            seen.add(key)
            import torch
            torch.cuda.current_stream(dev).synchronize()


class Device:
    """One bgv_ctx: a HIP device, its stream and its HBM pubkey table."""

    def __init__(self, device: int = 0, **cfg):
        """cfg: bgv_cfg overrides (tests and A/B tools only), e.g. miller=36, split=0"""
        self.lib = load_library()
        h = ctypes.c_void_p()
        if cfg:
            self._check(self.lib.bgv_open_cfg(device, ctypes.byref(BgvCfg.make(**cfg)), ctypes.byref(h)))
        else:
            self._check(self.lib.bgv_open(device, ctypes.byref(h)))
        self.h = h
        self.device = device
        self.last_stats = BgvStats()

    # -------------------------------------------------------------- helpers
    def _check(self, st: int):
        if st != BGV_OK:
            raise BgvNativeError(st, self.lib.bgv_last_error().decode())

    def stage_name(self, i: int) -> str:
        return self.lib.bgv_stage_name(i).decode()

    def close(self):
        if getattr(self, "h", None):
            self.lib.bgv_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------- pubkey table
    def pubkeys_set(self, first: int, data: bytes | np.ndarray, fmt: int):
        w = 48 if fmt == PK_COMPRESSED_48 else 96
        arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
        n = arr.size // w
        self._check(self.lib.bgv_pubkeys_set(self.h, first, n, arr.ctypes.data, fmt))

    def pubkeys_count(self) -> int:
        c = ctypes.c_uint32()
        self._check(self.lib.bgv_pubkeys_count(self.h, ctypes.byref(c)))
        return c.value

    def pubkeys_get(self, first: int, n: int) -> bytes:
        out = np.zeros(n * 96, dtype=np.uint8)
        self._check(self.lib.bgv_pubkeys_get(self.h, first, n, out.ctypes.data))
        return out.tobytes()

    def pubkeys_validate(self, pk48: bytes) -> np.ndarray:
        """PublicKey.fromBytes(pk, affine, validate=true) for each 48-byte key
        (processDeposit.ts:59): per-key bgv_set_code (0 = valid)."""
        n = len(pk48) // 48
        buf = np.frombuffer(pk48, dtype=np.uint8).copy()
        codes = np.zeros(max(n, 1), dtype=np.int32)
        self._check(self.lib.bgv_pubkeys_validate(self.h, buf.ctypes.data, n, codes.ctypes.data))
        return codes[:n]

    def gen_keys(self, first: int, n: int, seed: int):
        self._check(self.lib.bgv_gen_keys(self.h, first, n, seed))

    # --------------------------------------------------------------- batches
    @staticmethod
    def make_batch(arrays: dict, on_device: bool = False, sync_inputs: bool = True) -> BgvBatch:
        """sync_inputs=False: the caller guarantees device-resident inputs are
        complete (e.g. one torch.cuda.synchronize() after they were written, for
        inputs that are only read afterwards), and the per-call wait for torch's
        current stream is skipped; that wait can sit behind other contexts'
        kernels on a shared hardware queue."""
        b = BgvBatch()
        b.n_sets = int(arrays["n_sets"])
        b.n_jobs = int(arrays["n_jobs"])
        b.job_offsets = _ptr(arrays["job_offsets"])
        b.pk_offsets = _ptr(arrays["pk_offsets"])
        b.pk_indices = _ptr(arrays["pk_indices"])
        b.raw_pks = _ptr(arrays.get("raw_pks"))
        b.n_raw = int(arrays.get("n_raw", 0))
        b.msgs = _ptr(arrays["msgs"])
        b.sigs = _ptr(arrays.get("sigs"))
        b.sig_len = _ptr(arrays.get("sig_len"))
        b.scalars = _ptr(arrays.get("scalars"))
        b.on_device = 1 if on_device else 0
        if on_device and sync_inputs:
            _sync_producers(arrays)
        return b

    def verify(self, arrays: dict, on_device: bool = False, want_set_codes: bool = True, sync_inputs: bool = True):
        """returns (job_result int32[n_jobs], set_code int32[n_sets] | None)"""
        b = self.make_batch(arrays, on_device, sync_inputs)
        jr = np.zeros(max(b.n_jobs, 1), dtype=np.int32)
        sc = np.zeros(max(b.n_sets, 1), dtype=np.int32) if want_set_codes else None
        self._check(self.lib.bgv_verify(self.h, ctypes.byref(b), jr.ctypes.data,
                                        sc.ctypes.data if sc is not None else None, ctypes.byref(self.last_stats)))
        return jr[: b.n_jobs], (sc[: b.n_sets] if sc is not None else None)

    def partial(self, arrays: dict, on_device: bool = False, sync_inputs: bool = True):
        """bgv_partial: (miller576 bytes, set codes, provisional job results
        (-code rejected / 1 pending the combined check), no-job-rejected)."""
        b = self.make_batch(arrays, on_device, sync_inputs)
        out = np.zeros(576, dtype=np.uint8)
        sc = np.zeros(max(b.n_sets, 1), dtype=np.int32)
        jr = np.zeros(max(b.n_jobs, 1), dtype=np.int32)
        ok = ctypes.c_int32()
        self._check(self.lib.bgv_partial(self.h, ctypes.byref(b), out.ctypes.data, sc.ctypes.data, jr.ctypes.data,
                                         ctypes.byref(ok)))
        self._partial_jobs = b.n_jobs
        self._check(self.lib.bgv_last_stats(self.h, ctypes.byref(self.last_stats)))
        return out.tobytes(), sc[: b.n_sets], jr[: b.n_jobs], bool(ok.value)

    def partial_finish(self) -> np.ndarray:
        """bgv_partial_finish: per-job verdicts of the shard left by partial()."""
        n = getattr(self, "_partial_jobs", 0)
        jr = np.zeros(max(n, 1), dtype=np.int32)
        self._check(self.lib.bgv_partial_finish(self.h, jr.ctypes.data, ctypes.byref(self.last_stats)))
        return jr[:n]

    def debug_stages(self, arrays: dict, on_device: bool = False) -> dict:
        """bgv_debug_stages (test only): per-stage canonical values as numpy arrays."""
        b = self.make_batch(arrays, on_device)
        n, J = b.n_sets, b.n_jobs
        bufs = {"sig_aff": np.zeros((max(n, 1), 192), np.uint8), "h_aff": np.zeros((max(n, 1), 192), np.uint8),
                "pk_agg": np.zeros((max(n, 1), 96), np.uint8), "rpk_aff": np.zeros((max(n, 1), 96), np.uint8),
                "s_aff": np.zeros((max(J, 1), 192), np.uint8), "pair_fe": np.zeros((max(n + J, 1), 576), np.uint8),
                "job_fe": np.zeros((max(J, 1), 576), np.uint8), "batch_fe": np.zeros(576, np.uint8)}
        dbg = BgvDebug(**{k: v.ctypes.data for k, v in bufs.items()})
        jr = np.zeros(max(J, 1), dtype=np.int32)
        sc = np.zeros(max(n, 1), dtype=np.int32)
        self._check(self.lib.bgv_debug_stages(self.h, ctypes.byref(b), jr.ctypes.data, sc.ctypes.data, ctypes.byref(dbg)))
        out = {k: (v[: n] if k in ("sig_aff", "h_aff", "pk_agg", "rpk_aff") else v[: J] if k in ("s_aff", "job_fe")
                   else v[: n + J] if k == "pair_fe" else v) for k, v in bufs.items()}
        out["job_result"] = jr[:J]
        out["set_code"] = sc[:n]
        return out

    def combine_final(self, partials: list[bytes]) -> bool:
        buf = np.frombuffer(b"".join(partials), dtype=np.uint8) if partials else np.zeros(1, np.uint8)
        r = ctypes.c_int32()
        self._check(self.lib.bgv_combine_final(self.h, buf.ctypes.data, len(partials), ctypes.byref(r)))
        return bool(r.value)

    def gen_sign(self, arrays: dict, out, on_device: bool = False):
        _sync_producers(out)
        b = self.make_batch(arrays, on_device)
        self._check(self.lib.bgv_gen_sign(self.h, ctypes.byref(b), _ptr(out)))

    def debug_fp_ops(self, ab: np.ndarray) -> np.ndarray:
        """Device modular add/sub primitives (test only): ab is (n, 2, 12) u32
        limbs; returns (n, FP_OPS_N, 12) u32 (include/bgv.h bgv_debug_fp_ops)."""
        ab = np.ascontiguousarray(ab, dtype=np.uint32)
        n = ab.shape[0]
        out = np.zeros((n, FP_OPS_N, 12), np.uint32)
        self._check(self.lib.bgv_debug_fp_ops(self.h, ab.ctypes.data, n, out.ctypes.data))
        return out

    def debug_g2_decode(self, sigs192: np.ndarray, sig_len: np.ndarray):
        """Signature decode without the subgroup check (test only): sigs192 is
        (n, 192) u8, sig_len (n,) u32; returns ((n, 192) u8 affine points as
        x.c0 || x.c1 || y.c0 || y.c1 big-endian, (n,) i32 set codes)
        (include/bgv.h bgv_debug_g2_decode)."""
        sigs192 = np.ascontiguousarray(sigs192, dtype=np.uint8)
        sig_len = np.ascontiguousarray(sig_len, dtype=np.uint32)
        n = sig_len.shape[0]
        assert sigs192.shape == (n, 192)
        out = np.zeros((n, 192), np.uint8)
        codes = np.zeros(n, np.int32)
        self._check(self.lib.bgv_debug_g2_decode(self.h, sigs192.ctypes.data, sig_len.ctypes.data, n, out.ctypes.data,
                                                 codes.ctypes.data))
        return out, codes

    # ---------------------------------------------------------- microbench
    def bench_fpmul(self, lanes: int, iters: int) -> float:
        ms = ctypes.c_float()
        self._check(self.lib.bgv_bench_fpmul(self.h, lanes, iters, ctypes.byref(ms)))
        return ms.value

    def bench_mad(self, lanes: int, iters: int) -> float:
        ms = ctypes.c_float()
        self._check(self.lib.bgv_bench_mad(self.h, lanes, iters, ctypes.byref(ms)))
        return ms.value
