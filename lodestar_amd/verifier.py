"""Host-side mirror of Lodestar's BLS verifier interface, backed by the gfx950
HIP library through the C ABI (lodestar_amd/native.py -> include/bgv.h).

Reference interface (maschad/lodestar, packages/beacon-node/src/chain/bls/):

* ``IBlsVerifier`` (interface.ts:20-51): ``verifySignatureSets(sets, opts)``
  -> Promise<boolean>, ``close()``, ``canAcceptWork()``.  Here:
  ``BlsGpuVerifier.verify_signature_sets`` (a coroutine), ``close``,
  ``can_accept_work``.
* ``VerifySignatureOpts`` {batchable, verifyOnMainThread} (interface.ts:3-18).
* ``ISignatureSet`` single / aggregate (state-transition/src/util/
  signatureSets.ts:5-22).  Pubkeys are references into the HBM-resident
  ``index2pubkey`` table (``PubkeyTable``), so a set carries index lists
  instead of serialized points (BASELINE north_star); raw pubkeys outside
  the table are still accepted (``PublicKey.from_bytes``).
* Pool semantics of ``BlsMultiThreadWorkerPool`` (multithread/index.ts:
  151-431): sets chunked into jobs of <= 128 (``chunkify_maximize_chunk_size``,
  multithread/utils.ts:4-19), batchable jobs buffered up to 100 ms or until
  more than 32 sigs are waiting, job verdict = AND of its sets, the call's
  verdict = AND of its jobs, a job whose signature does not parse rejects
  with ``BLST_ERROR: BLST_<CODE>``, an empty aggregate rejects with
  ``EMPTY_AGGREGATE_ARRAY``, a job of zero sets rejects with
  ``Empty signature set`` (maybeBatch.ts:29-31), ``close()`` rejects pending
  jobs with ``QueueError(QUEUE_ABORTED)`` (multithread/index.ts:193-214).

What differs on purpose: the worker pool packs <= 128 sigs per worker
message (prepareWork, index.ts:405-420) because a CPU worker verifies one
batch at a time; a GPU wants one large batch, so every queued job is packed
into one device batch (bounded by ``max_sets_per_device_batch``).  Verdicts
are unaffected: the device checks the whole batch once and falls back to
per-job checks exactly where the worker retries (worker.ts:64-85).
"""
from __future__ import annotations

import asyncio
import enum
import math
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from . import native
from .dist import RESERVED_CAP, job_work, shard_jobs

MAX_SIGNATURE_SETS_PER_JOB = 128  # multithread/index.ts:39
MAX_BUFFERED_SIGS = 32            # multithread/index.ts:48
MAX_BUFFER_WAIT_MS = 100          # multithread/index.ts:57
MAX_JOBS_CAN_ACCEPT_WORK = 512    # multithread/index.ts:62
PRIORITY_CUS = 32  # CUs of the first device kept for verifyOnMainThread (bgv_cfg.cu_split; one per SE)
# device batches in flight per GPU, one context each (napi/index.js
# CONTEXTS_PER_DEVICE): the next batches' phase 1 fills the SIMDs a batch's
# Miller phase leaves idle (profiles/r06b_overlap_sizes.txt)
CONTEXTS_PER_DEVICE = 3
# the priority context's sizing job (BlsGpuVerifier._warm_priority)
G1_GENERATOR_96 = bytes.fromhex(
    "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"
    "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1")
IDENTITY_SIG_96 = bytes([0xC0]) + bytes(95)
MAX_SETS_PER_DEVICE_BATCH = 1 << 17
# a device batch of at least this many sets (and >= 2 jobs) is split by job
# over the idle devices: each returns a partial Miller product and ONE final
# exponentiation checks their product.  Below it the batch runs
# whole on one device and other devices take the next batch: one GPU verifies
# 2,000-4,000 sets in 7-10 ms, within ~2 ms of the split, which pays a host
# round trip and the combined final exponentiation
SHARD_MIN_SETS = 4096


class BlsError(Exception):
    """Rejection raised by verify_signature_sets; ``message`` follows the
    strings the reference's tests match (multithread.test.ts:97,
    test/spec/general/bls.ts:37)."""

    def __init__(self, message: str, code: int | None = None):
        super().__init__(message)
        self.message = message
        self.code = code


class QueueErrorCode(str, enum.Enum):
    QUEUE_ABORTED = "QUEUE_ERROR_QUEUE_ABORTED"  # util/queue/errors.ts


class QueueError(Exception):
    def __init__(self, code: QueueErrorCode = QueueErrorCode.QUEUE_ABORTED):
        super().__init__(code.value)
        self.code = code


def error_for_code(code: int) -> BlsError:
    if code == 10:
        return BlsError("Empty signature set", code)
    return BlsError(f"BLST_ERROR: {native.SET_CODE_NAMES.get(code, 'BLST_UNKNOWN')}", code)


# --------------------------------------------------------------- data types
class SignatureSetType(str, enum.Enum):
    single = "single"
    aggregate = "aggregate"


@dataclass(frozen=True)
class PublicKey:
    """A trusted pubkey: either a row of the device index2pubkey table
    (``index``) or raw bytes (96 B uncompressed x||y, or 48 B compressed)."""

    index: int | None = None
    raw: bytes | None = None

    @staticmethod
    def from_bytes(b: bytes) -> "PublicKey":
        if len(b) not in (48, 96):
            raise BlsError("BLST_ERROR: BLST_INVALID_SIZE", 8)
        return PublicKey(raw=bytes(b))


@dataclass
class VerifySignatureOpts:
    batchable: bool = False
    verifyOnMainThread: bool = False


@dataclass
class ISignatureSet:
    type: SignatureSetType
    signingRoot: bytes
    signature: bytes
    pubkey: PublicKey | None = None
    pubkeys: list[PublicKey] = field(default_factory=list)


def create_single_signature_set_from_components(pubkey: PublicKey, signing_root: bytes, signature: bytes) -> ISignatureSet:
    """util/signatureSets.ts:40-51"""
    return ISignatureSet(SignatureSetType.single, bytes(signing_root), bytes(signature), pubkey=pubkey)


def create_aggregate_signature_set_from_components(pubkeys, signing_root: bytes, signature: bytes) -> ISignatureSet:
    """util/signatureSets.ts:53-64"""
    return ISignatureSet(SignatureSetType.aggregate, bytes(signing_root), bytes(signature), pubkeys=list(pubkeys))


def get_aggregated_pubkeys_count(sets) -> int:
    """chain/bls/utils.ts:18-26"""
    return sum(len(s.pubkeys) for s in sets if s.type == SignatureSetType.aggregate)


def chunkify_maximize_chunk_size(arr: list, min_per_chunk: int) -> list[list]:
    """multithread/utils.ts:4-19: split maximizing the smallest chunk."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [arr]
    per_chunk = math.ceil(len(arr) / chunk_count)
    return [arr[i : i + per_chunk] for i in range(0, len(arr), per_chunk)]


# ------------------------------------------------------------ pubkey table
class PubkeyTable:
    """``index2pubkey`` resident in HBM (state-transition/src/cache/
    pubkeyCache.ts:6,56-77 syncPubkeys; cache/epochContext.ts:701-704
    addPubkey).  One replica per device."""

    def __init__(self, devices: list[native.Device]):
        self.devices = devices
        self.pubkey2index: dict[bytes, int] = {}

    def __len__(self):
        return self.devices[0].pubkeys_count()

    def sync_pubkeys(self, pubkeys48: list[bytes]):
        """Append every validator pubkey not yet in the table (compressed).
        A key that does not deserialize throws like PublicKey.fromBytes and
        leaves the table unchanged."""
        if len(self.pubkey2index) != len(self):  # pubkeyCache.ts:61-63
            raise BlsError(f"Pubkey indices have fallen out of sync: {len(self.pubkey2index)} != {len(self)}")
        start = len(self)
        new = pubkeys48[start:]
        if not new:
            return
        blob = b"".join(new)
        self._set(start, blob)
        for i, pk in enumerate(new):
            self.pubkey2index[bytes(pk)] = start + i

    def add_pubkey(self, index: int, pubkey48: bytes):
        """epochContext.ts:701-704.  The device table is append-only: index
        may rewrite a row or append the next one, not leave a gap."""
        self._set(index, pubkey48)
        self.pubkey2index[bytes(pubkey48)] = index

    def _set(self, first: int, blob: bytes):
        for d in self.devices:
            try:
                d.pubkeys_set(first, blob, native.PK_COMPRESSED_48)
            except native.BgvNativeError as e:
                if e.status == native.BGV_E_BAD_PUBKEY:
                    raise BlsError(str(e).split(": ", 1)[-1]) from e
                raise

    def __getitem__(self, index: int) -> PublicKey:
        return PublicKey(index=index)


# ------------------------------------------------------- batch marshalling
def encode_jobs(jobs: list[list[ISignatureSet]], scalars: np.ndarray | None = None) -> dict:
    """Flatten jobs of sets into the SoA arrays of bgv_batch (include/bgv.h).
    Raises BlsError("EMPTY_AGGREGATE_ARRAY") like PublicKey.aggregate."""
    job_off = [0]
    pk_off = [0]
    idx: list[int] = []
    raw: list[bytes] = []
    raw_pos: dict[bytes, int] = {}
    n = sum(len(j) for j in jobs)
    msgs = np.zeros((max(n, 1), 32), dtype=np.uint8)
    sigs = np.zeros((max(n, 1), 192), dtype=np.uint8)
    sig_len = np.zeros(max(n, 1), dtype=np.uint32)
    i = 0
    for job in jobs:
        for s in job:
            pks = [s.pubkey] if s.type == SignatureSetType.single else s.pubkeys
            if len(pks) == 0:
                raise BlsError("EMPTY_AGGREGATE_ARRAY")
            for pk in pks:
                if pk.index is not None:
                    idx.append(pk.index)
                else:
                    r = pk.raw if len(pk.raw) == 96 else _decompress_raw48(pk.raw)
                    if r not in raw_pos:
                        raw_pos[r] = len(raw)
                        raw.append(r)
                    idx.append(0x80000000 | raw_pos[r])
            pk_off.append(len(idx))
            if len(s.signingRoot) != 32:
                raise BlsError("signingRoot must be 32 bytes")
            msgs[i] = np.frombuffer(s.signingRoot, dtype=np.uint8)
            sl = len(s.signature)
            sig_len[i] = sl
            if sl in (96, 192):
                sigs[i, :sl] = np.frombuffer(s.signature, dtype=np.uint8)
            i += 1
        job_off.append(i)
    out = {
        "n_sets": n,
        "n_jobs": len(jobs),
        "job_offsets": np.array(job_off, dtype=np.uint32),
        "pk_offsets": np.array(pk_off, dtype=np.uint32),
        "pk_indices": np.array(idx if idx else [0], dtype=np.uint32),
        "raw_pks": np.frombuffer(b"".join(raw), dtype=np.uint8).copy() if raw else None,
        "n_raw": len(raw),
        "msgs": msgs,
        "sigs": sigs,
        "sig_len": sig_len,
        "scalars": scalars,
    }
    return out


def _decompress_raw48(b: bytes) -> bytes:
    raise BlsError("raw compressed pubkeys must be added to the table (PubkeyTable.add_pubkey)")


def check_sets(sets: list[ISignatureSet]) -> None:
    """Caller-side checks of one verifySignatureSets call: PublicKey.aggregate
    throws EMPTY_AGGREGATE_ARRAY (chain/bls/utils.ts:11); a raw key must be a
    96-byte uncompressed point (compressed keys live in the table); a signing
    root is 32 bytes.  Pubkey indices past the table are reported per set by
    the device (BGV_INDEX_RANGE rejects only that job)."""
    for s in sets:
        pks = [s.pubkey] if s.type == SignatureSetType.single else s.pubkeys
        if s.type == SignatureSetType.aggregate and len(pks) == 0:
            raise BlsError("EMPTY_AGGREGATE_ARRAY")
        for pk in pks:
            if pk is None:
                raise BlsError("EMPTY_AGGREGATE_ARRAY")
            if pk.index is None and len(pk.raw) != 96:
                _decompress_raw48(pk.raw)
            if pk.index is not None and not (0 <= pk.index < 0x80000000):
                raise BlsError(f"pubkey index {pk.index} out of range")
        if len(s.signingRoot) != 32:
            raise BlsError("signingRoot must be 32 bytes")


# ----------------------------------------------------------------- verifier
@dataclass
class _Job:
    sets: list
    opts: VerifySignatureOpts
    future: asyncio.Future
    added: float


class BlsGpuVerifier:
    """``IBlsVerifier`` on one or more MI355X devices, one context per device
    (one host process owns them all, as the reference's pool owns its workers,
    chain/chain.ts:199-202).

    devices: HIP device ordinals; every device holds a replica of the pubkey
    table.  Every idle device takes a device batch of the queued jobs; a batch
    of >= ``shard_min_sets`` sets is split by job over all idle devices instead,
    each returning a partial Miller product (bgv_partial), combined by ONE
    final exponentiation (bgv_combine_final); when that check fails every
    shard localises its own failing jobs (bgv_partial_finish)."""

    def __init__(self, devices=(0,), metrics: dict | None = None, scalar_seed: int | None = None,
                 max_sets_per_device_batch: int = MAX_SETS_PER_DEVICE_BATCH, shard_min_sets: int = SHARD_MIN_SETS,
                 priority_cus: int | None = None, bls_verify_all_multi_thread: bool = False,
                 contexts_per_device: int = CONTEXTS_PER_DEVICE):
        # priority_cus CUs of the first device (a multiple of 8) are kept for
        # verifyOnMainThread (bgv_cfg.cu_split): its own context runs there,
        # the first bulk context leaves them free; 0 shares every CU.  Default:
        # PRIORITY_CUS on a pool of two or more devices (sharded batches give
        # device 0 a RESERVED_CAP-weighted shard), 0 on one device, whose bulk
        # batches would otherwise run ~13-20% slower.
        # bls_verify_all_multi_thread (chain/options.ts:14, multithread/index.ts:124):
        # verifyOnMainThread calls join the queue like any other, no CUs are
        # reserved and no priority context is opened
        devices = list(devices)
        if priority_cus is None:
            priority_cus = PRIORITY_CUS if len(devices) > 1 else 0
        if bls_verify_all_multi_thread:
            priority_cus = 0
        self.bls_verify_all_multi_thread = bls_verify_all_multi_thread
        self.priority_cus = priority_cus
        # contexts_per_device device batches in flight per GPU (one context
        # each, own table replica); every bulk context of the first device
        # leaves the reserved CUs free.  Context k runs on device entry _ctx_dev[k]
        if contexts_per_device < 1:
            raise ValueError(f"contexts_per_device {contexts_per_device}")
        self.contexts_per_device = contexts_per_device
        self.n_devices = len(devices)
        self._ctx_dev = [i for i in range(len(devices)) for _ in range(contexts_per_device)]
        self.devices = [native.Device(devices[i], cu_split=-priority_cus) if i == 0 and priority_cus > 0
                        else native.Device(devices[i]) for i in self._ctx_dev]
        if bls_verify_all_multi_thread:
            self.prio = None
        else:
            self.prio = native.Device(devices[0], cu_split=priority_cus) if priority_cus > 0 else native.Device(devices[0])
        self.prio_reserved = priority_cus > 0  # device 0's bulk context runs at RESERVED_CAP (shard_jobs caps)
        if self.prio is not None:
            self._warm_priority()
        self._prio_lock = threading.Lock()
        self._shard_min = shard_min_sets
        self._idle = [True] * len(self.devices)
        self.table = PubkeyTable(self._contexts())
        self.metrics = metrics if metrics is not None else _new_metrics()
        self._rng = np.random.default_rng(scalar_seed) if scalar_seed is not None else None
        self._max_batch = max_sets_per_device_batch
        self._jobs: list[_Job] = []
        self._buffered: list[_Job] = []
        self._buffered_sigs = 0
        self._buffer_handle = None
        self._closed = False
        self._busy = 0
        self._exec = ThreadPoolExecutor(max_workers=len(self.devices) + 1)  # + the main-thread path
        self._dev_locks = [threading.Lock() for _ in self.devices]

    # -- IBlsVerifier ---------------------------------------------------
    def can_accept_work(self) -> bool:
        """multithread/index.ts:143-149.  A queued job joins the next device
        batch, so work is accepted while the queue holds fewer than
        MAX_JOBS_CAN_ACCEPT_WORK jobs and less than one full device batch of
        sets, whether or not a batch is in flight (a GPU wants large batches;
        gating on idle devices would stall the network processor for every
        batch, network/processor/index.ts:406)."""
        return (not self._closed and len(self._jobs) < MAX_JOBS_CAN_ACCEPT_WORK
                and sum(len(j.sets) for j in self._jobs) < self._max_batch)

    async def verify_signature_sets(self, sets: list[ISignatureSet], opts: VerifySignatureOpts | None = None) -> bool:
        opts = opts or VerifySignatureOpts()
        self.metrics["aggregated_pubkeys_total"] += get_aggregated_pubkeys_count(sets)
        # the checks the reference makes on the caller's side before queueing
        # (getAggregatedPubkey, utils.ts:5-16), so a bad call cannot fail a
        # device batch it shares with other callers
        check_sets(sets)
        if opts.verifyOnMainThread and not self.bls_verify_all_multi_thread:
            # unbuffered, high priority (multithread/index.ts:155-167): one
            # device batch on the priority context, off the event loop; it
            # never waits for the bulk contexts' locks or waves
            r = await asyncio.get_running_loop().run_in_executor(self._exec, self._run_priority, sets)
            if isinstance(r, Exception):
                raise r
            return r
        chunks = chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB)
        results = await asyncio.gather(*[self._queue_work(c, opts) for c in chunks])
        if len(results) == 0:
            raise BlsError("Empty results array")
        return all(r is True for r in results)

    async def close(self):
        self._closed = True
        if self._buffer_handle is not None:
            self._buffer_handle.cancel()
            self._buffer_handle = None
        for j in self._jobs + self._buffered:
            if not j.future.done():
                j.future.set_exception(QueueError(QueueErrorCode.QUEUE_ABORTED))
        self._jobs.clear()
        self._buffered.clear()
        self._exec.shutdown(wait=True)
        for d in self._contexts():
            d.close()

    # -- synchronous helpers ------------------------------------------------
    def verify_signature_sets_maybe_batch(self, sets: list[ISignatureSet]) -> bool:
        """maybeBatch.ts:16-38 for one job, synchronously (BlsSingleThreadVerifier
        path, singleThread.ts:14-35)."""
        check_sets(sets)
        r = self._run_device_batch([sets], [0])[0]
        if isinstance(r, Exception):
            raise r
        return r

    def verify_signature_set(self, s: ISignatureSet) -> bool:
        """util/signatureSets.ts:24-38 verifySignatureSet: the signature is
        parsed and group-checked; single -> verify(pk, root), aggregate ->
        verifyAggregate(pks, root).  One set, one device batch (n = 1): the
        random scalar of the batch equation cannot change the verdict (GT has
        prime order r and the scalar is nonzero mod r)."""
        if s.type == SignatureSetType.aggregate and len(s.pubkeys) == 0:
            raise BlsError("EMPTY_AGGREGATE_ARRAY")
        return self.verify_signature_sets_maybe_batch([s])

    def is_valid_bls_aggregate(self, public_keys: list[PublicKey], message: bytes, signature: bytes) -> bool:
        """light-client/src/validation.ts:152-175 isValidBlsAggregate: aggregate
        the keys, deserialize + group-check the signature, verify; each failure
        re-thrown with the reference's prefix."""
        if len(public_keys) == 0:
            raise BlsError("Error aggregating pubkeys: EMPTY_AGGREGATE_ARRAY")
        s = create_aggregate_signature_set_from_components(list(public_keys), message, signature)
        try:
            return self.verify_signature_sets_maybe_batch([s])
        except BlsError as e:
            raise BlsError(f"Error deserializing signature: {e}", getattr(e, "code", None)) from e

    # -- queueing -------------------------------------------------------------
    async def _queue_work(self, sets, opts) -> bool:
        if self._closed:
            raise QueueError(QueueErrorCode.QUEUE_ABORTED)
        loop = asyncio.get_running_loop()
        job = _Job(sets, opts, loop.create_future(), time.monotonic())
        if opts.batchable:
            if not self._buffered:
                self._buffer_handle = loop.call_later(MAX_BUFFER_WAIT_MS / 1000, self._run_buffered)
            self._buffered.append(job)
            self._buffered_sigs += len(sets)
            if self._buffered_sigs > MAX_BUFFERED_SIGS:
                self._buffer_handle.cancel()
                self._run_buffered()
        else:
            self._jobs.append(job)
            loop.call_soon(self._schedule)
        return await job.future

    def _run_buffered(self):
        self._jobs.extend(self._buffered)
        self._buffered = []
        self._buffered_sigs = 0
        self._buffer_handle = None
        asyncio.get_running_loop().call_soon(self._schedule)

    def _schedule(self):
        """every idle device takes a device batch of the queued jobs; a large
        batch is split over all idle devices (SHARD_MIN_SETS)"""
        while not self._closed and self._jobs and any(self._idle):
            take, n = [], 0
            while self._jobs and (n == 0 or n + len(self._jobs[0].sets) <= self._max_batch):
                j = self._jobs.pop(0)
                take.append(j)
                n += len(j.sets)
            idle = self._spread_contexts(idle_only=True)
            devs = idle if (len(idle) > 1 and len(take) > 1 and n >= self._shard_min) else [self._best_idle_context()]
            for d in devs:
                self._idle[d] = False
            self._busy += 1
            self.peak_busy = max(getattr(self, "peak_busy", 0), self._busy)  # batches in flight at once (test hook)
            asyncio.ensure_future(self._run(take, devs))

    async def _run(self, jobs: list[_Job], devs: list[int]):
        loop = asyncio.get_running_loop()
        try:
            now = time.monotonic()
            for j in jobs:
                self.metrics["job_wait_time_s"].append(now - j.added)
            results = await loop.run_in_executor(self._exec, self._run_device_batch, [j.sets for j in jobs], devs)
            for j, r in zip(jobs, results):
                if j.future.done():
                    continue
                if isinstance(r, Exception):
                    j.future.set_exception(r)
                else:
                    j.future.set_result(r)
        except Exception as e:  # device failure rejects the whole package (index.ts:386-393)
            for j in jobs:
                if not j.future.done():
                    j.future.set_exception(e)
        finally:
            self._busy -= 1
            for d in devs:
                self._idle[d] = True
            loop.call_soon(self._schedule)

    # -- device -------------------------------------------------------------
    def _scalars(self, n: int) -> np.ndarray | None:
        if self._rng is None:
            return None  # drawn inside the library (device ChaCha20 keyed by getrandom)
        s = self._rng.integers(1, 2**64 - 1, size=max(n, 1), dtype=np.uint64, endpoint=True)
        return s

    @staticmethod
    def _verdict(r: int):
        return True if r == 1 else False if r == 0 else error_for_code(-r)

    def _record(self, st: native.BgvStats, seconds: float):
        self.metrics["batch_retries"] += int(st.batch_retries)
        self.metrics["batch_sigs_success"] += int(st.batch_sigs_success)
        self.metrics["device_time_s"] += seconds

    def _warm_priority(self):
        """sizes the priority context's work buffers for a full job (128 sets)
        at construction, so a verifyOnMainThread call never frees and regrows
        them (a hipFree synchronises the device and would wait for the bulk
        contexts' batches).  One dummy job: the G1 generator as a raw key and
        the identity signature; its verdict is ignored."""
        one = create_single_signature_set_from_components(PublicKey(raw=G1_GENERATOR_96), bytes(32), IDENTITY_SIG_96)
        self.prio.verify(encode_jobs([[one] * MAX_SIGNATURE_SETS_PER_JOB], np.ones(MAX_SIGNATURE_SETS_PER_JOB, np.uint64)),
                         want_set_codes=False)

    def _contexts(self) -> list:
        return self.devices + ([self.prio] if self.prio is not None else [])

    def _spread_contexts(self, idle_only: bool = False) -> list[int]:
        """the first (idle) context of each device: where a sharded batch goes"""
        out, seen = [], set()
        for k, dv in enumerate(self._ctx_dev):
            if dv not in seen and (not idle_only or self._idle[k]):
                seen.add(dv)
                out.append(k)
        return out

    def _best_idle_context(self) -> int:
        """an idle context on the device with the fewest batches in flight"""
        busy = [0] * self.n_devices
        for k, f in enumerate(self._idle):
            if not f:
                busy[self._ctx_dev[k]] += 1
        return min((k for k, f in enumerate(self._idle) if f), key=lambda k: (busy[self._ctx_dev[k]], k))

    def _run_priority(self, sets: list[ISignatureSet]):
        """verifyOnMainThread's device batch on the priority context"""
        t0 = time.perf_counter()
        try:
            arrays = encode_jobs([sets], self._scalars(len(sets)))
            with self._prio_lock:
                t1 = time.perf_counter()
                jr, _ = self.prio.verify(arrays, want_set_codes=False)
                self._record(self.prio.last_stats, time.perf_counter() - t1)
        except Exception as e:  # noqa: BLE001 -- a device error rejects the call
            return e
        finally:
            # mainThreadDurationInThreadPool (multithread/index.ts:156-167): timed
            # in a finally, so calls that throw are observed too
            self.metrics["main_thread_time_s"] += time.perf_counter() - t0
            self.metrics["main_thread_calls"] += 1
        return self._verdict(int(jr[0]))

    def _run_device_batch(self, jobs: list[list[ISignatureSet]], devs: list[int] | None = None) -> list:
        """Verify a list of jobs on the devices `devs` (default: all); returns
        per job True / False / BlsError.  One device: bgv_verify.  Several: the
        jobs are sharded by work, sets + pubkey references (dist.job_work,
        dist.shard_jobs), every shard reduced to
        a partial Miller product, the partials combined by one final
        exponentiation, and only when that fails each shard localised on its
        own device."""
        if not jobs:
            return []
        devs = self._spread_contexts() if devs is None else list(devs)
        if len(devs) > 1:
            refs = [sum(1 if s.type == SignatureSetType.single else len(s.pubkeys) for s in j) for j in jobs]
            caps = [RESERVED_CAP if self._ctx_dev[d] == 0 and self.prio_reserved else 1.0 for d in devs]
            shards = shard_jobs(job_work([len(j) for j in jobs], refs), len(devs), caps)
        else:
            shards = [list(range(len(jobs)))]
        live = [(devs[r], ids) for r, ids in enumerate(shards) if ids]
        out: list = [None] * len(jobs)
        self.metrics["sets_started"] += sum(len(j) for j in jobs)
        self.metrics["jobs_started"] += len(jobs)
        if len(live) == 1:
            d, ids = live[0]
            try:
                arrays = encode_jobs(jobs, self._scalars(sum(len(j) for j in jobs)))
                with self._dev_locks[d]:
                    t0 = time.perf_counter()
                    jr, _ = self.devices[d].verify(arrays, want_set_codes=False)
                    self._record(self.devices[d].last_stats, time.perf_counter() - t0)
            except Exception as e:  # noqa: BLE001 -- a device error rejects the package (index.ts:386-393)
                return [e] * len(jobs)
            return [self._verdict(r) for r in jr.tolist()]
        # every participating context stays locked from its partial to its
        # localisation (the partial's intermediates live on the context)
        locks = [self._dev_locks[d] for d, _ in sorted(live)]
        for lk in locks:
            lk.acquire()
        try:
            t0 = time.perf_counter()
            parts: list = [None] * len(live)

            def run_partial(k):
                d, ids = live[k]
                try:
                    sub = [jobs[i] for i in ids]
                    parts[k] = self.devices[d].partial(encode_jobs(sub, self._scalars(sum(len(j) for j in sub))))
                except Exception as e:  # noqa: BLE001
                    parts[k] = e

            self._parallel(run_partial, len(live))
            failed = [k for k in range(len(live)) if isinstance(parts[k], Exception)]
            for k in failed:  # a device error rejects that shard's jobs
                for i in live[k][1]:
                    out[i] = parts[k]
            ok_shards = [k for k in range(len(live)) if k not in failed]
            if not ok_shards:
                return out
            d0 = live[ok_shards[0]][0]
            valid = self.devices[d0].combine_final([parts[k][0] for k in ok_shards])
            finals: list = [None] * len(live)
            if valid:
                for k in ok_shards:
                    finals[k] = parts[k][2]  # provisional: 1, or -code for a rejected job (final)
            else:
                def run_finish(k):
                    try:
                        finals[k] = self.devices[live[k][0]].partial_finish()
                    except Exception as e:  # noqa: BLE001
                        finals[k] = e

                self._parallel(run_finish, len(live), only=ok_shards)
            valid_sets = 0
            for k in ok_shards:
                ids = live[k][1]
                if isinstance(finals[k], Exception):
                    for i in ids:
                        out[i] = finals[k]
                    continue
                for i, r in zip(ids, np.asarray(finals[k]).tolist()):
                    out[i] = self._verdict(int(r))
                    if valid and r == 1:
                        valid_sets += len(jobs[i])
            self.metrics["batch_retries"] += 0 if valid else 1
            self.metrics["batch_sigs_success"] += valid_sets
            self.metrics["device_time_s"] += time.perf_counter() - t0
        finally:
            for lk in locks:
                lk.release()
        return out

    @staticmethod
    def _parallel(fn, n: int, only=None):
        ks = list(range(n)) if only is None else list(only)
        if len(ks) == 1:
            fn(ks[0])
            return
        ths = [threading.Thread(target=fn, args=(k,)) for k in ks]
        for t in ths:
            t.start()
        for t in ths:
            t.join()


class BlsGpuSingleThreadVerifier:
    """BlsSingleThreadVerifier (chain/bls/singleThread.ts:7-46), which
    chain.ts:200-202 builds instead of the pool when blsVerifyAllMainThread is
    set: maybeBatch on one device context in the calling thread (the event loop
    waits, as it does for blst on the main thread); can_accept_work() is always
    True.  Its pubkey table is its own replica."""

    def __init__(self, device: int = 0, metrics: dict | None = None):
        self.device = native.Device(device)
        self.table = PubkeyTable([self.device])
        self.metrics = metrics if metrics is not None else {"aggregated_pubkeys_total": 0, "main_thread_time_s": 0.0,
                                                            "main_thread_calls": 0}
        self._closed = False

    async def verify_signature_sets(self, sets: list[ISignatureSet], opts: VerifySignatureOpts | None = None) -> bool:
        if self._closed:
            raise QueueError(QueueErrorCode.QUEUE_ABORTED)
        self.metrics["aggregated_pubkeys_total"] += get_aggregated_pubkeys_count(sets)
        check_sets(sets)  # getAggregatedPubkey's checks (utils.ts:5-16)
        t0 = time.perf_counter()
        jr, _ = self.device.verify(encode_jobs([sets]), want_set_codes=False)
        r = BlsGpuVerifier._verdict(int(jr[0]))
        if isinstance(r, Exception):
            raise r  # only runs without exceptions are timed, as in the reference
        self.metrics["main_thread_time_s"] += time.perf_counter() - t0
        self.metrics["main_thread_calls"] += 1
        return r

    def can_accept_work(self) -> bool:
        return True

    async def close(self):
        if not self._closed:
            self._closed = True
            self.device.close()


async def reject_first_invalid_resolve_all_valid(is_valid_awaitables) -> dict:
    """chain/blocks/verifyBlocksSignatures.ts:69-89: resolves {"allValid": False,
    "index": i} at the first False to arrive, {"allValid": True} when all are
    True; an exception rejects."""
    tasks = [asyncio.ensure_future(a) for a in is_valid_awaitables]
    idx = {t: i for i, t in enumerate(tasks)}
    pending = set(tasks)
    try:
        while pending:
            done, pending = await asyncio.wait(pending, return_when=asyncio.FIRST_COMPLETED)
            for t in sorted(done, key=lambda t: idx[t]):
                if not t.result():
                    return {"allValid": False, "index": idx[t]}
        return {"allValid": True}
    finally:
        for t in pending:
            t.cancel()


async def verify_blocks_signatures(bls: "BlsGpuVerifier", blocks_sets: list[list[ISignatureSet]],
                                   coalesce: bool = True) -> dict:
    """verifyBlocksSignatures (chain/blocks/verifyBlocksSignatures.ts:16-60) for
    a segment of blocks.  coalesce=False issues one verifySignatureSets per
    block exactly like the reference; coalesce=True sends
    the whole segment as ONE device batch with one job per block (each block
    <= 128 sets is exactly one reference job), so the per-block verdicts come
    from a single whole-segment pairing check plus per-block checks only on
    failure.  Verdict semantics are the same; with every block result
    arriving at once, the first invalid block by index is reported."""
    if not coalesce:
        return await reject_first_invalid_resolve_all_valid([bls.verify_signature_sets(s) for s in blocks_sets])
    jobs = []
    owner = []
    for b, sets in enumerate(blocks_sets):
        check_sets(sets)
        for chunk in chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB):
            jobs.append(chunk)
            owner.append(b)
    res = await asyncio.get_running_loop().run_in_executor(bls._exec, bls._run_device_batch, jobs, None)
    ok = [True] * len(blocks_sets)
    for b, r in zip(owner, res):
        if isinstance(r, Exception):
            raise r
        ok[b] = ok[b] and r
    for b, v in enumerate(ok):
        if not v:
            return {"allValid": False, "index": b}
    return {"allValid": True}


def _new_metrics() -> dict:
    """Counterparts of lodestar_bls_thread_pool_* (metrics/metrics/lodestar.ts:350-430)."""
    return {
        "aggregated_pubkeys_total": 0,
        "jobs_started": 0,
        "main_thread_time_s": 0.0,
        "main_thread_calls": 0,
        "sets_started": 0,
        "batch_retries": 0,
        "batch_sigs_success": 0,
        "device_time_s": 0.0,
        "job_wait_time_s": [],
    }
