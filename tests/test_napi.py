"""The N-API addon (lodestar_amd/napi/bgv.node over libbgv.so) driven from
Node: the binding a Lodestar maintainer adds.

CPU: the addon builds, loads in Node, exports every entry point, maps the
BLST code names and rejects `open` cleanly without a GPU.
GPU: tests/js/addon_golden_test.js verifies the golden batch through
addon.verify (libuv pool) and addon.verifySync, and drives the IBlsVerifier
wrapper with the reference e2e semantics."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _addon():
    from tools import build as B

    path = B.build_addon()
    if path is None:
        pytest.skip("node_api.h not found")
    return path


def test_addon_loads_and_exports():
    addon = _addon()
    script = f"""
const a = require({addon!r});
const want = ["abiVersion","codeName","open","close","pubkeysSet","pubkeysCount","pubkeysValidate","verify","verifySync"];
for (const k of want) if (typeof a[k] !== "function") throw Error("missing " + k);
if (a.abiVersion() !== 4) throw Error("abi " + a.abiVersion());
if (a.codeName(8) !== "BLST_INVALID_SIZE" || a.codeName(3) !== "BLST_POINT_NOT_IN_GROUP") throw Error("names");
// without a GPU open() throws a bgv error; with one it yields a working context
let ctx = null;
try {{ ctx = a.open(0); }} catch (e) {{ if (!/bgv error -3/.test(e.message)) throw e; }}
if (ctx !== null) {{ if (a.pubkeysCount(ctx) !== 0) throw Error("fresh table"); a.close(ctx); }}
console.log("ok");
"""
    r = subprocess.run([NODE, "-e", script], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "ok"


@pytest.mark.gpu
def test_addon_golden_batch_and_verifier():
    _addon()
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "addon_golden_test.js")],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "addon golden test OK" in r.stdout


@pytest.mark.gpu
def test_verify_on_main_thread_priority_path(tmp_path):
    """verifyOnMainThread with a 100,352-set bulk batch in flight: resolves
    first, the event loop never stalls >= 2 ms, verdicts right
    (tests/js/priority_test.js; multithread/index.ts:155-167)"""
    import json

    import numpy as np

    from lodestar_amd import native
    _addon()
    n, k, table_n = 100_353, 4, 4096
    d = native.Device(0)
    try:
        d.gen_keys(0, table_n, 0x5EED)
        rng = np.random.default_rng(5)
        arrays = {"n_sets": n, "n_jobs": n, "job_offsets": np.arange(n + 1, dtype=np.uint32),
                  "pk_offsets": (np.arange(n + 1) * k).astype(np.uint32),
                  "pk_indices": rng.integers(0, table_n, size=n * k).astype(np.uint32),
                  "msgs": rng.integers(0, 256, size=(n, 32), dtype=np.uint8)}
        sigs = np.zeros((n, 192), np.uint8)
        d.gen_sign(arrays, sigs)
        table = d.pubkeys_get(0, table_n)
    finally:
        d.close()
    (tmp_path / "table96.bin").write_bytes(table)
    (tmp_path / "msgs.bin").write_bytes(arrays["msgs"].tobytes())
    (tmp_path / "sigs.bin").write_bytes(np.ascontiguousarray(sigs[:, :96]).tobytes())
    (tmp_path / "pk_offsets.bin").write_bytes(arrays["pk_offsets"].tobytes())
    (tmp_path / "pk_indices.bin").write_bytes(arrays["pk_indices"].tobytes())
    (tmp_path / "meta.json").write_text(json.dumps({"n_sets": n}))
    r = subprocess.run([NODE, "--max-old-space-size=4096", "--expose-gc", os.path.join(ROOT, "tests", "js", "priority_test.js"), str(tmp_path)],
                       capture_output=True, text=True, timeout=150, env={**os.environ, "UV_THREADPOOL_SIZE": "8"})
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "priority test OK" in r.stdout
