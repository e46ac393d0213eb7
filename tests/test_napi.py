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
if (a.abiVersion() !== 3) throw Error("abi " + a.abiVersion());
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
