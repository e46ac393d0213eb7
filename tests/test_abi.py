"""The C-ABI library: builds for gfx950, loads without a GPU, exports every
symbol include/bgv.h declares, and its struct layout matches the ctypes
mirror.  No compute calls here (no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bgv.h")


@pytest.fixture(scope="module")
def lib():
    from tools import build
    build.build()
    from lodestar_amd import native
    return native.load_library()


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(bgv_\w+)\s*\(", src, re.M)))


def test_every_declared_symbol_is_exported(lib):
    names = declared_functions()
    assert len(names) >= 16
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(ROOT, "lodestar_amd", "libbgv.so")]).decode()
    exported = set(re.findall(r" T (bgv_\w+)", out))
    assert set(names) <= exported, set(names) - exported
    from lodestar_amd import native
    assert set(native.EXPORTS) == set(names)


def test_struct_layout_matches_ctypes(tmp_path):
    from lodestar_amd import native
    c = tmp_path / "layout.c"
    fields_b = [f for f, _ in native.BgvBatch._fields_]
    fields_s = [f for f, _ in native.BgvStats._fields_]
    fields_d = [f for f, _ in native.BgvDebug._fields_]
    fields_c = [f for f, _ in native.BgvCfg._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "bgv.h"', "int main(void){"]
    lines.append('printf("%zu %zu %zu %zu\\n", sizeof(bgv_batch), sizeof(bgv_stats), sizeof(bgv_debug), sizeof(bgv_cfg));')
    for f in fields_b:
        lines.append(f'printf("%zu\\n", offsetof(bgv_batch, {f}));')
    for f in fields_s:
        lines.append(f'printf("%zu\\n", offsetof(bgv_stats, {f}));')
    for f in fields_d:
        lines.append(f'printf("%zu\\n", offsetof(bgv_debug, {f}));')
    for f in fields_c:
        lines.append(f'printf("%zu\\n", offsetof(bgv_cfg, {f}));')
    lines.append("return 0;}")
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)])
    vals = subprocess.check_output([str(exe)]).decode().split()
    assert int(vals[0]) == ctypes.sizeof(native.BgvBatch)
    assert int(vals[1]) == ctypes.sizeof(native.BgvStats)
    assert int(vals[2]) == ctypes.sizeof(native.BgvDebug)
    assert int(vals[3]) == ctypes.sizeof(native.BgvCfg)
    offs = [int(v) for v in vals[4:]]
    nb, ns, nd = len(fields_b), len(fields_s), len(fields_d)
    assert offs[:nb] == [getattr(native.BgvBatch, f).offset for f in fields_b]
    assert offs[nb:nb + ns] == [getattr(native.BgvStats, f).offset for f in fields_s]
    assert offs[nb + ns:nb + ns + nd] == [getattr(native.BgvDebug, f).offset for f in fields_d]
    assert offs[nb + ns + nd:] == [getattr(native.BgvCfg, f).offset for f in fields_c]


def test_metadata_and_no_silent_fallback(lib):
    from lodestar_amd import native
    assert lib.bgv_abi_version() == native.ABI_VERSION == 4
    assert lib.bgv_set_code_name(8) == b"BLST_INVALID_SIZE"
    assert lib.bgv_set_code_name(3) == b"BLST_POINT_NOT_IN_GROUP"
    assert lib.bgv_stage_name(6) == b"miller_loop"
    assert lib.bgv_stage_name(2) == b"pk_gather"
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        # the product path fails loudly without a HIP device: no CPU fallback
        with pytest.raises(native.BgvNativeError):
            native.Device(0)


def test_gfx950_code_object_present(lib):
    blob = open(os.path.join(ROOT, "lodestar_amd", "libbgv.so"), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the fat binary carries a gfx950 code object


def test_no_environment_steers_the_pipeline(lib):
    """The pipeline variant is chosen per batch (prepare()) or forced by an
    explicit bgv_cfg; the library reads no environment variable."""
    out = subprocess.check_output(["nm", "-D", "--undefined-only", os.path.join(ROOT, "lodestar_amd", "libbgv.so")]).decode()
    assert "getenv" not in out
    src = "".join(open(os.path.join(ROOT, "lodestar_amd", "csrc", f)).read()
                  for f in os.listdir(os.path.join(ROOT, "lodestar_amd", "csrc")))
    assert "getenv" not in src


def test_cfg_defaults_and_validation(lib):
    from lodestar_amd import native
    c = native.BgvCfg()
    lib.bgv_cfg_default(ctypes.byref(c))
    assert c.struct_size == ctypes.sizeof(native.BgvCfg)
    assert {k: getattr(c, k) for k in native.BgvCfg.AUTO} == native.BgvCfg.AUTO
    h = ctypes.c_void_p()
    # invalid overrides are refused before any device call (no GPU needed)
    for bad in ({"miller": 7}, {"job_lanes": 5}, {"pairs": 3}, {"defer_pct": 101}, {"split": 2}, {"prefold": -2},
                {"lines": 2}, {"timing": 5}, {"miller": 4, "pairs": 2}, {"miller": 36, "pairs": 2},
                {"cu_split": 65}, {"cu_split": -65}, {"clear_lanes": 2}, {"miller_kv": 4}):
        st = lib.bgv_open_cfg(0, ctypes.byref(native.BgvCfg.make(**bad)), ctypes.byref(h))
        assert st == native.BGV_E_INVALID_ARG, bad
    c2 = native.BgvCfg.make()
    c2.struct_size = 4
    assert lib.bgv_open_cfg(0, ctypes.byref(c2), ctypes.byref(h)) == native.BGV_E_INVALID_ARG
    with pytest.raises(ValueError):
        native.BgvCfg.make(overlap=0)


def test_library_id_matches_the_sources(lib):
    """tools/build.py compiles the SHA-256 of csrc/ + include/bgv.h into the
    library; load_library refuses a library built from other sources."""
    from lodestar_amd import native
    assert lib.bgv_build_id().decode() == native.source_hash()


def test_stale_library_refuses_to_load(lib, tmp_path):
    import shutil

    from lodestar_amd import native
    lib_id = lib.bgv_build_id().decode()
    # a tree whose sources differ from the ones the library was built from
    for rel in native.source_files():
        dst = tmp_path / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(ROOT, rel), dst)
    native.check_build_id(lib_id, root=str(tmp_path))  # same sources: accepted
    fp = tmp_path / "lodestar_amd" / "csrc" / "fp.h"
    fp.write_text(fp.read_text() + "\n// edited\n")
    with pytest.raises(native.BgvNativeError, match="other sources"):
        native.check_build_id(lib_id, root=str(tmp_path))
    # and in a fresh interpreter the stale tree's library does not load at all
    shutil.copytree(os.path.join(ROOT, "lodestar_amd"), tmp_path / "pkg" / "lodestar_amd",
                    ignore=shutil.ignore_patterns("__pycache__", "napi"))
    (tmp_path / "pkg" / "include").mkdir()
    shutil.copy(HEADER, tmp_path / "pkg" / "include" / "bgv.h")
    hdr = tmp_path / "pkg" / "lodestar_amd" / "csrc" / "fp.h"
    hdr.write_text(hdr.read_text() + "\n// edited\n")
    code = ("import sys; sys.path.insert(0, %r)\nfrom lodestar_amd import native\n"
            "try:\n    native.load_library()\nexcept native.BgvNativeError as e:\n    print('refused', e)\n") % str(tmp_path / "pkg")
    env = dict(os.environ)
    env.pop("BGV_LIB", None)
    out = subprocess.check_output([__import__("sys").executable, "-c", code], env=env).decode()
    assert out.startswith("refused") and "other sources" in out


def test_device_inputs_wait_for_their_producing_stream(monkeypatch):
    """native._sync_producers: one current-stream synchronize per CUDA device a
    tensor argument lives on; numpy arrays, None and scalars need none"""
    import types

    import numpy as np
    import torch

    from lodestar_amd import native
    calls = []

    class _Stream:
        def __init__(self, dev):
            self.dev = dev

        def synchronize(self):
            calls.append(self.dev)

    monkeypatch.setattr(torch.cuda, "current_stream", lambda dev=None: _Stream(dev))
    d0 = types.SimpleNamespace(type="cuda", index=0)
    d1 = types.SimpleNamespace(type="cuda", index=1)
    cpu = types.SimpleNamespace(type="cpu", index=None)
    t = lambda dev: types.SimpleNamespace(device=dev, data_ptr=lambda: 0)
    native._sync_producers({"a": np.zeros(3), "b": None, "n": 5, "c": t(d0), "d": t(d0), "e": t(d1), "f": t(cpu)})
    assert calls == [d0, d1]
    calls.clear()
    native._sync_producers({"a": np.zeros(3)}, None)
    assert calls == []
    native._sync_producers(t(d1))
    assert calls == [d1]
