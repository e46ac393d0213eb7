"""Build the gfx950 shared library lodestar_amd/libbgv.so in-tree.

hipcc compiles the kernels and the C-ABI host code (both .hip translation
units) for gfx950 only.  The SHA-256 of the sources (lodestar_amd.native
source_hash) is compiled in as bgv_build_id(); the library is rebuilt when
its id is not the tree's, and the bindings refuse to load it in that case,
so a library built from other sources never runs.  Used by
__graft_entry__.build() and the test suite."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
from lodestar_amd.native import source_hash  # noqa: E402
CSRC = os.path.join(ROOT, "lodestar_amd", "csrc")
LIB = os.path.join(ROOT, "lodestar_amd", "libbgv.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["bgv_kernels.hip", "bgv_miller.hip", "bgv_latency.hip", "bgv_tail.hip", "bgv_gather.hip", "bgv_api.hip"]


def deps():
    return (glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip"))
            + [os.path.join(ROOT, "include", "bgv.h"), os.path.abspath(__file__)])


def build_id(defines=()):
    h = source_hash(ROOT)
    return h + ("+" + ",".join(defines) if defines else "")


def stale(lib=LIB, defines=()):
    """True unless the library carries the id of the current sources"""
    if not os.path.exists(lib):
        return True
    with open(lib, "rb") as f:
        return (build_id(defines).encode() + b"\0") not in f.read()


def build(force=False, verbose=False, lib=LIB, defines=()):
    if not force and not stale(lib, defines):
        return lib
    bid = build_id(defines)
    objs = []
    procs = []
    for s in SOURCES:
        o = os.path.join(CSRC, os.path.basename(lib) + "." + s.replace(".hip", ".o"))
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
               "-I" + os.path.join(ROOT, "include")] + ["-D" + x for x in defines] + [f'-DBGV_SRC_HASH="{bid}"', "-c", os.path.join(CSRC, s), "-o", o]
        if defines and os.environ.get("BGV_VARIANT_FLAGS"):  # variant builds only (A/B experiments)
            cmd[1:1] = os.environ["BGV_VARIANT_FLAGS"].split()
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
        objs.append(o)
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    tmp = lib + ".tmp"
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


NAPI_DIR = os.path.join(ROOT, "lodestar_amd", "napi")
ADDON = os.path.join(NAPI_DIR, "bgv.node")
NODE_INCLUDE = [d for d in ("/usr/include/node", "/usr/include/nodejs/src") if os.path.exists(os.path.join(d, "node_api.h"))]


def build_addon(force=False):
    """N-API addon lodestar_amd/napi/bgv.node over libbgv.so (INTEGRATION.md
    section 3).  gcc against the system node_api.h; rpath points at the
    library one directory up.  Returns None when no Node headers exist."""
    if not NODE_INCLUDE:
        return None
    build()
    src = os.path.join(NAPI_DIR, "bgv_addon.c")
    if (not force and os.path.exists(ADDON) and os.path.getmtime(ADDON) >= os.path.getmtime(src)
            and os.path.getmtime(ADDON) >= os.path.getmtime(os.path.join(ROOT, "include", "bgv.h"))):
        return ADDON
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-DNODE_GYP_MODULE_NAME=bgv",
                           "-I" + NODE_INCLUDE[0], "-I" + os.path.join(ROOT, "include"), src, "-o", ADDON,
                           "-L" + os.path.dirname(LIB), "-lbgv", "-lpthread", "-Wl,-rpath,$ORIGIN/.."])
    return ADDON


if __name__ == "__main__":
    if "--variant" in sys.argv:  # --variant NAME DEF [DEF ...]
        k = sys.argv.index("--variant")
        name, defs = sys.argv[k + 1], sys.argv[k + 2:]
        print(build(force=True, lib=LIB.replace(".so", f"_{name}.so"), defines=defs))
    elif "--variants" in sys.argv:  # occupancy experiment builds
        for w in (1, 2, 4):
            print(build(force=True, lib=LIB.replace(".so", f"_w{w}.so"), defines=[f"BGV_WAVES={w}"]))
    else:
        build(force="--force" in sys.argv, verbose=True)
        print(LIB)
        print(build_addon(force="--force" in sys.argv))
