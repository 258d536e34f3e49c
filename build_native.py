"""Build every native extension of ray_memory_management_amd IN-TREE.

* ``_store``  — shared-memory object store (C++17, g++)
* ``_sched``  — scheduler core: resource sets, policies, dependency-gated queue (C++17, g++)
* ``_envs``   — native env cores (synthetic Atari vector env) for CPU rollout workers (C++17, g++)
* ``_hip``    — CDNA4 kernels + HBM GPU object store + native hybrid rollout loop (HIP, hipcc --offload-arch=gfx950)

Usage: ``python build_native.py [--force] [--only NAME]``. Rebuilds an extension only when a
source is newer than the built ``.so``. hipcc cross-compiles for gfx950 without a GPU.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ray_memory_management_amd")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RMM_OFFLOAD_ARCH", "gfx950")


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _torch_lib() -> str | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = os.path.join(os.path.dirname(spec.origin), "lib")
            if os.path.exists(os.path.join(d, "libamdhip64.so")):
                return d
    except Exception:
        pass
    return None


def _ext(name, sources, compiler, flags, ldflags, headers=()):
    return dict(name=name, sources=[os.path.join(ROOT, s) for s in sources], compiler=compiler,
                flags=flags, ldflags=ldflags, headers=[os.path.join(ROOT, h) for h in headers])


def extensions():
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall",
              "-Wno-unused-function", f"-I{py_inc}", f"-I{_pybind_include()}"]
    exts = [
        _ext("_store", ["csrc/store/shm_store.cc", "csrc/store/store_py.cc"], "g++",
             common + ["-march=x86-64-v2"], ["-lrt", "-lpthread"], ["csrc/store/shm_store.h"]),
        _ext("_sched", ["csrc/sched/scheduler.cc", "csrc/sched/sched_py.cc"], "g++",
             common, ["-lpthread"], ["csrc/sched/scheduler.h"]),
        _ext("_envs", ["csrc/rl/envs_py.cc"], "g++", common, [], ["csrc/rl/synth_env.h"]),
    ]
    tl = _torch_lib()
    hip_ld = ["-lpthread"]
    # Link against the HIP runtime torch ships with (same soname as /opt/rocm's) so one runtime
    # is loaded per process.
    if tl:
        hip_ld = [f"-L{tl}", f"-Wl,-rpath,{tl}", "-lamdhip64"] + hip_ld
    exts.append(
        _ext("_hip", ["csrc/hip/kernels.hip", "csrc/hip/rl_kernels.hip", "csrc/hip/conv_kernels.hip", "csrc/hip/dense_kernels.hip", "csrc/hip/x3_kernels.hip", "csrc/hip/shuffle_kernels.hip", "csrc/hip/ingest_kernels.hip", "csrc/hip/vtrace_kernels.hip", "csrc/hip/gpu_store.hip", "csrc/hip/peer_allreduce.hip", "csrc/hip/rollout_server.hip", "csrc/hip/rccl_comm.cc", "csrc/hip/rollout_loop.cc", "csrc/hip/hip_py.cc",
              "csrc/store/shm_store.cc"], HIPCC,
             common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-Wno-unused-result"]
             # RMM_X3_PROBE=1: the x3 kernels' phase timestamps (benchmarks/x3_phase_probe.py; build with --force)
             + (["-DRMM_X3_PROBE"] if os.environ.get("RMM_X3_PROBE") == "1" else []),
             hip_ld, ["csrc/hip/kernels.h", "csrc/hip/gpu_store.h", "csrc/hip/rccl_comm.h", "csrc/hip/peer_allreduce.h", "csrc/hip/common.h", "csrc/store/shm_store.h",
                     "csrc/hip/rollout_loop.h", "csrc/rl/synth_env.h", "csrc/hip/trunk_device.h",
                     "csrc/hip/dense_device.h", "csrc/hip/adam_device.h", "csrc/hip/x3_device.h"]))
    return exts


def _out(name):
    return os.path.join(PKG, name + EXT_SUFFIX)


def _stale(e) -> bool:
    out = _out(e["name"])
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in e["sources"] + e["headers"] if os.path.exists(s))


def _compile_obj(e, src, verbose):
    """Compile one source of a multi-source extension to build/obj (cached by mtime)."""
    od = os.path.join(ROOT, "build", "obj", e["name"])
    os.makedirs(od, exist_ok=True)
    obj = os.path.join(od, os.path.basename(src) + ".o")
    deps = [src] + e["headers"]
    if os.path.exists(obj) and all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in deps if os.path.exists(d)):
        return obj
    flags = [f for f in e["flags"] if f != "-shared"]
    cmd = [e["compiler"]] + flags + ["-c", src, "-o", obj + ".tmp"]
    if verbose:
        print("[build_native]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compiling {src} failed:\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def build_one(e, force=False, verbose=True):
    if not force and not _stale(e):
        return e["name"], "up-to-date"
    missing = [s for s in e["sources"] if not os.path.exists(s)]
    if missing:
        return e["name"], f"skipped (missing {missing})"
    out = _out(e["name"])
    tmp = out + ".tmp"
    if force:
        import shutil

        shutil.rmtree(os.path.join(ROOT, "build", "obj", e["name"]), ignore_errors=True)
    # per-source objects in parallel (hipcc is single-threaded per file), then one link
    with ThreadPoolExecutor(max_workers=min(8, len(e["sources"]))) as ex:
        objs = list(ex.map(lambda s: _compile_obj(e, s, verbose), e["sources"]))
    link = [f for f in e["flags"] if f.startswith("--offload-arch") or f in ("-shared", "-fPIC")]
    cmd = [e["compiler"]] + link + objs + ["-o", tmp] + e["ldflags"]
    if verbose:
        print("[build_native]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"linking {e['name']} failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    return e["name"], "built"


def build(force=False, only=None, verbose=True):
    exts = [e for e in extensions() if only is None or e["name"] in only]
    with ThreadPoolExecutor(max_workers=3) as ex:
        results = list(ex.map(lambda e: build_one(e, force, verbose), exts))
    for n, s in results:
        if verbose:
            print(f"[build_native] {n}: {s}", flush=True)
    return results


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    try:
        build(a.force, a.only)
    except RuntimeError as err:
        print(err, file=sys.stderr)
        sys.exit(1)
