"""Loader for the in-tree native extensions (built by ``build_native.py``).

``_store`` and ``_sched`` are required everywhere. ``_hip`` is imported lazily (after torch, so
the process uses ONE HIP runtime) and is REQUIRED whenever a GPU is visible: on a GPU box a
missing/broken ``_hip`` raises rather than silently falling back to eager PyTorch.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_hip = None
_hip_err = None
_tried = False


def _maybe_build(name: str) -> None:
    if os.environ.get("RMM_NO_AUTOBUILD"):
        return
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = os.path.join(root, "build_native.py")
    if os.path.exists(script):
        import subprocess
        import sys

        subprocess.run([sys.executable, script, "--only", name], check=False, capture_output=True)


def load(name: str):
    try:
        return importlib.import_module(f"ray_memory_management_amd.{name}")
    except ImportError:
        _maybe_build(name)
        return importlib.import_module(f"ray_memory_management_amd.{name}")


def store_ext():
    return load("_store")


def sched_ext():
    return load("_sched")


def hip_ext():
    """The HIP extension module, or None if it cannot be loaded (CPU-only hosts)."""
    global _hip, _hip_err, _tried
    if _tried:
        return _hip
    with _lock:
        if _tried:
            return _hip
        try:
            import torch  # noqa: F401  (load torch's HIP runtime first)

            _hip = load("_hip")
        except Exception as e:  # pragma: no cover - depends on host
            _hip_err = e
            _hip = None
        _tried = True
    return _hip


def gpu_visible() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def require_hip():
    h = hip_ext()
    if h is None:
        raise RuntimeError(
            f"ray_memory_management_amd: the native HIP extension (_hip) is required for GPU ops but failed "
            f"to load: {_hip_err!r}. Run `python build_native.py`.")
    return h
