"""Loader for the in-tree native libraries (built by ``__graft_entry__.build()``).

The HIP libraries are loaded with ``ctypes``.  When PyTorch is imported in the same process the
HIP runtime is shared (``libamdhip64.so.7`` is one soname), so streams created here can be handed
to ``torch.cuda.ExternalStream`` and vice versa.

On a machine with a GPU a missing library is an error (``require``), never a silent fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict

NATIVE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")

_lock = threading.Lock()
_libs: Dict[str, ctypes.CDLL] = {}


class NativeUnavailable(RuntimeError):
    pass


def lib_path(name: str) -> str:
    # NOS_NATIVE_DIR: an alternative build of the same libraries (A/B timing runs only; such a build
    # is not stamp-verified, so it also needs NOS_ALLOW_STALE_NATIVE=1)
    return os.path.join(os.environ.get("NOS_NATIVE_DIR") or NATIVE_DIR, name)


def available(name: str) -> bool:
    return os.path.exists(lib_path(name))


def load(name: str) -> ctypes.CDLL:
    with _lock:
        if name in _libs:
            return _libs[name]
        p = lib_path(name)
        if not os.path.exists(p):
            raise NativeUnavailable(f"native library {name} is not built ({p}); run `python -c "
                                    f"'import __graft_entry__ as g; g.build()'` from the repo root")
        if os.environ.get("NOS_ALLOW_STALE_NATIVE") != "1":
            from .build import verify
            try:
                verify(name)  # the library must be the build of the sources next to it
            except (RuntimeError, StopIteration) as e:
                raise NativeUnavailable(str(e)) from None
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        _libs[name] = lib
        return lib


def gpu_present() -> bool:
    """True when a GPU is visible, without initialising HIP in this process."""
    if os.environ.get("HIP_VISIBLE_DEVICES") == "" or os.environ.get("CUDA_VISIBLE_DEVICES") == "":
        return False
    return os.path.exists("/dev/kfd") and any(n.startswith("renderD") for n in os.listdir("/dev/dri")) \
        if os.path.isdir("/dev/dri") else False
