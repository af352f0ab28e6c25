"""bm25mi — MI355X-native BM25 CSC query engine (host side).

The product path is libbm25mi.so (HIP kernels for gfx950 + C-ABI), reached
through ``bm25mi._capi``.  Importing :class:`GpuIndex` requires the built
library; there is no CPU fallback.

Drop-in modules of the reference API live next to this package
(``mojo-bm25_amd/bm25_native.py``, ``bm25.py``, ``gpu_bm25/common.py``).
"""
from .build import LIB, SYNTH_LIB, build  # noqa: F401


def __getattr__(name):
    if name in ("GpuIndex", "merge_topk_device", "device_count"):
        from . import index
        return getattr(index, name)
    raise AttributeError(name)
