"""ctypes binding of libbm25mi.so (include/bm25mi.h).

This is the Python side of the drop-in boundary: the reference's MAX custom-op
ABI (operations/graph_operation.mojo:27-45, graph.py:55-73) is replaced by a
plain C-ABI called through ctypes (ctypes releases the GIL during calls).
There is no fallback: if the HIP library is missing, importing this module
raises ImportError.
"""
from __future__ import annotations

import ctypes
import os
import re

from .build import LIB

BM25_OK, BM25_EINVAL, BM25_EHIP, BM25_ENOMEM = 0, 1, 2, 4  # 3: unused (no RCCL inside the library)
HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                      "include", "bm25mi.h")

if not os.path.exists(LIB):
    raise ImportError(
        f"libbm25mi.so not found at {LIB}: run __graft_entry__.build() "
        "(python mojo-bm25_amd/bm25mi/build.py) — there is no CPU fallback")

# One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64
# (SONAME libamdhip64.so.7, loaded through its RPATH under a different NEEDED
# name), so if libbm25mi.so bound /opt/rocm's copy first, torch would later load
# a second runtime that sees no GPU.  Importing torch first makes the dynamic
# linker satisfy libbm25mi's NEEDED libamdhip64.so.7 with the copy already
# mapped, so device pointers and streams are shared with torch.
try:  # pragma: no cover - depends on the environment
    import torch  # noqa: F401
except ImportError:
    pass

lib = ctypes.CDLL(LIB)

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PD = ctypes.POINTER(ctypes.c_double)

_SIGS = {
    "bm25_abi_version": ([], ctypes.c_int),
    "bm25_last_error": ([], ctypes.c_char_p),
    "bm25_device_count": ([], ctypes.c_int),
    "bm25_index_create": ([ctypes.c_int, _I64, _I64, _I64, _P, ctypes.c_int, _P, _P, _I64,
                           ctypes.POINTER(_P)], ctypes.c_int),
    "bm25_index_destroy": ([_P], ctypes.c_int),
    "bm25_index_fork": ([_P, ctypes.POINTER(_P)], ctypes.c_int),
    "bm25_index_info": ([_P, _PI64, _PI64, _PI64, _PI32, _PI64, _PI64], ctypes.c_int),
    "bm25_index_segments": ([_P, _PI32, _PI64], ctypes.c_int),
    "bm25_index_bounds": ([_P, _PI32, _PI64], ctypes.c_int),
    "bm25_search": ([_P, _P, _I64, _I64, _I32, _P, _P], ctypes.c_int),
    "bm25_search_device": ([_P, _P, _I64, _I64, _I32, _P, _P, _P], ctypes.c_int),
    "bm25_max_token_device": ([_P, _P, _I64, _I64, _P, _P], ctypes.c_int),
    "bm25_scores_dense": ([_P, _P, _I64, _P], ctypes.c_int),
    "bm25_index_set_values_f64": ([_P, _P], ctypes.c_int),
    "bm25_scores_dense_f64": ([_P, _P, _I64, _P], ctypes.c_int),
    "bm25_topn_f64": ([_P, _P, _I64, _I64, _P, _P], ctypes.c_int),
    "bm25_merge_topk_device": ([ctypes.c_int, _P, _P, _I64, _I64, _I32, _P, _P, _P],
                               ctypes.c_int),
    "bm25_merge_sorted_device": ([ctypes.c_int, _P, _P, _I64, _I64, _I32, _I64, _P, _P, _P],
                                 ctypes.c_int),
    "bm25_profile_enable": ([_P, ctypes.c_int], ctypes.c_int),
    "bm25_profile_read": ([_P, _PD, _PI64, _PD, _PI64, _PI64], ctypes.c_int),
    "bm25_search_stats": ([_P, _PI64, _PI64], ctypes.c_int),
    "bm25_search_stats_ex": ([_P, _PI64, _PI64, _PI64], ctypes.c_int),
    "bm25_search_counters": ([_P, _PI64, _I32], ctypes.c_int),
    "bm25_index_set_option": ([_P, ctypes.c_char_p, _I64], ctypes.c_int),
    "bm25_index_get_option": ([_P, ctypes.c_char_p, _PI64], ctypes.c_int),
    "bm25_search_dispatch": ([_P, ctypes.POINTER(ctypes.c_uint32), _PI32, _PI32, _PI32],
                             ctypes.c_int),
    "bm25_sharded_create": ([ctypes.c_int, _P, _I64, _I64, _I64, _P, ctypes.c_int, _P, _P,
                             ctypes.POINTER(_P)], ctypes.c_int),
    "bm25_sharded_search": ([_P, _P, _I64, _I64, _I32, _P, _P], ctypes.c_int),
    "bm25_sharded_info": ([_P, _PI64, _P, _P], ctypes.c_int),
    "bm25_sharded_destroy": ([_P], ctypes.c_int),
    "bm25_sample_width": ([_P, _I64, _I32, _I32, _PI64], ctypes.c_int),
    "bm25_search_sample_device": ([_P, _P, _I64, _I64, _I32, _I32, _I64, _P, _P], ctypes.c_int),
    "bm25_search_finish_streams_device": ([_P, _P, _I64, _I64, _I32, _I32, _I64, _P, _P, _P, _P,
                                           _P, _P], ctypes.c_int),
    "bm25_search_finish_device": ([_P, _P, _I64, _I64, _I32, _I32, _I64, _P, _P, _P, _P],
                                  ctypes.c_int),
    "bm25_index_bounds_export": ([_P, _P, _I64, _P], ctypes.c_int),
    "bm25_index_set_world_bounds": ([_P, _P, _I32, _I64, _I64], ctypes.c_int),
    "bm25_search_shard_device": ([_P, _P, _I64, _I64, _I32, _P, _P, _P], ctypes.c_int),
    "bm25_build_scores": ([ctypes.c_int, _I64, _I64, _I64, _P, _P, _P, _P, ctypes.c_double,
                           ctypes.c_double, ctypes.c_double, ctypes.c_int, _P, _P, _P, _P, _P],
                          ctypes.c_int),
}
for _name, (_args, _res) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.argtypes = _args
    _f.restype = _res


class HipError(RuntimeError):
    """A HIP runtime failure inside libbm25mi (BM25_EHIP)."""


def check(rc: int) -> None:
    if rc == BM25_OK:
        return
    msg = (lib.bm25_last_error() or b"").decode(errors="replace")
    if rc == BM25_EINVAL:
        raise ValueError(msg)
    if rc == BM25_ENOMEM:
        raise MemoryError(msg)
    if rc == BM25_EHIP:
        raise HipError(msg)
    raise RuntimeError(f"libbm25mi error {rc}: {msg}")


def header_symbols(path: str = HEADER):
    """Function names declared in include/bm25mi.h."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bm25_[a-z0-9_]+)\s*\(", text)))


def abi_version() -> int:
    return lib.bm25_abi_version()


def device_count() -> int:
    return lib.bm25_device_count()
