"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/liboracle.so).

The oracle is a bit-exact C++ restatement of the reference render path (oracle.cpp);
it is pinned by tests/golden/ (hashes generated from the unmodified reference, see
tests/golden/make_golden.py).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("trace_rays", "shadow_rays", "reflect_rays", "refract_rays",
                                               "sphere_tests", "mesh_tests", "bbox_pass", "face_tests")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class OracleError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(msg)
        self.rc = rc


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so", "oracle_cli"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(Counters)]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_last_warnings.restype = ctypes.c_char_p
        L.oracle_to_rgb8.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        _lib = L
    return _lib


def render(files: Sequence[str], width: int, height: int, bdepth: int = 10, intersection_only: bool = False,
           threads: int = 8, rows: Tuple[int, ...] = None) -> Tuple[np.ndarray, dict]:
    """Renders rows r0, r0+step, ... < r1 (rows=(r0, r1[, step]), default all)
    -> (float64 (n_rows, W, 3), counters dict)."""
    L = lib()
    if isinstance(files, (str, os.PathLike)):
        files = [files]
    r0, r1, step = (tuple(rows) + (1,))[:3] if rows else (0, height, 1)
    out = np.empty((max(0, -(-(r1 - r0) // step)), width, 3), dtype=np.float64)
    arr = (ctypes.c_char_p * len(files))(*[os.fsencode(str(f)) for f in files])
    cnt = Counters()
    rc = L.oracle_render(arr, len(files), width, height, bdepth, int(intersection_only), threads, r0, r1, step,
                         out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cnt))
    if rc:
        raise OracleError(rc, L.oracle_last_error().decode())
    return out, cnt.as_dict()


def warnings() -> str:
    return lib().oracle_last_warnings().decode()


def to_rgb8(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.float64)
    out = np.empty(img.shape, dtype=np.uint8)
    lib().oracle_to_rgb8(img.ctypes.data_as(ctypes.c_void_p), img.size // 3, out.ctypes.data_as(ctypes.c_void_p))
    return out
