"""FETCH_SIZE calibration run (profile with rocprofv3 --pmc FETCH_SIZE): librtamd's
rt_debug_fetch_calibration reads a 1 GiB buffer once per access width 1, 4, 8, 16 bytes
per lane (each read preceded by a 16-B streaming read of another 1 GiB buffer that
evicts the first from L2 and the Infinity Cache).  tools/make_traffic.py turns the
counter into bytes-per-counted-byte factors per width."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import rtamd  # noqa: E402

BYTES = 1 << 30
L = rtamd.lib(diag=True)
L.rt_debug_fetch_calibration.restype = ctypes.c_int
L.rt_debug_fetch_calibration.argtypes = [ctypes.c_int, ctypes.c_int64]
rc = L.rt_debug_fetch_calibration(0, BYTES)
print({"rc": rc, "bytes": BYTES, "widths": [1, 4, 8, 16]})
sys.exit(0 if rc == 0 else 1)
