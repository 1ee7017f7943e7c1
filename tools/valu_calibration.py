"""VALU issue calibration run (profile with rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU):
librtamd's rt_debug_valu_calibration runs fma chains in fp32 and fp64 on every CU
(k_valu_peak, 16 waves per CU); tools/make_valu.py turns instructions / duration into the
VALU roof's peak."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import rtamd  # noqa: E402

L = rtamd.lib()
L.rt_debug_valu_calibration.restype = ctypes.c_int
L.rt_debug_valu_calibration.argtypes = [ctypes.c_int, ctypes.c_int]
rc = L.rt_debug_valu_calibration(0, int(sys.argv[1]) if len(sys.argv) > 1 else 2000)
print({"rc": rc})
sys.exit(0 if rc == 0 else 1)
