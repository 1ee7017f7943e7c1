"""VALU issue calibration run (profile with rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU):
librtamd's rt_debug_valu_calibration runs fma chains in fp32 and fp64 on every CU
(k_valu_peak, 16 waves per CU); tools/make_valu.py turns instructions / duration into the
VALU roof's peak.

--mix: every instruction kind of k_valu_peak (trace.hip kValuKinds) at 1, 2, 4 and 8 waves
per SIMD, timed with HIP events (rt_debug_valu_rate, no profiler): one JSON line per run with
the wave-instruction rate and the SIMD cycles per wave64 instruction at 2.4 GHz."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import rtamd  # noqa: E402

KINDS = ["v_fma_f32", "v_pk_fma_f32", "v_fma_f64", "v_add_f64", "v_mul_f64", "v_max_f64", "v_cmp_gt_f64",
         "v_cndmask_b32", "v_add_u32", "v_mov_b32", "v_cmp_gt_f32", "v_mov_b64", "v_rcp_f64",
         "v_cndmask_b32_e64 (SGPR mask)", "v_cndmask_b32 (VCC set)", "v_cndmask_b32_e64 (2 VGPRs)",
         "v_cmp_gt_f64_e64 (SGPR dst)", "v_cndmask_b32_e32 (2 VGPRs, VCC)", "v_cndmask_b32_e64 (2 VGPRs, VCC)",
         "v_div_fmas_f64", "v_div_scale_f64", "v_div_fixup_f64", "v_addc_co_u32_e32", "v_readlane_b32", "v_writelane_b32",
         "v_sqrt_f64"]
SIMDS, CLOCK_GHZ = 1024, 2.4

L = rtamd.lib(diag=True)
args = [a for a in sys.argv[1:] if not a.startswith("--")]
iters = int(args[0]) if args else 2000
if "--mix" in sys.argv:
    L.rt_debug_valu_rate.restype = ctypes.c_int
    L.rt_debug_valu_rate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double)]
    only = {int(k) for a in sys.argv if a.startswith("--kinds=") for k in a.split("=")[1].split(",")}
    for kind, name in enumerate(KINDS):
        if only and kind not in only:
            continue
        for waves in (1, 2, 4, 8):
            it = max(1, iters * 8 // waves)
            ms = ctypes.c_double()
            rc = L.rt_debug_valu_rate(0, kind, waves, it, ctypes.byref(ms))
            if rc != 0:
                print(json.dumps({"kind": name, "waves": waves, "rc": rc}))
                sys.exit(1)
            instr = 256 * waves * 4 * it * 128
            rate = instr / (ms.value * 1e-3)
            print(json.dumps({"kind": name, "waves_per_simd": waves, "ms": round(ms.value, 4),
                              "wave_instr_per_s": round(rate), "simd_cycles_per_instr":
                              round(SIMDS * CLOCK_GHZ * 1e9 / rate, 3)}), flush=True)
    sys.exit(0)
L.rt_debug_valu_calibration.restype = ctypes.c_int
L.rt_debug_valu_calibration.argtypes = [ctypes.c_int, ctypes.c_int]
rc = L.rt_debug_valu_calibration(0, iters)
print({"rc": rc})
sys.exit(0 if rc == 0 else 1)
