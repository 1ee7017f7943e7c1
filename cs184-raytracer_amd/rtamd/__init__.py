"""rtamd — Python mirror of the reference's render interface over the C-ABI.

The reference (gh2o/CS184-Raytracer) is a C++ program; its render path is driven by

    Scene scene;                                   // scene.h:9-39
    RTIParser(scene).parseFile(filename);          // parsers.cpp:93
    scene.renderScene(image, progressHandler);     // scene.cpp:10-59
    PNGWriter(filename).writeImage(image);         // writers.cpp:11-21

with flags in the global ``programOptions`` (options.h:10-16).  This module exposes the
same names over ``librtamd.so`` (include/rtamd.h), whose render runs as HIP kernels on
an MI355X.  There is no CPU fallback: rendering without a HIP device raises
``DeviceError`` (the CPU restatement under ``oracle/`` is test infrastructure only).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RTAMD_LIB: an alternative build of the same library (e.g. the phase-profile build, make prof)
LIB_PATH = os.environ.get("RTAMD_LIB") or os.path.join(_HERE, "librtamd.so")
# the same library with the test and measurement hooks (csrc/diag.cpp: rt_debug_*, not in
# rtamd.h): only tests that inject failures and the profiling tools load it
DIAG_LIB_PATH = os.path.join(_HERE, "librtamd_diag.so")

RT_OK, RT_ERR_PARSE, RT_ERR_MATH, RT_ERR_ARG, RT_ERR_DEVICE, RT_ERR_IO = 0, -1, -2, -3, -4, -5


class RTError(RuntimeError):
    """Base class of rtamd errors."""


class ParseException(RTError):
    """ParseException (exceptions.h:6-21)."""


class MathException(RTError):
    """MathException (exceptions.h:23-26): what() text of the reference."""


class WriteException(RTError):
    """WriteException (exceptions.h:28-31)."""


class DeviceError(RTError):
    """HIP runtime failure or no HIP device."""


class ArgumentError(RTError, ValueError):
    pass


class rt_render_params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("bounce_depth", ctypes.c_int32),
                ("intersection_only", ctypes.c_int32), ("row_begin", ctypes.c_int32), ("row_end", ctypes.c_int32),
                ("row_step", ctypes.c_int32), ("chunk_pixels", ctypes.c_int32), ("row_block", ctypes.c_int32),
                ("work_stats", ctypes.c_int32)]


class rt_counters(ctypes.Structure):
    _fields_ = [("trace_rays", ctypes.c_int64), ("shadow_rays", ctypes.c_int64), ("reflect_rays", ctypes.c_int64),
                ("refract_rays", ctypes.c_int64), ("pixels", ctypes.c_int64), ("intersection_max", ctypes.c_double),
                ("kernel_ms", ctypes.c_double), ("levels", ctypes.c_int32), ("trace_launches", ctypes.c_int32),
                ("node_visits", ctypes.c_int64), ("tri_tests", ctypes.c_int64), ("candidates", ctypes.c_int64),
                ("sphere_tests", ctypes.c_int64), ("stage_ms", ctypes.c_double * 3),
                ("stage_launches", ctypes.c_int32 * 3), ("stage_node_visits", ctypes.c_int64 * 2),
                ("stage_tri_tests", ctypes.c_int64 * 2), ("stage_candidates", ctypes.c_int64 * 2),
                ("stage_sphere_tests", ctypes.c_int64 * 2), ("stage_bvh_traversals", ctypes.c_int64 * 2),
                ("stage_max_node_visits", ctypes.c_int64 * 2), ("shadow_rays_zero_terms", ctypes.c_int64),
                ("host_ms", ctypes.c_double), ("copy_ms", ctypes.c_double)]


class rt_scene_info(ctypes.Structure):
    _fields_ = [("n_geometries", ctypes.c_int32), ("n_spheres", ctypes.c_int32), ("n_meshes", ctypes.c_int32),
                ("n_lights", ctypes.c_int32), ("n_faces", ctypes.c_int64), ("n_bvh_nodes", ctypes.c_int64),
                ("device_bytes", ctypes.c_int64), ("max_bvh_depth", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("level_bytes", ctypes.c_int64), ("build_ms", ctypes.c_double), ("upload_ms", ctypes.c_double),
                ("level_bytes_peak", ctypes.c_int64), ("level_budget", ctypes.c_int64)]


class rt_xform_desc(ctypes.Structure):
    """Transformable (rtbase.h:41-64): Eigen Transform4d storage, column-major."""
    _fields_ = [("fwd", ctypes.c_double * 16), ("inv", ctypes.c_double * 16), ("det", ctypes.c_double),
                ("derive", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class rt_material_desc(ctypes.Structure):
    """Material (rtbase.h:30-39)."""
    _fields_ = [("ambient", ctypes.c_double * 3), ("diffuse", ctypes.c_double * 3), ("specular", ctypes.c_double * 3),
                ("reflective", ctypes.c_double * 3), ("specular_coefficient", ctypes.c_double),
                ("translucency", ctypes.c_double * 3), ("index_of_refractivity", ctypes.c_double)]


class rt_face_desc(ctypes.Structure):
    """Mesh::Face (geometry.h:32)."""
    _fields_ = [("points", (ctypes.c_double * 4) * 3), ("normals", (ctypes.c_double * 4) * 3)]


class rt_geometry_desc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("reserved", ctypes.c_int32), ("xf", rt_xform_desc),
                ("material", rt_material_desc), ("center", ctypes.c_double * 4), ("radius", ctypes.c_float),
                ("reserved_f", ctypes.c_float), ("faces", ctypes.POINTER(rt_face_desc)), ("n_faces", ctypes.c_int64),
                ("bbox_min", ctypes.c_double * 4), ("bbox_max", ctypes.c_double * 4)]


class rt_light_desc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("reserved", ctypes.c_int32), ("xf", rt_xform_desc),
                ("color", ctypes.c_double * 3), ("vec", ctypes.c_double * 4), ("falloff", ctypes.c_double)]


class rt_camera_desc(ctypes.Structure):
    _fields_ = [("xf", rt_xform_desc), ("eye", ctypes.c_double * 4), ("lower_left", ctypes.c_double * 4),
                ("lower_right", ctypes.c_double * 4), ("upper_left", ctypes.c_double * 4),
                ("upper_right", ctypes.c_double * 4)]


class rt_scene_desc(ctypes.Structure):
    """Scene (scene.h:35-38) as flat arrays (include/rtamd.h)."""
    _fields_ = [("has_camera", ctypes.c_int32), ("n_geometries", ctypes.c_int32), ("n_lights", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("camera", rt_camera_desc),
                ("geometries", ctypes.POINTER(rt_geometry_desc)), ("lights", ctypes.POINTER(rt_light_desc))]


RT_GEOM_SPHERE, RT_GEOM_MESH = 0, 1
RT_LIGHT_POINT, RT_LIGHT_DIRECTIONAL, RT_LIGHT_AMBIENT = 0, 1, 2

PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)

_libs: dict = {}
RTAMD_ABI_VERSION = 5  # include/rtamd.h


def lib(diag: bool = False) -> ctypes.CDLL:
    """Loads librtamd.so (built in-tree by ``make -C cs184-raytracer_amd``); fails loudly.
    ``diag``: librtamd_diag.so instead, the same library with the rt_debug_* hooks (a separate
    instance: its scenes are its own)."""
    path = DIAG_LIB_PATH if diag else LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with `make -C cs184-raytracer_amd` "
                          "(or __graft_entry__.build())")
    try:
        # One HIP runtime per process: when PyTorch is present its libamdhip64.so.7 must be
        # the one librtamd binds to (same soname), so torch buffers/streams/RCCL interoperate.
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    vp, cp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
    sig = {
        "rt_builder_create": (vp, []),
        "rt_builder_destroy": (None, [vp]),
        "rt_builder_parse_rti": (i32, [vp, cp]),
        "rt_builder_has_camera": (i32, [vp]),
        "rt_builder_warnings": (cp, [vp]),
        "rt_scene_create": (i32, [vp, i32, ctypes.POINTER(vp)]),
        "rt_scene_destroy": (None, [vp]),
        "rt_scene_get_info": (i32, [vp, ctypes.POINTER(rt_scene_info)]),
        "rt_render": (i32, [vp, ctypes.POINTER(rt_render_params), vp, PROGRESS_FN, vp, ctypes.POINTER(rt_counters)]),
        "rt_render_rgb8": (i32, [vp, ctypes.POINTER(rt_render_params), vp, PROGRESS_FN, vp,
                                 ctypes.POINTER(rt_counters)]),
        "rt_render_device": (i32, [vp, ctypes.POINTER(rt_render_params), vp, vp, vp, ctypes.POINTER(rt_counters)]),
        "rt_builder_get_desc": (i32, [vp, ctypes.POINTER(rt_scene_desc)]),
        "rt_builder_set_desc": (i32, [vp, ctypes.POINTER(rt_scene_desc)]),
        "rt_scene_create_desc": (i32, [ctypes.POINTER(rt_scene_desc), i32, ctypes.POINTER(vp)]),
        "rt_partition_row": (None, [i64, i32, i32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64)]),
        "rt_render_batch_device": (i32, [vp, i32, ctypes.POINTER(rt_render_params), ctypes.POINTER(vp),
                                         ctypes.POINTER(vp), vp, ctypes.POINTER(rt_counters)]),
        "rt_normalize_device": (i32, [vp, vp, i64, dbl, vp, vp]),
        "rt_to_rgb8": (None, [vp, i64, vp]),
        "rt_write_png": (i32, [cp, vp, i32, i32]),
        "rt_last_error": (cp, []),
        "rt_version": (cp, []),
        "rt_device_count": (i32, []),
        "rt_selftest_math": (i32, [i32, i32, vp, vp, vp, i64]),
    }
    if diag:
        sig.update({
            "rt_debug_builder_digest": (i32, [vp, ctypes.POINTER(ctypes.c_uint64)]),
            "rt_debug_fail_after": (i32, [vp, i32]),
            "rt_debug_corrupt_rows": (i32, [vp]),
            "rt_debug_plan_chunks": (i32, [i32, ctypes.POINTER(rt_render_params), i32, i64, i32,
                                           ctypes.POINTER(ctypes.c_int64), i32]),
            "rt_debug_phase_profile": (i32, [i32, vp]),
            "rt_debug_wave_times": (i32, [i32, vp, i32]),
            "rt_debug_fetch_calibration": (i32, [i32, i64]),
            "rt_debug_valu_calibration": (i32, [i32, i32]),
            "rt_debug_valu_rate": (i32, [i32, i32, i32, i32, ctypes.POINTER(dbl)]),
        })
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    # the ctypes structs above mirror include/rtamd.h of this ABI version (RTAMD_ABI_CHECK=0
    # loads a library of an older revision for a bisection: its structs must be a prefix of these)
    if os.environ.get("RTAMD_ABI_CHECK") == "0" and not hasattr(L, "rt_abi_version"):
        _libs[path] = L
        return L
    L.rt_abi_version.restype, L.rt_abi_version.argtypes = i32, []
    if L.rt_abi_version() != RTAMD_ABI_VERSION:
        raise ImportError(f"{path} has ABI version {L.rt_abi_version()}, this binding expects "
                          f"{RTAMD_ABI_VERSION} (include/rtamd.h RTAMD_ABI_VERSION): rebuild it")
    _libs[path] = L
    return L


def _rows4(rows, height):
    """(begin, end, step[, block]) row selection (rt_render_params); None = every row."""
    if rows is None:
        return 0, height, 1, 1
    return (tuple(rows) + (1,))[:4]


def selected_rows(begin: int, end: int, step: int, block: int = 1) -> List[int]:
    """The image rows a row selection renders, in order (rt_render_params: blocks of
    `block` rows, one block every step * block rows)."""
    block = max(1, block)
    return [r for r in range(begin, end) if ((r - begin) // block) % step == 0]


def selected_count(begin: int, end: int, step: int, block: int = 1) -> int:
    return len(selected_rows(begin, end, step, block))


def _raise(rc: int, what: str = "", L: Optional[ctypes.CDLL] = None) -> None:
    if rc == RT_OK:
        return
    msg = (L or lib()).rt_last_error().decode(errors="replace")
    cls = {RT_ERR_PARSE: ParseException, RT_ERR_MATH: MathException, RT_ERR_ARG: ArgumentError,
           RT_ERR_DEVICE: DeviceError, RT_ERR_IO: WriteException}.get(rc, RTError)
    raise cls(msg or what)


@dataclass
class Options:
    """Options (options.h:10-16); ``programOptions`` below is the module-wide instance."""
    inputFilenames_: List[str] = field(default_factory=list)
    outputFilename_: str = ""
    renderThreadsCount_: int = 1
    renderWidth_: int = 500
    renderHeight_: int = 500
    bounceDepth_: int = 10
    intersectionOnly_: bool = False


programOptions = Options()


@dataclass
class RenderStats:
    trace_rays: int
    shadow_rays: int
    reflect_rays: int
    refract_rays: int
    pixels: int
    intersection_max: float
    kernel_ms: float
    levels: int
    trace_launches: int
    node_visits: int
    tri_tests: int
    candidates: int
    sphere_tests: int
    stage_ms: tuple = ()            # (k_closest, k_shadow, k_shade) device ms
    stage_launches: tuple = ()
    stage_node_visits: tuple = ()   # (closest, shadow)
    stage_tri_tests: tuple = ()
    stage_candidates: tuple = ()
    stage_sphere_tests: tuple = ()
    stage_bvh_traversals: tuple = ()
    stage_max_node_visits: tuple = ()
    shadow_rays_zero_terms: int = 0  # shadow rays decided without traversal (zero Phong terms)

    @property
    def rays(self) -> int:
        """Rays in the Mrays/s metric: traceRay calls + shadow rays."""
        return self.trace_rays + self.shadow_rays


def _stats(c: rt_counters) -> RenderStats:
    return RenderStats(c.trace_rays, c.shadow_rays, c.reflect_rays, c.refract_rays, c.pixels, c.intersection_max,
                       c.kernel_ms, c.levels, c.trace_launches, c.node_visits, c.tri_tests, c.candidates,
                       c.sphere_tests, tuple(c.stage_ms), tuple(c.stage_launches), tuple(c.stage_node_visits),
                       tuple(c.stage_tri_tests), tuple(c.stage_candidates), tuple(c.stage_sphere_tests),
                       tuple(c.stage_bvh_traversals), tuple(c.stage_max_node_visits),
                       c.shadow_rays_zero_terms)


class Scene:
    """Scene (scene.h:9-39): accumulates parsed files; uploads to HBM on first render."""

    def __init__(self, device: int = 0, diag: bool = False):
        """``diag``: the scene lives in librtamd_diag.so (test hooks: digest, debug_*)."""
        self._L = lib(diag)
        self._b = self._L.rt_builder_create()
        self._scene = None
        self.device = device
        self.last_stats: Optional[RenderStats] = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def close(self) -> None:
        if getattr(self, "_scene", None):
            self._L.rt_scene_destroy(self._scene)
            self._scene = None
        if getattr(self, "_b", None):
            self._L.rt_builder_destroy(self._b)
            self._b = None

    def hasCamera(self) -> bool:  # scene.h:20
        return bool(self._L.rt_builder_has_camera(self._b))

    def warnings(self) -> str:
        return self._L.rt_builder_warnings(self._b).decode()

    def _parse(self, filename: str) -> None:
        if self._scene:
            raise ArgumentError("scene already uploaded; parse all files before rendering")
        _raise(self._L.rt_builder_parse_rti(self._b, os.fsencode(filename)), L=self._L)

    def upload(self) -> None:
        """rt_scene_create: build the LBVHs and upload the scene to the device once."""
        if self._scene:
            return
        p = ctypes.c_void_p()
        _raise(self._L.rt_scene_create(self._b, self.device, ctypes.byref(p)), L=self._L)
        self._scene = p

    @property
    def handle(self) -> ctypes.c_void_p:
        self.upload()
        return self._scene

    def info(self) -> rt_scene_info:
        i = rt_scene_info()
        _raise(self._L.rt_scene_get_info(self.handle, ctypes.byref(i)), L=self._L)
        return i

    def params(self, width: int, height: int, bounce_depth: int, intersection_only: bool, row_begin: int = 0,
               row_end: Optional[int] = None, row_step: int = 1, chunk_pixels: int = 0,
               row_block: int = 1, work_stats: bool = False) -> rt_render_params:
        """``work_stats``: count the traversal work (RenderStats.node_visits ...; rt_render_params)."""
        return rt_render_params(width, height, bounce_depth, int(bool(intersection_only)), row_begin,
                                height if row_end is None else row_end, row_step, chunk_pixels, row_block,
                                int(bool(work_stats)))

    def renderScene(self, output: Optional[np.ndarray] = None,
                    phandler: Optional[Callable[[int, int], None]] = None, options: Optional[Options] = None,
                    rows: Optional[tuple] = None, chunk_pixels: int = 0) -> np.ndarray:
        """Scene::renderScene (scene.cpp:10-59).

        ``output`` is the RasterImage: float64 array of shape (H, W, 3), caller-owned (allocated
        here from ``options`` when None).  ``rows = (begin, end, step[, block])`` renders a
        row-interleaved subset (blocks of ``block`` rows) into an (n_rows, W, 3) array (multi-GPU
        partition).
        """
        o = options or programOptions
        W, H = o.renderWidth_, o.renderHeight_
        rb, re_, rs, blk = _rows4(rows, H)
        n_rows = selected_count(rb, re_, rs, blk)
        if output is None:
            output = np.empty((n_rows, W, 3), dtype=np.float64)
        if output.dtype != np.float64 or output.shape != (n_rows, W, 3) or not output.flags.c_contiguous:
            raise ArgumentError(f"output must be a C-contiguous float64 array of shape {(n_rows, W, 3)}")
        prm = self.params(W, H, o.bounceDepth_, o.intersectionOnly_, rb, re_, rs, chunk_pixels, blk)
        cb = PROGRESS_FN((lambda c, t, u: phandler(c, t)) if phandler else (lambda c, t, u: None))
        cnt = rt_counters()
        _raise(self._L.rt_render(self.handle, ctypes.byref(prm), output.ctypes.data_as(ctypes.c_void_p), cb, None,
                               ctypes.byref(cnt)), L=self._L)
        self.last_stats = _stats(cnt)
        return output

    def render_rgb8(self, options: Optional[Options] = None, rows: Optional[tuple] = None,
                    phandler: Optional[Callable[[int, int], None]] = None, chunk_pixels: int = 0) -> np.ndarray:
        """rt_render_rgb8: renderScene + convertToRGBImage (writers.cpp:4-9) quantised on the device;
        returns a uint8 (n_rows, W, 3) array."""
        o = options or programOptions
        W, H = o.renderWidth_, o.renderHeight_
        rb, re_, rs, blk = _rows4(rows, H)
        n_rows = selected_count(rb, re_, rs, blk)
        out = np.empty((n_rows, W, 3), dtype=np.uint8)
        prm = self.params(W, H, o.bounceDepth_, o.intersectionOnly_, rb, re_, rs, chunk_pixels, blk)
        cb = PROGRESS_FN((lambda c, t, u: phandler(c, t)) if phandler else (lambda c, t, u: None))
        cnt = rt_counters()
        _raise(self._L.rt_render_rgb8(self.handle, ctypes.byref(prm), out.ctypes.data_as(ctypes.c_void_p), cb, None,
                                    ctypes.byref(cnt)), L=self._L)
        self.last_stats = _stats(cnt)
        return out

    def desc(self) -> rt_scene_desc:
        """rt_builder_get_desc: the parsed scene as a flat descriptor (views into the builder,
        valid while this Scene lives and parses nothing more)."""
        d = rt_scene_desc()
        _raise(self._L.rt_builder_get_desc(self._b, ctypes.byref(d)), L=self._L)
        return d

    def set_desc(self, d: rt_scene_desc) -> None:
        """rt_builder_set_desc: replace the (not yet uploaded) scene by a descriptor's."""
        if self._scene:
            raise ArgumentError("scene already uploaded")
        _raise(self._L.rt_builder_set_desc(self._b, ctypes.byref(d)), L=self._L)

    @classmethod
    def from_desc(cls, d: rt_scene_desc, device: int = 0, diag: bool = False) -> "Scene":
        """rt_scene_create_desc: a device scene straight from a descriptor (no builder scene)."""
        s = cls(device, diag)
        p = ctypes.c_void_p()
        _raise(s._L.rt_scene_create_desc(ctypes.byref(d), device, ctypes.byref(p)), L=s._L)
        s._scene = p
        return s

    def digest(self) -> int:
        """Host-side digest of the device scene rt_scene_create would upload (diag scenes)."""
        h = ctypes.c_uint64()
        _raise(self._L.rt_debug_builder_digest(self._b, ctypes.byref(h)), L=self._L)
        return h.value

    def debug_fail_after(self, launches: int) -> None:
        """Fault injection (diag scenes): the next render fails after `launches` closest-hit launches."""
        _raise(self._L.rt_debug_fail_after(self.handle, launches), L=self._L)

    def debug_corrupt_rows(self) -> None:
        """Fault injection (diag scenes): the next chunk's row descriptors name rows no frame has."""
        _raise(self._L.rt_debug_corrupt_rows(self.handle), L=self._L)

    def render_device(self, params: rt_render_params, out_rgb_ptr: int = 0, out_rgb8_ptr: int = 0,
                      stream_ptr: int = 0) -> RenderStats:
        """rt_render_device into device buffers (e.g. torch tensors' data_ptr())."""
        cnt = rt_counters()
        _raise(self._L.rt_render_device(self.handle, ctypes.byref(params), out_rgb_ptr or None, out_rgb8_ptr or None,
                                      stream_ptr or None, ctypes.byref(cnt)), L=self._L)
        self.last_stats = _stats(cnt)
        return self.last_stats

    def render_batch_device(self, params: Sequence[rt_render_params], out_rgb_ptrs: Sequence[int] = (),
                            out_rgb8_ptrs: Sequence[int] = (), stream_ptr: int = 0) -> RenderStats:
        """rt_render_batch_device: len(params) renders, images pipelined over the scene's lanes;
        missing/0 pointers are NULL.  Stats are sums over the batch."""
        n = len(params)
        prm = (rt_render_params * max(n, 1))(*params)
        ptrs = lambda xs: (ctypes.c_void_p * max(n, 1))(*[(xs[k] if k < len(xs) else 0) or None for k in range(n)])
        cnt = rt_counters()
        _raise(self._L.rt_render_batch_device(self.handle, n, prm, ptrs(out_rgb_ptrs), ptrs(out_rgb8_ptrs),
                                            stream_ptr or None, ctypes.byref(cnt)), L=self._L)
        self.last_stats = _stats(cnt)
        return self.last_stats

    def normalize_device(self, rgb_ptr: int, n_pixels: int, max_value: float, out_rgb8_ptr: int = 0,
                         stream_ptr: int = 0) -> None:
        _raise(self._L.rt_normalize_device(self.handle, rgb_ptr, n_pixels, max_value, out_rgb8_ptr or None,
                                         stream_ptr or None), L=self._L)


class RTIParser:
    """RTIParser (parsers.h:5-47): one instance per file, transform/material restart."""

    def __init__(self, scene: Scene):
        self.scene = scene

    def parseFile(self, filename: str) -> None:
        self.scene._parse(filename)


def to_rgb8(image: np.ndarray) -> np.ndarray:
    """PNGWriter::convertToRGBImage (writers.cpp:4-9)."""
    img = np.ascontiguousarray(image, dtype=np.float64)
    out = np.empty(img.shape, dtype=np.uint8)
    lib().rt_to_rgb8(img.ctypes.data_as(ctypes.c_void_p), img.size // 3, out.ctypes.data_as(ctypes.c_void_p))
    return out


class PNGWriter:
    """PNGWriter (writers.h:5-16): byte-identical to libpng 1.6.13's simplified writer."""

    def __init__(self, filename: str):
        self.filename = filename

    def writeImage(self, image: np.ndarray) -> None:
        rgb = image if image.dtype == np.uint8 else to_rgb8(image)
        rgb = np.ascontiguousarray(rgb)
        h, w = rgb.shape[0], rgb.shape[1]
        _raise(lib().rt_write_png(os.fsencode(self.filename), rgb.ctypes.data_as(ctypes.c_void_p), w, h))


def partition_row(row: int, n_devices: int, row_block: int):
    """rt_partition_row: (device, local row) of image row `row` in the multi-GPU partition."""
    d, l = ctypes.c_int(), ctypes.c_int64()
    lib().rt_partition_row(row, n_devices, row_block, ctypes.byref(d), ctypes.byref(l))
    return d.value, l.value


def device_count() -> int:
    return int(lib().rt_device_count())


def selftest_math(op: str, x: np.ndarray, y: Optional[np.ndarray] = None, device: int = 0) -> np.ndarray:
    """Runs the kernels' device pow/sqrt/div on the GPU for comparison with the host libm.
    "norm_x|y|z": component of normalized3 of the vector (x[i], y[i], x[(i + n/2) % n])."""
    code = {"pow": 0, "sqrt": 1, "div": 2, "norm_x": 4, "norm_y": 5, "norm_z": 6}[op]
    x = np.ascontiguousarray(x, dtype=np.float64)
    yy = np.ascontiguousarray(y if y is not None else x, dtype=np.float64)
    out = np.empty_like(x)
    _raise(lib().rt_selftest_math(device, code, x.ctypes.data_as(ctypes.c_void_p), yy.ctypes.data_as(ctypes.c_void_p),
                                  out.ctypes.data_as(ctypes.c_void_p), x.size))
    return out


def load_scene(files, device: int = 0, diag: bool = False) -> Scene:
    """main.cpp:53-66: one RTIParser per file, camera required (``diag``: in librtamd_diag.so)."""
    s = Scene(device, diag)
    for f in ([files] if isinstance(files, (str, os.PathLike)) else files):
        RTIParser(s).parseFile(str(f))
    if not s.hasCamera():
        raise ArgumentError("At least one camera must be specified.")
    return s
