"""Host-side (CPU) checks of librtamd: ABI exports, PNG writer, ingest, pow restatement, CLI.

No GPU is needed: these load librtamd.so and call only its host functions.
"""
import os
import re
import subprocess

import numpy as np
import pytest

from cases import REPO, SCENES, SHIPPED, scene_files

HEADER = os.path.join(REPO, "include", "rtamd.h")
CLI = os.path.join(REPO, "cs184-raytracer_amd", "bin", "rtamd")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rt_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_function(rt):
    names = declared_functions()
    assert len(names) >= 17
    for n in names:
        assert hasattr(rt.lib(), n), f"{n} declared in include/rtamd.h but not exported"


DIAG_HOOKS = ["rt_debug_builder_digest", "rt_debug_fail_after", "rt_debug_corrupt_rows",
              "rt_debug_plan_chunks", "rt_debug_phase_profile",
              "rt_debug_wave_times", "rt_debug_fetch_calibration", "rt_debug_valu_calibration", "rt_debug_valu_rate"]


def test_production_library_has_no_debug_hooks(rt):
    """The test and measurement hooks live in librtamd_diag.so only (csrc/diag.cpp): the
    product library exports the rtamd.h surface and nothing named rt_debug_*."""
    names = subprocess.run(["nm", "-D", "--defined-only", rt.LIB_PATH], capture_output=True, text=True,
                           check=True).stdout
    assert "rt_debug_" not in names
    diag = rt.lib(diag=True)
    for n in DIAG_HOOKS:
        assert hasattr(diag, n), n
    for n in declared_functions():
        assert hasattr(diag, n), n


def test_multi_library_exports_every_declared_function(rt):
    """librtamd_multi.so (RCCL multi-GPU render) exports include/rtamd_multi.h; loading it
    needs no GPU."""
    import ctypes
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "rtamd_multi.h")).read(), flags=re.S)
    names = sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rt_multi\w+)\s*\(", text, flags=re.M)))
    assert len(names) == 5
    L = ctypes.CDLL(os.path.join(REPO, "cs184-raytracer_amd", "rtamd", "librtamd_multi.so"))
    for n in names:
        assert hasattr(L, n), n


@pytest.mark.parametrize("n,block", [(1, 8), (2, 8), (3, 8), (8, 8), (4, 1), (3, 5), (16, 16)])
def test_partition_row_matches_dist(rt, n, block):
    """The multi-GPU de-interleave map (rt_partition_row, k_deinterleave's index math) is the
    inverse of every device's row selection (rtamd.dist.rows_of / rt_render_params)."""
    from rtamd import dist as rd
    H = 1080
    owner = {}
    for d in range(n):
        for k, r in enumerate(rd.rows_of(H, d, n, block)):
            owner[r] = (d, k)
    assert sorted(owner) == list(range(H))
    for r in range(H):
        assert rt.partition_row(r, n, block) == owner[r]


@pytest.mark.parametrize("png", sorted(SHIPPED))
def test_png_writer_is_byte_identical_to_libpng(rt, tmp_path, png):
    from PIL import Image
    ref = os.path.join(REPO, "tests", "golden", "shipped", png)
    rgb = np.ascontiguousarray(np.asarray(Image.open(ref).convert("RGB")))
    out = tmp_path / png
    rt.PNGWriter(str(out)).writeImage(rgb)
    assert out.read_bytes() == open(ref, "rb").read()


def test_png_writer_small_images_use_reduced_window(rt, tmp_path):
    """Images <= 16 KiB take libpng's windowBits reduction + CMF rewrite (pngwutil.c:251-288,370-385)."""
    from PIL import Image
    for w, h in [(1, 1), (7, 5), (40, 30), (73, 74)]:
        rgb = (np.arange(w * h * 3, dtype=np.uint32).reshape(h, w, 3) * 37 % 251).astype(np.uint8)
        out = tmp_path / f"s{w}x{h}.png"
        rt.PNGWriter(str(out)).writeImage(rgb)
        assert np.array_equal(np.asarray(Image.open(out).convert("RGB")), rgb)


def test_to_rgb8_matches_writer_conversion(rt, oracle):
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.normal(0.5, 0.7, 30000), [np.nan, np.inf, -np.inf, 0.0, -0.0, 1.0, 255 / 255]])
    v = np.resize(v, (v.size // 3) * 3).reshape(-1, 1, 3)
    assert np.array_equal(rt.to_rgb8(v), oracle.to_rgb8(v))


@pytest.mark.parametrize("scene", scene_files())
def test_ingest_errors_and_warnings_match_oracle(rt, oracle, scene):
    path = os.path.join(SCENES, scene)
    s = rt.Scene()
    err = None
    try:
        rt.RTIParser(s).parseFile(path)
    except rt.RTError as e:
        err = str(e)
    try:
        oracle.render(path, 2, 2, bdepth=0)
        oerr = None
    except oracle.OracleError as e:
        oerr = str(e)
    assert err == oerr
    assert s.warnings() == oracle.warnings()
    if err is None:
        assert s.hasCamera()


def test_pow_restatement_matches_libm(tmp_path):
    exe = tmp_path / "pow_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I" + os.path.join(REPO, "cs184-raytracer_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "pow_check.cpp"), "-o", str(exe)], check=True)
    p = subprocess.run([str(exe), "2000000"], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout


@pytest.mark.parametrize("args,msg", [
    ([], "Error: At least one input file must be specified."),
    (["x.rti"], "Error: An output file must be specified."),
    (["-o", "/tmp/x.png", "-w", "abc", "x.rti"], "Error: Width and/or height is invalid."),
    (["-o", "/tmp/x.png", "-h", "0", "x.rti"], "Error: Width and/or height must be positive."),
    (["-o", "/tmp/x.png", "-t", "-2", "x.rti"], "Error: Thread count must be positive."),
    (["-o", "/tmp/x.png", "--bdepth", "-1", "x.rti"], "Error: Bounce depth must be non-negative."),
    (["-o", "/nonexistent_dir/x.png", "x.rti"], "Error: Output file is not writable."),
    (["-o", "/tmp/rtamd_cli_test.png", "/nonexistent.rti"], "Error: file not found: /nonexistent.rti"),
    (["-o", "/tmp/x.png", "--gpus", "0", "x.rti"], "Error: GPU count is invalid."),
])
def test_cli_option_errors_match_reference(args, msg):
    """options.cpp:18-86 / main.cpp:40-66 messages and exit status 1 (checked before any GPU use)."""
    if not os.path.exists(CLI):
        pytest.skip("CLI not built")
    p = subprocess.run([CLI] + args, capture_output=True, text=True)
    assert p.returncode == 1
    assert msg in p.stderr


def test_libm_pow_identities_used_by_shading():
    """k_shade skips pow for exponents -0/+0 (falloff 0) and 1 (ns 1): glibc's pow returns
    exactly 1 and exactly x there (trace.hip k_shade)."""
    import ctypes
    m = ctypes.CDLL("libm.so.6")
    m.pow.restype = ctypes.c_double
    m.pow.argtypes = [ctypes.c_double, ctypes.c_double]
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(0, 1, 20000), np.exp(rng.uniform(-700, 700, 20000)), [0.0, 1.0, np.inf]])
    for x in xs:
        x = float(x)
        assert m.pow(x, 1.0) == x
        assert m.pow(x, -0.0) == 1.0 and m.pow(x, 0.0) == 1.0
    assert np.isnan(m.pow(float("nan"), 1.0)) and m.pow(float("nan"), -0.0) == 1.0


def _plan(rt, params, lanes, chunk=1 << 22, balance=1):
    """rt_debug_plan_chunks: [(chunk, job, r0, rows)] of a render call (no device needed)."""
    import ctypes
    f = rt.lib(diag=True).rt_debug_plan_chunks
    arr = (rt.rt_render_params * len(params))(*params)
    out = (ctypes.c_int64 * (4 * 100000))()
    q = f(len(params), arr, lanes, chunk, balance, out, 100000)
    assert q >= 0
    return [tuple(out[4 * k:4 * k + 4]) for k in range(q)]


def _rows(p):
    from rtamd import dist as rd
    if p.row_block > 1:
        return rd.n_rows(p.height, p.row_begin // p.row_block, p.row_step, p.row_block)
    return len(range(p.row_begin, p.row_end, p.row_step))


@pytest.mark.parametrize("frames,ways,lanes", [(32, 1, 3), (32, 2, 3), (32, 4, 3), (32, 8, 3), (7, 1, 2), (5, 4, 3),
                                               (1, 1, 1), (3, 8, 3)])
def test_chunk_plan_covers_every_row_once(rt, frames, ways, lanes):
    """The chunk plan of a batch (render_jobs: packed and balanced chunks) covers every
    selected row of every frame exactly once, in order; a chunk holds at most one segment
    per frame and at most 4 M pixels; a balanced plan (fewer than two chunks per lane
    unbalanced) has a multiple of the lanes of chunks, cut on 8-row boundaries."""
    W, H = 1920, 1080
    mk = lambda: rt.rt_render_params(W, H, 4, 0, 0, H, 1, 0, 1, 0) if ways == 1 else \
        rt.rt_render_params(W, H, 4, 0, 8 * (ways - 1), H, ways, 0, 8, 0)  # the last rank's share
    params = [mk() for _ in range(frames)]
    plan = _plan(rt, params, lanes)
    for j, p in enumerate(params):
        segs = [(r0, n) for c, jj, r0, n in plan if jj == j]
        nxt = 0
        for r0, n in segs:
            assert r0 == nxt and n > 0
            nxt += n
        assert nxt == _rows(p)
    chunks = sorted({c for c, *_ in plan})
    assert chunks == list(range(len(chunks)))
    for c in chunks:
        segs = [s for s in plan if s[0] == c]
        assert len({s[1] for s in segs}) == len(segs)
        assert sum(s[3] for s in segs) * W <= 1 << 22
    total = sum(_rows(p) for p in params)
    lim = (1 << 22) // W // 8 * 8
    unbalanced = -(-total // lim)
    if frames > 1 and unbalanced < 2 * lanes and unbalanced % lanes:
        n = -(-unbalanced // lanes) * lanes                # a multiple of the lanes
        rows = min(lim, (-(-total // n) + 7) // 8 * 8)     # equal chunks, 8-row cuts
        assert len(chunks) == -(-total // rows) and len(chunks) <= n
        for c in chunks[:-1]:
            assert sum(s[3] for s in plan if s[0] == c) == rows


@pytest.mark.parametrize("frames", [32, 48])
def test_chunk_plan_unbalanced_whole_frames(rt, frames):
    """Whole frames of a 32- or 48-frame step (bench.py's default) keep their two-frame chunks
    (16 or 24 of them: many chunks per lane, so no balancing; 48 frames give every one of the
    3 lanes 8) and the balancing switch changes nothing there."""
    W, H = 1920, 1080
    params = [rt.rt_render_params(W, H, 4, 0, 0, H, 1, 0, 1, 0) for _ in range(frames)]
    a, b = _plan(rt, params, 3, balance=1), _plan(rt, params, 3, balance=0)
    assert a == b
    assert len({c for c, *_ in a}) == frames // 2 and all(n == H for *_, n in a)


def test_ctypes_structs_match_the_header_layout(rt, tmp_path):
    """The Python mirror's structures (rtamd/__init__.py) have the C header's field offsets
    and sizes: a C program compiled against include/rtamd.h prints offsetof / sizeof of every
    field the ctypes classes declare."""
    import ctypes
    structs = [getattr(rt, n) for n in dir(rt) if n.startswith("rt_") and isinstance(getattr(rt, n), type)
               and issubclass(getattr(rt, n), ctypes.Structure)]
    assert len(structs) >= 10
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "rtamd.h"', "int main(void) {"]
    want = []
    for st in structs:
        name = st.__name__
        lines.append(f'  printf("%zu\\n", sizeof({name}));')
        want.append((name, "sizeof", ctypes.sizeof(st)))
        for f, *_ in st._fields_:
            lines.append(f'  printf("%zu\\n", offsetof({name}, {f}));')
            want.append((name, f, getattr(st, f).offset))
    lines += ["  return 0;", "}"]
    src = tmp_path / "abi.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "abi"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert len(got) == len(want)
    bad = [(w, g) for w, g in zip(want, got) if w[2] != g]
    assert not bad, bad
