"""C ABI checks that need no GPU: libfvo.so builds, loads, and exports every entry point
include/fvo.h declares; the product refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, gpu_available


def _declared():
    src = open(os.path.join(ROOT, "include", "fvo.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fvo_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_reference_entry_points():
    names = _declared()
    for n in ["fvo_orb_detect_compute", "fvo_bf_match", "fvo_sgbm", "fvo_backproject", "fvo_pnp_ransac",
              "fvo_create", "fvo_destroy", "fvo_last_error", "fvo_config_default", "fvo_gather_matches",
              "fvo_find_essential", "fvo_recover_pose"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    import forest_slam_amd.build as b
    path = b.build()
    lib = ctypes.CDLL(path)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.fvo_abi_version() == 7


def test_binding_signatures_cover_header():
    from forest_slam_amd import _lib
    assert set(_declared()) <= set(_lib.SIGNATURES)


def test_config_default_matches_reference_constants():
    from forest_slam_amd import _lib
    L = _lib.load()
    cfg = _lib.FvoConfig()
    L.fvo_config_default(ctypes.byref(cfg), 960, 600)
    # cv2.ORB_create() defaults and stereo_slam.py:109-115
    assert (cfg.nfeatures, cfg.nlevels, cfg.edge_threshold, cfg.patch_size, cfg.fast_threshold) == (500, 8, 31, 31, 20)
    assert abs(cfg.scale_factor - 1.2) < 1e-6
    assert (cfg.num_disparities, cfg.min_disparity, cfg.block_size, cfg.P1, cfg.P2) == (96, 0, 7, 392, 1568)
    assert cfg.sgbm_stripes == 4
    assert cfg.stages == 63  # FVO_STAGE_ALL
    assert (cfg.ba_window, cfg.ba_max_landmarks, cfg.ba_max_obs) == (10, 4096, 32768)
    # the SGBM schedule: classic, default launch shape, default hand-off bound
    assert (cfg.sgbm_mode, cfg.sgbm_lanes, cfg.sgbm_cols, cfg.sgbm_handoff_us) == (_lib.SGBM_CLASSIC, 0, 0, 0)


def test_library_reads_no_environment():
    """the SGBM schedule was chosen by FVO_SG_* environment variables read on every
    launch; it is fvo_config's now (ABI 7), and no source of the library reads the environment."""
    csrc = os.path.join(ROOT, "forest-slam_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        text = open(os.path.join(csrc, f)).read()
        assert "getenv" not in text and "FVO_SG_" not in text, f


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_context_fails_loudly_without_gpu():
    from forest_slam_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.Context(960, 600)


def test_config_layout_matches_binding():
    """the ctypes FvoConfig must match the compiled struct exactly (size and
    every field offset), or fvo_config_default writes past the Python object."""
    from forest_slam_amd import _lib
    L = _lib.load()
    assert L.fvo_config_size() == ctypes.sizeof(_lib.FvoConfig) == 31 * 4
    for name, _ in _lib.FvoConfig._fields_:
        assert L.fvo_config_offset(name.encode()) == getattr(_lib.FvoConfig, name).offset, name
    assert L.fvo_config_offset(b"no_such_field") == -1
    # every field the header declares is in the binding (and nothing else)
    src = open(os.path.join(ROOT, "include", "fvo.h")).read()
    body = src[src.index("typedef struct fvo_config {"):src.index("} fvo_config;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    declared = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*(?:,|;)", body.split("{", 1)[1])
    assert declared == [n for n, _ in _lib.FvoConfig._fields_]


def test_integration_raw_binding_snippet_runs_to_create():
    """The raw ctypes binding printed in INTEGRATION.md, executed verbatim up to its device
    calls: layout asserts pass, fvo_config_default fills the reference constants without
    overrunning the struct, and fvo_create returns a status (no GPU here: < 0, cleanly)."""
    import forest_slam_amd.build as b
    b.build()
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(import ctypes\n.*?)```", md, flags=re.S).group(1)
    code = block.split("# --- device calls")[0]
    code = code.replace('"forest-slam_amd/libfvo.so"', repr(os.path.join(ROOT, "forest-slam_amd", "libfvo.so")))
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    cfg = ns["cfg"]
    assert (cfg.width, cfg.height, cfg.nfeatures, cfg.num_disparities, cfg.P2, cfg.sgbm_max_batch) == \
        (960, 600, 500, 96, 1568, 0)
    if gpu_available():
        assert ns["rc"] == 0
    else:
        assert ns["rc"] < 0 and not ns["ctx"].value
