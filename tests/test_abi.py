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
    assert lib.fvo_abi_version() == 4


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


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_context_fails_loudly_without_gpu():
    from forest_slam_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.Context(960, 600)
