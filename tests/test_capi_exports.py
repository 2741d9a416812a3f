"""The product C-ABI library loads on a CPU-only host and exports every function that
include/eray_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header="eray_hip.h"):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(eray_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("eray_render", "eray_node_wave", "eray_node_rgb", "eray_node_flat_color",
                 "eray_node_mix_color", "eray_scene_add_object", "eray_pack_ppm", "eray_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from eray_amd import capi
    lib = capi.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared_functions()) == set(capi.SIGNATURES), "ctypes signatures out of sync"
    assert lib.eray_abi_version() == 6


def test_debug_exports_are_declared_apart():
    """The test-only diagnostics are declared in include/eray_hip_debug.h, not in the boundary
    header, and the library exports exactly those (ADVICE/VERDICT r02 W9)."""
    from eray_amd import capi
    lib = capi.lib()
    debug = [n for n in declared_functions("eray_hip_debug.h") if n.startswith("eray_debug_")]
    assert debug and set(debug) == set(capi.DEBUG_SIGNATURES)
    assert not [n for n in declared_functions() if n.startswith("eray_debug_")]
    assert all(hasattr(lib, n) for n in debug)


def test_no_gpu_fails_loudly():
    """Without a GPU the context cannot be created: an error, never a silent CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from eray_amd import capi
    with pytest.raises(capi.ErayError) as e:
        capi.Context(0)
    assert e.value.status == capi.E_HIP


def test_ppm_header_and_camera_size_are_host_only():
    from eray_amd import capi
    assert capi.ppm_header(1920, 1080) == b"P6 1920 1080 255\n"
    assert capi.camera_size(capi.make_camera(fov=(16.0, 9.0), width=1920)) == (1920, 1080)
