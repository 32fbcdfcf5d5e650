"""The C ABI boundary: the library loads, exports exactly what include/rt.h
declares, and reports errors as codes (no GPU needed)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT


def declared_functions():
    src = open(os.path.join(ROOT, "include", "rt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(rt_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol(rt):
    names = declared_functions()
    assert len(names) >= 40
    so = os.path.join(ROOT, "02562_raytracer_amd", "lib02562rt.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    # and the Python binding declares a signature for each
    assert set(names) == set(rt._ffi.SIGNATURES), set(names) ^ set(rt._ffi.SIGNATURES)


def test_library_contains_gfx950_code_object():
    so = os.path.join(ROOT, "02562_raytracer_amd", "lib02562rt.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data


def test_struct_sizes(rt):
    F = rt._ffi
    assert C.sizeof(F.Material) == 64        # src/mesh.rs:12-20
    assert C.sizeof(F.GpuNode) == 32         # hlbvh.rs:508-528
    assert C.sizeof(F.Uniform) == 80         # uniform.rs:6-34
    assert C.sizeof(F.RayCounts) == 23 * 8


def test_error_codes_without_gpu(rt):
    L = rt.lib()
    h = C.c_void_p()
    # no context: invalid / device error codes, message available
    assert L.rt_create(-1, C.byref(h)) in (rt._ffi.RT_E_DEVICE, rt._ffi.RT_E_INVALID)
    assert L.rt_last_error(None)
    assert L.rt_mesh_load_obj(b"/nonexistent.obj", C.byref(h)) == rt._ffi.RT_E_IO
    assert L.rt_bsp_build(None, 20, 4, 0, C.byref(h)) == rt._ffi.RT_E_INVALID
    assert L.rt_tileset_local_tiles(1920, 1080, 8) == (240 * 135 + 7) // 8
    assert L.rt_tileset_local_tiles(70, 45, 3) == (9 * 6 + 2) // 3
    assert L.rt_tileset_local_tiles(16, 16, 0) == 0
    m = C.c_int(-1)
    assert L.rt_bsp_cull_in_use(None, C.byref(m), None, None) == rt._ffi.RT_E_INVALID


def test_scene_table_mirrors_reference(rt):
    sc = rt.get_scenes()
    assert len(sc) == 44                                      # src/scenes.rs:98-487
    names = [s.name for s in sc]
    assert names[0] == "W1 E1" and names[-1] == "Project: Dragon BSP"
    hot = [s for s in sc if s.mode]
    assert {s.mode for s in hot} == {"W1E6", "W6E1", "PROJECT", "W7E3", "W9E1", "W8E1", "W8E2", "W8E3", "W9E2", "W6E2",
                                      "W7E1", "W7E2", "W6E3", "W9E3"}
    w8 = rt.find_scene("W8 E3 Absorption")
    assert w8.mode == "W8E3" and w8.model == "CornellBox.obj"
    w7 = rt.find_scene("W7 E3 Cornell Box")
    assert w7.mode == "W7E3" and w7.traverse_type == "BSP" and w7.camera.eye == (277.0, 275.0, -570.0)
    assert rt.find_scene("Project: Bunny").traverse_type == "BVH"
    with pytest.raises(KeyError):
        rt.find_scene("nope")
