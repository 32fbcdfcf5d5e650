"""The C++ host layer (include/raytracer.hpp, 02562_raytracer_amd/host/) through
its headless driver bin/rt_render, CPU-only parts: the scene table, the camera
controller and the jitter table must equal the Python mirror bit for bit
(both restate src/scenes.rs, src/camera.rs and src/bindings/uniform.rs)."""
import importlib
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "02562_raytracer_amd", "bin", "rt_render")

pytestmark = pytest.mark.skipif(not os.path.exists(BIN), reason="bin/rt_render not built (make -C 02562_raytracer_amd)")


def run(*args):
    r = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def f32(x):
    return np.float32(float.fromhex(x) if isinstance(x, str) else x)


def test_scene_table_equals_python(rt):
    cpp = [json.loads(l) for l in run("--list-scenes").splitlines()]
    py = rt.get_scenes()
    assert len(cpp) == len(py) == 44
    for c, p in zip(cpp, py):
        assert c["name"] == p.name and c["shader"] == p.shader and c["mode"] == p.mode
        assert c["model"] == p.model and tuple(c["res"]) == tuple(p.res)
        assert c["vertex_type"] == p.vertex_type and c["traverse_type"] == p.traverse_type
        assert c["background_hdri"] == p.background_hdri
        for k, v in (("eye", p.camera.eye), ("target", p.camera.target), ("up", p.camera.up)):
            assert [f32(x) for x in c["camera"][k]] == [np.float32(x) for x in v], (p.name, k)
        assert f32(c["camera"]["constant"]) == np.float32(p.camera.constant)


@pytest.mark.parametrize("keys,n", [("W", 30), ("S", 7), ("A", 40), ("D", 40), ("W,D", 25), ("Up,Left", 60),
                                    ("W,A,S,D", 12), ("Down,Right", 3)])
def test_camera_controller_equals_python(keys, n):
    cam_mod = importlib.import_module("02562_raytracer_amd.camera")
    c = json.loads(run("--camera-test", keys, str(n)))
    cam = cam_mod.Camera()
    ctl = cam_mod.CameraController()
    for k in keys.split(","):
        ctl.handle_camera_commands(k, True)
    for _ in range(n):
        ctl.update_camera(cam)
    assert [f32(x) for x in c["eye"]] == [np.float32(x) for x in cam.eye]


@pytest.mark.parametrize("subdiv,h", [(1, 512), (2, 450), (3, 512), (10, 1080)])
def test_jitter_table_equals_python(subdiv, h):
    J = importlib.import_module("02562_raytracer_amd.jitter")
    rows = [l.split() for l in run("--jitter", str(subdiv), str(h)).splitlines()]
    cpp = np.array([[f32(x.strip('"')) for x in r] for r in rows], np.float32)
    assert np.array_equal(cpp.view(np.uint32), J.jitters_for(h, subdiv).view(np.uint32))


def test_scene_errors():
    r = subprocess.run([BIN, "--scene", "W1 E1"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
