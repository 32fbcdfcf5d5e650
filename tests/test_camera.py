"""Headless camera controller (02562_raytracer_amd/camera.py) vs src/camera.rs
CameraController::update_camera, restated here in float64 from the Rust source
text and rounded: the f32 result must lie within a few ulp of the float64
path, and the invariants the controller states hold (forward stops one step
short of the target; left/right keep the eye on its circle about the target)."""
import importlib

import numpy as np
import pytest

cam_mod = importlib.import_module("02562_raytracer_amd.camera")


def _f64_update(eye, target, up, speed, keys):
    eye, target, up = (np.asarray(v, np.float64) for v in (eye, target, up))
    fwd = target - eye
    fn = fwd / np.linalg.norm(fwd)
    fm = np.linalg.norm(fwd)
    if "forward" in keys and fm > speed:
        eye = eye + fn * speed
    if "backward" in keys:
        eye = eye - fn * speed
    right = np.cross(fn, up)
    fwd = target - eye
    fm = np.linalg.norm(fwd)
    if "right" in keys:
        v = fwd + right * speed
        eye = target - v / np.linalg.norm(v) * fm
    if "left" in keys:
        v = fwd - right * speed
        eye = target - v / np.linalg.norm(v) * fm
    return eye


@pytest.mark.parametrize("keys", [("W",), ("S",), ("A",), ("D",), ("Up", "Right"), ("Down", "Left"),
                                  ("W", "S", "A", "D")])
def test_update_matches_float64(keys):
    cam = cam_mod.Camera()
    ctl = cam_mod.CameraController()
    for k in keys:
        assert ctl.handle_camera_commands(k, True)
    names = {ctl.KEYS[k] for k in keys}
    want = np.array(cam.eye, np.float64)
    for _ in range(25):
        want = _f64_update(want, cam.target, cam.up, 0.05, names)
        ctl.update_camera(cam)
        assert cam.eye.dtype == np.float32
    assert np.allclose(cam.eye, want, rtol=0, atol=2e-5)


def test_unknown_key_and_release():
    ctl = cam_mod.CameraController()
    assert not ctl.handle_camera_commands("Q", True)
    assert ctl.handle_camera_commands("W", True) and ctl.pressed["forward"]
    assert ctl.handle_camera_commands("W", False) and not ctl.pressed["forward"]
    cam = cam_mod.Camera()
    before = cam.eye.copy()
    ctl.update_camera(cam)
    assert np.array_equal(cam.eye, before)   # nothing pressed: the eye stays


def test_forward_stops_short_of_target():
    cam = cam_mod.Camera()
    ctl = cam_mod.CameraController()
    ctl.handle_camera_commands("W", True)
    for _ in range(200):
        ctl.update_camera(cam)
    d = np.linalg.norm(cam.target.astype(np.float64) - cam.eye)
    assert 0 < d <= 0.05 + 1e-6


def test_orbit_keeps_radius():
    cam = cam_mod.Camera()
    ctl = cam_mod.CameraController()
    r0 = np.linalg.norm(cam.target.astype(np.float64) - cam.eye)
    ctl.handle_camera_commands("D", True)
    for _ in range(100):
        ctl.update_camera(cam)
    r = np.linalg.norm(cam.target.astype(np.float64) - cam.eye)
    assert abs(r - r0) < 1e-4
