"""Camera and CameraController: mirror of src/camera.rs (Camera :13-34,
CameraController :36-112) for a headless RenderState.

Key events arrive as (key, pressed) pairs instead of winit's
Command::KeyEvent; the key names are winit's VirtualKeyCode names the
controller matches (W/Up, A/Left, S/Down, D/Right).  update_camera runs in f32
with cgmath's operation order (InnerSpace::normalize = v * (1 / |v|),
magnitude = sqrt(x*x + y*y + z*z)), so a camera moved here sits where the
reference's camera would, bit for bit.
"""
from dataclasses import dataclass, field

import numpy as np

F32 = np.float32
CAMERA_SPEED = 0.05   # src/render_state.rs:31


def _v(x):
    return np.asarray(x, dtype=F32).reshape(3)


def _dot(a, b):
    # cgmath Vector3::dot: mul_element_wise(...).sum(), summed x + y + z
    p = a * b
    return F32(F32(p[0] + p[1]) + p[2])


def _magnitude(a):
    return F32(np.sqrt(_dot(a, a), dtype=F32))


def _normalize(a):
    # InnerSpace::normalize -> normalize_to(1) = self * (1 / magnitude)
    return a * F32(F32(1.0) / _magnitude(a))


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], F32)


@dataclass
class Camera:
    """src/camera.rs:13-34 (Default: eye (2, 1.5, 2), target (0, 0.5, 0), up +y)."""
    eye: np.ndarray = field(default_factory=lambda: _v((2.0, 1.5, 2.0)))
    target: np.ndarray = field(default_factory=lambda: _v((0.0, 0.5, 0.0)))
    up: np.ndarray = field(default_factory=lambda: _v((0.0, 1.0, 0.0)))
    aspect: float = 1.0
    constant: float = 1.0

    @classmethod
    def from_tuple(cls, cam):
        """From a scenes.Camera (eye, target, up, constant)."""
        return cls(_v(cam.eye), _v(cam.target), _v(cam.up), 1.0, float(cam.constant))

    def as_args(self):
        """(eye, target, up, constant) for make_uniform."""
        return (tuple(float(x) for x in self.eye), tuple(float(x) for x in self.target),
                tuple(float(x) for x in self.up), float(self.constant))


class CameraController:
    """src/camera.rs:36-112."""

    KEYS = {"W": "forward", "Up": "forward", "A": "left", "Left": "left", "S": "backward", "Down": "backward",
            "D": "right", "Right": "right"}

    def __init__(self, speed=CAMERA_SPEED):
        self.speed = F32(speed)
        self.pressed = {"forward": False, "backward": False, "left": False, "right": False}

    def handle_camera_commands(self, key, pressed):
        """Command::KeyEvent -> True when the key is one the controller owns (:56-81)."""
        which = self.KEYS.get(key)
        if which is None:
            return False
        self.pressed[which] = bool(pressed)
        return True

    def update_camera(self, camera):
        """:83-111: forward/backward along the view ray (not closer than one
        step to the target), left/right around the target at fixed radius."""
        s = self.speed
        forward = camera.target - camera.eye
        forward_norm = _normalize(forward)
        forward_mag = _magnitude(forward)
        if self.pressed["forward"] and forward_mag > s:
            camera.eye = camera.eye + forward_norm * s
        if self.pressed["backward"]:
            camera.eye = camera.eye - forward_norm * s
        right = _cross(forward_norm, camera.up)
        forward = camera.target - camera.eye
        forward_mag = _magnitude(forward)
        if self.pressed["right"]:
            camera.eye = camera.target - _normalize(forward + right * s) * forward_mag
        if self.pressed["left"]:
            camera.eye = camera.target - _normalize(forward - right * s) * forward_mag
        return camera
