"""Headless RenderState (render_state.py) driving the kernel the way the
reference's rendering_thread does (src/lib.rs:321-489): SetSamples-limited
progressive stepping, scene reloads restarting the iteration, and the camera
controller moving the camera between frames (src/camera.rs).  Compared with
direct rt_render calls and with the CPU oracle."""
import numpy as np
import pytest

from parity_util import Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu


def test_progressive_steps_stop_at_max_iterations(rt):
    rs = rt.RenderState(rt.find_scene("W7 E3 Cornell Box"), resolution=(64, 48))
    try:
        rs.set_samples(3, True)
        n = 0
        while rs.step():
            n += 1
            assert n <= 3
        assert n == 3 and rs.iteration == 3
        frame = rs.frame().copy()
        # the same three iterations in one launch from a cleared buffer
        rs.reset_iteration()
        rs.accum.zero()
        rs.render(3)
        assert np.array_equal(frame.view(np.uint32), rs.frame().view(np.uint32))
        # a reload restarts the iteration
        rs.load_scene(rs.scene)
        assert rs.iteration == 0 and rs.step()
    finally:
        rs.ctx.close()


def test_camera_controller_moves_the_rendered_camera(rt):
    scene = rt.find_scene("W7 E3 Cornell Box")
    rs = rt.RenderState(scene, resolution=(48, 48))
    try:
        assert rs.input("D", True) and rs.input("W", True)
        rs.update()   # RenderState::update: the controller moves the camera
        rs.update()
        eye, target, up, constant = rs.camera.as_args()
        assert eye != scene.camera.eye
        rs.accum.zero()
        rs.render(2)
        got = (rs.frame(), rs.hit_ids(), None)
        s = Scene(rt, rs.mesh, "BSP")
        o = s.render_oracle("W7E3", (eye, target, up, constant), 48, 48, (0, 0, 48, 48), 0, 2)
        check((got[0], got[1], o[2]), o, counts=False)
    finally:
        rs.ctx.close()


def test_subdivision_jitter_table(rt):
    # "Project: Utah Teapot BSP" with subdivision_level 3: the kernel takes the
    # 9 stratified samples of the PCG jitter table (jitter.py) per pixel
    from importlib import import_module
    J = import_module("02562_raytracer_amd.jitter")
    rs = rt.RenderState(rt.find_scene("Project: Utah Teapot BSP"), resolution=(200, 120))
    try:
        rs.set_subdivision_level(3)
        rs.update()
        assert rs.uniform.subdivision_level == 3
        rs.render(1)
        got = (rs.frame(), rs.hit_ids(), None)
        eye, target, up, constant = rs.camera.as_args()
        s = Scene(rt, rs.mesh, "BSP")
        o = s.render_oracle("PROJECT", (eye, target, up, constant), 200, 120, (0, 0, 200, 120), 0, 1,
                            jitter=J.jitters_for(120, 3))
        check((got[0], got[1], o[2]), o, counts=False)
        rs.set_subdivision_level(42)
        assert rs.subdivision_level == 10
    finally:
        rs.ctx.close()
