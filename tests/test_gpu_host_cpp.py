"""The C++ host layer on the GPU: bin/rt_render (C++ RenderState over the C
ABI) renders the reference's scenes, and its frames equal the Python
RenderState's and the CPU oracle's bit for bit -- the two host mirrors drive
the same kernels with the same uniforms, jitter tables and iteration order."""
import json
import os
import subprocess

import numpy as np
import pytest

from parity_util import Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "02562_raytracer_amd", "bin", "rt_render")


def cpp_render(tmp_path, scene, W, H, *args):
    out = str(tmp_path / "frame")
    r = subprocess.run([BIN, "--scene", scene, "--res", f"{W}x{H}", "--out", out, *args], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    acc = np.fromfile(out + ".accum.f32", np.float32).reshape(H, W, 4)
    ids = np.fromfile(out + ".ids.u32", np.uint32).reshape(H, W)
    rgba = np.fromfile(out + ".rgba8", np.uint8).reshape(H, W, 4)
    return acc, ids, rgba, info


def test_cornell_progressive_samples(rt, tmp_path):
    acc, ids, rgba, info = cpp_render(tmp_path, "W7 E3 Cornell Box", 64, 48, "--samples", "3")
    assert info["iteration"] == 3 and info["frames"] == 3 and info["mode"] == "W7E3"
    rs = rt.RenderState(rt.find_scene("W7 E3 Cornell Box"), resolution=(64, 48))
    try:
        rs.set_samples(3, True)
        while rs.step():
            pass
        assert np.array_equal(acc.view(np.uint32), rs.frame().view(np.uint32))
        assert np.array_equal(ids, rs.hit_ids())
        assert np.array_equal(rgba, rs.frame_rgba8())
        s = Scene(rt, rs.mesh, "BSP")
        c = rt.find_scene("W7 E3 Cornell Box").camera
        o = s.render_oracle("W7E3", (c.eye, c.target, c.up, c.constant), 64, 48, (0, 0, 64, 48), 0, 3)
        check((acc, ids, o[2]), o, counts=False)
    finally:
        rs.ctx.close()


def test_keys_move_the_camera_like_python(rt, tmp_path):
    acc, ids, _, info = cpp_render(tmp_path, "W8 E2 Cornell Box Balls", 48, 48, "--keys", "A,W", "--updates", "3",
                                   "--spp", "2")
    rs = rt.RenderState(rt.find_scene("W8 E2 Cornell Box Balls"), resolution=(48, 48))
    try:
        rs.input("A", True)
        rs.input("W", True)
        for _ in range(3):
            rs.update()
        eye = [float.fromhex(x) for x in info["camera"]["eye"]]
        rs.render(2)   # rendered before render's own update() moved the camera again
        assert np.array_equal(acc.view(np.uint32), rs.frame().view(np.uint32))
        assert np.array_equal(ids, rs.hit_ids())
        assert eye != list(rt.find_scene("W8 E2 Cornell Box Balls").camera.eye)
    finally:
        rs.ctx.close()


def test_w9e1_teapot_with_campus_texture(rt, tmp_path):
    # the C++ host takes the decoded background_hdri texels (the reference decodes
    # with the `image` crate; both mirrors here use the same PIL decode)
    path = os.path.join(ROOT, "assets", "textures", "luxo_pxr_campus.jpg")
    if not os.path.exists(path):
        pytest.skip("texture asset missing")
    tex = rt.load_texture_rgba8(path)
    raw = tmp_path / "env.rgba"
    tex.tofile(raw)
    acc, ids, _, _ = cpp_render(tmp_path, "W9 E1 Teapot", 200, 112, "--spp", "2", "--env-rgba", str(raw),
                                "--env-size", f"{tex.shape[1]}x{tex.shape[0]}")
    rs = rt.RenderState(rt.find_scene("W9 E1 Teapot"), resolution=(200, 112))
    try:
        rs.render(2)
        assert np.array_equal(acc.view(np.uint32), rs.frame().view(np.uint32))
        assert np.array_equal(ids, rs.hit_ids())
    finally:
        rs.ctx.close()


def test_project_subdivision_and_device_build(rt, tmp_path):
    acc, ids, _, _ = cpp_render(tmp_path, "Project: Bunny", 96, 96, "--subdiv", "2", "--device-build")
    rs = rt.RenderState(rt.find_scene("Project: Bunny"), resolution=(96, 96), device_build=True)
    try:
        rs.set_subdivision_level(2)
        rs.update()
        rs.render(1)
        assert np.array_equal(acc.view(np.uint32), rs.frame().view(np.uint32))
        assert np.array_equal(ids, rs.hit_ids())
    finally:
        rs.ctx.close()


@pytest.mark.parametrize("scene,args", [("W7 E3 Cornell Box", ("--samples", "3")), ("W6 E1 Teapot", ())])
def test_tiled_one_rank_communicator_equals_plain_frame(rt, tmp_path, scene, args):
    # rt_render --nranks 1 --rank 0 --comm-file: the C++ RenderState renders its
    # tiles (rt_render_tiles, packed accumulation across the progressive
    # iterations) and gathers them through the library's RCCL communicator
    # (rt_comm_unique_id published in a file, rt_comm_init, rt_gather_tiles):
    # the frame equals the plain region render's bit for bit
    plain = cpp_render(tmp_path, scene, 72, 40, *args)
    # a file left by an earlier launch (another token) is replaced, never used
    (tmp_path / "comm.id").write_bytes(b"RTCOMMID old-launch\n" + bytes(128))
    tiled = cpp_render(tmp_path, scene, 72, 40, *args, "--nranks", "1", "--rank", "0", "--comm-file",
                       str(tmp_path / "comm.id"), "--comm-token", "job-42")
    blob = (tmp_path / "comm.id").read_bytes()
    assert blob.startswith(b"RTCOMMID job-42\n") and len(blob) == len(b"RTCOMMID job-42\n") + 128
    assert blob[-128:] != bytes(128)
    for a, b in zip(plain[:3], tiled[:3]):
        assert np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                              b.view(np.uint32) if b.dtype == np.float32 else b)
    assert plain[3]["iteration"] == tiled[3]["iteration"]
