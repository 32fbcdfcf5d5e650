"""INTEGRATION.md's call sequence, performed by a C program through include/rt.h
(tests/native/integration_seq.c): it compiles and links against lib02562rt.so on
the CPU, and on the GPU its frame -- `iters` render() calls of one progressive
iteration each -- equals one fused rt_render of `iters` iterations (the Python
binding) and the CPU oracle, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, model
from parity_util import CORNELL_CAM, compare

SRC = os.path.join(ROOT, "tests", "native", "integration_seq.c")
PKG = os.path.join(ROOT, "02562_raytracer_amd")


def build(out_dir):
    exe = os.path.join(out_dir, "integration_seq")
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), SRC, "-o", exe,
                    "-L", PKG, "-l:lib02562rt.so", f"-Wl,-rpath,{PKG}"], check=True, capture_output=True)
    return exe


def test_integration_sequence_compiles_and_links(tmp_path):
    exe = build(str(tmp_path))
    assert os.path.exists(exe)
    # usage error path: no device needed
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
def test_integration_sequence_frame(tmp_path, rt, oracle):
    exe = build(str(tmp_path))
    W, H, IT = 96, 80, 3
    out = str(tmp_path / "frame.bin")
    r = subprocess.run([exe, model("CornellBoxWithBlocks.obj"), str(W), str(H), str(IT), out], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, dtype=np.uint8)
    acc = raw[:W * H * 16].view(np.float32).reshape(H, W, 4)
    ids = raw[W * H * 16:].view(np.uint32).reshape(H, W)
    # the fused launch of the Python binding
    ctx = rt.Context(0)
    try:
        mesh = rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj"))
        ctx.upload_mesh(mesh)
        ctx.upload_bsp(mesh.bsp_tree())
        ctx.set_uniforms(rt.make_uniform(*CORNELL_CAM, W, H))
        a = ctx.alloc(W * H * 16)
        i = ctx.alloc(W * H * 4)
        a.zero()
        ctx.render("W7E3", "BSP", (0, 0, W, H), 0, IT, a.ptr, i.ptr)
        fa, fi = a.to_numpy(np.float32, (H, W, 4)), i.to_numpy(np.uint32, (H, W))
    finally:
        ctx.close()
    assert np.array_equal(ids, fi) and np.array_equal(acc.view(np.uint32), fa.view(np.uint32))
    m = oracle.load_obj(model("CornellBoxWithBlocks.obj"))
    o = oracle.render(oracle.SceneRef(m, oracle.build_bsp(m)), oracle.make_uniform(*CORNELL_CAM, W, H), "W7E3", "BSP",
                      (0, 0, W, H), 0, IT)
    linf, bits, idm = compare((acc, ids, None), o)
    assert idm == 0 and bits == 0, (idm, bits, linf)
