"""Headless RenderState: mirror of src/render_state.rs (setup_rendering
:161-265, update :467-481, render :483-561) and of the progressive loop of
src/lib.rs:321-363, on top of the C ABI.

Differences from the windowed reference, all deliberate:
  * no window/surface: aspect = W/H of SceneDescriptor.res (the reference
    uses the window's inner size, render_state.rs:563-566);
  * the accumulation "texture" is an HBM float4 array (linear RGBA32F), and
    the display transform pow(., 1.5) is left to the caller;
  * the W9E1 equirectangular hdri0 is the scene's background_hdri texture
    when the file is in assets/textures (decoded with PIL, sampled as
    include/rt_detmath.h pins it), else a constant environment colour;
  * a missing bunny.obj can be replaced by the deterministic stand-in
    (bunny_standin=True), since the reference checkout lacks it.
"""
import os

import numpy as np

from . import _ffi as F
from .camera import Camera, CameraController
from .jitter import MAX_SUBDIVISION, jitters_for
from .core import BspTree, Bvh, Context, Mesh, make_uniform

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(REPO, "assets", "models")


class RenderState:
    def __init__(self, scene, device=0, ctx=None, models_dir=ASSETS, bunny_standin=True, selection1=0,
                 env=(1.0, 1.0, 1.0), resolution=None, device_build=False):
        self.ctx = ctx if ctx is not None else Context(device)
        self.models_dir = models_dir
        self.bunny_standin = bunny_standin
        self.selection1 = selection1
        self.env = env
        self.resolution = resolution
        self.device_build = device_build   # build the BSP / HLBVH on the GPU (same arrays)
        self.progressive = True
        self.iteration = 0
        self.max_iterations = 2   # Uniform::max_iterations, SetSamples (lib.rs:472-479)
        self.subdivision_level = 1   # Uniform.subdivision_level (uniform.rs:122-129)
        self.camera_controller = CameraController()
        self.setup_rendering(scene)

    def _background(self, scene):
        """render_state.rs:191-206: the scene's background_hdri, if present."""
        if not getattr(scene, "background_hdri", None):
            return None
        path = os.path.join(REPO, "assets", "textures", os.path.basename(scene.background_hdri))
        if not os.path.exists(path):
            return None
        from .core import load_texture_rgba8
        return load_texture_rgba8(path)

    # render_state.rs:161-265
    def setup_rendering(self, scene):
        if scene.mode is None:
            raise F.RtError(F.RT_E_UNSUPPORTED, f"{scene.shader} is outside the hot path (SURVEY.md section 2)")
        self.scene = scene
        self.camera = Camera.from_tuple(scene.camera)
        self.mode = scene.mode
        self.width, self.height = self.resolution or scene.res
        self.mesh = self.bsp = self.bvh = None
        if scene.mode == "W1E6":
            self.trav = "NONE"
        else:
            self.trav = scene.traverse_type
            self.mesh = self._load_model(scene.model)
            self.ctx.upload_mesh(self.mesh)
            if self.trav == "BSP":
                if self.device_build:
                    self.ctx.build_bsp_device(20, 4)
                else:
                    self.bsp = self.mesh.bsp_tree()   # Mesh::bsp_tree, mesh.rs:229-231 (depth 20, leaf 4)
                    self.ctx.upload_bsp(self.bsp)
            else:
                if self.device_build:
                    self.ctx.build_bvh_device(4)
                else:
                    self.bvh = self.mesh.bvh()        # Mesh::bvh, mesh.rs:233-239 (leaf 4)
                    self.ctx.upload_bvh(self.bvh)
        self.ctx.set_environment(self.env)
        self.ctx.set_environment_map(None)
        tex = self._background(scene)
        if tex is not None:
            self.ctx.set_environment_map(tex)
        npx = self.width * self.height
        self.accum = self.ctx.alloc(npx * 16)
        self.accum.zero()
        self.ids = self.ctx.alloc(npx * 4)
        self.iteration = 0
        self.update()

    def _load_model(self, model):
        path = os.path.join(self.models_dir, model)
        if not os.path.exists(path) and model == "bunny.obj" and self.bunny_standin:
            return Mesh.synth_bunny()
        return Mesh.from_obj(path)

    def load_scene(self, scene):
        """RenderState::load_scene (render_state.rs:314-334): full rebuild;
        the iteration restarts (Command::LoadScene, lib.rs:464-469)."""
        self.iteration = 0
        self.setup_rendering(scene)

    # render_state.rs:467-481: the controller moves the camera, then the uniform follows
    def update(self):
        self.camera.aspect = float(np.float32(self.width) / np.float32(self.height))
        self.camera_controller.update_camera(self.camera)
        eye, target, up, constant = self.camera.as_args()
        self.uniform = make_uniform(eye, target, up, constant, self.width, self.height,
                                    selection1=self.selection1, iteration=self.iteration,
                                    subdiv=self.subdivision_level)
        # UniformGpu::update_buffer (uniform.rs:163-175): the jitter table with the uniforms
        self.ctx.set_uniforms(self.uniform, jitters_for(self.height, self.subdivision_level))

    def set_subdivision_level(self, level):
        """Uniform::update_subdivision_level (uniform.rs:122-129): clamped to 10;
        W6E1/PROJECT take level^2 stratified samples per pixel."""
        self.subdivision_level = min(int(level), MAX_SUBDIVISION)

    def input(self, key, pressed=True):
        """RenderState::input_alt (render_state.rs:462-465): a key event for the
        camera controller; takes effect at the next update()."""
        return self.camera_controller.handle_camera_commands(key, pressed)

    def set_camera_constant(self, constant):
        """Command::SetCameraConstant (lib.rs:401-403)."""
        self.camera.constant = float(constant)

    def set_samples(self, samples, enabled):
        """Command::SetSamples (lib.rs:472-479): progressive rendering up to
        `samples` iterations, or (disabled) a frame per step at a fixed iteration."""
        self.progressive = bool(enabled)
        self.max_iterations = int(samples) if enabled else 2

    def step(self):
        """One pass of rendering_thread (lib.rs:331-363): render while
        progressive and below max_iterations (or always when not progressive),
        advance the iteration when progressive, then update().  Returns whether
        a frame was rendered."""
        if self.progressive and self.iteration >= self.max_iterations:
            return False
        self.render(1)
        return True

    # render_state.rs:483-561 (+ lib.rs:349-354 iteration advance)
    def render(self, spp=1, counts=False):
        first = self.iteration   # not progressive: the iteration stays (lib.rs:350-355)
        c = self.ctx.render(self.mode, self.trav, (0, 0, self.width, self.height), first, spp, self.accum.ptr,
                            self.ids.ptr, counts=counts)
        if self.progressive and self.mode in F.PATH_MODES:
            self.iteration += spp
        self.update()
        return c

    def reset_iteration(self):
        self.iteration = 0
        self.update()

    def frame(self):
        """Linear accumulation [H, W, 4] float32 (the RenderDestination texture)."""
        return self.accum.to_numpy(np.float32, (self.height, self.width, 4))

    def hit_ids(self):
        return self.ids.to_numpy(np.uint32, (self.height, self.width))

    def frame_rgba8(self):
        """The displayed frame as the sRGB surface holds it: uint8 [H, W, 4]
        (rt_frame_rgba8, on the device)."""
        npx = self.width * self.height
        out = self.ctx.alloc(npx * 4)
        self.ctx.frame_rgba8(self.accum.ptr, npx, out.ptr)
        img = out.to_numpy(np.uint8, (self.height, self.width, 4))
        out.free()
        return img

    def save_png(self, path):
        """Write the displayed frame (PIL)."""
        from PIL import Image
        Image.fromarray(self.frame_rgba8(), "RGBA").save(path)

    @staticmethod
    def display(accum):
        """fs_main's frame output: saturate(pow(accum, 1.5)) (w7e3.wgsl:265)."""
        return np.clip(np.power(np.maximum(accum[..., :3], 0), 1.5), 0, 1)
