"""MI355X-native (gfx950) hot path of cakarsubasi/02562_raytracer.

The per-pixel BSP/BVH ray-triangle traversal + shading that the reference runs
as WGSL fragment shaders, as hand-written HIP kernels behind a C ABI
(include/rt.h, lib02562rt.so), with the host-side mirror of the reference's
dispatch surface (src/scenes.rs, src/render_state.rs).

The package directory name starts with a digit; import it with
``importlib.import_module("02562_raytracer_amd")``.
"""
from . import _ffi
from ._ffi import MODES, TRAVERSALS, RtError, lib
from .core import BspTree, Bvh, Context, DeviceBuffer, Mesh, load_texture_rgba8, local_tiles, make_uniform
from .render_state import ASSETS, RenderState
from .camera import CameraController
from .scenes import Camera, SceneDescriptor, find_scene, get_scenes

__all__ = ["BspTree", "Bvh", "Camera", "CameraController", "Context", "DeviceBuffer", "Mesh", "RenderState", "RtError",
           "SceneDescriptor", "ASSETS", "MODES", "TRAVERSALS", "find_scene", "get_scenes", "lib", "local_tiles",
           "load_texture_rgba8",
           "make_uniform", "_ffi"]
