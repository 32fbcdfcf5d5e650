"""SceneDescriptor table: mirror of src/scenes.rs (get_scenes, :46-488).

Each descriptor names the scene shader; `mode` maps it to the HIP kernel that
restates that shader (None = a course-exercise shader outside the hot path,
SURVEY.md section 2).  Paths are relative to the model directory
(assets/models in this repo; res/models in the reference).
"""
from dataclasses import dataclass, field, replace
from typing import Optional, Tuple

# shader file -> rt_mode name (include/rt.h)
SHADER_MODES = {
    "w1e6.wgsl": "W1E6",
    "w6e1.wgsl": "W6E1",
    "project.wgsl": "PROJECT",
    "w7e3.wgsl": "W7E3",
    "w9e1.wgsl": "W9E1",
    "w8e1.wgsl": "W8E1",
    "w8e2.wgsl": "W8E2",
    "w8e3.wgsl": "W8E3",
    "w9e2.wgsl": "W9E2",
    "w6e2.wgsl": "W6E2",
    "w7e1.wgsl": "W7E1",
    "w7e2.wgsl": "W7E2",
    "w6e3.wgsl": "W6E3",
    "w9e3.wgsl": "W9E3",
}


@dataclass(frozen=True)
class Camera:
    """src/camera.rs:13-19 (aspect comes from the frame, render_state.rs:468)."""
    eye: Tuple[float, float, float] = (2.0, 1.5, 2.0)
    target: Tuple[float, float, float] = (0.0, 0.5, 0.0)
    up: Tuple[float, float, float] = (0.0, 1.0, 0.0)
    constant: float = 1.0


@dataclass(frozen=True)
class SceneDescriptor:
    """src/scenes.rs:19-29."""
    name: str
    shader: str
    model: Optional[str] = None
    camera: Camera = field(default_factory=Camera)
    res: Tuple[int, int] = (512, 512)
    vertex_type: str = "Split"          # Split | Combined (storage layout only)
    traverse_type: str = "BSP"          # BSP | BVH
    background_hdri: Optional[str] = None

    @property
    def mode(self):
        return SHADER_MODES.get(self.shader)

    def with_(self, **kw):
        return replace(self, **kw)


BASIC = Camera((2.0, 1.5, 2.0), (0.0, 0.5, 0.0), (0.0, 1.0, 0.0), 1.0)           # scenes.rs:47-53
TEAPOT = Camera((0.15, 1.5, 10.0), (0.15, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5)       # :55-61
CORNELL = Camera((277.0, 275.0, -570.0), (277.0, 275.0, 0.0), (0.0, 1.0, 0.0), 1.0)   # :63-69
BUNNY = Camera((-0.02, 0.11, 0.6), (-0.02, 0.11, 0.0), (0.0, 1.0, 0.0), 3.5)     # :71-77
DRAGON = Camera((-0.02, 0.11, 0.6), (-0.02, 0.11, 0.0), (0.0, 1.0, 0.0), 3.5)    # :79-85

CAMPUS = "luxo_pxr_campus.jpg"
CAMPUS_HDR = "luxo_pxr_campus.hdr.png"


def get_scenes():
    """The reference's 44 scenes in order (src/scenes.rs:98-487)."""
    S = SceneDescriptor
    sc = []
    for w, e in [(1, 1), (1, 2), (1, 3), (1, 4), (1, 5), (1, 6), (2, 1), (2, 2), (2, 3), (2, 4), (2, 5),
                 (3, 1), (3, 2), (3, 3), (3, 4)]:
        sc.append(S(f"W{w} E{e}", f"w{w}e{e}.wgsl", None, BASIC, (512, 512)))
    sc += [
        S("W5 E2 Teapot", "w5e2.wgsl", "teapot.obj", TEAPOT, (800, 450)),
        S("W5 E3 Teapot", "w5e3.wgsl", "teapot.obj", TEAPOT, (800, 450)),
        S("W5 E4 Cornell Box", "w5e4.wgsl", "CornellBoxWithBlocks.obj", CORNELL, (512, 512)),
        S("W5 E5 Cornell Box", "w5e5.wgsl", "CornellBoxWithBlocks.obj", CORNELL, (512, 512)),
        S("W6 E1 Teapot", "w6e1.wgsl", "teapot.obj", TEAPOT, (800, 450)),
        S("W6 E1 Bunny", "w6e1.wgsl", "bunny.obj", BUNNY, (512, 512)),
        S("W6 E1 Dragon", "w6e1.wgsl", "dragon.obj", DRAGON, (800, 450)),
        S("W6 E2 Cornell Box", "w6e2.wgsl", "CornellBoxWithBlocks.obj", CORNELL, (512, 512), "Combined"),
        S("W6 E3 Cornell Box", "w6e3.wgsl", "CornellBox.obj", CORNELL, (512, 512), "Combined"),
        S("W7 E1 Cornell Box", "w7e1.wgsl", "CornellBoxWithBlocks.obj", CORNELL, (512, 512), "Combined"),
        S("W7 E2 Cornell Box", "w7e2.wgsl", "CornellBoxWithBlocks.obj", CORNELL, (512, 512), "Combined"),
        S("W7 E3 Cornell Box", "w7e3.wgsl", "CornellBoxWithBlocks.obj", CORNELL, (512, 512), "Combined"),
        S("W8 E1 Cornell Box Balls", "w8e1.wgsl", "CornellBox.obj", CORNELL, (512, 512), "Combined"),
        S("W8 E2 Cornell Box Balls", "w8e2.wgsl", "CornellBox.obj", CORNELL, (512, 512), "Combined"),
        S("W8 E3 Absorption", "w8e3.wgsl", "CornellBox.obj", CORNELL, (512, 512), "Combined"),
        S("W9 E1 Teapot", "w9e1.wgsl", "teapot.obj", TEAPOT, (800, 450), "Combined", "BSP", CAMPUS),
        S("W9 E1 Bunny", "w9e1.wgsl", "bunny.obj", BUNNY, (512, 512), "Combined", "BSP", CAMPUS),
        S("W9 E2 Teapot", "w9e2.wgsl", "teapot.obj", TEAPOT, (800, 450), "Combined", "BSP", CAMPUS_HDR),
        S("W9 E2 Bunny", "w9e2.wgsl", "bunny.obj", BUNNY, (512, 512), "Combined", "BSP", CAMPUS_HDR),
        S("W9 E3 Teapot", "w9e3.wgsl", "teapot.obj", TEAPOT, (800, 450), "Combined", "BSP", CAMPUS),
        S("Project: Quad", "project.wgsl", "plane.obj", BASIC, (512, 512), "Combined", "BVH"),
        S("Project: Three Quads", "project.wgsl", "test_object.obj", BASIC, (512, 512), "Combined", "BVH"),
        S("Project: Cornell Box", "project.wgsl", "CornellBoxWithBlocks.obj", CORNELL, (512, 512), "Combined", "BVH"),
        S("Project: Utah Teapot", "project.wgsl", "teapot.obj", TEAPOT, (800, 450), "Combined", "BVH"),
        S("Project: Utah Teapot BSP", "project.wgsl", "teapot.obj", TEAPOT, (800, 450), "Combined", "BSP"),
        S("Project: Bunny", "project.wgsl", "bunny.obj", BUNNY, (512, 512), "Combined", "BVH"),
        S("Project: Bunny BSP", "project.wgsl", "bunny.obj", BUNNY, (512, 512), "Combined", "BSP"),
        S("Project: Dragon", "project.wgsl", "dragon.obj", DRAGON, (800, 450), "Combined", "BVH"),
        S("Project: Dragon BSP", "project.wgsl", "dragon.obj", DRAGON, (800, 450), "Combined", "BSP"),
    ]
    return sc


def find_scene(name):
    for s in get_scenes():
        if s.name == name:
            return s
    raise KeyError(name)
