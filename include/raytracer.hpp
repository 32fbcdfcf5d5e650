/* C++ host layer of the drop-in: the reference's Rust host types above its
 * GPU boundary (src/gpu_handles.rs, src/scenes.rs, src/camera.rs,
 * src/bindings/uniform.rs, src/render_state.rs, the progressive loop of
 * src/lib.rs:321-489), restated in C++ over the C ABI of include/rt.h -- the
 * calls a Rust host would make through its extern "C" block.
 *
 * Headless: no window, surface or egui panel.  A RenderState renders into an
 * HBM RGBA32F accumulation buffer (the RenderDestination texture) and hands
 * back the linear accumulation, the primary-hit ids and the sRGB frame.
 * Errors from the C ABI surface as raytracer::Error (code + rt_last_error).
 */
#pragma once

#include <array>
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rt.h"

namespace raytracer {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& what) : std::runtime_error(what), code(code) {}
    int code;
};

/* ---- src/gpu_handles.rs: the device + stream wrapper (GPUHandles::new, self_test) */
class GpuHandles {
public:
    explicit GpuHandles(int device = 0);
    ~GpuHandles();
    GpuHandles(const GpuHandles&) = delete;
    GpuHandles& operator=(const GpuHandles&) = delete;
    rt_ctx* ctx() const { return ctx_; }
    int device() const { return device_; }
    /* gpu_handles.rs:72-90: is there a device to render on? */
    static bool self_test();
    void check(int rc, const char* what) const;

private:
    rt_ctx* ctx_ = nullptr;
    int device_ = 0;
};

/* ---- src/camera.rs */
using Vec3 = std::array<float, 3>;

struct Camera {   /* :13-34 */
    Vec3 eye{2.0f, 1.5f, 2.0f};
    Vec3 target{0.0f, 0.5f, 0.0f};
    Vec3 up{0.0f, 1.0f, 0.0f};
    float aspect = 1.0f;
    float constant = 1.0f;
};

/* winit VirtualKeyCode values the controller reacts to (camera.rs:56-81) */
enum class Key { W, A, S, D, Up, Down, Left, Right, Other };
Key key_from_name(const std::string& name);

class CameraController {   /* :36-112 */
public:
    explicit CameraController(float speed = 0.05f) : speed_(speed) {}   // CAMERA_SPEED, render_state.rs:31
    /* Command::KeyEvent: true when the key is one the controller owns */
    bool handle_camera_commands(Key key, bool pressed);
    /* f32 in cgmath's operation order (normalize = v * (1/|v|)) */
    void update_camera(Camera& camera) const;

private:
    float speed_;
    bool forward_ = false, backward_ = false, left_ = false, right_ = false;
};

/* ---- src/scenes.rs */
enum class VertexType { Split, Combined };
enum class TraverseType { Bsp, Bvh };

struct SceneDescriptor {   /* :20-44 */
    std::string name;
    std::string shader;                            // res/shaders/<file>
    VertexType vertex_type = VertexType::Split;
    std::optional<std::string> model;              // res/models/<file>
    std::optional<std::string> background_hdri;    // res/textures/<file>
    Camera camera;
    std::pair<uint32_t, uint32_t> res{512, 512};
    TraverseType traverse_type = TraverseType::Bsp;
    /* the HIP kernel that restates the shader; nullopt = a worksheet shader
     * outside the hot path */
    std::optional<rt_mode> mode() const;
};

std::vector<SceneDescriptor> get_scenes();            /* :46-488, the 44 scenes in order */
const SceneDescriptor& find_scene(const std::string& name);

/* ---- src/bindings/uniform.rs */
constexpr uint32_t MAX_SUBDIVISION = 10;
/* compute_jitters (:254-277): PCG32 Lcg64Xsh32::new(0, 0), rand's f64 gen_range */
std::vector<std::array<float, 2>> compute_jitters(double pixel_size, uint32_t subdivs);
rt_uniform make_uniform(const Camera& cam, uint32_t width, uint32_t height, uint32_t selection1 = 0,
                        uint32_t subdivision_level = 1, uint32_t iteration = 0);

/* PCG32 (XSH RR), as rand_pcg 0.3.1's Lcg64Xsh32 */
class Lcg64Xsh32 {
public:
    Lcg64Xsh32(uint64_t state, uint64_t stream);
    uint32_t next_u32();
    uint64_t next_u64();
    double gen_unit_f64();   // gen_range(0.0..1.0)

private:
    uint64_t state_, increment_;
};

/* ---- src/mesh.rs + src/data_structures (host builders behind the C ABI) */
class Mesh {
public:
    static Mesh load(const std::string& path);                   /* Mesh::from_obj */
    static Mesh synth_bunny(uint32_t ntris = 69451, uint32_t seed = 0x0B0B);
    Mesh(Mesh&& o) noexcept : m_(o.m_) { o.m_ = nullptr; }
    ~Mesh();
    rt_mesh_host* get() const { return m_; }
    uint32_t ntris() const;

private:
    explicit Mesh(rt_mesh_host* m) : m_(m) {}
    rt_mesh_host* m_;
};

/* ---- src/render_state.rs + src/lib.rs rendering_thread */
struct RenderOptions {
    std::string models_dir;                               // where scene models live
    std::optional<std::pair<uint32_t, uint32_t>> resolution;   // override SceneDescriptor.res
    bool bunny_standin = true;                            // bunny.obj is absent from the reference
    bool device_build = false;                            // build BSP / HLBVH on the GPU
    Vec3 environment{1.0f, 1.0f, 1.0f};                   // W9 escape radiance without a texture
};

class RenderState {
public:
    RenderState(GpuHandles& gpu, const SceneDescriptor& scene, RenderOptions opts);
    ~RenderState();
    RenderState(const RenderState&) = delete;
    RenderState& operator=(const RenderState&) = delete;

    void load_scene(const SceneDescriptor& scene);   /* :314-334 (+ iteration reset, lib.rs:464-469) */
    void update();                                   /* :467-481 */
    void render(uint32_t spp = 1);                   /* :483-561, spp progressive iterations */
    bool step();                                     /* one pass of rendering_thread, lib.rs:331-363 */

    bool input_alt(Key key, bool pressed);           /* :462-465 */
    void update_camera_constant(float constant);     /* :591-593 */
    void set_samples(uint32_t samples, bool enabled);   /* Command::SetSamples, lib.rs:472-479 */
    void set_subdivision_level(uint32_t level);      /* uniform.rs:122-129 */
    void set_selection1(uint32_t shader);            /* Command::SetSphereMaterial, lib.rs:405-409 */
    /* the scene's background_hdri, decoded by the caller (render_state.rs:191-206):
     * RGBA8 equirectangular texels, or nullptr for the constant environment */
    void set_environment_map(const uint8_t* rgba8, uint32_t width, uint32_t height);
    void reset_iteration();
    /* Framebuffer tiling across the GPUs of a node: this state
     * renders only rank `rank`'s interleaved 8x8 tiles of every frame
     * (rt_render_tiles, into a packed accumulation kept across iterations) and
     * gathers all ranks' tiles into rank 0's frame over RCCL (rt_comm_init with
     * the communicator id rank 0 made, rt_gather_tiles).  Collective: every rank
     * calls it, then render()/step() in lockstep; frame()/hit_ids() are rank 0's. */
    void set_tiling(uint32_t nranks, uint32_t rank, const uint8_t comm_id[RT_COMM_ID_BYTES]);

    std::vector<float> frame() const;        /* linear RGBA32F accumulation, H x W x 4 */
    std::vector<uint32_t> hit_ids() const;   /* primary-hit triangle ids, H x W */
    std::vector<uint8_t> frame_rgba8() const;   /* the sRGB surface frame, H x W x 4 */

    uint32_t width() const { return width_; }
    uint32_t height() const { return height_; }
    uint32_t iteration() const { return iteration_; }
    const Camera& camera() const { return camera_; }
    const SceneDescriptor& scene() const { return scene_; }
    rt_ray_counts last_counts() const;

private:
    void setup_rendering(const SceneDescriptor& scene);   /* :161-265 */
    void release();

    GpuHandles& gpu_;
    RenderOptions opts_;
    SceneDescriptor scene_;
    Camera camera_;
    CameraController controller_;
    rt_mode mode_ = RT_MODE_W7E3;
    rt_traverse trav_ = RT_TRAVERSE_BSP;
    uint32_t width_ = 0, height_ = 0;
    uint32_t iteration_ = 0, max_iterations_ = 2, subdivision_ = 1, selection1_ = 0;
    bool progressive_ = true;
    void* accum_ = nullptr;
    void* ids_ = nullptr;
    void alloc_tiles();
    uint32_t nranks_ = 1, rank_ = 0;   // set_tiling
    bool tiled_ = false;
    void* tile_accum_ = nullptr;       // this rank's packed tiles (rt_render_tiles)
    void* tile_ids_ = nullptr;
};

}  // namespace raytracer
