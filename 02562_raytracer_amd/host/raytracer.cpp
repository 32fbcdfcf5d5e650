// C++ host layer (include/raytracer.hpp) over the C ABI of include/rt.h: the
// reference's Rust host types restated for a C++ caller.  Every GPU action
// goes through rt_* entry points, exactly as the Rust binding of
// INTEGRATION.md would make them.
#include "raytracer.hpp"

#include <cmath>
#include <cstring>
#include <sys/stat.h>

namespace raytracer {

// ------------------------------------------------------------------ GpuHandles
GpuHandles::GpuHandles(int device) : device_(device)
{
    const int rc = rt_create(device, &ctx_);
    if (rc != RT_OK) throw Error(rc, "GPUHandles::new: no usable HIP device " + std::to_string(device));
}

GpuHandles::~GpuHandles()
{
    if (ctx_) rt_destroy(ctx_);
}

bool GpuHandles::self_test()
{
    int n = 0;
    return rt_device_count(&n) == RT_OK && n > 0;
}

void GpuHandles::check(int rc, const char* what) const
{
    if (rc != RT_OK) throw Error(rc, std::string(what) + ": " + (ctx_ ? rt_last_error(ctx_) : "no context"));
}

// ------------------------------------------------------------------ camera.rs
Key key_from_name(const std::string& n)
{
    if (n == "W") return Key::W;
    if (n == "A") return Key::A;
    if (n == "S") return Key::S;
    if (n == "D") return Key::D;
    if (n == "Up") return Key::Up;
    if (n == "Down") return Key::Down;
    if (n == "Left") return Key::Left;
    if (n == "Right") return Key::Right;
    return Key::Other;
}

bool CameraController::handle_camera_commands(Key key, bool pressed)
{
    switch (key) {
    case Key::W:
    case Key::Up: forward_ = pressed; return true;
    case Key::A:
    case Key::Left: left_ = pressed; return true;
    case Key::S:
    case Key::Down: backward_ = pressed; return true;
    case Key::D:
    case Key::Right: right_ = pressed; return true;
    default: return false;
    }
}

namespace {
// cgmath's f32 vector operations, in its order of evaluation
inline Vec3 vsub(const Vec3& a, const Vec3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
inline Vec3 vadd(const Vec3& a, const Vec3& b) { return {a[0] + b[0], a[1] + b[1], a[2] + b[2]}; }
inline Vec3 vmul(const Vec3& a, float s) { return {a[0] * s, a[1] * s, a[2] * s}; }
inline float vdot(const Vec3& a, const Vec3& b)
{
    const float x = a[0] * b[0], y = a[1] * b[1], z = a[2] * b[2];
    return (x + y) + z;
}
inline float vmag(const Vec3& a) { return std::sqrt(vdot(a, a)); }
inline Vec3 vnormalize(const Vec3& a) { return vmul(a, 1.0f / vmag(a)); }
inline Vec3 vcross(const Vec3& a, const Vec3& b)
{
    return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
}  // namespace

void CameraController::update_camera(Camera& c) const
{
    const float s = speed_;
    Vec3 forward = vsub(c.target, c.eye);
    const Vec3 forward_norm = vnormalize(forward);
    float forward_mag = vmag(forward);
    if (forward_ && forward_mag > s) c.eye = vadd(c.eye, vmul(forward_norm, s));
    if (backward_) c.eye = vsub(c.eye, vmul(forward_norm, s));
    const Vec3 right = vcross(forward_norm, c.up);
    forward = vsub(c.target, c.eye);
    forward_mag = vmag(forward);
    if (right_) c.eye = vsub(c.target, vmul(vnormalize(vadd(forward, vmul(right, s))), forward_mag));
    if (left_) c.eye = vsub(c.target, vmul(vnormalize(vsub(forward, vmul(right, s))), forward_mag));
}

// ------------------------------------------------------------------ scenes.rs
std::optional<rt_mode> SceneDescriptor::mode() const
{
    if (shader == "w1e6.wgsl") return RT_MODE_W1E6;
    if (shader == "w6e1.wgsl") return RT_MODE_W6E1;
    if (shader == "project.wgsl") return RT_MODE_PROJECT;
    if (shader == "w7e3.wgsl") return RT_MODE_W7E3;
    if (shader == "w9e1.wgsl") return RT_MODE_W9E1;
    if (shader == "w8e1.wgsl") return RT_MODE_W8E1;
    if (shader == "w8e2.wgsl") return RT_MODE_W8E2;
    if (shader == "w8e3.wgsl") return RT_MODE_W8E3;
    if (shader == "w9e2.wgsl") return RT_MODE_W9E2;
    if (shader == "w6e2.wgsl") return RT_MODE_W6E2;
    if (shader == "w7e1.wgsl") return RT_MODE_W7E1;
    if (shader == "w7e2.wgsl") return RT_MODE_W7E2;
    if (shader == "w6e3.wgsl") return RT_MODE_W6E3;
    if (shader == "w9e3.wgsl") return RT_MODE_W9E3;
    return std::nullopt;
}

std::vector<SceneDescriptor> get_scenes()
{
    // cameras, scenes.rs:47-85 (aspect comes from the frame)
    auto cam = [](Vec3 e, Vec3 t, Vec3 u, float k) {
        Camera c;
        c.eye = e;
        c.target = t;
        c.up = u;
        c.constant = k;
        return c;
    };
    const Camera basic = cam({2.0f, 1.5f, 2.0f}, {0.0f, 0.5f, 0.0f}, {0.0f, 1.0f, 0.0f}, 1.0f);
    const Camera teapot = cam({0.15f, 1.5f, 10.0f}, {0.15f, 1.5f, 0.0f}, {0.0f, 1.0f, 0.0f}, 2.5f);
    const Camera cornell = cam({277.0f, 275.0f, -570.0f}, {277.0f, 275.0f, 0.0f}, {0.0f, 1.0f, 0.0f}, 1.0f);
    const Camera bunny = cam({-0.02f, 0.11f, 0.6f}, {-0.02f, 0.11f, 0.0f}, {0.0f, 1.0f, 0.0f}, 3.5f);
    const Camera dragon = bunny;   // scenes.rs:79-85 uses the bunny framing
    const std::string campus = "luxo_pxr_campus.jpg", campus_hdr = "luxo_pxr_campus.hdr.png";
    const auto C = VertexType::Combined, Sp = VertexType::Split;
    const auto BSP = TraverseType::Bsp, BVH = TraverseType::Bvh;

    std::vector<SceneDescriptor> v;
    auto S = [&](std::string name, std::string shader, std::optional<std::string> model, const Camera& c,
                 uint32_t w, uint32_t h, VertexType vt = VertexType::Split, TraverseType tt = TraverseType::Bsp,
                 std::optional<std::string> hdri = std::nullopt) {
        SceneDescriptor d;
        d.name = std::move(name);
        d.shader = std::move(shader);
        d.model = std::move(model);
        d.camera = c;
        d.res = {w, h};
        d.vertex_type = vt;
        d.traverse_type = tt;
        d.background_hdri = std::move(hdri);
        v.push_back(std::move(d));
    };
    const int we[15][2] = {{1, 1}, {1, 2}, {1, 3}, {1, 4}, {1, 5}, {1, 6}, {2, 1}, {2, 2},
                           {2, 3}, {2, 4}, {2, 5}, {3, 1}, {3, 2}, {3, 3}, {3, 4}};
    for (const auto& p : we)
        S("W" + std::to_string(p[0]) + " E" + std::to_string(p[1]),
          "w" + std::to_string(p[0]) + "e" + std::to_string(p[1]) + ".wgsl", std::nullopt, basic, 512, 512);
    S("W5 E2 Teapot", "w5e2.wgsl", "teapot.obj", teapot, 800, 450);
    S("W5 E3 Teapot", "w5e3.wgsl", "teapot.obj", teapot, 800, 450);
    S("W5 E4 Cornell Box", "w5e4.wgsl", "CornellBoxWithBlocks.obj", cornell, 512, 512);
    S("W5 E5 Cornell Box", "w5e5.wgsl", "CornellBoxWithBlocks.obj", cornell, 512, 512);
    S("W6 E1 Teapot", "w6e1.wgsl", "teapot.obj", teapot, 800, 450);
    S("W6 E1 Bunny", "w6e1.wgsl", "bunny.obj", bunny, 512, 512);
    S("W6 E1 Dragon", "w6e1.wgsl", "dragon.obj", dragon, 800, 450);
    S("W6 E2 Cornell Box", "w6e2.wgsl", "CornellBoxWithBlocks.obj", cornell, 512, 512, C);
    S("W6 E3 Cornell Box", "w6e3.wgsl", "CornellBox.obj", cornell, 512, 512, C);
    S("W7 E1 Cornell Box", "w7e1.wgsl", "CornellBoxWithBlocks.obj", cornell, 512, 512, C);
    S("W7 E2 Cornell Box", "w7e2.wgsl", "CornellBoxWithBlocks.obj", cornell, 512, 512, C);
    S("W7 E3 Cornell Box", "w7e3.wgsl", "CornellBoxWithBlocks.obj", cornell, 512, 512, C);
    S("W8 E1 Cornell Box Balls", "w8e1.wgsl", "CornellBox.obj", cornell, 512, 512, C);
    S("W8 E2 Cornell Box Balls", "w8e2.wgsl", "CornellBox.obj", cornell, 512, 512, C);
    S("W8 E3 Absorption", "w8e3.wgsl", "CornellBox.obj", cornell, 512, 512, C);
    S("W9 E1 Teapot", "w9e1.wgsl", "teapot.obj", teapot, 800, 450, C, BSP, campus);
    S("W9 E1 Bunny", "w9e1.wgsl", "bunny.obj", bunny, 512, 512, C, BSP, campus);
    S("W9 E2 Teapot", "w9e2.wgsl", "teapot.obj", teapot, 800, 450, C, BSP, campus_hdr);
    S("W9 E2 Bunny", "w9e2.wgsl", "bunny.obj", bunny, 512, 512, C, BSP, campus_hdr);
    S("W9 E3 Teapot", "w9e3.wgsl", "teapot.obj", teapot, 800, 450, C, BSP, campus);
    S("Project: Quad", "project.wgsl", "plane.obj", basic, 512, 512, C, BVH);
    S("Project: Three Quads", "project.wgsl", "test_object.obj", basic, 512, 512, C, BVH);
    S("Project: Cornell Box", "project.wgsl", "CornellBoxWithBlocks.obj", cornell, 512, 512, C, BVH);
    S("Project: Utah Teapot", "project.wgsl", "teapot.obj", teapot, 800, 450, C, BVH);
    S("Project: Utah Teapot BSP", "project.wgsl", "teapot.obj", teapot, 800, 450, C, BSP);
    S("Project: Bunny", "project.wgsl", "bunny.obj", bunny, 512, 512, C, BVH);
    S("Project: Bunny BSP", "project.wgsl", "bunny.obj", bunny, 512, 512, C, BSP);
    S("Project: Dragon", "project.wgsl", "dragon.obj", dragon, 800, 450, C, BVH);
    S("Project: Dragon BSP", "project.wgsl", "dragon.obj", dragon, 800, 450, C, BSP);
    (void)Sp;
    return v;
}

const SceneDescriptor& find_scene(const std::string& name)
{
    static const std::vector<SceneDescriptor> table = get_scenes();
    for (const auto& s : table)
        if (s.name == name) return s;
    throw Error(RT_E_INVALID, "no scene named '" + name + "'");
}

// ------------------------------------------------------------------ uniform.rs
Lcg64Xsh32::Lcg64Xsh32(uint64_t state, uint64_t stream)
{
    increment_ = (stream << 1) | 1u;
    state_ = state + increment_;
    state_ = state_ * 6364136223846793005ull + increment_;
}

uint32_t Lcg64Xsh32::next_u32()
{
    const uint64_t s = state_;
    state_ = state_ * 6364136223846793005ull + increment_;
    const uint32_t rot = (uint32_t)(s >> 59);
    const uint32_t xsh = (uint32_t)(((s >> 18) ^ s) >> 27);
    return (xsh >> rot) | (xsh << ((32u - rot) & 31u));
}

uint64_t Lcg64Xsh32::next_u64()
{
    const uint64_t lo = next_u32();
    const uint64_t hi = next_u32();
    return (hi << 32) | lo;
}

double Lcg64Xsh32::gen_unit_f64()
{
    const uint64_t bits = (next_u64() >> 12) | 0x3FF0000000000000ull;
    double v;
    std::memcpy(&v, &bits, sizeof v);
    return v - 1.0;
}

std::vector<std::array<float, 2>> compute_jitters(double pixel_size, uint32_t subdivs)
{
    if (subdivs == 0 || subdivs > MAX_SUBDIVISION || pixel_size == 0.0)
        throw Error(RT_E_INVALID, "compute_jitters: subdivs must be in 1..10 and pixel_size nonzero");
    std::vector<std::array<float, 2>> out;
    if (subdivs == 1) {
        out.push_back({0.0f, 0.0f});
        return out;
    }
    Lcg64Xsh32 rng(0, 0);
    const double step = pixel_size / subdivs;
    for (uint32_t i = 0; i < subdivs; i++)
        for (uint32_t j = 0; j < subdivs; j++) {
            const double u1 = rng.gen_unit_f64();
            const double u2 = rng.gen_unit_f64();
            out.push_back({(float)((u1 + j) * step - pixel_size * 0.5), (float)((u2 + i) * step - pixel_size * 0.5)});
        }
    return out;
}

rt_uniform make_uniform(const Camera& cam, uint32_t width, uint32_t height, uint32_t selection1,
                        uint32_t subdivision_level, uint32_t iteration)
{
    rt_uniform u;
    std::memset(&u, 0, sizeof u);
    for (int i = 0; i < 3; i++) {
        u.camera_pos[i] = cam.eye[i];
        u.camera_look_at[i] = cam.target[i];
        u.camera_up[i] = cam.up[i];
    }
    u.camera_constant = cam.constant;
    u.aspect_ratio = (float)width / (float)height;   // headless: the frame's W/H (render_state.rs:563-566)
    u.selection1 = selection1;
    u.subdivision_level = subdivision_level;
    u.iteration = iteration;
    u.uv_scale[0] = u.uv_scale[1] = 1.0f;
    u.resolution[0] = width;
    u.resolution[1] = height;
    return u;
}

// ------------------------------------------------------------------ mesh.rs
Mesh Mesh::load(const std::string& path)
{
    rt_mesh_host* m = nullptr;
    const int rc = rt_mesh_load_obj(path.c_str(), &m);
    if (rc != RT_OK) throw Error(rc, "Mesh::from_obj: cannot load " + path);
    return Mesh(m);
}

Mesh Mesh::synth_bunny(uint32_t ntris, uint32_t seed)
{
    rt_mesh_host* m = nullptr;
    const int rc = rt_mesh_synth_bunny(ntris, seed, &m);
    if (rc != RT_OK) throw Error(rc, "synth_bunny failed");
    return Mesh(m);
}

Mesh::~Mesh()
{
    if (m_) rt_mesh_free(m_);
}

uint32_t Mesh::ntris() const
{
    rt_mesh_view v;
    if (rt_mesh_view_get(m_, &v) != RT_OK) return 0;
    return v.ntris;
}

// ------------------------------------------------------------------ render_state.rs
RenderState::RenderState(GpuHandles& gpu, const SceneDescriptor& scene, RenderOptions opts)
    : gpu_(gpu), opts_(std::move(opts))
{
    setup_rendering(scene);
}

RenderState::~RenderState() { release(); }

void RenderState::release()
{
    if (accum_) rt_device_free(gpu_.ctx(), accum_);
    if (ids_) rt_device_free(gpu_.ctx(), ids_);
    if (tile_accum_) rt_device_free(gpu_.ctx(), tile_accum_);
    if (tile_ids_) rt_device_free(gpu_.ctx(), tile_ids_);
    accum_ = ids_ = tile_accum_ = tile_ids_ = nullptr;
}

void RenderState::set_tiling(uint32_t nranks, uint32_t rank, const uint8_t comm_id[RT_COMM_ID_BYTES])
{
    if (tiled_) throw Error(RT_E_INVALID, "set_tiling: already tiled");
    gpu_.check(rt_comm_init(gpu_.ctx(), nranks, rank, comm_id), "communicator");
    nranks_ = nranks;
    rank_ = rank;
    tiled_ = true;
    alloc_tiles();
}

// the packed tile buffers of this rank for the current resolution (zeroed: the
// accumulation of iteration 0 is not read)
void RenderState::alloc_tiles()
{
    if (!tiled_) return;
    rt_ctx* c = gpu_.ctx();
    if (tile_accum_) rt_device_free(c, tile_accum_);
    if (tile_ids_) rt_device_free(c, tile_ids_);
    tile_accum_ = tile_ids_ = nullptr;
    const size_t px = (size_t)rt_tileset_local_tiles(width_, height_, nranks_) * 64u;
    gpu_.check(rt_device_alloc(c, px * 16, &tile_accum_), "tile accumulation buffer");
    gpu_.check(rt_device_alloc(c, px * 4, &tile_ids_), "tile id buffer");
    gpu_.check(rt_memset_device(c, tile_accum_, 0, px * 16), "clear tile accumulation");
}

void RenderState::setup_rendering(const SceneDescriptor& scene)
{
    const auto m = scene.mode();
    if (!m) throw Error(RT_E_UNSUPPORTED, scene.shader + " is outside the hot path (SURVEY.md section 2)");
    scene_ = scene;
    camera_ = scene.camera;
    mode_ = *m;
    width_ = opts_.resolution ? opts_.resolution->first : scene.res.first;
    height_ = opts_.resolution ? opts_.resolution->second : scene.res.second;
    rt_ctx* c = gpu_.ctx();
    if (mode_ == RT_MODE_W1E6) {
        trav_ = RT_TRAVERSE_NONE;
    } else {
        trav_ = scene.traverse_type == TraverseType::Bsp ? RT_TRAVERSE_BSP : RT_TRAVERSE_BVH;
        const std::string path = opts_.models_dir + "/" + scene.model.value_or("");
        struct stat st;
        const bool exists = ::stat(path.c_str(), &st) == 0;
        Mesh mesh = (!exists && scene.model == std::string("bunny.obj") && opts_.bunny_standin) ? Mesh::synth_bunny()
                                                                                                 : Mesh::load(path);
        gpu_.check(rt_upload_mesh_host(c, mesh.get()), "upload mesh");
        if (trav_ == RT_TRAVERSE_BSP) {
            if (opts_.device_build) {
                gpu_.check(rt_build_bsp_device(c, 20, 4, nullptr), "BSP device build");
            } else {   // Mesh::bsp_tree, mesh.rs:229-231 (depth 20, leaf 4)
                rt_bsp_host* b = nullptr;
                gpu_.check(rt_bsp_build(mesh.get(), 20, 4, 0, &b), "BSP build");
                const int rc = rt_upload_bsp_host(c, b);
                rt_bsp_free(b);
                gpu_.check(rc, "upload BSP");
            }
        } else {
            if (opts_.device_build) {
                gpu_.check(rt_build_bvh_device(c, 4, nullptr), "HLBVH device build");
            } else {   // Mesh::bvh, mesh.rs:233-239 (leaf 4)
                rt_bvh_host* b = nullptr;
                gpu_.check(rt_bvh_build(mesh.get(), 4, &b), "HLBVH build");
                const int rc = rt_upload_bvh_host(c, b);
                rt_bvh_free(b);
                gpu_.check(rc, "upload BVH");
            }
        }
    }
    gpu_.check(rt_set_environment(c, opts_.environment.data()), "environment");
    gpu_.check(rt_set_environment_map(c, nullptr, 0, 0), "environment map");
    release();
    const size_t npx = (size_t)width_ * height_;
    gpu_.check(rt_device_alloc(c, npx * 16, &accum_), "accumulation buffer");
    gpu_.check(rt_device_alloc(c, npx * 4, &ids_), "id buffer");
    gpu_.check(rt_memset_device(c, accum_, 0, npx * 16), "clear accumulation");
    alloc_tiles();
    iteration_ = 0;
    update();
}

void RenderState::load_scene(const SceneDescriptor& scene)
{
    iteration_ = 0;
    setup_rendering(scene);
}

void RenderState::update()
{
    camera_.aspect = (float)width_ / (float)height_;
    controller_.update_camera(camera_);
    const rt_uniform u = make_uniform(camera_, width_, height_, selection1_, subdivision_, iteration_);
    const auto jit = compute_jitters(1.0 / (double)height_, subdivision_);
    gpu_.check(rt_set_uniforms(gpu_.ctx(), &u, &jit[0][0]), "set uniforms");
}

void RenderState::render(uint32_t spp)
{
    if (tiled_) {
        // this rank's tiles, then every rank's tiles into rank 0's frame
        const rt_tileset ts{rank_, nranks_};
        gpu_.check(rt_render_tiles(gpu_.ctx(), mode_, trav_, &ts, iteration_, spp, static_cast<float*>(tile_accum_),
                                   static_cast<uint32_t*>(tile_ids_), nullptr),
                   "render tiles");
        const bool root = rank_ == 0;
        gpu_.check(rt_gather_tiles(gpu_.ctx(), width_, height_, static_cast<const float*>(tile_accum_),
                                   static_cast<const uint32_t*>(tile_ids_), root ? static_cast<float*>(accum_) : nullptr,
                                   root ? static_cast<uint32_t*>(ids_) : nullptr),
                   "gather tiles");
    } else {
        const rt_tile region{0, 0, width_, height_};
        gpu_.check(rt_render(gpu_.ctx(), mode_, trav_, &region, iteration_, spp, static_cast<float*>(accum_),
                             static_cast<uint32_t*>(ids_), nullptr),
                   "render");
    }
    const bool path = mode_ == RT_MODE_W7E3 || mode_ == RT_MODE_W9E1 || mode_ == RT_MODE_W8E1 ||
                      mode_ == RT_MODE_W8E2 || mode_ == RT_MODE_W8E3 || mode_ == RT_MODE_W9E2 ||
                      mode_ == RT_MODE_W7E1 || mode_ == RT_MODE_W7E2 || mode_ == RT_MODE_W9E3;
    if (progressive_ && path) iteration_ += spp;
    update();
}

bool RenderState::step()
{
    if (progressive_ && iteration_ >= max_iterations_) return false;
    render(1);
    return true;
}

bool RenderState::input_alt(Key key, bool pressed) { return controller_.handle_camera_commands(key, pressed); }
void RenderState::update_camera_constant(float constant) { camera_.constant = constant; }

void RenderState::set_samples(uint32_t samples, bool enabled)
{
    progressive_ = enabled;
    max_iterations_ = enabled ? samples : 2;
}

void RenderState::set_subdivision_level(uint32_t level) { subdivision_ = level <= MAX_SUBDIVISION ? level : MAX_SUBDIVISION; }
void RenderState::set_selection1(uint32_t shader) { selection1_ = shader; }

void RenderState::set_environment_map(const uint8_t* rgba8, uint32_t width, uint32_t height)
{
    gpu_.check(rt_set_environment_map(gpu_.ctx(), rgba8, width, height), "environment map");
}

void RenderState::reset_iteration()
{
    iteration_ = 0;
    update();
}

std::vector<float> RenderState::frame() const
{
    std::vector<float> out((size_t)width_ * height_ * 4);
    gpu_.check(rt_memcpy_to_host(gpu_.ctx(), out.data(), accum_, out.size() * 4), "download frame");
    return out;
}

std::vector<uint32_t> RenderState::hit_ids() const
{
    std::vector<uint32_t> out((size_t)width_ * height_);
    gpu_.check(rt_memcpy_to_host(gpu_.ctx(), out.data(), ids_, out.size() * 4), "download ids");
    return out;
}

std::vector<uint8_t> RenderState::frame_rgba8() const
{
    const size_t npx = (size_t)width_ * height_;
    void* d = nullptr;
    gpu_.check(rt_device_alloc(gpu_.ctx(), npx * 4, &d), "frame buffer");
    std::vector<uint8_t> out(npx * 4);
    int rc = rt_frame_rgba8(gpu_.ctx(), static_cast<const float*>(accum_), (uint32_t)npx, static_cast<uint8_t*>(d));
    if (rc == RT_OK) rc = rt_memcpy_to_host(gpu_.ctx(), out.data(), d, out.size());
    rt_device_free(gpu_.ctx(), d);
    gpu_.check(rc, "frame_rgba8");
    return out;
}

rt_ray_counts RenderState::last_counts() const
{
    rt_ray_counts c;
    gpu_.check(rt_last_counts(gpu_.ctx(), &c), "counts");
    return c;
}

}  // namespace raytracer
