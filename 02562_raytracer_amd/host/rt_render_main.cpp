// rt_render: headless driver of the C++ host layer (include/raytracer.hpp) --
// what the reference's binary does per frame, minus the window: pick a scene
// from the table, set it up (load OBJ, build BSP/HLBVH, upload), feed camera
// keys and commands, render progressive iterations, and write the frame.
//
//   rt_render --list-scenes
//   rt_render --scene NAME [--res WxH] [--spp N | --samples N] [--keys K1,K2 --updates N]
//             [--selection K] [--subdiv K] [--camera-constant C] [--device-build]
//             [--env-rgba FILE --env-size WxH] [--models DIR] [--out PREFIX]
//   rt_render ... --nranks N --rank R --comm-file PATH [--comm-token T] [--device D]
//                                        (one process per GPU: rank R renders its
//                                        interleaved tiles, rank 0 gathers the frame
//                                        over RCCL and writes it; rank 0 publishes the
//                                        communicator id in PATH, tagged with T -- any
//                                        string unique to the launch, e.g. a job id, the
//                                        same on every rank; default $RT_COMM_TOKEN --
//                                        and the other ranks take only a file with
//                                        their T, never a previous launch's; without a
//                                        token PATH must be fresh; device defaults to R)
//   rt_render --camera-test K1,K2 N      (CPU: eye after N controller updates)
//   rt_render --jitter SUBDIV HEIGHT     (CPU: the jitter table)
//
// --out writes PREFIX.accum.f32 (H*W*4 float32), PREFIX.ids.u32 (H*W) and
// PREFIX.rgba8 (the sRGB frame); one JSON summary line goes to stdout.
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <fstream>
#include <iterator>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "raytracer.hpp"

using namespace raytracer;

static std::vector<std::string> split(const std::string& s, char c)
{
    std::vector<std::string> out;
    std::stringstream ss(s);
    std::string t;
    while (std::getline(ss, t, c))
        if (!t.empty()) out.push_back(t);
    return out;
}

static std::string jstr(const std::string& s)
{
    std::string o = "\"";
    for (char ch : s) {
        if (ch == '"' || ch == '\\') o += '\\';
        o += ch;
    }
    return o + "\"";
}

static std::string hexf(float f)
{
    char b[32];
    std::snprintf(b, sizeof b, "%a", (double)f);
    return jstr(b);
}

static const char* mode_name(std::optional<rt_mode> m)
{
    if (!m) return nullptr;
    switch (*m) {
    case RT_MODE_W1E6: return "W1E6";
    case RT_MODE_W6E1: return "W6E1";
    case RT_MODE_PROJECT: return "PROJECT";
    case RT_MODE_W7E3: return "W7E3";
    case RT_MODE_W9E1: return "W9E1";
    case RT_MODE_W8E1: return "W8E1";
    case RT_MODE_W8E2: return "W8E2";
    case RT_MODE_W8E3: return "W8E3";
    case RT_MODE_W9E2: return "W9E2";
    case RT_MODE_W6E2: return "W6E2";
    case RT_MODE_W7E1: return "W7E1";
    case RT_MODE_W7E2: return "W7E2";
    case RT_MODE_W6E3: return "W6E3";
    case RT_MODE_W9E3: return "W9E3";
    }
    return nullptr;
}

static std::string cam_json(const Camera& c)
{
    auto v = [](const Vec3& a) { return "[" + hexf(a[0]) + "," + hexf(a[1]) + "," + hexf(a[2]) + "]"; };
    return "{\"eye\":" + v(c.eye) + ",\"target\":" + v(c.target) + ",\"up\":" + v(c.up) +
           ",\"constant\":" + hexf(c.constant) + "}";
}

static void write_file(const std::string& path, const void* p, size_t n)
{
    std::ofstream f(path, std::ios::binary);
    f.write(static_cast<const char*>(p), (std::streamsize)n);
    if (!f) throw Error(RT_E_INVALID, "cannot write " + path);
}

// the communicator id through a file: rank 0 writes "RTCOMMID <token>\n" and the
// id (to PATH.tmp, then renames, so a reader never sees a partial file), the
// other ranks wait for a file that carries their own token.  A file left by an
// earlier launch (another token) is never taken: its id has no rank 0 any more,
// and ncclCommInitRank would wait for it forever.
static void publish_comm_id(const std::string& path, const std::string& token, uint8_t id[RT_COMM_ID_BYTES],
                            uint32_t rank)
{
    if (token.find('\n') != std::string::npos) throw Error(RT_E_INVALID, "--comm-token: no newlines");
    const std::string head = "RTCOMMID " + token + "\n";
    if (rank == 0) {
        std::remove(path.c_str());   // a stale file goes before the new id exists
        if (int r = rt_comm_unique_id(id)) throw Error(r, rt_last_error(nullptr));
        std::string buf = head;
        buf.append(reinterpret_cast<const char*>(id), RT_COMM_ID_BYTES);
        write_file(path + ".tmp", buf.data(), buf.size());
        if (std::rename((path + ".tmp").c_str(), path.c_str()) != 0) throw Error(RT_E_INVALID, "cannot publish " + path);
        return;
    }
    for (int i = 0; i < 1200; i++) {   // up to 2 minutes
        std::ifstream f(path, std::ios::binary);
        std::string buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        if (buf.size() == head.size() + RT_COMM_ID_BYTES && buf.compare(0, head.size(), head) == 0) {
            std::memcpy(id, buf.data() + head.size(), RT_COMM_ID_BYTES);
            return;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    throw Error(RT_E_NOT_READY, "no communicator id for token '" + token + "' in " + path);
}

static std::string default_models_dir(const char* argv0)
{
    // <repo>/02562_raytracer_amd/bin/rt_render -> <repo>/assets/models
    std::string p(argv0);
    const size_t k = p.rfind('/');
    std::string dir = k == std::string::npos ? "." : p.substr(0, k);
    return dir + "/../../assets/models";
}

int main(int argc, char** argv)
{
    try {
        std::vector<std::string> a(argv + 1, argv + argc);
        auto arg = [&](const std::string& name) -> const std::string* {
            for (size_t i = 0; i + 1 < a.size(); i++)
                if (a[i] == name) return &a[i + 1];
            return nullptr;
        };
        auto flag = [&](const std::string& name) {
            for (const auto& s : a)
                if (s == name) return true;
            return false;
        };
        if (flag("--list-scenes")) {
            for (const auto& s : get_scenes()) {
                const char* m = mode_name(s.mode());
                std::printf("{\"name\":%s,\"shader\":%s,\"mode\":%s,\"model\":%s,\"res\":[%u,%u],\"vertex_type\":%s,"
                            "\"traverse_type\":%s,\"background_hdri\":%s,\"camera\":%s}\n",
                            jstr(s.name).c_str(), jstr(s.shader).c_str(), m ? jstr(m).c_str() : "null",
                            s.model ? jstr(*s.model).c_str() : "null", s.res.first, s.res.second,
                            s.vertex_type == VertexType::Combined ? "\"Combined\"" : "\"Split\"",
                            s.traverse_type == TraverseType::Bsp ? "\"BSP\"" : "\"BVH\"",
                            s.background_hdri ? jstr(*s.background_hdri).c_str() : "null",
                            cam_json(s.camera).c_str());
            }
            return 0;
        }
        if (const std::string* k = arg("--camera-test")) {
            CameraController ctl;
            for (const auto& name : split(*k, ',')) ctl.handle_camera_commands(key_from_name(name), true);
            Camera c;
            const int n = std::atoi(argc > 3 ? argv[3] : "1");
            for (int i = 0; i < n; i++) ctl.update_camera(c);
            std::printf("%s\n", cam_json(c).c_str());
            return 0;
        }
        if (const std::string* sd = arg("--jitter")) {
            const uint32_t subdiv = (uint32_t)std::atoi(sd->c_str());
            const double h = argc > 3 ? std::atof(argv[3]) : 512.0;
            for (const auto& j : compute_jitters(1.0 / h, subdiv)) std::printf("%s %s\n", hexf(j[0]).c_str(), hexf(j[1]).c_str());
            return 0;
        }
        const std::string* name = arg("--scene");
        if (!name) {
            std::fprintf(stderr, "usage: rt_render --list-scenes | --scene NAME [options] (see the source header)\n");
            return 2;
        }
        RenderOptions opt;
        opt.models_dir = arg("--models") ? *arg("--models") : default_models_dir(argv[0]);
        if (const std::string* r = arg("--res")) {
            unsigned w = 0, h = 0;
            if (std::sscanf(r->c_str(), "%ux%u", &w, &h) != 2) throw Error(RT_E_INVALID, "--res WxH");
            opt.resolution = std::make_pair(w, h);
        }
        opt.device_build = flag("--device-build");
        const uint32_t nranks = arg("--nranks") ? (uint32_t)std::atoi(arg("--nranks")->c_str()) : 1;
        const uint32_t rank = arg("--rank") ? (uint32_t)std::atoi(arg("--rank")->c_str()) : 0;
        if (nranks == 0 || rank >= nranks) throw Error(RT_E_INVALID, "--rank must be below --nranks");
        if (nranks > 1 && !arg("--comm-file")) throw Error(RT_E_INVALID, "--nranks needs --comm-file PATH");
        GpuHandles gpu(arg("--device") ? std::atoi(arg("--device")->c_str()) : (int)rank);
        RenderState rs(gpu, find_scene(*name), opt);
        if (const std::string* cf = arg("--comm-file")) {
            uint8_t id[RT_COMM_ID_BYTES];
            const char* et = std::getenv("RT_COMM_TOKEN");
            const std::string token = arg("--comm-token") ? *arg("--comm-token") : (et ? et : "");
            publish_comm_id(*cf, token, id, rank);
            rs.set_tiling(nranks, rank, id);
        }
        std::vector<uint8_t> env;
        if (const std::string* ef = arg("--env-rgba")) {
            unsigned w = 0, h = 0;
            if (!arg("--env-size") || std::sscanf(arg("--env-size")->c_str(), "%ux%u", &w, &h) != 2)
                throw Error(RT_E_INVALID, "--env-rgba needs --env-size WxH");
            std::ifstream f(*ef, std::ios::binary);
            env.resize((size_t)w * h * 4);
            f.read(reinterpret_cast<char*>(env.data()), (std::streamsize)env.size());
            if (!f) throw Error(RT_E_INVALID, "cannot read " + *ef);
            rs.set_environment_map(env.data(), w, h);
        }
        if (const std::string* s = arg("--selection")) rs.set_selection1((uint32_t)std::atoi(s->c_str()));
        if (const std::string* s = arg("--subdiv")) rs.set_subdivision_level((uint32_t)std::atoi(s->c_str()));
        if (const std::string* s = arg("--camera-constant")) rs.update_camera_constant((float)std::atof(s->c_str()));
        if (const std::string* k = arg("--keys")) {
            for (const auto& kn : split(*k, ',')) rs.input_alt(key_from_name(kn), true);
            const int n = arg("--updates") ? std::atoi(arg("--updates")->c_str()) : 1;
            for (int i = 0; i < n; i++) rs.update();
        } else {
            rs.update();
        }
        uint32_t frames = 0;
        if (const std::string* s = arg("--samples")) {   // the progressive loop, SetSamples
            rs.set_samples((uint32_t)std::atoi(s->c_str()), true);
            while (rs.step()) frames++;
        } else {
            const uint32_t spp = arg("--spp") ? (uint32_t)std::atoi(arg("--spp")->c_str()) : 1;
            rs.render(spp);
            frames = 1;
        }
        const rt_ray_counts c = rs.last_counts();
        if (rank != 0) return 0;   // the frame is rank 0's
        if (const std::string* out = arg("--out")) {
            const auto f = rs.frame();
            const auto ids = rs.hit_ids();
            const auto rgba = rs.frame_rgba8();
            write_file(*out + ".accum.f32", f.data(), f.size() * 4);
            write_file(*out + ".ids.u32", ids.data(), ids.size() * 4);
            write_file(*out + ".rgba8", rgba.data(), rgba.size());
        }
        std::printf("{\"scene\":%s,\"mode\":%s,\"width\":%u,\"height\":%u,\"iteration\":%u,\"frames\":%u,"
                    "\"last_launch\":{\"samples\":%llu,\"primary\":%llu,\"shadow\":%llu,\"bounce\":%llu},\"camera\":%s}\n",
                    jstr(rs.scene().name).c_str(), jstr(mode_name(rs.scene().mode())).c_str(), rs.width(), rs.height(),
                    rs.iteration(), frames, (unsigned long long)c.samples, (unsigned long long)c.primary,
                    (unsigned long long)c.shadow, (unsigned long long)c.bounce, cam_json(rs.camera()).c_str());
        return 0;
    } catch (const Error& e) {
        std::fprintf(stderr, "rt_render: error %d: %s\n", e.code, e.what());
        return 1;
    }
}
