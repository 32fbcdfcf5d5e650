// host_mesh.cpp -- Mesh::from_obj (src/mesh.rs:78-202) and synthetic meshes.
//
// The reference parses OBJ with tobj 4.0.0 (LoadOptions {single_index,
// triangulate}); this loader implements that behaviour: models split at o/g and
// at material changes, (v, vt, vn) tuples deduplicated per model in first-use
// order, quads/polygons fan-triangulated, MTL Kd/Ka/Ks/illum.  Triangle order
// (the BSP/BVH primitive ids) is face order across models.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "host_types.h"

namespace rthost {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* get_error() { return g_err.c_str(); }

rt_material default_material()   // Material::default(), src/mesh.rs:22-31
{
    rt_material m;
    memset(&m, 0, sizeof m);
    m.diffuse[0] = m.diffuse[1] = m.diffuse[2] = 0.5f;
    m.diffuse[3] = 1.0f;
    return m;
}

std::vector<uint32_t> light_list(const std::vector<uint32_t>& idx, const std::vector<rt_material>& mats)
{
    std::vector<uint32_t> l;
    l.push_back(0xFFFFFFFFu);
    const size_t nt = idx.size() / 4;
    for (size_t i = 0; i < nt; i++) {
        uint32_t m = idx[i * 4 + 3];
        if (m < mats.size() && mats[m].emissive == 1) l.push_back((uint32_t)i);
    }
    return l;
}

namespace {

struct MtlEntry {
    std::string name;
    bool kd = false, ka = false, ks = false, il = false;
    float Kd[3] = {0, 0, 0}, Ka[3] = {0, 0, 0}, Ks[3] = {0, 0, 0};
    int illum = 0;
};

bool read_floats(const char* s, float* out, int n)
{
    char* end = nullptr;
    for (int i = 0; i < n; i++) {
        out[i] = strtof(s, &end);
        if (end == s) return false;
        s = end;
    }
    return true;
}

bool load_mtl(const std::string& path, std::vector<MtlEntry>& out)
{
    std::ifstream f(path);
    if (!f) return false;
    std::string line;
    MtlEntry* cur = nullptr;
    while (std::getline(f, line)) {
        const char* s = line.c_str();
        while (*s == ' ' || *s == '\t') s++;
        if (!*s || *s == '#') continue;
        const char* k = s;
        while (*s && *s != ' ' && *s != '\t' && *s != '\r') s++;
        std::string key(k, s - k);
        while (*s == ' ' || *s == '\t') s++;
        std::string rest(s);
        while (!rest.empty() && (rest.back() == '\r' || rest.back() == ' ' || rest.back() == '\t')) rest.pop_back();
        if (key == "newmtl") {
            out.emplace_back();
            cur = &out.back();
            cur->name = rest;
        } else if (cur && key == "Kd") {
            cur->kd = read_floats(rest.c_str(), cur->Kd, 3);
        } else if (cur && key == "Ka") {
            cur->ka = read_floats(rest.c_str(), cur->Ka, 3);
        } else if (cur && key == "Ks") {
            cur->ks = read_floats(rest.c_str(), cur->Ks, 3);
        } else if (cur && key == "illum") {
            cur->il = sscanf(rest.c_str(), "%d", &cur->illum) == 1;
        }
    }
    return true;
}

struct Tuple {
    long v, vt, vn;
    bool operator==(const Tuple& o) const { return v == o.v && vt == o.vt && vn == o.vn; }
};
struct TupleHash {
    size_t operator()(const Tuple& t) const
    {
        uint64_t h = (uint64_t)(t.v + 1) * 0x9E3779B97F4A7C15ull;
        h ^= (uint64_t)(t.vt + 1) * 0xC2B2AE3D27D4EB4Full + (h << 6) + (h >> 2);
        h ^= (uint64_t)(t.vn + 1) * 0x165667B19E3779F9ull + (h << 6) + (h >> 2);
        return (size_t)h;
    }
};

struct Model {
    std::vector<float> pos, nrm;
    std::vector<uint32_t> tri;
    long mat = -1;
};

bool parse_tuple(const char* tok, size_t np, size_t nt, size_t nn, Tuple& out)
{
    long a[3] = {0, 0, 0};
    bool have[3] = {false, false, false};
    int k = 0;
    const char* p = tok;
    while (k < 3) {
        if (*p && *p != '/') {
            char* end;
            a[k] = strtol(p, &end, 10);
            have[k] = true;
            p = end;
        }
        if (*p == '/') {
            p++;
            k++;
            continue;
        }
        break;
    }
    const size_t cnt[3] = {np, nt, nn};
    long r[3] = {-1, -1, -1};
    for (int i = 0; i < 3; i++) {
        if (!have[i]) continue;
        if (a[i] < 0) r[i] = (long)cnt[i] + a[i];
        else if (a[i] > 0) r[i] = a[i] - 1;
        else return false;
    }
    if (r[0] < 0) return false;
    out = Tuple{r[0], r[1], r[2]};
    return true;
}

// tobj export_faces with single_index + triangulate
bool export_model(const std::vector<Tuple>& faces, const std::vector<uint32_t>& arity, const std::vector<float>& P,
                  const std::vector<float>& N, long mat, std::vector<Model>& models)
{
    models.emplace_back();
    Model& m = models.back();
    m.mat = mat;
    std::unordered_map<Tuple, uint32_t, TupleHash> map;
    map.reserve(faces.size());
    auto add = [&](const Tuple& t) -> bool {
        auto it = map.find(t);
        if (it != map.end()) {
            m.tri.push_back(it->second);
            return true;
        }
        if ((size_t)t.v * 3 + 2 >= P.size()) return false;
        m.pos.insert(m.pos.end(), {P[t.v * 3], P[t.v * 3 + 1], P[t.v * 3 + 2]});
        if (!N.empty() && t.vn >= 0 && (size_t)t.vn * 3 + 2 < N.size())
            m.nrm.insert(m.nrm.end(), {N[t.vn * 3], N[t.vn * 3 + 1], N[t.vn * 3 + 2]});
        uint32_t id = (uint32_t)map.size();
        map.emplace(t, id);
        m.tri.push_back(id);
        return true;
    };
    size_t at = 0;
    for (uint32_t n : arity) {
        const Tuple* t = faces.data() + at;
        at += n;
        if (n < 3) continue;
        for (uint32_t c = 2; c < n; c++)
            if (!add(t[0]) || !add(t[c - 1]) || !add(t[c])) return false;
    }
    return true;
}

}  // namespace
}  // namespace rthost

using namespace rthost;

extern "C" int rt_mesh_load_obj(const char* path, rt_mesh_host** out)
{
    if (!path || !out) {
        set_error("rt_mesh_load_obj: null argument");
        return RT_E_INVALID;
    }
    std::ifstream f(path);
    if (!f) {
        set_error(std::string("rt_mesh_load_obj: cannot open ") + path);
        return RT_E_IO;
    }
    std::string dir(path);
    size_t sl = dir.rfind('/');
    dir = sl == std::string::npos ? std::string() : dir.substr(0, sl + 1);

    std::vector<float> P, N;
    size_t ntex = 0;
    std::vector<Tuple> faces;
    std::vector<uint32_t> arity;
    std::vector<Model> models;
    std::vector<MtlEntry> mtl;
    bool mtl_err = false;
    long mat = -1;
    std::string line;
    auto flush = [&]() -> bool {
        if (arity.empty()) return true;
        bool ok = export_model(faces, arity, P, N, mat, models);
        faces.clear();
        arity.clear();
        return ok;
    };
    while (std::getline(f, line)) {
        const char* s = line.c_str();
        while (*s == ' ' || *s == '\t') s++;
        if (!*s || *s == '#') continue;
        const char* k = s;
        while (*s && *s != ' ' && *s != '\t' && *s != '\r') s++;
        const size_t klen = s - k;
        while (*s == ' ' || *s == '\t') s++;
        if (klen == 1 && k[0] == 'v') {
            float v[3];
            if (!read_floats(s, v, 3)) {
                set_error("rt_mesh_load_obj: bad vertex");
                return RT_E_IO;
            }
            P.insert(P.end(), v, v + 3);
        } else if (klen == 2 && k[0] == 'v' && k[1] == 'n') {
            float v[3];
            if (!read_floats(s, v, 3)) {
                set_error("rt_mesh_load_obj: bad normal");
                return RT_E_IO;
            }
            N.insert(N.end(), v, v + 3);
        } else if (klen == 2 && k[0] == 'v' && k[1] == 't') {
            ntex++;
        } else if (klen == 1 && k[0] == 'f') {
            uint32_t n = 0;
            std::string rest(s);
            char* save = nullptr;
            for (char* tok = strtok_r(&rest[0], " \t\r", &save); tok; tok = strtok_r(nullptr, " \t\r", &save)) {
                Tuple t;
                if (!parse_tuple(tok, P.size() / 3, ntex, N.size() / 3, t)) {
                    set_error("rt_mesh_load_obj: bad face index");
                    return RT_E_IO;
                }
                faces.push_back(t);
                n++;
            }
            arity.push_back(n);
        } else if (klen == 1 && (k[0] == 'o' || k[0] == 'g')) {
            if (!flush()) {
                set_error("rt_mesh_load_obj: face vertex out of bounds");
                return RT_E_IO;
            }
        } else if (klen == 6 && !strncmp(k, "usemtl", 6)) {
            std::string name(s);
            while (!name.empty() && (name.back() == '\r' || name.back() == ' ' || name.back() == '\t')) name.pop_back();
            if (name.empty()) {
                set_error("rt_mesh_load_obj: empty usemtl");
                return RT_E_IO;
            }
            long nm = -1;
            for (size_t i = 0; i < mtl.size(); i++)
                if (mtl[i].name == name) {
                    nm = (long)i;
                    break;
                }
            if (nm != mat && !flush()) {
                set_error("rt_mesh_load_obj: face vertex out of bounds");
                return RT_E_IO;
            }
            mat = nm;
        } else if (klen == 6 && !strncmp(k, "mtllib", 6)) {
            std::string name(s);
            while (!name.empty() && (name.back() == '\r' || name.back() == ' ' || name.back() == '\t')) name.pop_back();
            if (!load_mtl(dir + name, mtl)) mtl_err = true;
        }
    }
    if (!flush()) {
        set_error("rt_mesh_load_obj: face vertex out of bounds");
        return RT_E_IO;
    }

    rt_mesh_host* m = new rt_mesh_host();
    if (mtl_err || mtl.empty()) {   // mesh.rs:127-133
        m->mats.push_back(default_material());
    } else {
        for (const MtlEntry& e : mtl) {
            rt_material x;
            memset(&x, 0, sizeof x);
            for (int c = 0; c < 3; c++) {
                x.diffuse[c] = e.kd ? e.Kd[c] : 1.0f;
                x.ambient[c] = e.ka ? e.Ka[c] : 0.0f;
                x.specular[c] = e.ks ? e.Ks[c] : 0.0f;
            }
            x.emissive = e.il ? (uint32_t)e.illum : 0u;
            m->mats.push_back(x);
        }
    }
    size_t nv = 0, nt = 0;
    for (const Model& md : models) {
        nv += md.pos.size() / 3;
        nt += md.tri.size() / 3;
    }
    m->pos.assign(nv * 4, 0.0f);
    m->nrm.assign(nv * 4, 0.0f);
    m->idx.assign(nt * 4, 0u);
    size_t vb = 0, tb = 0;
    for (const Model& md : models) {   // mesh.rs:139-194
        const size_t pn = md.pos.size() / 3, nn = md.nrm.size() / 3;
        for (size_t i = 0; i < pn; i++) {
            for (int c = 0; c < 3; c++) m->pos[(vb + i) * 4 + c] = md.pos[i * 3 + c];
            if (nn == pn)
                for (int c = 0; c < 3; c++) m->nrm[(vb + i) * 4 + c] = md.nrm[i * 3 + c];
        }
        const size_t tn = md.tri.size() / 3;
        for (size_t t = 0; t < tn; t++) {
            for (int c = 0; c < 3; c++) m->idx[(tb + t) * 4 + c] = (uint32_t)vb + md.tri[t * 3 + c];
            m->idx[(tb + t) * 4 + 3] = md.mat < 0 ? 0xFFFFFFFFu : (uint32_t)md.mat;
        }
        vb += pn;
        tb += tn;
    }
    m->lights = light_list(m->idx, m->mats);
    *out = m;
    return RT_OK;
}

extern "C" int rt_mesh_from_arrays(const float* pos_vec4, const float* nrm_vec4, uint32_t nverts,
                                   const uint32_t* idx_vec4u, uint32_t ntris, const rt_material* mats, uint32_t nmats,
                                   rt_mesh_host** out)
{
    if (!out || (!pos_vec4 && nverts) || (!idx_vec4u && ntris)) {
        set_error("rt_mesh_from_arrays: null argument");
        return RT_E_INVALID;
    }
    for (uint32_t t = 0; t < ntris; t++)
        for (int c = 0; c < 3; c++)
            if (idx_vec4u[t * 4 + c] >= nverts) {
                set_error("rt_mesh_from_arrays: vertex index out of range");
                return RT_E_INVALID;
            }
    rt_mesh_host* m = new rt_mesh_host();
    m->pos.assign(pos_vec4, pos_vec4 + (size_t)nverts * 4);
    if (nrm_vec4) m->nrm.assign(nrm_vec4, nrm_vec4 + (size_t)nverts * 4);
    else m->nrm.assign((size_t)nverts * 4, 0.0f);
    m->idx.assign(idx_vec4u, idx_vec4u + (size_t)ntris * 4);
    if (mats && nmats) m->mats.assign(mats, mats + nmats);
    else m->mats.push_back(default_material());
    m->lights = light_list(m->idx, m->mats);
    *out = m;
    return RT_OK;
}

// ------------------------------------------------------------------ synthetic meshes

// Displaced UV sphere standing in for the Stanford bunny (res/models/bunny.obj
// is missing from the reference checkout, .MISSING_LARGE_BLOBS:8): S segments x
// (R-2) rings plus two poles, 2*S*(R-2) triangles, scaled to the bunny's bounding box
// (centre (-0.0168, 0.110, -0.0015), extent 0.155 x 0.154 x 0.121) with
// smooth deterministic bumps; white Kd 0.9 material (res/models/bunny.mtl:1-5);
// area-weighted vertex normals.
extern "C" int rt_mesh_synth_bunny(uint32_t ntris_target, uint32_t seed, rt_mesh_host** out)
{
    if (!out || ntris_target < 8) {
        set_error("rt_mesh_synth_bunny: bad argument");
        return RT_E_INVALID;
    }
    // choose S ~ R with 2*S*(R-1) ~ ntris_target
    uint32_t S = (uint32_t)ceil(sqrt((double)ntris_target / 2.0));
    if (S < 3) S = 3;
    uint32_t R = (uint32_t)llround((double)ntris_target / (2.0 * S)) + 2;   // 2*S*(R-2) triangles
    if (R < 4) R = 4;
    std::mt19937 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 6.283185307179586);
    double ph[6];
    for (double& p : ph) p = U(rng);
    const double cx = -0.0168, cy = 0.110, cz = -0.0015, ex = 0.155 / 2, ey = 0.154 / 2, ez = 0.121 / 2;
    rt_mesh_host* m = new rt_mesh_host();
    // vertices: north pole, (R-2) rings of S, south pole
    auto radius = [&](double th, double phi) {
        return 1.0 + 0.12 * sin(3 * th + ph[0]) * cos(2 * phi + ph[1]) + 0.06 * sin(7 * th + ph[2]) * sin(5 * phi + ph[3]) +
               0.03 * cos(11 * th + ph[4]) * cos(9 * phi + ph[5]);
    };
    auto push_v = [&](double th, double phi) {
        double r = radius(th, phi);
        double x = r * sin(th) * cos(phi), y = r * cos(th), z = r * sin(th) * sin(phi);
        m->pos.insert(m->pos.end(), {(float)(cx + ex * x), (float)(cy + ey * y), (float)(cz + ez * z), 0.0f});
    };
    push_v(0.0, 0.0);
    for (uint32_t i = 1; i + 1 < R; i++) {
        double th = M_PI * i / (R - 1);
        for (uint32_t j = 0; j < S; j++) push_v(th, 2 * M_PI * j / S);
    }
    push_v(M_PI, 0.0);
    const uint32_t north = 0, south = (uint32_t)(m->pos.size() / 4 - 1);
    auto ring = [&](uint32_t i, uint32_t j) { return 1 + (i - 1) * S + (j % S); };   // i in [1, R-2]
    auto tri = [&](uint32_t a, uint32_t b, uint32_t c) { m->idx.insert(m->idx.end(), {a, b, c, 0u}); };
    for (uint32_t j = 0; j < S; j++) tri(north, ring(1, j + 1), ring(1, j));
    for (uint32_t i = 1; i + 2 < R; i++)
        for (uint32_t j = 0; j < S; j++) {
            tri(ring(i, j), ring(i, j + 1), ring(i + 1, j + 1));
            tri(ring(i, j), ring(i + 1, j + 1), ring(i + 1, j));
        }
    for (uint32_t j = 0; j < S; j++) tri(south, ring(R - 2, j), ring(R - 2, j + 1));
    // area-weighted vertex normals (outward)
    const size_t nv = m->pos.size() / 4;
    std::vector<double> acc(nv * 3, 0.0);
    for (size_t t = 0; t < m->idx.size() / 4; t++) {
        const uint32_t* ix = &m->idx[t * 4];
        double v[3][3];
        for (int k = 0; k < 3; k++)
            for (int c = 0; c < 3; c++) v[k][c] = m->pos[ix[k] * 4 + c];
        double e0[3], e1[3], n[3];
        for (int c = 0; c < 3; c++) {
            e0[c] = v[1][c] - v[0][c];
            e1[c] = v[2][c] - v[0][c];
        }
        n[0] = e0[1] * e1[2] - e0[2] * e1[1];
        n[1] = e0[2] * e1[0] - e0[0] * e1[2];
        n[2] = e0[0] * e1[1] - e0[1] * e1[0];
        for (int k = 0; k < 3; k++)
            for (int c = 0; c < 3; c++) acc[ix[k] * 3 + c] += n[c];
    }
    m->nrm.assign(nv * 4, 0.0f);
    for (size_t i = 0; i < nv; i++) {
        double l = sqrt(acc[i * 3] * acc[i * 3] + acc[i * 3 + 1] * acc[i * 3 + 1] + acc[i * 3 + 2] * acc[i * 3 + 2]);
        if (l > 0)
            for (int c = 0; c < 3; c++) m->nrm[i * 4 + c] = (float)(acc[i * 3 + c] / l);
    }
    rt_material w;
    memset(&w, 0, sizeof w);
    w.diffuse[0] = w.diffuse[1] = w.diffuse[2] = 0.9f;
    m->mats.push_back(w);
    m->lights = light_list(m->idx, m->mats);
    *out = m;
    return RT_OK;
}

// 10M-style random triangle soup: centres U[-1,1]^3,
// vertices = centre + U[-0.01,0.01]^3; 64-bit LCG (PCG32 output) seeded by `seed`.
// Triangle t takes draws 12t .. 12t+11 of the one stream, so threads fill disjoint
// triangle ranges from a jumped-ahead state (the same mesh, bit for bit, as one pass).
static constexpr uint64_t SOUP_MUL = 6364136223846793005ull, SOUP_INC = 1442695040888963407ull;

// the LCG state `delta` steps after `state` (Brown, "Random number generation with
// arbitrary strides": the affine map's powers by squaring)
static uint64_t lcg_advance(uint64_t state, uint64_t delta)
{
    uint64_t acc_mul = 1, acc_inc = 0, mul = SOUP_MUL, inc = SOUP_INC;
    while (delta) {
        if (delta & 1) {
            acc_mul *= mul;
            acc_inc = acc_inc * mul + inc;
        }
        inc = (mul + 1) * inc;
        mul *= mul;
        delta >>= 1;
    }
    return acc_mul * state + acc_inc;
}

extern "C" int rt_mesh_synth_soup(uint32_t ntris, uint32_t seed, rt_mesh_host** out)
{
    if (!out || ntris == 0) {
        set_error("rt_mesh_synth_soup: bad argument");
        return RT_E_INVALID;
    }
    const uint64_t state0 = 0x853c49e6748fea9bull ^ ((uint64_t)seed << 1);
    rt_mesh_host* m = new rt_mesh_host();
    m->pos.resize((size_t)ntris * 12);
    m->idx.resize((size_t)ntris * 4);
    m->nrm.resize((size_t)ntris * 12);
    auto fill = [&](uint32_t lo, uint32_t hi) {
        uint64_t state = lcg_advance(state0, 12ull * lo);
        auto pcg = [&]() {
            uint64_t old = state;
            state = old * SOUP_MUL + SOUP_INC;
            uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
            uint32_t rot = (uint32_t)(old >> 59u);
            return (xs >> rot) | (xs << ((-rot) & 31));
        };
        auto uni = [&](float a, float b) { return a + (b - a) * (float)((pcg() >> 8) * (1.0 / 16777216.0)); };
        for (uint32_t t = lo; t < hi; t++) {
            float* p = &m->pos[(size_t)t * 12];
            const float c0 = uni(-1, 1), c1 = uni(-1, 1), c2 = uni(-1, 1);
            for (int k = 0; k < 3; k++) {   // (the three offsets in argument order x, y, z)
                const float ox = uni(-0.01f, 0.01f), oy = uni(-0.01f, 0.01f), oz = uni(-0.01f, 0.01f);
                p[4 * k] = c0 + ox;
                p[4 * k + 1] = c1 + oy;
                p[4 * k + 2] = c2 + oz;
                p[4 * k + 3] = 0.0f;
            }
            uint32_t* ix = &m->idx[(size_t)t * 4];
            ix[0] = 3 * t;
            ix[1] = 3 * t + 1;
            ix[2] = 3 * t + 2;
            ix[3] = 0u;
            double e0[3], e1[3], n[3];   // face normal as vertex normal
            for (int c = 0; c < 3; c++) {
                e0[c] = p[4 + c] - p[c];
                e1[c] = p[8 + c] - p[c];
            }
            n[0] = e0[1] * e1[2] - e0[2] * e1[1];
            n[1] = e0[2] * e1[0] - e0[0] * e1[2];
            n[2] = e0[0] * e1[1] - e0[1] * e1[0];
            const double l = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            float* q = &m->nrm[(size_t)t * 12];
            for (int k = 0; k < 3; k++) {
                for (int c = 0; c < 3; c++) q[k * 4 + c] = l > 0 ? (float)(n[c] / l) : 0.0f;
                q[k * 4 + 3] = 0.0f;
            }
        }
    };
    // (16 threads at most: the GPU box's per-GPU share of the host)
    const uint32_t nthr = std::min<uint32_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
    if (ntris < 65536 || nthr == 1) {
        fill(0, ntris);
    } else {
        std::vector<std::thread> th;
        const uint32_t chunk = (ntris + nthr - 1) / nthr;
        for (uint32_t k = 0; k < nthr; k++) {
            const uint32_t lo = k * chunk, hi = std::min<uint32_t>(ntris, lo + chunk);
            if (lo < hi) th.emplace_back(fill, lo, hi);
        }
        for (auto& t : th) t.join();
    }
    rt_material w;
    memset(&w, 0, sizeof w);
    w.diffuse[0] = w.diffuse[1] = w.diffuse[2] = 0.9f;
    m->mats.push_back(w);
    m->lights = light_list(m->idx, m->mats);
    *out = m;
    return RT_OK;
}

// nx x nz grid of translated copies (x/z spacing), flattened into one mesh.
extern "C" int rt_mesh_synth_grid(const rt_mesh_host* src, uint32_t nx, uint32_t nz, float spacing,
                                  rt_mesh_host** out)
{
    if (!src || !out || nx == 0 || nz == 0) {
        set_error("rt_mesh_synth_grid: bad argument");
        return RT_E_INVALID;
    }
    const uint64_t total = (uint64_t)src->ntris() * nx * nz;
    if (total >= 0xFFFFFFFFull / 2) {
        set_error("rt_mesh_synth_grid: too many triangles");
        return RT_E_INVALID;
    }
    rt_mesh_host* m = new rt_mesh_host();
    const uint32_t nv = src->nverts();
    m->pos.reserve(src->pos.size() * nx * nz);
    m->nrm.reserve(src->nrm.size() * nx * nz);
    m->idx.reserve(src->idx.size() * nx * nz);
    const float ox = -0.5f * spacing * (float)(nx - 1), oz = -0.5f * spacing * (float)(nz - 1);
    for (uint32_t gz = 0; gz < nz; gz++)
        for (uint32_t gx = 0; gx < nx; gx++) {
            const uint32_t base = (uint32_t)(m->pos.size() / 4);
            const float dx = ox + spacing * (float)gx, dz = oz + spacing * (float)gz;
            for (uint32_t v = 0; v < nv; v++) {
                const float* p = &src->pos[(size_t)v * 4];
                m->pos.insert(m->pos.end(), {p[0] + dx, p[1], p[2] + dz, 0.0f});
                m->nrm.insert(m->nrm.end(), &src->nrm[(size_t)v * 4], &src->nrm[(size_t)v * 4] + 4);
            }
            for (size_t t = 0; t < src->idx.size() / 4; t++) {
                const uint32_t* ix = &src->idx[t * 4];
                m->idx.insert(m->idx.end(), {base + ix[0], base + ix[1], base + ix[2], ix[3]});
            }
        }
    m->mats = src->mats;
    m->lights = light_list(m->idx, m->mats);
    *out = m;
    return RT_OK;
}

extern "C" int rt_mesh_scale(rt_mesh_host* m, float factor)
{
    if (!m) return RT_E_INVALID;
    for (size_t v = 0; v < m->pos.size() / 4; v++)   // Mesh::scale, mesh.rs:246-252
        for (int c = 0; c < 3; c++) m->pos[v * 4 + c] = m->pos[v * 4 + c] * factor;
    return RT_OK;
}

extern "C" int rt_mesh_view_get(const rt_mesh_host* m, rt_mesh_view* v)
{
    if (!m || !v) return RT_E_INVALID;
    v->vertices = m->pos.data();
    v->normals = m->nrm.data();
    v->indices = m->idx.data();
    v->materials = m->mats.data();
    v->lights = m->lights.data();
    v->nverts = m->nverts();
    v->ntris = m->ntris();
    v->nmats = (uint32_t)m->mats.size();
    v->nlights = (uint32_t)m->lights.size();
    return RT_OK;
}

extern "C" void rt_mesh_free(rt_mesh_host* m) { delete m; }
