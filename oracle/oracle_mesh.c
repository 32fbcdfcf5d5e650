/*
 * oracle_mesh.c -- TEST INFRASTRUCTURE (see oracle.h header).
 *
 * Restatement of Mesh::from_obj / Mesh::load (src/mesh.rs:78-202) on top of a
 * restatement of the third-party OBJ loader it calls: tobj 4.0.0
 * (Cargo.lock pin; not vendored under /root/reference) with LoadOptions
 * {single_index: true, triangulate: true}.  tobj's published behaviour used here:
 *   - a new model starts at `o`/`g` (when faces are pending) and at `usemtl`
 *     naming a different material (when faces are pending);
 *   - single_index: each distinct (v, vt, vn) tuple of a model becomes one
 *     vertex, numbered in first-use order; a normal is exported only for
 *     tuples that carry one;
 *   - triangulate: quads (a,b,c,d) -> (a,b,c),(a,c,d); polygons are fans
 *     (a, b_i, b_{i+1});
 *   - 1-based indices, negative indices relative to the current count;
 *   - mtllib is resolved relative to the .obj directory; if it fails the
 *     material result is an Err (mesh.rs:127-129 then uses one default material).
 * Parity of the parsed values vs tobj is unpinned (no reference test checks
 * loaded values).
 */
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct { float* a; size_t n, cap; } fvec;
typedef struct { uint32_t* a; size_t n, cap; } uvec;

static void fpush(fvec* v, float x)
{
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 64;
        v->a = (float*)realloc(v->a, v->cap * sizeof(float));
    }
    v->a[v->n++] = x;
}
static void upush(uvec* v, uint32_t x)
{
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 64;
        v->a = (uint32_t*)realloc(v->a, v->cap * sizeof(uint32_t));
    }
    v->a[v->n++] = x;
}

/* one (v, vt, vn) tuple; -1 = absent */
typedef struct { long v, vt, vn; } vtx3;
typedef struct { vtx3* a; size_t n, cap; } tvec;
static void tpush(tvec* v, vtx3 x)
{
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 64;
        v->a = (vtx3*)realloc(v->a, v->cap * sizeof(vtx3));
    }
    v->a[v->n++] = x;
}

typedef struct {
    char name[256];
    int has_kd, has_ka, has_ks, has_illum;
    float kd[3], ka[3], ks[3];
    int illum;
} mtl_entry;

typedef struct { mtl_entry* a; size_t n, cap; } mvec;

/* a model = the triangle list exported for one tobj::Model */
typedef struct {
    fvec pos, nrm;        /* per exported vertex (3 floats) */
    uvec tri;             /* 3 per triangle, model-local vertex ids */
    long mat;             /* -1 = None */
} model_t;

typedef struct { model_t* a; size_t n, cap; } modvec;

static char* trim(char* s)
{
    while (*s && isspace((unsigned char)*s)) s++;
    size_t l = strlen(s);
    while (l && isspace((unsigned char)s[l - 1])) s[--l] = 0;
    return s;
}

static int load_mtl(const char* path, mvec* out)
{
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    char line[4096];
    mtl_entry* cur = NULL;
    while (fgets(line, sizeof line, f)) {
        char* s = trim(line);
        if (!*s || *s == '#') continue;
        char key[64];
        int off = 0;
        if (sscanf(s, "%63s%n", key, &off) != 1) continue;
        char* rest = trim(s + off);
        if (!strcmp(key, "newmtl")) {
            if (out->n == out->cap) {
                out->cap = out->cap ? out->cap * 2 : 8;
                out->a = (mtl_entry*)realloc(out->a, out->cap * sizeof(mtl_entry));
            }
            cur = &out->a[out->n++];
            memset(cur, 0, sizeof *cur);
            strncpy(cur->name, rest, sizeof cur->name - 1);
        } else if (cur && !strcmp(key, "Kd")) {
            cur->has_kd = sscanf(rest, "%f %f %f", &cur->kd[0], &cur->kd[1], &cur->kd[2]) == 3;
        } else if (cur && !strcmp(key, "Ka")) {
            cur->has_ka = sscanf(rest, "%f %f %f", &cur->ka[0], &cur->ka[1], &cur->ka[2]) == 3;
        } else if (cur && !strcmp(key, "Ks")) {
            cur->has_ks = sscanf(rest, "%f %f %f", &cur->ks[0], &cur->ks[1], &cur->ks[2]) == 3;
        } else if (cur && !strcmp(key, "illum")) {
            cur->has_illum = sscanf(rest, "%d", &cur->illum) == 1;
        }
    }
    fclose(f);
    return 0;
}

/* parse "v", "v/vt", "v//vn", "v/vt/vn"; 1-based, negative relative */
static int parse_tuple(const char* tok, size_t npos, size_t ntex, size_t nnrm, vtx3* out)
{
    long a[3] = {0, 0, 0};
    int have[3] = {0, 0, 0};
    int k = 0;
    const char* p = tok;
    while (k < 3) {
        if (*p && *p != '/') {
            char* end;
            a[k] = strtol(p, &end, 10);
            have[k] = 1;
            p = end;
        }
        if (*p == '/') {
            p++;
            k++;
            continue;
        }
        break;
    }
    size_t cnt[3] = {npos, ntex, nnrm};
    long r[3] = {-1, -1, -1};
    for (int i = 0; i < 3; i++) {
        if (!have[i]) continue;
        if (a[i] < 0) r[i] = (long)cnt[i] + a[i];
        else if (a[i] > 0) r[i] = a[i] - 1;
        else return -1;
    }
    if (r[0] < 0) return -1;
    out->v = r[0];
    out->vt = r[1];
    out->vn = r[2];
    return 0;
}

/* tobj export_faces (single_index): dedup tuples in first-use order */
typedef struct { vtx3 key; uint32_t id; int used; } hent;

static uint64_t hkey(vtx3 k)
{
    uint64_t h = (uint64_t)(k.v + 1) * 0x9E3779B97F4A7C15ull;
    h ^= (uint64_t)(k.vt + 1) * 0xC2B2AE3D27D4EB4Full + (h << 6) + (h >> 2);
    h ^= (uint64_t)(k.vn + 1) * 0x165667B19E3779F9ull + (h << 6) + (h >> 2);
    return h;
}

static int export_model(const tvec* faces, const uvec* arity, const fvec* P, const fvec* N, long mat,
                        modvec* models)
{
    if (models->n == models->cap) {
        models->cap = models->cap ? models->cap * 2 : 8;
        models->a = (model_t*)realloc(models->a, models->cap * sizeof(model_t));
    }
    model_t* m = &models->a[models->n++];
    memset(m, 0, sizeof *m);
    m->mat = mat;
    size_t cap = 16;
    while (cap < faces->n * 2 + 16) cap <<= 1;
    hent* tab = (hent*)calloc(cap, sizeof(hent));
    uint32_t next = 0;
    size_t at = 0;
    int err = 0;
#define ADD_VERTEX(T)                                                                      \
    do {                                                                                   \
        vtx3 k_ = (T);                                                                     \
        size_t h_ = (size_t)(hkey(k_) & (cap - 1));                                        \
        while (tab[h_].used && !(tab[h_].key.v == k_.v && tab[h_].key.vt == k_.vt &&       \
                                 tab[h_].key.vn == k_.vn))                                 \
            h_ = (h_ + 1) & (cap - 1);                                                     \
        if (tab[h_].used) {                                                                \
            upush(&m->tri, tab[h_].id);                                                    \
        } else {                                                                           \
            if ((size_t)k_.v * 3 + 2 >= P->n) { err = 1; break; }                         \
            fpush(&m->pos, P->a[k_.v * 3]);                                                \
            fpush(&m->pos, P->a[k_.v * 3 + 1]);                                            \
            fpush(&m->pos, P->a[k_.v * 3 + 2]);                                            \
            if (N->n && k_.vn >= 0 && (size_t)k_.vn * 3 + 2 < N->n) {                      \
                fpush(&m->nrm, N->a[k_.vn * 3]);                                           \
                fpush(&m->nrm, N->a[k_.vn * 3 + 1]);                                       \
                fpush(&m->nrm, N->a[k_.vn * 3 + 2]);                                       \
            }                                                                              \
            tab[h_].used = 1;                                                              \
            tab[h_].key = k_;                                                              \
            tab[h_].id = next;                                                             \
            upush(&m->tri, next);                                                          \
            next++;                                                                        \
        }                                                                                  \
    } while (0)
    for (size_t f = 0; f < arity->n && !err; f++) {
        uint32_t n = arity->a[f];
        const vtx3* t = faces->a + at;
        at += n;
        if (n < 3) continue; /* points / lines carry no triangles */
        /* Triangle: a b c; Quad: a b c, a c d; Polygon: fan a, b, c (tobj 4.0) */
        for (uint32_t c = 2; c < n && !err; c++) {
            ADD_VERTEX(t[0]);
            if (err) break;
            ADD_VERTEX(t[c - 1]);
            if (err) break;
            ADD_VERTEX(t[c]);
        }
    }
#undef ADD_VERTEX
    free(tab);
    return err ? -1 : 0;
}

int or_light_list(const uint32_t* idx, uint32_t ntris, const or_material* mats, uint32_t nmats,
                  uint32_t** out, uint32_t* nout)
{
    /* storage_mesh.rs:316-326: triangles whose material exists and has
     * emissive == 1, prefixed with the u32::MAX sentinel */
    uint32_t* l = (uint32_t*)malloc(sizeof(uint32_t) * (ntris + 1));
    uint32_t n = 0;
    l[n++] = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < ntris; i++) {
        uint32_t m = idx[i * 4 + 3];
        if (m < nmats && mats[m].emissive == 1) l[n++] = i;
    }
    *out = l;
    *nout = n;
    return 0;
}

int or_load_obj(const char* path, or_mesh* out)
{
    memset(out, 0, sizeof *out);
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    char dir[4096];
    strncpy(dir, path, sizeof dir - 1);
    dir[sizeof dir - 1] = 0;
    char* slash = strrchr(dir, '/');
    if (slash) slash[1] = 0;
    else dir[0] = 0;

    fvec P = {0}, N = {0};
    size_t ntex = 0;
    tvec faces = {0};
    uvec arity = {0};
    modvec models = {0};
    mvec mtl = {0};
    int mtl_err = 0;
    long mat = -1;
    char* line = (char*)malloc(1 << 16);
    int err = 0;
    while (fgets(line, 1 << 16, f)) {
        char* s = trim(line);
        if (!*s || *s == '#') continue;
        char key[64];
        int off = 0;
        if (sscanf(s, "%63s%n", key, &off) != 1) continue;
        char* rest = trim(s + off);
        if (!strcmp(key, "v")) {
            float x, y, z;
            if (sscanf(rest, "%f %f %f", &x, &y, &z) != 3) { err = 1; break; }
            fpush(&P, x); fpush(&P, y); fpush(&P, z);
        } else if (!strcmp(key, "vn")) {
            float x, y, z;
            if (sscanf(rest, "%f %f %f", &x, &y, &z) != 3) { err = 1; break; }
            fpush(&N, x); fpush(&N, y); fpush(&N, z);
        } else if (!strcmp(key, "vt")) {
            ntex++;
        } else if (!strcmp(key, "f")) {
            uint32_t n = 0;
            char* save = NULL;
            for (char* tok = strtok_r(rest, " \t", &save); tok; tok = strtok_r(NULL, " \t", &save)) {
                vtx3 t;
                if (parse_tuple(tok, P.n / 3, ntex, N.n / 3, &t)) { err = 1; break; }
                tpush(&faces, t);
                n++;
            }
            if (err) break;
            upush(&arity, n);
        } else if (!strcmp(key, "o") || !strcmp(key, "g")) {
            if (arity.n) {
                if (export_model(&faces, &arity, &P, &N, mat, &models)) { err = 1; break; }
                faces.n = 0;
                arity.n = 0;
            }
        } else if (!strcmp(key, "usemtl")) {
            if (!*rest) { err = 1; break; }
            long nm = -1;
            for (size_t i = 0; i < mtl.n; i++)
                if (!strcmp(mtl.a[i].name, rest)) { nm = (long)i; break; }
            if (nm != mat && arity.n) {
                if (export_model(&faces, &arity, &P, &N, mat, &models)) { err = 1; break; }
                faces.n = 0;
                arity.n = 0;
            }
            mat = nm;
        } else if (!strcmp(key, "mtllib")) {
            char mp[8192];
            snprintf(mp, sizeof mp, "%s%s", dir, rest);
            if (load_mtl(mp, &mtl)) mtl_err = 1;
        }
    }
    fclose(f);
    free(line);
    if (!err && arity.n) err = export_model(&faces, &arity, &P, &N, mat, &models);
    if (err) {
        for (size_t i = 0; i < models.n; i++) {
            free(models.a[i].pos.a); free(models.a[i].nrm.a); free(models.a[i].tri.a);
        }
        free(models.a); free(P.a); free(N.a); free(faces.a); free(arity.a); free(mtl.a);
        return -2;
    }

    /* mesh.rs:95-133 materials */
    if (mtl_err || mtl.n == 0) {
        out->nmats = 1;
        out->mats = (or_material*)calloc(1, sizeof(or_material));
        /* Material::default(), mesh.rs:22-31 */
        out->mats[0].diffuse[0] = out->mats[0].diffuse[1] = out->mats[0].diffuse[2] = 0.5f;
        out->mats[0].diffuse[3] = 1.0f;
    } else {
        out->nmats = (uint32_t)mtl.n;
        out->mats = (or_material*)calloc(mtl.n, sizeof(or_material));
        for (size_t i = 0; i < mtl.n; i++) {
            or_material* m = &out->mats[i];
            for (int c = 0; c < 3; c++) {
                m->diffuse[c] = mtl.a[i].has_kd ? mtl.a[i].kd[c] : 1.0f;
                m->ambient[c] = mtl.a[i].has_ka ? mtl.a[i].ka[c] : 0.0f;
                m->specular[c] = mtl.a[i].has_ks ? mtl.a[i].ks[c] : 0.0f;
            }
            m->emissive = mtl.a[i].has_illum ? (uint32_t)mtl.a[i].illum : 0u;
        }
    }

    /* mesh.rs:139-194: concatenate models; indices offset by the running
     * vertex total; normals zero unless one per position */
    size_t nv = 0, nt = 0;
    for (size_t i = 0; i < models.n; i++) {
        nv += models.a[i].pos.n / 3;
        nt += models.a[i].tri.n / 3;
    }
    out->nverts = (uint32_t)nv;
    out->ntris = (uint32_t)nt;
    out->pos = (float*)calloc(nv * 4 + 4, sizeof(float));
    out->nrm = (float*)calloc(nv * 4 + 4, sizeof(float));
    out->idx = (uint32_t*)calloc(nt * 4 + 4, sizeof(uint32_t));
    size_t vbase = 0, tbase = 0;
    for (size_t i = 0; i < models.n; i++) {
        model_t* m = &models.a[i];
        size_t pn = m->pos.n / 3, nn = m->nrm.n / 3;
        for (size_t k = 0; k < pn; k++) {
            for (int c = 0; c < 3; c++) out->pos[(vbase + k) * 4 + c] = m->pos.a[k * 3 + c];
            if (nn == pn)
                for (int c = 0; c < 3; c++) out->nrm[(vbase + k) * 4 + c] = m->nrm.a[k * 3 + c];
        }
        for (size_t t = 0; t < m->tri.n / 3; t++) {
            for (int c = 0; c < 3; c++) out->idx[(tbase + t) * 4 + c] = (uint32_t)vbase + m->tri.a[t * 3 + c];
            out->idx[(tbase + t) * 4 + 3] = m->mat < 0 ? 0xFFFFFFFFu : (uint32_t)m->mat;
        }
        vbase += pn;
        tbase += m->tri.n / 3;
        free(m->pos.a); free(m->nrm.a); free(m->tri.a);
    }
    free(models.a); free(P.a); free(N.a); free(faces.a); free(arity.a); free(mtl.a);
    or_light_list(out->idx, out->ntris, out->mats, out->nmats, &out->lights, &out->nlights);
    return 0;
}

void or_free_mesh(or_mesh* m)
{
    free(m->pos); free(m->nrm); free(m->idx); free(m->mats); free(m->lights);
    memset(m, 0, sizeof *m);
}
