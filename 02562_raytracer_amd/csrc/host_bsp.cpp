// host_bsp.cpp -- BspTree::new + bsp_array + primitive_ids
// (src/data_structures/bsp_tree.rs:45-189), multi-threaded.
//
// Output is bit-identical to the reference's single-threaded f32 build: the
// node slot of every subtree is fixed by (depth, branch) (idx = 2^depth +
// branch - 1, :137), so subtrees are built concurrently straight into the
// shared arrays; only the leaf first-ids depend on DFS order and are assigned
// in a sequential pass over the DFS-ordered leaf list afterwards.
// Compiled with -ffp-contract=off (Rust never contracts a*b+c).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <future>
#include <thread>
#include <vector>

#include "../../include/rt_detmath.h"
#include "host_types.h"

namespace {

struct Box {
    float mn[3], mx[3];
};

inline bool intersects(const Box& s, const Box& o)   // bbox.rs:151-155
{
    return !(o.mn[0] > s.mx[0] || o.mx[0] < s.mn[0]) && !(o.mn[1] > s.mx[1] || o.mx[1] < s.mn[1]) &&
           !(o.mn[2] > s.mx[2] || o.mx[2] < s.mn[2]);
}
inline float area(const Box& b)   // bbox.rs:117-125
{
    const float d0 = b.mx[0] - b.mn[0], d1 = b.mx[1] - b.mn[1], d2 = b.mx[2] - b.mn[2];
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}

struct Leaf {
    size_t idx;
    std::vector<uint32_t> objs;
};

struct Builder {
    const Box* boxes;
    uint32_t* tree;
    float* planes;
    uint32_t max_depth, max_leaf;
    int par_depth;   // spawn a task for the left subtree above this depth

    void build(const Box& bbox, uint32_t depth, size_t branch, std::vector<uint32_t>&& objs, std::vector<Leaf>& out)
    {
        const size_t idx = ((size_t)1 << depth) + branch - 1;
        uint32_t* node = tree + 4 * idx;
        node[1] = 0;
        node[2] = (uint32_t)(((size_t)1 << (depth + 1)) + 2 * branch - 1);
        node[3] = (uint32_t)(((size_t)1 << (depth + 1)) + 2 * branch);
        planes[idx] = 0.0f;
        const uint32_t n = (uint32_t)objs.size();
        if (n <= max_leaf || depth == max_depth) {   // :204-211
            node[0] = 3u + (n << 2);
            out.push_back(Leaf{idx, std::move(objs)});
            return;
        }
        // gather the node's boxes contiguously (SoA) for the 9 candidate sweeps
        std::vector<float> lo[3], hi[3];
        for (int a = 0; a < 3; a++) {
            lo[a].resize(n);
            hi[a].resize(n);
        }
        for (uint32_t j = 0; j < n; j++) {
            const Box& b = boxes[objs[j]];
            for (int a = 0; a < 3; a++) {
                lo[a][j] = b.mn[a];
                hi[a][j] = b.mx[a];
            }
        }
        auto count_in = [&](const Box& s) {
            uint32_t c = 0;
            const float *l0 = lo[0].data(), *l1 = lo[1].data(), *l2 = lo[2].data();
            const float *h0 = hi[0].data(), *h1 = hi[1].data(), *h2 = hi[2].data();
            for (uint32_t j = 0; j < n; j++)
                c += (uint32_t)(!(l0[j] > s.mx[0] || h0[j] < s.mn[0]) && !(l1[j] > s.mx[1] || h1[j] < s.mn[1]) &&
                                !(l2[j] > s.mx[2] || h2[j] < s.mn[2]));
            return c;
        };
        const int tests = 4;
        int axis_leaf = 0;
        float plane = 0.0f;
        uint32_t lnc = 0, rnc = 0;
        float min_cost = 1E+27f;
        for (int i = 0; i < 3; i++)   // :220-249
            for (int k = 1; k < tests; k++) {
                Box lb = bbox, rb = bbox;
                const float max_corner = bbox.mx[i], min_corner = bbox.mn[i];
                const float center = (max_corner - min_corner) * (float)k / (float)tests + min_corner;
                lb.mx[i] = center;
                rb.mn[i] = center;
                const uint32_t lc = count_in(lb), rc = count_in(rb);
                const float cost = (float)(int32_t)lc * area(lb) + (float)(int32_t)rc * area(rb);
                if (cost < min_cost) {
                    min_cost = cost;
                    axis_leaf = i;
                    plane = center;
                    lnc = lc;
                    rnc = rc;
                }
            }
        const float max_corner = bbox.mx[axis_leaf], min_corner = bbox.mn[axis_leaf];   // :252-282
        const float size = max_corner - min_corner;
        const float diff = 1e-6f < (size / 8.0f) ? size / 8.0f : 1e-6f;
        float center = plane;
        if (lnc == 0) {
            center = max_corner;
            for (uint32_t j = 0; j < n; j++)
                if (lo[axis_leaf][j] < center) center = lo[axis_leaf][j];
            center -= diff;
        }
        if (rnc == 0) {
            center = min_corner;
            for (uint32_t j = 0; j < n; j++)
                if (hi[axis_leaf][j] > center) center = hi[axis_leaf][j];
            center += diff;
        }
        plane = center;
        Box lb = bbox, rb = bbox;
        lb.mx[axis_leaf] = center;
        rb.mn[axis_leaf] = center;
        std::vector<uint32_t> lobj, robj;
        lobj.reserve(n);
        robj.reserve(n);
        for (uint32_t j = 0; j < n; j++) {   // :293-300
            const Box& b = boxes[objs[j]];
            if (intersects(lb, b)) lobj.push_back(objs[j]);
            if (intersects(rb, b)) robj.push_back(objs[j]);
        }
        node[0] = (uint32_t)axis_leaf + (n << 2);
        planes[idx] = plane;
        std::vector<uint32_t>().swap(objs);
        for (int a = 0; a < 3; a++) {
            std::vector<float>().swap(lo[a]);
            std::vector<float>().swap(hi[a]);
        }
        if ((int)depth < par_depth && lobj.size() + robj.size() > 4096) {
            std::vector<Leaf> lout;
            auto fut = std::async(std::launch::async, [&]() { build(lb, depth + 1, branch * 2, std::move(lobj), lout); });
            std::vector<Leaf> rout;
            build(rb, depth + 1, branch * 2 + 1, std::move(robj), rout);
            fut.get();
            for (Leaf& l : lout) out.push_back(std::move(l));
            for (Leaf& l : rout) out.push_back(std::move(l));
        } else {
            build(lb, depth + 1, branch * 2, std::move(lobj), out);
            build(rb, depth + 1, branch * 2 + 1, std::move(robj), out);
        }
    }
};

}  // namespace

extern "C" int rt_bsp_build(const rt_mesh_host* mesh, uint32_t max_depth, uint32_t max_leaf, int nthreads,
                            rt_bsp_host** out)
{
    if (!mesh || !out) {
        rthost::set_error("rt_bsp_build: null argument");
        return RT_E_INVALID;
    }
    if (max_depth == 0 || max_depth >= 32 || max_leaf == 0) {   // bsp_tree.rs:51-58
        rthost::set_error("rt_bsp_build: max_depth must be in [1,31], max_leaf > 0");
        return RT_E_INVALID;
    }
    const uint32_t nt = mesh->ntris();
    std::vector<Box> boxes(nt);
    Box root = {{1.0e37f, 1.0e37f, 1.0e37f}, {-1.0e37f, -1.0e37f, -1.0e37f}};   // Bbox::new
    for (uint32_t t = 0; t < nt; t++) {   // Mesh::bboxes, mesh.rs:212-227
        const uint32_t* ix = &mesh->idx[(size_t)t * 4];
        const float* v0 = &mesh->pos[(size_t)ix[0] * 4];
        const float* v1 = &mesh->pos[(size_t)ix[1] * 4];
        const float* v2 = &mesh->pos[(size_t)ix[2] * 4];
        for (int i = 0; i < 3; i++) {
            boxes[t].mn[i] = rt_minf(v0[i], rt_minf(v1[i], v2[i]));
            boxes[t].mx[i] = rt_maxf(v0[i], rt_maxf(v1[i], v2[i]));
        }
        for (int i = 0; i < 3; i++) {
            root.mn[i] = rt_minf(root.mn[i], boxes[t].mn[i]);
            root.mx[i] = rt_maxf(root.mx[i], boxes[t].mx[i]);
        }
    }
    const size_t nn = ((size_t)1 << (max_depth + 1)) - 1;
    rt_bsp_host* b = new rt_bsp_host();
    b->tree.assign(nn * 4, 0u);
    b->planes.assign(nn, 0.0f);
    b->max_depth = max_depth;
    int hw = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    if (hw < 1) hw = 1;
    int pd = 0;
    while ((1 << pd) < hw && pd < 12) pd++;
    Builder B{boxes.data(), b->tree.data(), b->planes.data(), max_depth, max_leaf, pd + 1};
    std::vector<uint32_t> objs(nt);
    for (uint32_t t = 0; t < nt; t++) objs[t] = t;
    std::vector<Leaf> leaves;
    B.build(root, 0, 0, std::move(objs), leaves);
    // DFS pass: leaf first-ids (bsp_array, :143-147) and treeIds (primitive_ids, :79-101)
    size_t total = 0;
    for (const Leaf& l : leaves) total += l.objs.size();
    b->ids.reserve(total);
    uint32_t node_id = 0;
    for (const Leaf& l : leaves) {
        b->tree[4 * l.idx + 1] = node_id;
        node_id += (uint32_t)l.objs.size();
        b->ids.insert(b->ids.end(), l.objs.begin(), l.objs.end());
    }
    b->aabb[0] = root.mn[0];
    b->aabb[1] = root.mn[1];
    b->aabb[2] = root.mn[2];
    b->aabb[3] = 0.0f;
    b->aabb[4] = root.mx[0];
    b->aabb[5] = root.mx[1];
    b->aabb[6] = root.mx[2];
    b->aabb[7] = 0.0f;
    *out = b;
    return RT_OK;
}

extern "C" int rt_bsp_view_get(const rt_bsp_host* b, rt_bsp_view* v)
{
    if (!b || !v) return RT_E_INVALID;
    v->tree = b->tree.data();
    v->planes = b->planes.data();
    v->ids = b->ids.data();
    memcpy(v->aabb, b->aabb, sizeof v->aabb);
    v->nnodes = (uint32_t)b->planes.size();
    v->nids = (uint32_t)b->ids.size();
    v->max_depth = b->max_depth;
    return RT_OK;
}

extern "C" void rt_bsp_free(rt_bsp_host* b) { delete b; }
