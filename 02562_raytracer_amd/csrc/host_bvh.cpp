// host_bvh.cpp -- hlbvh::Bvh::new + flatten + triangles
// (src/data_structures/hlbvh.rs:36-239).
//
// Morton codes (10 bits/axis of the centroid offset, Rust `as u32` saturating
// cast), sort by code, treelets on the top 12 code bits, emit_lbvh per treelet
// (in parallel; each returns its own node count), median-split upper tree,
// DFS flatten.  Orders the reference leaves implementation-defined are fixed:
// equal Morton codes by primitive index, equal centroids by input order.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <future>
#include <memory>
#include <thread>
#include <vector>

#include "../../include/rt_detmath.h"
#include "host_types.h"

namespace {

struct Box {
    float mn[3], mx[3];
};
inline Box box_new() { return Box{{1.0e37f, 1.0e37f, 1.0e37f}, {-1.0e37f, -1.0e37f, -1.0e37f}}; }
inline void include(Box& b, const Box& o)
{
    for (int i = 0; i < 3; i++) {
        b.mn[i] = rt_minf(b.mn[i], o.mn[i]);
        b.mx[i] = rt_maxf(b.mx[i], o.mx[i]);
    }
}
inline void include_v(Box& b, const float* v)
{
    for (int i = 0; i < 3; i++) {
        b.mn[i] = rt_minf(b.mn[i], v[i]);
        b.mx[i] = rt_maxf(b.mx[i], v[i]);
    }
}
inline void center(const Box& b, float* c)
{
    for (int i = 0; i < 3; i++) c[i] = (b.mn[i] + b.mx[i]) * 0.5f;
}

struct MP {
    uint32_t index, code;
};

uint32_t left_shift_3(uint32_t x)   // hlbvh.rs:489-498
{
    if (x == (1u << 10)) x -= 1;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}
uint32_t as_u32(float f)   // Rust `f as u32`
{
    if (!(f > 0.0f)) return 0;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

struct BNode {
    Box bbox;
    bool leaf;
    uint32_t first, n;
    std::unique_ptr<BNode> l, r;
};

std::unique_ptr<BNode> make_internal(std::unique_ptr<BNode> a, std::unique_ptr<BNode> b)
{
    auto x = std::make_unique<BNode>();
    x->bbox = a->bbox;
    include(x->bbox, b->bbox);
    x->leaf = false;
    x->l = std::move(a);
    x->r = std::move(b);
    return x;
}

struct Lbvh {
    const Box* boxes;
    const MP* mp;
    uint32_t max_prims;
    std::unique_ptr<BNode> emit(uint32_t off, uint32_t n, int bit, uint32_t& nodes)   // :348-442
    {
        nodes++;
        if (bit <= -1 || n < max_prims) {
            auto x = std::make_unique<BNode>();
            x->bbox = box_new();
            for (uint32_t i = 0; i < n; i++) include(x->bbox, boxes[mp[off + i].index]);
            x->leaf = true;
            x->first = off;
            x->n = n;
            return x;
        }
        const uint32_t mask = 1u << bit;
        if ((mp[off].code & mask) == (mp[off + n - 1].code & mask)) return emit(off, n, bit - 1, nodes);
        long size = (long)n - 2;
        uint32_t first = 1;
        while (size > 0) {
            const long half = size >> 1;
            const uint32_t middle = first + (uint32_t)half;
            if ((mp[off].code & mask) == (mp[off + middle].code & mask)) {
                first = middle + 1;
                size -= half + 1;
            } else {
                size = half;
            }
        }
        const uint32_t hi = n >= 2 ? n - 2 : 0;
        const uint32_t offset = first > hi ? hi : first;
        auto a = emit(off, offset, bit - 1, nodes);
        auto b = emit(off + offset, n - offset, bit - 1, nodes);
        return make_internal(std::move(a), std::move(b));
    }
};

bool center_less(const Box& a, const Box& b, int dim)   // f32::total_cmp on the centroid
{
    const float ca = (a.mn[dim] + a.mx[dim]) * 0.5f, cb = (b.mn[dim] + b.mx[dim]) * 0.5f;
    if (ca < cb) return true;
    if (ca > cb) return false;
    return signbit(ca) && !signbit(cb);
}

// collapse_build_nodes_recursive + mid_partition (:252-291) over entry indices
// ids[lo, hi); returns the entry index of the subtree root.
int32_t collapse(std::vector<rthost::UpperNode>& e, std::vector<int32_t>& ids, size_t lo, size_t hi, uint32_t& total)
{
    const size_t n = hi - lo;
    if (n == 1) return ids[lo];
    total++;
    Box cb = box_new();
    for (size_t i = lo; i < hi; i++) {
        const Box bx{{e[ids[i]].mn[0], e[ids[i]].mn[1], e[ids[i]].mn[2]}, {e[ids[i]].mx[0], e[ids[i]].mx[1], e[ids[i]].mx[2]}};
        float c[3];
        center(bx, c);
        include_v(cb, c);
    }
    const float d0 = cb.mx[0] - cb.mn[0], d1 = cb.mx[1] - cb.mn[1], d2 = cb.mx[2] - cb.mn[2];
    const int dim = d0 > d1 ? (d0 > d2 ? 0 : 2) : (d1 > d2 ? 1 : 2);   // longest_axis, bbox.rs:128-143
    std::stable_sort(ids.begin() + lo, ids.begin() + hi, [&e, dim](int32_t a, int32_t b) {
        const Box ba{{e[a].mn[0], e[a].mn[1], e[a].mn[2]}, {e[a].mx[0], e[a].mx[1], e[a].mx[2]}};
        const Box bb{{e[b].mn[0], e[b].mn[1], e[b].mn[2]}, {e[b].mx[0], e[b].mx[1], e[b].mx[2]}};
        return center_less(ba, bb, dim);
    });
    const size_t mid = lo + n / 2;
    const int32_t a = collapse(e, ids, lo, mid, total);
    const int32_t b = collapse(e, ids, mid, hi, total);
    rthost::UpperNode x;   // BvhBuildNode::new_internal: bbox = child0's, include child1's
    for (int i = 0; i < 3; i++) {
        x.mn[i] = rt_minf(e[a].mn[i], e[b].mn[i]);
        x.mx[i] = rt_maxf(e[a].mx[i], e[b].mx[i]);
    }
    x.root = -1;
    x.left = a;
    x.right = b;
    e.push_back(x);
    return (int32_t)e.size() - 1;
}

// the root's subtree, rebuilt as BNodes from the upper-tree entries
std::unique_ptr<BNode> to_bnodes(const std::vector<rthost::UpperNode>& e, int32_t i,
                                 std::vector<std::unique_ptr<BNode>>& roots)
{
    if (e[i].root >= 0) return std::move(roots[e[i].root]);
    auto a = to_bnodes(e, e[i].left, roots);
    auto b = to_bnodes(e, e[i].right, roots);
    return make_internal(std::move(a), std::move(b));
}

uint32_t flatten(std::vector<rt_gpu_node>& out, const BNode* b, uint32_t& offset)   // :198-230
{
    const uint32_t cur = offset++;
    uint32_t np, optr;
    if (b->leaf) {
        np = b->n;
        optr = b->first;
    } else {
        flatten(out, b->l.get(), offset);
        optr = flatten(out, b->r.get(), offset);
        np = 0;
    }
    for (int i = 0; i < 3; i++) {
        out[cur].min[i] = b->bbox.mn[i];
        out[cur].max[i] = b->bbox.mx[i];
    }
    out[cur].n_prims = np;
    out[cur].offset_ptr = optr;
    return cur;
}

}  // namespace

extern "C" int rt_bvh_build(const rt_mesh_host* mesh, uint32_t max_prims, rt_bvh_host** out)
{
    if (!mesh || !out || mesh->ntris() == 0) {
        rthost::set_error("rt_bvh_build: empty mesh");
        return RT_E_INVALID;
    }
    if (max_prims == 0) {   // emit_lbvh would read morton_primitives[offset - 1] for an empty range
        rthost::set_error("rt_bvh_build: max_prims must be >= 1");
        return RT_E_INVALID;
    }
    const uint32_t nt = mesh->ntris();
    std::vector<Box> boxes(nt);
    for (uint32_t t = 0; t < nt; t++) {
        const uint32_t* ix = &mesh->idx[(size_t)t * 4];
        const float* v0 = &mesh->pos[(size_t)ix[0] * 4];
        const float* v1 = &mesh->pos[(size_t)ix[1] * 4];
        const float* v2 = &mesh->pos[(size_t)ix[2] * 4];
        for (int i = 0; i < 3; i++) {
            boxes[t].mn[i] = rt_minf(v0[i], rt_minf(v1[i], v2[i]));
            boxes[t].mx[i] = rt_maxf(v0[i], rt_maxf(v1[i], v2[i]));
        }
    }
    Box bound = box_new();
    for (uint32_t t = 0; t < nt; t++) {
        float c[3];
        center(boxes[t], c);
        include_v(bound, c);
    }
    std::vector<MP> mp(nt);
    for (uint32_t t = 0; t < nt; t++) {   // :54-68 with Bbox::offset (bbox.rs:169-181)
        float c[3], o[3];
        center(boxes[t], c);
        for (int i = 0; i < 3; i++) {
            o[i] = c[i] - bound.mn[i];
            if (bound.mx[i] > bound.mn[i]) o[i] /= bound.mx[i] - bound.mn[i];
            o[i] = o[i] * 1024.0f;
        }
        mp[t].index = t;
        mp[t].code = (left_shift_3(as_u32(o[2])) << 2) | (left_shift_3(as_u32(o[1])) << 1) | left_shift_3(as_u32(o[0]));
    }
    std::sort(mp.begin(), mp.end(), [](const MP& a, const MP& b) {
        return a.code != b.code ? a.code < b.code : a.index < b.index;
    });
    // treelets (:100-117)
    const uint32_t mask = 0x3FFC0000u;
    std::vector<std::pair<uint32_t, uint32_t>> tl;
    uint32_t start = 0;
    for (uint32_t end = 1; end <= nt; end++)
        if (end == nt || (mp[start].code & mask) != (mp[end].code & mask)) {
            tl.emplace_back(start, end - start);
            start = end;
        }
    std::vector<std::unique_ptr<BNode>> roots(tl.size());
    std::vector<uint32_t> counts(tl.size(), 0);
    Lbvh L{boxes.data(), mp.data(), max_prims};
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nthr = std::min<size_t>(hw, tl.size());
    std::vector<std::thread> th;
    for (size_t w = 0; w < nthr; w++)
        th.emplace_back([&, w]() {
            for (size_t i = w; i < tl.size(); i += nthr) roots[i] = L.emit(tl[i].first, tl[i].second, 29 - 12, counts[i]);
        });
    for (auto& t : th) t.join();
    uint32_t total = 0;
    for (uint32_t c : counts) total += c;
    std::vector<float> rb(roots.size() * 6);
    for (size_t i = 0; i < roots.size(); i++)
        for (int k = 0; k < 3; k++) {
            rb[i * 6 + k] = roots[i]->bbox.mn[k];
            rb[i * 6 + 3 + k] = roots[i]->bbox.mx[k];
        }
    std::vector<rthost::UpperNode> upper;
    total += rthost::bvh_upper_tree(rb, upper);
    auto root = to_bnodes(upper, 0, roots);
    rt_bvh_host* b = new rt_bvh_host();
    rt_gpu_node filler;   // GpuNode::new(root bbox), :518-525
    for (int i = 0; i < 3; i++) {
        filler.min[i] = root->bbox.mn[i];
        filler.max[i] = root->bbox.mx[i];
    }
    filler.offset_ptr = 9999;
    filler.n_prims = 9999;
    b->nodes.assign(total, filler);
    uint32_t off = 0;
    flatten(b->nodes, root.get(), off);
    b->tri_ids.resize(nt);
    for (uint32_t k = 0; k < nt; k++) b->tri_ids[k] = mp[k].index;
    *out = b;
    return RT_OK;
}

uint32_t rthost::bvh_upper_tree(const std::vector<float>& root_boxes, std::vector<UpperNode>& out)
{
    const size_t n = root_boxes.size() / 6;
    out.clear();
    out.reserve(2 * n);
    std::vector<int32_t> ids(n);
    for (size_t i = 0; i < n; i++) {
        UpperNode x;
        for (int k = 0; k < 3; k++) {
            x.mn[k] = root_boxes[i * 6 + k];
            x.mx[k] = root_boxes[i * 6 + 3 + k];
        }
        x.root = (int32_t)i;
        x.left = x.right = -1;
        out.push_back(x);
        ids[i] = (int32_t)i;
    }
    uint32_t total = 0;
    if (n == 0) return 0;
    const int32_t r = collapse(out, ids, 0, n, total);
    // put the root first: entry 0 <-> r
    if (r != 0) {
        std::swap(out[0], out[(size_t)r]);
        for (auto& x : out) {
            if (x.left == 0) x.left = r; else if (x.left == r) x.left = 0;
            if (x.right == 0) x.right = r; else if (x.right == r) x.right = 0;
        }
    }
    return total;
}

extern "C" int rt_bvh_view_get(const rt_bvh_host* b, rt_bvh_view* v)
{
    if (!b || !v) return RT_E_INVALID;
    v->nodes = b->nodes.data();
    v->tri_ids = b->tri_ids.data();
    v->nnodes = (uint32_t)b->nodes.size();
    v->nids = (uint32_t)b->tri_ids.size();
    return RT_OK;
}

extern "C" void rt_bvh_free(rt_bvh_host* b) { delete b; }
