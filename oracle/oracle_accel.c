/*
 * oracle_accel.c -- TEST INFRASTRUCTURE (see oracle.h header).
 *
 * Literal f32 restatements of the reference's acceleration-structure builders:
 *   - Bbox                src/data_structures/bbox.rs:13-182
 *   - Mesh::bboxes        src/mesh.rs:212-227
 *   - BspTree             src/data_structures/bsp_tree.rs:45-347
 *   - HLBVH               src/data_structures/hlbvh.rs:36-503
 * Rust does not contract a*b+c, so this file must be compiled with
 * -ffp-contract=off to reproduce the reference's f32 results.
 *
 * HLBVH ordering that the reference leaves implementation-defined (rdst radix
 * sort of equal Morton codes, select_nth_unstable of equal centroids) is fixed
 * here as "stable by input order"; the product uses the same rule.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "../include/rt_detmath.h"

typedef struct { float min[3], max[3]; } bbox_t;

static bbox_t bbox_new(void)   /* bbox.rs:45-50 */
{
    bbox_t b = {{1.0e37f, 1.0e37f, 1.0e37f}, {-1.0e37f, -1.0e37f, -1.0e37f}};
    return b;
}
static void bbox_include_bbox(bbox_t* b, const bbox_t* o)   /* bbox.rs:73-81 */
{
    for (int i = 0; i < 3; i++) {
        b->min[i] = rt_minf(b->min[i], o->min[i]);
        b->max[i] = rt_maxf(b->max[i], o->max[i]);
    }
}
static void bbox_include_vertex(bbox_t* b, const float v[3])   /* bbox.rs:62-70 */
{
    for (int i = 0; i < 3; i++) {
        b->min[i] = rt_minf(b->min[i], v[i]);
        b->max[i] = rt_maxf(b->max[i], v[i]);
    }
}
static float bbox_area(const bbox_t* b)   /* bbox.rs:117-125 */
{
    float d0 = b->max[0] - b->min[0], d1 = b->max[1] - b->min[1], d2 = b->max[2] - b->min[2];
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}
static int bbox_intersects(const bbox_t* s, const bbox_t* o)   /* bbox.rs:151-155 */
{
    return !(o->min[0] > s->max[0] || o->max[0] < s->min[0]) &&
           !(o->min[1] > s->max[1] || o->max[1] < s->min[1]) &&
           !(o->min[2] > s->max[2] || o->max[2] < s->min[2]);
}
static void bbox_center(const bbox_t* b, float c[3])   /* bbox.rs:90-92 */
{
    for (int i = 0; i < 3; i++) c[i] = (b->min[i] + b->max[i]) * 0.5f;
}
static int bbox_longest_axis(const bbox_t* b)   /* bbox.rs:128-143 */
{
    float d0 = b->max[0] - b->min[0], d1 = b->max[1] - b->min[1], d2 = b->max[2] - b->min[2];
    if (d0 > d1) return d0 > d2 ? 0 : 2;
    return d1 > d2 ? 1 : 2;
}

/* Mesh::bboxes, mesh.rs:212-227 with Bbox::from_triangle, bbox.rs:54-59 */
static bbox_t* mesh_bboxes(const float* pos, const uint32_t* idx, uint32_t ntris)
{
    bbox_t* b = (bbox_t*)malloc(sizeof(bbox_t) * (ntris ? ntris : 1));
    for (uint32_t t = 0; t < ntris; t++) {
        const float* v0 = pos + 4 * (size_t)idx[4 * t];
        const float* v1 = pos + 4 * (size_t)idx[4 * t + 1];
        const float* v2 = pos + 4 * (size_t)idx[4 * t + 2];
        for (int i = 0; i < 3; i++) {
            b[t].min[i] = rt_minf(v0[i], rt_minf(v1[i], v2[i]));
            b[t].max[i] = rt_maxf(v0[i], rt_maxf(v1[i], v2[i]));
        }
    }
    return b;
}

/* ------------------------------------------------------------------ BSP */

typedef struct {
    const bbox_t* boxes;
    uint32_t* tree;
    float* planes;
    uint32_t* ids;
    size_t nids, cap_ids;
    uint32_t max_depth, max_leaf;
    uint32_t node_id;   /* bsp_array's running leaf id (bsp_tree.rs:145-146) */
} bsp_ctx;

static void push_id(bsp_ctx* c, uint32_t id)
{
    if (c->nids == c->cap_ids) {
        c->cap_ids = c->cap_ids ? c->cap_ids * 2 : 1024;
        c->ids = (uint32_t*)realloc(c->ids, c->cap_ids * sizeof(uint32_t));
    }
    c->ids[c->nids++] = id;
}

/* Node::subdivide_node (bsp_tree.rs:195-323) fused with the DFS of
 * primitive_ids (:79-101) and bsp_array (:120-189): both walk left-first, so
 * leaf first-ids equal the running id count. */
static void subdivide(bsp_ctx* c, bbox_t bbox, uint32_t depth, uint32_t branch, const uint32_t* objs,
                      uint32_t n)
{
    size_t idx = ((size_t)1 << depth) + branch - 1;
    uint32_t* node = c->tree + 4 * idx;
    node[1] = 0;
    node[2] = (uint32_t)(((size_t)1 << (depth + 1)) + 2 * (size_t)branch - 1);
    node[3] = (uint32_t)(((size_t)1 << (depth + 1)) + 2 * (size_t)branch);
    c->planes[idx] = 0.0f;
    if (n <= c->max_leaf || depth == c->max_depth) {
        node[0] = 3u + (n << 2);   /* NODE_TYPE_LEAF + (count << 2), :144 */
        node[1] = c->node_id;
        c->node_id += n;
        for (uint32_t i = 0; i < n; i++) push_id(c, objs[i]);
        return;
    }
    const int tests = 4;
    int axis_leaf = 0;
    float plane = 0.0f;
    int left_node_count = 0, right_node_count = 0;
    float min_cost = 1E+27f;
    for (int i = 0; i < 3; i++) {
        for (int k = 1; k < tests; k++) {
            bbox_t lb = bbox, rb = bbox;
            float max_corner = bbox.max[i], min_corner = bbox.min[i];
            float center = (max_corner - min_corner) * (float)k / (float)tests + min_corner;
            lb.max[i] = center;
            rb.min[i] = center;
            int lc = 0, rc = 0;
            for (uint32_t j = 0; j < n; j++) {
                lc += bbox_intersects(&lb, &c->boxes[objs[j]]);
                rc += bbox_intersects(&rb, &c->boxes[objs[j]]);
            }
            float cost = (float)lc * bbox_area(&lb) + (float)rc * bbox_area(&rb);
            if (cost < min_cost) {
                min_cost = cost;
                axis_leaf = i;
                plane = center;
                left_node_count = lc;
                right_node_count = rc;
            }
        }
    }
    float max_corner = bbox.max[axis_leaf], min_corner = bbox.min[axis_leaf];
    float size = max_corner - min_corner;
    float diff = 1e-6f < (size / 8.0f) ? size / 8.0f : 1e-6f;
    float center = plane;
    if (left_node_count == 0) {
        center = max_corner;
        for (uint32_t j = 0; j < n; j++) {
            float m = c->boxes[objs[j]].min[axis_leaf];
            if (m < center) center = m;
        }
        center -= diff;
    }
    if (right_node_count == 0) {
        center = min_corner;
        for (uint32_t j = 0; j < n; j++) {
            float m = c->boxes[objs[j]].max[axis_leaf];
            if (m > center) center = m;
        }
        center += diff;
    }
    plane = center;
    bbox_t lb = bbox, rb = bbox;
    lb.max[axis_leaf] = center;
    rb.min[axis_leaf] = center;
    uint32_t* lo = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t* ro = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t ln = 0, rn = 0;
    for (uint32_t j = 0; j < n; j++) {
        if (bbox_intersects(&lb, &c->boxes[objs[j]])) lo[ln++] = objs[j];
        if (bbox_intersects(&rb, &c->boxes[objs[j]])) ro[rn++] = objs[j];
    }
    node[0] = (uint32_t)axis_leaf + (n << 2);   /* split + (count << 2), :154 */
    c->planes[idx] = plane;
    subdivide(c, lb, depth + 1, branch * 2, lo, ln);
    free(lo);
    subdivide(c, rb, depth + 1, branch * 2 + 1, ro, rn);
    free(ro);
}

int or_bsp_build(const float* pos, uint32_t nverts, const uint32_t* idx, uint32_t ntris,
                 uint32_t max_depth, uint32_t max_leaf, or_bsp* out)
{
    (void)nverts;
    memset(out, 0, sizeof *out);
    if (max_depth == 0 || max_depth >= 32 || max_leaf == 0) return -1;   /* :46-58 */
    bbox_t* boxes = mesh_bboxes(pos, idx, ntris);
    bbox_t root = bbox_new();
    for (uint32_t t = 0; t < ntris; t++) bbox_include_bbox(&root, &boxes[t]);
    size_t nn = ((size_t)1 << (max_depth + 1)) - 1;
    bsp_ctx c;
    memset(&c, 0, sizeof c);
    c.boxes = boxes;
    c.tree = (uint32_t*)calloc(nn * 4, sizeof(uint32_t));
    c.planes = (float*)calloc(nn, sizeof(float));
    c.max_depth = max_depth;
    c.max_leaf = max_leaf;
    uint32_t* objs = (uint32_t*)malloc(sizeof(uint32_t) * (ntris ? ntris : 1));
    for (uint32_t t = 0; t < ntris; t++) objs[t] = t;
    subdivide(&c, root, 0, 0, objs, ntris);
    free(objs);
    free(boxes);
    out->tree = c.tree;
    out->planes = c.planes;
    out->ids = c.ids ? c.ids : (uint32_t*)calloc(1, sizeof(uint32_t));
    out->nids = (uint32_t)c.nids;
    out->nnodes = (uint32_t)nn;
    out->max_depth = max_depth;
    /* BboxGpu from Bbox (bbox.rs:28-37) */
    out->aabb[0] = root.min[0]; out->aabb[1] = root.min[1]; out->aabb[2] = root.min[2]; out->aabb[3] = 0.0f;
    out->aabb[4] = root.max[0]; out->aabb[5] = root.max[1]; out->aabb[6] = root.max[2]; out->aabb[7] = 0.0f;
    return 0;
}

/* ------------------------------------------------------------------ BSP, f64 (JS) semantics
 * The reference ships a second, runnable implementation of the same builder:
 * the instructor JavaScript js/bsp_tree/modules/BspTree_interleaved.js:28-188
 * (identical copy in js/bsp_tree/BspRunner.js).  It computes in f64 on f32
 * inputs, keeps the f64 plane for the child boxes and stores it rounded to
 * f32 in bspPlanes, and writes an interior node's count as the count its
 * parent evaluated for the chosen candidate (:89-92; the root: all objects).
 * This variant exists only to pin the restatement's structure (candidate
 * order, strict-< cost ties, empty-side handling, inclusive intersects, DFS
 * ids) against fixtures produced by running that JavaScript. */
typedef struct { double min[3], max[3]; } dbox_t;

static int dbox_intersects(const dbox_t* s, const bbox_t* o)
{
    return !((double)o->min[0] > s->max[0] || (double)o->max[0] < s->min[0]) &&
           !((double)o->min[1] > s->max[1] || (double)o->max[1] < s->min[1]) &&
           !((double)o->min[2] > s->max[2] || (double)o->max[2] < s->min[2]);
}
static double dbox_area(const dbox_t* b)
{
    double d0 = b->max[0] - b->min[0], d1 = b->max[1] - b->min[1], d2 = b->max[2] - b->min[2];
    return 2.0 * (d0 * d1 + d1 * d2 + d2 * d0);
}

static void subdivide_js(bsp_ctx* c, dbox_t bbox, uint32_t depth, uint32_t branch, const uint32_t* objs, uint32_t n,
                         uint32_t count_field)
{
    size_t idx = ((size_t)1 << depth) + branch - 1;
    uint32_t* node = c->tree + 4 * idx;
    node[1] = 0;
    node[2] = (uint32_t)(((size_t)1 << (depth + 1)) + 2 * (size_t)branch - 1);
    node[3] = (uint32_t)(((size_t)1 << (depth + 1)) + 2 * (size_t)branch);
    c->planes[idx] = 0.0f;
    if (n <= c->max_leaf || depth == c->max_depth) {
        node[0] = 3u + (n << 2);
        node[1] = (uint32_t)c->nids;   /* node.id = tree_objects.length */
        for (uint32_t i = 0; i < n; i++) push_id(c, objs[i]);
        return;
    }
    int axis_leaf = 0;
    double plane = 0.0;
    int lc_best = 0, rc_best = 0;
    double min_cost = 1.0e27;
    for (int i = 0; i < 3; i++) {
        for (int k = 1; k < 4; k++) {
            dbox_t lb = bbox, rb = bbox;
            double center = (bbox.max[i] - bbox.min[i]) * k / 4 + bbox.min[i];
            lb.max[i] = center;
            rb.min[i] = center;
            int lc = 0, rc = 0;
            for (uint32_t j = 0; j < n; j++) {
                lc += dbox_intersects(&lb, &c->boxes[objs[j]]);
                rc += dbox_intersects(&rb, &c->boxes[objs[j]]);
            }
            double cost = lc * dbox_area(&lb) + rc * dbox_area(&rb);
            if (cost < min_cost) {
                min_cost = cost;
                axis_leaf = i;
                plane = center;
                lc_best = lc;
                rc_best = rc;
            }
        }
    }
    double max_corner = bbox.max[axis_leaf], min_corner = bbox.min[axis_leaf];
    double size = max_corner - min_corner;
    double diff = 1.0e-6 < size / 8.0 ? size / 8.0 : 1.0e-6;
    double center = plane;
    if (lc_best == 0) {
        center = max_corner;
        for (uint32_t j = 0; j < n; j++)
            if ((double)c->boxes[objs[j]].min[axis_leaf] < center) center = c->boxes[objs[j]].min[axis_leaf];
        center -= diff;
    }
    if (rc_best == 0) {
        center = min_corner;
        for (uint32_t j = 0; j < n; j++)
            if ((double)c->boxes[objs[j]].max[axis_leaf] > center) center = c->boxes[objs[j]].max[axis_leaf];
        center += diff;
    }
    dbox_t lb = bbox, rb = bbox;
    lb.max[axis_leaf] = center;
    rb.min[axis_leaf] = center;
    uint32_t* lo = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t* ro = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t ln = 0, rn = 0;
    for (uint32_t j = 0; j < n; j++) {
        if (dbox_intersects(&lb, &c->boxes[objs[j]])) lo[ln++] = objs[j];
        if (dbox_intersects(&rb, &c->boxes[objs[j]])) ro[rn++] = objs[j];
    }
    node[0] = (uint32_t)axis_leaf + (count_field << 2);
    c->planes[idx] = (float)center;
    subdivide_js(c, lb, depth + 1, branch * 2, lo, ln, (uint32_t)lc_best);
    free(lo);
    subdivide_js(c, rb, depth + 1, branch * 2 + 1, ro, rn, (uint32_t)rc_best);
    free(ro);
}

int or_bsp_build_js64(const float* pos, uint32_t nverts, const uint32_t* idx, uint32_t ntris, uint32_t max_depth,
                      uint32_t max_leaf, or_bsp* out)
{
    (void)nverts;
    memset(out, 0, sizeof *out);
    if (max_depth == 0 || max_depth >= 32 || max_leaf == 0) return -1;
    bbox_t* boxes = mesh_bboxes(pos, idx, ntris);
    dbox_t root = {{1.0e37, 1.0e37, 1.0e37}, {-1.0e37, -1.0e37, -1.0e37}};
    for (uint32_t t = 0; t < ntris; t++)
        for (int i = 0; i < 3; i++) {
            if ((double)boxes[t].min[i] < root.min[i]) root.min[i] = boxes[t].min[i];
            if ((double)boxes[t].max[i] > root.max[i]) root.max[i] = boxes[t].max[i];
        }
    size_t nn = ((size_t)1 << (max_depth + 1)) - 1;
    bsp_ctx c;
    memset(&c, 0, sizeof c);
    c.boxes = boxes;
    c.tree = (uint32_t*)calloc(nn * 4, sizeof(uint32_t));
    c.planes = (float*)calloc(nn, sizeof(float));
    c.max_depth = max_depth;
    c.max_leaf = max_leaf;
    uint32_t* objs = (uint32_t*)malloc(sizeof(uint32_t) * (ntris ? ntris : 1));
    for (uint32_t t = 0; t < ntris; t++) objs[t] = t;
    subdivide_js(&c, root, 0, 0, objs, ntris, ntris);
    free(objs);
    free(boxes);
    out->tree = c.tree;
    out->planes = c.planes;
    out->ids = c.ids ? c.ids : (uint32_t*)calloc(1, sizeof(uint32_t));
    out->nids = (uint32_t)c.nids;
    out->nnodes = (uint32_t)nn;
    out->max_depth = max_depth;
    for (int i = 0; i < 3; i++) {
        out->aabb[i] = (float)root.min[i];
        out->aabb[4 + i] = (float)root.max[i];
    }
    return 0;
}

void or_free_bsp(or_bsp* b)
{
    free(b->tree); free(b->planes); free(b->ids);
    memset(b, 0, sizeof *b);
}

/* ------------------------------------------------------------------ HLBVH */

typedef struct { uint32_t index, code; } morton_t;

typedef struct bnode {
    bbox_t bbox;
    int leaf;
    uint32_t first, n;          /* leaf */
    struct bnode *left, *right; /* interior */
} bnode;

static uint32_t left_shift_3(uint32_t x)   /* hlbvh.rs:489-498 */
{
    if (x == (1u << 10)) x -= 1;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}
static uint32_t rust_as_u32(float f)   /* Rust `f as u32`: saturating, NaN -> 0 */
{
    if (!(f > 0.0f)) return 0;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}
static uint32_t encode_morton_3(float x, float y, float z)   /* hlbvh.rs:501-503 */
{
    return (left_shift_3(rust_as_u32(z)) << 2) | (left_shift_3(rust_as_u32(y)) << 1) |
           left_shift_3(rust_as_u32(x));
}

typedef struct {
    const bbox_t* boxes;
    const morton_t* mp;
    uint32_t max_prims;
    uint32_t total_nodes;
} lbvh_ctx;

static bnode* new_leaf(uint32_t first, uint32_t n, bbox_t b)
{
    bnode* x = (bnode*)calloc(1, sizeof(bnode));
    x->leaf = 1;
    x->first = first;
    x->n = n;
    x->bbox = b;
    return x;
}
static bnode* new_internal(bnode* a, bnode* b)   /* hlbvh.rs:332-344 */
{
    bnode* x = (bnode*)calloc(1, sizeof(bnode));
    x->bbox = a->bbox;
    bbox_include_bbox(&x->bbox, &b->bbox);
    x->left = a;
    x->right = b;
    return x;
}

/* emit_lbvh, hlbvh.rs:348-442 */
static bnode* emit_lbvh(lbvh_ctx* c, uint32_t off, uint32_t n, int bit)
{
    c->total_nodes++;
    if (bit <= -1 || n < c->max_prims) {
        bbox_t b = bbox_new();
        for (uint32_t i = 0; i < n; i++) bbox_include_bbox(&b, &c->boxes[c->mp[off + i].index]);
        return new_leaf(off, n, b);
    }
    uint32_t mask = 1u << bit;
    if ((c->mp[off].code & mask) == (c->mp[off + n - 1].code & mask))
        return emit_lbvh(c, off, n, bit - 1);
    /* binary search for the split (:389-408) */
    long size = (long)n - 2;
    uint32_t first = 1;
    while (size > 0) {
        long half = size >> 1;
        uint32_t middle = first + (uint32_t)half;
        int result = (c->mp[off].code & mask) == (c->mp[off + middle].code & mask);
        if (result) {
            first = middle + 1;
            size = size - (half + 1);
        } else {
            size = half;
        }
    }
    uint32_t hi = n >= 2 ? n - 2 : 0;
    uint32_t offset = first > hi ? hi : first;
    bnode* l = emit_lbvh(c, off, offset, bit - 1);
    bnode* r = emit_lbvh(c, off + offset, n - offset, bit - 1);
    return new_internal(l, r);
}

static int center_cmp_dim;
static int cmp_center(const void* a, const void* b)
{
    /* f32::total_cmp on the centroid; ties keep input order (index tie-break) */
    const bnode* x = *(bnode* const*)((const char*)a);
    const bnode* y = *(bnode* const*)((const char*)b);
    float cx = (x->bbox.min[center_cmp_dim] + x->bbox.max[center_cmp_dim]) * 0.5f;
    float cy = (y->bbox.min[center_cmp_dim] + y->bbox.max[center_cmp_dim]) * 0.5f;
    if (cx < cy) return -1;
    if (cx > cy) return 1;
    int sx = signbit(cx) != 0, sy = signbit(cy) != 0;
    if (sx != sy) return sx ? -1 : 1;
    return 0;
}

/* stable merge sort of node pointers by centroid[dim] */
static void sort_nodes(bnode** a, size_t n, int dim)
{
    if (n < 2) return;
    bnode** tmp = (bnode**)malloc(n * sizeof(bnode*));
    center_cmp_dim = dim;
    for (size_t w = 1; w < n; w *= 2) {
        for (size_t lo = 0; lo < n; lo += 2 * w) {
            size_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
            size_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi) tmp[k++] = cmp_center(&a[j], &a[i]) < 0 ? a[j++] : a[i++];
            while (i < mid) tmp[k++] = a[i++];
            while (j < hi) tmp[k++] = a[j++];
        }
        memcpy(a, tmp, n * sizeof(bnode*));
    }
    free(tmp);
}

/* collapse_build_nodes_recursive + mid_partition, hlbvh.rs:252-291 */
static bnode* collapse(bnode** nodes, size_t n, uint32_t* total)
{
    if (n == 1) return nodes[0];
    (*total)++;
    bbox_t cb = bbox_new();
    for (size_t i = 0; i < n; i++) {
        float c[3];
        bbox_center(&nodes[i]->bbox, c);
        bbox_include_vertex(&cb, c);
    }
    int dim = bbox_longest_axis(&cb);
    size_t mid = n / 2;
    sort_nodes(nodes, n, dim);
    bnode* l = collapse(nodes, mid, total);
    bnode* r = collapse(nodes + mid, n - mid, total);
    return new_internal(l, r);
}

static uint32_t flatten_rec(or_gpu_node* out, const bnode* b, uint32_t* offset)   /* :198-230 */
{
    uint32_t cur = (*offset)++;
    uint32_t np, optr;
    if (b->leaf) {
        np = b->n;
        optr = b->first;
    } else {
        flatten_rec(out, b->left, offset);
        optr = flatten_rec(out, b->right, offset);
        np = 0;
    }
    for (int i = 0; i < 3; i++) {
        out[cur].min[i] = b->bbox.min[i];
        out[cur].max[i] = b->bbox.max[i];
    }
    out[cur].n_prims = np;
    out[cur].offset_ptr = optr;
    return cur;
}

static void free_tree(bnode* b)
{
    if (!b) return;
    free_tree(b->left);
    free_tree(b->right);
    free(b);
}

static int cmp_morton(const void* a, const void* b)
{
    const morton_t* x = (const morton_t*)a;
    const morton_t* y = (const morton_t*)b;
    if (x->code != y->code) return x->code < y->code ? -1 : 1;
    return x->index < y->index ? -1 : (x->index > y->index);
}

int or_bvh_build(const float* pos, uint32_t nverts, const uint32_t* idx, uint32_t ntris,
                 uint32_t max_prims, or_bvh* out)
{
    (void)nverts;
    memset(out, 0, sizeof *out);
    if (ntris == 0) return -1;
    bbox_t* boxes = mesh_bboxes(pos, idx, ntris);
    bbox_t bound = bbox_new();   /* :41-44 */
    for (uint32_t t = 0; t < ntris; t++) {
        float c[3];
        bbox_center(&boxes[t], c);
        bbox_include_vertex(&bound, c);
    }
    morton_t* mp = (morton_t*)malloc(sizeof(morton_t) * ntris);
    for (uint32_t t = 0; t < ntris; t++) {   /* :54-68 with Bbox::offset, bbox.rs:169-181 */
        float c[3], o[3];
        bbox_center(&boxes[t], c);
        for (int i = 0; i < 3; i++) {
            o[i] = c[i] - bound.min[i];
            if (bound.max[i] > bound.min[i]) o[i] /= bound.max[i] - bound.min[i];
            o[i] = o[i] * 1024.0f;
        }
        mp[t].index = t;
        mp[t].code = encode_morton_3(o[0], o[1], o[2]);
    }
    qsort(mp, ntris, sizeof(morton_t), cmp_morton);   /* :75-90, ties by index */

    /* treelets on the top 12 bits (:100-117) */
    const uint32_t mask = 0x3FFC0000u;
    lbvh_ctx c = {boxes, mp, max_prims, 0};
    size_t cap = 64, nt = 0;
    bnode** roots = (bnode**)malloc(cap * sizeof(bnode*));
    uint32_t start = 0;
    for (uint32_t end = 1; end <= ntris; end++) {
        if (end == ntris || (mp[start].code & mask) != (mp[end].code & mask)) {
            if (nt == cap) {
                cap *= 2;
                roots = (bnode**)realloc(roots, cap * sizeof(bnode*));
            }
            roots[nt++] = emit_lbvh(&c, start, end - start, 29 - 12);
            start = end;
        }
    }
    uint32_t total = c.total_nodes;
    bnode** work = (bnode**)malloc(nt * sizeof(bnode*));
    memcpy(work, roots, nt * sizeof(bnode*));
    bnode* root = collapse(work, nt, &total);
    free(work);
    free(roots);

    out->nnodes = total;
    out->nodes = (or_gpu_node*)malloc(sizeof(or_gpu_node) * total);
    for (uint32_t i = 0; i < total; i++) {   /* GpuNode::new(root bbox), :518-525 */
        for (int k = 0; k < 3; k++) {
            out->nodes[i].min[k] = root->bbox.min[k];
            out->nodes[i].max[k] = root->bbox.max[k];
        }
        out->nodes[i].offset_ptr = 9999;
        out->nodes[i].n_prims = 9999;
    }
    uint32_t offset = 0;
    flatten_rec(out->nodes, root, &offset);
    out->nids = ntris;
    out->tri_ids = (uint32_t*)malloc(sizeof(uint32_t) * ntris);
    for (uint32_t k = 0; k < ntris; k++) out->tri_ids[k] = mp[k].index;   /* triangles(), :237-239 */
    free_tree(root);
    free(mp);
    free(boxes);
    return 0;
}

void or_free_bvh(or_bvh* b)
{
    free(b->nodes); free(b->tri_ids);
    memset(b, 0, sizeof *b);
}
