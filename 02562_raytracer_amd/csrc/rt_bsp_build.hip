// rt_bsp_build.hip -- BSP construction on the GPU:
// BspTree::new + bsp_array + primitive_ids (src/data_structures/bsp_tree.rs:
// 45-189, subdivide_node :195-323) producing the same arrays as the host
// builder (host_bsp.cpp, pinned to the oracle and the reference's JS builder).
//
// subdivide_node is breadth-first here: one pass per depth over every node of
// that depth, with the node's objects as one contiguous segment of a per-level
// slot array (in the reference's order).  Per level:
//   k_bsp_count     the 9 candidate planes x (left, right) membership counts
//                   of every splittable node (wave-level segmented popcounts,
//                   block-level accumulation for the block's first node)
//   k_bsp_decide    leaf test (:204), the strict-< min-cost candidate in
//                   (axis, k) order (:220-249), leaf records
//   k_bsp_extent    min lo / max hi along the chosen axis, only for nodes
//                   with an empty side (:251-282)
//   k_bsp_finalize  the moved plane, bsp_array node + plane
//   k_bsp_flags     membership of every object in the two children (:293-300)
//   scans           per-slot ranks, per-node child counts and child offsets
//   k_bsp_children, k_bsp_scatter   next level's nodes and segments (left
//                   child then right child, objects in order)
// Finally the leaves are sorted into DFS order (key = branch << (D - depth))
// and their first ids (:143-147) and primitive_ids (:79-101) follow from one
// scan.  Node slots are fixed by (depth, branch) (idx = 2^depth + branch - 1),
// so only the first ids depend on DFS order.
// Numerics: the same f32 expressions as the host builder, -ffp-contract=off.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/rt_detmath.h"
#include "rt_internal.h"

namespace rtbsp {

struct LNode {                 // a node of the current level
    uint32_t idx;              // bsp_array slot (0-based heap index)
    uint32_t seg, cnt;         // its objects: slots[seg, seg + cnt)
    uint32_t flags;            // 1: split, 2: needs the extent along its axis
    float mn[3], mx[3];        // node box
    uint32_t axis;
    float plane;
    uint32_t lnc, rnc;         // candidate counts (empty-side test)
    uint32_t cntL, cntR;       // final child object counts
    uint32_t child, cseg;      // next level: left child's node index and first slot
};
struct Leaf {
    uint32_t idx, level, seg, cnt;
};
constexpr uint32_t F_SPLIT = 1u, F_EXT = 2u;

__device__ __forceinline__ uint32_t ord_f(float f)   // monotone float -> u32 (non-NaN)
{
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord_f(uint32_t u)
{
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ __forceinline__ float area6(const float* mn, const float* mx)   // bbox.rs:117-125
{
    const float d0 = mx[0] - mn[0], d1 = mx[1] - mn[1], d2 = mx[2] - mn[2];
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}
__device__ __forceinline__ bool isect(const float* smn, const float* smx, const float4 omn, const float4 omx)
{   // bbox.rs:151-155, s.intersects(o)
    return !(omn.x > smx[0] || omx.x < smn[0]) && !(omn.y > smx[1] || omx.y < smn[1]) &&
           !(omn.z > smx[2] || omx.z < smn[2]);
}
__device__ __forceinline__ float comp4(const float4 v, uint32_t a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

// ---- triangle boxes and the root box (Mesh::bboxes; BspTree::new :59-63)
// The root box fold is evaluated as the reference's sequential fold: each
// thread folds a contiguous range from Bbox::new(), and partial results are
// combined left (earlier) to right in adjacent pairs, so ties keep the
// earliest value exactly as include_bbox in index order does.
__global__ void __launch_bounds__(256) k_tri_boxes(const float4* pos, const uint4* idx, uint32_t nt, uint32_t per,
                                                   float4* boxes, float* partial)
{
    __shared__ float red[6][256];
    const uint32_t t0 = (blockIdx.x * 256u + threadIdx.x) * per;
    float bmn[3] = {1.0e37f, 1.0e37f, 1.0e37f}, bmx[3] = {-1.0e37f, -1.0e37f, -1.0e37f};
    for (uint32_t t = t0; t < t0 + per && t < nt; t++) {
        const uint4 ix = idx[t];
        const float4 a = pos[ix.x], b = pos[ix.y], c = pos[ix.z];
        const float mn[3] = {rt_minf(a.x, rt_minf(b.x, c.x)), rt_minf(a.y, rt_minf(b.y, c.y)),
                             rt_minf(a.z, rt_minf(b.z, c.z))};
        const float mx[3] = {rt_maxf(a.x, rt_maxf(b.x, c.x)), rt_maxf(a.y, rt_maxf(b.y, c.y)),
                             rt_maxf(a.z, rt_maxf(b.z, c.z))};
        boxes[2u * t] = make_float4(mn[0], mn[1], mn[2], 0.0f);
        boxes[2u * t + 1u] = make_float4(mx[0], mx[1], mx[2], 0.0f);
        for (int i = 0; i < 3; i++) {
            bmn[i] = rt_minf(bmn[i], mn[i]);
            bmx[i] = rt_maxf(bmx[i], mx[i]);
        }
    }
    for (int i = 0; i < 3; i++) {
        red[i][threadIdx.x] = bmn[i];
        red[3 + i][threadIdx.x] = bmx[i];
    }
    __syncthreads();
    for (uint32_t s = 1; s < 256u; s <<= 1) {   // adjacent pairs: [t] op [t+s], t % 2s == 0
        if ((threadIdx.x & (2u * s - 1u)) == 0u)
            for (int i = 0; i < 3; i++) {
                red[i][threadIdx.x] = rt_minf(red[i][threadIdx.x], red[i][threadIdx.x + s]);
                red[3 + i][threadIdx.x] = rt_maxf(red[3 + i][threadIdx.x], red[3 + i][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) partial[blockIdx.x * 6u + threadIdx.x] = red[threadIdx.x][0];
}

// final fold of the per-block partials (in block order) into the root node
__global__ void k_root(const float* partial, uint32_t nparts, uint32_t nt, LNode* nodes, uint32_t* slots,
                       uint32_t* nos, float* aabb)
{
    if (threadIdx.x != 0) return;
    float v[6] = {1.0e37f, 1.0e37f, 1.0e37f, -1.0e37f, -1.0e37f, -1.0e37f};
    for (uint32_t p = 0; p < nparts; p++)
        for (int i = 0; i < 3; i++) {
            v[i] = rt_minf(v[i], partial[p * 6u + i]);
            v[3 + i] = rt_maxf(v[3 + i], partial[p * 6u + 3 + i]);
        }
    LNode r;
    r.idx = 0;
    r.seg = 0;
    r.cnt = nt;
    r.flags = 0;
    for (int i = 0; i < 3; i++) {
        r.mn[i] = v[i];
        r.mx[i] = v[3 + i];
    }
    r.axis = 0;
    r.plane = 0.0f;
    r.lnc = r.rnc = r.cntL = r.cntR = r.child = r.cseg = 0;
    nodes[0] = r;
    aabb[0] = v[0];
    aabb[1] = v[1];
    aabb[2] = v[2];
    aabb[3] = 0.0f;
    aabb[4] = v[3];
    aabb[5] = v[4];
    aabb[6] = v[5];
    aabb[7] = 0.0f;
}

__global__ void __launch_bounds__(256) k_iota(uint32_t* slots, uint32_t* nos, uint32_t n)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        slots[i] = i;
        nos[i] = 0;
    }
}

__device__ __forceinline__ bool splittable(const LNode& nd, uint32_t depth, uint32_t max_depth, uint32_t max_leaf)
{
    return !(nd.cnt <= max_leaf || depth == max_depth);   // :204
}

// ---- candidate counts: 18 per node, counts[node * 18 + c], c = axis*3 + (k-1) (left), 9 + ... (right)
constexpr uint32_t kSlotsPerBlock = 4096;   // 4 waves x 16 rounds x 64
__global__ void __launch_bounds__(256) k_bsp_count(const uint32_t* slots, const uint32_t* nos, uint32_t n,
                                                   const LNode* nodes, const float4* boxes, uint32_t depth,
                                                   uint32_t max_depth, uint32_t max_leaf, uint32_t* counts)
{
    __shared__ uint32_t acc[18];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t base = blockIdx.x * kSlotsPerBlock;
    if (threadIdx.x < 18) acc[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t first = nos[base];   // base < n by the grid
    for (uint32_t r = 0; r < 16u; r++) {
        const uint32_t slot = base + wave * 1024u + r * 64u + lane;
        const bool valid = slot < n;
        const uint32_t node = valid ? nos[slot] : 0xFFFFFFFFu;
        uint32_t bits = 0;
        if (valid) {
            const LNode& nd = nodes[node];
            if (splittable(nd, depth, max_depth, max_leaf)) {
                const uint32_t o = slots[slot];
                const float4 omn = boxes[2u * o], omx = boxes[2u * o + 1u];
                const bool ok0 = !(omn.x > nd.mx[0] || omx.x < nd.mn[0]);
                const bool ok1 = !(omn.y > nd.mx[1] || omx.y < nd.mn[1]);
                const bool ok2 = !(omn.z > nd.mx[2] || omx.z < nd.mn[2]);
                for (uint32_t i = 0; i < 3; i++) {
                    const bool others = (i == 0 ? ok1 && ok2 : (i == 1 ? ok0 && ok2 : ok0 && ok1));
                    const float lo = comp4(omn, i), hi = comp4(omx, i);
                    for (uint32_t k = 1; k < 4; k++) {
                        const float c = (nd.mx[i] - nd.mn[i]) * (float)k / (float)4 + nd.mn[i];
                        const bool inl = others && !(lo > c || hi < nd.mn[i]);
                        const bool inr = others && !(lo > nd.mx[i] || hi < c);
                        bits |= (inl ? 1u : 0u) << (i * 3u + k - 1u);
                        bits |= (inr ? 1u : 0u) << (9u + i * 3u + k - 1u);
                    }
                }
            }
        }
        const uint32_t prev = __shfl_up(node, 1, 64);
        const bool head = valid && (lane == 0 || prev != node);
        const uint64_t heads = __ballot(head);
        const uint64_t vmask = __ballot(valid);
        uint64_t seg = 0;
        if (head) {
            const uint64_t above = lane == 63 ? 0ull : (heads >> (lane + 1u)) << (lane + 1u);
            const uint32_t end = above ? (uint32_t)__ffsll((unsigned long long)above) - 1u : 64u;
            const uint64_t upto = end >= 64u ? ~0ull : ((1ull << end) - 1ull);
            seg = upto & ~((1ull << lane) - 1ull) & vmask;
        }
        for (uint32_t c = 0; c < 18u; c++) {
            const uint64_t b = __ballot((bits >> c) & 1u);
            if (head && b) {
                const uint32_t cnt = (uint32_t)__popcll(b & seg);
                if (cnt) {
                    if (node == first) atomicAdd(&acc[c], cnt);
                    else atomicAdd(&counts[(size_t)node * 18u + c], cnt);
                }
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < 18 && acc[threadIdx.x]) atomicAdd(&counts[(size_t)first * 18u + threadIdx.x], acc[threadIdx.x]);
}

// ---- leaf test and the candidate choice (:204-249); leaves are final here
__global__ void __launch_bounds__(256) k_bsp_decide(LNode* nodes, uint32_t nn, const uint32_t* counts, uint32_t depth,
                                                    uint32_t max_depth, uint32_t max_leaf, uint32_t* tree,
                                                    float* planes, uint32_t* ext, Leaf* leaves, uint32_t* leaf_keys,
                                                    uint32_t* leaf_ctr)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nn; i += gridDim.x * 256u) {
        LNode nd = nodes[i];
        uint32_t* t = tree + 4u * (size_t)nd.idx;
        t[1] = 0u;
        t[2] = 2u * nd.idx + 1u;
        t[3] = 2u * nd.idx + 2u;
        planes[nd.idx] = 0.0f;
        if (!splittable(nd, depth, max_depth, max_leaf)) {
            t[0] = 3u + (nd.cnt << 2);
            const uint32_t li = atomicAdd(leaf_ctr, 1u);
            leaves[li] = Leaf{nd.idx, depth, nd.seg, nd.cnt};
            const uint32_t branch = nd.idx + 1u - (1u << depth);
            leaf_keys[li] = branch << (max_depth - depth);   // DFS order of the leaves
            nd.flags = 0;
            nodes[i] = nd;
            continue;
        }
        const uint32_t* cn = counts + (size_t)i * 18u;
        uint32_t axis_leaf = 0, lnc = 0, rnc = 0;
        float plane = 0.0f, min_cost = 1E+27f;
        for (uint32_t a = 0; a < 3; a++)
            for (uint32_t k = 1; k < 4; k++) {
                float lmn[3] = {nd.mn[0], nd.mn[1], nd.mn[2]}, lmx[3] = {nd.mx[0], nd.mx[1], nd.mx[2]};
                float rmn[3] = {nd.mn[0], nd.mn[1], nd.mn[2]}, rmx[3] = {nd.mx[0], nd.mx[1], nd.mx[2]};
                const float c = (nd.mx[a] - nd.mn[a]) * (float)k / (float)4 + nd.mn[a];
                lmx[a] = c;
                rmn[a] = c;
                const uint32_t lc = cn[a * 3u + k - 1u], rc = cn[9u + a * 3u + k - 1u];
                const float cost = (float)(int32_t)lc * area6(lmn, lmx) + (float)(int32_t)rc * area6(rmn, rmx);
                if (cost < min_cost) {
                    min_cost = cost;
                    axis_leaf = a;
                    plane = c;
                    lnc = lc;
                    rnc = rc;
                }
            }
        nd.axis = axis_leaf;
        nd.plane = plane;
        nd.lnc = lnc;
        nd.rnc = rnc;
        nd.flags = F_SPLIT | ((lnc == 0u || rnc == 0u) ? F_EXT : 0u);
        ext[2u * i] = ord_f(nd.mx[axis_leaf]);        // lnc == 0: min(max_corner, objects' lo)
        ext[2u * i + 1u] = ord_f(nd.mn[axis_leaf]);   // rnc == 0: max(min_corner, objects' hi)
        nodes[i] = nd;
    }
}

__global__ void __launch_bounds__(256) k_bsp_extent(const uint32_t* slots, const uint32_t* nos, uint32_t n,
                                                    const LNode* nodes, const float4* boxes, uint32_t* ext)
{
    for (uint32_t s = blockIdx.x * 256u + threadIdx.x; s < n; s += gridDim.x * 256u) {
        const uint32_t node = nos[s];
        const LNode& nd = nodes[node];
        if (!(nd.flags & F_EXT)) continue;
        const uint32_t o = slots[s];
        if (nd.lnc == 0u) atomicMin(&ext[2u * node], ord_f(comp4(boxes[2u * o], nd.axis)));
        if (nd.rnc == 0u) atomicMax(&ext[2u * node + 1u], ord_f(comp4(boxes[2u * o + 1u], nd.axis)));
    }
}

// the moved plane (:251-282) and the split node's bsp_array entry
__global__ void __launch_bounds__(256) k_bsp_finalize(LNode* nodes, uint32_t nn, const uint32_t* ext, uint32_t* tree,
                                                      float* planes)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nn; i += gridDim.x * 256u) {
        LNode nd = nodes[i];
        if (!(nd.flags & F_SPLIT)) continue;
        const float max_corner = nd.mx[nd.axis], min_corner = nd.mn[nd.axis];
        const float size = max_corner - min_corner;
        const float diff = 1e-6f < (size / 8.0f) ? size / 8.0f : 1e-6f;
        float center = nd.plane;
        if (nd.lnc == 0u) center = unord_f(ext[2u * i]) - diff;
        if (nd.rnc == 0u) center = unord_f(ext[2u * i + 1u]) + diff;
        nd.plane = center;
        tree[4u * (size_t)nd.idx] = nd.axis + (nd.cnt << 2);
        planes[nd.idx] = center;
        nodes[i] = nd;
    }
}

// membership in the two children (:293-300): fl/fr[slot] in {0, 1}; fl[n] = fr[n] = 0
__global__ void __launch_bounds__(256) k_bsp_flags(const uint32_t* slots, const uint32_t* nos, uint32_t n,
                                                   const LNode* nodes, const float4* boxes, uint32_t* fl, uint32_t* fr)
{
    for (uint32_t s = blockIdx.x * 256u + threadIdx.x; s <= n; s += gridDim.x * 256u) {
        uint32_t l = 0, r = 0;
        if (s < n) {
            const LNode& nd = nodes[nos[s]];
            if (nd.flags & F_SPLIT) {
                const uint32_t o = slots[s];
                const float4 omn = boxes[2u * o], omx = boxes[2u * o + 1u];
                float lmx[3] = {nd.mx[0], nd.mx[1], nd.mx[2]}, rmn[3] = {nd.mn[0], nd.mn[1], nd.mn[2]};
                lmx[nd.axis] = nd.plane;
                rmn[nd.axis] = nd.plane;
                l = isect(nd.mn, lmx, omn, omx) ? 1u : 0u;
                r = isect(rmn, nd.mx, omn, omx) ? 1u : 0u;
            }
        }
        fl[s] = l;
        fr[s] = r;
    }
}

// child object counts from the scanned flags; a[i] = 2 children, b[i] = their objects
__global__ void __launch_bounds__(256) k_bsp_child_counts(LNode* nodes, uint32_t nn, const uint32_t* el,
                                                          const uint32_t* er, uint32_t* a, uint32_t* b)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i <= nn; i += gridDim.x * 256u) {
        if (i == nn) {
            a[i] = 0;
            b[i] = 0;
            continue;
        }
        LNode nd = nodes[i];
        if (!(nd.flags & F_SPLIT)) {
            a[i] = 0;
            b[i] = 0;
            continue;
        }
        nd.cntL = el[nd.seg + nd.cnt] - el[nd.seg];
        nd.cntR = er[nd.seg + nd.cnt] - er[nd.seg];
        a[i] = 2;
        b[i] = nd.cntL + nd.cntR;
        nodes[i] = nd;
    }
}

// next level's nodes: left child then right child, boxes split at the plane
__global__ void __launch_bounds__(256) k_bsp_children(LNode* nodes, uint32_t nn, const uint32_t* ea, const uint32_t* eb,
                                                      LNode* next)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nn; i += gridDim.x * 256u) {
        LNode nd = nodes[i];
        if (!(nd.flags & F_SPLIT)) continue;
        nd.child = ea[i];
        nd.cseg = eb[i];
        nodes[i] = nd;
        LNode l, r;
        for (int k = 0; k < 3; k++) {
            l.mn[k] = r.mn[k] = nd.mn[k];
            l.mx[k] = r.mx[k] = nd.mx[k];
        }
        l.mx[nd.axis] = nd.plane;
        r.mn[nd.axis] = nd.plane;
        l.idx = 2u * nd.idx + 1u;
        r.idx = 2u * nd.idx + 2u;
        l.seg = nd.cseg;
        l.cnt = nd.cntL;
        r.seg = nd.cseg + nd.cntL;
        r.cnt = nd.cntR;
        l.flags = r.flags = 0;
        l.axis = r.axis = 0;
        l.plane = r.plane = 0.0f;
        l.lnc = l.rnc = l.cntL = l.cntR = l.child = l.cseg = 0;
        r.lnc = r.rnc = r.cntL = r.cntR = r.child = r.cseg = 0;
        next[nd.child] = l;
        next[nd.child + 1u] = r;
    }
}

__global__ void __launch_bounds__(256) k_bsp_scatter(const uint32_t* slots, const uint32_t* nos, uint32_t n,
                                                     const LNode* nodes, const uint32_t* el, const uint32_t* er,
                                                     uint32_t* nslots, uint32_t* nnos)
{
    for (uint32_t s = blockIdx.x * 256u + threadIdx.x; s < n; s += gridDim.x * 256u) {
        const LNode& nd = nodes[nos[s]];
        if (!(nd.flags & F_SPLIT)) continue;
        const uint32_t o = slots[s];
        if (el[s + 1u] != el[s]) {
            const uint32_t p = nd.cseg + (el[s] - el[nd.seg]);
            nslots[p] = o;
            nnos[p] = nd.child;
        }
        if (er[s + 1u] != er[s]) {
            const uint32_t p = nd.cseg + nd.cntL + (er[s] - er[nd.seg]);
            nslots[p] = o;
            nnos[p] = nd.child + 1u;
        }
    }
}

// ---- flatten: leaves in DFS order -> first ids and primitive_ids
__global__ void __launch_bounds__(256) k_leaf_counts(const Leaf* leaves, const uint32_t* order, uint32_t nl,
                                                     uint32_t* cnt)
{
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < nl; j += gridDim.x * 256u) cnt[j] = leaves[order[j]].cnt;
}

__global__ void __launch_bounds__(256) k_leaf_finish(const Leaf* leaves, const uint32_t* order, uint32_t nl,
                                                     const uint32_t* first, uint32_t* const* level_slots,
                                                     uint32_t* tree, uint32_t* ids)
{
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < nl; j += gridDim.x * 256u) {
        const Leaf lf = leaves[order[j]];
        const uint32_t f = first[j];
        tree[4u * (size_t)lf.idx + 1u] = f;
        const uint32_t* src = level_slots[lf.level] + lf.seg;
        for (uint32_t t = 0; t < lf.cnt; t++) ids[f + t] = src[t];
    }
}

}  // namespace rtbsp

namespace rtk {

// rt_upload_bsp's repack on device: the 96-B treelet of every 1-based node M
// (M's content box and certification data, nodes M, 2M, 2M+1, 4M..4M+3 as 8-B
// entries) and the 48-B triangle records.
// Content box of every node's subtree: the union of the bounding boxes of the
// triangles its leaves reference (2 x float4 per node: min, max; empty: +inf /
// -inf).  The BSP walk skips a subtree whose box the ray interval misses
// (rt_kernels.hip bsp_walk, DESIGN.md section 4 "Subtree culling").
// Certification data of every node's subtree (2 x float4 per node), for the
// certified margin of bsp_box_miss (DESIGN.md section 4 "Certified culling"):
//   {E2, nlo.xyz}, {0, nhi.xyz}: E2 = the largest max(|e0|inf, |e1|inf)^2 over
//   its triangles (e0, e1: the records' f32 edges), [nlo, nhi] = a box holding
//   every triangle's exact normal n* = e0 x e1 (rounded outward to f32).
// Leaves first (a leaf range outside ids -- an unreachable node -- stays empty),
// then the interior nodes one depth at a time, bottom-up.
__device__ __forceinline__ float f_rd(double x) { return __double2float_rd(x); }
__device__ __forceinline__ float f_ru(double x) { return __double2float_ru(x); }
__global__ void __launch_bounds__(256) k_leaf_boxes(const uint32_t* tree, uint32_t nnodes, const float4* pos,
                                                    const uint4* idx, const uint32_t* ids, uint32_t nids, float4* box,
                                                    float4* cert)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nnodes; i += gridDim.x * 256u) {
        const uint32_t n0 = tree[4 * (size_t)i], first = tree[4 * (size_t)i + 1];
        float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
        float4 c0 = make_float4(0.0f, INFINITY, INFINITY, INFINITY), c1 = make_float4(0.0f, -INFINITY, -INFINITY, -INFINITY);
        const uint32_t cnt = (n0 & 3u) == 3u ? n0 >> 2 : 0u;
        if ((uint64_t)first + cnt <= nids) {
            for (uint32_t k = 0; k < cnt; k++) {
                const uint4 ix = idx[ids[first + k]];
                const float4 v[3] = {pos[ix.x], pos[ix.y], pos[ix.z]};
                for (int j = 0; j < 3; j++) {
                    lo.x = fminf(lo.x, v[j].x);
                    lo.y = fminf(lo.y, v[j].y);
                    lo.z = fminf(lo.z, v[j].z);
                    hi.x = fmaxf(hi.x, v[j].x);
                    hi.y = fmaxf(hi.y, v[j].y);
                    hi.z = fmaxf(hi.z, v[j].z);
                }
                // the record's f32 edges (k_tri_records2) and their exact cross
                // product: the f32 products are exact in f64, the differences
                // carry a 2^-53 relative error, covered by the outward rounding
                const float e0[3] = {v[1].x - v[0].x, v[1].y - v[0].y, v[1].z - v[0].z};
                const float e1[3] = {v[2].x - v[0].x, v[2].y - v[0].y, v[2].z - v[0].z};
                const double n[3] = {(double)e0[1] * e1[2] - (double)e0[2] * e1[1],
                                     (double)e0[2] * e1[0] - (double)e0[0] * e1[2],
                                     (double)e0[0] * e1[1] - (double)e0[1] * e1[0]};
                const double E = fmax(fmax(fmax(fabs((double)e0[0]), fabs((double)e0[1])), fabs((double)e0[2])),
                                      fmax(fmax(fabs((double)e1[0]), fabs((double)e1[1])), fabs((double)e1[2])));
                c0.x = fmaxf(c0.x, f_ru(E * E));
                const double sl = 0x1p-50;
                c0.y = fminf(c0.y, f_rd(n[0] - fabs(n[0]) * sl));
                c0.z = fminf(c0.z, f_rd(n[1] - fabs(n[1]) * sl));
                c0.w = fminf(c0.w, f_rd(n[2] - fabs(n[2]) * sl));
                c1.y = fmaxf(c1.y, f_ru(n[0] + fabs(n[0]) * sl));
                c1.z = fmaxf(c1.z, f_ru(n[1] + fabs(n[1]) * sl));
                c1.w = fmaxf(c1.w, f_ru(n[2] + fabs(n[2]) * sl));
            }
        }
        box[2 * (size_t)i] = lo;
        box[2 * (size_t)i + 1] = hi;
        cert[2 * (size_t)i] = c0;
        cert[2 * (size_t)i + 1] = c1;
    }
}
__global__ void __launch_bounds__(256) k_node_boxes(const uint32_t* tree, uint32_t nnodes, uint32_t lo_i, uint32_t hi_i,
                                                    float4* box, float4* cert)
{
    for (uint32_t i = lo_i + blockIdx.x * 256u + threadIdx.x; i < hi_i; i += gridDim.x * 256u) {
        if ((tree[4 * (size_t)i] & 3u) == 3u || 2ull * i + 2 >= nnodes) continue;   // a leaf (done) / no children
        const size_t l = 2 * (2 * (size_t)i + 1), r = 2 * (2 * (size_t)i + 2);
        const float4 a0 = box[l], a1 = box[l + 1], b0 = box[r], b1 = box[r + 1];
        box[2 * (size_t)i] = make_float4(fminf(a0.x, b0.x), fminf(a0.y, b0.y), fminf(a0.z, b0.z), 0.0f);
        box[2 * (size_t)i + 1] = make_float4(fmaxf(a1.x, b1.x), fmaxf(a1.y, b1.y), fmaxf(a1.z, b1.z), 0.0f);
        const float4 p0 = cert[l], p1 = cert[l + 1], q0 = cert[r], q1 = cert[r + 1];
        cert[2 * (size_t)i] = make_float4(fmaxf(p0.x, q0.x), fminf(p0.y, q0.y), fminf(p0.z, q0.z), fminf(p0.w, q0.w));
        cert[2 * (size_t)i + 1] = make_float4(0.0f, fmaxf(p1.y, q1.y), fmaxf(p1.z, q1.z), fmaxf(p1.w, q1.w));
    }
}

// f16 bits of x rounded toward -inf (down) or +inf (up)
__device__ __forceinline__ uint32_t h_rd(float x) { return __half_as_ushort(__float2half_rd(x)); }
__device__ __forceinline__ uint32_t h_ru(float x) { return __half_as_ushort(__float2half_ru(x)); }

// The 96-B treelet of 1-based node M at 96*M (rt_internal.h BSP_TREELET_BYTES):
// {box min.xyz, max.x | max.y, max.z, node M | nodes 2M, 2M+1 | 4M, 4M+1 |
//  4M+2, 4M+3 | F G, c.xy, c.z r.x, r.yz}
// -- node M's content box, expanded by `margin` on every side, the 8-B nodes a
// three-level walk from M reads (interior {axis, plane bits}; leaf {3 |
// (48*count) << 2, byte offset of its first record}), and the certification
// data: F = 1e-10 / E2 rounded down to a bf16 (+inf for a subtree without a
// triangle of non-zero extent) with the camera term G (f16, k_treelet_hcam)
// in the same dword, and the normal box divided by E2 (|x| <= 2: |n*_i| <=
// 2 E2) as its centre c (f16, nearest) and radius r (f16, rounded up, so that
// the box lies inside [c - r, c + r]).
__global__ void __launch_bounds__(256) k_bsp_repack(const uint32_t* tree, const float* planes, uint32_t nnodes,
                                                    uint32_t rec_off, const float4* box, const float4* cert,
                                                    float margin, uint32_t* tl)
{
    const size_t slots = (size_t)nnodes + 1;
    constexpr uint32_t W = BSP_TREELET_BYTES / 4;
    for (size_t m = (size_t)blockIdx.x * 256u + threadIdx.x; m < slots; m += (size_t)gridDim.x * 256u) {
        auto node8 = [&](size_t q) -> uint2 {
            if (q == 0 || q > nnodes) return make_uint2(0u, 0u);
            const uint32_t* n = tree + 4 * (q - 1);
            if ((n[0] & 3u) == 3u) return make_uint2(3u | ((48u * (n[0] >> 2)) << 2), rec_off + 48u * n[1]);
            return make_uint2(n[0] & 3u, __float_as_uint(planes[q - 1]));
        };
        uint32_t* o = tl + W * m;
        if (m == 0) {
            for (uint32_t k = 0; k < W; k++) o[k] = 0u;
            continue;
        }
        const float4 lo = box[2 * (m - 1)], hi = box[2 * (m - 1) + 1];
        const float b[6] = {lo.x - margin, lo.y - margin, lo.z - margin, hi.x + margin, hi.y + margin, hi.z + margin};
        for (int k = 0; k < 6; k++) o[k] = __float_as_uint(b[k]);
        const uint2 n[7] = {node8(m), node8(2 * m), node8(2 * m + 1), node8(4 * m), node8(4 * m + 1), node8(4 * m + 2),
                            node8(4 * m + 3)};
        for (int k = 0; k < 7; k++) {
            o[6 + 2 * k] = n[k].x;
            o[7 + 2 * k] = n[k].y;
        }
        const float4 c0 = cert[2 * (m - 1)], c1 = cert[2 * (m - 1) + 1];
        const double E2 = c0.x;
        uint32_t hb[6] = {0u, 0u, 0u, 0u, 0u, 0u};
        float F = INFINITY;
        if (E2 > 0.0 && E2 < INFINITY) {
            F = f_rd(1e-10 / E2 * (1.0 - 0x1p-40));
            // centre c (nearest f16) and radius r (rounded up) with [lo, hi] inside [c - r, c + r]
            const double s = 1.0 / E2, sl = 0x1p-50;
            const float nl[3] = {c0.y, c0.z, c0.w}, nh[3] = {c1.y, c1.z, c1.w};
            for (int k = 0; k < 3; k++) {
                const double a = nl[k] * s, z = nh[k] * s;
                const double lo = a - fabs(a) * sl, hi = z + fabs(z) * sl;
                const uint32_t cb = __half_as_ushort(__float2half_rn((float)(0.5 * (lo + hi))));
                const double c = (double)__half2float(__ushort_as_half((unsigned short)cb));
                const double r = fmax(hi - c, c - lo);
                hb[k] = cb;
                hb[3 + k] = h_ru(f_ru(r * (1.0 + 0x1p-40)));
            }
        }
        // F as a bf16 (the float's high half: truncation, i.e. rounded down for a
        // positive F); the high half is the camera term G (k_treelet_hcam), 0 until set
        o[20] = __float_as_uint(F) >> 16;
        o[21] = hb[0] | (hb[1] << 16);
        o[22] = hb[2] | (hb[3] << 16);
        o[23] = hb[4] | (hb[5] << 16);
    }
}

// The 48-B triangle records in treeIds order, and beside them each slot's
// {triangle id, material} (tm: what shading resolves a BSP hit to, one load
// instead of treeIds -> tri_idx; rt_kernels.hip resolve)
__global__ void __launch_bounds__(256) k_tri_records2(const float4* pos, const uint4* idx, const uint32_t* ids,
                                                      uint32_t nids, float4* recs, uint2* tm)
{
    for (uint32_t k = blockIdx.x * 256u + threadIdx.x; k < nids; k += gridDim.x * 256u) {
        const uint4 ix = idx[ids[k]];
        if (tm) tm[k] = make_uint2(ids[k], ix.w);
        const float4 a = pos[ix.x], b = pos[ix.y], c = pos[ix.z];
        const float e0[3] = {b.x - a.x, b.y - a.y, b.z - a.z};
        const float e1[3] = {c.x - a.x, c.y - a.y, c.z - a.z};
        const float n[3] = {e0[1] * e1[2] - e0[2] * e1[1], e0[2] * e1[0] - e0[0] * e1[2], e0[0] * e1[1] - e0[1] * e1[0]};
        recs[3u * k] = make_float4(a.x, a.y, a.z, e0[0]);
        recs[3u * k + 1u] = make_float4(e0[1], e0[2], e1[0], e1[1]);
        recs[3u * k + 2u] = make_float4(e1[2], n[0], n[1], n[2]);
    }
}

// The camera term of the certified margin (rt_kernels.hip bsp_box_miss,
// DESIGN.md section 4 "Certified culling"): for the eye E of the camera rays,
// H = min over a subtree's triangles of |(v0 - E) . n*| / E_T^2, a lower bound,
// rounded down (the f64 dot product's error subtracted, a 2^-19 relative slack
// for the kernel's f32 evaluation).  A triangle whose edges are zero cannot be
// accepted (its denominator is 0) and constrains nothing (+inf).
__device__ __forceinline__ float tri_hcam(const float4 v[3], const double E[3])
{
    const float e0[3] = {v[1].x - v[0].x, v[1].y - v[0].y, v[1].z - v[0].z};
    const float e1[3] = {v[2].x - v[0].x, v[2].y - v[0].y, v[2].z - v[0].z};
    const double n[3] = {(double)e0[1] * e1[2] - (double)e0[2] * e1[1], (double)e0[2] * e1[0] - (double)e0[0] * e1[2],
                         (double)e0[0] * e1[1] - (double)e0[1] * e1[0]};
    const double Em = fmax(fmax(fmax(fabs((double)e0[0]), fabs((double)e0[1])), fabs((double)e0[2])),
                           fmax(fmax(fabs((double)e1[0]), fabs((double)e1[1])), fabs((double)e1[2])));
    if (!(Em > 0.0)) return INFINITY;
    const double d[3] = {(double)v[0].x - E[0], (double)v[0].y - E[1], (double)v[0].z - E[2]};
    const double dot = d[0] * n[0] + d[1] * n[1] + d[2] * n[2];
    const double err = 0x1p-45 * (fabs(d[0] * n[0]) + fabs(d[1] * n[1]) + fabs(d[2] * n[2]));
    const double eta = fabs(dot) - err;
    if (!(eta > 0.0)) return 0.0f;
    return f_rd(eta / (Em * Em) * (1.0 - 0x1p-19));
}
// Per node, the three smallest H of its subtree with their triangles (distinct,
// ascending; H = +inf / triangle ~0 where fewer): the camera term excludes the
// first two (they are bounded per ray by their own normals instead) and takes
// the third as the rest's minimum -- any other triangle's H is at least that.
// Scratch: 6 words per node {h0, h1, h2, t0, t1, t2}.
struct Top3 {
    float h[3];
    uint32_t t[3];
};
__device__ __forceinline__ void top3_add(Top3& a, float h, uint32_t t)
{
    if (t == ~0u) return;
    for (int j = 0; j < 3; j++)
        if (a.t[j] == t) return;   // (a triangle referenced by two leaves)
    if (!(h < a.h[2])) return;
    int j = 2;
    while (j > 0 && h < a.h[j - 1]) {
        a.h[j] = a.h[j - 1];
        a.t[j] = a.t[j - 1];
        j--;
    }
    a.h[j] = h;
    a.t[j] = t;
}
__device__ __forceinline__ Top3 top3_load(const float* s, size_t i)
{
    Top3 a;
    for (int j = 0; j < 3; j++) {
        a.h[j] = s[6 * i + j];
        a.t[j] = __float_as_uint(s[6 * i + 3 + j]);
    }
    return a;
}
__device__ __forceinline__ void top3_store(float* s, size_t i, const Top3& a)
{
    for (int j = 0; j < 3; j++) {
        s[6 * i + j] = a.h[j];
        s[6 * i + 3 + j] = __uint_as_float(a.t[j]);
    }
}
__global__ void __launch_bounds__(256) k_leaf_hcam(const uint32_t* tree, uint32_t nnodes, const float4* pos,
                                                   const uint4* idx, const uint32_t* ids, uint32_t nids, double ex,
                                                   double ey, double ez, float* h)
{
    const double E[3] = {ex, ey, ez};
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nnodes; i += gridDim.x * 256u) {
        const uint32_t n0 = tree[4 * (size_t)i], first = tree[4 * (size_t)i + 1];
        Top3 a = {{INFINITY, INFINITY, INFINITY}, {~0u, ~0u, ~0u}};
        const uint32_t cnt = (n0 & 3u) == 3u ? n0 >> 2 : 0u;
        if ((uint64_t)first + cnt <= nids)
            for (uint32_t k = 0; k < cnt; k++) {
                const uint4 ix = idx[ids[first + k]];
                const float4 v[3] = {pos[ix.x], pos[ix.y], pos[ix.z]};
                top3_add(a, tri_hcam(v, E), ids[first + k]);
            }
        top3_store(h, i, a);
    }
}
__global__ void __launch_bounds__(256) k_node_hcam(const uint32_t* tree, uint32_t nnodes, uint32_t lo_i, uint32_t hi_i,
                                                   float* h)
{
    for (uint32_t i = lo_i + blockIdx.x * 256u + threadIdx.x; i < hi_i; i += gridDim.x * 256u) {
        if ((tree[4 * (size_t)i] & 3u) == 3u || 2ull * i + 2 >= nnodes) continue;
        Top3 a = top3_load(h, 2 * (size_t)i + 1);
        const Top3 b = top3_load(h, 2 * (size_t)i + 2);
        for (int j = 0; j < 3; j++) top3_add(a, b.h[j], b.t[j]);
        top3_store(h, i, a);
    }
}
// n*/E_t^2 of triangle t (the records' f32 edges, the exact cross product in f64,
// E_t its largest edge component) as three f16 rounded to nearest; NaN where the
// triangle has no extent (it cannot be accepted: its denominator is 0)
__device__ __forceinline__ void tri_nrm_h(const float4* pos, const uint4* idx, uint32_t t, uint32_t h[3])
{
    const uint4 ix = idx[t];
    const float4 v[3] = {pos[ix.x], pos[ix.y], pos[ix.z]};
    const float e0[3] = {v[1].x - v[0].x, v[1].y - v[0].y, v[1].z - v[0].z};
    const float e1[3] = {v[2].x - v[0].x, v[2].y - v[0].y, v[2].z - v[0].z};
    const double n[3] = {(double)e0[1] * e1[2] - (double)e0[2] * e1[1], (double)e0[2] * e1[0] - (double)e0[0] * e1[2],
                         (double)e0[0] * e1[1] - (double)e0[1] * e1[0]};
    const double Em = fmax(fmax(fmax(fabs((double)e0[0]), fabs((double)e0[1])), fabs((double)e0[2])),
                           fmax(fmax(fabs((double)e1[0]), fabs((double)e1[1])), fabs((double)e1[2])));
    for (int a = 0; a < 3; a++)
        h[a] = Em > 0.0 ? __half_as_ushort(__float2half_rn((float)(n[a] / (Em * Em)))) : 0x7E00u;
}
// The camera term G of treelet M, into the high half of its q5.x as an f16
// rounded down (G <= 2 sqrt(3): |n*| <= 2 E_T^2, |v0 - E| <= sqrt(3) Dinf): with D1 and Dinf the L1 and L-inf bounds of
// |x - E| over the treelet's box (f64, rounded up) and H the subtree's minimum
// above, a camera ray's |denom| / E_T^2 >= ((H - 14u D1) |w|inf - 38u D1 |w|1) / Dinf
// >= |w|inf (H - 128u D1) / Dinf = G |w|inf, since |w|1 <= 3 |w|inf (u = 2^-24;
// the factor 1 - 2^-20 covers the kernel's one rounding of G |w|inf).
// The silhouette data of RT_BSP_CULL_SILHOUETTE (16 B per 1-based node M in
// `sil`): {x0.xy | x0.z x1.x | x1.yz | G_x}.  G_x, from the third smallest H, is
// the camera bound for every triangle but the two excluded ones, whose normals
// x = n*/E_t^2 (f16, nearest) the kernel dots with the ray:
// |w . n*| / E_t^2 >= |w . x| - |w|1 (2 2^-11 + 2^-25 + 10u + rounding) >= |w . x| - 2^-9 |w|1
// (|n*| / E_t^2 <= 2 per component; 10u: the test's own error of its denominator).
__global__ void __launch_bounds__(256) k_treelet_hcam(const float* h, uint32_t nnodes, double ex, double ey, double ez,
                                                      const float4* pos, const uint4* idx, uint32_t* tl, uint32_t* sil)
{
    constexpr uint32_t W = BSP_TREELET_BYTES / 4;
    const double E[3] = {ex, ey, ez};
    for (size_t m = 1 + (size_t)blockIdx.x * 256u + threadIdx.x; m <= nnodes; m += (size_t)gridDim.x * 256u) {
        uint32_t* t = tl + W * m;
        double D1 = 0.0, Dinf = 0.0;
        for (int a = 0; a < 3; a++) {
            const double d = fmax(fabs((double)__uint_as_float(t[a]) - E[a]), fabs((double)__uint_as_float(t[3 + a]) - E[a]));
            D1 += d;
            Dinf = fmax(Dinf, d);
        }
        D1 *= 1.0 + 0x1p-40;
        Dinf *= 1.0 + 0x1p-40;
        auto gterm = [&](double H) -> float {
            if (H == INFINITY) return INFINITY;   // no triangle of non-zero extent: F is +inf too
            if (Dinf > 0.0 && H - 128.0 * 0x1p-24 * D1 > 0.0) return f_rd((H - 128.0 * 0x1p-24 * D1) / Dinf * (1.0 - 0x1p-20));
            return 0.0f;
        };
        const Top3 a = top3_load(h, m - 1);
        t[20] = (t[20] & 0xFFFFu) | (h_rd(gterm(a.h[0])) << 16);
        // the two excluded triangles (NaN slots: none) and the rest's term G_x
        uint32_t x[6] = {0x7E00u, 0x7E00u, 0x7E00u, 0x7E00u, 0x7E00u, 0x7E00u};
        for (int j = 0; j < 2; j++)
            if (a.t[j] != ~0u && a.h[j] < INFINITY) tri_nrm_h(pos, idx, a.t[j], x + 3 * j);
        uint32_t* q = sil + 4 * m;
        q[0] = x[0] | (x[1] << 16);
        q[1] = x[2] | (x[3] << 16);
        q[2] = x[4] | (x[5] << 16);
        q[3] = h_rd(gterm(a.h[2]));
    }
}
int launch_bsp_camera(const uint32_t* tree, uint32_t nnodes, const float4* pos, const uint4* idx, const uint32_t* ids,
                      uint32_t nids, const float eye[3], void* blob, uint32_t* sil, void* scratch, hipStream_t s)
{
    float* h = reinterpret_cast<float*>(scratch);
    const uint32_t g0 = std::min<uint32_t>(16384, (nnodes + 255) / 256);
    hipLaunchKernelGGL(k_leaf_hcam, dim3(g0), dim3(256), 0, s, tree, nnodes, pos, idx, ids, nids, (double)eye[0],
                       (double)eye[1], (double)eye[2], h);
    uint32_t depth = 0;
    while ((2ull << depth) - 1 < nnodes) depth++;
    for (int d = (int)depth - 1; d >= 0; d--) {
        const uint32_t lo = (1u << d) - 1u, hi = std::min<uint32_t>(nnodes, (2u << d) - 1u);
        const uint32_t g = std::min<uint32_t>(16384, (hi - lo + 255) / 256);
        hipLaunchKernelGGL(k_node_hcam, dim3(g), dim3(256), 0, s, tree, nnodes, lo, hi, h);
    }
    hipLaunchKernelGGL(k_treelet_hcam, dim3(g0), dim3(256), 0, s, h, nnodes, (double)eye[0], (double)eye[1], (double)eye[2],
                       pos, idx, reinterpret_cast<uint32_t*>(blob), sil);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

// Whether the walk's plane divisions need their range check (rt_kernels.hip bsp_decide):
// rt_div_by_recip is exact for x = plane - o with x == 0 or 2^-100 <= |x| <= 2^100
// (include/rt_detmath.h).  That holds for every ray origin coordinate o that is 0 or
// in [2^-76, 2^99] in magnitude (k_path checks those per ray) when every interior
// plane is too: the difference of two such floats is 0, or a nonzero multiple of
// 2^-99, or at most 2^100.  flag |= 1 for a plane outside that range.
__global__ void __launch_bounds__(256) k_plane_range(const uint32_t* tree, const float* planes, uint32_t nnodes,
                                                     uint32_t* flag)
{
    bool out = false;
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < nnodes; i += (size_t)gridDim.x * 256u) {
        if ((tree[4 * i] & 3u) == 3u) continue;   // a leaf: no plane
        const float a = fabsf(planes[i]);
        out |= !(a == 0.0f || (a >= 0x1p-76f && a <= 0x1p99f));
    }
    if (__ballot(out) != 0 && (threadIdx.x & 63u) == 0u) atomicOr(flag, 1u);
}

int launch_plane_range(const uint32_t* tree, const float* planes, uint32_t nnodes, uint32_t* flag, hipStream_t s)
{
    if (hipMemsetAsync(flag, 0, 4, s) != hipSuccess) return RT_E_DEVICE;
    const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(4096, (nnodes + 255) / 256));
    hipLaunchKernelGGL(k_plane_range, dim3(g), dim3(256), 0, s, tree, planes, nnodes, flag);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

int launch_bsp_repack(const uint32_t* tree, const float* planes, uint32_t nnodes, uint32_t rec_off, void* blob,
                      const float4* pos, const uint4* idx, const uint32_t* ids, uint32_t nids, float margin,
                      void* box_scratch, uint2* tm, hipStream_t s)
{
    // content boxes: leaves, then each depth bottom-up (depth d holds nodes [2^d - 1, 2^(d+1) - 1))
    float4* box = reinterpret_cast<float4*>(box_scratch);
    float4* cert = box + 2 * (size_t)nnodes;
    const uint32_t g0 = std::min<uint32_t>(16384, (nnodes + 255) / 256);
    hipLaunchKernelGGL(k_leaf_boxes, dim3(g0), dim3(256), 0, s, tree, nnodes, pos, idx, ids, nids, box, cert);
    uint32_t depth = 0;
    while ((2ull << depth) - 1 < nnodes) depth++;   // the deepest level
    for (int d = (int)depth - 1; d >= 0; d--) {
        const uint32_t lo = (1u << d) - 1u, hi = std::min<uint32_t>(nnodes, (2u << d) - 1u);
        const uint32_t g = std::min<uint32_t>(16384, (hi - lo + 255) / 256);
        hipLaunchKernelGGL(k_node_boxes, dim3(g), dim3(256), 0, s, tree, nnodes, lo, hi, box, cert);
    }
    const uint32_t g1 = std::min<uint32_t>(16384, (nnodes + 256) / 256 + 1);
    hipLaunchKernelGGL(k_bsp_repack, dim3(g1), dim3(256), 0, s, tree, planes, nnodes, rec_off, box, cert, margin,
                       reinterpret_cast<uint32_t*>(blob));
    if (nids) {
        const uint32_t g2 = std::min<uint32_t>(16384, (nids + 255) / 256 + 1);
        hipLaunchKernelGGL(k_tri_records2, dim3(g2), dim3(256), 0, s, pos, idx, ids, nids,
                           reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(blob) + rec_off), tm);
    }
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

namespace {
struct DBufs {   // device allocations freed at scope exit
    std::vector<void*> p;
    hipError_t e = hipSuccess;
    ~DBufs()
    {
        for (void* q : p) (void)hipFree(q);
    }
    template <class T>
    T* alloc(size_t count)
    {
        void* q = nullptr;
        if (e == hipSuccess) e = hipMalloc(&q, std::max<size_t>(16, count * sizeof(T)));
        if (e == hipSuccess) p.push_back(q);
        return reinterpret_cast<T*>(q);
    }
};
inline uint32_t blocks_for(size_t n, uint32_t cap) { return (uint32_t)std::max<size_t>(1, std::min<size_t>(cap, (n + 255) / 256)); }
}  // namespace

int build_bsp_device(const float4* pos, const uint4* idx, uint32_t nt, uint32_t max_depth, uint32_t max_leaf,
                     int num_cus, hipStream_t s, BspDeviceOut& out, rt_bsp_build_times* times, std::string& err)
{
    using namespace rtbsp;
    if (nt == 0) {
        err = "rt_build_bsp_device: empty mesh";
        return RT_E_INVALID;
    }
    if (max_depth == 0 || max_depth > 24 || max_leaf == 0) {
        err = "rt_build_bsp_device: max_depth must be in [1,24] (the traversal layout's limit), max_leaf > 0";
        return RT_E_INVALID;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t cap = (uint32_t)std::max(1, num_cus) * 16u;
    const size_t nnodes = ((size_t)1 << (max_depth + 1)) - 1;
    DBufs D;
    float4* boxes = D.alloc<float4>((size_t)nt * 2);
    const uint32_t per = (nt + 65535u) / 65536u;   // triangles per thread: <= 256 blocks of contiguous ranges
    const uint32_t rblocks = (nt + 256u * per - 1) / (256u * per);
    float* partial = D.alloc<float>((size_t)rblocks * 6);
    uint32_t* leaf_ctr = D.alloc<uint32_t>(4);
    Leaf* leaves = D.alloc<Leaf>(nnodes);
    uint32_t* lkeys = D.alloc<uint32_t>(nnodes);
    uint32_t* d_aabb_u = D.alloc<uint32_t>(8);
    if (D.e != hipSuccess) {
        err = std::string("rt_build_bsp_device: allocation: ") + hipGetErrorString(D.e);
        return RT_E_OOM;
    }
    if (hipMalloc(&out.tree, nnodes * 16) != hipSuccess || hipMalloc(&out.planes, nnodes * 4) != hipSuccess) {
        err = "rt_build_bsp_device: output allocation failed";
        return RT_E_OOM;
    }
    out.nnodes = (uint32_t)nnodes;
    (void)hipMemsetAsync(out.tree, 0, nnodes * 16, s);   // unused slots (0,0,0,0) / plane 0
    (void)hipMemsetAsync(out.planes, 0, nnodes * 4, s);
    (void)hipMemsetAsync(leaf_ctr, 0, 16, s);
    // level 0
    std::vector<uint32_t*> level_slots;
    uint32_t nn = 1, ns = nt;
    LNode* nodes = D.alloc<LNode>(1);
    uint32_t* slots = D.alloc<uint32_t>(ns);
    uint32_t* nos = D.alloc<uint32_t>(ns);
    hipLaunchKernelGGL(k_tri_boxes, dim3(rblocks), dim3(256), 0, s, pos, idx, nt, per, boxes, partial);
    hipLaunchKernelGGL(k_iota, dim3(blocks_for(ns, cap)), dim3(256), 0, s, slots, nos, ns);
    hipLaunchKernelGGL(k_root, dim3(1), dim3(64), 0, s, partial, rblocks, nt, nodes, slots, nos,
                       reinterpret_cast<float*>(d_aabb_u));
    uint32_t levels = 0;
    for (uint32_t depth = 0; depth <= max_depth && nn > 0; depth++) {
        levels++;
        level_slots.push_back(slots);
        uint32_t* counts = D.alloc<uint32_t>((size_t)nn * 18);
        uint32_t* ext = D.alloc<uint32_t>((size_t)nn * 2);
        uint32_t* el = D.alloc<uint32_t>((size_t)ns + 2);   // scans of ns+1 flags: ns+2 words
        uint32_t* er = D.alloc<uint32_t>((size_t)ns + 2);
        uint32_t* na = D.alloc<uint32_t>((size_t)nn + 2);
        uint32_t* nb = D.alloc<uint32_t>((size_t)nn + 2);
        uint32_t* sc = D.alloc<uint32_t>(scan_scratch_words(std::max(ns, nn) + 1));
        if (D.e != hipSuccess) {
            err = std::string("rt_build_bsp_device: level allocation: ") + hipGetErrorString(D.e);
            return RT_E_OOM;
        }
        (void)hipMemsetAsync(counts, 0, (size_t)nn * 18 * 4, s);
        if (ns > 0) {
            const uint32_t cblocks = (ns + kSlotsPerBlock - 1) / kSlotsPerBlock;
            hipLaunchKernelGGL(k_bsp_count, dim3(cblocks), dim3(256), 0, s, slots, nos, ns, nodes, boxes, depth,
                               max_depth, max_leaf, counts);
        }
        hipLaunchKernelGGL(k_bsp_decide, dim3(blocks_for(nn, cap)), dim3(256), 0, s, nodes, nn, counts, depth,
                           max_depth, max_leaf, out.tree, out.planes, ext, leaves, lkeys, leaf_ctr);
        hipLaunchKernelGGL(k_bsp_extent, dim3(blocks_for(ns, cap)), dim3(256), 0, s, slots, nos, ns, nodes, boxes,
                           ext);
        hipLaunchKernelGGL(k_bsp_finalize, dim3(blocks_for(nn, cap)), dim3(256), 0, s, nodes, nn, ext, out.tree,
                           out.planes);
        hipLaunchKernelGGL(k_bsp_flags, dim3(blocks_for((size_t)ns + 1, cap)), dim3(256), 0, s, slots, nos, ns, nodes,
                           boxes, el, er);
        int r = scan_exclusive_u32(el, el, ns + 1, sc, s);
        if (!r) r = scan_exclusive_u32(er, er, ns + 1, sc, s);
        hipLaunchKernelGGL(k_bsp_child_counts, dim3(blocks_for((size_t)nn + 1, cap)), dim3(256), 0, s, nodes, nn, el,
                           er, na, nb);
        if (!r) r = scan_exclusive_u32(na, na, nn + 1, sc, s);
        if (!r) r = scan_exclusive_u32(nb, nb, nn + 1, sc, s);
        uint32_t tot[2] = {0, 0};
        hipError_t e = hipGetLastError();
        if (e == hipSuccess && !r) e = hipMemcpyAsync(&tot[0], na + nn + 1, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&tot[1], nb + nn + 1, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess || r) {
            err = std::string("rt_build_bsp_device: level ") + std::to_string(depth) + ": " + hipGetErrorString(e);
            return RT_E_DEVICE;
        }
        const uint32_t nn2 = tot[0], ns2 = tot[1];
        if (nn2 == 0) break;
        LNode* next = D.alloc<LNode>(nn2);
        uint32_t* nslots = D.alloc<uint32_t>(ns2);
        uint32_t* nnos = D.alloc<uint32_t>(ns2);
        if (D.e != hipSuccess) {
            err = std::string("rt_build_bsp_device: level allocation: ") + hipGetErrorString(D.e);
            return RT_E_OOM;
        }
        hipLaunchKernelGGL(k_bsp_children, dim3(blocks_for(nn, cap)), dim3(256), 0, s, nodes, nn, na, nb, next);
        hipLaunchKernelGGL(k_bsp_scatter, dim3(blocks_for(ns, cap)), dim3(256), 0, s, slots, nos, ns, nodes, el, er,
                           nslots, nnos);
        nodes = next;
        slots = nslots;
        nos = nnos;
        nn = nn2;
        ns = ns2;
    }
    // ---- flatten: leaves in DFS order
    uint32_t nl = 0;
    if (hipMemcpyAsync(&nl, leaf_ctr, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
        err = "rt_build_bsp_device: leaf count readback failed";
        return RT_E_DEVICE;
    }
    const auto t1 = std::chrono::steady_clock::now();
    uint32_t* ord = D.alloc<uint32_t>(nl);
    uint32_t* k1 = D.alloc<uint32_t>(nl);
    uint32_t* v1 = D.alloc<uint32_t>(nl);
    uint32_t* hist = D.alloc<uint32_t>(radix_hist_words(nl));
    uint32_t* lc = D.alloc<uint32_t>((size_t)nl + 1);
    uint32_t* sc = D.alloc<uint32_t>(scan_scratch_words(nl + 1));
    uint32_t** d_levels = D.alloc<uint32_t*>(level_slots.size());
    if (D.e != hipSuccess) {
        err = "rt_build_bsp_device: flatten allocation failed";
        return RT_E_OOM;
    }
    (void)hipMemcpyAsync(d_levels, level_slots.data(), level_slots.size() * sizeof(uint32_t*), hipMemcpyHostToDevice, s);
    if (nl) {
        hipLaunchKernelGGL(k_iota, dim3(blocks_for(nl, cap)), dim3(256), 0, s, ord, v1, nl);
        int second = 0;
        const uint32_t passes = (max_depth + 7u) / 8u;   // keys < 2^max_depth
        if (radix_sort_pairs(lkeys, ord, k1, v1, nl, passes, hist, s, second)) {
            err = "rt_build_bsp_device: leaf sort failed";
            return RT_E_DEVICE;
        }
        const uint32_t* order = second ? v1 : ord;
        hipLaunchKernelGGL(k_leaf_counts, dim3(blocks_for(nl, cap)), dim3(256), 0, s, leaves, order, nl, lc);
        (void)hipMemsetAsync(lc + nl, 0, 4, s);
        if (scan_exclusive_u32(lc, lc, nl, sc, s)) {
            err = "rt_build_bsp_device: leaf scan failed";
            return RT_E_DEVICE;
        }
        uint32_t nids = 0;
        if (hipMemcpyAsync(&nids, lc + nl, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            err = "rt_build_bsp_device: id count readback failed";
            return RT_E_DEVICE;
        }
        if (hipMalloc(&out.ids, std::max<size_t>(16, (size_t)nids * 4)) != hipSuccess) {
            err = "rt_build_bsp_device: id allocation failed";
            return RT_E_OOM;
        }
        out.nids = nids;
        hipLaunchKernelGGL(k_leaf_finish, dim3(blocks_for(nl, cap)), dim3(256), 0, s, leaves, order, nl, lc,
                           d_levels, out.tree, out.ids);
    } else if (hipMalloc(&out.ids, 16) != hipSuccess) {
        return RT_E_OOM;
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out.aabb, d_aabb_u, 32, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        err = std::string("rt_build_bsp_device: flatten: ") + hipGetErrorString(e);
        return RT_E_DEVICE;
    }
    if (times) {
        const auto t2 = std::chrono::steady_clock::now();
        times->subdivision_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        times->flattening_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
        times->total_ms = std::chrono::duration<double, std::milli>(t2 - t0).count();
        times->levels = levels;
        times->leaves = nl;
        times->nids = out.nids;
    }
    return RT_OK;
}

}  // namespace rtk
