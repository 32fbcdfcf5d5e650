// rt_build.hip -- HLBVH construction on the GPU:
// hlbvh::Bvh::new + flatten + triangles (src/data_structures/hlbvh.rs:36-239)
// as gfx950 kernels, producing the same arrays as the host builder
// (host_bvh.cpp, pinned to the oracle) bit for bit.
//
// Phases (the reference's BvhConstructionTime split, bvh_util.rs):
//   morton_codes  k_boxes (triangle boxes + per-block centroid bounds),
//                 k_bound, k_morton (10 bits/axis, Rust `as u32` saturation)
//   radix_sort    4 LSD passes of 8 bits over the 30-bit codes: k_rs_hist,
//                 k_rs_scan, k_rs_scatter (stable: equal codes stay in
//                 primitive-index order, the host builder's tie order)
//   treelet_init  k_treelet_count / k_treelet_list: treelets = runs of equal
//                 top-12 code bits (mask 0x3FFC0000), in code order
//   treelet_build emit_lbvh for all treelets at once, one kernel per bit level
//                 (bit 17 .. -1: at most 19 levels); each work item is one
//                 emit_lbvh call; then k_bottom_up per level (subtree sizes and
//                 boxes: leaf = fold of its primitive boxes in order, internal =
//                 child0's box including child1's)
//   upper_tree    k_upper_tree: the reference's median-split collapse over the
//                 <= 4096 treelet roots in one workgroup (a bitonic sort per
//                 level), the DFS offsets of the roots and the upper nodes' records
//   flattening    k_top_down per level (DFS index of every node: left child
//                 = parent+1, right = parent+1+size(left)), k_write_nodes, the
//                 upper nodes, the GpuNode::new(root box) filler of the
//                 over-allocated array, and the traversal repack (node records
//                 with byte offsets + 48-B triangle records)
// Numerics: min/max folds with the reference's operand order, -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/rt_detmath.h"
#include "host_types.h"
#include "rt_internal.h"

namespace rtb {

constexpr int kLevels = 19;          // emit_lbvh bits 17 .. -1
constexpr uint32_t kTreeletMask = 0x3FFC0000u;
constexpr int kTile = 2048;          // radix sort keys per block (256 threads x 8)

struct BNode {                       // build node (pool)
    float mn[3], mx[3];
    int32_t left, right;             // -1 for a leaf
    uint32_t first, n;               // leaf: sorted range
    uint32_t size, dfs;
};
struct Item {                        // one pending emit_lbvh call
    uint32_t off, n;
    int32_t bit;
    uint32_t node;
};
struct Ctl {                         // device-side counters
    uint32_t items[2];               // ping-pong item counts
    uint32_t pool;                   // pool nodes allocated
    uint32_t res;                    // internal nodes resolved (res list length)
    uint32_t ntreelets;
    uint32_t emits;                  // emit_lbvh calls (the reference's total_nodes increments)
    uint32_t lvl_end[kLevels + 1];   // res list length after each level
};

__device__ __forceinline__ void box_include(float* mn, float* mx, const float* omn, const float* omx)
{
    for (int i = 0; i < 3; i++) {
        mn[i] = rt_minf(mn[i], omn[i]);
        mx[i] = rt_maxf(mx[i], omx[i]);
    }
}

// ------------------------------------------------------------ morton codes
// Mesh::bboxes (src/mesh.rs:212-227, Bbox::from_triangle) and the per-block
// bound of the centroids (hlbvh.rs:42-45).  Bounds use min/max (exact; the
// sign of a zero bound cannot change a code: c - (+-0) and the extent agree).
__global__ void __launch_bounds__(256) k_boxes(const float4* pos, const uint4* idx, uint32_t nt, float4* boxes,
                                               float* partial)
{
    __shared__ float red[6][256];
    float bmn[3] = {1.0e37f, 1.0e37f, 1.0e37f}, bmx[3] = {-1.0e37f, -1.0e37f, -1.0e37f};
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < nt; t += gridDim.x * 256u) {
        const uint4 ix = idx[t];
        const float4 a = pos[ix.x], b = pos[ix.y], c = pos[ix.z];
        const float mn[3] = {rt_minf(a.x, rt_minf(b.x, c.x)), rt_minf(a.y, rt_minf(b.y, c.y)),
                             rt_minf(a.z, rt_minf(b.z, c.z))};
        const float mx[3] = {rt_maxf(a.x, rt_maxf(b.x, c.x)), rt_maxf(a.y, rt_maxf(b.y, c.y)),
                             rt_maxf(a.z, rt_maxf(b.z, c.z))};
        boxes[2u * t] = make_float4(mn[0], mn[1], mn[2], 0.0f);
        boxes[2u * t + 1u] = make_float4(mx[0], mx[1], mx[2], 0.0f);
        for (int i = 0; i < 3; i++) {
            const float cc = (mn[i] + mx[i]) * 0.5f;
            bmn[i] = rt_minf(bmn[i], cc);
            bmx[i] = rt_maxf(bmx[i], cc);
        }
    }
    for (int i = 0; i < 3; i++) {
        red[i][threadIdx.x] = bmn[i];
        red[3 + i][threadIdx.x] = bmx[i];
    }
    __syncthreads();
    for (uint32_t s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s)
            for (int i = 0; i < 3; i++) {
                red[i][threadIdx.x] = rt_minf(red[i][threadIdx.x], red[i][threadIdx.x + s]);
                red[3 + i][threadIdx.x] = rt_maxf(red[3 + i][threadIdx.x], red[3 + i][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) partial[blockIdx.x * 6u + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void __launch_bounds__(256) k_bound(const float* partial, uint32_t nparts, float* bound)
{
    __shared__ float red[6][256];
    float v[6] = {1.0e37f, 1.0e37f, 1.0e37f, -1.0e37f, -1.0e37f, -1.0e37f};
    for (uint32_t p = threadIdx.x; p < nparts; p += 256u)
        for (int i = 0; i < 3; i++) {
            v[i] = rt_minf(v[i], partial[p * 6u + i]);
            v[3 + i] = rt_maxf(v[3 + i], partial[p * 6u + 3 + i]);
        }
    for (int i = 0; i < 6; i++) red[i][threadIdx.x] = v[i];
    __syncthreads();
    for (uint32_t s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s)
            for (int i = 0; i < 3; i++) {
                red[i][threadIdx.x] = rt_minf(red[i][threadIdx.x], red[i][threadIdx.x + s]);
                red[3 + i][threadIdx.x] = rt_maxf(red[3 + i][threadIdx.x], red[3 + i][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) bound[threadIdx.x] = red[threadIdx.x][0];
}

__device__ __forceinline__ uint32_t left_shift_3(uint32_t x)   // hlbvh.rs:489-498
{
    if (x == (1u << 10)) x -= 1;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}
__device__ __forceinline__ uint32_t as_u32(float f)   // Rust `f as u32` (saturating, NaN -> 0)
{
    if (!(f > 0.0f)) return 0;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

// hlbvh.rs:54-68 with Bbox::offset (bbox.rs:169-181)
__global__ void __launch_bounds__(256) k_morton(const float4* boxes, const float* bound, uint32_t nt, uint32_t* keys,
                                                uint32_t* vals)
{
    const float bmn[3] = {bound[0], bound[1], bound[2]}, bmx[3] = {bound[3], bound[4], bound[5]};
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < nt; t += gridDim.x * 256u) {
        const float4 a = boxes[2u * t], b = boxes[2u * t + 1u];
        const float c[3] = {(a.x + b.x) * 0.5f, (a.y + b.y) * 0.5f, (a.z + b.z) * 0.5f};
        uint32_t q[3];
        for (int i = 0; i < 3; i++) {
            float o = c[i] - bmn[i];
            if (bmx[i] > bmn[i]) o = o / (bmx[i] - bmn[i]);
            q[i] = as_u32(o * 1024.0f);
        }
        keys[t] = (left_shift_3(q[2]) << 2) | (left_shift_3(q[1]) << 1) | left_shift_3(q[0]);
        vals[t] = t;
    }
}

// ------------------------------------------------------------ radix sort
// Stable LSD radix sort of (code, index) pairs, 8-bit digits.  Per pass:
// per-tile digit histograms (digit-major), one exclusive scan, and a stable
// scatter: each tile ranks its keys in order, 256 at a time, with wave64
// match masks (8 ballots) and a per-digit running count across the 4 waves.
__global__ void __launch_bounds__(256) k_rs_hist(const uint32_t* keys, uint32_t n, uint32_t shift, uint32_t ntiles,
                                                 uint32_t* hist)
{
    __shared__ uint32_t cnt[256];
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * (uint32_t)kTile;
    for (uint32_t i = threadIdx.x; i < (uint32_t)kTile; i += 256u) {
        const uint32_t k = base + i;
        if (k < n) atomicAdd(&cnt[(keys[k] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * ntiles + blockIdx.x] = cnt[threadIdx.x];
}

// exclusive scan of m words in place, one block of 1024 threads
__global__ void __launch_bounds__(1024) k_rs_scan(uint32_t* a, uint32_t m)
{
    __shared__ uint32_t part[1024];
    const uint32_t per = (m + 1023u) / 1024u;
    const uint32_t lo = threadIdx.x * per, hi = min(m, lo + per);
    uint32_t s = 0;
    for (uint32_t i = lo; i < hi; i++) s += a[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {   // Hillis-Steele inclusive scan
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t v = a[i];
        a[i] = run;
        run += v;
    }
}

__global__ void __launch_bounds__(256) k_rs_scatter(const uint32_t* kin, const uint32_t* vin, uint32_t n,
                                                    uint32_t shift, uint32_t ntiles, const uint32_t* offs,
                                                    uint32_t* kout, uint32_t* vout)
{
    __shared__ uint32_t gbase[256], running[256], wcnt[4][256], wbase[4][256];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    gbase[threadIdx.x] = offs[threadIdx.x * ntiles + blockIdx.x];
    running[threadIdx.x] = 0;
    for (int w = 0; w < 4; w++) wcnt[w][threadIdx.x] = 0;
    __syncthreads();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
    for (uint32_t r = 0; r < (uint32_t)kTile / 256u; r++) {
        const uint32_t k = blockIdx.x * (uint32_t)kTile + r * 256u + threadIdx.x;
        const bool valid = k < n;
        const uint32_t key = valid ? kin[k] : 0u, val = valid ? vin[k] : 0u;
        const uint32_t d = (key >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t m = __ballot(((d >> b) & 1u) != 0u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        {
            const uint32_t dd = threadIdx.x;
            uint32_t s = running[dd];
            for (int w = 0; w < 4; w++) {
                const uint32_t c = wcnt[w][dd];
                wbase[w][dd] = s;
                s += c;
                wcnt[w][dd] = 0;
            }
            running[dd] = s;
        }
        __syncthreads();
        if (valid) {
            const uint32_t pos = gbase[d] + wbase[wave][d] + rank;
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------ treelets
__global__ void __launch_bounds__(256) k_treelet_count(const uint32_t* keys, uint32_t n, uint32_t* counts)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        atomicAdd(&counts[(keys[i] & kTreeletMask) >> 18], 1u);
}

// runs of equal top-12 bits in code order = the non-empty prefixes in order
// (hlbvh.rs:100-117); writes the level-0 items (emit_lbvh(start, n, 17)) with
// pool slot j for treelet j
__global__ void __launch_bounds__(1024) k_treelet_list(const uint32_t* counts, Item* items, Ctl* ctl)
{
    __shared__ uint32_t ne[1024], st[1024];
    uint32_t c[4], nonempty = 0, total = 0;
    for (int i = 0; i < 4; i++) {
        c[i] = counts[threadIdx.x * 4u + i];
        nonempty += c[i] != 0u;
        total += c[i];
    }
    ne[threadIdx.x] = nonempty;
    st[threadIdx.x] = total;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {
        const uint32_t a = threadIdx.x >= off ? ne[threadIdx.x - off] : 0u;
        const uint32_t b = threadIdx.x >= off ? st[threadIdx.x - off] : 0u;
        __syncthreads();
        ne[threadIdx.x] += a;
        st[threadIdx.x] += b;
        __syncthreads();
    }
    uint32_t j = ne[threadIdx.x] - nonempty, start = st[threadIdx.x] - total;
    for (int i = 0; i < 4; i++) {
        if (c[i]) {
            items[j] = Item{start, c[i], 17, j};
            j++;
        }
        start += c[i];
    }
    if (threadIdx.x == 1023u) {
        ctl->ntreelets = ne[1023];
        ctl->items[0] = ne[1023];
        ctl->items[1] = 0;
        ctl->pool = ne[1023];
        ctl->res = 0;
        ctl->emits = 0;
    }
}

// ------------------------------------------------------------ emit_lbvh, one bit level
// hlbvh.rs:348-442 for every pending call of this level.
__global__ void __launch_bounds__(256) k_lbvh_level(const Item* in, uint32_t in_sel, Item* out, Ctl* ctl,
                                                    const uint32_t* keys, const uint32_t* vals, const float4* boxes,
                                                    uint32_t max_prims, BNode* pool, uint32_t* res)
{
    const uint32_t nin = ctl->items[in_sel];
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nin; i += gridDim.x * 256u) {
        const Item it = in[i];
        BNode& nd = pool[it.node];
        if (it.bit <= -1 || it.n < max_prims) {   // leaf
            float mn[3] = {1.0e37f, 1.0e37f, 1.0e37f}, mx[3] = {-1.0e37f, -1.0e37f, -1.0e37f};
            for (uint32_t k = 0; k < it.n; k++) {
                const uint32_t p = vals[it.off + k];
                const float4 a = boxes[2u * p], b = boxes[2u * p + 1u];
                const float omn[3] = {a.x, a.y, a.z}, omx[3] = {b.x, b.y, b.z};
                box_include(mn, mx, omn, omx);
            }
            for (int k = 0; k < 3; k++) {
                nd.mn[k] = mn[k];
                nd.mx[k] = mx[k];
            }
            nd.left = nd.right = -1;
            nd.first = it.off;
            nd.n = it.n;
            nd.size = 1;
            continue;
        }
        const uint32_t mask = 1u << it.bit;
        const uint32_t k0 = keys[it.off] & mask;
        if (k0 == (keys[it.off + it.n - 1u] & mask)) {   // same call with the bit dropped
            const uint32_t o = atomicAdd(&ctl->items[in_sel ^ 1u], 1u);
            out[o] = Item{it.off, it.n, it.bit - 1, it.node};
            continue;
        }
        int64_t size = (int64_t)it.n - 2;
        uint32_t first = 1;
        while (size > 0) {
            const int64_t half = size >> 1;
            const uint32_t middle = first + (uint32_t)half;
            if (k0 == (keys[it.off + middle] & mask)) {
                first = middle + 1;
                size -= half + 1;
            } else {
                size = half;
            }
        }
        const uint32_t hi = it.n >= 2u ? it.n - 2u : 0u;   // usize::clamp(first, 0, n - 2)
        const uint32_t offset = first > hi ? hi : first;
        const uint32_t c = atomicAdd(&ctl->pool, 2u);
        nd.left = (int32_t)c;
        nd.right = (int32_t)c + 1;
        const uint32_t o = atomicAdd(&ctl->items[in_sel ^ 1u], 2u);
        out[o] = Item{it.off, offset, it.bit - 1, c};
        out[o + 1u] = Item{it.off + offset, it.n - offset, it.bit - 1, c + 1u};
        res[atomicAdd(&ctl->res, 1u)] = it.node;
    }
}

// between levels: count this level's calls, mark the res list, reset the input count
__global__ void k_level_end(Ctl* ctl, uint32_t in_sel, uint32_t level)
{
    ctl->emits += ctl->items[in_sel];
    ctl->items[in_sel] = 0;
    ctl->lvl_end[level] = ctl->res;
}

// internal nodes resolved at `level` (children resolve later): size and box
// (BvhBuildNode::new_internal: child0's box including child1's)
__global__ void __launch_bounds__(256) k_bottom_up(const Ctl* ctl, uint32_t level, const uint32_t* res, BNode* pool)
{
    const uint32_t lo = level ? ctl->lvl_end[level - 1] : 0u, hi = ctl->lvl_end[level];
    for (uint32_t i = lo + blockIdx.x * 256u + threadIdx.x; i < hi; i += gridDim.x * 256u) {
        BNode& nd = pool[res[i]];
        const BNode& a = pool[nd.left];
        const BNode& b = pool[nd.right];
        for (int k = 0; k < 3; k++) {
            nd.mn[k] = rt_minf(a.mn[k], b.mn[k]);
            nd.mx[k] = rt_maxf(a.mx[k], b.mx[k]);
        }
        nd.size = 1u + a.size + b.size;
    }
}

__global__ void __launch_bounds__(256) k_top_down(const Ctl* ctl, uint32_t level, const uint32_t* res, BNode* pool)
{
    const uint32_t lo = level ? ctl->lvl_end[level - 1] : 0u, hi = ctl->lvl_end[level];
    for (uint32_t i = lo + blockIdx.x * 256u + threadIdx.x; i < hi; i += gridDim.x * 256u) {
        const BNode& nd = pool[res[i]];
        BNode& a = pool[nd.left];
        pool[nd.right].dfs = nd.dfs + 1u + a.size;
        a.dfs = nd.dfs + 1u;
    }
}

// flatten (hlbvh.rs:195-234): GpuNode {min, offset_ptr, max, number_of_prims}
__global__ void __launch_bounds__(256) k_write_nodes(const Ctl* ctl, const BNode* pool, rt_gpu_node* out)
{
    const uint32_t np = ctl->pool;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < np; i += gridDim.x * 256u) {
        const BNode& nd = pool[i];
        rt_gpu_node g;
        for (int k = 0; k < 3; k++) {
            g.min[k] = nd.mn[k];
            g.max[k] = nd.mx[k];
        }
        if (nd.left < 0) {
            g.offset_ptr = nd.first;
            g.n_prims = nd.n;
        } else {
            g.offset_ptr = pool[nd.right].dfs;
            g.n_prims = 0;
        }
        out[nd.dfs] = g;
    }
}

__global__ void __launch_bounds__(256) k_scatter_nodes(const rt_gpu_node* src, const uint32_t* at, uint32_t n,
                                                       rt_gpu_node* out)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) out[at[i]] = src[i];
}

// ------------------------------------------------------------ upper tree (device)
// collapse_build_nodes_recursive + mid_partition (hlbvh.rs:252-291) over the
// <= 4096 treelet roots, in one workgroup.  The recursion's segments are the
// nodes of the midpoint tree over positions [0, n) (children [lo, mid) and
// [mid, hi), mid = lo + (hi - lo) / 2): its shape does not depend on the data.
// Level by level, every segment with >= 2 members takes the longest axis of
// its members' centroid bound (bbox.rs longest_axis) and is sorted stably by
// the centroid on that axis (f32::total_cmp order; ties keep the order the
// level above left, as the host builder's stable_sort does): one bitonic sort
// of (segment start, key, position) per level.  Then, from the final order:
//   * pre-order DFS index of node (lo, hi) at depth d with r right turns on its
//     path: prefix(lo) + d + lo - r, prefix = the subtree sizes of the leaves
//     before it (each right turn passes a left sibling subtree of size - 1
//     internal nodes; the ancestors are the other d);
//   * internal node <-> the boundary m = its mid (1 <= m < n, one each);
//   * boxes bottom-up: child0's box including child1's (rt_minf keeps the left
//     operand on ties, so a fold is the leftmost minimum in position order).
// Bit-identical to rthost::bvh_upper_tree for meshes without NaN coordinates
// (tests/test_gpu_build.py).
namespace upper {
constexpr uint32_t kMax = 4096;   // treelets: 12-bit Morton prefixes
__device__ __forceinline__ uint32_t fkey(float f)   // f32::total_cmp order (-0 < +0)
{
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float funkey(uint32_t k)
{
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
struct Seg {
    uint32_t lo, hi, depth, rights, ord;
};
// the deepest segment containing position p at depth <= lev
__device__ __forceinline__ Seg descend(uint32_t n, uint32_t p, uint32_t lev)
{
    Seg g{0u, n, 0u, 0u, 0u};
    while (g.depth < lev && g.hi - g.lo >= 2u) {
        const uint32_t mid = g.lo + (g.hi - g.lo) / 2u;
        g.ord <<= 1;
        if (p < mid) {
            g.hi = mid;
        } else {
            g.lo = mid;
            g.ord |= 1u;
            g.rights++;
        }
        g.depth++;
    }
    return g;
}
// the internal node whose mid is m (1 <= m < n)
__device__ __forceinline__ Seg node_of(uint32_t n, uint32_t m)
{
    Seg g{0u, n, 0u, 0u, 0u};
    for (;;) {
        const uint32_t mid = g.lo + (g.hi - g.lo) / 2u;
        if (mid == m) return g;
        if (m < mid) {
            g.hi = mid;
        } else {
            g.lo = mid;
            g.rights++;
        }
        g.depth++;
    }
}
__device__ __forceinline__ float centre(const BNode& b, uint32_t k) { return (b.mn[k] + b.mx[k]) * 0.5f; }
}  // namespace upper

__global__ void __launch_bounds__(1024) k_upper_tree(const Ctl* ctl, BNode* pool, rt_gpu_node* up, uint32_t* up_at,
                                                     float* root_box)
{
    using namespace upper;
    __shared__ uint32_t perm[kMax], pre[kMax + 1];
    // sort phase: keys (segments padded to a power of two) + per-segment
    // centroid bounds; output phase: node boxes
    __shared__ __attribute__((aligned(16))) uint8_t pool_lds[2 * kMax * 8 + 6 * (kMax / 2) * 4];
    uint64_t* key = reinterpret_cast<uint64_t*>(pool_lds);                     // [2 kMax]
    uint32_t* bmn = reinterpret_cast<uint32_t*>(pool_lds + 2 * kMax * 8);      // [3][kMax/2]
    uint32_t* bmx = bmn + 3 * (kMax / 2);
    float* box = reinterpret_cast<float*>(pool_lds);                           // [kMax-1][6]
    const uint32_t tid = threadIdx.x, n = ctl->ntreelets;
    if (n == 0u) return;
    uint32_t np = 1, L = 0;
    while (np < n) {
        np <<= 1;
        L++;
    }
    for (uint32_t p = tid; p < n; p += 1024u) perm[p] = p;
    __syncthreads();
    for (uint32_t lev = 0; lev < L; lev++) {
        for (uint32_t i = tid; i < 3u * (kMax / 2); i += 1024u) {
            bmn[i] = 0xFFFFFFFFu;
            bmx[i] = 0u;
        }
        __syncthreads();
        // this thread's positions p = tid + 1024 r: their centroids, loaded together
        // (one round of global loads per level)
        float cc[4][3];
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t p = tid + 1024u * r;
            if (p < n) {
                const BNode& b = pool[perm[p]];
                for (uint32_t k = 0; k < 3; k++) cc[r][k] = centre(b, k);
            }
        }
        for (uint32_t r = 0; r < 4; r++) {   // centroid bounds (Bbox::include_vertex)
            const uint32_t p = tid + 1024u * r;
            if (p >= n) break;
            const Seg g = descend(n, p, lev);
            if (g.hi - g.lo >= 2u)
                for (uint32_t k = 0; k < 3; k++) {
                    const uint32_t c = fkey(cc[r][k]);
                    atomicMin(&bmn[k * (kMax / 2) + g.ord], c);
                    atomicMax(&bmx[k * (kMax / 2) + g.ord], c);
                }
        }
        __syncthreads();
        // every segment of this level in its own block of B (a power of two >= the
        // largest segment, ceil(n / 2^lev)) slots: B << lev <= 2 np keys, sorted block
        // by block -- log2(B) stages instead of log2(np)
        uint32_t B = 1;
        while (B < ((n + (1u << lev) - 1u) >> lev)) B <<= 1;
        const uint32_t tot = B << lev;
        for (uint32_t i = tid; i < tot; i += 1024u) key[i] = ~0ull;
        __syncthreads();
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t p = tid + 1024u * r;
            if (p >= n) break;
            const Seg g = descend(n, p, lev);
            uint32_t k32 = 0;
            if (g.hi - g.lo >= 2u) {
                float d[3];
                for (uint32_t k = 0; k < 3; k++)
                    d[k] = funkey(bmx[k * (kMax / 2) + g.ord]) - funkey(bmn[k * (kMax / 2) + g.ord]);
                const uint32_t dim = d[0] > d[1] ? (d[0] > d[2] ? 0u : 2u) : (d[1] > d[2] ? 1u : 2u);
                k32 = fkey(dim == 0u ? cc[r][0] : dim == 1u ? cc[r][1] : cc[r][2]);
            }
            // a single-member segment that stopped above this level keeps its block at
            // its ordinal scaled to this depth (no real segment lives under it)
            key[(g.ord << (lev - g.depth)) * B + (p - g.lo)] = ((uint64_t)k32 << 12) | p;   // ties: the order above
        }
        __syncthreads();
        for (uint32_t k = 2; k <= B; k <<= 1)        // bitonic sort of each block, ascending
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t q = tid; q < tot / 2u; q += 1024u) {   // compare-exchange pair q: (i, i + j)
                    const uint32_t i = ((q & ~(j - 1u)) << 1) | (q & (j - 1u));
                    const uint64_t a = key[i], b = key[i + j];
                    if ((a > b) == ((k == B) | ((i & k) == 0u))) {
                        key[i] = b;
                        key[i + j] = a;
                    }
                }
                __syncthreads();
            }
        for (uint32_t p = tid; p < n; p += 1024u) {
            const Seg g = descend(n, p, lev);
            pre[p] = perm[(uint32_t)(key[(g.ord << (lev - g.depth)) * B + (p - g.lo)] & 0xFFFu)];
        }
        __syncthreads();
        for (uint32_t p = tid; p < n; p += 1024u) perm[p] = pre[p];
        __syncthreads();
    }
    // exclusive prefix of the leaves' subtree sizes, in position order
    {
        uint32_t loc[4], sum = 0;
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t p = tid * 4u + r;
            loc[r] = p < n ? pool[perm[p]].size : 0u;
            sum += loc[r];
        }
        uint32_t* part = bmn;   // 1024 partial sums (the sort scratch is free)
        part[tid] = sum;
        __syncthreads();
        for (uint32_t off = 1; off < 1024u; off <<= 1) {
            const uint32_t v = tid >= off ? part[tid - off] : 0u;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        uint32_t run = part[tid] - sum;
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t p = tid * 4u + r;
            if (p <= n) pre[p] = run;
            run += loc[r];
        }
        __syncthreads();
    }
    // treelet roots: DFS index of each leaf position
    for (uint32_t p = tid; p < n; p += 1024u) {
        const Seg g = descend(n, p, 32u);
        pool[perm[p]].dfs = pre[p] + g.depth + p - g.rights;
    }
    // internal nodes: boxes bottom-up by depth (deepest first), then the records
    for (int dep = (int)L - 1; dep >= 0; dep--) {
        for (uint32_t m = 1u + tid; m < n; m += 1024u) {
            const Seg g = node_of(n, m);
            if ((int)g.depth != dep) continue;
            float cb[2][6];
            const uint32_t cl[2] = {g.lo, m}, ch[2] = {m, g.hi};
            for (int c = 0; c < 2; c++) {
                if (ch[c] - cl[c] == 1u) {
                    const BNode& b = pool[perm[cl[c]]];
                    for (int k = 0; k < 3; k++) {
                        cb[c][k] = b.mn[k];
                        cb[c][3 + k] = b.mx[k];
                    }
                } else {
                    const uint32_t cm = cl[c] + (ch[c] - cl[c]) / 2u;
                    for (int k = 0; k < 6; k++) cb[c][k] = box[(cm - 1u) * 6u + k];
                }
            }
            for (int k = 0; k < 3; k++) {
                box[(m - 1u) * 6u + k] = rt_minf(cb[0][k], cb[1][k]);
                box[(m - 1u) * 6u + 3 + k] = rt_maxf(cb[0][3 + k], cb[1][3 + k]);
            }
        }
        __syncthreads();
    }
    for (uint32_t m = 1u + tid; m < n; m += 1024u) {
        const Seg g = node_of(n, m);
        const uint32_t dfs = pre[g.lo] + g.depth + g.lo - g.rights;
        rt_gpu_node r;
        for (int k = 0; k < 3; k++) {
            r.min[k] = box[(m - 1u) * 6u + k];
            r.max[k] = box[(m - 1u) * 6u + 3 + k];
        }
        r.offset_ptr = dfs + 1u + (m - g.lo - 1u) + pre[m] - pre[g.lo];   // right child: after the left subtree
        r.n_prims = 0;
        up[m - 1u] = r;
        up_at[m - 1u] = dfs;
    }
    if (tid == 0) {   // GpuNode::new(root bbox) filler (hlbvh.rs:518-525)
        if (n == 1u) {
            for (int k = 0; k < 3; k++) {
                root_box[k] = pool[0].mn[k];
                root_box[3 + k] = pool[0].mx[k];
            }
        } else {
            const uint32_t m = n / 2u;
            for (int k = 0; k < 6; k++) root_box[k] = box[(m - 1u) * 6u + k];
        }
    }
}

__global__ void __launch_bounds__(256) k_fill_nodes_dev(rt_gpu_node* out, uint32_t n, const float* root_box)
{
    rt_gpu_node f;
    for (int k = 0; k < 3; k++) {
        f.min[k] = root_box[k];
        f.max[k] = root_box[3 + k];
    }
    f.offset_ptr = 9999;
    f.n_prims = 9999;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) out[i] = f;
}

// ------------------------------------------------------------ device-wide exclusive scan
// out[0..n] = exclusive prefix sums of in[0..n), out[n] = total (in == out allowed).
// Reduce-then-scan: 4096-element blocks (256 threads x 16), one-block scan of
// the block sums, then each block scans its elements with its offset.
constexpr uint32_t kScanBlock = 4096;
__global__ void __launch_bounds__(256) k_scan_reduce(const uint32_t* in, uint32_t n, uint32_t* bsum)
{
    __shared__ uint32_t red[256];
    const uint32_t base = blockIdx.x * kScanBlock;
    uint32_t s = 0;
    for (uint32_t i = threadIdx.x; i < kScanBlock; i += 256u)
        if (base + i < n) s += in[base + i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) k_scan_down(const uint32_t* in, uint32_t n, const uint32_t* bsum,
                                                   uint32_t* out)
{
    __shared__ uint32_t part[256];
    const uint32_t base = blockIdx.x * kScanBlock + threadIdx.x * 16u;
    uint32_t v[16], s = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        v[i] = base + i < n ? in[base + i] : 0u;
        s += v[i];
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 256u; off <<= 1) {
        const uint32_t a = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += a;
        __syncthreads();
    }
    uint32_t run = bsum[blockIdx.x] + part[threadIdx.x] - s;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (blockIdx.x == gridDim.x - 1u && threadIdx.x == 255u) out[n] = run;
}

}  // namespace rtb

namespace rtk {

int scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* scratch, hipStream_t s)
{
    using namespace rtb;
    const uint32_t nb = n ? (n + kScanBlock - 1) / kScanBlock : 1;
    if (n == 0) {
        (void)hipMemsetAsync(out, 0, 4, s);
        return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
    }
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(256), 0, s, in, n, scratch);
    hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, s, scratch, nb);
    hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(256), 0, s, in, n, scratch, out);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}
size_t scan_scratch_words(uint32_t n) { return (size_t)(n + rtb::kScanBlock - 1) / rtb::kScanBlock + 16; }

// Stable LSD radix sort of (key, value) pairs over the low 8*passes key bits;
// ping-pongs between (k0,v0) and (k1,v1); returns which pair holds the result.
int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, uint32_t passes,
                     uint32_t* hist, hipStream_t s, int& result_in_second)
{
    using namespace rtb;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    result_in_second = 0;
    for (uint32_t pass = 0; pass < passes && n; pass++) {
        const uint32_t sh = pass * 8u;
        hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(256), 0, s, k0, n, sh, ntiles, hist);
        hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, s, hist, 256u * ntiles);
        hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(256), 0, s, k0, v0, n, sh, ntiles, hist, k1, v1);
        std::swap(k0, k1);
        std::swap(v0, v1);
        result_in_second ^= 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}
size_t radix_hist_words(uint32_t n) { return (size_t)256 * ((n + rtb::kTile - 1) / rtb::kTile) + 16; }

// Traversal layout (rt_api.cpp rt_upload_bvh): node record {min.xyz, w0}{max.xyz, w1}
// with byte offsets, and 48-B triangle records {v0, e0, e1, n} in tri_ids order.
__global__ void __launch_bounds__(256) k_bvh_repack(const rt_gpu_node* nodes, uint32_t nnodes, uint32_t rec_off,
                                                    uint4* blob)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nnodes; i += gridDim.x * 256u) {
        const rt_gpu_node n = nodes[i];
        uint32_t w0, w1;
        if (n.n_prims > 0) {
            w0 = rec_off + 48u * n.offset_ptr;
            w1 = 48u * n.n_prims;
        } else {
            w0 = 32u * n.offset_ptr;
            w1 = 0u;
        }
        blob[2u * i] = make_uint4(__float_as_uint(n.min[0]), __float_as_uint(n.min[1]), __float_as_uint(n.min[2]), w0);
        blob[2u * i + 1u] =
            make_uint4(__float_as_uint(n.max[0]), __float_as_uint(n.max[1]), __float_as_uint(n.max[2]), w1);
    }
}

__global__ void __launch_bounds__(256) k_tri_records(const float4* pos, const uint4* idx, const uint32_t* ids,
                                                     uint32_t nids, float4* recs)
{
    for (uint32_t k = blockIdx.x * 256u + threadIdx.x; k < nids; k += gridDim.x * 256u) {
        const uint4 ix = idx[ids[k]];
        const float4 a = pos[ix.x], b = pos[ix.y], c = pos[ix.z];
        const float e0[3] = {b.x - a.x, b.y - a.y, b.z - a.z};
        const float e1[3] = {c.x - a.x, c.y - a.y, c.z - a.z};
        const float n[3] = {e0[1] * e1[2] - e0[2] * e1[1], e0[2] * e1[0] - e0[0] * e1[2], e0[0] * e1[1] - e0[1] * e1[0]};
        recs[3u * k] = make_float4(a.x, a.y, a.z, e0[0]);
        recs[3u * k + 1u] = make_float4(e0[1], e0[2], e1[0], e1[1]);
        recs[3u * k + 2u] = make_float4(e1[2], n[0], n[1], n[2]);
    }
}

int launch_bvh_repack(const rt_gpu_node* nodes, uint32_t nnodes, uint32_t rec_off, void* blob, const float4* pos,
                      const uint4* idx, const uint32_t* ids, uint32_t nids, hipStream_t s)
{
    const uint32_t g1 = std::min<uint32_t>(8192, (nnodes + 255) / 256 + 1);
    hipLaunchKernelGGL(k_bvh_repack, dim3(g1), dim3(256), 0, s, nodes, nnodes, rec_off, reinterpret_cast<uint4*>(blob));
    const uint32_t g2 = std::min<uint32_t>(8192, (nids + 255) / 256 + 1);
    hipLaunchKernelGGL(k_tri_records, dim3(g2), dim3(256), 0, s, pos, idx, ids, nids,
                       reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(blob) + rec_off));
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

namespace {
struct Scratch {   // freed at scope exit
    std::vector<void*> p;
    ~Scratch()
    {
        for (void* q : p) (void)hipFree(q);
    }
    template <class T>
    T* alloc(size_t count, hipError_t& e)
    {
        void* q = nullptr;
        if (e == hipSuccess) e = hipMalloc(&q, std::max<size_t>(16, count * sizeof(T)));
        if (e == hipSuccess) p.push_back(q);
        return reinterpret_cast<T*>(q);
    }
};
}  // namespace

int build_bvh_device(const float4* pos, const uint4* idx, uint32_t nt, uint32_t max_prims, int num_cus,
                     hipStream_t s, BvhDeviceOut& out, rt_bvh_build_times* times, std::string& err)
{
    using namespace rtb;
    if (nt == 0) {
        err = "rt_build_bvh_device: empty mesh";
        return RT_E_INVALID;
    }
    hipError_t e = hipSuccess;
    // node pool bound: with max_prims >= 3 every split leaves both sides
    // non-empty (<= 2 nodes per primitive); with 1 or 2 the clamp of
    // hlbvh.rs:408 can split n = 2 into an empty leaf and the same pair one
    // bit lower, so up to 2 new nodes per item per level
    const size_t pool_cap = (max_prims >= 3 ? (size_t)2 * nt : (size_t)2 * kLevels * nt) + 4096;
    const size_t item_cap = (max_prims >= 3 ? (size_t)nt : (size_t)2 * nt) + 4096;
    Scratch S;
    const uint32_t grid = (uint32_t)std::max(1, num_cus) * 8u;
    const uint32_t ntiles = (nt + kTile - 1) / kTile;
    float4* boxes = S.alloc<float4>((size_t)nt * 2, e);
    float* partial = S.alloc<float>((size_t)grid * 6, e);
    float* bound = S.alloc<float>(8, e);
    uint32_t* k0 = S.alloc<uint32_t>(nt, e);
    uint32_t* v0 = S.alloc<uint32_t>(nt, e);
    uint32_t* k1 = S.alloc<uint32_t>(nt, e);
    uint32_t* v1 = S.alloc<uint32_t>(nt, e);
    uint32_t* hist = S.alloc<uint32_t>((size_t)256 * ntiles, e);
    uint32_t* tcount = S.alloc<uint32_t>(4096, e);
    Item* items0 = S.alloc<Item>(item_cap, e);
    Item* items1 = S.alloc<Item>(item_cap, e);
    BNode* pool = S.alloc<BNode>(pool_cap, e);
    uint32_t* res = S.alloc<uint32_t>(pool_cap, e);
    Ctl* ctl = S.alloc<Ctl>(1, e);
    rt_gpu_node* d_up = S.alloc<rt_gpu_node>(upper::kMax, e);   // upper-tree records and their DFS slots
    uint32_t* d_upat = S.alloc<uint32_t>(upper::kMax, e);
    float* d_rootbox = S.alloc<float>(8, e);
    if (e != hipSuccess) {
        err = std::string("rt_build_bvh_device: scratch allocation: ") + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? RT_E_OOM : RT_E_DEVICE;
    }
    hipEvent_t ev[7];
    for (auto& x : ev) (void)hipEventCreate(&x);
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard()
        {
            for (int i = 0; i < 7; i++) (void)hipEventDestroy(e[i]);
        }
    } evg{ev};
    auto chk = [&](const char* what) {
        const hipError_t r = hipGetLastError();
        if (r != hipSuccess && e == hipSuccess) {
            e = r;
            err = std::string("rt_build_bvh_device: ") + what + ": " + hipGetErrorString(r);
        }
    };
    const auto t_start = std::chrono::steady_clock::now();
    (void)hipEventRecord(ev[0], s);
    // -- morton codes
    hipLaunchKernelGGL(k_boxes, dim3(grid), dim3(256), 0, s, pos, idx, nt, boxes, partial);
    hipLaunchKernelGGL(k_bound, dim3(1), dim3(256), 0, s, partial, grid, bound);
    hipLaunchKernelGGL(k_morton, dim3(grid), dim3(256), 0, s, boxes, bound, nt, k0, v0);
    chk("morton");
    (void)hipEventRecord(ev[1], s);
    // -- radix sort (stable; 30-bit codes: 4 passes)
    for (uint32_t pass = 0; pass < 4; pass++) {
        const uint32_t sh = pass * 8u;
        hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(256), 0, s, k0, nt, sh, ntiles, hist);
        hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, s, hist, 256u * ntiles);
        hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(256), 0, s, k0, v0, nt, sh, ntiles, hist, k1, v1);
        std::swap(k0, k1);
        std::swap(v0, v1);
    }
    chk("radix sort");
    (void)hipEventRecord(ev[2], s);
    // -- treelets
    (void)hipMemsetAsync(tcount, 0, 4096 * 4, s);
    hipLaunchKernelGGL(k_treelet_count, dim3(grid), dim3(256), 0, s, k0, nt, tcount);
    hipLaunchKernelGGL(k_treelet_list, dim3(1), dim3(1024), 0, s, tcount, items0, ctl);
    chk("treelets");
    (void)hipEventRecord(ev[3], s);
    // -- emit_lbvh, one level per bit
    Item* bufs[2] = {items0, items1};
    for (uint32_t L = 0; L < (uint32_t)kLevels; L++) {
        const uint32_t sel = L & 1u;
        hipLaunchKernelGGL(k_lbvh_level, dim3(grid), dim3(256), 0, s, bufs[sel], sel, bufs[sel ^ 1u], ctl, k0, v0,
                           boxes, max_prims, pool, res);
        hipLaunchKernelGGL(k_level_end, dim3(1), dim3(1), 0, s, ctl, sel, L);
    }
    for (int L = kLevels - 1; L >= 0; L--)
        hipLaunchKernelGGL(k_bottom_up, dim3(grid), dim3(256), 0, s, ctl, (uint32_t)L, res, pool);
    chk("treelet build");
    (void)hipEventRecord(ev[4], s);
    // -- upper tree on the device (<= 4096 treelet roots, k_upper_tree); the host
    //    only reads the two counts that size the output (the reference's total_nodes)
    Ctl hc;
    if (e == hipSuccess) e = hipMemcpyAsync(&hc, ctl, sizeof hc, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        if (err.empty()) err = std::string("rt_build_bvh_device: ") + hipGetErrorString(e);
        return RT_E_DEVICE;
    }
    if (hc.ntreelets == 0u || hc.ntreelets > upper::kMax) {
        err = "rt_build_bvh_device: treelet count out of range";
        return RT_E_DEVICE;
    }
    const uint32_t n_up = hc.ntreelets - 1u;            // internal nodes of the upper tree
    const uint32_t total = hc.emits + n_up;             // the reference's total_nodes (array length)
    hipLaunchKernelGGL(k_upper_tree, dim3(1), dim3(1024), 0, s, ctl, pool, d_up, d_upat, d_rootbox);
    chk("upper tree");
    (void)hipEventRecord(ev[5], s);
    // -- flattening
    out.nnodes = total;
    out.nids = nt;
    if ((e = hipMalloc(&out.nodes, (size_t)total * sizeof(rt_gpu_node))) != hipSuccess ||
        (e = hipMalloc(&out.ids, (size_t)nt * 4)) != hipSuccess) {
        err = "rt_build_bvh_device: output allocation failed";
        return RT_E_OOM;
    }
    for (uint32_t L = 0; L < (uint32_t)kLevels; L++)
        hipLaunchKernelGGL(k_top_down, dim3(grid), dim3(256), 0, s, ctl, L, res, pool);
    hipLaunchKernelGGL(k_fill_nodes_dev, dim3(grid), dim3(256), 0, s, out.nodes, total, d_rootbox);
    hipLaunchKernelGGL(k_write_nodes, dim3(grid), dim3(256), 0, s, ctl, pool, out.nodes);
    if (n_up)
        hipLaunchKernelGGL(k_scatter_nodes, dim3(grid), dim3(256), 0, s, d_up, d_upat, n_up, out.nodes);
    (void)hipMemcpyAsync(out.ids, v0, (size_t)nt * 4, hipMemcpyDeviceToDevice, s);
    chk("flatten");
    (void)hipEventRecord(ev[6], s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        if (err.empty()) err = std::string("rt_build_bvh_device: ") + hipGetErrorString(e);
        return RT_E_DEVICE;
    }
    if (times) {
        float ms[6] = {0, 0, 0, 0, 0, 0};
        for (int i = 0; i < 4; i++) (void)hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]);
        (void)hipEventElapsedTime(&ms[5], ev[5], ev[6]);
        times->morton_codes_ms = ms[0];
        times->radix_sort_ms = ms[1];
        times->treelet_init_ms = ms[2];
        times->treelet_build_ms = ms[3];
        // upper tree: the count read-back + k_upper_tree (no host work left)
        float up_ms = 0.0f;
        (void)hipEventElapsedTime(&up_ms, ev[4], ev[5]);
        times->upper_tree_ms = up_ms;
        times->upper_tree_host_ms = 0.0;
        times->flattening_ms = ms[5];
        times->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        times->treelets = hc.ntreelets;
        times->nodes = total;
    }
    return RT_OK;
}

}  // namespace rtk
