// host_types.h -- host-side containers behind the opaque rt_*_host handles.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt.h"

struct rt_mesh_host {
    std::vector<float> pos;        // nverts x 4
    std::vector<float> nrm;        // nverts x 4
    std::vector<uint32_t> idx;     // ntris x 4 (v0, v1, v2, material)
    std::vector<rt_material> mats;
    std::vector<uint32_t> lights;  // [0] = UINT32_MAX sentinel
    uint32_t nverts() const { return (uint32_t)(pos.size() / 4); }
    uint32_t ntris() const { return (uint32_t)(idx.size() / 4); }
};

struct rt_bsp_host {
    std::vector<uint32_t> tree;    // nnodes x 4
    std::vector<float> planes;
    std::vector<uint32_t> ids;
    float aabb[8];
    uint32_t max_depth;
};

struct rt_bvh_host {
    std::vector<rt_gpu_node> nodes;
    std::vector<uint32_t> tri_ids;
};

namespace rthost {
// StorageMeshGpu light list (src/bindings/storage_mesh.rs:316-326).
std::vector<uint32_t> light_list(const std::vector<uint32_t>& idx, const std::vector<rt_material>& mats);
rt_material default_material();
// hlbvh.rs upper tree (collapse_build_nodes_recursive + mid_partition,
// src/data_structures/hlbvh.rs:252-291) over the treelet roots' boxes
// (mn.xyz, mx.xyz each): nodes[0] is the root when there are >= 2 roots.
// An entry with root >= 0 stands for treelet root `root`; otherwise it is an
// internal node whose children are entries `left` and `right` (child0 first).
// Returns the number of internal nodes (the `total_nodes` increments).
struct UpperNode {
    float mn[3], mx[3];
    int32_t root;          // treelet index, or -1 for an internal node
    int32_t left, right;   // entry indices (internal nodes)
};
uint32_t bvh_upper_tree(const std::vector<float>& root_boxes, std::vector<UpperNode>& out);
// thread-local last error for context-less calls
void set_error(const std::string& msg);
const char* get_error();
}  // namespace rthost
