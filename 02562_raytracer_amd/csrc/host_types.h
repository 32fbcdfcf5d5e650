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
// thread-local last error for context-less calls
void set_error(const std::string& msg);
const char* get_error();
}  // namespace rthost
