/*
 * integration_seq.c -- the call sequence INTEGRATION.md gives a maintainer of the
 * reference (the Rust `RenderState` hooks), performed through include/rt.h in C:
 *
 *   gpu_handles::self_test        -> rt_device_count
 *   GPUHandles::new               -> rt_create
 *   Mesh::from_obj                -> (stand-in: rt_mesh_load_obj + rt_mesh_view_get; the
 *                                    reference's Mesh has the same four public arrays)
 *   MaterialsGpu::new light list  -> computed here as storage_mesh.rs:316-332 does
 *   StorageMeshGpu::new_*         -> rt_upload_mesh  (raw pointers)
 *   BspTreeIntermediate::new      -> (stand-in: rt_bsp_build + rt_bsp_view_get; the reference's
 *                                    intermediate has the same public fields)
 *   BspTreeGpu::new               -> rt_upload_bsp   (raw pointers)
 *   UniformGpu::update_buffer     -> rt_set_uniforms (iteration = the frame index)
 *   RenderState::render (x iters) -> rt_render, one progressive iteration per call
 *   reading the accumulation      -> rt_memcpy_to_host
 *
 * usage: integration_seq <model.obj> <W> <H> <iterations> <out.bin>
 * out.bin: W*H float4 accumulation, then W*H u32 primary-hit ids.
 * Exit status 0 on success; a failing call prints rt_last_error and exits 1.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt.h"

static rt_ctx* g_ctx;

static void check(int rc, const char* what)
{
    if (rc != RT_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, rt_last_error(g_ctx));
        exit(1);
    }
}

int main(int argc, char** argv)
{
    if (argc != 6) {
        fprintf(stderr, "usage: %s <model.obj> <W> <H> <iterations> <out.bin>\n", argv[0]);
        return 2;
    }
    const uint32_t W = (uint32_t)atoi(argv[2]), H = (uint32_t)atoi(argv[3]), iters = (uint32_t)atoi(argv[4]);

    int ndev = 0;
    check(rt_device_count(&ndev), "rt_device_count");
    if (ndev < 1) {
        fprintf(stderr, "no HIP device\n");
        return 1;
    }
    check(rt_create(0, &g_ctx), "rt_create");

    rt_mesh_host* mesh = NULL;
    check(rt_mesh_load_obj(argv[1], &mesh), "rt_mesh_load_obj");
    rt_mesh_view mv;
    check(rt_mesh_view_get(mesh, &mv), "rt_mesh_view_get");

    /* MaterialsGpu::new (storage_mesh.rs:316-332): triangles whose material has
     * emissive == 1, after a u32::MAX sentinel */
    uint32_t* lights = (uint32_t*)malloc(sizeof(uint32_t) * (mv.ntris + 1));
    uint32_t nlights = 0;
    lights[nlights++] = 0xFFFFFFFFu;
    for (uint32_t t = 0; t < mv.ntris; t++) {
        const uint32_t m = mv.indices[4 * t + 3];
        if (m < mv.nmats && mv.materials[m].emissive == 1) lights[nlights++] = t;
    }
    check(rt_upload_mesh(g_ctx, mv.vertices, mv.normals, mv.nverts, mv.indices, mv.ntris, mv.materials, mv.nmats,
                         lights, nlights),
          "rt_upload_mesh");

    rt_bsp_host* bsp = NULL;
    check(rt_bsp_build(mesh, 20, 4, 0, &bsp), "rt_bsp_build");   /* Mesh::bsp_tree: depth 20, leaf 4 */
    rt_bsp_view bv;
    check(rt_bsp_view_get(bsp, &bv), "rt_bsp_view_get");
    check(rt_upload_bsp(g_ctx, bv.aabb, bv.tree, bv.planes, bv.nnodes, bv.ids, bv.nids, bv.max_depth),
          "rt_upload_bsp");

    /* Uniform of the W7 E3 Cornell Box scene (scenes.rs:63-69), aspect = W/H */
    rt_uniform u;
    memset(&u, 0, sizeof u);
    const float eye[3] = {277.0f, 275.0f, -570.0f}, at[3] = {277.0f, 275.0f, 0.0f}, up[3] = {0.0f, 1.0f, 0.0f};
    memcpy(u.camera_pos, eye, sizeof eye);
    memcpy(u.camera_look_at, at, sizeof at);
    memcpy(u.camera_up, up, sizeof up);
    u.camera_constant = 1.0f;
    u.aspect_ratio = (float)W / (float)H;
    u.selection1 = 0;
    u.subdivision_level = 1;
    u.uv_scale[0] = u.uv_scale[1] = 1.0f;
    u.resolution[0] = W;
    u.resolution[1] = H;

    void* accum = NULL;
    void* ids = NULL;
    check(rt_device_alloc(g_ctx, (size_t)W * H * 16, &accum), "rt_device_alloc");
    check(rt_device_alloc(g_ctx, (size_t)W * H * 4, &ids), "rt_device_alloc");
    check(rt_memset_device(g_ctx, accum, 0, (size_t)W * H * 16), "rt_memset_device");
    const rt_tile full = {0, 0, W, H};
    for (uint32_t it = 0; it < iters; it++) {   /* rendering_thread: render(), then iteration += 1 */
        u.iteration = it;
        check(rt_set_uniforms(g_ctx, &u, NULL), "rt_set_uniforms");
        check(rt_render(g_ctx, RT_MODE_W7E3, RT_TRAVERSE_BSP, &full, it, 1, (float*)accum, (uint32_t*)ids, NULL),
              "rt_render");
    }
    float* h_acc = (float*)malloc((size_t)W * H * 16);
    uint32_t* h_ids = (uint32_t*)malloc((size_t)W * H * 4);
    check(rt_memcpy_to_host(g_ctx, h_acc, accum, (size_t)W * H * 16), "rt_memcpy_to_host");
    check(rt_memcpy_to_host(g_ctx, h_ids, ids, (size_t)W * H * 4), "rt_memcpy_to_host");
    FILE* f = fopen(argv[5], "wb");
    if (!f || fwrite(h_acc, 16, (size_t)W * H, f) != (size_t)W * H || fwrite(h_ids, 4, (size_t)W * H, f) != (size_t)W * H) {
        fprintf(stderr, "cannot write %s\n", argv[5]);
        return 1;
    }
    fclose(f);
    check(rt_device_free(g_ctx, accum), "rt_device_free");
    check(rt_device_free(g_ctx, ids), "rt_device_free");
    rt_bsp_free(bsp);
    rt_mesh_free(mesh);
    free(lights);
    free(h_acc);
    free(h_ids);
    rt_destroy(g_ctx);
    return 0;
}
