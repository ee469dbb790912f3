/*
 * rt_oracle.h -- CPU ORACLE for the render hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline -- the product path
 * (librt_hip.so) never links, loads or calls anything under oracle/.
 *
 * What it is: a line-by-line C restatement of the reference GLSL compute shaders and of
 * the host code that feeds them (paths relative to /root/reference/Raytracing-Sandbox/Src/):
 *   IOW-00  In-One-Weekend/base.cpp:7-28 (default compute shader)          (orc_render_iow00)
 *   IOW-01  In-One-Weekend/01_Adding_Sphere/computeShaderSrc.glsl            (orc_render_iow01)
 *   IOW-02  In-One-Weekend/02_Groups/computeShaderSrc.glsl                   (orc_render_iow02)
 *   IOW-03  In-One-Weekend/03_Shadows_and_Materials/computeShaderSrc.glsl    (orc_render_iow03)
 *   INW-01  In-Next-Week/01_BoundingVolumeHierarchy/computeShaderSrc.glsl    (orc_render_inw, layout 1;
 *           its "#if MULTIFOCUS" branch: orc_render_inw_mf)
 *   INW-04  In-Next-Week/04_Lights_Camera_And_Action/computeShaderSrc.glsl   (orc_render_inw, layout 4)
 *   LBVH    In-Next-Week/LBVH/lbvh.h                                         (orc_lbvh_build)
 *   packers materials.h:48-86, base.h:24-71, BVH.h:47-58, lights.h:40-141, utility.cpp:489-516
 *
 * PARITY STATUS: UNPINNED against the reference itself.  The reference has no CPU
 * renderer, no tests, no golden images and no known-answer vectors; its
 * shaders need an OpenGL 4.4 context and its harness #errors on Linux; lbvh.h needs glm,
 * an un-vendored submodule, so it is unbuildable here.  The oracle is pinned only by
 * analytic known-answer tests (tests/test_oracle_kat.py) and by structural properties.
 *
 * Numerics contract (identical in the HIP kernels):
 *   IEEE binary32; GLSL evaluation order; no FMA contraction (-ffp-contract=off);
 *   GLSL a/b  ==  a * RN(1/b);  sqrt correctly rounded;  normalize(v) == v*RN(1/sqrt(dot(v,v)));
 *   min/max == fminf/fmaxf;  pow(x,5) == ((((x*x)*x)*x)*x);  pow(x,1) == x;
 *   sin/cos/tan only in host tables computed in double and rounded to float;
 *   uninitialised GLSL values == 0; out-of-range local-array reads == 0;
 *   float -> uint of a negative value truncates toward zero (clamps to 0).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Same memory layout as rt_camera / rt_params / rt_stats / rt_geom_desc in include/. */
typedef struct { float pos[3]; float dir[3]; float fov_y_rad, aperture, focus_dist; } orc_camera;
typedef struct { int width, height, spp, max_bounces; int tile_x0, tile_y0, tile_w, tile_h;
                 int show_normal; int device; } orc_params;
typedef struct { uint64_t segments, node_visits, prim_tests, shadow_queries, stack_drops,
                 nan_drops; double ms; } orc_stats;
typedef struct {
    int type; float position[3], last_position[3], rotation_deg[3], scale[3], color[3];
    float refractivity, reflectivity, refractive_index, scat_refract, scat_reflect;
    int emissive, texture_index;
} orc_geom_desc;

int orc_num_threads(void);
void orc_set_threads(int n);

int orc_render_iow00(const orc_params *p, float *rgba);
int orc_render_iow01(const orc_camera *cam, const float sphere[4], const orc_params *p,
                     float *rgba, orc_stats *st);
/* IOW-02 records: N x 18 floats = position, inverse rotation (glm column-major), scale, colour
 * (groups.h:11-17, the first 18 floats of an IOW-03 record); types 1 = CUBOID, 2 = ELLIPSOID */
int orc_render_iow02(const float *types, const float *records, uint32_t n, const orc_camera *cam,
                     const orc_params *p, int cull_front, int cull_back, float *rgba, orc_stats *st);
int orc_render_iow03(const float *types, const float *records, uint32_t n,
                     const orc_camera *cam, const orc_params *p, float *rgba, orc_stats *st);
int orc_render_inw(const float *geom, uint32_t n, int layout, const float *nodes,
                   const float *lights, uint32_t n_lights, const orc_camera *cam,
                   const orc_params *p, float *rgba, float *depth, orc_stats *st);
/* INW-01 (layout 1) with MULTIFOCUS compiled in: focus[0..n_focus-1], 1 <= n_focus <= 9 */
int orc_render_inw_mf(const float *geom, uint32_t n, const float *nodes, const orc_camera *cam,
                      const float *focus, int n_focus, const orc_params *p, float *rgba, float *depth,
                      orc_stats *st);

/* INW-04 material textures: texels row 0 first (GL upload order), channels 3 (RGB8) or 4 (RGBA8) */
typedef struct { const uint8_t *texels; int width, height, channels; } orc_texture;
int orc_render_inw_tex(const float *geom, uint32_t n, int layout, const float *nodes,
                       const float *lights, uint32_t n_lights, const orc_texture *tex, uint32_t n_tex,
                       const orc_camera *cam, const orc_params *p, float *rgba, float *depth, orc_stats *st);
/* Helper::Noise::MakeTexture<glm::vec3> (utility.h:69-192): RGB8 texels, width*height*3 */
int orc_noise_texture(int width, int height, int type, const float *gradient, int n_grad, float freq,
                      float lac, float gain, int octaves, uint8_t *rgb_out);
/* TEXTURE_2D::LoadFromDiskToGPU's re-projection (utility.cpp:266-463): load_as / map_to 0 =
 * MERCATOR, 1 = CUBIC */
int orc_texture_remap(const uint8_t *in, int width, int height, int channels, int load_as, int map_to,
                      uint8_t *out);
int orc_lbvh_build(const float *aabbs, uint32_t n, float *nodes_out);
int orc_pack_iow03(const orc_geom_desc *g, uint32_t n, float *types, float *records);
int orc_pack_inw(const orc_geom_desc *g, uint32_t n, int layout, float *geom, float *aabbs,
                 float *lights, uint32_t *n_lights);
int orc_sample_tables(int spp, float *sunflower, float *fib, int *ring);

#ifdef __cplusplus
}
#endif
#endif
