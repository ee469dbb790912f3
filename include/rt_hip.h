/*
 * rt_hip.h -- C ABI of the MI355X-native render path (librt_hip.so).
 *
 * This is the drop-in boundary for the reference's per-pixel render loop.  In the
 * reference the boundary is the OpenGL compute-dispatch contract: sampler units 0/1
 * bound to the geometry / LBVH "buffer textures", a set of uniforms, an optional light
 * SSBO, then glDispatchCompute.  Each entry point below replaces one such dispatch
 * (file:line citations are relative to /root/reference/Raytracing-Sandbox/Src/):
 *
 *   rt_render_iow01  <- In_One_Weekend::Sphere::OnUpdate             01_Adding_Sphere/Sphere.cpp:51-64
 *                       (uniforms Sphere.cpp:54-61, dispatch (W,H,1) Sphere.cpp:63)
 *   rt_render_iow03  <- In_One_Weekend::Adding_Materials::OnUpdate   03_Shadows_and_Materials/materials.cpp:118-146
 *                       (uniforms :121-135, textures :137-140, per-tile dispatch :142-143)
 *   rt_render_inw    <- In_Next_Week::RT_Base<>::OnUpdateBase        In-Next-Week/base.h:148-173
 *                       (layout 1 = BVH stage, 01_BoundingVolumeHierarchy/BVH.cpp:26-43;
 *                        layout 4 = Lights stage + SSBO, 04_Lights_Camera_And_Action/lights.cpp:15-37)
 *   rt_lbvh_build    <- LBVH::ConstructLBVH_Buff                      In-Next-Week/LBVH/lbvh.h:215-269
 *                       (called from base.h:135 on every redraw)
 *
 * Conventions:
 *   - POD structs, caller-owned host memory, library-owned device memory.
 *   - int status: 0 = ok, negative = error (RT_E_*); no exceptions cross the ABI.
 *   - Output images are row-major, row y = pixel_coords.y (GL bottom row first),
 *     RGBA float32 with alpha = 1, exactly the reference's rgba32f image memory.
 *     The depth image (INW only) is one float per pixel (the reference's r32f image).
 *   - The *_async variants take DEVICE pointers (inputs already resident in HBM) and a
 *     hipStream_t passed as void*; they never allocate or synchronise (graph-capturable).
 *   - Threading: calls are reentrant per distinct output buffer.
 *
 * Numerics contract shared with the CPU oracle (DESIGN.md "Numerics contract"):
 * IEEE binary32, GLSL evaluation order, no FMA contraction, GLSL a/b == a*RN(1/b),
 * correctly rounded sqrt and reciprocal, transcendentals only in host-built double
 * precision tables.  Under this contract the GPU image is bit-identical to the oracle's.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 5

/* status codes */
#define RT_OK            0
#define RT_E_ARG        -1   /* bad argument (null pointer, non-positive size, bad layout) */
#define RT_E_HIP        -2   /* a HIP runtime call failed */
#define RT_E_NODEVICE   -3   /* no usable gfx950 device */
#define RT_E_UNSUPPORTED -4  /* a feature the call cannot serve (e.g. TextureIndex > 0 with no texture bound) */

/* Camera uniforms.
 *   IOW-01: u_CameraPosn, u_CameraDirn, u_FocusDist            (01_Adding_Sphere/computeShaderSrc.glsl:5-7)
 *   IOW-03: u_CameraPosn, u_CameraDirn, u_FOV_y, u_CamAperture, u_CamFocusDist (03...glsl:7-13)
 *   INW   : u_Camera{Position, Direction, FOV_y, FocusDist[0], Aperture} (01_BoundingVolumeHierarchy/computeShaderSrc.glsl:221-228)
 * dir is passed exactly as the reference host computes it (IOW: normalized FrontFromPitchYaw,
 * materials.cpp:321-328; INW: RT_Base::m_Camera.Front(), NOT normalized, base.h:274-281). */
typedef struct rt_camera {
    float pos[3];
    float dir[3];
    float fov_y_rad;
    float aperture;
    float focus_dist;
} rt_camera;

/* Render parameters.
 *   width, height : full image size (imageSize(img_output))
 *   spp           : IOW-03 u_NumOfSamples; INW local_size_x (samples per pixel, any value >= 1)
 *   max_bounces   : IOW-03 u_NumOfBounce; INW u_NumOfBounces
 *   tile_*        : rectangle of pixels to render (IOW-03 u_TileIndex*u_TileSize and the
 *                   per-tile dispatch size, materials.cpp:126-143).  tile_w/tile_h <= 0 => full image.
 *   show_normal   : IOW-01/IOW-03 u_ShowNormal
 *   device        : HIP device ordinal for the blocking entry points (-1 = current) */
typedef struct rt_params {
    int width, height, spp, max_bounces;
    int tile_x0, tile_y0, tile_w, tile_h;
    int show_normal;
    int device;
} rt_params;

/* Counters, identical definitions in the kernels and in the oracle (DESIGN.md "Counters"). */
typedef struct rt_stats {
    uint64_t segments;        /* rays cast (primary + secondary), i.e. closest-hit queries   */
    uint64_t node_visits;     /* LBVH nodes fetched+tested (closest-hit, shadow, RI walks)   */
    uint64_t prim_tests;      /* primitive tests (IOW linear loop, INW leaves, RI inside)    */
    uint64_t shadow_queries;  /* INW-04 shadow rays                                          */
    uint64_t stack_drops;     /* pushes silently dropped by a full stack                     */
    uint64_t nan_drops;       /* secondary directions that came out NaN                      */
    double   ms;              /* device time of the render launch(es), milliseconds          */
} rt_stats;

/* ---- options ------------------------------------------------------------------------
 * The strategy switches of the render path.  Every strategy is exact: the image, the depth
 * and the ray-level counters are bit-identical whatever the options (tests/test_gpu_bvh_exact.py);
 * only speed and the build's own node / primitive counts change.  The defaults (rt_options_default)
 * are the measured-best settings; nothing else (no environment variable) changes what the
 * library runs.  rt_options_set sets the library-wide options; a device scene copies them when
 * it is created (rt_dev_scene_*) and rt_dev_scene_set_options replaces its copy.  The blocking
 * entry points build a scene per call, so they use the options current at the call.
 * Options marked [build] shape the scene's device structures and are read at scene creation only. */
typedef struct rt_options {
    uint32_t size;          /* sizeof(rt_options), set by rt_options_default; checked by the setters */
    /* INW (In-Next-Week 01 / 04) */
    int inw_wide_walk;      /* [build] 1: 4-wide culling walk with the reference's leaf tests; 0: the LBVH walk as the shader does it */
    int inw_order;          /* fold kernel: 0 = the probe picks, 1 = pixel-major, 2 = sample-major, -1 = per-pixel k_inw */
    int inw_beams;          /* per-pixel candidate lists for primary rays (pixel-major frames); 1: entries of
                               32 bits (16-bit object id, entry t rounded down) when ids fit, 2: (id, t) pairs */
    int inw_ri_grid;        /* surrounding-RI queries through the uniform grid */
    int inw_lds_nodes;      /* top of the wide BVH staged in LDS (768-lane blocks) */
    int inw_fused_cull;     /* one fma per culling plane where the error bound holds */
    int inw_claim_order;    /* pixel-major claims costliest 8x8 blocks first */
    int inw_ring_pm;        /* pixel-major fold ring: 0 (default) in LDS, 256 entries per wave, the walks
                               reading every node from L1 / L2; else a global ring of that many entries
                               per wave (power of two >= 64) beside 236 staged nodes */
    int inw_ring_sm;        /* sample-major fold ring: 0 (default) in LDS, 256 entries per wave, when the
                               scene's BVH top fits the 5 nodes staged beside it (nothing lost), else a
                               global ring of 256; else a global ring of that many entries per wave */
    int inw_stackless;      /* the reference's LBVH walks (closest hit, surrounding RI) without their stack, by
                               the node buffer's parent links, wherever no push could drop; their top
                               nodes staged in LDS when there is no wide walk (DESIGN.md "Stackless") */
    int inw_device_build;   /* rt_dev_scene_inw_update with the LBVH built on the device: the wide walk's
                               4-wide BVH (binned SAH), ranks and RI grid built on the device too (0: on
                               the host from the read-back LBVH, as rt_dev_scene_inw does) */
    int inw_claim_xcd;      /* pixel-major claims from 8 queues, one per XCD (an 8x8 block's pixels are
                               written by one XCD's L2, whole lines), idle XCDs taking from the others */
    int inw_qnodes;         /* 1: pixel-major INW-01 frames with the fused cull run k_inw_pm's GQ instance
                               (DESIGN.md §5.1): the reference's 40-float stacks in global memory with the
                               top ray in registers, the wide walk's node stack and the top of the culling
                               BVH in LDS (quantised 64-B nodes, 1,168 of them); 0 (default, measured faster):
                               the FStack instance */
    int inw_time_bins;      /* moving objects: the wide walk culls with one of this many extra culling trees,
                               each over the boxes the objects sweep in its share of the shutter interval
                               (the ray's time ratio picks it; DESIGN.md §5.2 "Time-binned culling trees");
                               0 or 1: the swept tree only.  Default 2 (4 and 8 measured slower: their trees crowd
                               the L2); scenes built on the host */
    int inw_walk_bins;      /* 1 (default): the wide closest-hit walks use the time-bin trees */
    int inw_beam_bins;      /* 1 (default): a pixel's beam lists per time bin, from the time-bin trees */
    int inw_sphere_records; /* 1 (default): in scenes of equal-scale ellipsoids with the identity rotation, the
                               wide walk, beam lists and RI grid read 3-float4 sphere records */
    int inw_compact_nodes;  /* 1 (default): the wide walk reads its nodes from global memory as 7 float4
                               (112 B) instead of 10 (the repeated low planes dropped) */
    /* IOW-03 (In-One-Weekend 03) */
    int iow_spec;           /* sample-parallel speculation (0: the sequential per-pixel kernel) */
    int iow_linear;         /* [build] the shader's linear object loop instead of the culling BVH */
    int iow_narrow;         /* byte bounce counts / 12-deep BVH stack variant (u_NumOfBounce <= 255) */
    int iow_lds_bvh;        /* culling BVH staged in LDS when it fits */
    int iow_leaf_batch;     /* test postponed leaves once this many lanes hold one (1..65) */
    int iow_coop_max;       /* wave-cooperative closest hits when at most this many lanes trace (0 = off) */
    int iow_chunks_lpt;     /* sequential kernel: a short first sample chunk, then longest-first */
    int rounds_seq;         /* tail-compaction rounds per pass, sequential kernels (0..14) */
    int rounds_spec;        /* ... sample-parallel passes (0..14) */
    int park_min;           /* park lanes only while at least this many units remain (-1: resident lanes / 8) */
    int spec_iters;         /* resolve + re-run passes */
    int spec_probe;         /* heavy-first: every spec_probe-th pixel probes all sample indices */
    int spec_heavy;         /* heavy-first: costliest sample indices run first (-1: (spp - 1) / 20,
                               (spp - 1) / 10 for a render of at most half the frame) */
    int spec_rounds;        /* checkpoint rounds of the speculative pass (0 = one launch) */
    int spec_tail_rounds;   /* budgeted tail rounds */
    int spec_tail_budget;   /* segments per unit and budgeted tail round */
    int spec_scan;          /* anchored scan past the frontier, samples (0 = off) */
    int spec_chain;         /* exact restarts follow their pixel's chain */
    int spec_alt;           /* alternative runs for long samples that read one stale entry */
    int spec_alt_cap;       /* alternative-run records */
    int spec_alt_seg;       /* segments that make a sample long enough for alternatives (0: 16384,
                               2048 for a render of at most half the frame) */
    int spec_alt_every;     /* also spawn alternatives after every k-th budgeted tail round (0 = once) */
    int spec_spread;        /* the last round of a pass gives long samples a wave each */
    int spec_prior_from;    /* first sample whose stale entries are guessed as the scene's RI prior */
    int spec_sort;          /* run the first re-execution list longest first */
    int spec_solo;          /* re-run pass: the longest samples take a wave each, up to this many */
    int spec_validate;      /* the sequential leftover pass reuses still-exact records */
    double spec_max_gb;     /* device memory cap of the speculation records, GB */
} rt_options;
void rt_options_default(rt_options *o);
int  rt_options_set(const rt_options *o);   /* RT_E_ARG: null, wrong size or a value out of range */
int  rt_options_get(rt_options *o);

/* ---- version / device ------------------------------------------------------------ */
int  rt_abi_version(void);
/* Returns RT_OK if a gfx950 device is visible; writes its name (<=255 chars). */
int  rt_device_info(int device, char *name_out, int name_cap, int *cu_count);

/* ---- blocking entry points (host buffers in, host buffers out) -------------------- */
int rt_render_iow01(const rt_camera *cam, const float sphere[4] /* centre xyz, radius */,
                    const rt_params *p, float *rgba /* W*H*4 */, rt_stats *st);

/* IOW-00: the base stage's default compute shader (In-One-Weekend/base.cpp:7-28, dispatched
 * W x H by 00_Image/image.cpp:46-53): rgba = (x/(W-1), y/(H-1), 0.25, 1). */
int rt_render_iow00(const rt_params *p, float *rgba /* W*H*4 */);

/* IOW-02 groups stage (02_Groups/computeShaderSrc.glsl; host groups.cpp:56-84, CopyObjBuffer
 * :250-285): records N x 18 = position, inverse rotation (glm column-major), scale, colour
 * (groups.h:11-17 GeometryBuff; the first 18 floats of an IOW-03 record), types 1 = CUBOID,
 * 2 = ELLIPSOID; u_Cull_Front / u_Cull_Back; u_NumOfBounce = p->max_bounces, u_FocusDist =
 * cam->focus_dist.  st->segments = bounce iterations (closest-hit queries). */
int rt_render_iow02(const float *types, const float *records /* N*18 */, uint32_t n, const rt_camera *cam,
                    const rt_params *p, int cull_front, int cull_back, float *rgba, rt_stats *st);

int rt_render_iow03(const float *types /* N, float(Geom_type) */,
                    const float *records /* N*24, materials.h:11-19 */, uint32_t n,
                    const rt_camera *cam, const rt_params *p, float *rgba, rt_stats *st);

int rt_render_inw(const float *geom /* N*28, layout 1 (BVH.h:12-19) or 4 (lights.h:15-21) */,
                  uint32_t n, int layout,
                  const float *nodes /* (2N-1)*8, BFS, lbvh.h:48-54 */,
                  const float *lights /* L*7: BBmin[3] BBmax[3] uint idx (bit-cast), lights.h:187-192 */,
                  uint32_t n_lights,
                  const rt_camera *cam, const rt_params *p,
                  float *rgba /* W*H*4 */, float *depth /* W*H, may be NULL */, rt_stats *st);

/* INW-01 (layout 1) with the shader's "#if MULTIFOCUS" branch compiled in
 * (01_BoundingVolumeHierarchy/computeShaderSrc.glsl:388-404, 424-428, 479-481, 505-549; the
 * reference never defines MULTIFOCUS): u_Camera.FocusDist[0..n_focus-1] = focus, 1..9 values
 * (u_NumOfFocusDist, In-Next-Week/base.h:458-473).  cam->focus_dist is not used. */
int rt_render_inw_mf(const float *geom /* N*28, layout 1 */, uint32_t n, const float *nodes, const rt_camera *cam,
                     const float *focus, int n_focus, const rt_params *p, float *rgba, float *depth, rt_stats *st);

/* ---- textures --------------------------------------------------------
 * INW-04 material textures, u_MaterialTextures[u_NumOfTexture2D]
 * (04_Lights_Camera_And_Action/computeShaderSrc.glsl:10, bound from slot 2 by
 * GeometryData_04::BindExtraData, lights.cpp:18-22).  texels: row 0 first (the GL upload
 * order; stbi flips on load, utility.cpp:217), channels 3 (GL_RGB8) or 4 (GL_RGBA8),
 * tightly packed.  An object with TextureIndex k in 1..n_tex multiplies its colour by the
 * nearest texel (GL_NEAREST, GL_REPEAT: a compute shader samples level 0 with the
 * magnification filter, utility.cpp:182-193) of its cube-projected object-space hit point
 * (04...glsl:416-464); TextureIndex > n_tex leaves the colour as is. */
typedef struct rt_texture {
    const uint8_t *texels;
    int width, height, channels;
} rt_texture;

int rt_render_inw_tex(const float *geom, uint32_t n, int layout, const float *nodes, const float *lights,
                      uint32_t n_lights, const rt_texture *tex, int n_tex, const rt_camera *cam,
                      const rt_params *p, float *rgba, float *depth, rt_stats *st);

/* Noise textures <- Helper::Noise::MakeTexture<glm::vec3>  Utilities/utility.h:69-192
 * (Snoise2 / Fbm2 / Turbulance, Utilities/utility.cpp:609-769; the stage UI calls it with
 * 600 x 100, gradient {0, 1}, lights.cpp:206).  rgb_out: width*height*3 bytes (GL_RGB8 texels,
 * row 0 first).  gradient: n_grad rgb triples (a list shorter than 2 gets black in front,
 * then white at the end, as MakeTexture does).  width must be one the reference's four
 * column batches tile exactly (600 is; others index out of bounds there): RT_E_ARG
 * otherwise, and for a constant noise field (the reference divides by zero). */
#define RT_NOISE_SIMPLEX    0
#define RT_NOISE_FBM        1
#define RT_NOISE_TURBULENCE 2
int rt_noise_texture(int width, int height, int type, const float *gradient, int n_grad, float freq, float lac,
                     float gain, int octaves, uint8_t *rgb_out, int device, double *ms);
size_t rt_noise_workspace_bytes(int width, int height);
/* Device pointers, never synchronises.  A constant noise field writes zeros and sets the
 * third uint32 of d_ws to 1. */
int rt_noise_texture_async(int width, int height, int type, const float *gradient, int n_grad, float freq,
                           float lac, float gain, int octaves, uint8_t *d_rgb_out, void *d_ws, size_t ws_bytes,
                           void *stream);

/* Re-projection <- TEXTURE_2D::LoadFromDiskToGPU(location, loadAs, mapTo)
 * Utilities/utility.cpp:266-463 (MercatorToCubic / CubicToMercator); load_as == map_to copies.
 * Where the reference is undefined: the output starts zeroed, the later loop position wins a
 * texel two positions store to, a load past the last texel reads the last texel. */
#define RT_MAP_MERCATOR 0
#define RT_MAP_CUBIC    1
int rt_texture_remap(const uint8_t *in, int width, int height, int channels, int load_as, int map_to,
                     uint8_t *out, int device, double *ms);
size_t rt_remap_workspace_bytes(int width, int height);
int rt_texture_remap_async(const uint8_t *d_in, int width, int height, int channels, int load_as, int map_to,
                           uint8_t *d_out, void *d_ws, size_t ws_bytes, void *stream);

/* LBVH builder: aabbs = N*(min xyz, max xyz) in geometry order -> (2N-1)*8 floats. */
int rt_lbvh_build(const float *aabbs, uint32_t n, float *nodes_out);

/* The same LBVH built on the GPU, node-for-node identical to rt_lbvh_build:
 * Morton keys + radix sort, the level merge as a Cartesian tree over the highest differing
 * bits, bottom-up boxes, breadth-first numbering.  Device pointers; d_ws holds
 * rt_lbvh_workspace_bytes(n) of scratch; never synchronises.  N <= 2^24 (ids are floats). */
size_t rt_lbvh_workspace_bytes(uint32_t n);
int rt_lbvh_build_async(const float *d_aabbs, uint32_t n, float *d_nodes_out, void *d_ws, size_t ws_bytes,
                        void *stream);
/* Blocking convenience wrapper (host buffers); *ms (may be NULL) receives the device time. */
int rt_lbvh_build_gpu(const float *aabbs, uint32_t n, float *nodes_out, int device, double *ms);

/* Host-side builds of a device scene's acceleration structures, without a device (what
 * rt_dev_scene_inw / rt_dev_scene_iow03 build on the host and upload):
 *   INW: the wide walk's 4-wide culling BVH over the LBVH leaf boxes, the depth-first ranks and
 *        leaf boxes, and the surrounding-RI grid; info = {wide nodes, dfs_high, wide depth,
 *        RI grid built, RI cells, RI ids, 0, 0} (all 0 when the wide walk does not apply);
 *   IOW-03: the culling BVH over the records; info = {wide nodes (0: linear loop), 0, 0, 0}.
 * info may be NULL; *ms (may be NULL) receives the host time. */
int rt_inw_host_build(const float *nodes /* (2N-1)*8 */, uint32_t n, uint32_t info[8], double *ms);
int rt_iow_host_build(const float *types, const float *records /* N*24 */, uint32_t n, uint32_t info[4], double *ms);

/* ---- asynchronous device entry points (bench / multi-GPU path) ---------------------
 * A prepared scene owns its device buffers (scene records, LBVH nodes, sample tables).
 * rt_scene_dev_* return an opaque handle; render calls enqueue on `stream`.
 * Counters are accumulated atomically into d_counters (6 x uint64, device memory). */
typedef struct rt_dev_scene rt_dev_scene;

rt_dev_scene *rt_dev_scene_iow03(const float *types, const float *records, uint32_t n,
                                 int spp, int device);
rt_dev_scene *rt_dev_scene_inw(const float *geom, uint32_t n, int layout, const float *nodes,
                               const float *lights, uint32_t n_lights, int spp, int device);
/* The same with material textures bound (see rt_texture); copied to the device. */
rt_dev_scene *rt_dev_scene_inw_tex(const float *geom, uint32_t n, int layout, const float *nodes,
                                   const float *lights, uint32_t n_lights, const rt_texture *tex, int n_tex,
                                   int spp, int device);
void rt_dev_scene_free(rt_dev_scene *s);
/* The next frame's geometry for an INW scene: RT_Base<>::OnUpdateBase's per-redraw work
 * (In-Next-Week/base.h:96-175: FillBuffer, LBVH::ConstructLBVH_Buff at :135-142, the texture
 * uploads) on the scene's existing device buffers.  geom: N*28 records of the scene's layout;
 * nodes: the caller's LBVH ((2N-1)*8), or NULL to build it on the device from aabbs (N*6, the
 * swept boxes rt_pack_inw writes) with rt_lbvh_build_async; lights: the layout-4 light SSBO.
 * The wide walk's structures and the RI grid are rebuilt on the device from a device-built LBVH
 * (rt_options.inw_device_build, the default), else on the host.  Synchronises the device first.
 * timing_ms (may be NULL) receives the host time of {records, LBVH (upload + device build, +
 * read-back for the host builders), the wide walk's structures (device or host build), their
 * upload (0 for the device build)}.  If any step fails the scene keeps its
 * previous object count but its buffers may be partly replaced: every render of it then returns
 * RT_E_ARG until a later update succeeds. */
int rt_dev_scene_inw_update(rt_dev_scene *s, const float *geom, uint32_t n, const float *nodes, const float *aabbs,
                            const float *lights, uint32_t n_lights, double timing_ms[4]);
/* Replace the scene's options (the [build] ones keep the values the scene was built with). */
int rt_dev_scene_set_options(rt_dev_scene *s, const rt_options *o);

/* The path the scene's last render took (bench line): the main kernel as
 * rocprofv3 names it and its launches per frame, the resolved fold order and which exact
 * shortcuts were on for that frame (some are decided per frame: the probe's pick, the fused
 * cull's error bound, the beam lists' memory and geometry conditions).  Synchronises when the
 * fold order was left to the device probe. */
typedef struct rt_path_info {
    char kernel[64];
    int launches;
    int order;            /* INW: 1 pixel-major, 2 sample-major, 3 per-pixel k_inw; IOW-03: 4 sample-parallel, 5 sequential */
    int order_forced;     /* 1 when rt_options.inw_order chose it, 0 when the probe did */
    int wide_walk, beams, ri_grid, fused_cull;
    int lds_nodes;        /* wide BVH nodes staged in LDS (0: none) */
    int claim_order;
    int ring_entries;     /* fold window of the kernel that ran */
    int iow_bvh;          /* IOW-03: 0 linear loop, 1 culling BVH, 2 culling BVH in LDS */
    int ring_lds;         /* 1: the fold ring was in LDS (k_inw_pm: inw_ring_pm = 0; k_inw_sm: inw_ring_sm = 0 and a BVH top of <= 5 nodes) */
    int stackless;        /* 1: the reference LBVH walks ran stackless where no push could drop */
    int lbvh_lds_nodes;   /* LBVH nodes the stackless walks read from LDS (no wide walk) */
    int qnodes;           /* 1: the wide closest-hit walks read quantised nodes (inw_qnodes) */
    int global_stack;     /* 1: the reference's 40-float stacks lived in global memory, not in LDS */
    int walk_stack;       /* entries of the wide walks' own node stack per lane (LDS) */
    uint64_t ref_walks;   /* INW: the last frame's closest-hit queries (segments + shadow rays) that the wide
                             walk or beam list handed to the reference's LBVH walks (stackless or stack) */
    int time_bins;        /* INW: time-bin culling trees the wide closest-hit walks chose from (0: the swept
                             tree; inw_time_bins, moving objects, walks that read no LDS-staged nodes) */
    int beam_bins;        /* INW: beam lists per pixel (one per time bin; 0: one list over the swept boxes) */
    int sphere_records;   /* INW: 1 when the object tests read the sphere records (inw_sphere_records) */
} rt_path_info;
int rt_debug_path(rt_dev_scene *s, rt_path_info *out);

/* Render one tile list.  tiles: device int array of n_tiles (tx, ty) pairs of tile_size^2
 * tiles; out_packed: device float array n_tiles*tile_size*tile_size*4 (tile-major, row-major
 * inside a tile; pixels outside the image are written as 0).  out_depth may be NULL. */
int rt_render_tiles_async(rt_dev_scene *s, const rt_camera *cam, const rt_params *p,
                          const int *d_tiles, int n_tiles, int tile_size,
                          float *d_out_packed, float *d_out_depth_packed,
                          uint64_t *d_counters, void *stream);

/* Render the rectangle in p->tile_* into a full W*H image resident on the device. */
int rt_render_image_async(rt_dev_scene *s, const rt_camera *cam, const rt_params *p,
                          float *d_rgba, float *d_depth, uint64_t *d_counters, void *stream);

/* ---- multi-GPU partition (BASELINE configs[3]) -----------------------------
 * One host thread drives several devices of this process: the frame's tiles are dealt
 * across the devices, each renders its share with rt_render_tiles_async on a stream of its own,
 * and one RCCL exchange over xGMI (grouped ncclSend / ncclRecv) brings the packed tiles to device
 * 0, which unpacks them into the W x H image.  This generalises the reference's per-tile
 * dispatch (In-One-Weekend/03_Shadows_and_Materials/materials.cpp:98-152) to devices, for the
 * host that replaces RT_Base<>::OnUpdateBase (In-Next-Week/base.h:148-173).
 *
 * rt_tile_deal: the frame's ceil(W/T) x ceil(H/T) tiles in deal order as (tx, ty) int pairs,
 * row-major for one device, else row-major permuted by the multiplicative hash
 * i * 2654435761 mod 2^32 (ties by i); entry k goes to device k % n_dev.  Writes up to cap pairs
 * to order_out (may be NULL) and returns the tile count. */
int rt_tile_deal(int width, int height, int tile_size, int n_dev, int *order_out, int cap);
/* A group of distinct devices with one RCCL communicator each (ncclCommInitAll) and a stream per
 * device.  NULL when a device is missing, not gfx950, repeated, or RCCL fails. */
typedef struct rt_group rt_group;
rt_group *rt_group_create(const int *devices, int n_dev);
void rt_group_free(rt_group *g);   /* synchronises the group's devices first */
/* Render the whole frame p->width x p->height (p->tile_* ignored) of scenes[r] (one device scene
 * per group device r, built from the same records and spp) in tile_size^2 tiles (a multiple of
 * 16) dealt by rt_tile_deal.  d_rgba (W*H*4 floats), d_depth (W*H, may be NULL) and d_counters
 * (6 x u64, added to; may be NULL) are device-0 pointers; stream is device 0's stream (the other
 * devices use the group's).  The first call for a frame size allocates the group's buffers. */
int rt_render_multi_async(rt_group *g, rt_dev_scene *const *scenes, const rt_camera *cam, const rt_params *p,
                          int tile_size, float *d_rgba, float *d_depth, uint64_t *d_counters, void *stream);
/* Blocking form of rt_render_inw over devices[0..n_dev): the scene replicated on every device, a
 * group, one partitioned frame, the image copied back (st->ms: device-0 time of the render). */
int rt_render_inw_multi(const float *geom, uint32_t n, int layout, const float *nodes, const float *lights,
                        uint32_t n_lights, const rt_camera *cam, const rt_params *p, const int *devices, int n_dev,
                        int tile_size, float *rgba, float *depth, rt_stats *st);

/* ---- progressive display -------------------------------------------------
 * Tile order <- Adding_Materials::OnUpdate  In-One-Weekend/03_Shadows_and_Materials/materials.cpp:84-152:
 * the drawable tiles of the centre-out square spiral over tile_w x tile_h tiles, each as
 * (tx, ty, dispatch_w, dispatch_h); the last tile index of an axis is dispatched W % tile wide
 * (materials.cpp:142-143; 0 when the tile divides W, as in the reference).  Writes up to cap
 * quadruples to out (may be NULL) and returns the number of tiles. */
int rt_tile_spiral(int width, int height, int tile_w, int tile_h, int *out, int cap);
/* One progressive update (OnUpdate with m_NumberOfTilesAtATime = count): renders tiles
 * [first, first + count) of that order into the full W*H device image (p->tile_* ignored).
 * Returns the next cursor (== rt_tile_spiral's count when the frame is complete) or an
 * error. */
int rt_render_spiral_async(rt_dev_scene *s, const rt_camera *cam, const rt_params *p, int tile_w, int tile_h,
                           int first, int count, float *d_rgba, float *d_depth, uint64_t *d_counters,
                           void *stream);
/* Display pass <- the fullscreen-quad blit into the RGBA8 framebuffer
 * (In-Next-Week/01_BoundingVolumeHierarchy/BVH.cpp:6-43; materials.cpp:154-161): the colour
 * image, or with use_depth the depth image as (d, d, d, 1), converted as GL stores unorm8
 * (clamp to [0,1], round to nearest, NaN -> 0).  d_out: W*H*4 bytes. */
int rt_display_rgba8_async(const float *d_rgba, const float *d_depth, int width, int height, int use_depth,
                           uint8_t *d_out, void *stream);

/* ---- diagnostics ---------------------------------------------------------------------
 * d_buf: device array of 16 uint64 (or NULL to disable).  While set, the IOW-03 kernel adds
 *   [0..7]  per wave iteration of each phase (outer work loop, BVH walk, postponed-leaf tests,
 *           ray segments): 1 and the number of lanes taking part (lane occupancy);
 *   [8..13] wave shader-clock cycles in: the work loop's camera-ray part, closest-hit queries,
 *           their BVH walk, leaf tests, ray segments, (unused).
 * Diagnostics cost time; never enable them for a measured run. */
int rt_debug_counters(uint64_t *d_buf);
/* d_buf: device array with one uint32 per work unit (or NULL to disable): the IOW-03 kernel
 * writes the rays each pixel cast when the pixel completes (unit = tile-major pixel index in
 * tile mode, 8x8-block-major in rect mode).  The INW fold kernels instead ADD the rays of each
 * output pixel (index = the pixel's position in the output image: y * W + x, or the packed
 * tile index), so the buffer must be zeroed before the render. */
int rt_debug_pixel_rays(uint32_t *d_buf);
/* Lanes parked by each tail-compaction round of the scene's last render (synchronises the
 * device).  Returns the number of rounds written to out (<= cap). */
int rt_debug_rounds(rt_dev_scene *s, uint32_t *out, int cap);
/* Rays per sample over the scene's last sample-parallel IOW-03 render (synchronises):
 * out[0] = max, out[1] = samples, out[2+b] = samples with 2^b <= rays < 2^(b+1),
 * out[34+b] = rays in those samples.  66 entries. */
int rt_debug_spec_hist(rt_dev_scene *s, uint64_t *out);
/* Per pixel unit of the last sample-parallel IOW-03 render, 4 x u32: sample-0 rays, the most
 * rays of one sample, that sample's index, and (column 3 of row r) the pixel at rank r of the
 * heaviest-first order.  Returns the number of units (<= cap_units) or an error. */
int rt_debug_spec_pixels(rt_dev_scene *s, uint32_t *out, uint32_t cap_units);
/* Same 66 x u64 layout as rt_debug_spec_hist, over the samples of group 0's last re-execution
 * list (their final executions). */
int rt_debug_spec_list_hist(rt_dev_scene *s, uint64_t *out);
/* With RT_DEBUG_FIRST_STALE=1 (which repurposes the stack-drop counter): out[b] / out[16+b] =
 * samples / rays of the re-execution list whose first stale stack read came in the b-th 16th
 * of their segments. */
int rt_debug_spec_list_stale(rt_dev_scene *s, uint64_t *out);
/* Rays of every (pixel unit, sample) record of the last sample-parallel IOW-03 render
 * (rays_out[s * P + pu], cap >= P * S), group 0's last re-execution list (up to list_cap
 * units) and dims = {P, S, list count, sequential-leftover count}. */
int rt_debug_spec_dump(rt_dev_scene *s, uint32_t *rays_out, size_t cap, uint32_t *list_out, uint32_t list_cap,
                       uint32_t *dims);
/* With RT_DEBUG_TIMES=1 set before the render: per (pixel unit, sample) record of the last
 * sample-parallel IOW-03 render, start_out[s * P + pu] = launch of the sample's last start
 * (bits 0-15) and its start count (bits 16-31), end_out = launch it finished in (synchronises). */
int rt_debug_spec_times(rt_dev_scene *s, uint32_t *start_out, uint32_t *end_out, size_t cap);
/* Main render kernel of the scene's last render and how many times it was launched (the
 * bench's per-launch roofline figures divide by this).  Returns the count; writes the name. */
int rt_debug_launches(rt_dev_scene *s, char *name_out, int name_cap);
/* Sample chunks of the scene's last render: the sample-parallel paths split the samples into
 * chunks whose records fit the device's free memory (INW: RT_SPEC_MAX_GB), and the per-pixel
 * paths split them by chunk_plan.  1 = one pass over all samples. */
int rt_debug_chunks(rt_dev_scene *s);
/* Kernel timing (diagnostics / bench): with rt_debug_time_kernels(1), every launch of the main
 * sample-parallel IOW-03 kernel (rt_debug_launches' name) is bracketed by HIP events on its
 * stream; rt_debug_kernel_time returns the summed durations and the launch count of the
 * scene's last render (waits for it). */
int rt_debug_time_kernels(int on);
/* Numerics self-check of the shortened correctly rounded sequences in rt_math.hpp against the
 * compiler's, for all 2^32 float bit patterns x: which 0 = rcp_sqrt_domain(sqrtf(x)) (the
 * reciprocal normalize() uses) vs 1.0f / sqrtf(x); other values are RT_E_ARG.
 * Writes the mismatch count and the lowest mismatching x (0xffffffff if none); synchronous. */
int rt_debug_check_fastmath(int which, uint64_t *mismatches, uint32_t *first_bad);
int rt_debug_kernel_time(rt_dev_scene *s, double *ms_total, int *launches);
/* The INW scene's walk structures (synchronises): info = {wide nodes, dfs_high, wide depth, RI grid
 * built, RI cells, stackless layout, objects, where the walk structures were built: 0 host, 1 device,
 * 2 host after the device build ran past its level cap}; rank_out (2n, may be NULL) receives the objects'
 * depth-first ranks (invert 0, then 1) when the wide walk is built.  Lets the tests compare the
 * device build (rt_dev_scene_inw_update) with the host build of a fresh scene. */
int rt_debug_wide_info(rt_dev_scene *s, uint32_t info[8], uint32_t *rank_out);
/* Test hook: the device build of the walk structures (rt_dev_scene_inw_update) launches at most
 * `levels` SAH / collapse levels (0 = its own cap, 256); a deeper tree is built on the host instead
 * (rt_debug_wide_info info[7] = 2), which lets a test reach that fallback with an ordinary scene. */
int rt_debug_build_level_cap(int levels);
/* Test hooks for the host build of the time-bin culling trees and the sphere records (no device;
 * DESIGN.md §5.2).  rt_debug_time_bins builds the wide walk's trees from the reference's LBVH nodes
 * and GeometryBuff records (28 floats each) with `bins` time bins and copies the 4-wide nodes (40
 * floats each, links as int bits) into wnodes_out when wnodes_cap holds them; info = {nodes of the
 * swept tree, bins built (1: none), nodes per bin tree, all nodes}.  rt_debug_bin_boxes writes the
 * culling boxes (lo xyz, hi xyz per object) of bin b of `bins`.  rt_debug_sphere_records writes the
 * 3-float4 sphere records (12 floats per object) and returns 1, or 0 when some object does not
 * qualify. */
int rt_debug_time_bins(const float *nodes, const float *geom, uint32_t n, uint32_t bins, float *wnodes_out,
                       uint32_t wnodes_cap, uint32_t info[4]);
int rt_debug_bin_boxes(const float *geom, uint32_t n, uint32_t bins, uint32_t b, float *boxes_out);
int rt_debug_sphere_records(const float *geom, uint32_t n, int layout, float *out);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
