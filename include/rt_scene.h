/*
 * rt_scene.h -- host-side scene description surface of librt_hip.so.
 *
 * Mirrors the reference's scene classes so a caller keeps the same vocabulary:
 *   rt_geom_desc  <- In_One_Weekend::Adding_Materials::Geometry   (03_Shadows_and_Materials/materials.h:43-98)
 *                    In_Next_Week::Transform_Data + GeometryData  (In-Next-Week/base.h:19-81, 01_BoundingVolumeHierarchy/BVH.h:26-76)
 *                    In_Next_Week::GeometryData_04                (04_Lights_Camera_And_Action/lights.h:28-207)
 *   rt_cam_desc   <- RT_Base::m_Camera / pitch-yaw camera members (In-Next-Week/base.h:256-282, materials.h:140-145)
 *   rt_pack_*     <- Geometry::FillBuffer / GeometryData::FillBuffer / GeometryData_04::FillBuffer,
 *                    Transform_Data::CalculateBBMinMax, Lights::FillBuffer light SSBO (lights.cpp:255-271)
 *   rt_scene_preset <- the scenes the reference stages build in OnAttach / "Set Configration" /
 *                    'R' key, plus the seeded synthetic scenes of SURVEY.md 8d.
 * Paths relative to /root/reference/Raytracing-Sandbox/Src/.
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <stdint.h>
#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Stage (which shader / record layout a description is packed for). */
#define RT_STAGE_IOW01 1
#define RT_STAGE_IOW02 2
#define RT_STAGE_IOW03 3
#define RT_STAGE_INW01 11
#define RT_STAGE_INW04 14

/* Geometry type codes as the reference stores them (note the two enums differ):
 * IOW-03: CUBOID = 1, ELLIPSOID = 2 (materials.h:37-42); INW: Ellipsoid = 1, Cuboid = 2 (BVH.h:20-25). */
#define RT_IOW_CUBOID    1
#define RT_IOW_ELLIPSOID 2
#define RT_INW_ELLIPSOID 1
#define RT_INW_CUBOID    2

typedef struct rt_geom_desc {
    int   type;               /* stage-specific code above                                  */
    float position[3];
    float last_position[3];   /* INW motion: DeltaPosition = position - last_position       */
    float rotation_deg[3];    /* (x = pitch, y = yaw, z = roll), degrees, Rz*Rx*Ry          */
    float scale[3];
    float color[3];
    float refractivity, reflectivity, refractive_index;
    float scat_refract, scat_reflect;
    int   emissive;           /* INW-04 isEmissive                                          */
    int   texture_index;      /* INW-04 TextureIndex (0 = none)                             */
} rt_geom_desc;

typedef struct rt_cam_desc {
    float position[3];
    float pitch_deg, yaw_deg;
    float fov_y_deg;
    float aperture;
    float focus_dist;
} rt_cam_desc;

/* Presets */
#define RT_PRESET_IOW03_REF3     1   /* materials.cpp:46-65 + materials.h:136-150 defaults          */
#define RT_PRESET_IOW03_FINAL    2   /* config C2: ~500 spheres "final scene", SURVEY 8d, seed       */
#define RT_PRESET_INW01_GRID     3   /* BVH stage, 'R' key grid layout (BVH.cpp:83-112), n objects  */
#define RT_PRESET_INW01_RANDOM   4   /* config C3: n random moving ellipsoids, SURVEY 8d, seed       */
#define RT_PRESET_INW04_REFSET   5   /* Lights stage "Set Configration" (lights.cpp:116-146)         */
#define RT_PRESET_INW04_CORNELL  6   /* config C5: Cornell-style emissive box, SURVEY 8d, seed       */

/* Fill up to `cap` descriptions; returns the object count (or <0 on error).  cam / params
 * receive the preset's default camera and render parameters (either may be NULL).
 * n_hint: object count for presets that take one (GRID, RANDOM); ignored otherwise. */
int rt_scene_preset(int preset, uint32_t seed, int n_hint, rt_geom_desc *out, int cap,
                    rt_cam_desc *cam, rt_params *params);

/* Camera uniforms exactly as the stage's host computes them. */
int rt_camera_from_desc(const rt_cam_desc *d, int stage, rt_camera *out);

/* IOW-03: types[N] (float type code), records[N*24] (Geometry::FillBuffer). */
int rt_pack_iow03(const rt_geom_desc *g, uint32_t n, float *types, float *records);
/* IOW-02: types[N], records[N*18] (Groups::Geometry::FillBuffer, groups.h:45-64). */
int rt_pack_iow02(const rt_geom_desc *g, uint32_t n, float *types, float *records);

/* INW: geom[N*28] in layout 1 or 4, aabbs[N*6] (CalculateBBMinMax of that layout),
 * lights[N*7] (only the first *n_lights used; LightClass with idx bit-cast) may be NULL. */
int rt_pack_inw(const rt_geom_desc *g, uint32_t n, int layout, float *geom, float *aabbs,
                float *lights, uint32_t *n_lights);

/* Host-built sample tables (transcendentals evaluated once in double, rounded to float).
 * sunflower: spp*2 floats, unit-aperture golden-angle disk (03...glsl:153-163, 01_BVH...glsl:15-27)
 * fib:       spp*3 floats, unit Fibonacci sphere (03...glsl:164-184) before scatter scaling
 * ring:      spp*2 ints, IOW-03 ring-ordered stratified sub-pixel indices (03...glsl:383-397) */
int rt_sample_tables(int spp, float *sunflower, float *fib, int *ring);

#ifdef __cplusplus
}
#endif
#endif /* RT_SCENE_H */
