// rt_host.hpp -- host-side C++ of the MI355X render path: the scene-description surface
// the reference stages keep on the CPU (Geometry / Transform_Data / GeometryData /
// GeometryData_04 / camera), their record packers, the LBVH builder and the sample tables.
// Everything here is product code (it is what librt_hip.so ships); the CPU oracle under
// oracle/ is an independent restatement used only by tests to check these bytes.
//
// Reference files (relative to /root/reference/Raytracing-Sandbox/Src/):
//   Utilities/utility.cpp:489-516    Helper::MATH::MakeRotation{X,Y,Z}
//   In-One-Weekend/03_Shadows_and_Materials/materials.h:43-98   IOW-03 Geometry
//   In-Next-Week/base.h:12-81        Transform_Buff / Transform_Data
//   In-Next-Week/01_BoundingVolumeHierarchy/BVH.h:6-76           GeometryBuff / GeometryData
//   In-Next-Week/04_Lights_Camera_And_Action/lights.h:6-207      GeometryBuff_04 / GeometryData_04
//   In-Next-Week/LBVH/lbvh.h:11-269  LBVH::ConstructLBVH(_Buff)
#pragma once
#include <array>
#include <cstdint>
#include <utility>
#include <vector>

#include "../../include/rt_hip.h"
#include "../../include/rt_scene.h"

namespace rtamd {

// ---- the slice of glm the reference's host code relies on (column-major mat3) ----------
struct Vec3 {
    float x = 0, y = 0, z = 0;
    Vec3() = default;
    Vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline Vec3 operator+(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec3 operator-(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec3 operator*(Vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }

struct Mat3 {
    Vec3 col[3];  // glm::mat3 m; m[c][r]
    static Mat3 identity() { Mat3 m; m.col[0] = {1, 0, 0}; m.col[1] = {0, 1, 0}; m.col[2] = {0, 0, 1}; return m; }
    // glm::mat3(x0,y0,z0, x1,y1,z1, x2,y2,z2) -- nine scalars fill the columns
    static Mat3 from_cols(float a, float b, float c, float d, float e, float f, float g, float h, float i) {
        Mat3 m; m.col[0] = {a, b, c}; m.col[1] = {d, e, f}; m.col[2] = {g, h, i}; return m;
    }
    float at(int c, int r) const { return col[c][r]; }
};
Mat3 operator*(const Mat3 &a, const Mat3 &b);  // glm mat3 product
Vec3 operator*(const Mat3 &m, Vec3 v);         // glm mat3 * vec3
Mat3 inverse(const Mat3 &m);                   // glm::inverse (adjugate form)
float radians(float deg);                      // glm::radians
Mat3 make_rotation_x(float rad);               // utility.cpp:491-498
Mat3 make_rotation_y(float rad);               // utility.cpp:500-507
Mat3 make_rotation_z(float rad);               // utility.cpp:508-515
Mat3 rotation_zxy(const Vec3 &deg);            // Rz * Rx * Ry (materials.h:80-84, base.h:26-29)

// ---- IOW-03 stage scene description (materials.h:43-98) --------------------------------
struct IowGeometry {
    int type = RT_IOW_CUBOID;                     // Typ
    Vec3 position{0, 0, 0}, rotation{0, 0, 0}, scale{1, 1, 1};
    Vec3 color{1, 0, 0};
    Vec3 material{0.2f, 0.3f, 1.5f};              // refractivity, reflectivity, refractive index
    Vec3 scatteritivity{0, 0, 0};                 // (refract, reflect)
    Mat3 inv_rotation = Mat3::identity();         // _inv_rotation_matrix
    void reset_inv_rotation();                    // ResetInvRotationMatrix
    void fill_buffer(float rec[24]) const;        // FillBuffer
};

// ---- INW scene description (base.h:19-81, BVH.h:26-76, lights.h:28-207) -----------------
struct TransformData {
    Vec3 position{3, 3, 3}, last_position{0, 0, 0}, rotation{0, 0, 0}, scale{1, 1, 1};
    std::pair<Vec3, Vec3> bb_min_max() const;     // CalculateBBMinMax (base version)
    void fill_transform(float buf[18]) const;     // FillTransformBuff
};
struct GeometryData : TransformData {               // layout 1
    int type = RT_INW_ELLIPSOID;
    Vec3 color{0, 0, 0};
    float refractive_index = 1.5f, refractivity = 0.65f, reflectivity = 0.15f;
    float scat[2] = {0, 0};
    void fill_buffer(float buf[28]) const;
};
struct GeometryData04 : TransformData {             // layout 4
    int type = RT_INW_ELLIPSOID;
    bool emissive = false;
    Vec3 color{0, 0, 0};
    int texture_index = 0;
    float refractive_index = 1.5f, refractivity = 0.65f, reflectivity = 0.15f;
    float scat[2] = {0, 0};
    std::pair<Vec3, Vec3> bb_min_max() const;     // override: corner-exact cuboid
    void fill_buffer(float buf[28]) const;
};

IowGeometry to_iow(const rt_geom_desc &d);
GeometryData to_inw01(const rt_geom_desc &d);
GeometryData04 to_inw04(const rt_geom_desc &d);

// ---- LBVH (lbvh.h) --------------------------------------------------------------------
// aabbs: N x (min xyz, max xyz).  Returns (2N-1) x 8 floats in the reference's BFS layout.
std::vector<float> lbvh_build(const float *aabbs, uint32_t n);

// Full-sweep SAH BVH over boxes (acceleration structure for IOW-03's closest-hit search; the
// reference has none there).  Same node layout as the LBVH (children contiguous, leftData
// = first child or -objectID, rightData = parent).  *depth receives the tree depth.
std::vector<float> sah_build(const float *aabbs, uint32_t n, int *depth);

// 4-wide BVH from a binary one (sah_build / lbvh layout, n >= 2).  Node = 32 floats, SoA over
// the 4 children: lo_x[4] lo_y[4] lo_z[4] hi_x[4] hi_y[4] hi_z[4] link[4] pad[4]; link > 0 is
// (wide node index + 1), link <= 0 is -objectID, empty slots hold a far-away box and link 1e9.
// *depth receives the number of wide levels.
std::vector<float> bvh4_collapse(const std::vector<float> &bin, int *depth);

// ---- device-scene structures built on the host -------------------------
// IOW-03 culling BVH (the reference loops linearly over the objects, 03...glsl:196-256): a SAH
// tree over conservative world boxes of the records, collapsed to 4-wide nodes whose child
// links are int bits (float 24..27 of a node), and the leaves' boxes as n float4 (lo.xyz, hi.x)
// followed by n float2 (hi.yz).  Returns false (linear loop) for fewer than 2 or 16384+ objects.
struct IowCull {
    std::vector<float> wide, obox;
    uint32_t n_wide = 0;
};
bool iow_cull_build(const float *types, const float *rec, uint32_t n, IowCull &out);

// INW wide walk: from the reference's LBVH nodes ((2n-1) x 8), each object's
// leaf box, its rank in the LBVH's depth-first order for both child orders, the walk's stack
// high-water mark dfs_high, and a 4-wide culling BVH over the leaf boxes (inflated), 40 floats
// per node (lx ly lz hx hy hz lx ly lz links).  Returns false (reference walk only) for fewer
// than 2 objects or an LBVH that is not well formed.
struct InwWide {
    uint32_t dfs_high = 0;
    int depth = 0;
    float wbound = 0.0f;           // largest |coordinate| of the culling boxes
    std::vector<float> wnodes;     // 40 floats per node
    std::vector<uint32_t> rank;    // 2n: rank[inv * n + g]
    std::vector<float> leafbox;    // 8n: object g's LBVH leaf node
    // Shutter-time bins (DESIGN.md §5.2 "Time-binned culling trees"): after the tree over the swept
    // boxes (n_tree0 nodes) come `bins` trees of bin_stride nodes each (padded), tree b over the
    // boxes the objects sweep while the ray time ratio lies in [b / bins, (b + 1) / bins]; their
    // links are rebased to the concatenated array.  bins = 1: the swept tree only.
    uint32_t n_tree0 = 0, bins = 1, bin_stride = 0;
};
bool inw_wide_build(const float *nodes, uint32_t n, InwWide &out);
// Append the time-bin trees to a built InwWide from the reference's GeometryBuff records (28
// floats: position, rotation, scale, position - last_position at 15..17).  false (nothing
// appended): bins < 2, no object moves, or the records are malformed.
bool inw_wide_add_bins(const float *geom, uint32_t n, uint32_t bins, InwWide &w);
// The culling boxes of bin b of `bins` (6 floats per object: lo xyz, hi xyz), rounded outward; the
// largest |coordinate| goes into wbound (max).  false: a record's extent is not finite.
bool inw_bin_boxes(const float *geom, uint32_t n, uint32_t bins, uint32_t b, std::vector<float> &boxes, float &wbound);
// The reference walk's stack high-water mark over both child orders (high; its pushes can only
// drop while size + high > 40) and whether the node buffer has the layout the stackless LBVH walks
// rely on (stackless: every internal node's children at L (odd), L + 1 with rightData = the node,
// leaf ids < n; lbvh.h:236-269 writes it so).  false: not a walkable LBVH (no shortcut applies).
bool lbvh_walk_info(const float *nodes, uint32_t n, uint32_t &high, bool &stackless);

// The surrounding-RI grid (DESIGN.md §5 "RI grid") over the leaf boxes: about two cells per
// object, every object entered in each cell its leaf box overlaps once widened by a thousandth of
// a cell.  ok = false when some cell would list more than 64 objects (the walk answers instead).
struct RiGrid {
    bool ok = false;
    float lo[3] = {}, hi[3] = {}, inv[3] = {};
    int dim[3] = {};
    std::vector<uint32_t> cells, ids;  // cell offsets (cells + 1), object ids
};
RiGrid ri_grid_build(const float *leafbox, uint32_t n);
// its cell counts per axis over the leaf boxes' bounds [lo, hi] (false: not finite), shared with
// the device build (rt_build.hip)
bool ri_grid_dims(const double lo[3], const double hi[3], uint32_t n, int dim[3], double inv[3]);

// ---- camera (materials.cpp:321-328, base.h:274-281) ------------------------------------
Vec3 front_from_pitch_yaw(float pitch_deg, float yaw_deg, bool normalize);

// ---- sample tables ----------------------------------------------------------------------
void sample_tables(int spp, float *sunflower, float *fib, int *ring);

// Progressive tile order of Adding_Materials::OnUpdate (materials.cpp:84-152): the drawable
// tiles of the centre-out square spiral, each (tx, ty, dispatch_w, dispatch_h)
struct SpiralTile { int tx, ty, w, h; };
std::vector<SpiralTile> tile_spiral(int W, int H, int tw, int th);

// ---- presets ----------------------------------------------------------------------------
int scene_preset(int preset, uint32_t seed, int n_hint, std::vector<rt_geom_desc> &out,
                 rt_cam_desc &cam, rt_params &params);

// The tile deal of the multi-GPU partition: the frame's ceil(W/T) x ceil(H/T) tiles
// in row-major order, permuted for n_dev > 1 by a multiplicative hash of their index (a plain
// round robin over rows hands a rank whole tile columns when the row length is a multiple of
// n_dev, and a glass sphere's columns to a few ranks); entry k goes to device k % n_dev.
// bench.py deal_order is the same function.
std::vector<std::pair<int, int>> tile_deal(int W, int H, int T, int n_dev);

// the device a device scene was built on (rt_capi.hip; the multi-GPU group checks its scene list)
int scene_device(const struct rt_dev_scene *s);

}  // namespace rtamd
