// rt_host.cpp -- scene description, packers, LBVH builder, sample tables, presets.
// See rt_host.hpp for the reference map.  Compiled with -ffp-contract=off: every float
// expression here must round exactly as the reference's host code (glm) does.
#include "rt_host.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <random>

namespace rtamd {

// ----------------------------------------------------------------------------- glm slice
Mat3 operator*(const Mat3 &a, const Mat3 &b) {
    Mat3 r;
    for (int j = 0; j < 3; j++)  // glm: Result[j] = A[0]*B[j][0] + A[1]*B[j][1] + A[2]*B[j][2]
        r.col[j] = a.col[0] * b.col[j].x + a.col[1] * b.col[j].y + a.col[2] * b.col[j].z;
    return r;
}
Vec3 operator*(const Mat3 &m, Vec3 v) {
    return {m.col[0].x * v.x + m.col[1].x * v.y + m.col[2].x * v.z,
            m.col[0].y * v.x + m.col[1].y * v.y + m.col[2].y * v.z,
            m.col[0].z * v.x + m.col[1].z * v.y + m.col[2].z * v.z};
}
Mat3 inverse(const Mat3 &m) {
    auto M = [&](int c, int r) { return m.at(c, r); };
    float det = +M(0, 0) * (M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) -
                M(1, 0) * (M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) +
                M(2, 0) * (M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2));
    float o = 1.0f / det;
    Mat3 r;
    r.col[0].x = +(M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * o;
    r.col[1].x = -(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * o;
    r.col[2].x = +(M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * o;
    r.col[0].y = -(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * o;
    r.col[1].y = +(M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * o;
    r.col[2].y = -(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * o;
    r.col[0].z = +(M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * o;
    r.col[1].z = -(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * o;
    r.col[2].z = +(M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * o;
    return r;
}
float radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }
Mat3 make_rotation_x(float rad) {
    float c = std::cos(rad), s = std::sin(rad);
    return Mat3::from_cols(1.0f, 0.0f, 0.0f, 0.0f, c, -s, 0.0f, s, c);
}
Mat3 make_rotation_y(float rad) {
    float c = std::cos(rad), s = std::sin(rad);
    return Mat3::from_cols(c, 0.0f, s, 0.0f, 1.0f, 0.0f, -s, 0.0f, c);
}
Mat3 make_rotation_z(float rad) {
    float c = std::cos(rad), s = std::sin(rad);
    return Mat3::from_cols(c, -s, 0.0f, s, c, 0.0f, 0.0f, 0.0f, 1.0f);
}
Mat3 rotation_zxy(const Vec3 &deg) {
    return make_rotation_z(radians(deg.z)) * make_rotation_x(radians(deg.x)) * make_rotation_y(radians(deg.y));
}

static inline float rmin(float x, float y) { return x > y ? y : x; }  // MIN, utility.h:10
static inline float rmax(float x, float y) { return x > y ? x : y; }  // MAX, utility.h:11

// ------------------------------------------------------------------------------- IOW-03
void IowGeometry::reset_inv_rotation() { inv_rotation = inverse(rotation_zxy(rotation)); }
void IowGeometry::fill_buffer(float r[24]) const {
    for (int i = 0; i < 3; i++) r[i] = position[i];
    for (int i = 0; i < 9; i++) r[3 + i] = inv_rotation.at(i / 3, i % 3);
    for (int i = 0; i < 3; i++) r[12 + i] = scale[i];
    for (int i = 0; i < 3; i++) r[15 + i] = color[i];
    for (int i = 0; i < 3; i++) r[18 + i] = material[i];
    r[21] = scatteritivity[0];
    r[22] = scatteritivity[1];
    r[23] = 0.0f;
}

// ---------------------------------------------------------------------------------- INW
std::pair<Vec3, Vec3> TransformData::bb_min_max() const {
    Mat3 m = rotation_zxy(rotation) * Mat3::from_cols(scale.x, 0, 0, 0, scale.y, 0, 0, 0, scale.z);
    float x = std::sqrt(m.at(0, 0) * m.at(0, 0) + m.at(1, 0) * m.at(1, 0) + m.at(2, 0) * m.at(2, 0));
    float y = std::sqrt(m.at(0, 1) * m.at(0, 1) + m.at(1, 1) * m.at(1, 1) + m.at(2, 1) * m.at(2, 1));
    float z = std::sqrt(m.at(0, 2) * m.at(0, 2) + m.at(1, 2) * m.at(1, 2) + m.at(2, 2) * m.at(2, 2));
    Vec3 mn(rmin(position.x, last_position.x), rmin(position.y, last_position.y), rmin(position.z, last_position.z));
    Vec3 mx(rmax(position.x, last_position.x), rmax(position.y, last_position.y), rmax(position.z, last_position.z));
    return {Vec3(-x, -y, -z) + mn, Vec3(x, y, z) + mx};
}
void TransformData::fill_transform(float b[18]) const {
    for (int i = 0; i < 3; i++) { b[i] = position[i]; b[15 + i] = position[i] - last_position[i]; }
    Mat3 m = rotation_zxy(rotation);
    for (int i = 0; i < 9; i++) b[3 + i] = m.at(i / 3, i % 3);
    for (int i = 0; i < 3; i++) b[12 + i] = scale[i];
}
void GeometryData::fill_buffer(float b[28]) const {
    fill_transform(b);
    b[18] = float(type);
    b[19] = 0.0f;  // _padding
    b[20] = refractive_index; b[21] = refractivity; b[22] = reflectivity;
    b[23] = scat[0]; b[24] = scat[1];
    b[25] = color.x; b[26] = color.y; b[27] = color.z;
}
std::pair<Vec3, Vec3> GeometryData04::bb_min_max() const {
    if (type == RT_INW_ELLIPSOID) return TransformData::bb_min_max();
    if (type == RT_INW_CUBOID) {
        Mat3 m = rotation_zxy(rotation);
        Vec3 bmin(0, 0, 0), bmax(0, 0, 0);
        for (int i = 0; i < 8; i++) {
            Vec3 co;
            int bit = 1;
            for (int a = 0; a < 3; a++) { co[a] = (i & bit) ? 0.5f * scale[a] : -0.5f * scale[a]; bit <<= 1; }
            co = m * co;
            for (int a = 0; a < 3; a++) { bmin[a] = rmin(co[a], bmin[a]); bmax[a] = rmax(co[a], bmax[a]); }
        }
        Vec3 mn(rmin(position.x, last_position.x), rmin(position.y, last_position.y), rmin(position.z, last_position.z));
        Vec3 mx(rmax(position.x, last_position.x), rmax(position.y, last_position.y), rmax(position.z, last_position.z));
        return {bmin + mn, bmax + mx};
    }
    return {Vec3(0, 0, 0), Vec3(0, 0, 0)};
}
void GeometryData04::fill_buffer(float b[28]) const {
    fill_transform(b);
    b[18] = float(type);
    b[27] = float(texture_index);
    if (!emissive) {
        b[24] = color.x; b[25] = color.y; b[26] = color.z;
        b[19] = refractive_index; b[21] = reflectivity; b[20] = refractivity;
    } else {  // lights.h:134-139: emissive objects are white, RI 1, no reflect/refract
        b[24] = 1.0f; b[25] = 1.0f; b[26] = 1.0f;
        b[19] = 1.0f; b[21] = 0.0f; b[20] = 0.0f;
    }
    b[22] = scat[0]; b[23] = scat[1];
}

static Vec3 v3(const float *f) { return Vec3(f[0], f[1], f[2]); }
IowGeometry to_iow(const rt_geom_desc &d) {
    IowGeometry g;
    g.type = d.type;
    g.position = v3(d.position); g.rotation = v3(d.rotation_deg); g.scale = v3(d.scale);
    g.color = v3(d.color);
    g.material = Vec3(d.refractivity, d.reflectivity, d.refractive_index);
    g.scatteritivity = Vec3(d.scat_refract, d.scat_reflect, 0.0f);
    // the default inverse is glm::mat3(1); ImGui edits call ResetInvRotationMatrix
    if (d.rotation_deg[0] != 0 || d.rotation_deg[1] != 0 || d.rotation_deg[2] != 0) g.reset_inv_rotation();
    return g;
}
template <class G> static void fill_common(G &g, const rt_geom_desc &d) {
    g.type = d.type;
    g.position = v3(d.position); g.last_position = v3(d.last_position);
    g.rotation = v3(d.rotation_deg); g.scale = v3(d.scale); g.color = v3(d.color);
    g.refractive_index = d.refractive_index; g.refractivity = d.refractivity; g.reflectivity = d.reflectivity;
    g.scat[0] = d.scat_refract; g.scat[1] = d.scat_reflect;
}
GeometryData to_inw01(const rt_geom_desc &d) { GeometryData g; fill_common(g, d); return g; }
GeometryData04 to_inw04(const rt_geom_desc &d) {
    GeometryData04 g;
    fill_common(g, d);
    g.emissive = d.emissive != 0;
    g.texture_index = d.texture_index;
    return g;
}

// --------------------------------------------------------------------------------- LBVH
// The reference merges adjacent leaf clusters level by level: every internal node i sits
// between sorted leaves i and i+1 and is solved in the pass whose level reaches its
// "highest differing bit" (lbvh.h:162-210); within a pass the FIFO keeps index order and
// a solved node adopts the current top-most ancestors of leaves i and i+1.  That is the
// same as merging nodes in (bit, index) order while tracking each contiguous leaf
// cluster's root, which this does with a disjoint-set in O(N log N).
static inline uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
static inline uint32_t morton30(Vec3 p) {
    const float res = 1024.0f;
    auto q = [&](float f) { return static_cast<uint32_t>(std::fmin(std::fmax(f * res, 0.0f), res - 1.0f)); };
    return expand_bits(q(p.x)) * 4 + expand_bits(q(p.y)) * 2 + expand_bits(q(p.z));
}

std::vector<float> lbvh_build(const float *aabbs, uint32_t n) {
    std::vector<float> out(size_t(2 * n - 1) * 8, 0.0f);
    if (n == 1) {
        std::memcpy(out.data(), aabbs, 6 * sizeof(float));
        out[6] = -float(0u);
        out[7] = 0.0f;
        return out;
    }
    Vec3 smin = v3(aabbs), smax = v3(aabbs + 3);
    for (uint32_t i = 1; i < n; i++)
        for (int a = 0; a < 3; a++) {
            smin[a] = rmin(smin[a], aabbs[size_t(i) * 6 + a]);
            smax[a] = rmax(smax[a], aabbs[size_t(i) * 6 + 3 + a]);
        }
    struct Key { uint32_t code, id; float diag2; };
    std::vector<Key> keys(n);
    for (uint32_t i = 0; i < n; i++) {
        const float *b = aabbs + size_t(i) * 6;
        Vec3 p((b[0] + b[3]) * 0.5f, (b[1] + b[4]) * 0.5f, (b[2] + b[5]) * 0.5f);
        p = p - smin;
        p.x /= (smax.x - smin.x);
        p.y /= (smax.y - smin.y);
        p.z /= (smax.z - smin.z);
        Vec3 d(b[3] - b[0], b[4] - b[1], b[5] - b[2]);
        keys[i] = {morton30(p), i, d.x * d.x + d.y * d.y + d.z * d.z};
    }
    std::sort(keys.begin(), keys.end(), [](const Key &a, const Key &b) {
        if (a.code != b.code) return a.code < b.code;
        if (a.diag2 < b.diag2) return true;
        if (b.diag2 < a.diag2) return false;
        return a.id < b.id;  // contract tie-break (std::sort order of equal keys is unspecified)
    });
    std::vector<uint8_t> bit(n - 1);
    for (uint32_t i = 1; i < n; i++) {
        uint32_t x = keys[i - 1].code ^ keys[i].code;
        uint8_t h = 0;
        while (x) { x >>= 1; h++; }
        bit[i - 1] = h;
    }
    const uint32_t total = 2 * n - 1;
    struct Node { int32_t left = -1, right = -1; uint32_t obj = 0; Vec3 mn, mx; };
    std::vector<Node> nd(total);
    for (uint32_t i = 0; i < n; i++) {
        nd[i].obj = keys[i].id;
        nd[i].mn = v3(aabbs + size_t(keys[i].id) * 6);
        nd[i].mx = v3(aabbs + size_t(keys[i].id) * 6 + 3);
    }
    // disjoint set over leaves; croot[rep] = tree node at the top of that cluster
    std::vector<uint32_t> dsu(n), croot(n);
    std::iota(dsu.begin(), dsu.end(), 0u);
    std::iota(croot.begin(), croot.end(), 0u);
    auto find = [&](uint32_t x) {
        while (dsu[x] != x) { dsu[x] = dsu[dsu[x]]; x = dsu[x]; }
        return x;
    };
    std::vector<uint32_t> order(n - 1);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return bit[a] < bit[b]; });
    uint32_t last = 0;
    for (uint32_t i : order) {
        uint32_t ra = find(i), rb = find(i + 1);
        uint32_t L = croot[ra], R = croot[rb], me = n + i;
        nd[me].left = int32_t(L);
        nd[me].right = int32_t(R);
        for (int a = 0; a < 3; a++) {
            nd[me].mn[a] = rmin(nd[L].mn[a], nd[R].mn[a]);
            nd[me].mx[a] = rmax(nd[L].mx[a], nd[R].mx[a]);
        }
        dsu[rb] = ra;
        croot[ra] = me;
        last = me;
    }
    // ConstructLBVH_Buff: breadth-first write, children contiguous, rightData = parent
    std::vector<std::pair<uint32_t, uint32_t>> q;
    q.reserve(total);
    q.push_back({last, 0u});
    for (size_t head = 0, index = 0; head < q.size(); head++, index++) {
        auto [cn, parent] = q[head];
        uint32_t L = 0;
        if (nd[cn].left >= 0) {
            q.push_back({uint32_t(nd[cn].left), uint32_t(index)});
            L = uint32_t(index + (q.size() - head - 1));
            q.push_back({uint32_t(nd[cn].right), uint32_t(index)});
        }
        float *o = out.data() + index * 8;
        o[0] = nd[cn].mn.x; o[1] = nd[cn].mn.y; o[2] = nd[cn].mn.z;
        o[3] = nd[cn].mx.x; o[4] = nd[cn].mx.y; o[5] = nd[cn].mx.z;
        o[6] = (L == 0) ? -float(nd[cn].obj) : float(L);
        o[7] = float(parent);
    }
    return out;
}

// ----------------------------------------------------------------------------- SAH BVH
namespace {
struct Box {
    float mn[3] = {1e30f, 1e30f, 1e30f}, mx[3] = {-1e30f, -1e30f, -1e30f};
    void grow(const Box &b) { for (int a = 0; a < 3; a++) { mn[a] = std::fmin(mn[a], b.mn[a]); mx[a] = std::fmax(mx[a], b.mx[a]); } }
    float area() const {
        float d[3];
        for (int a = 0; a < 3; a++) d[a] = std::fmax(mx[a] - mn[a], 0.0f);
        return d[0] * d[1] + d[1] * d[2] + d[2] * d[0];
    }
};
struct SahBuilder {
    std::vector<Box> prim;
    std::vector<float> cen;  // 3 per prim
    std::vector<uint32_t> ids;
    std::vector<float> out;  // 8 floats per node
    uint32_t next = 1;
    int depth = 0;
    void node(uint32_t at, uint32_t parent, uint32_t lo, uint32_t hi, int d) {
        depth = std::max(depth, d);
        Box b;
        for (uint32_t i = lo; i < hi; i++) b.grow(prim[ids[i]]);
        float *o = out.data() + size_t(at) * 8;
        for (int a = 0; a < 3; a++) { o[a] = b.mn[a]; o[3 + a] = b.mx[a]; }
        o[7] = float(parent);
        const uint32_t cnt = hi - lo;
        if (cnt == 1) { o[6] = -float(ids[lo]); return; }
        // full sweep SAH over the three axes (N is small: hundreds to thousands)
        float best = 1e38f;
        int best_axis = 0;
        uint32_t best_split = lo + cnt / 2;
        std::vector<float> right_area(cnt);
        for (int a = 0; a < 3; a++) {
            std::sort(ids.begin() + lo, ids.begin() + hi, [&](uint32_t x, uint32_t y) {
                return cen[3 * x + a] < cen[3 * y + a] || (cen[3 * x + a] == cen[3 * y + a] && x < y);
            });
            Box r;
            for (uint32_t i = hi; i-- > lo + 1;) { r.grow(prim[ids[i]]); right_area[i - lo] = r.area(); }
            Box l;
            for (uint32_t i = lo; i + 1 < hi; i++) {
                l.grow(prim[ids[i]]);
                const uint32_t nl = i + 1 - lo, nr = hi - i - 1;
                const float c = l.area() * float(nl) + right_area[i + 1 - lo] * float(nr);
                if (c < best) { best = c; best_axis = a; best_split = i + 1; }
            }
        }
        std::sort(ids.begin() + lo, ids.begin() + hi, [&](uint32_t x, uint32_t y) {
            return cen[3 * x + best_axis] < cen[3 * y + best_axis] ||
                   (cen[3 * x + best_axis] == cen[3 * y + best_axis] && x < y);
        });
        const uint32_t c0 = next;
        next += 2;
        o[6] = float(c0);
        node(c0, at, lo, best_split, d + 1);
        node(c0 + 1, at, best_split, hi, d + 1);
    }
};
}  // namespace

std::vector<float> sah_build(const float *aabbs, uint32_t n, int *depth) {
    SahBuilder b;
    b.prim.resize(n);
    b.cen.resize(size_t(n) * 3);
    b.ids.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        for (int a = 0; a < 3; a++) {
            b.prim[i].mn[a] = aabbs[size_t(i) * 6 + a];
            b.prim[i].mx[a] = aabbs[size_t(i) * 6 + 3 + a];
            b.cen[3 * i + a] = 0.5f * (b.prim[i].mn[a] + b.prim[i].mx[a]);
        }
        b.ids[i] = i;
    }
    b.out.assign(size_t(2 * n - 1) * 8, 0.0f);
    b.node(0, 0, 0, n, 0);
    if (depth) *depth = b.depth;
    return b.out;
}

// Collapse the binary tree into 4-wide nodes: a node's children are gathered by repeatedly
// opening the largest-area internal child until there are four (or only leaves remain).
std::vector<float> bvh4_collapse(const std::vector<float> &bin, int *depth) {
    auto is_leaf = [&](int i) { return !(bin[size_t(i) * 8 + 6] > 0.1f); };
    auto first = [&](int i) { return int(bin[size_t(i) * 8 + 6]); };
    auto area = [&](int i) {
        const float *b = &bin[size_t(i) * 8];
        const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
        return dx * dy + dy * dz + dz * dx;
    };
    std::vector<std::array<int, 4>> kids;  // binary node ids per wide node (-1 = empty)
    std::vector<int> lvl;
    std::vector<float> out;
    struct Item { int bin, wide, level; };
    std::vector<Item> work{{0, 0, 1}};
    kids.push_back({-1, -1, -1, -1});
    lvl.push_back(1);
    int maxd = 1;
    for (size_t w = 0; w < work.size(); w++) {
        const Item it = work[w];
        std::vector<int> ch{first(it.bin), first(it.bin) + 1};
        for (;;) {
            if (ch.size() >= 4) break;
            int pick = -1;
            for (size_t k = 0; k < ch.size(); k++)
                if (!is_leaf(ch[k]) && (pick < 0 || area(ch[k]) > area(ch[size_t(pick)]))) pick = int(k);
            if (pick < 0) break;
            const int b = ch[size_t(pick)];
            ch.erase(ch.begin() + pick);
            ch.push_back(first(b));
            ch.push_back(first(b) + 1);
        }
        for (size_t k = 0; k < ch.size(); k++) kids[size_t(it.wide)][k] = ch[k];
        for (int b : ch)
            if (!is_leaf(b)) {
                const int id = int(kids.size());
                kids.push_back({-1, -1, -1, -1});
                work.push_back({b, id, it.level + 1});
                maxd = std::max(maxd, it.level + 1);
            }
    }
    // children that are internal binary nodes map to wide ids in `work` order
    std::vector<int> wide_of(bin.size() / 8, -1);
    for (const Item &it : work) wide_of[size_t(it.bin)] = it.wide;
    out.assign(kids.size() * 32, 0.0f);
    for (size_t w = 0; w < kids.size(); w++) {
        float *o = &out[w * 32];
        for (int k = 0; k < 4; k++) {
            const int b = kids[w][size_t(k)];
            if (b < 0) {  // empty slot: a far-away point box, culled by every ray
                for (int a = 0; a < 6; a++) o[a * 4 + k] = 1e30f;
                o[24 + k] = 1e9f;
                continue;
            }
            const float *bb = &bin[size_t(b) * 8];
            o[0 * 4 + k] = bb[0]; o[1 * 4 + k] = bb[1]; o[2 * 4 + k] = bb[2];
            o[3 * 4 + k] = bb[3]; o[4 * 4 + k] = bb[4]; o[5 * 4 + k] = bb[5];
            // link: wide node index + 1 (> 0) or -objectID (<= 0)
            o[24 + k] = is_leaf(b) ? bb[6] : float(wide_of[size_t(b)] + 1);
        }
    }
    if (depth) *depth = maxd;
    return out;
}

// ------------------------------------------------------------------------------- camera
Vec3 front_from_pitch_yaw(float pitch, float yaw, bool normalize) {
    Vec3 f;
    f.x = std::cos(radians(yaw)) * std::cos(radians(pitch));
    f.y = std::sin(radians(pitch));
    f.z = std::sin(radians(yaw)) * std::cos(radians(pitch));
    if (!normalize) return f;  // RT_Base::m_Camera.Front(), base.h:274-281
    float k = 1.0f / std::sqrt(f.x * f.x + f.y * f.y + f.z * f.z);  // glm::normalize
    return f * k;
}

// ------------------------------------------------------------------------ sample tables
void sample_tables(int spp, float *sunflower, float *fib, int *ring) {
    const double kPI = 3.1415926538;              // the shaders' #define PI
    const double kPHI = kPI * (3.0 - std::sqrt(5.0));
    const double b = std::floor(2.0 * std::sqrt(double(spp)) + 0.5);
    for (int i = 0; i < spp; i++) {
        const double th = kPHI * double(i);
        if (sunflower) {
            if (i == 0) { sunflower[0] = 0.0f; sunflower[1] = 0.0f; }
            else {
                double rho = (double(i) > double(spp) - b) ? 1.0
                             : std::sqrt((double(i) - 0.5) / (double(spp) - (b + 1.0) / 2.0));
                sunflower[2 * i] = float(rho * std::cos(th));
                sunflower[2 * i + 1] = float(rho * std::sin(th));
            }
        }
        if (fib) {
            double y = 1.0 - (double(i) / double(spp - 1));
            double radius = std::sqrt(1.0 - y * y);
            fib[3 * i] = float(std::cos(th) * radius);
            fib[3 * i + 1] = float(y);
            fib[3 * i + 2] = float(std::sin(th) * radius);
        }
    }
    if (ring) {  // closed-form walk of the ring schedule (03...glsl:383-397)
        int grid = 1;
        while (grid * grid < spp) grid++;
        int focus = 0, x = 0, y = 0;
        for (int s = 0; s < spp; s++) {
            int *o = ring + 2 * s;
            if (focus >= grid) { o[0] = o[1] = -1; continue; }
            if (x == 0 && y == 0) { ++focus; x = y = focus; o[0] = o[1] = focus; }
            else if (x < y) { --y; o[0] = focus; o[1] = y; }
            else { --x; o[0] = x; o[1] = focus; }
        }
    }
}

// ------------------------------------------------------------------------------ presets
namespace {
struct Rng {  // mt19937 raw words -> 24-bit uniform floats (portable, no std::distribution)
    std::mt19937 g;
    explicit Rng(uint32_t s) : g(s) {}
    float u() { return float(g() >> 8) * (1.0f / 16777216.0f); }
    float u(float a, float b) { return a + (b - a) * u(); }
};
rt_geom_desc blank() {
    rt_geom_desc d;
    std::memset(&d, 0, sizeof(d));
    d.scale[0] = d.scale[1] = d.scale[2] = 1.0f;
    d.refractive_index = 1.5f;
    return d;
}
void set3(float *f, float a, float b, float c) { f[0] = a; f[1] = b; f[2] = c; }
rt_cam_desc cam_at(float px, float py, float pz, float pitch, float yaw, float fov, float ap, float focus) {
    rt_cam_desc c;
    set3(c.position, px, py, pz);
    c.pitch_deg = pitch; c.yaw_deg = yaw; c.fov_y_deg = fov; c.aperture = ap; c.focus_dist = focus;
    return c;
}
rt_params params_of(int w, int h, int spp, int bounces) {
    rt_params p;
    std::memset(&p, 0, sizeof(p));
    p.width = w; p.height = h; p.spp = spp; p.max_bounces = bounces; p.device = -1;
    return p;
}
// pitch/yaw (degrees) of the direction from `from` to `to`, inverse of FrontFromPitchYaw
void look(const float from[3], const float to[3], float &pitch, float &yaw) {
    double dx = to[0] - from[0], dy = to[1] - from[1], dz = to[2] - from[2];
    double l = std::sqrt(dx * dx + dy * dy + dz * dz);
    pitch = float(std::asin(dy / l) * 180.0 / 3.14159265358979323846);
    yaw = float(std::atan2(dz, dx) * 180.0 / 3.14159265358979323846);
}
}  // namespace

int scene_preset(int preset, uint32_t seed, int n_hint, std::vector<rt_geom_desc> &out,
                 rt_cam_desc &cam, rt_params &params) {
    out.clear();
    switch (preset) {
    case RT_PRESET_IOW03_REF3: {  // materials.cpp:46-65 on top of Geometry defaults (materials.h:89-95)
        for (int i = 0; i < 3; i++) {
            rt_geom_desc d = blank();
            d.type = RT_IOW_CUBOID;
            set3(d.color, 1, 0, 0);
            d.refractivity = 0.2f; d.reflectivity = 0.3f; d.refractive_index = 1.5f;
            out.push_back(d);
        }
        out[0].type = RT_IOW_ELLIPSOID; set3(out[0].color, 0, 0, 0); set3(out[0].scale, 2, 2, 2);
        out[0].position[1] = 1; out[0].refractivity = 1; out[0].reflectivity = 0; out[0].refractive_index = 1.5f;
        out[1].type = RT_IOW_CUBOID; out[1].position[1] = -1.5f; out[1].scale[0] = 12; out[1].scale[2] = 11;
        set3(out[1].color, 0.02f, 0.0125f, 0.08f);
        out[2].type = RT_IOW_ELLIPSOID; set3(out[2].position, -1, -.5f, 1.75f); set3(out[2].scale, .5f, .5f, .5f);
        out[2].reflectivity = 0.8f; out[2].scat_reflect = 0.8f; set3(out[2].color, 0, 0, 0);
        cam = cam_at(3, 2, 10, -13, -120, 90.0f, 2.0f, 10.0f);  // materials.h:140-145
        params = params_of(300, 300, 36, 5);                    // materials.h:137-149
        return int(out.size());
    }
    case RT_PRESET_IOW03_FINAL: {  // config C2: the "final scene" as IOW records
        Rng r(seed);
        rt_geom_desc g = blank();
        g.type = RT_IOW_CUBOID;
        set3(g.position, 0, -0.5f, 0); set3(g.scale, 100, 1, 100); set3(g.color, 0.1f, 0.1f, 0.1f);
        g.reflectivity = 0.5f; g.scat_reflect = 1.0f;
        out.push_back(g);
        for (int a = -11; a < 11; a++)
            for (int b = -11; b < 11; b++) {
                float choose = r.u();
                float cx = float(a) + 0.9f * r.u(), cz = float(b) + 0.9f * r.u();
                float dx = cx - 4.0f, dz = cz;
                if (std::sqrt(dx * dx + dz * dz) <= 0.9f) continue;
                rt_geom_desc d = blank();
                d.type = RT_IOW_ELLIPSOID;
                set3(d.position, cx, 0.2f, cz); set3(d.scale, 0.2f, 0.2f, 0.2f);
                if (choose < 0.8f) {  // "diffuse": broad-cone reflector
                    float c0 = r.u() * r.u(), c1 = r.u() * r.u(), c2 = r.u() * r.u();
                    set3(d.color, c0, c1, c2);
                    d.reflectivity = 0.5f; d.scat_reflect = 1.0f;
                } else if (choose < 0.95f) {  // "metal": fuzzed mirror
                    float c0 = r.u(0.25f, 0.5f), c1 = r.u(0.25f, 0.5f), c2 = r.u(0.25f, 0.5f);
                    set3(d.color, c0, c1, c2);
                    d.reflectivity = 0.8f; d.scat_reflect = r.u(0.0f, 0.5f);
                } else {  // "dielectric"
                    d.refractivity = 1.0f; d.refractive_index = 1.5f;
                }
                out.push_back(d);
            }
        rt_geom_desc s1 = blank(); s1.type = RT_IOW_ELLIPSOID; set3(s1.position, 0, 1, 0);
        s1.refractivity = 1.0f; s1.refractive_index = 1.5f; out.push_back(s1);
        rt_geom_desc s2 = blank(); s2.type = RT_IOW_ELLIPSOID; set3(s2.position, -4, 1, 0);
        set3(s2.color, 0.4f, 0.2f, 0.1f); s2.reflectivity = 0.5f; s2.scat_reflect = 1.0f; out.push_back(s2);
        rt_geom_desc s3 = blank(); s3.type = RT_IOW_ELLIPSOID; set3(s3.position, 4, 1, 0);
        set3(s3.color, 0.35f, 0.3f, 0.25f); s3.reflectivity = 0.8f; out.push_back(s3);
        float from[3] = {13, 2, 3}, to[3] = {0, 0, 0}, pitch, yaw;
        look(from, to, pitch, yaw);
        cam = cam_at(13, 2, 3, pitch, yaw, 20.0f, 0.1f, 10.0f);
        params = params_of(1200, 800, 100, 50);
        return int(out.size());
    }
    case RT_PRESET_INW01_GRID: {  // BVH.cpp:83-112 ('R' key) over GeometryData defaults
        int n = n_hint > 0 ? n_hint : 4;
        uint32_t grid = 1;
        while (grid * grid < uint32_t(n)) grid++;
        grid /= 2;
        int x = -int(grid), y = -int(grid);
        for (int i = 0; i < n; i++) {
            rt_geom_desc d = blank();
            d.type = RT_INW_ELLIPSOID;
            d.refractivity = 0.65f; d.reflectivity = 0.15f; d.refractive_index = 1.5f;
            d.position[0] = float(x) * 1.0f; d.position[1] = float(y) * 1.0f; d.position[2] = 0.0f;
            d.scale[0] = 1.0f + 0.2f * float(x) * (1.0f / float(grid));
            d.scale[1] = 1.0f + 0.2f * float(y) * (1.0f / float(grid));
            d.scale[2] = 1.0f;
            std::memcpy(d.last_position, d.position, sizeof(d.position));
            out.push_back(d);
            if (++x > int(grid)) { x = -int(grid); y++; }
        }
        cam = cam_at(-3, 6.5f, -3, -30, 45, 60.0f, 1.0f, 10.0f);  // BVH.cpp:50-52, base.h:268-272, :590
        params = params_of(100, 100, 1, 5);                       // base.h:249-255
        return int(out.size());
    }
    case RT_PRESET_INW01_RANDOM: {  // config C3
        int n = n_hint > 0 ? n_hint : 10000;
        Rng r(seed);
        for (int i = 0; i < n; i++) {
            rt_geom_desc d = blank();
            d.type = RT_INW_ELLIPSOID;
            float px = r.u(-50, 50), py = r.u(-5, 5), pz = r.u(-50, 50);
            float rad = r.u(0.1f, 0.4f);
            float mx = r.u(-0.2f, 0.2f), my = r.u(-0.2f, 0.2f), mz = r.u(-0.2f, 0.2f);
            set3(d.position, px, py, pz);
            set3(d.last_position, px - mx, py - my, pz - mz);
            set3(d.scale, rad, rad, rad);
            if (r.u() < 0.7f) {
                d.refractivity = 0.0f; d.reflectivity = r.u(0.5f, 0.9f); d.scat_reflect = r.u(0.0f, 0.3f);
                float c0 = r.u(0, 0.6f), c1 = r.u(0, 0.6f), c2 = r.u(0, 0.6f);
                set3(d.color, c0, c1, c2);
            } else {
                d.refractivity = 0.65f; d.reflectivity = 0.15f; d.refractive_index = r.u(1.3f, 1.7f);
                d.scat_refract = r.u(0.0f, 0.3f);
                float c0 = r.u(0, 0.2f), c1 = r.u(0, 0.2f), c2 = r.u(0, 0.2f);
                set3(d.color, c0, c1, c2);
            }
            out.push_back(d);
        }
        cam = cam_at(-60, 15, -60, -12, 45, 60.0f, 0.1f, 40.0f);
        params = params_of(1920, 1080, 500, 50);
        return int(out.size());
    }
    case RT_PRESET_INW04_REFSET: {  // lights.cpp:116-146 over GeometryData_04 defaults (lights.h:194-201)
        for (int i = 0; i < 5; i++) {
            rt_geom_desc d = blank();
            d.type = RT_INW_ELLIPSOID;
            d.refractivity = 0.65f; d.reflectivity = 0.15f; d.refractive_index = 1.5f;
            set3(d.position, 3, 3, 3);
            out.push_back(d);
        }
        out[0].emissive = 1;
        set3(out[1].position, -1.52f, 3.0f, 1.4f); out[1].emissive = 1;
        set3(out[2].position, 9, 0, 9); set3(out[2].color, 0.3f, 0.4f, 1.0f);
        set3(out[3].position, 7, 0, 8); set3(out[3].color, 0.3f, 0.4f, 1.0f);
        set3(out[4].position, 0, -2, 0); set3(out[4].scale, 100, 1, 100); set3(out[4].color, 0.3f, 0.4f, 1.0f);
        out[4].refractivity = 0.1f; out[4].reflectivity = 0.6f; out[4].type = RT_INW_CUBOID;
        for (auto &d : out) std::memcpy(d.last_position, d.position, sizeof(d.position));
        cam = cam_at(-6.1f, 6.2f, -0.2f, -30, 45, 60.0f, 1.0f, 10.0f);
        params = params_of(100, 100, 1, 5);
        return int(out.size());
    }
    case RT_PRESET_INW04_CORNELL: {  // config C5; deterministic, seed unused
        (void)seed;
        auto wall = [&](float px, float py, float pz, float sx, float sy, float sz, float r, float g, float b) {
            rt_geom_desc d = blank();
            d.type = RT_INW_CUBOID;
            set3(d.position, px, py, pz); set3(d.scale, sx, sy, sz); set3(d.color, r, g, b);
            d.refractivity = 0.0f; d.reflectivity = 0.5f; d.scat_reflect = 1.0f;
            out.push_back(d);
            return out.size() - 1;
        };
        const float S = 5.55f, h = S * 0.5f;
        wall(h, -0.05f, h, S, 0.1f, S, .73f, .73f, .73f);          // floor
        wall(h, S + 0.05f, h, S, 0.1f, S, .73f, .73f, .73f);       // ceiling
        wall(h, h, S + 0.05f, S, S, 0.1f, .73f, .73f, .73f);       // back
        wall(-0.05f, h, h, 0.1f, S, S, .65f, .05f, .05f);          // left (red)
        wall(S + 0.05f, h, h, 0.1f, S, S, .12f, .45f, .15f);       // right (green)
        size_t li = wall(2.78f, S - 0.01f, 2.795f, 1.3f, 0.02f, 1.05f, 1, 1, 1);
        out[li].emissive = 1;                                       // ceiling light
        size_t tb = wall(3.68f, 1.65f, 3.51f, 1.65f, 3.30f, 1.65f, .73f, .73f, .73f);
        out[tb].rotation_deg[1] = 15.0f;                           // tall block
        size_t sb = wall(1.85f, 0.825f, 1.69f, 1.65f, 1.65f, 1.65f, .73f, .73f, .73f);
        out[sb].rotation_deg[1] = -18.0f;                          // short block
        rt_geom_desc gl = blank();
        gl.type = RT_INW_ELLIPSOID;
        set3(gl.position, 1.85f, 2.25f, 1.69f); set3(gl.scale, 0.6f, 0.6f, 0.6f);
        gl.refractivity = 0.9f; gl.reflectivity = 0.1f; gl.refractive_index = 1.5f;
        out.push_back(gl);
        for (auto &d : out) std::memcpy(d.last_position, d.position, sizeof(d.position));
        cam = cam_at(2.78f, 2.78f, -8.0f, 0, 90, 40.0f, 0.05f, 10.0f);
        params = params_of(4096, 4096, 2000, 50);
        return int(out.size());
    }
    default:
        return RT_E_ARG;
    }
}

// materials.cpp:84-152.  The state has the reference's widths (materials.h:110-116: int16
// indices and ring corners, uint16 maxima, int8 steps); every OnUpdate draws
// m_NumberOfTilesAtATime drawable tiles, skipping undrawable spiral positions (the goto), so
// the sequence of drawable tiles is the whole schedule.  The last index of an axis is the
// partial tile, dispatched W % tile wide (0 when the tile divides W; kept).
std::vector<SpiralTile> tile_spiral(int W, int H, int tw, int th) {
    std::vector<SpiralTile> out;
    const uint16_t mx0 = uint16_t(W / tw), mx1 = uint16_t(H / th);
    int16_t i0 = int16_t((mx0 - 0.1f) / 2), i1 = int16_t((mx1 - 0.1f) / 2);
    int16_t r00[2] = {i0, i1}, r01[2] = {i0, int16_t(i1 + 1)};
    int16_t r10[2] = {int16_t(i0 + 1), int16_t(i1 - 1)}, r11[2] = {int16_t(i0 + 1), int16_t(i1 + 1)};
    int8_t st[2] = {0, 0};
    const int lim = (mx0 > mx1 ? mx0 : mx1) + 1;
    while ((i0 < i1 ? i0 : i1) < lim) {
        if (i1 == r00[1] && i0 == r00[0]) { r00[0]--; r00[1]--; st[0] = 0; st[1] = 1; }
        if (i1 == r01[1] && i0 == r01[0]) { r01[0]--; r01[1]++; st[0] = 1; st[1] = 0; }
        if (i1 == r11[1] && i0 == r11[0]) { r11[0]++; r11[1]++; st[0] = 0; st[1] = -1; }
        if (i1 == r10[1] && i0 == r10[0]) { r10[0]++; r10[1]--; st[0] = -1; st[1] = 0; }
        if (i1 > -1 && i1 < mx1 + 1 && i0 > -1 && i0 < mx0 + 1)
            out.push_back({i0, i1, i0 >= mx0 ? W % tw : tw, i1 >= mx1 ? H % th : th});
        i0 = int16_t(i0 + st[0]);
        i1 = int16_t(i1 + st[1]);
    }
    return out;
}

// ---------------------------------------------------------------- device-scene structures
bool iow_cull_build(const float *types, const float *rec, uint32_t n, IowCull &out) {
    // links travel as int16 on the IOW traversal stack: wide node ids < n, object ids < n
    if (n < 2 || n >= 16384) return false;
    // world box of each record = |M^T| * local half extents, inflated so it is conservative
    std::vector<float> boxes(size_t(n) * 6);
    for (uint32_t j = 0; j < n; j++) {
        const float *r = rec + size_t(j) * 24;
        const bool ell = int(types[j]) == RT_IOW_ELLIPSOID;
        float h[3];
        for (int k = 0; k < 3; k++) h[k] = std::fabs(r[12 + k]) * (ell ? 1.0f : 0.5f);
        const float big = std::fmax(std::fabs(r[0]), std::fmax(std::fabs(r[1]), std::fabs(r[2])));
        for (int k = 0; k < 3; k++) {
            const float *col = r + 3 + 3 * k;  // column k of M: M_{row j, col k} = col[j]
            float e = std::fabs(col[0]) * h[0] + std::fabs(col[1]) * h[1] + std::fabs(col[2]) * h[2];
            e = e * 1.001f + 1e-3f + big * 1e-5f;
            boxes[size_t(j) * 6 + k] = r[k] - e;
            boxes[size_t(j) * 6 + 3 + k] = r[k] + e;
        }
    }
    int depth = 0, depth4 = 0;
    out.wide = bvh4_collapse(sah_build(boxes.data(), n, &depth), &depth4);
    for (size_t w = 0; w < out.wide.size() / 32; w++)  // the kernels read the links as int bits
        for (int k = 0; k < 4; k++) {
            const int link = int(out.wide[w * 32 + 24 + size_t(k)]);
            std::memcpy(&out.wide[w * 32 + 24 + size_t(k)], &link, sizeof(link));
        }
    out.n_wide = uint32_t(out.wide.size() / 32);
    out.obox.assign(size_t(n) * 6, 0.0f);
    for (uint32_t j = 0; j < n; j++) {
        const float *b = boxes.data() + size_t(j) * 6;
        for (int k = 0; k < 4; k++) out.obox[size_t(j) * 4 + k] = b[k];
        out.obox[size_t(n) * 4 + size_t(j) * 2] = b[4];
        out.obox[size_t(n) * 4 + size_t(j) * 2 + 1] = b[5];
    }
    return true;
}

// A 4-wide culling tree over `boxes` (6 floats each) appended to `out` as 10 float4 per node: lx ly
// lz hx hy hz lx ly lz, child links as int bits; node links are rebased by `base` (the index of
// the tree's first node in the whole array), empty slots keep their far-away link.  Returns nodes.
static size_t wide_tree(const float *boxes, uint32_t n, size_t base, std::vector<float> &out, int *depth4) {
    int depth = 0;
    const std::vector<float> wide = bvh4_collapse(sah_build(boxes, n, &depth), depth4);
    const size_t nw = wide.size() / 32, o0 = out.size();
    out.resize(o0 + nw * 40, 0.0f);
    for (size_t w = 0; w < nw; w++) {
        float *o = &out[o0 + w * 40];
        std::memcpy(o, &wide[w * 32], 24 * sizeof(float));
        std::memcpy(o + 24, &wide[w * 32], 12 * sizeof(float));
        for (int k = 0; k < 4; k++) {
            int link = int(wide[w * 32 + 24 + size_t(k)]);
            if (link > 0 && size_t(link) <= nw) link += int(base);
            std::memcpy(o + 36 + k, &link, sizeof(link));
        }
    }
    return nw;
}

bool inw_wide_build(const float *nodes, uint32_t n, InwWide &out) {
    if (n < 2) return false;
    const uint32_t nn = 2 * n - 1;
    std::vector<uint32_t> leaf(n, 0xffffffffu);
    out.rank.assign(size_t(2) * n, 0);
    for (uint32_t i = 0; i < nn; i++) {
        const float left = nodes[size_t(i) * 8 + 6];
        if (!(left > 0.1f)) {
            const float g = -left;
            if (!(g >= 0.0f) || g >= float(n)) return false;  // not a well-formed LBVH: exact walk only
            leaf[uint32_t(g)] = i;
        }
    }
    for (uint32_t g = 0; g < n; g++)
        if (leaf[g] == 0xffffffffu) return false;
    // depth-first order of the leaves and the stack high-water mark, both child orders
    // (01_BVH...glsl:456-460: push(invert ? right : left), push(invert ? left : right))
    uint32_t high = 0;
    for (int inv = 0; inv < 2; inv++) {
        std::vector<uint32_t> st{0};
        uint32_t r = 0;
        high = std::max<uint32_t>(high, 1);
        while (!st.empty()) {
            const uint32_t i = st.back();
            st.pop_back();
            const float left = nodes[size_t(i) * 8 + 6];
            if (left > 0.1f) {
                const uint32_t l = uint32_t(left), rr = l + 1;
                if (rr >= nn || st.size() + 2 > size_t(nn)) return false;
                st.push_back(inv ? rr : l);
                st.push_back(inv ? l : rr);
                high = std::max<uint32_t>(high, uint32_t(st.size()));
            } else {
                if (r == n) return false;
                out.rank[size_t(inv) * n + uint32_t(-left)] = r++;
            }
        }
        if (r != n) return false;
    }
    // culling boxes: the leaf boxes, inflated as the IOW culling BVH's
    std::vector<float> boxes(size_t(n) * 6);
    float wbound = 0.0f;
    for (uint32_t g = 0; g < n; g++) {
        const float *b = nodes + size_t(leaf[g]) * 8;  // bbmin xyz, bbmax xyz
        float big = 0.0f;
        for (int k = 0; k < 6; k++) big = std::fmax(big, std::fabs(b[k]));
        for (int k = 0; k < 3; k++) {
            const float e = (b[3 + k] - b[k]) * 1e-3f + 1e-3f + big * 1e-5f;
            boxes[size_t(g) * 6 + k] = b[k] - e;
            boxes[size_t(g) * 6 + 3 + k] = b[3 + k] + e;
            wbound = std::fmax(wbound, std::fmax(std::fabs(b[k] - e), std::fabs(b[3 + k] + e)));
        }
    }
    int depth4 = 0;
    out.wnodes.clear();
    wide_tree(boxes.data(), n, 0, out.wnodes, &depth4);
    out.n_tree0 = uint32_t(out.wnodes.size() / 40);
    out.bins = 1;
    out.bin_stride = 0;
    out.leafbox.assign(size_t(n) * 8, 0.0f);
    for (uint32_t g = 0; g < n; g++) std::memcpy(&out.leafbox[size_t(g) * 8], nodes + size_t(leaf[g]) * 8, 8 * sizeof(float));
    out.dfs_high = high;
    out.depth = depth4;
    out.wbound = wbound;
    return true;
}

// Time-bin trees.  Object g's centre at time ratio r is p - delta (1 - r) (the kernels' object
// offset (o - p) + delta (1 - r), 01_BVH...glsl), so over [r0, r1] it sweeps the segment between
// its centres at r0 and r1; its box there is that segment's box widened by the object's own half
// extent, sqrt(sum_c (M_ic s_c)^2) under either orientation convention of the rotation M (the
// ellipsoid's exact extent, and above a cuboid's), inflated as the swept culling boxes are.  A ray
// that hits the object at a time in the bin hits it inside that box, so culling with it is as
// conservative as with the swept box (the tree only decides which leaves get the
// exact test).
bool inw_bin_boxes(const float *geom, uint32_t n, uint32_t bins, uint32_t b, std::vector<float> &boxes, float &wbound) {
    boxes.assign(size_t(n) * 6, 0.0f);
    const double r0 = double(b) / bins, r1 = double(b + 1) / bins;
    for (uint32_t g = 0; g < n; g++) {
        const float *f = geom + size_t(g) * 28;
        double lo[3], hi[3];
        float big = 0.0f;
        for (int a = 0; a < 3; a++) {
            double row = 0.0, col = 0.0;  // the half extent along axis a under either orientation of M
            for (int c = 0; c < 3; c++) {
                const double x = double(f[3 + 3 * a + c]) * f[12 + c], y = double(f[3 + 3 * c + a]) * f[12 + c];
                row += x * x;
                col += y * y;
            }
            const double e = std::sqrt(std::fmax(row, col));
            if (!std::isfinite(e)) return false;
            const double c0 = double(f[a]) - double(f[15 + a]) * (1.0 - r0);
            const double c1 = double(f[a]) - double(f[15 + a]) * (1.0 - r1);
            lo[a] = std::fmin(c0, c1) - e;
            hi[a] = std::fmax(c0, c1) + e;
            big = std::fmax(big, float(std::fmax(std::fabs(lo[a]), std::fabs(hi[a]))));
        }
        for (int a = 0; a < 3; a++) {
            const double e = (hi[a] - lo[a]) * 1e-3 + 1e-3 + double(big) * 1e-5;  // as the swept boxes
            float l = float(lo[a] - e), h = float(hi[a] + e);  // rounded outward to float
            if (double(l) > lo[a] - e) l = std::nextafter(l, -INFINITY);
            if (double(h) < hi[a] + e) h = std::nextafter(h, INFINITY);
            boxes[size_t(g) * 6 + a] = l;
            boxes[size_t(g) * 6 + 3 + a] = h;
            wbound = std::fmax(wbound, std::fmax(std::fabs(l), std::fabs(h)));
        }
    }
    return true;
}

// Time-bin trees (see inw_bin_boxes for the boxes).  Object g's centre at time ratio r is
// p - delta (1 - r) (the kernels' object offset (o - p) + delta (1 - r), 01_BVH...glsl), so over
// [r0, r1] it sweeps the segment between its centres at r0 and r1; its box there is that segment's
// box widened by the object's own half extent, sqrt(sum_c (M_ic s_c)^2) under either orientation
// convention of the rotation M (the ellipsoid's exact extent, and above a cuboid's), inflated as
// the swept culling boxes are.  A ray that hits the object at a time in the bin hits it inside that
// box, so culling with it is as conservative as with the swept box (the tree only
// decides which leaves get the exact test).
bool inw_wide_add_bins(const float *geom, uint32_t n, uint32_t bins, InwWide &w) {
    if (bins < 2 || bins > 16 || n < 2 || w.wnodes.empty() || w.bins != 1) return false;
    bool moving = false;
    for (uint32_t g = 0; g < n && !moving; g++)
        for (int a = 0; a < 3; a++) moving = moving || geom[size_t(g) * 28 + 15 + a] != 0.0f;
    if (!moving) return false;
    std::vector<std::vector<float>> trees(bins);
    size_t stride = 0;
    std::vector<float> boxes;
    float wbound = w.wbound;
    for (uint32_t b = 0; b < bins; b++) {
        if (!inw_bin_boxes(geom, n, bins, b, boxes, wbound)) return false;
        int d4 = 0;
        stride = std::max(stride, wide_tree(boxes.data(), n, 0, trees[b], &d4));
    }
    // concatenate: tree b's first node at n_tree0 + b * stride (links rebased), padding nodes empty
    const size_t n0 = w.wnodes.size() / 40;
    w.wnodes.resize((n0 + bins * stride) * 40, 0.0f);
    for (uint32_t b = 0; b < bins; b++) {
        const size_t base = n0 + b * stride, nw = trees[b].size() / 40;
        float *o = &w.wnodes[base * 40];
        std::memcpy(o, trees[b].data(), trees[b].size() * sizeof(float));
        for (size_t k = 0; k < nw; k++)
            for (int j = 0; j < 4; j++) {
                int link;
                std::memcpy(&link, o + k * 40 + 36 + j, sizeof(link));
                if (link > 0 && size_t(link) <= nw) link += int(base);
                std::memcpy(o + k * 40 + 36 + j, &link, sizeof(link));
            }
        for (size_t k = nw; k < stride; k++) {  // padding: empty slots only
            float *p = o + k * 40;
            for (int j = 0; j < 36; j++) p[j] = 1e30f;
            const int link = 1000000000;
            for (int j = 0; j < 4; j++) std::memcpy(p + 36 + j, &link, sizeof(link));
        }
    }
    w.bins = bins;
    w.bin_stride = uint32_t(stride);
    w.wbound = wbound;
    return true;
}

bool lbvh_walk_info(const float *nodes, uint32_t n, uint32_t &high, bool &stackless) {
    high = 0;
    stackless = false;
    if (n == 0 || n > (1u << 24)) return false;
    const uint32_t nn = 2 * n - 1;
    bool lay = true;
    for (uint32_t i = 0; i < nn && lay; i++) {
        const float left = nodes[size_t(i) * 8 + 6];
        if (left > 0.1f) {
            const uint32_t L = uint32_t(left);
            lay = float(L) == left && (L & 1u) && L + 1 < nn && nodes[size_t(L) * 8 + 7] == float(i) &&
                  nodes[size_t(L + 1) * 8 + 7] == float(i);
        } else {
            lay = -left >= 0.0f && -left < float(n) && float(uint32_t(-left)) == -left;
        }
    }
    for (int inv = 0; inv < 2; inv++) {  // 01_BVH...glsl:456-460 push order
        std::vector<uint32_t> st{0};
        uint32_t pops = 0;
        high = std::max<uint32_t>(high, 1);
        while (!st.empty()) {
            const uint32_t i = st.back();
            st.pop_back();
            if (++pops > nn) return false;  // a cycle: not a tree
            const float left = nodes[size_t(i) * 8 + 6];
            if (left > 0.1f) {
                const uint32_t l = uint32_t(left), r = l + 1;
                if (r >= nn) return false;
                st.push_back(inv ? r : l);
                st.push_back(inv ? l : r);
                high = std::max<uint32_t>(high, uint32_t(st.size()));
            }
        }
    }
    stackless = lay;
    return true;
}

bool ri_grid_dims(const double lo[3], const double hi[3], uint32_t n, int dim[3], double inv[3]) {
    double ext[3], vol = 1.0;
    for (int a = 0; a < 3; a++) {
        if (!(hi[a] >= lo[a]) || !std::isfinite(lo[a]) || !std::isfinite(hi[a])) return false;
        ext[a] = std::fmax(hi[a] - lo[a], 1e-6 * (1.0 + std::fabs(lo[a])));
        vol *= ext[a];
    }
    const double cell = std::cbrt(vol / (2.0 * n));
    for (int a = 0; a < 3; a++) {
        dim[a] = int(std::fmin(512.0, std::fmax(1.0, std::ceil(ext[a] / cell))));
        inv[a] = double(dim[a]) / ext[a];
    }
    return true;
}

RiGrid ri_grid_build(const float *lbox, uint32_t n) {
    RiGrid G;
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (uint32_t g = 0; g < n; g++)
        for (int a = 0; a < 3; a++) {
            lo[a] = std::fmin(lo[a], double(lbox[size_t(g) * 8 + a]));
            hi[a] = std::fmax(hi[a], double(lbox[size_t(g) * 8 + 3 + a]));
        }
    int dim[3];
    double inv[3];
    if (!ri_grid_dims(lo, hi, n, dim, inv)) return G;
    const size_t nc = size_t(dim[0]) * dim[1] * dim[2];
    std::vector<uint32_t> cnt(nc + 1, 0);
    auto range = [&](uint32_t g, int a, int &c0, int &c1) {
        const double m = 1e-3 / inv[a];
        c0 = std::max(0, std::min(dim[a] - 1, int(std::floor((double(lbox[size_t(g) * 8 + a]) - m - lo[a]) * inv[a]))));
        c1 = std::max(0, std::min(dim[a] - 1, int(std::floor((double(lbox[size_t(g) * 8 + 3 + a]) + m - lo[a]) * inv[a]))));
    };
    std::vector<uint32_t> fill, ids;
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
            for (size_t c = 0; c < nc; c++) cnt[c + 1] += cnt[c];
            fill.assign(cnt.begin(), cnt.end() - 1);
            ids.resize(cnt[nc]);
        }
        for (uint32_t g = 0; g < n; g++) {
            int r0[3], r1[3];
            for (int a = 0; a < 3; a++) range(g, a, r0[a], r1[a]);
            for (int z = r0[2]; z <= r1[2]; z++)
                for (int y = r0[1]; y <= r1[1]; y++)
                    for (int x = r0[0]; x <= r1[0]; x++) {
                        const size_t c = (size_t(z) * dim[1] + y) * dim[0] + x;
                        if (pass == 0) {
                            if (++cnt[c + 1] > 64) return G;
                        } else ids[fill[c]++] = g;
                    }
        }
    }
    for (int a = 0; a < 3; a++) {
        // float bounds: a point outside them is outside every leaf box
        G.lo[a] = float(lo[a]);
        G.hi[a] = float(hi[a]);
        G.inv[a] = float(inv[a]);
        G.dim[a] = dim[a];
    }
    G.cells = std::move(cnt);
    G.ids = std::move(ids);
    G.ok = true;
    return G;
}

std::vector<std::pair<int, int>> tile_deal(int W, int H, int T, int n_dev) {
    const int nx = (W + T - 1) / T, ny = (H + T - 1) / T;
    std::vector<uint32_t> idx(size_t(nx) * size_t(ny));
    for (size_t i = 0; i < idx.size(); i++) idx[i] = uint32_t(i);
    if (n_dev > 1)  // key (i * 2654435761 mod 2^32, i): Knuth's multiplicative hash, ties by index
        std::sort(idx.begin(), idx.end(), [](uint32_t a, uint32_t b) {
            const uint32_t ha = a * 2654435761u, hb = b * 2654435761u;
            return ha < hb || (ha == hb && a < b);
        });
    std::vector<std::pair<int, int>> out;
    out.reserve(idx.size());
    for (uint32_t i : idx) out.push_back({int(i % uint32_t(nx)), int(i / uint32_t(nx))});
    return out;
}

}  // namespace rtamd
