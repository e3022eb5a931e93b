// pfref: LaserMappingClass, the global map of src/laserMappingNode.cpp.
// TEST INFRASTRUCTURE (oracle) — see pfref.h header.
//
// Restates src/laserMappingClass.cpp (init :7-33, checkPoints :105-147, updateCurrentPointsToMap
// :151-189, getMap :194-206; include/laserMappingClass.h:13-20) with the map held as a dictionary of
// 50 m cubes keyed by their global cube coordinates (the reference's growing 3-D vector of cubes
// indexes the same cubes through origin_in_map_*; getMap walks them in the same x, y, z order, and
// cubes that were never allocated or are empty contribute nothing either way).
//
// Third-party arithmetic (parity unpinned):
//   pcl::transformPointCloud<PointXYZI>(..., Affine3f): PCL 1.10's SSE Transformer<float>::se3,
//     out = x c0 + (y c1 + (z c2 + c3)) in f32, c = columns of pose.cast<float>().matrix()
//   pcl::VoxelGrid<PointXYZI> (downsample_all_data): as pfref_odom.cpp's voxel_grid, with the
//     intensity averaged like x, y, z; ties in the (idx, point) sort kept in input order (the
//     reference's std::sort is unstable: VG_STABLE).
#include "pfref_internal.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <map>
#include <set>
#include <tuple>

namespace pfref {
namespace {

constexpr double kCell = 50.0;    // LASER_CELL_WIDTH / HEIGHT / DEPTH
constexpr int kRangeH = 2;        // LASER_CELL_RANGE_HORIZONTAL
constexpr int kRangeV = 2;        // LASER_CELL_RANGE_VERTICAL

struct P4 { float x, y, z, i; };
using Cube = std::tuple<int, int, int>;

// pcl::VoxelGrid<PointXYZI>::applyFilter (B.1), in place
void voxel_grid_xyzi(std::vector<P4>& pts, float leaf) {
    if (pts.empty()) return;
    const float inv = 1.0f / leaf;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (const P4& p : pts) {
        const float v[3] = {p.x, p.y, p.z};
        for (int d = 0; d < 3; ++d) { mn[d] = std::min(mn[d], v[d]); mx[d] = std::max(mx[d], v[d]); }
    }
    const int64_t dx = static_cast<int64_t>((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = static_cast<int64_t>((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = static_cast<int64_t>((mx[2] - mn[2]) * inv) + 1;
    if (dx * dy * dz > static_cast<int64_t>(INT32_MAX)) return;    // "leaf size too small": unchanged
    int min_b[3], mul[3];
    for (int d = 0; d < 3; ++d) min_b[d] = static_cast<int>(std::floor(mn[d] * inv));
    const int div0 = static_cast<int>(std::floor(mx[0] * inv)) - min_b[0] + 1;
    const int div1 = static_cast<int>(std::floor(mx[1] * inv)) - min_b[1] + 1;
    mul[0] = 1; mul[1] = div0; mul[2] = div0 * div1;
    std::vector<std::pair<unsigned, unsigned>> iv(pts.size());
    for (size_t i = 0; i < pts.size(); ++i) {
        const P4& p = pts[i];
        const int i0 = static_cast<int>(std::floor(p.x * inv) - static_cast<float>(min_b[0]));
        const int i1 = static_cast<int>(std::floor(p.y * inv) - static_cast<float>(min_b[1]));
        const int i2 = static_cast<int>(std::floor(p.z * inv) - static_cast<float>(min_b[2]));
        iv[i] = {static_cast<unsigned>(i0 * mul[0] + i1 * mul[1] + i2 * mul[2]), static_cast<unsigned>(i)};
    }
    std::stable_sort(iv.begin(), iv.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    std::vector<P4> out;
    for (size_t s = 0; s < iv.size();) {
        size_t e = s + 1;
        while (e < iv.size() && iv[e].first == iv[s].first) ++e;
        float sx = 0, sy = 0, sz = 0, si = 0;
        for (size_t k = s; k < e; ++k) {
            const P4& p = pts[iv[k].second];
            sx += p.x; sy += p.y; sz += p.z; si += p.i;
        }
        const float n = static_cast<float>(e - s);
        out.push_back({sx / n, sy / n, sz / n, si / n});
        s = e;
    }
    pts.swap(out);
}

int cube_of(float v) { return static_cast<int>(std::floor(v / kCell + 0.5)); }   // float promoted
int cube_of_d(double v) { return static_cast<int>(std::floor(v / kCell + 0.5)); }

}  // namespace
}  // namespace pfref

using namespace pfref;

struct pfref_map {
    float leaf = 0.4f;
    std::map<Cube, std::vector<P4>> cubes;   // allocated cubes (possibly empty), ordered x, y, z
};

extern "C" {

// LaserMappingClass::init (:7-33): the 5 x 5 x 5 cubes around the origin, VoxelGrid leaf
pfref_map* pfref_map_create(double map_resolution) {
    pfref_map* m = new pfref_map();
    m->leaf = static_cast<float>(map_resolution);                   // setLeafSize(float, float, float)
    for (int i = -kRangeH; i <= kRangeH; ++i)
        for (int j = -kRangeH; j <= kRangeH; ++j)
            for (int k = -kRangeV; k <= kRangeV; ++k) m->cubes[Cube(i, j, k)];
    return m;
}

void pfref_map_destroy(pfref_map* m) { delete m; }

// updateCurrentPointsToMap (:151-189). pose = qx, qy, qz, qw, tx, ty, tz (the odometry message's
// orientation and position). Returns 0, or -1 when a point falls into a cube the reference never
// allocated (it dereferences a null cloud there).
int pfref_map_update(pfref_map* m, const float* xyzi, size_t n, size_t stride, const double pose[7]) {
    const double tx = pose[4], ty = pose[5], tz = pose[6];
    const int cx = cube_of_d(tx), cy = cube_of_d(ty), cz = cube_of_d(tz);
    for (int i = cx - kRangeH; i <= cx + kRangeH; ++i)                 // checkPoints (:105-147)
        for (int j = cy - kRangeH; j <= cy + kRangeH; ++j)
            for (int k = cz - kRangeV; k <= cz + kRangeV; ++k) m->cubes[Cube(i, j, k)];
    // Isometry3d: rotate(Quaterniond(w, x, y, z)) then pretranslate(t); cast<float>()
    const M3 R = q2m(Quat{pose[0], pose[1], pose[2], pose[3]});
    float c[4][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) c[b][a] = static_cast<float>(R.m[a][b]);   // column b
    c[3][0] = static_cast<float>(tx); c[3][1] = static_cast<float>(ty); c[3][2] = static_cast<float>(tz);
    std::vector<std::pair<Cube, P4>> add;
    add.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        const float* p = reinterpret_cast<const float*>(reinterpret_cast<const char*>(xyzi) + i * stride);
        P4 q;
        float o[3];
        for (int a = 0; a < 3; ++a) o[a] = p[0] * c[0][a] + (p[1] * c[1][a] + (p[2] * c[2][a] + c[3][a]));
        q.x = o[0]; q.y = o[1]; q.z = o[2];
        q.i = static_cast<float>(std::min(1.0, std::max(static_cast<double>(p[2]) + 2.0, 0.0) / 5));   // :167
        const Cube cb(cube_of(q.x), cube_of(q.y), cube_of(q.z));
        if (!m->cubes.count(cb)) return -1;
        add.emplace_back(cb, q);
    }
    for (const auto& e : add) m->cubes[e.first].push_back(e.second);
    for (int i = cx - kRangeH; i <= cx + kRangeH; ++i)                 // :176-187
        for (int j = cy - kRangeH; j <= cy + kRangeH; ++j)
            for (int k = cz - kRangeV; k <= cz + kRangeV; ++k) voxel_grid_xyzi(m->cubes[Cube(i, j, k)], m->leaf);
    return 0;
}

// getMap (:194-206): x, y, z, intensity of every cube's points, cubes in x, then y, then z order
int pfref_map_get(const pfref_map* m, float* xyzi, size_t cap, size_t* n) {
    size_t tot = 0;
    for (const auto& e : m->cubes) tot += e.second.size();
    if (n) *n = tot;
    if (!xyzi) return 0;
    if (tot > cap) return -1;
    size_t k = 0;
    for (const auto& e : m->cubes)
        for (const P4& p : e.second) {
            xyzi[4 * k] = p.x; xyzi[4 * k + 1] = p.y; xyzi[4 * k + 2] = p.z; xyzi[4 * k + 3] = p.i;
            ++k;
        }
    return 0;
}

}  // extern "C"
