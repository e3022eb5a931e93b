// pfref: curvedVoxel (DCVC, Dynamic Curved-Voxel Clustering) restated — src/additionClass.cpp:1-497,
// include/additionClass.hpp:95-120. TEST INFRASTRUCTURE (oracle) — see pfref.h header.
//
// The reference runs its loops under `#pragma omp parallel for` with up to 6 threads, and the loop
// bodies write shared variables (cur, polarIndex, ... declared outside the loops, label_info relabelled
// from several threads): its output is not a function of its input. This restatement is the serial
// execution of the same source (one OpenMP thread), the only deterministic reading of it, quirks
// included:
//   * out-of-range points (r >= sensorMaxRange or r <= sensorMinRange, :112-113) keep a zero polar
//     coordinate and are clustered as (r 0, pitch 0, azimuth 0) (:96, :113-114);
//   * minPitch / maxPitch start at 0 every frame, minPolar / maxPolar at 5 on the first frame and at 0
//     after it (member defaults .hpp:103-106, resetParams :445-449);
//   * the neighbour search (searchKNN :196-225) skips pitch layers above `height` (so the top layer,
//     index round((maxPitch - minPitch) / deltaP) = height + 1, never finds its own voxel), wraps
//     azimuth -1 to width - 1 but clamps azimuth 301 to 300 (no wrap the other way);
//   * voxelFilter (:232-318) skips points already labelled, so clusters are the label classes of that
//     greedy pass, not connected components.
// labelAnalysis (:325-355) orders clusters by size with std::sort over an unordered_map's iteration
// order; for equal sizes that order is implementation-defined (parity unpinned). Here equal sizes are
// ordered by their smallest point index (the device does the same). Output: the points of clusters
// larger than minSeg, cluster by cluster, each cluster's points in input order (colorSegmentation
// :360-372, serial).
#include "pfref_internal.h"

#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

namespace {

struct Polar { double r, pitch, az; };

}  // namespace

extern "C" {

void pfref_dcvc_default_params(pfref_dcvc_params* p) {
    p->start_r = 1.0;          // config/config.yaml:50 startR
    p->delta_r = 0.003;        // :51 deltaR
    p->delta_p = 1.2;          // :52 deltaP
    p->delta_a = 1.2;          // :53 deltaA
    p->min_seg = 80;           // :54 minSeg
    p->min_range = 1.0;        // :7 sensorMinRange
    p->max_range = 120.0;      // :8 sensorMaxRange
}

int pfref_dcvc(const float* xyz, size_t n, size_t stride, const pfref_dcvc_params* p, int first_frame,
               int32_t* out_idx, size_t* n_out, int32_t* label) {
    return pfref_dcvc_mode(xyz, n, stride, p, first_frame, 0, out_idx, n_out, label);
}

// mode 0: the serial reading of voxelFilter (the reference-faithful restatement); mode 1: the connected
// components of the same voxel neighbourhood relation (every occupied voxel unioned with each occupied
// position of its searchKNN), which the device computes
int pfref_dcvc_mode(const float* xyz, size_t n, size_t stride, const pfref_dcvc_params* p, int first_frame,
                    int mode, int32_t* out_idx, size_t* n_out, int32_t* label) {
    if (!p || (!xyz && n) || stride < 12) return -1;
    if (n_out) *n_out = 0;
    if (n == 0) return 0;                                                    // :462-466 (error, no output)
    const char* b = reinterpret_cast<const char*>(xyz);
    auto pt = [&](size_t i) { return reinterpret_cast<const float*>(b + i * stride); };
    // convertToPolar (:85-136)
    double minPitch = 0.0, maxPitch = 0.0;
    double minPolar = first_frame ? 5.0 : 0.0, maxPolar = first_frame ? 5.0 : 0.0;
    std::vector<Polar> pc(n, Polar{0.0, 0.0, 0.0});
    for (size_t i = 0; i < n; ++i) {
        const double x = pt(i)[0], y = pt(i)[1], z = pt(i)[2];              // Eigen::Vector3d from float
        const double r = std::sqrt((x * x + y * y) + z * z);               // cur.norm()
        const double pitch = std::asin(z / r) * 180.0 / M_PI;
        const double ang = std::atan2(y, x);
        const double az = ang > 0.0 ? ang * 180 / M_PI : (ang + 2 * M_PI) * 180 / M_PI;
        if (r >= p->max_range || r <= p->min_range) continue;
        minPitch = pitch < minPitch ? pitch : minPitch;
        maxPitch = pitch > maxPitch ? pitch : maxPitch;
        minPolar = r < minPolar ? r : minPolar;
        maxPolar = r > maxPolar ? r : maxPolar;
        pc[i] = Polar{r, pitch, az};
    }
    const int width = static_cast<int>(std::round(360.0 / p->delta_a) + 1);
    const int height = static_cast<int>((maxPitch - minPitch) / p->delta_p);
    std::vector<double> bounds;
    {
        double range = minPolar;
        int step = 1;
        while (range <= maxPolar) {
            range += (p->start_r - step * p->delta_r);
            bounds.push_back(range);
            step++;
            if (bounds.size() > 100000) return -1;                          // non-terminating parameters
        }
    }
    const int polarNum = (int)bounds.size();
    auto polar_index = [&](double r) {                                      // getPolarIndex (:69-78)
        for (int k = 0; k < polarNum; ++k)
            if (r < bounds[k]) return k;
        return polarNum - 1;
    };
    // createHashTable (:143-177)
    std::vector<int> pol(n), pit(n), azi(n);
    std::map<long long, std::vector<int>> vmap;                             // voxelMap (unordered in the reference)
    auto vindex = [&](long long a, long long y, long long z) {
        return (a * (polarNum + 1) + y) + z * (long long)(polarNum + 1) * (width + 1);
    };
    for (size_t i = 0; i < n; ++i) {
        pol[i] = polar_index(pc[i].r);
        pit[i] = static_cast<int>(std::round((pc[i].pitch - minPitch) / p->delta_p));
        azi[i] = static_cast<int>(std::round(pc[i].az / p->delta_a));
        vmap[vindex(azi[i], pol[i], pit[i])].push_back((int)i);
    }
    std::vector<int> lab(n, -1);
    // searchKNN (:196-225): the occupied search positions of a voxel, in the reference's loop order
    auto search = [&](int pz, int py, int pa, std::vector<const std::vector<int>*>& out) {
        out.clear();
        for (int z = pz - 1; z <= pz + 1; ++z) {
            if (z < 0 || z > height) continue;
            for (int y = py - 1; y <= py + 1; ++y) {
                if (y < 0 || y > polarNum) continue;
                for (int x = pa - 1; x <= pa + 1; ++x) {
                    int ax = x;
                    if (ax < 0) ax = width - 1;
                    if (ax > 300) ax = 300;
                    auto it = vmap.find(vindex(ax, y, z));
                    if (it != vmap.end()) out.push_back(&it->second);
                }
            }
        }
    };
    std::vector<const std::vector<int>*> vs;
    if (mode == 1) {                                                        // connected components
        std::vector<int> parent(n);
        for (size_t i = 0; i < n; ++i) parent[i] = (int)i;
        auto find = [&](int a) {
            while (parent[a] != a) a = parent[a] = parent[parent[a]];
            return a;
        };
        for (auto& kv : vmap) {
            const int i = kv.second.front();
            search(pit[i], pol[i], azi[i], vs);
            vs.push_back(&kv.second);                                       // a voxel's own points belong together
            for (const std::vector<int>* v : vs)
                for (int j : *v) {
                    const int a = find(i), c = find(j);
                    if (a != c) parent[std::max(a, c)] = std::min(a, c);
                }
        }
        for (size_t i = 0; i < n; ++i) lab[i] = find((int)i);
    }
    // voxelFilter (:232-318), serial
    int labelCount = 0;
    std::vector<int> nb;
    for (size_t i = 0; i < n && mode == 0; ++i) {
        if (lab[i] != -1) continue;
        nb.clear();
        search(pit[i], pol[i], azi[i], vs);
        for (const std::vector<int>* v : vs) nb.insert(nb.end(), v->begin(), v->end());
        for (int id : nb) {
            const int cur = lab[i], nei = lab[id];
            if (cur != -1 && nei != -1 && cur != nei) {
                for (int& s : lab)
                    if (s == cur) s = nei;
            } else if (nei != -1) {
                lab[i] = nei;
            } else if (cur != -1) {
                lab[id] = cur;
            }
        }
        if (lab[i] == -1) {
            labelCount++;
            lab[i] = labelCount;
            for (int id : nb) lab[id] = labelCount;
        }
    }
    // labelAnalysis (:325-355): clusters larger than minSeg, by size, then by their first point
    std::map<int, std::vector<int>> cl;
    for (size_t i = 0; i < n; ++i) cl[lab[i]].push_back((int)i);
    std::vector<const std::vector<int>*> keep;
    for (auto& kv : cl)
        if ((int)kv.second.size() > p->min_seg) keep.push_back(&kv.second);
    std::sort(keep.begin(), keep.end(), [](const std::vector<int>* a, const std::vector<int>* b) {
        return a->size() != b->size() ? a->size() > b->size() : a->front() < b->front();
    });
    if (label) std::fill(label, label + n, 0);
    size_t k = 0;
    for (size_t c = 0; c < keep.size(); ++c)
        for (int i : *keep[c]) {
            if (out_idx) out_idx[k] = i;
            if (label) label[i] = (int32_t)(c + 1);
            ++k;
        }
    if (n_out) *n_out = k;
    return 0;
}

}  // extern "C"
