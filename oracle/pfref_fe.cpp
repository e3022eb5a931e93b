// pfref: LaserProcessingClass::featureExtraction restated (src/laserProcessingClass.cpp:10-209).
// TEST INFRASTRUCTURE (oracle) — see pfref.h header.
#include "pfref_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdio>

namespace pfref {

namespace {
struct Double2d {          // include/laserProcessingClass.h:17-22
    int id;
    double value;
};

// featureExtractionFromSector (src/laserProcessingClass.cpp:99-209)
void from_sector(const std::vector<PtI>& ring, std::vector<Double2d>& cc, bool stable_ties,
                 std::vector<PtI>& edge, std::vector<PtI>& surf) {
    if (stable_ties)
        std::sort(cc.begin(), cc.end(), [](const Double2d& a, const Double2d& b) {
            return a.value < b.value || (a.value == b.value && a.id < b.id);
        });
    else
        std::sort(cc.begin(), cc.end(), [](const Double2d& a, const Double2d& b) { return a.value < b.value; });

    int largestPickedNum = 0;
    std::vector<int> picked;
    for (int i = (int)cc.size() - 1; i >= 0; i--) {           // :110-148
        int ind = cc[i].id;
        if (std::find(picked.begin(), picked.end(), ind) == picked.end()) {
            if (cc[i].value <= 0.1) break;                     // :114-116
            largestPickedNum++;
            picked.push_back(ind);
            if (largestPickedNum <= 20) {
                edge.push_back(ring[ind]);
            } else {
                break;                                         // :124-126 (21st: neither edge nor surf)
            }
            for (int k = 1; k <= 5; k++) {                     // :128-136
                double dx = ring[ind + k].x - ring[ind + k - 1].x;   // float difference
                double dy = ring[ind + k].y - ring[ind + k - 1].y;
                double dz = ring[ind + k].z - ring[ind + k - 1].z;
                if (dx * dx + dy * dy + dz * dz > 0.05) break;
                picked.push_back(ind + k);
            }
            for (int k = -1; k >= -5; k--) {                   // :137-145
                double dx = ring[ind + k].x - ring[ind + k + 1].x;
                double dy = ring[ind + k].y - ring[ind + k + 1].y;
                double dz = ring[ind + k].z - ring[ind + k + 1].z;
                if (dx * dx + dy * dy + dz * dz > 0.05) break;
                picked.push_back(ind + k);
            }
        }
    }
    for (int i = 0; i <= (int)cc.size() - 1; i++) {           // :198-205
        int ind = cc[i].id;
        if (std::find(picked.begin(), picked.end(), ind) == picked.end()) surf.push_back(ring[ind]);
    }
}
}  // namespace

// Ring id of one point (src/laserProcessingClass.cpp:22-61); -1 = rejected.
int ring_id(const pfref_lidar& lp, const PtI& p, bool sqrt_double) {
    const int N_SCANS = lp.num_lines;
    float sq = p.x * p.x + p.y * p.y;                      // float arithmetic (:23)
    double distance = sqrt_double ? std::sqrt((double)sq) : (double)std::sqrt(sq);
    if (distance < lp.min_distance || distance > lp.max_distance) return -1;
    double angle = std::atan(p.z / distance) * 180 / M_PI;
    int scanID = 0;
    if (lp.ring_top > lp.ring_bottom) {    // extension: linear beam model (pf_fe_set_ring_model)
        const double scale = (double)N_SCANS / (lp.ring_top - lp.ring_bottom);
        scanID = int((lp.ring_top - angle) * scale);
        if (!(lp.ring_top - angle >= 0.0) || scanID > N_SCANS - 1) return -1;
    } else if (N_SCANS == 16) {
        scanID = int((angle + 15) / 2 + 0.5);
        if (scanID > (N_SCANS - 1) || scanID < 0) return -1;
    } else if (N_SCANS == 32) {
        scanID = int((angle + 92.0 / 3.0) * 3.0 / 4.0);
        if (scanID > (N_SCANS - 1) || scanID < 0) return -1;
    } else if (N_SCANS == 64) {
        if (angle >= -8.83)
            scanID = int((2 - angle) * 3.0 + 0.5);
        else
            scanID = N_SCANS / 2 + int((-8.83 - angle) * 2.0 + 0.5);
        if (angle > 2 || angle < -24.33 || scanID > 63 || scanID < 0) return -1;
    } else {
        // "wrong scan number" (:58-61): every point lands in ring 0
        scanID = 0;
    }
    return scanID;
}

// Curvature of ring point j (:73-77): the 11-tap sums are FLOAT expressions evaluated left to
// right (all operands are float), then widened; the squares are summed in double.
double curvature(const std::vector<PtI>& r, int j) {
    float dx = r[j - 5].x + r[j - 4].x + r[j - 3].x + r[j - 2].x + r[j - 1].x - 10 * r[j].x + r[j + 1].x +
               r[j + 2].x + r[j + 3].x + r[j + 4].x + r[j + 5].x;
    float dy = r[j - 5].y + r[j - 4].y + r[j - 3].y + r[j - 2].y + r[j - 1].y - 10 * r[j].y + r[j + 1].y +
               r[j + 2].y + r[j + 3].y + r[j + 4].y + r[j + 5].y;
    float dz = r[j - 5].z + r[j - 4].z + r[j - 3].z + r[j - 2].z + r[j - 1].z - 10 * r[j].z + r[j + 1].z +
               r[j + 2].z + r[j + 3].z + r[j + 4].z + r[j + 5].z;
    double diffX = dx, diffY = dy, diffZ = dz;
    return diffX * diffX + diffY * diffY + diffZ * diffZ;
}

void feature_extraction(const pfref_lidar& lp, int opts, const PtI* in, size_t n, std::vector<PtI>& edge,
                        std::vector<PtI>& surf) {
    const int N_SCANS = lp.num_lines;
    const bool sqrt_double = (opts & PFREF_FE_SQRT_DOUBLE) != 0;
    const bool stable = (opts & PFREF_FE_STABLE_TIES) != 0;
    // removeNaNFromPointCloud fills an index list only; the cloud is not modified (:13)
    std::vector<std::vector<PtI>> scans(N_SCANS > 0 ? N_SCANS : 1);
    bool warned = false;
    for (size_t i = 0; i < n; i++) {
        int id = ring_id(lp, in[i], sqrt_double);
        if (id < 0) continue;
        if (N_SCANS != 16 && N_SCANS != 32 && N_SCANS != 64 && !(lp.ring_top > lp.ring_bottom) && !warned) {
            std::printf("wrong scan number\n");
            warned = true;
        }
        scans[id].push_back(in[i]);
    }
    for (int i = 0; i < N_SCANS; i++) {                       // :66-93
        const std::vector<PtI>& ring = scans[i];
        if (ring.size() < 131) continue;
        std::vector<Double2d> cc;
        int total_points = (int)ring.size() - 10;
        for (int j = 5; j < (int)ring.size() - 5; j++) cc.push_back({j, curvature(ring, j)});
        for (int j = 0; j < 6; j++) {
            int sector_length = (int)(total_points / 6);
            int sector_start = sector_length * j;
            int sector_end = sector_length * (j + 1) - 1;
            if (j == 5) sector_end = total_points - 1;
            std::vector<Double2d> sub(cc.begin() + sector_start, cc.begin() + sector_end);
            from_sector(ring, sub, stable, edge, surf);
        }
    }
}

}  // namespace pfref
