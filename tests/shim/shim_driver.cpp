// Drives the C++ shim the way the ROS nodes do (src/laserProcessingNode.cpp:71-78 then
// src/odomEstimationNode copy.cpp:86-107): per frame, featureExtraction -> copy XYZI to XYZRGB ->
// initMapWithPoints (first frame) / updatePointsToMap -> read `odom`. Input: a binary file of frames
// (int64 n, then n x 4 float32). Output: one line per frame with the 7 pose values (%.17g).
//   shim_driver frames.bin poses.txt
#include <cstdio>
#include <vector>

#include "mock_pcl.hpp"
#define PFILTER_HIP_NO_EIGEN
#include "../../pfilter-noetic_amd/shim/pfilter_hip_shim.hpp"

using Fe = pfilter_hip::LaserProcessingClassT<mock::PointCloud<mock::PointXYZI>, mock::Lidar>;
using Odom = pfilter_hip::Odom_ES_EstimationClassT<mock::PointCloud<mock::PointXYZRGB>, mock::Lidar>;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    FILE* o = std::fopen(argv[2], "w");
    if (!f || !o) return 2;
    mock::Lidar lidar;
    Fe fe;
    fe.init(lidar);
    Odom odom;
    odom.init(lidar, 0.4, 0, 0.4f, 75, 0.0);
    bool inited = false;
    long long n;
    while (std::fread(&n, sizeof(n), 1, f) == 1) {
        std::vector<float> buf(4 * n);
        if (std::fread(buf.data(), sizeof(float), 4 * n, f) != (size_t)(4 * n)) return 3;
        auto in = std::make_shared<mock::PointCloud<mock::PointXYZI>>();
        for (long long i = 0; i < n; ++i) {
            mock::PointXYZI p;
            p.x = buf[4 * i]; p.y = buf[4 * i + 1]; p.z = buf[4 * i + 2]; p.intensity = buf[4 * i + 3];
            in->push_back(p);
        }
        auto e = std::make_shared<mock::PointCloud<mock::PointXYZI>>();
        auto s = std::make_shared<mock::PointCloud<mock::PointXYZI>>();
        fe.featureExtraction(in, e, s);
        auto e2 = std::make_shared<mock::PointCloud<mock::PointXYZRGB>>();   // pcl::copyPointCloud
        auto s2 = std::make_shared<mock::PointCloud<mock::PointXYZRGB>>();
        for (const auto& p : e->points) { mock::PointXYZRGB q; q.x = p.x; q.y = p.y; q.z = p.z; e2->push_back(q); }
        for (const auto& p : s->points) { mock::PointXYZRGB q; q.x = p.x; q.y = p.y; q.z = p.z; s2->push_back(q); }
        if (!inited) { odom.initMapWithPoints(e2, s2); inited = true; }
        else odom.updatePointsToMap(e2, s2);
        std::fprintf(o, "%.17g %.17g %.17g %.17g %.17g %.17g %.17g %zu %zu", odom.odom.q[0], odom.odom.q[1],
                     odom.odom.q[2], odom.odom.q[3], odom.odom.t[0], odom.odom.t[1], odom.odom.t[2],
                     odom.laserCloudCornerMap->size(), odom.laserCloudSurfMap->size());
        // the OdomBaseClass members (parameters, last_odom translation, optimization_count) and a
        // checksum of the surf map's ages / p-index bytes (refreshed through the pinned map export)
        for (int k = 0; k < 7; ++k) std::fprintf(o, " %.17g", odom.parameters[k]);
        std::fprintf(o, " %.17g %.17g %.17g %d", odom.last_odom[3], odom.last_odom[7], odom.last_odom[11],
                     odom.optimization_count);
        unsigned long long cs = 0;
        for (const auto& p : odom.laserCloudSurfMap->points) cs = cs * 1000003ull + (unsigned)p.r * 256u + p.g;
        std::fprintf(o, " %llu\n", cs);
    }
    std::fclose(f);
    std::fclose(o);
    return 0;
}
