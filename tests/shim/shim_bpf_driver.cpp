// Drives the C++ BPF shim the way src/odomEstimationNode.cpp:191-264 does: per frame, the classified
// beam / pillar / facade clouds (XYZINormal copied to XYZRGB) -> initMapWithPoints (first frame) /
// updatePointsToMap -> read `odom` and the map members. Input: a binary file of frames, each three
// clouds (int64 n, then n x 4 float32). Output: one line per frame with the 7 pose values (%.17g),
// the beam / pillar / facade map sizes and the merged map size.
//   shim_bpf_driver clouds.bin poses.txt
#include <cstdio>
#include <vector>

#include "mock_pcl.hpp"
#define PFILTER_HIP_NO_EIGEN
#include "../../pfilter-noetic_amd/shim/pfilter_hip_shim.hpp"

using Cloud = mock::PointCloud<mock::PointXYZRGB>;
using Odom = pfilter_hip::Odom_BPF_EstimationClassT<Cloud, mock::Lidar>;

static bool read_cloud(FILE* f, std::shared_ptr<Cloud>& out) {
    long long n;
    if (std::fread(&n, sizeof(n), 1, f) != 1) return false;
    std::vector<float> buf(4 * (n ? n : 1));
    if (n && std::fread(buf.data(), sizeof(float), 4 * n, f) != (size_t)(4 * n)) return false;
    out = std::make_shared<Cloud>();
    for (long long i = 0; i < n; ++i) {
        mock::PointXYZRGB q;
        q.x = buf[4 * i]; q.y = buf[4 * i + 1]; q.z = buf[4 * i + 2];
        out->push_back(q);
    }
    return true;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    FILE* o = std::fopen(argv[2], "w");
    if (!f || !o) return 2;
    mock::Lidar lidar;
    Odom odom;
    odom.init(lidar, 0.4, 0, 0.4f, 75, 0.0);
    bool inited = false;
    std::shared_ptr<Cloud> b, p, fa;
    while (read_cloud(f, b) && read_cloud(f, p) && read_cloud(f, fa)) {
        if (!inited) { odom.initMapWithPoints(b, p, fa); inited = true; }
        else odom.updatePointsToMap(b, p, fa);
        std::fprintf(o, "%.17g %.17g %.17g %.17g %.17g %.17g %.17g %zu %zu %zu %zu\n", odom.odom.q[0],
                     odom.odom.q[1], odom.odom.q[2], odom.odom.q[3], odom.odom.t[0], odom.odom.t[1], odom.odom.t[2],
                     odom.laserCloudBeamMap->size(), odom.laserCloudPillarMap->size(),
                     odom.laserCloudFacadeMap->size(), odom.laserCloudMergeMap->size());
    }
    std::fclose(f);
    std::fclose(o);
    return 0;
}
