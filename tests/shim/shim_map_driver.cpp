// Drives the LaserMappingClass shim the way src/laserMappingNode.cpp:72-86 does: per frame a cloud and
// the pose (row-major [R | t]) -> updateCurrentPointsToMap -> getMap. Input: frames (int64 n, 12
// doubles, then n x 4 float32). Output: the final map, n x 4 float32.
//   shim_map_driver frames.bin map.bin
#include <cstdio>
#include <vector>

#include "mock_pcl.hpp"
#define PFILTER_HIP_NO_EIGEN
#include "../../pfilter-noetic_amd/shim/pfilter_hip_shim.hpp"

using Cloud = mock::PointCloud<mock::PointXYZI>;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    FILE* o = std::fopen(argv[2], "wb");
    if (!f || !o) return 2;
    pfilter_hip::LaserMappingClassT<Cloud> mapping;
    mapping.init(0.4);
    long long n;
    while (std::fread(&n, sizeof(n), 1, f) == 1) {
        double T[12];
        if (std::fread(T, sizeof(double), 12, f) != 12) return 3;
        std::vector<float> buf(4 * (n ? n : 1));
        if (n && std::fread(buf.data(), sizeof(float), 4 * n, f) != (size_t)(4 * n)) return 3;
        Cloud::Ptr in = std::make_shared<Cloud>();
        for (long long i = 0; i < n; ++i) {
            mock::PointXYZI q;
            q.x = buf[4 * i]; q.y = buf[4 * i + 1]; q.z = buf[4 * i + 2]; q.intensity = buf[4 * i + 3];
            in->push_back(q);
        }
        mapping.updateCurrentPointsToMap(in, T);
    }
    Cloud::Ptr map = mapping.getMap();
    for (const auto& q : map->points) {
        const float v[4] = {q.x, q.y, q.z, q.intensity};
        std::fwrite(v, sizeof(float), 4, o);
    }
    std::fclose(o);
    return 0;
}
