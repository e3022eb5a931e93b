// Drives the curvedVoxel shim (pfilter_hip::CurvedVoxelT) the way src/additionNode.cpp:29-39 does:
// one object, run() per frame, then reads pointCloudSegPtr and labelRecords. Input: frames (int64 n,
// then n x 4 float32). Output per frame: the kept count and the cluster count, then per kept point its
// x, y, z (float32), per cluster its rank, size and first input index (int32), then per cluster the
// bounds clusterBoxes() gives colorSegmentation (lo xyz, hi xyz, float32).
//   shim_dcvc_driver scans.bin out.bin
#include <cstdio>
#include <vector>

#include "mock_pcl.hpp"
#define PFILTER_HIP_NO_EIGEN
#include "../../pfilter-noetic_amd/shim/pfilter_hip_shim.hpp"

using CloudI = mock::PointCloud<mock::PointXYZI>;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    FILE* o = std::fopen(argv[2], "wb");
    if (!f || !o) return 2;
    pfilter_hip::CurvedVoxelT<CloudI> curvedvoxel;
    pfilter_hip::CurvedVoxelT<CloudI> bound = curvedvoxel;    // boost::bind's copy shares the device handle
    long long n;
    while (std::fread(&n, sizeof(n), 1, f) == 1) {
        std::vector<float> buf(4 * (n ? n : 1));
        if (n && std::fread(buf.data(), sizeof(float), 4 * n, f) != (size_t)(4 * n)) return 3;
        CloudI::Ptr in = std::make_shared<CloudI>();
        for (long long i = 0; i < n; ++i) {
            mock::PointXYZI q;
            q.x = buf[4 * i]; q.y = buf[4 * i + 1]; q.z = buf[4 * i + 2]; q.intensity = buf[4 * i + 3];
            in->push_back(q);
        }
        bound.run(in);
        const long long hdr[2] = {(long long)bound.pointCloudSegPtr->size(), (long long)bound.labelRecords.size()};
        std::fwrite(hdr, sizeof(long long), 2, o);
        for (const auto& q : bound.pointCloudSegPtr->points) {
            const float v[3] = {q.x, q.y, q.z};
            std::fwrite(v, sizeof(float), 3, o);
        }
        for (const auto& r : bound.labelRecords) {
            const int32_t v[3] = {r.first, r.second.clusterNum, r.second.index.empty() ? -1 : r.second.index[0]};
            std::fwrite(v, sizeof(int32_t), 3, o);
        }
        for (const auto& b : bound.clusterBoxes()) {
            std::fwrite(b.lo, sizeof(float), 3, o);
            std::fwrite(b.hi, sizeof(float), 3, o);
        }
    }
    std::fclose(o);
    return 0;
}
