// Drives the front-end shim (groundSeg + nongroundExtract) the way src/additionNode.cpp:21-45 does:
// ground_seg with groundSeg's members, pc2pc of the non-ground cloud, featureExtract, then reads
// cloud_beam / cloud_pillar / cloud_facade. Input: frames (int64 n, then n x 4 float32). Output per
// frame: ground, non-ground, beam, pillar, facade sizes, then the xyz of the three clouds.
//   shim_cls_driver scans.bin out.bin
#include <cstdio>
#include <vector>

#include "mock_pcl.hpp"
#define PFILTER_HIP_NO_EIGEN
#include "../../pfilter-noetic_amd/shim/pfilter_hip_shim.hpp"

namespace mock {
struct PointXYZINormal {
    float x = 0, y = 0, z = 0, pad0 = 1;
    float normal_x = 0, normal_y = 0, normal_z = 0, curvature = 0;
    float intensity = 0, pad1[3] = {0, 0, 0};
};
}  // namespace mock

using CloudI = mock::PointCloud<mock::PointXYZI>;
using CloudN = mock::PointCloud<mock::PointXYZINormal>;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    FILE* o = std::fopen(argv[2], "wb");
    if (!f || !o) return 2;
    pfilter_hip::GroundSegT<CloudI> groundseg;
    pfilter_hip::NongroundExtractT<mock::PointCloud, mock::PointXYZINormal> extra;
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
        groundseg.groundInit(in);
        groundseg.ground_seg(groundseg.groundSeginputCloudPtr, groundseg.groundCloudPtr, groundseg.nonGroundCloudPtr,
                             groundseg.gf_grid_pt_num_thre, groundseg.gf_grid_resolution,
                             groundseg.gf_max_grid_height_diff, groundseg.gf_neighbor_height_diff,
                             groundseg.gf_max_ground_height, groundseg.gf_min_ground_height);
        extra.featureInit();
        extra.pc2pc<CloudI>(groundseg.nonGroundCloudPtr, extra.normalCloud);
        extra.featureExtract<mock::PointXYZINormal>(extra.normalCloud);
        const long long sz[5] = {(long long)groundseg.groundCloudPtr->size(), (long long)groundseg.nonGroundCloudPtr->size(),
                                 (long long)extra.cloud_beam->size(), (long long)extra.cloud_pillar->size(),
                                 (long long)extra.cloud_facade->size()};
        std::fwrite(sz, sizeof(long long), 5, o);
        for (const auto& c : {extra.cloud_beam, extra.cloud_pillar, extra.cloud_facade})
            for (const auto& q : c->points) {
                const float v[7] = {q.x, q.y, q.z, q.normal_x, q.normal_y, q.normal_z, q.curvature};
                std::fwrite(v, sizeof(float), 7, o);
            }
    }
    std::fclose(o);
    return 0;
}
