// pfref internal types. TEST INFRASTRUCTURE (oracle) — see pfref.h header.
#pragma once
#include "pfref.h"
#include "pfref_math.h"

#include <cstdint>
#include <vector>

extern "C" void pfref_introsort_stats(const uint32_t* keys, size_t n, long* st);   // pfref_sort.cpp
extern "C" void pfref_introsort_heapdep(const uint32_t* keys, const uint8_t* dep, size_t n, const char* tag);

namespace pfref {

struct PtI { float x, y, z, intensity; };                 // pcl::PointXYZI (fields used)
struct PtC {                                               // pcl::PointXYZRGB (fields used)
    float x, y, z;
    uint8_t r, g, b;
};

int ring_id(const pfref_lidar& lp, const PtI& p, bool sqrt_double);
double curvature(const std::vector<PtI>& ring, int j);
void feature_extraction(const pfref_lidar& lp, int opts, const PtI* in, size_t n, std::vector<PtI>& edge,
                        std::vector<PtI>& surf);

// PCL 1.10 VoxelGrid<PointXYZRGB>::applyFilter with downsample_all_data_
void voxel_grid(const std::vector<PtC>& in, float leaf, bool stable, std::vector<PtC>& out);
// OdomBaseClass::rgbds (src/odomEstimationClass.cpp:34-134)
void rgbds(const std::vector<PtC>& in, float dsleaf, bool stable, std::vector<PtC>& out);

// FLANN-style single kd-tree (leaf 15), exact kNN; ties resolved by (d2, index).
class KdTree {
public:
    void build(const std::vector<PtC>& pts);
    // k <= 8; returns found count; idx/d2 sorted ascending by (d2, idx)
    int knn(const float q[3], int k, int* idx, float* d2) const;
private:
    struct Node { int left, right; int divfeat; float divlow, divhigh; int child1, child2; };
    int build_rec(int lo, int hi, const float* bmin, const float* bmax);
    void search(int node, const float q[3], float mindist, float dists[3], struct KnnSet& rs) const;
    std::vector<float> xyz_;     // reordered copy, 3 floats/pt
    std::vector<int> vind_;      // original indices
    std::vector<Node> nodes_;
    int root_ = -1;
};

void knn_brute(const std::vector<PtC>& map, const float q[3], int k, int* idx, float* d2);

// FLANN L2_Simple<float>: sum of squared differences in dimension order, float
inline float l2f(const float* a, const float* b) {
    float r = 0.0f;
    float d = a[0] - b[0]; r += d * d;
    d = a[1] - b[1]; r += d * d;
    d = a[2] - b[2]; r += d * d;
    return r;
}

}  // namespace pfref
