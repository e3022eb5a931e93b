// Minimal stand-ins for the PCL / lidar types the C++ shim is instantiated with, so that the shim
// can be compiled and run without PCL (test only). Layouts follow PCL 1.10: 32-byte points with
// x, y, z at offsets 0, 4, 8; intensity at 16 (PointXYZI); b, g, r, a bytes at 16 (PointXYZRGB).
#pragma once
#include <cstdint>
#include <memory>
#include <vector>

namespace mock {
struct PointXYZI {
    float x = 0, y = 0, z = 0, pad0 = 1;
    float intensity = 0, pad1[3] = {0, 0, 0};
};
struct PointXYZRGB {
    float x = 0, y = 0, z = 0, pad0 = 1;
    uint8_t b = 0, g = 0, r = 0, a = 255;
    float pad1[3] = {0, 0, 0};
};
static_assert(sizeof(PointXYZI) == 32 && sizeof(PointXYZRGB) == 32, "PCL point layout");
template <class T>
struct PointCloud {
    using Ptr = std::shared_ptr<PointCloud<T>>;
    std::vector<T> points;
    void push_back(const T& p) { points.push_back(p); }
    void clear() { points.clear(); }
    size_t size() const { return points.size(); }
};
struct Lidar {
    int num_lines = 64;
    double min_distance = 3.0, max_distance = 90.0, scan_period = 0.1;
};
}  // namespace mock
