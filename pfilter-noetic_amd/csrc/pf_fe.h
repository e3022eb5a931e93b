// Feature extraction on the device: LaserProcessingClass::featureExtraction
// (src/laserProcessingClass.cpp:10-209) as six launches with device-resident counts.
#pragma once
#include "pf_common.h"

namespace pf {

constexpr int kMaxRings = 128;
constexpr int kSecLds = 2048;      // sectors up to this many curvature entries sort in LDS (KITTI-64: ~330);
                                   // larger ones (any size) sort in global scratch
constexpr int kEdgePerSector = 20; // src/laserProcessingClass.cpp:121

struct FeGPU {
    pf_lidar_params lidar{};
    int sqrt_double = 0;         // 0: sqrtf overload (default), 1: double sqrt
    // ring model extension (pf_fe_set_ring_model): scale > 0 selects a linear beam model, ring =
    // int((ring_top - elevation_deg) * ring_scale), for line counts the reference has no formula for
    double ring_top = 0.0, ring_scale = 0.0;
    int tie_order = 0;           // sectors with equal curvatures in libstdc++ std::sort's order (:101-104)
    size_t cap = 0;              // max input points
    int nblk_cap = 0;            // ceil(cap / 256)
    int rings = 0;               // number of ring lists (num_lines)
    // buffers
    int* ring = nullptr;         // [cap]  ring id or -1
    u32* blkhist = nullptr;      // [rings * nblk_cap]
    int* ring_start = nullptr;   // [kMaxRings + 1]
    float4* rp = nullptr;        // [cap] ring-ordered points
    int* sec_edge_ids = nullptr; // [rings*6*20]
    int* sec_surf_ids = nullptr; // [cap]  surf ids of the sector starting at ring point base + cs, from there
    double* big_val = nullptr;   // [2 cap] sort scratch of sectors above kSecLds entries
    int* big_id = nullptr;       // [2 cap]
    unsigned char* big_picked = nullptr, *big_gap = nullptr;   // [2 cap]
    int* sec_cnt = nullptr;      // [rings*6*2]  edge, surf counts
    int* sec_off = nullptr;      // [rings*6*2]  output offsets
    int* err = nullptr;          // [1] error flag (unused since sectors of any size are handled; kept for the ABI)
    float4* d_in_stage = nullptr;// [cap] staging for host inputs
};

int fe_alloc(FeGPU& f, const pf_lidar_params& lidar, size_t cap);
// linear beam model for L = num_lines rings between top_deg and bottom_deg (top > bottom), or the
// reference's ring formulas again (top == bottom == 0); PF_EINVAL otherwise
int fe_set_ring_model(FeGPU& f, double top_deg, double bottom_deg);
void fe_free(FeGPU& f);
// Enqueue feature extraction of *d_n device points (count read on the device). Outputs: edge/surf
// float4 arrays with device counts d_ne / d_ns (capacity: edge >= rings*120, surf >= n).
void fe_enqueue(FeGPU& f, const float4* d_in, const int* d_n, float4* edge, int* d_ne, float4* surf, int* d_ns,
                hipStream_t s);

}  // namespace pf
