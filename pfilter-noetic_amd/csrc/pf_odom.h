// Device-resident Odom_ES_EstimationClass (src/odomEstimationClass.cpp:182-647).
#pragma once
#include "pf_common.h"
#include "pf_fe.h"
#include "pf_knn.h"
#include "pf_prims.h"

namespace pf {

// device counter slots (int32, one array per handle)
enum CounterSlot {
    C_EIN = 0, C_SIN, C_VGN, C_EDS, C_SDS, C_NQ, C_ME, C_MS, C_NPAIR, C_NRG, C_NSEG, C_NSEG_E, C_NRG_VALID,
    C_KEEP_TOTAL, C_EDGE_KEPT, C_SURF_KEPT, C_EDGE_VALID, C_SURF_VALID, C_LM_ITERS, C_GATE, C_ERR,
    C_OUTER, C_PAD0, C_PAD1, C_NIN, C_FE_ERR, C_COUNT
};

// ordered-uint accumulator slots (float min/max via atomics)
enum AccSlot {
    A_VG = 0,        // [cloud][6]: min xyz, max xyz  (12)
    A_RG = 12,       // [cloud][6]                     (12)
    A_W = 24,        // [class][4]: obs min, obs max, spars min, spars max (8)
    A_COUNT = 32
};

struct DevState {
    double params[7];      // q (x,y,z,w), t: OdomBaseClass::parameters (.h:53-55)
    double odomR[9], odomt[3];
    double lastR[9], lastt[3];
    int optimization_count;
    int gate;
    int frame;
    int pad;
};

struct LMState {
    double x[7], cand[7], best[7];
    double scale[6];
    double cost, H[21], g[6];
    double D[6];
    double radius, decrease, x_norm, min_cost, mcc;
    double wmin[2][2], wmax[2][2];   // [class][observe, sparsity]
    int iteration, invalid, reuse, done, phase, n_res, pad0, pad1;
};

constexpr int kLmParts = 30;   // cost, g[6], H[21], bad_r, bad_J

struct OdomGPU {
    pf_lidar_params lidar{};
    pf_odom_params prm{};
    int device = 0;
    hipStream_t stream = nullptr;
    size_t in_cap = 0, map_cap = 0, sort_cap = 0, pose_cap = 0;
    int pidx_bits = 32;            // key bits the p-index pair sort needs
    int opt_count_host = 2;
    bool inited = false;
    int frames = 0;
    float leaf_vg[2] = {0, 0};     // downSizeFilterEdge/Surf leaf (double -> float)
    float leaf_rg[2] = {0, 0};     // rgbds leaves: map_resolution, map_resolution * 2 (float)

    FeGPU fe;
    GridGPU grid;
    PrimWork prim;

    DevState* st = nullptr;
    LMState* lm = nullptr;
    int* cnt = nullptr;
    u32* acc = nullptr;
    int* h_cnt = nullptr;          // pinned mirror
    double* h_pose = nullptr;      // pinned [7]

    float4 *in_edge = nullptr, *in_surf = nullptr;
    float4 *ds_edge = nullptr, *ds_surf = nullptr;
    float4 *map_e = nullptr, *map_s = nullptr;
    float4 *app_e = nullptr, *app_s = nullptr;
    float4* seg_out = nullptr;
    u32 *keys = nullptr, *vals = nullptr, *flags = nullptr, *scan_out = nullptr, *segstart = nullptr;

    int* nbr = nullptr;            // [5 * 2 * in_cap]
    int* qflag = nullptr;          // bit0 valid association, bit1 kept
    double* geo = nullptr;         // [8 * 2 * in_cap]
    float* spars = nullptr;
    float* roundv = nullptr;
    float* observe = nullptr;
    u32* pcnt = nullptr;           // [5 * 2 * in_cap]
    u32* tailinc = nullptr;        // [sort_cap]
    double* lm_part = nullptr;     // [kLmBlocks * 32] per-block LM partials
    u32* lm_ticket = nullptr;      // LM arrival counter
    unsigned long long* dbg = nullptr;   // [64] device timestamps (development probe)
    double* poses = nullptr;       // [pose_cap * 7]
    float4* stage = nullptr;       // [2 * in_cap] host staging target

    hipGraphExec_t graph = nullptr;
    bool graph_enabled = true;
    const float4* graph_in = nullptr;
    int graph_n = -1;
};

int odom_create(OdomGPU& o, const pf_lidar_params& lidar, const pf_odom_params& prm, int device, size_t in_cap,
                size_t map_cap);
void odom_destroy(OdomGPU& o);
// enqueue initMapWithPoints from in_edge/in_surf (counts in cnt[C_EIN], cnt[C_SIN])
void odom_enqueue_init(OdomGPU& o, hipStream_t s);
// enqueue updatePointsToMap from in_edge/in_surf (device counts); outer iteration count = host mirror
void odom_enqueue_update(OdomGPU& o, hipStream_t s);
// enqueue featureExtraction(d_in[0 .. cnt[C_NIN])) followed by init or update
void odom_enqueue_frame(OdomGPU& o, const float4* d_in, hipStream_t s);

}  // namespace pf
