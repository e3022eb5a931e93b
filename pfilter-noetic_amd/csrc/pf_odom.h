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

// One slot of the two-stage frame pipeline: a frame's features and their voxel-grid output, with
// the counters of that stage. Stage A (stream_a: featureExtraction + VoxelGrid, pose independent)
// fills slot k % 2 while stage B (stream: the odometry) still works on frame k - 1 in the other slot.
struct StageBuf {
    float4 *in_edge = nullptr, *in_surf = nullptr;   // featureExtraction output
    float4 *ds_edge = nullptr, *ds_surf = nullptr;   // VoxelGrid output (r, g written by the odometry)
    int* cnt = nullptr;                              // [C_COUNT] stage counters
};

// pipeline slots: frame k's stage A output lives in slot k % kSlots, so stage A may run up to
// kSlots - 1 frames ahead of stage B
constexpr int kSlots = 3;

struct OdomGPU {
    pf_lidar_params lidar{};
    pf_odom_params prm{};
    int device = 0;
    hipStream_t stream = nullptr;      // stage B: odometry
    hipStream_t stream_a = nullptr;    // stage A: featureExtraction + VoxelGrid
    size_t in_cap = 0, map_cap = 0, sort_cap = 0, pose_cap = 0;
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

    StageBuf sb[kSlots];
    u32* acc_a = nullptr;                                   // stage A min/max accumulators
    u32 *vkeys = nullptr, *vvals = nullptr, *vflags = nullptr, *vscan = nullptr, *vsegstart = nullptr;
    PrimWork vprim;                                         // stage A sort / scan scratch
    hipEvent_t ev_a[kSlots] = {};                           // stage A done with slot p
    hipEvent_t ev_b[kSlots] = {};                           // stage B done with slot p
    hipGraphExec_t graph_a[kSlots] = {};                    // steady-state replay per slot
    hipGraphExec_t graph_b[kSlots] = {};
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
    int* pnext = nullptr;          // [5 * 2 * in_cap] p-index lists: next pair sharing the map point
    int4* pbkt = nullptr;          // [2 * map_cap] p-index buckets {count, pair, pair, overflow head}
    u32* tailinc = nullptr;        // [5 * 2 * in_cap] increments of a map point, on its last pair
    double* lm_part = nullptr;     // [kLmBlocks * 32] per-block LM partials
    u32* lm_ticket = nullptr;      // LM arrival counter
    unsigned long long* dbg = nullptr;   // [64] device timestamps (development probe)
    double* poses = nullptr;       // [pose_cap * 7]
    float4* stage = nullptr;       // [2 * in_cap] host staging target

    bool graph_enabled = true;
};

int odom_create(OdomGPU& o, const pf_lidar_params& lidar, const pf_odom_params& prm, int device, size_t in_cap,
                size_t map_cap);
void odom_destroy(OdomGPU& o);
// stage A: featureExtraction of d_in[0 .. sb[p].cnt[C_NIN]) into slot p
void stage_enqueue_fe(OdomGPU& o, int p, const float4* d_in, hipStream_t s);
// stage A: VoxelGrid of slot p's features (counts sb[p].cnt[C_EIN], [C_SIN])
void stage_enqueue_vg(OdomGPU& o, int p, hipStream_t s);
// stage B: initMapWithPoints from slot p's features
void odom_enqueue_init(OdomGPU& o, int p, hipStream_t s);
// stage B: updatePointsToMap from slot p's down-sampled features; outer iteration count = host mirror
void odom_enqueue_update(OdomGPU& o, int p, hipStream_t s);

}  // namespace pf
