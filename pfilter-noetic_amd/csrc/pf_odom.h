// Device-resident Odom_ES_EstimationClass (src/odomEstimationClass.cpp:182-647) and
// Odom_BPF_EstimationClass (:649-1306): one pipeline over 2 or 3 map classes.
#pragma once
#include "pf_cls.h"
#include "pf_common.h"
#include "pf_fe.h"
#include "pf_knn.h"
#include "pf_prims.h"
#include "pf_tie.h"

namespace pf {

// Map classes. One class = one input cloud, its VoxelGrid leaf, its local map and its residual type.
//   ES  (Odom_ES_EstimationClass):  0 corner (line, leaf r), 1 surf (plane, leaf 2r)
//   BPF (Odom_BPF_EstimationClass): 0 beam (line, r), 1 pillar (line, r), 2 facade (plane, 2r)
// Queries, residuals and maps are concatenated in class order, the reference's factor order.
constexpr int kMaxC = 3;
// p-index bucket of a map point (the valid queries of an outer iteration that have it as a neighbour):
// 16 ints = {pair count, the first kBktInline pair ids, head of the overflow list}, read by k_observe
// in one round of loads (the overflow list only past kBktInline pairs)
#ifndef PF_BKT_QUADS
#define PF_BKT_QUADS 4
#endif
constexpr int kBktQuads = PF_BKT_QUADS;
constexpr int kBktInline = 4 * kBktQuads - 2;
constexpr int kBktHead = 4 * kBktQuads - 1;

// device counter slots (int32, one array per handle); per-class slots are kMaxC consecutive ints
enum CounterSlot {
    C_NIN = 0,                  // raw scan points (featureExtraction input)
    C_IN = 1,                   // [kMaxC] class input clouds (featureExtraction output / caller's clouds)
    C_VGN = C_IN + kMaxC,       // VoxelGrid batch size
    C_DS,                       // [kMaxC] down-sampled clouds (queries of each class)
    C_NQ = C_DS + kMaxC,        // all queries
    C_M,                        // [kMaxC] map sizes
    C_NPAIR = C_M + kMaxC,
    C_NRG, C_NSEG,
    C_NLT,                      // [3] per class bound b = 1, 2, 3: VoxelGrid segments of classes < b (stage A),
                                //     kept map voxels of classes < b (stage B, k_rg_tail)
    C_NRG_VALID = C_NLT + 3,
    C_KEEP_TOTAL,
    C_KEPT,                     // [kMaxC] residual blocks kept (last outer iteration)
    C_VALID = C_KEPT + kMaxC,   // [kMaxC] gated + fitted associations
    C_LM_ITERS = C_VALID + kMaxC,
    C_GATE, C_ERR, C_OUTER, C_FE_ERR, C_COUNT
};

// Sticky device error words of a handle (OdomGPU::errw). Kernels set a word when a bounded wait gave
// up or a capacity was exceeded; it stays set across frames until the host reports it (PF_EHIP for
// E_LM / E_SORT_*, PF_ECAPACITY for the rest) at the next pf_odom_sync / poses / pose read, and
// clears it. The feature, grid, sort and front-end flags of the sub-objects point into this array.
enum ErrWord {
    E_LM = 0,          // LM chunk wait gave up, or a p-index list was corrupt (C_ERR)
    E_FE_SECTOR,       // featureExtraction: a sector above kSecCap points was dropped
    E_GRID,            // map grid above its cell capacity: the frame's kNN saw an empty map
    E_SORT_B,          // stage B sort / scan look-back wait gave up
    E_SORT_A,          // stage A sort / scan look-back wait gave up
    E_FRONT,           // BPF front end: ground grid above its cell limit (CC_ERR)
    E_FRONT_GRID,      // BPF front end: U grid above its cell capacity
    E_MAP,             // a class map above map_cap after rgbds: the voxels past it were dropped
    E_COUNT = 8
};

// ordered-uint accumulator slots (float min/max via atomics)
enum AccSlot {
    A_VG = 0,                   // [class][6]: min xyz, max xyz
    A_RG = 6 * kMaxC,           // [class][6]
    A_W = 12 * kMaxC,           // [class][4]: obs min, obs max, spars min, spars max
    A_COUNT = 16 * kMaxC
};

// the class table every kernel sees: count and which classes are planes (bit c)
struct ClassCfg {
    int nc;
    u32 plane;
    __host__ __device__ __forceinline__ bool is_plane(int c) const { return (plane >> c) & 1u; }
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
    double wmin[kMaxC][2], wmax[kMaxC][2];   // [class][observe, sparsity]
    int iteration, invalid, reuse, done, phase, n_res, pad0, pad1;
};

constexpr int kDbgWords = 8192;   // development probe buffer (PF_PROBE): LM [0, 64), rgbds buckets after
constexpr int kLmParts = 31;   // cost, g[6], H[21], bad_r, bad_J, kept rows
constexpr int kLmEvalSlots = 8; // LM claim masks per solve (>= evaluations per solve)
constexpr int kLmEvals = 5;      // evaluations per solve: 1 + max_num_iterations (4)
constexpr int kLmBlocks = 32;    // LM workgroups = residual chunks per evaluation
constexpr int kLmBlkProbe = kDbgWords - 512;   // PF_PROBE: per-workgroup LM timestamps from here
// an LM partial not yet published (a NaN payload no arithmetic produces); k_assoc writes it over
// every partial slot before each solve
constexpr unsigned long long kPartSentinel = 0x7FF4C0DE5E47F00Dull;

// One slot of the two-stage frame pipeline: a frame's features and their voxel-grid output, with
// the counters of that stage. Stage A (stream_a: featureExtraction + VoxelGrid, pose independent)
// fills slot k % 2 while stage B (stream: the odometry) still works on frame k - 1 in the other slot.
struct StageBuf {
    float4* in[kMaxC] = {};      // class inputs (featureExtraction output or the caller's clouds)
    float4* ds[kMaxC] = {};      // VoxelGrid output (r, g written by the odometry)
    int* cnt = nullptr;          // [C_COUNT] stage counters
};

// pipeline slots: frame k's stage A output lives in slot k % kSlots, so stage A may run up to
// kSlots - 1 frames ahead of stage B
constexpr int kSlots = 3;

// What the host reads back after a call that reports a pose (read_pose): the counters, the sticky
// error words, the latest pose and the estimator state, gathered by one kernel into mapped pinned
// host memory, so a frame's report costs one stream synchronisation.
struct HostRead {
    int cnt[C_COUNT];
    int err[E_COUNT];
    double pose[7];
    DevState st;
};

// Host-input staging (pf_odom_frame_host / update / init_map): per pipeline slot a pinned host buffer
// (the repacked caller clouds) and a device buffer the copy stream fills by DMA; stage A's stream
// waits for the slot's copy event instead of the host waiting for the copy.
struct HostStage {
    hipStream_t stream = nullptr;          // copy stream (H2D)
    float4* h[kSlots] = {};                // pinned, kMaxC * in_cap points each
    float4* d[kSlots] = {};                // device, kMaxC * in_cap points each
    hipEvent_t ev[kSlots] = {};            // slot's copy done
};

struct OdomGPU {
    pf_lidar_params lidar{};
    pf_odom_params prm{};
    int device = 0;
    hipStream_t stream = nullptr;      // stage B: odometry
    hipStream_t stream_a = nullptr;    // stage A: featureExtraction + VoxelGrid
    // stage B's side stream (development switch pf_dev_set_tie_aux / PF_TIE_AUX=1, off by default): the
    // rgbds tie sort heap-sorts its partition tiers' depth-limit segments there beside k_tie_local
    // (TieAux, pf_tie.h). Measured on the headline: 844.9 frames/s on against 844.7 off -- the heap
    // workgroups need a whole CU's LDS and wait for k_tie_local's to drain -- and the stage-B timing
    // events then miss the side stream's work, so it stays off
    hipStream_t stream_bx = nullptr;
    hipEvent_t ev_bx_fork = nullptr, ev_bx_join = nullptr;
    bool tie_aux = false;
    // the radix route of a sort with big levels (configs[4]'s ~820k-key depth-limit segment) on stream_bx
    // beside the partition tiers (TieAux::hs); PF_TIE_HS=0 keeps it on stage B's stream (A/B checks)
    bool tie_hs = true;
    size_t in_cap = 0, map_cap = 0, sort_cap = 0, pose_cap = 0;
    int opt_count_host = 2;
    bool inited = false;
    int frames = 0;
    ClassCfg cls{2, 2u};
    float leaf_vg[kMaxC] = {};     // downSizeFilter leaves (double -> float)
    float leaf_rg[kMaxC] = {};     // rgbds leaves: map_resolution, map_resolution * 2 (float)

    FeGPU fe;
    GridGPU grid;
    PrimWork prim;

    DevState* st = nullptr;
    LMState* lm = nullptr;
    int* cnt = nullptr;
    u32* acc = nullptr;
    int* errw = nullptr;           // [E_COUNT] sticky error words (ErrWord)
    int err_seen = 0;              // bits of the words reported since create / reset (pf_odom_stats)
    int err_last[E_COUNT] = {};    // values of the words at their last report (pf_dev_errors)
    int* h_cnt = nullptr;          // pinned mirror
    double* h_pose = nullptr;      // pinned [7]
    HostRead* h_rd = nullptr;      // mapped pinned (read_pose)
    HostRead* h_rd_dev = nullptr;  // its device-side address
    int rd_frames = -1;            // `frames` at the last read_pose (-1: the cached state is stale)
    HostStage* hs = nullptr;       // host-input staging, allocated by the first host-input call
    // map export (pf_odom_set_map_export): after every update the maps are written straight into
    // mapped pinned host memory by k_map_export (device-resident sizes, no host round trip)
    bool export_maps = false;
    float4* h_map[kMaxC] = {};     // pinned, map_cap points each
    float4* h_map_dev[kMaxC] = {}; // their device-side addresses
    int* h_map_n = nullptr;        // pinned [kMaxC] sizes written with them
    int* h_map_n_dev = nullptr;

    StageBuf sb[kSlots];
    u32* acc_a = nullptr;                                   // stage A min/max accumulators
    u32 *vkeys = nullptr, *vvals = nullptr, *vflags = nullptr, *vscan = nullptr, *vsegstart = nullptr;
    PrimWork vprim;                                         // stage A sort / scan scratch
    hipEvent_t ev_a[kSlots] = {};                           // stage A done with slot p
    hipEvent_t ev_b[kSlots] = {};                           // stage B done with slot p
    hipGraphExec_t graph_a[kSlots] = {};                    // steady-state replay per slot
    hipGraphExec_t graph_b[2 * kSlots] = {};                // [slot + kSlots * mpar]
    ClsGPU* front = nullptr;                                // BPF raw-scan mode: the PCA front end
    hipGraphExec_t graph_as[kSlots] = {};                   // stage A replay in raw-scan mode
    // BPF raw-scan mode with two front-end lanes (pf_bpf_set_front_lanes; the default for a handle alone
    // on the host, as PF_GRAPH_AUTO: several handles' lanes oversubscribe the hardware queues): the front end of
    // frame k runs on stream_f[k & 1] with that lane's own instance (front / front2) and scan staging
    // (stage / stage2), so the front ends of consecutive frames overlap; VoxelGrid then runs on
    // stream_a in frame order once the frame's front end is done (ev_f). Allocated by the first
    // raw-scan frame. Lane 1's DCVC starts as "called before" (pf_dcvc.h dcvc_mark_called): the
    // reference's first-call defaults belong to frame 0 only, which lane 0 runs.
#ifndef PF_FRONT_LANES_DEFAULT
#define PF_FRONT_LANES_DEFAULT 0
#endif
    int front_lanes = PF_FRONT_LANES_DEFAULT;   // 1, 2, or 0 = auto: 2 while it is the process's only raw-scan handle
    int lanes_used = 0;                         // the lane count of the last raw-scan frame (0: none yet)
    bool dcvc_first = false;                    // no curvedfilter frame since DCVC was enabled / reset: the
                                                // next one starts the reference's single instance (first call)
    ClsGPU* front2 = nullptr;
    float4* stage2 = nullptr;                               // [kMaxC * in_cap]
    hipStream_t stream_f[2] = {};
    hipEvent_t ev_f[kSlots] = {};                           // frame in slot p: front end done
    hipGraphExec_t graph_f[2 * kSlots] = {};                // [slot + kSlots * lane] front-end replay
    // local maps, double-buffered: an update reads mapset[mpar] and writes the new maps into
    // mapset[mpar ^ 1] (rgbds cannot overwrite the map it is still reading), then the host flips mpar
    // (odom_update_done); graph B is captured per (slot, mpar)
    float4* mapset[2][kMaxC] = {};
    int mpar = 0;
    // the map grid's dims of map_cur() were computed by the update that wrote it (k_rgm_finish), so
    // the next update's grid build skips its bounds pass; false after any other map write
    bool dims_fresh = false;
    bool no_fuse_obs = false;      // development (pf_dev_set_fuse_observe): k_observe even at weightType 0
    float4* app[kMaxC] = {};       // this frame's transformed down-sampled points (appended)
    float4* seg_out = nullptr;
    u32 *keys = nullptr, *vals = nullptr;
    u64* tail_status = nullptr;   // k_rg_tail look-back words [tail_tiles] + arrival counter
    size_t tail_tiles = 0;
    // rgbds by merge (k_rgm_bucket / k_rgm_finish, the default order): the map is kept
    // in voxel order, so only this frame's appended points are sorted and then merged into it
    u64* rgm_okey = nullptr;       // [nc * map_cap] voxel keys of the map points, map order
    u64* rgm_key64 = nullptr;      // [sort_cap] voxel keys of every element, element order
    u32* rgm_vtag = nullptr;       // [sort_cap] element index | cropped << 31
    u32* rgm_bcount = nullptr;     // [kRgmBuckets] appended points per bucket (lists built by the LM)
    int* rgm_bmeta = nullptr;      // [kRgmBuckets][32] each bucket's merged base, length, kept voxels and
                                   // kept-voxel cell bounds per class
    int* dims_next = nullptr;      // [8 * kGridMaps + 1] the map grid dims and scan length of map_next(),
                                   // written by k_rgm_finish (copied into the grid by the next build)
    u64* rgm_bkey = nullptr;       // [kRgmBuckets * kRgmBucketCap] the lists: keys, tags
    u32* rgm_btag = nullptr;
    float4* rgm_vox = nullptr;     // [sort_cap] voxel outputs at merged positions
    u32* rgm_kflag = nullptr;      // [sort_cap] kept flags / ranks at merged positions
    u64* rgm_kout = nullptr;       // [sort_cap] fallback: sorted keys (vals: `vals`)
    u64* rgm_ktmp = nullptr;       // [sort_cap] fallback sort scratch
    u32* rgm_vtmp = nullptr;
    int* rgm_stat = nullptr;       // [8]: fallback this frame, fallbacks so far, largest append, spare,
                                   // kept voxels per class (accumulated over the buckets)

    int* nbr = nullptr;            // [5 * kMaxC * in_cap]
    int* qflag = nullptr;          // bit0 valid association, bit1 kept
    double* geo = nullptr;         // [8 * kMaxC * in_cap]
    float* spars = nullptr;
    float* roundv = nullptr;
    float* observe = nullptr;
    int* pnext = nullptr;          // [5 * kMaxC * in_cap] p-index lists: next pair sharing the map point
    int4* pbkt = nullptr;          // [nc * map_cap][kBktQuads] p-index buckets {count, kBktInline pairs, overflow head}
    u32* tailinc = nullptr;        // [5 * kMaxC * in_cap] increments of a map point, on its last pair
    double* lm_part = nullptr;     // [kLmBlocks * 32] per-block LM partials
    u32* lm_ticket = nullptr;      // LM arrival counter
    unsigned long long* dbg = nullptr;   // [64] device timestamps (development probe)
    double* poses = nullptr;       // [pose_cap * 7]
    float4* stage = nullptr;       // [kMaxC * in_cap] staging target of the frame entry points

    int graph_mode = PF_GRAPH_AUTO;      // pf_odom_set_graph
    int cu_reserve = 0;            // CUs stage A stays off (odom_stage_a_stream)
    // reference tie order (pf_odom_set_tie_order, pf_tie.h): VoxelGrid (stage A) and rgbds (stage B)
    // order equal keys as libstdc++'s std::sort does; each stage has its own scratch
    bool tie_order = false;
    bool rg_radix = false;         // development: rgbds by the full radix sort instead of the merge
    TieSort* tie_a = nullptr;
    TieSort* tie_b = nullptr;
    size_t tie_hint = 0;                        // largest class an rgbds tie sort may see (pf_odom_set_map)
    // rgbds voxel groups whose f32 centroid does not depend on the order of their points (pf_odom.hip
    // k_rg_dep): an open-addressing table key -> {count, first three elements}, empty between updates
    u32* dep_key = nullptr;        // [dep_h] voxel key, 0xFFFFFFFF = empty
    u32* dep_cnt = nullptr;        // [dep_h] elements with that key
    u32* dep_mem = nullptr;        // [3 * dep_h] the first three elements
    u32* dep_slot = nullptr;       // [sort_cap] each element's slot (0xFFFFFFFF: cropped)
    u8* dep_free = nullptr;        // [sort_cap] 1 = the element's group is order-free
    u32 dep_hbits = 0;             // dep_h = 1 << dep_hbits
    bool dep_force_full = false;   // pf_dev_set_dep_full
    u32* dep_dirty = nullptr;      // [2] the map may hold two points of a voxel / k_rg_tail's verdict (DepTab)
};
// the dependence table of the tie-order rgbds (allocated with the tie sorts, pf_odom_set_tie_order)
int odom_dep_alloc(OdomGPU& o);
void odom_dep_release(OdomGPU& o);                 // frees the table (also after a failed alloc)
void odom_dep_dirty(OdomGPU& o, hipStream_t s);   // the maps were written by the host or initMapWithPoints

// Stage A keeps off the last CUs of the device by default: with one sequence per GPU, stage B's LM
// (kLmBlocks co-resident workgroups) otherwise waits for stage A's waves to drain. Measured on one
// MI355X: ES 3.09k -> 3.24k frames/s at 128 CUs reserved (a cliff past 192); the BPF
// raw-scan chain 1.25k -> 1.79k at 32 (its front end needs the CUs); several concurrent sequences
// per GPU lose with any reservation (pf_odom_set_stage_a_reserve(h, 0)).
constexpr int kStageAReserveES = 128;
constexpr int kStageAReserveBPF = 32;
int odom_stage_a_stream(OdomGPU& o, int reserve);
// a stream restricted to all but the last `reserve` CUs (0: unrestricted, non-blocking)
int odom_masked_stream(int device, int reserve, hipStream_t* out);
// waits for everything enqueued on stage A's streams (the front-end lanes and stream_a)
hipError_t odom_sync_a(OdomGPU& o);

// nc = 2: the ES estimator; nc = 3: the BPF estimator (the last class is the plane class)
int odom_create(OdomGPU& o, const pf_lidar_params& lidar, const pf_odom_params& prm, int device, size_t in_cap,
                size_t map_cap, int nc = 2);
void odom_destroy(OdomGPU& o);
int odom_reset(OdomGPU& o);
// point a sub-object's error flag at a sticky error word (frees the flag's own allocation)
void alias_err(int*& flag, int* word);
// stage A: featureExtraction of d_in[0 .. sb[p].cnt[C_NIN]) into slot p's classes 0 / 1 (ES)
void stage_enqueue_fe(OdomGPU& o, int p, const float4* d_in, hipStream_t s);
// stage A: VoxelGrid of slot p's class clouds (counts sb[p].cnt[C_IN + c])
void stage_enqueue_vg(OdomGPU& o, int p, hipStream_t s);
// stage B: initMapWithPoints from slot p's features
void odom_enqueue_init(OdomGPU& o, int p, hipStream_t s);
// stage B: updatePointsToMap from slot p's down-sampled features; outer iteration count = host mirror
void odom_enqueue_update(OdomGPU& o, int p, hipStream_t s);
// after an update has been enqueued (or its graph launched): the maps it wrote become the current ones
inline void odom_update_done(OdomGPU& o) { o.mpar ^= 1; }
inline bool odom_merge_mode(const OdomGPU& o) { return !o.tie_order && !o.rg_radix; }
inline float4* const* map_cur(const OdomGPU& o) { return o.mapset[o.mpar]; }
inline float4* const* map_next(const OdomGPU& o) { return o.mapset[o.mpar ^ 1]; }
// stage B tail when map export is on: the maps and their sizes into the mapped pinned buffers
// the maps into the mapped pinned export buffers: after_update, the maps the update just wrote
// (enqueued before odom_update_done), else the current ones
void odom_enqueue_export(OdomGPU& o, hipStream_t s, bool after_update);
// k_assoc's kNN alone, `iters` times, on the last frame's queries and grid (pf_odom_probe_assoc)
int odom_probe_assoc(OdomGPU& o, int iters, double* avg_ms, double* alg_bytes, int* nq, float4* q_host, size_t q_cap);

}  // namespace pf
