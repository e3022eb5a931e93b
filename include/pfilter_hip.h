/* pfilter_hip — C ABI of the MI355X-native PFilter/FLOAM odometry hot path.
 *
 * One handle = one HIP stream = one caller thread (the reference classes are used by exactly one
 * worker thread each: src/odomEstimationNode copy.cpp:54-148, src/laserProcessingNode.cpp:53-106).
 * Handles on different devices are independent; that is the per-sequence multi-GPU model.
 * Every entry point returns a status code and never throws across the ABI.
 *
 * Reference interfaces replaced (the C++ drop-in shims in pfilter-noetic_amd/shim/ map 1:1):
 *   pf_fe_create/pf_fe_extract     LaserProcessingClass::init / featureExtraction
 *                                  (include/laserProcessingClass.h:36-37, src/laserProcessingClass.cpp:10-96)
 *   pf_odom_create                 Odom_ES_EstimationClass::init (include/odomEstimationClass.h:146,
 *                                  src/odomEstimationClass.cpp:182-208)
 *   pf_odom_init_map               Odom_ES_EstimationClass::initMapWithPoints (.h:148, .cpp:217-222)
 *   pf_odom_update                 Odom_ES_EstimationClass::updatePointsToMap (.h:149, .cpp:229-282)
 *   pf_odom_get_pose               public member `odom` as read by the node (copy.cpp:105-107)
 *   pf_odom_get_map                public members laserCloudCornerMap / laserCloudSurfMap (.h:151-152)
 *                                  and getMap (.h:147, .cpp:210-215)
 *   pf_bpf_create                  Odom_BPF_EstimationClass::init (.h:175, .cpp:649-681)
 *   pf_bpf_init_map                Odom_BPF_EstimationClass::initMapWithPoints (.h:177, .cpp:685-691)
 *   pf_bpf_update                  Odom_BPF_EstimationClass::updatePointsToMap (.h:178, .cpp:702-749)
 *   pf_odom_get_map (BPF handle)   laserCloudBeamMap / PillarMap / FacadeMap (.h:180-182), getMap (.cpp:683)
 *   pf_map_create / update / get   LaserMappingClass::init / updateCurrentPointsToMap / getMap
 *                                  (include/laserMappingClass.h:27-29, src/laserMappingClass.cpp:7-206)
 *   pf_cls_create / pf_cls_extract groundSeg::ground_seg + nongroundExtract::featureExtract, the BPF
 *                                  front end of src/additionNode.cpp:21-45 (include/preProcess.hpp:
 *                                  398-505, 646-689)
 */
#ifndef PFILTER_HIP_H
#define PFILTER_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: 0 ok, > 0 warnings (execution continued, as the reference prints and continues),
 * < 0 errors */
#define PF_OK 0
#define PF_W_MAP_TOO_SMALL 1     /* "not enough points in map to associate" (.cpp:274-277) */
#define PF_W_FEW_CORRESPONDENCES 2 /* "not enough correct points" (.cpp:428-431, 574-577) */
#define PF_EINVAL (-1)           /* bad argument, e.g. weight_type not in {0,1,2,12} (reference: UB) */
#define PF_EHIP (-2)             /* HIP runtime error */
#define PF_ENOMEM (-3)           /* device allocation failed */
#define PF_ECAPACITY (-4)        /* input or map larger than the handle's capacity */
#define PF_EUNSUPPORTED (-5)     /* configuration outside the implemented path */

typedef struct {                 /* lidar::Lidar fields read on the path (include/lidar.h:9-30) */
    int num_lines;               /* 16, 32 or 64 (others: every point in ring 0, as the reference) */
    double min_dist;
    double max_dist;
    double scan_period;
} pf_lidar_params;

typedef struct {                 /* Odom_ES_EstimationClass::init arguments */
    double map_res;              /* map_resolution (edge leaf; surf leaf = 2x) */
    int k_new;
    float theta_p;
    int theta_max;
    int weight_type;             /* 0 none, 1 observe, 2 sparsity, 12 both */
} pf_odom_params;

typedef struct {
    int64_t n_edge_in, n_surf_in;        /* E, S */
    int64_t n_edge_ds, n_surf_ds;        /* E', S' after VoxelGrid */
    int64_t n_edge_map, n_surf_map;      /* map sizes after the update */
    int64_t n_edge_res, n_surf_res;      /* residual blocks in the last outer iteration */
    int64_t n_edge_valid, n_surf_valid;  /* gated + fitted associations, last outer iteration */
    int32_t outer_iterations;
    int32_t lm_iterations;               /* summed over outer iterations */
    int32_t map_too_small;
    int32_t status;
    /* per map class (ES: 0 edge, 1 surf; BPF: 0 beam, 1 pillar, 2 facade); the n_edge_* / n_surf_*
     * fields above repeat classes 0 and 1 */
    int64_t n_in[3], n_ds[3], n_map[3], n_res[3], n_valid[3];
    /* sticky device error words seen since create / reset (bit k set = word k was raised):
     * 0 LM chunk wait gave up or corrupt p-index list, 1 featureExtraction sector above 4096 points
     * dropped, 2 map grid above its cell capacity, 3 / 4 stage B / A sort look-back wait gave up,
     * 5 BPF front end ground grid above its cell limit, 6 front end 1 m grid above its capacity */
    int32_t errors;
    int32_t pad_;
} pf_odom_stats;

/* ---------------- feature extraction (LaserProcessingClass) ---------------- */
typedef struct pf_fe pf_fe;
int pf_fe_create(const pf_lidar_params* lidar, int device, size_t max_points, pf_fe** out);
int pf_fe_destroy(pf_fe* h);
/* xyzi: n points, x,y,z at byte offsets 0,4,8 and intensity at 16 (PCL PointXYZI) or 12 (packed)
 * selected by stride_bytes (32 = PCL layout, 16 = packed float4). Outputs are packed float4
 * (x, y, z, intensity), bit-identical copies of input points in reference order
 * (ring -> sector -> edges by descending curvature / surfs ascending). `cap` is the capacity of
 * each output in points. */
int pf_fe_extract(pf_fe* h, const float* xyzi, size_t n, size_t stride_bytes, float* edge_out,
                  size_t* n_edge, float* surf_out, size_t* n_surf, size_t cap);
/* EXTENSION (not in the reference): a linear beam model for line counts the reference has no ring
 * formula for (src/laserProcessingClass.cpp:58-61 puts every point of such a scan into ring 0):
 * ring = int((top_deg - elevation_deg) * num_lines / (top_deg - bottom_deg)), points outside
 * [0, num_lines) dropped. SURVEY 8(d) config 5 (synthetic 128-line scans, -25..+15 deg) runs with it.
 * top_deg == bottom_deg == 0 restores the reference's formulas (the default). */
int pf_fe_set_ring_model(pf_fe* h, double top_deg, double bottom_deg);
/* Reference tie order (default ON since round 5): a sector whose curvature list holds equal values is
 * ordered as libstdc++'s std::sort leaves it (src/laserProcessingClass.cpp:101-104 sorts by value alone,
 * and the surf cloud is written in that order); 0 orders it by (value, ring position) instead. Sectors
 * without an exact tie are identical either way. pf_odom_set_tie_order switches the handle's
 * featureExtraction too. */
int pf_fe_set_tie_order(pf_fe* h, int enable);

/* ---------------- odometry (Odom_ES_EstimationClass) ---------------- */
typedef struct pf_odom pf_odom;
/* max_points: largest raw scan / edge / surf input; map_capacity: largest local map (per map).
 * Any number of handles may share a device (bounded by device memory): no kernel of the pipeline
 * depends on its workgroups being co-resident with each other or with other handles' kernels.
 *
 * Device memory per handle grows with map_capacity, about 280 B per map point per class (nc = 2 map
 * classes for ES, 3 for BPF): the p-index buckets take 64 B (pf_odom.h kBktQuads), the two map sets
 * 32 B, the map update's keys, sort buffers and voxel staging about 84 B, and the reference tie order's
 * sort structures (working copy, rank lists, heap scratch, radix route) and its dependence table the
 * rest (pf_odom.hip odom_create, pf_tie.hip tie_alloc, odom_dep_alloc). Measured (tools/mem_probe.py,
 * round 6): 3.2 GiB (ES) / 4.6 GiB (BPF) per handle at the defaults (max_points 300000, map_capacity
 * 1 << 22), 1.2 GiB for ES at map_capacity 1 << 18 (the per-scan buffers, which scale with max_points,
 * dominate there). bench.py's configs[3] runs 4 handles per GPU (about 13 GiB of the 288 GiB), the
 * 12-handle concurrency test about 39 GiB. Size map_capacity to the largest expected local map when
 * many handles share a device.
 *
 * Device-side failures (a bounded wait that gave up, a featureExtraction sector above 4096 points,
 * a map grid or front-end grid above capacity) latch sticky error words on the device. They are
 * reported once, at the next call that waits for the handle's work (pf_odom_sync, pf_odom_poses,
 * a frame / update call with pose_out, pf_odom_get_pose): PF_EHIP for a wait that gave up,
 * PF_ECAPACITY for a capacity overflow (the outputs of those calls are still written).
 * pf_odom_get_stats reports the words seen since create / reset in `errors`. */
int pf_odom_create(const pf_lidar_params* lidar, const pf_odom_params* params, int device,
                   size_t max_points, size_t map_capacity, pf_odom** out);
int pf_odom_destroy(pf_odom* h);
/* back to the state right after create/init (identity pose, empty maps; the next frame or init_map
 * seeds the maps), keeping allocations and captured graphs: the next sequence on the same handle */
int pf_odom_reset(pf_odom* h);
/* edge/surf: points with x,y,z at offsets 0,4,8 and the given stride (16 packed, 32 PCL). */
int pf_odom_init_map(pf_odom* h, const float* edge, size_t ne, size_t edge_stride, const float* surf,
                     size_t ns, size_t surf_stride);
int pf_odom_update(pf_odom* h, const float* edge, size_t ne, size_t edge_stride, const float* surf,
                   size_t ns, size_t surf_stride, double pose_out[7]);
/* pose = {qx, qy, qz, qw, tx, ty, tz} of `odom` (q = Quaterniond(odom.rotation())) */
int pf_odom_get_pose(pf_odom* h, double pose[7]);
/* which: the map class. ES: 0 = edge (corner) map, 1 = surf map; BPF: 0 beam, 1 pillar, 2 facade.
 * xyz 3 floats/pt, rg 2 bytes/pt (r=age, g=p-index).
 * Either output may be NULL; with cap too small *n is set and PF_ECAPACITY returned. */
int pf_odom_get_map(pf_odom* h, int which, float* xyz, uint8_t* rg, size_t cap, size_t* n);
int pf_odom_set_map(pf_odom* h, int which, const float* xyz, const uint8_t* rg, size_t n);
int pf_odom_get_stats(pf_odom* h, pf_odom_stats* s);

/* ---------------- odometry (Odom_BPF_EstimationClass) ----------------
 * The estimator the fork's built node runs (src/odomEstimationNode.cpp:191-331): three local maps,
 * beam and pillar (line residuals, leaf map_res) and facade (plane residuals, leaf 2 map_res), from
 * the classified clouds of the feature classifier. Residual order beam -> pillar -> facade (.cpp:733-735).
 * The handle type is pf_odom; pf_odom_get_pose / get_map / set_map / get_stats / poses / sync /
 * set_graph / destroy apply, the ES-only entry points return PF_EINVAL on a BPF handle and back. */
int pf_bpf_create(const pf_lidar_params* lidar, const pf_odom_params* params, int device,
                  size_t max_points, size_t map_capacity, pf_odom** out);
int pf_bpf_init_map(pf_odom* h, const float* beam, size_t nb, size_t beam_stride, const float* pillar,
                    size_t np, size_t pillar_stride, const float* facade, size_t nf, size_t facade_stride);
int pf_bpf_update(pf_odom* h, const float* beam, size_t nb, size_t beam_stride, const float* pillar,
                  size_t np, size_t pillar_stride, const float* facade, size_t nf, size_t facade_stride,
                  double pose_out[7]);
/* HBM-resident clouds (packed float4 device pointers): the first call seeds the maps, later calls
 * run updatePointsToMap; pose_out may be NULL (enqueue only), as pf_odom_frame_device */
int pf_bpf_frame_device(pf_odom* h, const float* d_beam, size_t nb, const float* d_pillar, size_t np,
                        const float* d_facade, size_t nf, double pose_out[7]);
/* number of map classes of a handle: 2 (ES) or 3 (BPF) */
int pf_odom_classes(pf_odom* h);

/* ---------------- BPF front end (groundSeg + nongroundExtract, src/additionNode.cpp:21-45) ----------------
 * ground_seg (include/preProcess.hpp:398-505): 2-D grid of gf_grid_res cells over the scan's x/y
 * bounds; per cell the lowest z in (gf_min_ground_height, gf_max_ground_height], the 3x3 neighbourhood
 * minimum, and the ground / non-ground split. featureExtract (:646-689): per non-ground point the
 * <= k nearest non-ground points with d^2 < radius^2, their PCA, and the pillar / beam / facade
 * decision. The DCVC `curvedfilter` stage the KITTI launch file inserts between them
 * (pfilter_kitti.launch:8) is enabled per handle with pf_cls_set_dcvc / pf_bpf_set_dcvc (below);
 * with it off the non-ground cloud feeds featureExtract directly. */
typedef struct {
    int ground_filter;                 /* additionNode `groundfilter` (pfilter_kitti.launch:10) */
    int gf_min_grid_pts;               /* gf_grid_pt_num_thre (preProcess.hpp:575) */
    float gf_grid_res, gf_max_height_diff, gf_neighbor_height_diff, gf_max_ground_height,
          gf_min_ground_height;        /* :601-605 (double members passed as float, :398-401) */
    float radius;                      /* neighbor_searching_radius (:703); must be <= 1 */
    int k, k_min;                      /* neighbor_k (:705; 1..32), neigh_k_min (:706) */
    float edge_thre, planar_thre, linear_vsin_high, linear_vsin_low, planar_vsin_low,
          beam_h_max, beam_h_min;      /* :708-715 */
} pf_cls_params;
typedef struct pf_cls pf_cls;
void pf_cls_default_params(pf_cls_params* p);   /* the reference's member defaults */
int pf_cls_create(const pf_cls_params* p, int device, size_t max_points, pf_cls** out);
int pf_cls_destroy(pf_cls* h);
/* One scan (x, y, z floats at the start of each stride-byte record). Outputs are indices into the
 * scan, in the order the reference publishes the clouds: beam / pillar / facade (cloud_beam /
 * cloud_pillar / cloud_facade, :660-684) and ground (cloud_ground, :480). Any output pair may be NULL;
 * each list holds at most cap entries (PF_ECAPACITY with the counts set when one does not fit). */
int pf_cls_extract(pf_cls* h, const float* xyz, size_t n, size_t stride_bytes, int32_t* beam, size_t* nb,
                   int32_t* pillar, size_t* np, int32_t* facade, size_t* nf, int32_t* ground, size_t* ng,
                   size_t cap);
/* ground_seg alone (:398-505): ground and non-ground input indices in the reference's push order */
int pf_cls_ground_seg(pf_cls* h, const float* xyz, size_t n, size_t stride_bytes, int32_t* ground, size_t* ng,
                      int32_t* unground, size_t* nu, size_t cap);
/* featureExtract alone on a cloud (no ground segmentation): per point the index_with_feature code
 * (0 none, 1 pillar, 2 beam, 3 facade, :663-682) and the neighbour count pt_num (:223); either may
 * be NULL */
int pf_cls_classify(pf_cls* h, const float* xyz, size_t n, size_t stride_bytes, uint8_t* cls, int32_t* pt_num);
/* The normals assign_normal (include/preProcess.hpp:327-346) leaves in the points, 4 floats per point:
 * (principal direction, linear_2) for pillar and beam points (featureExtract, :663-674); (normal
 * direction, planar_2) for every other point with more than 3 neighbours (get_pc_pca_feature,
 * :238-239); zeros with 0-3 neighbours (the zero-initialised feature; the reference leaves points with
 * 0-1 neighbours untouched, which the C++ shim does too, using the pt_num counts). Per point of the last
 * pf_cls_classify call (input order) or, after pf_cls_extract, per non-ground point in ground_seg's
 * push order. n = the number of points wanted (at most that call's point count). */
int pf_cls_normals(pf_cls* h, float* normal4, size_t n);

/* ---------------- curvedVoxel (DCVC, src/additionClass.cpp:1-497) ----------------
 * Polar (range, pitch, azimuth) voxels with range rings growing by start_r - k * delta_r, the 27-voxel
 * neighbourhood of searchKNN (:196-225, its azimuth wrap and pitch-layer quirks kept), clusters of
 * neighbouring occupied voxels, and the points of clusters larger than min_seg, cluster by cluster by
 * size (ties: first point), each in input order (pointCloudSegPtr, :360-372). The reference's loops
 * race under OpenMP; the device computes the connected components of the voxel neighbourhood (DESIGN.md
 * §2 gives the statistical bar against the serial reading). The first call of a handle starts the
 * range rings at 5 m (the member default, include/additionClass.hpp:105), later calls at 0. */
typedef struct {
    double start_r, delta_r, delta_p, delta_a;   /* config/config.yaml:50-53 (1, 0.003, 1.2, 1.2) */
    int min_seg;                                 /* :54 (80) */
    double min_range, max_range;                 /* velodyne sensorMinRange / sensorMaxRange (1, 120) */
} pf_dcvc_params;
typedef struct pf_dcvc pf_dcvc;
void pf_dcvc_default_params(pf_dcvc_params* p);
int pf_dcvc_create(const pf_dcvc_params* p, int device, size_t max_points, pf_dcvc** out);
int pf_dcvc_destroy(pf_dcvc* h);
/* curvedVoxel::run on one cloud (x, y, z floats at the start of each stride-byte record): the kept
 * points as input indices in the published order (out_idx, cap entries; *n_out = their count) and
 * per point its cluster's rank (1 = largest) or 0 (dropped); out_idx / label may be NULL. */
int pf_dcvc_run(pf_dcvc* h, const float* xyz, size_t n, size_t stride_bytes, int32_t* out_idx, size_t* n_out,
                int32_t* label, size_t cap);
/* the next call is a first call again (a new sequence) */
int pf_dcvc_reset(pf_dcvc* h);
/* grows the point capacity to max_points (no-op when already that large), keeping the call state: a
 * run after it is still a later call (curvedVoxel's members persist across scans) */
int pf_dcvc_reserve(pf_dcvc* h, size_t max_points);
/* curvedfilter in the front end: DCVC runs on the non-ground cloud and featureExtract on its output
 * (src/additionNode.cpp:29-39); p NULL turns it off (the default) */
int pf_cls_set_dcvc(pf_cls* h, const pf_dcvc_params* p);

/* BPF whole-frame mode: one raw scan (device pointer to n packed float4) per call; stage A runs the
 * front end above (ground_seg + featureExtract) into the beam / pillar / facade clouds, then the
 * VoxelGrid, stage B the odometry (the additionNode -> odomEstimationNode chain without ROS).
 * set_front_end fixes the front end's parameters (default: pf_cls_default_params); n <= the handle's
 * max_points. pose_out may be NULL (enqueue only), as pf_odom_frame_device; with pose_out the call
 * also reports PF_ECAPACITY when the front end's grids exceeded their limits (the frame then ran with
 * empty class clouds: a ground grid above 32,766 cells of gf_grid_res, or a 1 m grid above 2^23 cells). */
int pf_bpf_set_front_end(pf_odom* h, const pf_cls_params* p);
/* curvedfilter in the raw-scan BPF pipeline (the KITTI launch's default); p NULL turns it off */
int pf_bpf_set_dcvc(pf_odom* h, const pf_dcvc_params* p);
int pf_bpf_frame_scan_device(pf_odom* h, const float* d_xyzi, size_t n, double pose_out[7]);
/* EXTENSION (not in the reference): front-end lanes of the raw-scan mode. 2: the front ends of
 * consecutive frames run on two streams with one front-end instance each (about 2x the front end's
 * device memory), overlapping frame k + 1's front end with frame k's; VoxelGrid and the odometry still
 * run in frame order. 1: one front end, in line with VoxelGrid. 0 (the default): 2 while the handle is
 * the process's only handle with a raw-scan front end, else 1 (several such handles' lanes
 * oversubscribe the GPU's hardware queues).
 * Results are identical in every mode. */
int pf_bpf_set_front_lanes(pf_odom* h, int lanes);

/* ---------------- global map (LaserMappingClass, src/laserMappingClass.cpp) ----------------
 * The map of src/laserMappingNode.cpp: 50 m cubes; every update transforms the scan into the world
 * frame (pose = qx, qy, qz, qw, tx, ty, tz, the odometry message), appends it to its cubes and
 * VoxelGrid-filters the 5 x 5 x 5 cubes around the pose. max_points bounds the map, max_scan a scan.
 * update returns PF_EINVAL when a point falls into a cube the reference never allocated (it
 * dereferences a null cloud there, :171) or lies beyond +-25 km; the map is then unchanged.
 * pf_map_get: x, y, z, intensity of the whole map in getMap's cube order (xyzi may be NULL). */
typedef struct pf_map pf_map;
int pf_map_create(double map_resolution, int device, size_t max_points, size_t max_scan, pf_map** out); /* init :7-33 */
int pf_map_destroy(pf_map* h);
int pf_map_update(pf_map* h, const float* xyzi, size_t n, size_t stride_bytes, const double pose[7]); /* :151-189 */
int pf_map_update_device(pf_map* h, const float* d_xyzi, size_t n, const double pose[7]);
/* the same with the pose as the Isometry3d itself: row-major [R | t], 12 doubles (the C++ shim) */
int pf_map_update_mat(pf_map* h, const float* xyzi, size_t n, size_t stride_bytes, const double T[12]);
int pf_map_get(pf_map* h, float* xyzi, size_t cap, size_t* n);                                   /* getMap :194-206 */

/* ---------------- whole-frame device pipeline (featureExtraction -> odometry) ----------------
 * d_xyzi: device pointer to n packed float4 points (HBM-resident scan). The first frame seeds the
 * map (initMapWithPoints), later frames run updatePointsToMap. The pose of every frame is kept on
 * the device (pf_odom_poses). pose_out may be NULL, in which case the call only enqueues work on
 * the handle's stream and returns without waiting. */
int pf_odom_frame_device(pf_odom* h, const float* d_xyzi, size_t n, double pose_out[7]);
/* The same from host memory (stride as pf_fe_extract): the scan is uploaded by DMA on the handle's copy
 * stream, overlapping the previous frames' kernels; with pose_out NULL the call only enqueues, as
 * pf_odom_frame_device. The caller's buffer may change as soon as the call returns. */
int pf_odom_frame_host(pf_odom* h, const float* xyzi, size_t n, size_t stride_bytes, double pose_out[7]);
int pf_odom_sync(pf_odom* h);
/* poses of frames processed so far, 7 doubles each */
int pf_odom_poses(pf_odom* h, double* poses, size_t cap, size_t* n);
/* compute units stage A (features / front end + VoxelGrid) stays off, so that stage B (the odometry)
 * finds free CUs while stage A runs. Defaults: 128 (ES), 32 (BPF); 0 = unrestricted, which is better
 * when several handles share one GPU. A reserve leaving stage A fewer than 32 CUs is PF_EINVAL. */
int pf_odom_set_stage_a_reserve(pf_odom* h, int cus);
/* the ring model extension of pf_fe_set_ring_model for the handle's featureExtraction */
int pf_odom_set_ring_model(pf_odom* h, double top_deg, double bottom_deg);
/* The public members of OdomBaseClass (include/odomEstimationClass.h:52-58, 71): `parameters`
 * (q_w_curr = parameters[0..3] as x, y, z, w; t_w_curr = parameters[4..6]) after the last solve,
 * `last_odom` as a row-major 3 x 4 [R | t], and `optimization_count`. Any output may be NULL. */
int pf_odom_get_state(pf_odom* h, double parameters[7], double last_odom[12], int* optimization_count);
/* Sets those members from poses {qx, qy, qz, qw, tx, ty, tz}: odom = (R(q), t) and parameters =
 * odom_pose, last_odom from last_pose (NULL: the same pose), and optimization_count. With
 * pf_odom_set_map it resumes a handle from an externally held estimator state (a reference node's
 * members, or the oracle's in the per-frame parity test); the handle is marked initialised, so the
 * next frame runs updatePointsToMap. */
int pf_odom_set_state(pf_odom* h, const double odom_pose[7], const double last_pose[7], int optimization_count);
/* Snapshot of a handle's whole estimator state (pose, last pose, optimization count, the maps with
 * their age / p-index bytes, the counters), for golden-vector capture and checkpoint / resume. buf NULL:
 * *size = the bytes needed. restore() loads a snapshot into a handle created with the same parameters
 * (PF_EINVAL otherwise); the next frame continues exactly as the snapshot handle's next frame would
 * (its pose history restarts with the snapshot's pose). */
int pf_odom_snapshot(pf_odom* h, void* buf, size_t cap, size_t* size);
int pf_odom_restore(pf_odom* h, const void* buf, size_t size);
/* Map export: with enable, every frame / update writes the maps (x, y, z, bits(r | g << 8) as 4
 * floats per point) and their sizes straight into mapped pinned host memory at the end of the
 * odometry (one kernel, no extra host round trip). map_export returns the pointer and size of map
 * `which` for the last completed call (valid until the next one): what the C++ shim copies into
 * laserCloudCornerMap / laserCloudSurfMap (or the BPF maps) after every update. */
int pf_odom_set_map_export(pf_odom* h, int enable);
int pf_odom_map_export(pf_odom* h, int which, const float** xyzw, size_t* n);
/* hipGraph replay of the steady-state frame, per stage: a bit mask of PF_GRAPH_STAGE_A (the front
 * end / VoxelGrid stage) and PF_GRAPH_STAGE_B (the odometry stage), 0 = eager launches, or
 * PF_GRAPH_AUTO (the default): stage A replays its graph; stage B launches eagerly while this is the
 * process's only handle and replays its graph when several handles share the host's launch path.
 * The mode was a boolean before the per-stage bits existed; 1 (a caller's "true") is PF_GRAPH_AUTO and
 * the stage bits do not overlap it.
 * Measured on MI355X (configs[1], 4521 frames): a graph replay costs about 0.4 us more per kernel
 * boundary than eager launches (tools/mb/graph_gap.hip) and stage B is the critical path, so one
 * sequence runs 4525-4557 frames/s with stage B eager against 4404-4452 with both graphs; four
 * concurrent handles (configs[3]) run 6558 frames/s with both graphs against 5459 with stage B
 * eager (their host threads contend on the launch path). */
#define PF_GRAPH_AUTO 1
#define PF_GRAPH_STAGE_A 2
#define PF_GRAPH_STAGE_B 4
int pf_odom_set_graph(pf_odom* h, int mode);
/* Reference tie order (default ON since round 5: pf_odom_create / pf_bpf_create enable it, so a handle
 * gives the reference's results frame by frame unless the caller opts out): VoxelGrid (stage A) and
 * rgbds (stage B) order the points of a voxel as libstdc++'s std::sort leaves them -- the reference's own
 * sorts (PCL 1.10 VoxelGrid; src/odomEstimationClass.cpp:74), which are not stable -- so that
 * every f32 centroid is summed in the reference's order. It runs introsort's recursion on the device
 * (pf_tie.h) in place of the radix sorts. enable = 0 is the faster stable mode: stable radix sorts
 * (VoxelGrid) and a merge of the voxel-ordered map with the sorted appended points (rgbds); its
 * centroids' last bits differ from the reference's in 0.5-1 % of frames.
 * Capacity limit: the tie sort keeps one level's big segments (> 65536 keys each) in a 512-entry list,
 * so a handle whose rgbds sort capacity (the maps plus appended points, about 2 x map_capacity for ES,
 * 3 x for BPF) exceeds about 32M elements cannot run it: pf_odom_set_tie_order(h, 1) returns PF_EINVAL
 * and leaves the handle unchanged, and pf_odom_create / pf_bpf_create create such a handle in the stable
 * order instead of failing. A failed allocation (PF_ENOMEM) leaves the handle in its previous order. */
int pf_odom_set_tie_order(pf_odom* h, int enable);
/* Measurement: the association's kNN alone (the exact 5-NN of k_assoc, src/odomEstimationClass.cpp:299,
 * 447) on the last frame's queries -- its down-sampled points through the solved pose -- against the
 * grid that frame searched, `iters` launches timed with HIP events on the handle's stream. avg_ms: per
 * launch; alg_bytes: SURVEY 8(d)'s algorithmic bytes of those queries (16 + 40 + 27 x 8 + 16 |C(q)| each);
 * nq: the query count; queries (optional, 4 floats each: x, y, z, bits(class)) when cap >= nq. The
 * estimator's state is not changed. PF_EINVAL before the second frame. */
int pf_odom_probe_assoc(pf_odom* h, int iters, double* avg_ms, double* alg_bytes, size_t* nq, float* queries,
                        size_t cap);
/* rgbds bookkeeping (the default order merges this frame's sorted appended points into the map, which
 * stays in voxel order): how many updates since create / reset had to sort every element instead (the
 * first update after initMapWithPoints or pf_odom_set_map, a centroid that rounded into a neighbouring
 * voxel, or more than 2048 appended points falling into one of the 512 map-key buckets), and the
 * largest appended-point count seen. Waits for the handle's work. */
int pf_odom_merge_stats(pf_odom* h, int* full_sorts, int* max_appended);
/* Per-stage device time (the reference's per-stage timers, src/laserProcessingNode.cpp:71-79 and
 * src/odomEstimationNode copy.cpp:92-100, as HIP events on the handle's two streams): with enable,
 * every frame records when stage A (featureExtraction / front end + VoxelGrid) and stage B (the
 * odometry) start and end on the device. stage_times waits for the handle's work and returns the mean
 * stage A and stage B durations (us) over the frames since the last enable, and how many. Adds four
 * event records per frame: leave it off in timed runs. */
int pf_odom_set_stage_timing(pf_odom* h, int enable);
int pf_odom_stage_times(pf_odom* h, double* a_us, double* b_us, size_t* frames);

/* ---------------- device memory helpers (scan staging without a framework) ---------------- */
int pf_device_count(int* n);
int pf_dev_malloc(int device, size_t bytes, void** d);
int pf_dev_free(int device, void* d);
int pf_memcpy_h2d(int device, void* dst, const void* src, size_t bytes);
/* Pinned (page-locked), device-mapped host memory usable with any device. The host-input entry points
 * (pf_fe_extract, pf_odom_frame_host, pf_odom_init_map / update, pf_bpf_init_map / update) DMA a
 * 16-byte-stride cloud straight from such a block, and pf_fe_extract writes its outputs straight into
 * one; other memory is repacked into the handle's own pinned staging first. The reference's nodes
 * hold their clouds in host RAM (src/laserProcessingNode.cpp:62-66), so this is how a caller keeps
 * scans "preloaded in pinned host RAM" (SURVEY 8(d)). */
int pf_host_alloc(size_t bytes, void** p);
int pf_host_free(void* p);
int pf_memcpy_d2h(int device, void* dst, const void* src, size_t bytes);

/* ---------------- exact radius-gated 5-NN (the roofline kernel) ----------------
 * Exact 5 nearest map points with squared distance < 1 (f32, accumulated x->y->z), ties by map
 * index: the search of KdTreeFLANN::nearestKSearch(k=5) restricted to what the reference consumes
 * (src/odomEstimationClass.cpp:299-300, 447-451). Unfound slots get idx = -1, d2 = +inf. */
typedef struct pf_knn pf_knn;
int pf_knn_create(int device, size_t map_capacity, size_t query_capacity, pf_knn** out);
int pf_knn_destroy(pf_knn* h);
int pf_knn_set_map(pf_knn* h, const float* xyz4, size_t m);            /* host, 4 floats/pt */
int pf_knn_query(pf_knn* h, const float* q4, size_t nq, int32_t* idx, float* d2);
/* time `iters` launches of the query kernel on the resident map/queries with HIP events.
 * Returns the average kernel ms and the algorithmic bytes per launch. */
int pf_knn_bench(pf_knn* h, int iters, double* avg_ms, double* alg_bytes_per_launch);

#ifdef __cplusplus
}
#endif
#endif
