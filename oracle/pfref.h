/* pfref — CPU restatement of the PFilter/FLOAM ES odometry hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity oracle and the reported
 * single-core CPU baseline. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (pfilter-noetic_amd/) never links it.
 *
 * It restates, in plain C++17 with no third-party dependencies:
 *   - LaserProcessingClass::featureExtraction(+FromSector)   src/laserProcessingClass.cpp:10-209
 *   - Odom_ES_EstimationClass init/initMapWithPoints/updatePointsToMap/addEdgeCostFactor/
 *     addSurfCostFactor/addPointsToMap                       src/odomEstimationClass.cpp:182-647
 *   - groundSeg::ground_seg, nongroundExtract::featureExtract  include/preProcess.hpp:398-505,646-689
 *   - LaserMappingClass init/updateCurrentPointsToMap/getMap   src/laserMappingClass.cpp:7-206
 *   - Odom_BPF_EstimationClass init/initMapWithPoints/updatePointsToMap/addBeam|Pillar|Facade-
 *     CostFactor/addPointsToMap (the same sequence over 3 maps)  src/odomEstimationClass.cpp:649-1306
 *   - OdomBaseClass rgbds/extractstablepoint/observeMean/pointAssociateToMap
 *                                                            src/odomEstimationClass.cpp:7-174
 *   - pointSparsityMean                                      include/odomEstimationClass.h:111-126
 *   - Edge/SurfNormAnalyticCostFunction, PoseSE3Parameterization, getTransformFromSe3
 *                                                            src/lidarOptimization.cpp:12-155
 * and the third-party semantics those call: PCL 1.10 VoxelGrid,
 * CropBox, ExtractIndices, KdTreeFLANN (FLANN 1.9.1 single kd-tree, leaf 15), Eigen 3.3
 * quaternion/isometry formulas, a 3x3 symmetric eigensolver, column-pivoting Householder
 * least squares, and the Ceres 1.14 Levenberg-Marquardt trust-region loop with
 * HuberLoss(0.1), Jacobi scaling and DENSE_QR.
 *
 * PARITY STATUS: the reference ships no tests, golden vectors or fixtures and
 * its dependencies (ROS, PCL, FLANN, Eigen, Ceres) are absent here, so it cannot be run.
 * Arithmetic owned by the reference's own files is restated operation-for-operation
 * (float vs double exactly as the C++ source evaluates it). Arithmetic inside PCL/Eigen/
 * FLANN/Ceres is "parity unpinned": restated from their published algorithms, with the
 * ambiguous choices exposed as option bits below so their pose sensitivity can be bounded.
 */
#ifndef PFREF_H
#define PFREF_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {            /* lidar::Lidar fields read on the path (include/lidar.h:9-30) */
    int num_lines;
    double min_distance;
    double max_distance;
    double scan_period;
    /* EXTENSION (pf_fe_set_ring_model): ring_bottom < ring_top selects the linear beam model
     * ring = int((ring_top - elevation) * num_lines / (ring_top - ring_bottom)); 0, 0 = reference */
    double ring_top, ring_bottom;
} pfref_lidar;

typedef struct {            /* Odom_ES_EstimationClass::init arguments (include/odomEstimationClass.h:146) */
    double map_resolution;
    int k_new;
    float theta_p;
    int theta_max;
    double weight_type;     /* 0, 1, 2 or 12 */
} pfref_odom_params;

/* Option bits (0 = reference-faithful choice). */
enum {
    PFREF_FE_STABLE_TIES = 1,   /* sector sort by (curvature, id) instead of libstdc++ std::sort  */
    PFREF_FE_SQRT_DOUBLE = 2,   /* ring-binning range as sqrt((double)(x*x+y*y)) not sqrtf       */
    PFREF_VG_STABLE      = 4,   /* VoxelGrid/rgbds ties kept in input order (stable sort)        */
    PFREF_KNN_BRUTE      = 8,   /* brute-force kNN instead of the FLANN-style kd-tree            */
    PFREF_LM_NORMAL_EQ   = 16,  /* LM step by 6x6 normal equations instead of dense Householder QR */
    PFREF_LD_TRIG        = 32,  /* (experiment) the LM's sin / cos / cubes in long double, rounded once:
                                   another libm's last bit (tools/drift_probe.py)                   */
    PFREF_QR_REVSUM      = 64,  /* (experiment) the LM's Householder QR sums its rows in reverse order  */
    PFREF_LM_QUAD        = 128, /* (experiment) LM_NORMAL_EQ's products and step in binary128         */
    PFREF_COST_REVSUM    = 256, /* (experiment) the faithful LM sums its cost in reverse order           */
    PFREF_DEV_LIBM       = 512, /* (experiment) LM_NORMAL_EQ's SE(3) updates by libm sin/cos (se3_plus) */
    PFREF_DEV_HALFANGLE  = 1024,/* (experiment) LM_NORMAL_EQ's SE(3) update by round 3's half-angle
                                   identities instead of the reference's form                      */
    PFREF_GPU_EQUIV      = 1 | 4 | 16
};

typedef struct {
    int64_t n_edge_in, n_surf_in;        /* E, S */
    int64_t n_edge_ds, n_surf_ds;        /* E', S' */
    int64_t n_edge_map, n_surf_map;      /* map sizes after the update */
    int64_t n_edge_res, n_surf_res;      /* residuals in the last outer iteration */
    int64_t n_edge_valid, n_surf_valid;  /* associations passing the gate + fit test (last outer it.) */
    int32_t outer_iterations;            /* optimization_count used */
    int32_t lm_iterations;               /* summed over outer iterations */
    int32_t map_too_small;               /* 1 when the solve was skipped (odomEstimationClass.cpp:274-277) */
    int32_t status;
    double t_downsample, t_tree, t_assoc, t_solve, t_mapupdate;  /* seconds */
    /* per map class (ES: 0 corner, 1 surf; BPF: 0 beam, 1 pillar, 2 facade); the n_edge_* /
     * n_surf_* fields above repeat classes 0 and 1 */
    int64_t n_in[3], n_ds[3], n_map[3], n_res[3], n_valid[3];
} pfref_stats;

/* --- feature extraction: LaserProcessingClass::featureExtraction --------------------- */
/* xyzi: 4 floats per point (x, y, z, intensity). Outputs are XYZI copies of input points
 * in reference order (ring -> sector -> edge by descending curvature / surf ascending).
 * Returns 0, or -1 when cap is exceeded. */
int pfref_feature_extraction(const pfref_lidar* lidar, int opts, const float* xyzi, size_t n,
                             float* edge_out, size_t* n_edge, float* surf_out, size_t* n_surf,
                             size_t cap);

/* --- third-party semantics, exposed for unit tests ---------------------------------- */
/* PCL VoxelGrid<PointXYZRGB> (B.1): pts = 4 floats (x,y,z, rgb packed as uint32 bits r<<16|g<<8|b). */
int pfref_voxel_grid(const float* pts, size_t n, float leaf, int opts, float* out, size_t* n_out);
/* OdomBaseClass::rgbds (a15): same point layout. */
int pfref_rgbds(const float* pts, size_t n, float leaf, int opts, float* out, size_t* n_out);
/* exact kNN (d^2 in float accumulated x->y->z), ties by index. map/queries 4 floats/pt. */
/* sum over queries of the map points in the 27 1 m cells around each query (SURVEY 8(d) |C(q)|) */
unsigned long long pfref_knn_cellpop(const float* map, size_t m, const float* queries, size_t q);
int pfref_knn(const float* map, size_t m, const float* queries, size_t q, int k, int opts,
              int32_t* idx_out, float* d2_out);
/* 3x3 symmetric eigen (ascending). a = {a00,a01,a02,a11,a12,a22}. */
void pfref_eigen_sym3(const double a[6], double evals[3], double evecs[9] /* column-major */);
/* 5x3 column-pivoting Householder least squares of A n = -1 (A row-major 5x3). */
void pfref_plane_fit(const double A[15], double n_out[3]);
/* PoseSE3Parameterization::Plus */
void pfref_se3_plus(const double x[7], const double delta[6], double out[7]);
/* GPU_EQUIV SE(3) update: getTransformFromSe3 with one deterministic sincos of theta/2 and the
 * half-angle identities (the device's arithmetic, pf_geom.h se3_exp) */
void pfref_se3_plus_half(const double x[7], const double delta[6], double out[7]);
/* sin/cos from + - * and rint only (fdlibm kernels): bit-identical on the host and the device */
void pfref_det_sincos(double x, double* s, double* c);
/* Eigen 3.3 Isometry3d::rotation(): orthogonal polar factor of a 3x3 (row-major in/out) */
void pfref_rotation_polar(const double m[9], double out[9]);
/* Edge/SurfNormAnalyticCostFunction::Evaluate: returns residual, J[7] */
double pfref_edge_eval(const double x[7], const double cur[3], const double a[3], const double b[3],
                       double weight, double J[7]);
double pfref_surf_eval(const double x[7], const double cur[3], const double n[3], double d,
                       double weight, double J[7]);

/* --- odometry: Odom_ES_EstimationClass ------------------------------------------------ */
typedef struct pfref_odom pfref_odom;
pfref_odom* pfref_odom_create(const pfref_lidar* lidar, const pfref_odom_params* params, int opts);
void pfref_odom_destroy(pfref_odom* h);
/* edge/surf: 4 floats per point (x, y, z, intensity); r = g = 0 as after copyPointCloud */
int pfref_odom_init_map(pfref_odom* h, const float* edge, size_t ne, const float* surf, size_t ns);
int pfref_odom_update(pfref_odom* h, const float* edge, size_t ne, const float* surf, size_t ns,
                      double pose_out[7]);
/* pose = {qx,qy,qz,qw,tx,ty,tz} of odom (rotation via Quaterniond(odom.rotation())) */
void pfref_odom_get_pose(const pfref_odom* h, double pose[7]);
/* which: 0 edge (corner) map, 1 surf map. xyz: 3 floats/pt, rg: 2 bytes/pt (r, g). */
int pfref_odom_get_map(const pfref_odom* h, int which, float* xyz, uint8_t* rg, size_t cap, size_t* n);
int pfref_odom_set_map(pfref_odom* h, int which, const float* xyz, const uint8_t* rg, size_t n);
void pfref_odom_get_stats(const pfref_odom* h, pfref_stats* s);
/* set odom / last_odom (poses {qx,qy,qz,qw,tx,ty,tz}) e.g. to replay a fixture from a given state */
void pfref_odom_set_state(pfref_odom* h, const double odom_pose[7], const double last_pose[7]);
void pfref_odom_set_opt_count(pfref_odom* h, int n);

/* --- odometry: Odom_BPF_EstimationClass (src/odomEstimationClass.cpp:649-1306) ----------
 * Three map classes in residual order: 0 beam (line, leaf r), 1 pillar (line, leaf r),
 * 2 facade (plane, leaf 2r). The same handle type and accessors as the ES estimator; `which` of
 * get/set_map is the class index. */
pfref_odom* pfref_bpf_create(const pfref_lidar* lidar, const pfref_odom_params* params, int opts);
int pfref_odom_classes(const pfref_odom* h);   /* 2 (ES) or 3 (BPF) */
/* clouds[c]: 4 floats per point (x, y, z, intensity); n[c] points; one per class */
int pfref_odom_init_map_n(pfref_odom* h, const float* const* clouds, const size_t* n);
int pfref_odom_update_n(pfref_odom* h, const float* const* clouds, const size_t* n, double pose_out[7]);

/* --- BPF front end: groundSeg::ground_seg + nongroundExtract::featureExtract -------------
 * (include/preProcess.hpp:398-505, :646-689, driven by src/additionNode.cpp:21-45). Parameters
 * mirror the reference's member defaults (pfref_cls_default_params); same layout as the
 * product's pf_cls_params. Points: x, y, z floats at the start of each `stride`-byte record. */
typedef struct {
    int ground_filter;                 /* additionNode `groundfilter` (pfilter_kitti.launch:10) */
    int gf_min_grid_pts;               /* gf_grid_pt_num_thre (preProcess.hpp:575) */
    float gf_grid_res, gf_max_height_diff, gf_neighbor_height_diff, gf_max_ground_height,
          gf_min_ground_height;        /* :601-605 (double members passed as float) */
    float radius;                      /* neighbor_searching_radius (:703) */
    int k, k_min;                      /* neighbor_k, neigh_k_min (:705-706) */
    float edge_thre, planar_thre, linear_vsin_high, linear_vsin_low, planar_vsin_low,
          beam_h_max, beam_h_min;      /* :708-715 */
} pfref_cls_params;
void pfref_cls_default_params(pfref_cls_params* p);
/* ground / unground as input indices in the reference's push order */
int pfref_ground_seg(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, int32_t* ground,
                     size_t* ng, int32_t* unground, size_t* nu);
/* per point: 0 none, 1 pillar, 2 beam, 3 facade (index_with_feature); pt_num = neighbours found */
int pfref_pca_classify(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, uint8_t* cls,
                       int32_t* pt_num);
/* the same, and the normal the reference's assign_normal writes into each classified point (:327-346):
 * 4 floats per point, (principal direction, linear_2) for pillar / beam, (normal direction,
 * planar_2) for facade, zeros for unclassified points */
int pfref_pca_classify_normals(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, uint8_t* cls,
                               int32_t* pt_num, float* normal4);
/* curvedVoxel (DCVC, src/additionClass.cpp), serial semantics (pfref_dcvc.cpp header) */
typedef struct {
    double start_r, delta_r, delta_p, delta_a;   /* config/config.yaml:50-53 curvedVoxel */
    int min_seg;                                 /* :54 */
    double min_range, max_range;                 /* :7-8 velodyne sensorMinRange / sensorMaxRange */
} pfref_dcvc_params;
void pfref_dcvc_default_params(pfref_dcvc_params* p);
/* out_idx: input indices of the kept points in the published order (pointCloudSegPtr); label: per
 * point its cluster's rank (1 = largest) or 0 (dropped); first_frame: the node's first call (the
 * polar range starts from the member default 5 m instead of 0). Any output may be NULL. */
int pfref_dcvc(const float* xyz, size_t n, size_t stride, const pfref_dcvc_params* p, int first_frame,
               int32_t* out_idx, size_t* n_out, int32_t* label);
/* mode 0 = pfref_dcvc; mode 1 = connected components of the same neighbourhood (the device's reading) */
int pfref_dcvc_mode(const float* xyz, size_t n, size_t stride, const pfref_dcvc_params* p, int first_frame,
                    int mode, int32_t* out_idx, size_t* n_out, int32_t* label);
/* the additionNode chain with curvedfilter on (src/additionNode.cpp:21-45): ground_seg -> DCVC on the
 * non-ground cloud -> featureExtract on DCVC's output; class clouds as input indices */
int pfref_bpf_preprocess_dcvc(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p,
                              const pfref_dcvc_params* dp, int first_frame, int dcvc_mode, int32_t* beam, size_t* nb,
                              int32_t* pillar, size_t* np, int32_t* facade, size_t* nf, int32_t* ground,
                              size_t* ng);
/* the chain: class clouds (input indices, in the published order); any output may be NULL */
int pfref_bpf_preprocess(const float* xyz, size_t n, size_t stride, const pfref_cls_params* p, int32_t* beam,
                         size_t* nb, int32_t* pillar, size_t* np, int32_t* facade, size_t* nf, int32_t* ground,
                         size_t* ng);

/* --- LaserMappingClass (src/laserMappingClass.cpp): the global map of 50 m cubes ------------------
 * update: xyzi records of `stride` bytes in the sensor frame, pose = qx, qy, qz, qw, tx, ty, tz; returns
 * -1 when a point falls outside the allocated cubes (reference: null dereference). get: x, y, z,
 * intensity of the whole map in the reference's cube order (n = size; xyzi may be NULL). */
typedef struct pfref_map pfref_map;
pfref_map* pfref_map_create(double map_resolution);
void pfref_map_destroy(pfref_map* m);
int pfref_map_update(pfref_map* m, const float* xyzi, size_t n, size_t stride, const double pose[7]);
int pfref_map_get(const pfref_map* m, float* xyzi, size_t cap, size_t* n);

/* --- whole frame: featureExtraction then initMapWithPoints (first call) / updatePointsToMap */
int pfref_odom_frame(pfref_odom* h, const pfref_lidar* lidar, const float* xyzi, size_t n,
                     double pose_out[7]);

#ifdef __cplusplus
}
#endif
#endif
