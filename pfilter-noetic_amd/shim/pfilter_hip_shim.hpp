// Header-only C++ drop-in for the reference classes on the odometry hot path, over the C ABI of
// libpfilter_hip.so (include/pfilter_hip.h). Same names, same call signatures, same public members
// as the reference:
//
//   LaserProcessingClass::init / featureExtraction        include/laserProcessingClass.h:36-37
//   Odom_ES_EstimationClass::init / initMapWithPoints /
//       updatePointsToMap / getMap, members odom,
//       laserCloudCornerMap, laserCloudSurfMap            include/odomEstimationClass.h:140-152
//   Odom_BPF_EstimationClass::init / initMapWithPoints /
//       updatePointsToMap / getMap / mergeFeatures,
//       members odom, laserCloudBeamMap, laserCloudPillarMap,
//       laserCloudFacadeMap, laserCloudMergeMap            include/odomEstimationClass.h:169-202
//   groundSeg::groundInit / ground_seg, members
//       groundSeginputCloudPtr, groundCloudPtr, nonGroundCloudPtr, gf_*   include/preProcess.hpp:368-614
//   LaserMappingClass::init / updateCurrentPointsToMap / getMap          include/laserMappingClass.h:23-29
//   nongroundExtract::featureInit / pc2pc / featureExtract, members
//       cloud_pillar, cloud_beam, cloud_facade, index_with_feature, thresholds   :616-735
//   curvedVoxel::run, members pointCloudPtr, pointCloudSegPtr, labelRecords,
//       startR / deltaR / deltaP / deltaA / minSeg, sensorMinRange / MaxRange    include/additionClass.hpp:3-120
//
// The classes are templates over the point-cloud and lidar types so this header needs neither PCL nor
// ROS; shim/laserProcessingClass.h and shim/odomEstimationClass.h instantiate them with the PCL 1.10
// types the ROS nodes use. Requirements on the types:
//   Cloud:  Cloud::Ptr (shared pointer), `points` (contiguous vector of points), push_back, clear
//   Point:  standard layout with float x, y, z at offsets 0, 4, 8 (PCL's 32-byte points qualify);
//           PointXYZI also has `intensity`, PointXYZRGB the `r`, `g`, `b` bytes
//   Lidar:  num_lines, min_distance, max_distance, scan_period (lidar::Lidar, include/lidar.h:9-30)
//
// Error behaviour mirrors the reference, which prints and continues: the warnings of
// updatePointsToMap ("not enough points in map to associate, map error", "not enough correct
// points") are printed to stdout the same way; hard errors (bad arguments, HIP failures) throw
// pfilter_hip::Error, since the reference would crash or run into undefined behaviour there.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/pfilter_hip.h"

#ifndef PFILTER_HIP_NO_EIGEN
#include <Eigen/Geometry>
#endif

namespace pfilter_hip {

struct Error : std::runtime_error {
    int code;
    Error(const char* fn, int c) : std::runtime_error(std::string(fn) + " failed with status " + std::to_string(c)), code(c) {}
};

inline int check(const char* fn, int rc) {
    if (rc < 0) throw Error(fn, rc);
    return rc;
}

#ifdef PFILTER_HIP_NO_EIGEN
// minimal stand-in for Eigen::Isometry3d when Eigen is not available (tests)
struct Pose {
    double q[4] = {0, 0, 0, 1};   // x, y, z, w
    double t[3] = {0, 0, 0};
};
#endif

template <class Lidar>
inline pf_lidar_params lidar_params(const Lidar& l) {
    pf_lidar_params p;
    p.num_lines = l.num_lines;
    p.min_dist = l.min_distance;
    p.max_dist = l.max_distance;
    p.scan_period = l.scan_period;
    return p;
}

// --------------------------------------------------------------------------------------------
template <class CloudXYZI, class Lidar>
class LaserProcessingClassT {
public:
    using Ptr = typename CloudXYZI::Ptr;
    using Point = typename std::decay<decltype(std::declval<CloudXYZI>().points[0])>::type;

    explicit LaserProcessingClassT(int device = 0, size_t max_points = 300000) : device_(device), max_points_(max_points) {}
    ~LaserProcessingClassT() { if (h_) pf_fe_destroy(h_); }
    LaserProcessingClassT(const LaserProcessingClassT&) = delete;
    LaserProcessingClassT& operator=(const LaserProcessingClassT&) = delete;

    void init(Lidar lidar_param_in) {
        if (h_) { pf_fe_destroy(h_); h_ = nullptr; }
        const pf_lidar_params p = lidar_params(lidar_param_in);
        check("pf_fe_create", pf_fe_create(&p, device_, max_points_, &h_));
        check("pf_fe_set_tie_order", pf_fe_set_tie_order(h_, reference_tie_order ? 1 : 0));
    }

    // true (the default): equal curvatures in a sector come out as libstdc++'s std::sort leaves them
    // (src/laserProcessingClass.cpp:101-104), i.e. the reference's clouds; false: (value, ring position)
    // order. Read by init(); setReferenceTieOrder() switches a live handle.
    bool reference_tie_order = true;
    void setReferenceTieOrder(bool on) {
        reference_tie_order = on;
        if (h_) check("pf_fe_set_tie_order", pf_fe_set_tie_order(h_, on ? 1 : 0));
    }

    // appends to pc_out_edge / pc_out_surf, never modifies pc_in (laserProcessingClass.cpp:10-96)
    void featureExtraction(const Ptr& pc_in, Ptr& pc_out_edge, Ptr& pc_out_surf) {
        const size_t n = pc_in->points.size();
        buf_e_.resize(4 * (n ? n : 1));
        buf_s_.resize(4 * (n ? n : 1));
        size_t ne = 0, ns = 0;
        const float* src = n ? reinterpret_cast<const float*>(&pc_in->points[0]) : nullptr;
        check("pf_fe_extract", pf_fe_extract(h_, src, n, sizeof(Point), buf_e_.data(), &ne, buf_s_.data(), &ns,
                                             n ? n : 1));
        append(buf_e_, ne, *pc_out_edge);
        append(buf_s_, ns, *pc_out_surf);
    }

private:
    static void append(const std::vector<float>& b, size_t n, CloudXYZI& out) {
        for (size_t i = 0; i < n; ++i) {
            Point p;
            p.x = b[4 * i];
            p.y = b[4 * i + 1];
            p.z = b[4 * i + 2];
            p.intensity = b[4 * i + 3];
            out.push_back(p);
        }
    }
    int device_;
    size_t max_points_;
    pf_fe* h_ = nullptr;
    std::vector<float> buf_e_, buf_s_;
};

// --------------------------------------------------------------------------------------------
// OdomBaseClass's public optimisation members (include/odomEstimationClass.h:52-58, 71), refreshed
// from the device after every initMapWithPoints / updatePointsToMap (pf_odom_get_state), and the
// map copy both estimators share: with refresh_maps_every_frame the maps arrive in pinned host
// memory at the end of the device update (pf_odom_set_map_export), so refreshing the public clouds
// costs no extra device round trip.
class OdomBaseMembers {
public:
    double parameters[7] = {0, 0, 0, 1, 0, 0, 0};
#ifndef PFILTER_HIP_NO_EIGEN
    Eigen::Map<Eigen::Quaterniond> q_w_curr = Eigen::Map<Eigen::Quaterniond>(parameters);
    Eigen::Map<Eigen::Vector3d> t_w_curr = Eigen::Map<Eigen::Vector3d>(parameters + 4);
    Eigen::Isometry3d last_odom = Eigen::Isometry3d::Identity();
#else
    double last_odom[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};   // row-major [R | t]
#endif
    int optimization_count = 2;

    // true (the default): VoxelGrid, rgbds and featureExtraction's sector sort order equal keys as
    // libstdc++'s std::sort does (pf_odom_set_tie_order), so the poses and maps are the reference's frame
    // by frame; false: the faster stable-sort mode, whose centroids differ from the reference's in the
    // last bits. Read by init(); setReferenceTieOrder() switches a live handle.
    bool reference_tie_order = true;

protected:
    void apply_tie_order(pf_odom* h, bool on) {
        reference_tie_order = on;
        if (h) check("pf_odom_set_tie_order", pf_odom_set_tie_order(h, on ? 1 : 0));
    }

    void pull_state(pf_odom* h) {
        double lo[12];
        check("pf_odom_get_state", pf_odom_get_state(h, parameters, lo, &optimization_count));
#ifndef PFILTER_HIP_NO_EIGEN
        last_odom = Eigen::Isometry3d::Identity();
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) last_odom.linear()(i, j) = lo[4 * i + j];
            last_odom.translation()(i) = lo[4 * i + 3];
        }
#else
        for (int k = 0; k < 12; ++k) last_odom[k] = lo[k];
#endif
    }
    // keep the device-side map export in step with refresh_maps_every_frame (before each call)
    void sync_export(pf_odom* h, bool refresh) {
        if (refresh != export_on_) {
            check("pf_odom_set_map_export", pf_odom_set_map_export(h, refresh ? 1 : 0));
            export_on_ = refresh;
        }
    }
    // map `which` into a PointXYZRGB cloud: from the export buffer when the last call wrote it,
    // otherwise by pf_odom_get_map (r = age / rounds, g = p-index / observation count)
    template <class Cloud>
    void fill_map(pf_odom* h, int which, Cloud& out) {
        using Point = typename std::decay<decltype(out.points[0])>::type;
        out.clear();
        if (export_on_) {
            const float* a = nullptr;
            size_t n = 0;
            check("pf_odom_map_export", pf_odom_map_export(h, which, &a, &n));
            for (size_t i = 0; i < n; ++i) {
                Point p;
                p.x = a[4 * i];
                p.y = a[4 * i + 1];
                p.z = a[4 * i + 2];
                uint32_t w;
                std::memcpy(&w, a + 4 * i + 3, 4);
                p.r = (uint8_t)(w & 255u);
                p.g = (uint8_t)((w >> 8) & 255u);
                p.b = 0;
                out.push_back(p);
            }
            return;
        }
        size_t n = 0;
        check("pf_odom_get_map", pf_odom_get_map(h, which, nullptr, nullptr, 0, &n));
        xyz_.resize(3 * (n ? n : 1));
        rg_.resize(2 * (n ? n : 1));
        check("pf_odom_get_map", pf_odom_get_map(h, which, xyz_.data(), rg_.data(), n, &n));
        for (size_t i = 0; i < n; ++i) {
            Point p;
            p.x = xyz_[3 * i];
            p.y = xyz_[3 * i + 1];
            p.z = xyz_[3 * i + 2];
            p.r = rg_[2 * i];
            p.g = rg_[2 * i + 1];
            p.b = 0;
            out.push_back(p);
        }
    }
    bool export_on_ = false;
    std::vector<float> xyz_;
    std::vector<uint8_t> rg_;
};

template <class CloudXYZRGB, class Lidar>
class Odom_ES_EstimationClassT : public OdomBaseMembers {
public:
    using Ptr = typename CloudXYZRGB::Ptr;
    using Point = typename std::decay<decltype(std::declval<CloudXYZRGB>().points[0])>::type;

    explicit Odom_ES_EstimationClassT(int device = 0, size_t max_points = 300000, size_t map_capacity = (size_t)1 << 22)
        : laserCloudCornerMap(new CloudXYZRGB()), laserCloudSurfMap(new CloudXYZRGB()), device_(device),
          max_points_(max_points), map_capacity_(map_capacity) {}
    ~Odom_ES_EstimationClassT() { if (h_) pf_odom_destroy(h_); }
    Odom_ES_EstimationClassT(const Odom_ES_EstimationClassT&) = delete;
    Odom_ES_EstimationClassT& operator=(const Odom_ES_EstimationClassT&) = delete;

    // include/odomEstimationClass.h:146 (weightType is a double there; 0, 1, 2 or 12)
    void init(Lidar lidar_param, double map_resolution_in, int k_new_para, float theta_p_para, int theta_max_para,
              double weightType_para) {
        if (h_) { pf_odom_destroy(h_); h_ = nullptr; }
        const pf_lidar_params lp = lidar_params(lidar_param);
        pf_odom_params op;
        op.map_res = map_resolution_in;
        op.k_new = k_new_para;
        op.theta_p = theta_p_para;
        op.theta_max = theta_max_para;
        op.weight_type = (int)weightType_para;
        check("pf_odom_create", pf_odom_create(&lp, &op, device_, max_points_, map_capacity_, &h_));
        check("pf_odom_set_tie_order", pf_odom_set_tie_order(h_, reference_tie_order ? 1 : 0));
        export_on_ = false;
        set_identity();
        laserCloudCornerMap->clear();
        laserCloudSurfMap->clear();
    }

    void initMapWithPoints(const Ptr& edge_in, const Ptr& surf_in) {
        sync_export(h_, refresh_maps_every_frame);
        check("pf_odom_init_map", pf_odom_init_map(h_, data(edge_in), edge_in->points.size(), sizeof(Point),
                                                   data(surf_in), surf_in->points.size(), sizeof(Point)));
        refresh();
    }

    void updatePointsToMap(const Ptr& edge_in, const Ptr& surf_in) {
        double pose[7];
        sync_export(h_, refresh_maps_every_frame);
        const int rc = check("pf_odom_update", pf_odom_update(h_, data(edge_in), edge_in->points.size(), sizeof(Point),
                                                              data(surf_in), surf_in->points.size(), sizeof(Point),
                                                              pose));
        // the reference's messages (src/odomEstimationClass.cpp:276, 428-431, 574-577)
        if (rc == PF_W_MAP_TOO_SMALL) std::printf("not enough points in map to associate, map error\n");
        if (rc == PF_W_FEW_CORRESPONDENCES) std::printf("not enough correct points\n");
        set_pose(pose);
        refresh();
    }

    // surf map then corner map, appended (src/odomEstimationClass.cpp:210-215)
    void getMap(Ptr& laserCloudMap) {
        for (const auto& p : laserCloudSurfMap->points) laserCloudMap->push_back(p);
        for (const auto& p : laserCloudCornerMap->points) laserCloudMap->push_back(p);
    }

    // false: the map members are only refreshed by syncMaps() (saves the D2H copy per frame when no
    // subscriber reads them, as in src/odomEstimationNode copy.cpp:129-141)
    bool refresh_maps_every_frame = true;
    void syncMaps() { fill_map(h_, 0, *laserCloudCornerMap); fill_map(h_, 1, *laserCloudSurfMap); }
    void setReferenceTieOrder(bool on) { apply_tie_order(h_, on); }

#ifndef PFILTER_HIP_NO_EIGEN
    Eigen::Isometry3d odom = Eigen::Isometry3d::Identity();
#else
    Pose odom;
#endif
    Ptr laserCloudCornerMap;
    Ptr laserCloudSurfMap;

private:
    static const float* data(const Ptr& c) {
        return c->points.empty() ? nullptr : reinterpret_cast<const float*>(&c->points[0]);
    }
    void set_identity() {
        const double id[7] = {0, 0, 0, 1, 0, 0, 0};
        set_pose(id);
    }
    void set_pose(const double* p) {
#ifndef PFILTER_HIP_NO_EIGEN
        // odom = I; linear = q.toRotationMatrix(); translation = t (src/odomEstimationClass.cpp:278-280)
        const Eigen::Quaterniond q(p[3], p[0], p[1], p[2]);
        odom = Eigen::Isometry3d::Identity();
        odom.linear() = q.toRotationMatrix();
        odom.translation() = Eigen::Vector3d(p[4], p[5], p[6]);
#else
        for (int k = 0; k < 4; ++k) odom.q[k] = p[k];
        for (int k = 0; k < 3; ++k) odom.t[k] = p[4 + k];
#endif
    }
    void refresh() {
        pull_state(h_);
        if (refresh_maps_every_frame) syncMaps();
    }
    int device_;
    size_t max_points_, map_capacity_;
    pf_odom* h_ = nullptr;
};

// --------------------------------------------------------------------------------------------
template <class CloudXYZRGB, class Lidar>
class Odom_BPF_EstimationClassT : public OdomBaseMembers {
public:
    using Ptr = typename CloudXYZRGB::Ptr;
    using Point = typename std::decay<decltype(std::declval<CloudXYZRGB>().points[0])>::type;

    explicit Odom_BPF_EstimationClassT(int device = 0, size_t max_points = 300000, size_t map_capacity = (size_t)1 << 22)
        : laserCloudBeamMap(new CloudXYZRGB()), laserCloudPillarMap(new CloudXYZRGB()),
          laserCloudFacadeMap(new CloudXYZRGB()), laserCloudMergeMap(new CloudXYZRGB()), device_(device),
          max_points_(max_points), map_capacity_(map_capacity) {}
    ~Odom_BPF_EstimationClassT() { if (h_) pf_odom_destroy(h_); }
    Odom_BPF_EstimationClassT(const Odom_BPF_EstimationClassT&) = delete;
    Odom_BPF_EstimationClassT& operator=(const Odom_BPF_EstimationClassT&) = delete;

    // include/odomEstimationClass.h:175, src/odomEstimationClass.cpp:649-681
    void init(Lidar lidar_param, double map_resolution_in, int k_new_para, float theta_p_para, int theta_max_para,
              double weightType_para) {
        if (h_) { pf_odom_destroy(h_); h_ = nullptr; }
        const pf_lidar_params lp = lidar_params(lidar_param);
        pf_odom_params op;
        op.map_res = map_resolution_in;
        op.k_new = k_new_para;
        op.theta_p = theta_p_para;
        op.theta_max = theta_max_para;
        op.weight_type = (int)weightType_para;
        check("pf_bpf_create", pf_bpf_create(&lp, &op, device_, max_points_, map_capacity_, &h_));
        check("pf_odom_set_tie_order", pf_odom_set_tie_order(h_, reference_tie_order ? 1 : 0));
        export_on_ = false;
        set_pose(kIdentity);
        for (Ptr* m : maps()) (*m)->clear();
        laserCloudMergeMap->clear();
    }

    // src/odomEstimationClass.cpp:685-691
    void initMapWithPoints(const Ptr& beam_in, const Ptr& pillar_in, const Ptr& facade_in) {
        sync_export(h_, refresh_maps_every_frame);
        check("pf_bpf_init_map", pf_bpf_init_map(h_, data(beam_in), beam_in->points.size(), sizeof(Point),
                                                 data(pillar_in), pillar_in->points.size(), sizeof(Point),
                                                 data(facade_in), facade_in->points.size(), sizeof(Point)));
        refresh();
    }

    // src/odomEstimationClass.cpp:702-749
    void updatePointsToMap(const Ptr& beam_in, const Ptr& pillar_in, const Ptr& facade_in) {
        double pose[7];
        sync_export(h_, refresh_maps_every_frame);
        const int rc = check("pf_bpf_update",
                             pf_bpf_update(h_, data(beam_in), beam_in->points.size(), sizeof(Point), data(pillar_in),
                                           pillar_in->points.size(), sizeof(Point), data(facade_in),
                                           facade_in->points.size(), sizeof(Point), pose));
        // the reference's messages (:753, :908, :1058, :1204)
        if (rc == PF_W_MAP_TOO_SMALL) std::printf("not enough points in map to associate, map error\n");
        if (rc == PF_W_FEW_CORRESPONDENCES) {
            pf_odom_stats st;
            check("pf_odom_get_stats", pf_odom_get_stats(h_, &st));
            if (st.n_res[0] < 20) std::printf("not enough Beam points\n");
            if (st.n_res[1] < 20) std::printf("not enough Pillar points\n");
            if (st.n_res[2] < 20) std::printf("not enough correct points\n");
        }
        set_pose(pose);
        refresh();
    }

    // beam, pillar, then facade, appended (src/odomEstimationClass.cpp:683-689)
    void getMap(Ptr& laserCloudMap) {
        for (Ptr* m : maps())
            for (const auto& p : (*m)->points) laserCloudMap->push_back(p);
    }

    // laserCloudMergeMap = beam + facade + pillar (src/odomEstimationClass.cpp:1297-1302; called at the
    // end of every updatePointsToMap when the maps are refreshed)
    void mergeFeatures(int mergeGround = 1) {
        (void)mergeGround;
        laserCloudMergeMap->clear();
        for (Ptr m : {laserCloudBeamMap, laserCloudFacadeMap, laserCloudPillarMap})
            for (const auto& p : m->points) laserCloudMergeMap->push_back(p);
    }

    bool refresh_maps_every_frame = true;
    void setReferenceTieOrder(bool on) { apply_tie_order(h_, on); }
    void syncMaps() {
        int c = 0;
        for (Ptr* m : maps()) fill_map(h_, c++, **m);
        mergeFeatures(1);
    }

#ifndef PFILTER_HIP_NO_EIGEN
    Eigen::Isometry3d odom = Eigen::Isometry3d::Identity();
#else
    Pose odom;
#endif
    Ptr laserCloudBeamMap;
    Ptr laserCloudPillarMap;
    Ptr laserCloudFacadeMap;
    Ptr laserCloudMergeMap;

private:
    static constexpr double kIdentity[7] = {0, 0, 0, 1, 0, 0, 0};
    std::vector<Ptr*> maps() { return {&laserCloudBeamMap, &laserCloudPillarMap, &laserCloudFacadeMap}; }
    static const float* data(const Ptr& c) {
        return c->points.empty() ? nullptr : reinterpret_cast<const float*>(&c->points[0]);
    }
    void set_pose(const double* p) {
#ifndef PFILTER_HIP_NO_EIGEN
        const Eigen::Quaterniond q(p[3], p[0], p[1], p[2]);
        odom = Eigen::Isometry3d::Identity();
        odom.linear() = q.toRotationMatrix();
        odom.translation() = Eigen::Vector3d(p[4], p[5], p[6]);
#else
        for (int k = 0; k < 4; ++k) odom.q[k] = p[k];
        for (int k = 0; k < 3; ++k) odom.t[k] = p[4 + k];
#endif
    }
    void refresh() {
        pull_state(h_);
        if (refresh_maps_every_frame) syncMaps();
    }
    int device_;
    size_t max_points_, map_capacity_;
    pf_odom* h_ = nullptr;
};

// --------------------------------------------------------------------------------------------
// groundSeg (include/preProcess.hpp:368-614): the ground filter of src/additionNode.cpp:21-27. The
// ROS publishers of the reference class are added by shim/preProcess.hpp.
inline pf_cls_params cls_defaults() {
    pf_cls_params p;
    pf_cls_default_params(&p);
    return p;
}
inline bool same_params(const pf_cls_params& a, const pf_cls_params& b) { return std::memcmp(&a, &b, sizeof(a)) == 0; }

// one pf_cls handle, re-created when the parameters it was created with change
class ClsHandle {
public:
    ClsHandle(int device, size_t max_points) : device_(device), max_points_(max_points) {}
    ~ClsHandle() {
        if (h_) pf_cls_destroy(h_);
    }
    ClsHandle(const ClsHandle&) = delete;
    ClsHandle& operator=(const ClsHandle&) = delete;
    pf_cls* get(const pf_cls_params& p, size_t n) {
        if (!h_ || !same_params(p, prm_) || n > cap_) {
            if (h_) pf_cls_destroy(h_);
            h_ = nullptr;
            cap_ = n > max_points_ ? n : max_points_;
            check("pf_cls_create", pf_cls_create(&p, device_, cap_, &h_));
            prm_ = p;
        }
        return h_;
    }

private:
    int device_;
    size_t max_points_, cap_ = 0;
    pf_cls_params prm_{};
    pf_cls* h_ = nullptr;
};

template <class CloudXYZI>
class GroundSegT {
public:
    using Ptr = typename CloudXYZI::Ptr;
    using Point = typename std::decay<decltype(std::declval<CloudXYZI>().points[0])>::type;
    explicit GroundSegT(int device = 0, size_t max_points = 300000) : cls_(device, max_points) {}

    void groundInit(Ptr& inputCloud) {          // :373-380 (header kept by the ROS layer)
        groundSeginputCloudPtr = inputCloud;
        groundCloudPtr = Ptr(new CloudXYZI());
        nonGroundCloudPtr = Ptr(new CloudXYZI());
    }
    // :398-505: appends to cloud_ground / cloud_unground in the reference's push order
    bool ground_seg(Ptr& cloud_in, Ptr& cloud_ground, Ptr& cloud_unground, int min_grid_pt_num, float grid_resolution,
                    float max_height_difference, float neighbor_height_diff, float max_ground_height,
                    float min_ground_height) {
        static_assert(std::is_standard_layout<Point>::value, "point type must be standard layout");
        pf_cls_params p = cls_defaults();
        p.gf_min_grid_pts = min_grid_pt_num;
        p.gf_grid_res = grid_resolution;
        p.gf_max_height_diff = max_height_difference;
        p.gf_neighbor_height_diff = neighbor_height_diff;
        p.gf_max_ground_height = max_ground_height;
        p.gf_min_ground_height = min_ground_height;
        const size_t n = cloud_in->points.size();
        g_.resize(n ? n : 1);
        u_.resize(n ? n : 1);
        size_t ng = 0, nu = 0;
        check("pf_cls_ground_seg", pf_cls_ground_seg(cls_.get(p, n), n ? &cloud_in->points[0].x : nullptr, n,
                                                     sizeof(Point), g_.data(), &ng, u_.data(), &nu, n ? n : 1));
        for (size_t i = 0; i < ng; ++i) cloud_ground->push_back(cloud_in->points[(size_t)g_[i]]);
        for (size_t i = 0; i < nu; ++i) cloud_unground->push_back(cloud_in->points[(size_t)u_[i]]);
        std::printf("Ground: [%zu] Unground: [%zu].\n", ng, nu);     // :499
        return true;
    }

    // members read by src/additionNode.cpp:24 (include/preProcess.hpp:575, 600-605)
    int gf_grid_pt_num_thre = 8;
    double gf_max_ground_height = 5, gf_min_ground_height = -5, gf_neighbor_height_diff = 1.5,
           gf_max_grid_height_diff = 0.3, gf_grid_resolution = 3.0;
    Ptr groundSeginputCloudPtr, groundCloudPtr, nonGroundCloudPtr;

private:
    ClsHandle cls_;
    std::vector<int32_t> g_, u_;
};

// nongroundExtract (include/preProcess.hpp:616-735): featureExtract on the non-ground cloud. CloudTpl
// is the point-cloud template (pcl::PointCloud); PointN the output point (pcl::PointXYZINormal). As the
// reference's assign_normal (:327-346) does, every point of the input cloud with more than one
// neighbour gets the normal get_pc_pca_feature leaves (:238-239: the PCA normal direction and
// planar_2, zeros with 2-3 neighbours), and classified points the one featureExtract writes before it
// pushes them to their class cloud (normal_x / _y / _z and the fourth float of the normal block,
// pt.normal[3]: linear_2 for pillar / beam, planar_2 for facade).
template <class P>
auto set_pca_normal(P& pt, const float* n4, int) -> decltype((void)pt.normal_x, void()) {
    pt.normal_x = n4[0];
    pt.normal_y = n4[1];
    pt.normal_z = n4[2];
    (&pt.normal_x)[3] = n4[3];          // PCL's data_n[3], which the reference writes as pt.normal[3]
}
template <class P>
void set_pca_normal(P&, const float*, long) {}     // a point type without normals: xyz only

template <template <class> class CloudTpl, class PointN>
class NongroundExtractT {
public:
    using CloudN = CloudTpl<PointN>;
    using PtrN = typename CloudN::Ptr;
    explicit NongroundExtractT(int device = 0, size_t max_points = 300000) : cls_(device, max_points) {}

    void featureInit() {                                            // :621-631 (clouds reset)
        normalCloud = PtrN(new CloudN());
        cloud_pillar = PtrN(new CloudN());
        cloud_beam = PtrN(new CloudN());
        cloud_facade = PtrN(new CloudN());
        cloud_roof = PtrN(new CloudN());
    }
    template <class CloudIn>
    void pc2pc(typename CloudIn::Ptr& cloud_in, PtrN& cloud_out) {   // :633-644 (xyz only)
        for (const auto& q : cloud_in->points) {
            PointN pn;
            pn.x = q.x;
            pn.y = q.y;
            pn.z = q.z;
            cloud_out->push_back(pn);
        }
    }
    // :647-689: the <= neighbor_k nearest within neighbor_searching_radius, PCA, pillar / beam / facade
    template <class PointT>
    void featureExtract(typename CloudTpl<PointT>::Ptr& cloud_in) {
        static_assert(std::is_standard_layout<PointT>::value, "point type must be standard layout");
        pf_cls_params p = cls_defaults();
        p.ground_filter = 0;
        p.radius = neighbor_searching_radius;
        p.k = neighbor_k;
        p.k_min = neigh_k_min;
        p.edge_thre = edge_thre;
        p.planar_thre = planar_thre;
        p.linear_vsin_high = linear_vertical_sin_high_thre;
        p.linear_vsin_low = linear_vertical_sin_low_thre;
        p.planar_vsin_low = planar_vertical_sin_low_thre;
        p.beam_h_max = beam_height_max;
        p.beam_h_min = beam_height_min;
        const size_t n = cloud_in->points.size();
        code_.resize(n ? n : 1);
        pt_num_.resize(n ? n : 1);
        pf_cls* h = cls_.get(p, n);
        check("pf_cls_classify", pf_cls_classify(h, n ? &cloud_in->points[0].x : nullptr, n, sizeof(PointT),
                                                 code_.data(), pt_num_.data()));
        nrm_.resize(4 * (n ? n : 1));
        check("pf_cls_normals", pf_cls_normals(h, nrm_.data(), n));
        index_with_feature.assign(n, 0);
        for (size_t i = 0; i < n; ++i) {
            const int c = code_[i];
            index_with_feature[i] = c;
            if (pt_num_[i] > 1) set_pca_normal(cloud_in->points[i], &nrm_[4 * i], 0);   // min_k = 1 (:238)
            if (c == 0) continue;
            PointN pn;
            pn.x = cloud_in->points[i].x;
            pn.y = cloud_in->points[i].y;
            pn.z = cloud_in->points[i].z;
            set_pca_normal(pn, &nrm_[4 * i], 0);
            (c == 1 ? cloud_pillar : (c == 2 ? cloud_beam : cloud_facade))->push_back(pn);
        }
    }

    // members (include/preProcess.hpp:703-731)
    float neighbor_searching_radius = 1.0f;
    int neighbor_k = 25, neigh_k_min = 8, pca_down_rate = 2;
    float edge_thre = 0.65f, planar_thre = 0.65f, linear_vertical_sin_high_thre = 0.94f,
          linear_vertical_sin_low_thre = 0.17f, planar_vertical_sin_high_thre = 0.98f,
          planar_vertical_sin_low_thre = 0.34f, beam_height_max = 3.402823466e+38f, beam_height_min = 0.5f;
    PtrN normalCloud, cloud_pillar, cloud_beam, cloud_facade, cloud_roof;
    std::vector<int> index_with_feature;

private:
    ClsHandle cls_;
    std::vector<uint8_t> code_;
    std::vector<int32_t> pt_num_;
    std::vector<float> nrm_;
};

// --------------------------------------------------------------------------------------------
// LaserMappingClass (include/laserMappingClass.h:23-29, src/laserMappingClass.cpp): the global map of
// src/laserMappingNode.cpp, held on the device.
template <class CloudXYZI>
class LaserMappingClassT {
public:
    using Ptr = typename CloudXYZI::Ptr;
    using Point = typename std::decay<decltype(std::declval<CloudXYZI>().points[0])>::type;
    explicit LaserMappingClassT(int device = 0, size_t max_points = size_t(1) << 24, size_t max_scan = 300000)
        : device_(device), max_points_(max_points), max_scan_(max_scan) {}
    ~LaserMappingClassT() {
        if (h_) pf_map_destroy(h_);
    }
    LaserMappingClassT(const LaserMappingClassT&) = delete;
    LaserMappingClassT& operator=(const LaserMappingClassT&) = delete;

    void init(double map_resolution) {                                   // :7-33
        if (h_) pf_map_destroy(h_);
        h_ = nullptr;
        check("pf_map_create", pf_map_create(map_resolution, device_, max_points_, max_scan_, &h_));
    }
    // :151-189 with the pose as row-major [R | t]
    void updateCurrentPointsToMap(const Ptr& pc_in, const double T[12]) {
        static_assert(std::is_standard_layout<Point>::value, "point type must be standard layout");
        const size_t n = pc_in->points.size();
        check("pf_map_update_mat", pf_map_update_mat(h_, n ? &pc_in->points[0].x : nullptr, n, sizeof(Point), T));
    }
#ifndef PFILTER_HIP_NO_EIGEN
    void updateCurrentPointsToMap(const Ptr& pc_in, const Eigen::Isometry3d& pose_current) {
        double T[12];
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) T[4 * r + c] = pose_current.linear()(r, c);
            T[4 * r + 3] = pose_current.translation()(r);
        }
        updateCurrentPointsToMap(pc_in, T);
    }
#endif
    Ptr getMap() {                                                       // :194-206
        size_t n = 0;
        check("pf_map_get", pf_map_get(h_, nullptr, 0, &n));
        buf_.resize(4 * (n ? n : 1));
        check("pf_map_get", pf_map_get(h_, buf_.data(), n, &n));
        Ptr out(new CloudXYZI());
        for (size_t i = 0; i < n; ++i) {
            Point p;
            p.x = buf_[4 * i];
            p.y = buf_[4 * i + 1];
            p.z = buf_[4 * i + 2];
            p.intensity = buf_[4 * i + 3];
            out->push_back(p);
        }
        return out;
    }

private:
    int device_;
    size_t max_points_, max_scan_;
    pf_map* h_ = nullptr;
    std::vector<float> buf_;
};

// curvedVoxel (include/additionClass.hpp:3-120, src/additionClass.cpp:457-497): the DCVC clustering of
// additionNode's `curvedfilter` stage on the device (pf_dcvc_run). run() leaves in pointCloudSegPtr
// the points of the clusters larger than minSeg, cluster by cluster from the largest (ties: first
// point), each cluster's points in input order, and in labelRecords {rank, {size, input indices}} per
// kept cluster (labelAnalysis, :319-356). The reference fills pointCloudSegPtr from several OpenMP
// threads at once (colorSegmentation, :364-416), so its order is not defined; DESIGN.md §2 gives the
// statistical bar against its serial reading. The parameters are the members, as init() reads them
// from the yaml file (:17-52); the device handle is shared by copies of the object (the node binds
// the object by value, src/additionNode.cpp:88-89), and its first run starts the range rings at 5 m
// (minPolar's member default, .hpp:105), later runs at 0 (resetParams, :442-455).
template <class Cloud>
class CurvedVoxelT {
public:
    using Ptr = typename Cloud::Ptr;
    using Point = typename std::decay<decltype(std::declval<Cloud>().points[0])>::type;
    struct segInfo {                                                 // .hpp:69-73
        int clusterNum{-1};
        std::vector<int> index{};
    };
    explicit CurvedVoxelT(int device = 0, size_t max_points = 300000)
        : st_(std::make_shared<State>(device, max_points)) {}

    // :457-497 without the ROS publishing (the ROS layer adds init / colorSegmentation / publishData)
    bool run(Ptr& inputCloud) {
        static_assert(std::is_standard_layout<Point>::value, "point type must be standard layout");
        pointCloudPtr = inputCloud;
        labelRecords.clear();
        pointCloudSegPtr = Ptr(new Cloud());
        const size_t n = pointCloudPtr ? pointCloudPtr->points.size() : 0;
        if (n == 0) {
            std::printf("not enough point to convert\n");                    // :461-463 (ROS_ERROR)
            return false;
        }
        pf_dcvc* h = st_->get(params(), n);
        idx_.resize(n);
        lab_.resize(n);
        size_t nk = 0;
        check("pf_dcvc_run", pf_dcvc_run(h, &pointCloudPtr->points[0].x, n, sizeof(Point), idx_.data(), &nk,
                                         lab_.data(), n));
        pointCloudSegPtr->points.reserve(nk);
        for (size_t j = 0; j < nk; ++j) {
            const int i = idx_[j];
            const int r = lab_[(size_t)i];
            pointCloudSegPtr->push_back(pointCloudPtr->points[(size_t)i]);
            if (labelRecords.empty() || labelRecords.back().first != r) labelRecords.emplace_back(r, segInfo{0, {}});
            labelRecords.back().second.clusterNum++;
            labelRecords.back().second.index.push_back(i);
        }
        return true;
    }
    // per input point of the last run: its cluster's rank (1 = largest) or 0 when dropped
    const std::vector<int32_t>& labels() const { return lab_; }

    // the axis-aligned bounds of every cluster of the last run, in labelRecords order: the clustered
    // cloud holds each cluster as one contiguous run (the device publishes them rank by rank), so one
    // pass over pointCloudSegPtr, run by run, gives them all
    struct ClusterBox {
        int label;
        float lo[3], hi[3];
        size_t first, count;        // the cluster's run in pointCloudSegPtr
    };
    std::vector<ClusterBox> clusterBoxes() const {
        std::vector<ClusterBox> out;
        out.reserve(labelRecords.size());
        size_t at = 0;
        for (const auto& rec : labelRecords) {
            ClusterBox b{rec.first, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, at, rec.second.index.size()};
            for (size_t j = at; j < at + b.count; ++j) {
                const auto& q = pointCloudSegPtr->points[j];
                const float xyz[3] = {q.x, q.y, q.z};
                for (int a = 0; a < 3; ++a) {
                    b.lo[a] = j == at ? xyz[a] : std::min(b.lo[a], xyz[a]);
                    b.hi[a] = j == at ? xyz[a] : std::max(b.hi[a], xyz[a]);
                }
            }
            at += b.count;
            out.push_back(b);
        }
        return out;
    }

    // members (include/additionClass.hpp:73-115), defaults of config/config.yaml:7-8, 49-54
    Ptr pointCloudPtr, pointCloudSegPtr;
    std::vector<std::pair<int, segInfo>> labelRecords;
    double sensorMinRange{1.0}, sensorMaxRange{120.0};
    double startR{1.0}, deltaR{0.003}, deltaP{1.2}, deltaA{1.2};
    int minSeg{80};

private:
    pf_dcvc_params params() const {
        pf_dcvc_params p;
        pf_dcvc_default_params(&p);
        p.start_r = startR;
        p.delta_r = deltaR;
        p.delta_p = deltaP;
        p.delta_a = deltaA;
        p.min_seg = minSeg;
        p.min_range = sensorMinRange;
        p.max_range = sensorMaxRange;
        return p;
    }
    // the device handle: re-created (a first run again) when the parameters change; a scan above the
    // capacity grows it in place, keeping the call state (pf_dcvc_reserve)
    struct State {
        State(int device, size_t max_points) : device(device), max_points(max_points) {}
        ~State() {
            if (h) pf_dcvc_destroy(h);
        }
        pf_dcvc* get(const pf_dcvc_params& p, size_t n) {
            const bool same = p.start_r == prm.start_r && p.delta_r == prm.delta_r && p.delta_p == prm.delta_p &&
                              p.delta_a == prm.delta_a && p.min_seg == prm.min_seg && p.min_range == prm.min_range &&
                              p.max_range == prm.max_range;
            if (!h || !same) {
                if (h) pf_dcvc_destroy(h);
                h = nullptr;
                cap = n > max_points ? n : max_points;
                check("pf_dcvc_create", pf_dcvc_create(&p, device, cap, &h));
                prm = p;
            } else if (n > cap) {
                check("pf_dcvc_reserve", pf_dcvc_reserve(h, n));
                cap = n;
            }
            return h;
        }
        int device;
        size_t max_points, cap = 0;
        pf_dcvc_params prm{};
        pf_dcvc* h = nullptr;
    };
    std::shared_ptr<State> st_;
    std::vector<int32_t> idx_, lab_;
};

}  // namespace pfilter_hip
