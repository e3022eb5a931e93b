// Drop-in replacement for the estimators of the reference's include/odomEstimationClass.h:
// Odom_ES_EstimationClass (:140-163; members odom, laserCloudCornerMap, laserCloudSurfMap) for
// src/odomEstimationNode copy.cpp and Odom_BPF_EstimationClass (:169-202; members odom,
// laserCloudBeam/Pillar/Facade/MergeMap) for src/odomEstimationNode.cpp, with the whole
// updatePointsToMap on the MI355X through libpfilter_hip.so.
#ifndef _ODOM_ESTIMATION_CLASS_H_
#define _ODOM_ESTIMATION_CLASS_H_

#include <pcl/point_cloud.h>
#include <pcl/point_types.h>

#include <Eigen/Dense>
#include <Eigen/Geometry>

#include "lidar.h"
#include "pfilter_hip_shim.hpp"

typedef pcl::PointXYZRGB PointType;
using Odom_ES_EstimationClass = pfilter_hip::Odom_ES_EstimationClassT<pcl::PointCloud<PointType>, lidar::Lidar>;
using Odom_BPF_EstimationClass = pfilter_hip::Odom_BPF_EstimationClassT<pcl::PointCloud<PointType>, lidar::Lidar>;
// the north star's name for the ES estimator (the fork calls it Odom_ES_EstimationClass)
using OdomEstimationClass = Odom_ES_EstimationClass;

#endif  // _ODOM_ESTIMATION_CLASS_H_
