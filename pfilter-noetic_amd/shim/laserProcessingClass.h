// Drop-in replacement for the reference's include/laserProcessingClass.h (LaserProcessingClass,
// include/laserProcessingClass.h:32-41): the same class name and members for
// src/laserProcessingNode.cpp, running featureExtraction on the MI355X through libpfilter_hip.so.
#ifndef _LASER_PROCESSING_CLASS_H_
#define _LASER_PROCESSING_CLASS_H_

#include <pcl/point_cloud.h>
#include <pcl/point_types.h>

#include "lidar.h"
#include "pfilter_hip_shim.hpp"

using LaserProcessingClass = pfilter_hip::LaserProcessingClassT<pcl::PointCloud<pcl::PointXYZI>, lidar::Lidar>;

#endif  // _LASER_PROCESSING_CLASS_H_
