// Drop-in replacement for the reference's include/laserMappingClass.h (LaserMappingClass, :23-29) for
// src/laserMappingNode.cpp: the global map of 50 m cubes kept on the MI355X through libpfilter_hip.so.
#ifndef _LASER_MAPPING_H_
#define _LASER_MAPPING_H_

#include <pcl/point_cloud.h>
#include <pcl/point_types.h>

#include <Eigen/Dense>
#include <Eigen/Geometry>

#include "pfilter_hip_shim.hpp"

using LaserMappingClass = pfilter_hip::LaserMappingClassT<pcl::PointCloud<pcl::PointXYZI>>;

#endif  // _LASER_MAPPING_H_
