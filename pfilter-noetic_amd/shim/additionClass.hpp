// Drop-in replacement for the reference's include/additionClass.hpp as src/additionNode.cpp uses it:
// class curvedVoxel with the same constructor, run(cloud, header), members (pointCloudPtr,
// pointCloudSegPtr, pointCloudSegRGBLPtr, labelRecords, boxInfo, the yaml / topic strings and the three
// publishers) and the same yaml keys (src/additionClass.cpp:17-52); the clustering runs on the MI355X
// through libpfilter_hip.so (pfilter_hip::CurvedVoxelT in pfilter_hip_shim.hpp), so additionNode.cpp
// builds without src/additionClass.cpp (whose OpenMP loops race: SURVEY §2 row 9). The per-cluster
// colours and bounding boxes of colorSegmentation (:364-416) come from the device's clustered cloud
// (CurvedVoxelT::clusterBoxes: one pass over its contiguous cluster runs). The reference's distanceWeight / segmentation helper classes are not on the path
// and are not provided.
#ifndef PFILTER_HIP_ADDITIONCLASS_HPP
#define PFILTER_HIP_ADDITIONCLASS_HPP

#include <algorithm>
#include <cmath>
#include <limits>
#include <sstream>

#include <yaml-cpp/yaml.h>

#include "common.hpp"               // the package's ROS / PCL typedefs (pointTypeCloud, pointTypeRGBL, ...)
#include "pfilter_hip_shim.hpp"

class curvedVoxel : public pfilter_hip::CurvedVoxelT<pointTypeCloud> {
public:
    explicit curvedVoxel(ros::NodeHandle nh) : nh_(nh) {}

    void init(pointTypeCloud::Ptr& inputCloud, std_msgs::Header header) {           // :12-56
        YAML::Node node = YAML::LoadFile(yamlConfigFile);
        const YAML::Node lidar_config = node["velodyne"];
        const YAML::Node voxel_config = node["curvedVoxel"];
        sensorModel = lidar_config["sensorModel"].as<int>();
        scanPeriod = lidar_config["scanPeriod"].as<double>();
        verticalRes = lidar_config["verticalRes"].as<double>();
        initAngle = lidar_config["initAngle"].as<double>();
        sensorHeight = lidar_config["sensorHeight"].as<double>();
        sensorMinRange = lidar_config["sensorMinRange"].as<double>();
        sensorMaxRange = lidar_config["sensorMaxRange"].as<double>();
        near_dis = lidar_config["near_dis"].as<double>();
        startR = voxel_config["startR"].as<double>();
        deltaR = voxel_config["deltaR"].as<double>();
        deltaP = voxel_config["deltaP"].as<double>();
        deltaA = voxel_config["deltaA"].as<double>();
        minSeg = voxel_config["minSeg"].as<int>();
        colorList.clear();
        for (const auto& colorNode : node["colorlist"]) {
            std::istringstream cs(colorNode.as<std::string>());
            int r, g, b;
            char comma;
            cs >> r >> comma >> g >> comma >> b;
            colorList.push_back({r, g, b});
        }
        cloudHeader = header;
        pointCloudPtr = inputCloud;
    }

    void run(pointTypeCloud::Ptr& inputCloud, std_msgs::Header header) {            // :457-497
        init(inputCloud, header);
        if (!CurvedVoxelT::run(inputCloud)) {
            ROS_ERROR("not enough point to convert");
            return;
        }
        colorSegmentation();
        publishData();
    }

    // :364-416: the clusters' boxes from the device's clustered cloud (CurvedVoxelT::clusterBoxes, one
    // pass over its contiguous runs) and the cloud coloured run by run from the yaml colour list
    bool colorSegmentation() {
        const auto boxes = clusterBoxes();
        pointCloudSegRGBLPtr.reset(new pointTypeRGBLCloud());
        pointCloudSegRGBLPtr->points.resize(pointCloudSegPtr->points.size());
        boxInfo.assign(boxes.size(), jsk_recognition_msgs::BoundingBox());
        for (size_t c = 0; c < boxes.size(); ++c) {
            const auto& cb = boxes[c];
            const std::vector<int>* rgb = colorList.empty() ? nullptr : &colorList[cb.label % colorList.size()];
            for (size_t j = cb.first; j < cb.first + cb.count; ++j) {
                auto& out = pointCloudSegRGBLPtr->points[j];
                const auto& in = pointCloudSegPtr->points[j];
                out.x = in.x;
                out.y = in.y;
                out.z = in.z;
                if (rgb) {
                    out.r = (*rgb)[0];
                    out.g = (*rgb)[1];
                    out.b = (*rgb)[2];
                }
            }
            jsk_recognition_msgs::BoundingBox& box = boxInfo[c];
            box.header = cloudHeader;
            box.label = cb.label;
            // extent = hi - lo in float, widened; centre = lo + extent / 2 in double (the reference's types)
            const double ext[3] = {(double)(cb.hi[0] - cb.lo[0]), (double)(cb.hi[1] - cb.lo[1]),
                                   (double)(cb.hi[2] - cb.lo[2])};
            box.pose.position.x = cb.lo[0] + ext[0] / 2.0;
            box.pose.position.y = cb.lo[1] + ext[1] / 2.0;
            box.pose.position.z = cb.lo[2] + ext[2] / 2.0;
            box.dimensions.x = std::abs(ext[0]);
            box.dimensions.y = std::abs(ext[1]);
            box.dimensions.z = std::abs(ext[2]);
        }
        return true;
    }

    // :422-440: the boxes, then the coloured cloud, both stamped with the scan's header
    void publishData() {
        jsk_recognition_msgs::BoundingBoxArray boxArray;
        boxArray.header = cloudHeader;
        boxArray.boxes = boxInfo;
        pubBoundingBox.publish(boxArray);
        sensor_msgs::PointCloud2 coloured;
        pcl::toROSMsg(*pointCloudSegRGBLPtr, coloured);
        coloured.header = cloudHeader;
        pubCurvedPointCloudRGBA.publish(coloured);
    }
    void resetParams() {}                            // :442-455: the device handle carries the ring start

    pointTypeRGBLCloud::Ptr pointCloudSegRGBLPtr;
    std_msgs::Header cloudHeader;
    std::vector<jsk_recognition_msgs::BoundingBox> boxInfo{};
    std::string yamlConfigFile, velodyne_points, pfilter_input_cloud, sensorFrameId;
    ros::Publisher pubCurvedPointCloud, pubCurvedPointCloudRGBA, pubBoundingBox;

private:
    int sensorModel{64};
    double scanPeriod{0.0}, verticalRes{0.0}, initAngle{0.0}, sensorHeight{0.0}, near_dis{3.0};
    std::vector<std::vector<int>> colorList;
    ros::NodeHandle nh_;
};

#endif  // PFILTER_HIP_ADDITIONCLASS_HPP
