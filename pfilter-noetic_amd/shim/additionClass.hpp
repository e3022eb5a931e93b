// Drop-in replacement for the reference's include/additionClass.hpp as src/additionNode.cpp uses it:
// class curvedVoxel with the same constructor, run(cloud, header), members (pointCloudPtr,
// pointCloudSegPtr, pointCloudSegRGBLPtr, labelRecords, boxInfo, the yaml / topic strings and the three
// publishers) and the same yaml keys (src/additionClass.cpp:17-52); the clustering runs on the MI355X
// through libpfilter_hip.so (pfilter_hip::CurvedVoxelT in pfilter_hip_shim.hpp), so additionNode.cpp
// builds without src/additionClass.cpp (whose OpenMP loops race: SURVEY §2 row 9). The per-cluster
// colours and bounding boxes of colorSegmentation (:364-416) are computed here from the clusters the
// device returns. The reference's distanceWeight / segmentation helper classes are not on the path
// and are not provided.
#ifndef PFILTER_HIP_ADDITIONCLASS_HPP
#define PFILTER_HIP_ADDITIONCLASS_HPP

#include <algorithm>
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

    bool colorSegmentation() {                                                       // :364-416
        pointCloudSegRGBLPtr.reset(new pointTypeRGBLCloud());
        boxInfo.clear();
        for (auto& label : labelRecords) {
            jsk_recognition_msgs::BoundingBox box;
            float min_x = std::numeric_limits<float>::max(), max_x = -std::numeric_limits<float>::max();
            float min_y = min_x, max_y = max_x, min_z = min_x, max_z = max_x;
            for (int id : label.second.index) {
                const auto& p = pointCloudPtr->points[id];
                min_x = std::min(min_x, p.x); max_x = std::max(max_x, p.x);
                min_y = std::min(min_y, p.y); max_y = std::max(max_y, p.y);
                min_z = std::min(min_z, p.z); max_z = std::max(max_z, p.z);
                pointTypeRGBL pp;
                pp.x = p.x; pp.y = p.y; pp.z = p.z;
                if (!colorList.empty()) {
                    const std::vector<int>& c = colorList[label.first % colorList.size()];
                    pp.r = c[0]; pp.g = c[1]; pp.b = c[2];
                }
                pointCloudSegRGBLPtr->points.push_back(pp);
            }
            const double lx = max_x - min_x, ly = max_y - min_y, lz = max_z - min_z;
            box.header = cloudHeader;
            box.label = label.first;
            box.pose.position.x = min_x + lx / 2.0;
            box.pose.position.y = min_y + ly / 2.0;
            box.pose.position.z = min_z + lz / 2.0;
            box.dimensions.x = lx < 0 ? -lx : lx;
            box.dimensions.y = ly < 0 ? -ly : ly;
            box.dimensions.z = lz < 0 ? -lz : lz;
            boxInfo.emplace_back(box);
        }
        return true;
    }

    void publishData() {                                                             // :422-440
        jsk_recognition_msgs::BoundingBoxArray boxArray;
        for (auto& box : boxInfo) boxArray.boxes.emplace_back(box);
        boxArray.header = cloudHeader;
        pubBoundingBox.publish(boxArray);
        sensor_msgs::PointCloud2 msg;
        pcl::toROSMsg(*pointCloudSegRGBLPtr, msg);
        msg.header = cloudHeader;
        pubCurvedPointCloudRGBA.publish(msg);
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
