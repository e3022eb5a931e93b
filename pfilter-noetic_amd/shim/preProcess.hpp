// Drop-in replacement for the reference's include/preProcess.hpp as src/additionNode.cpp uses it:
// groundSeg (ground_seg, :398-505) and nongroundExtract (featureExtract, :646-689) with the same names,
// members and ROS publishers, the computation on the MI355X through libpfilter_hip.so
// (pfilter_hip::GroundSegT / NongroundExtractT in pfilter_hip_shim.hpp). The reference header's
// PrincipleComponentAnalysis helper and groundSeg's unused fast_ground_filter / random_downsample_pcl
// declarations are not part of the path and are not provided.
#ifndef PFILTER_HIP_PREPROCESS_HPP
#define PFILTER_HIP_PREPROCESS_HPP

#include "common.hpp"               // the package's ROS / PCL typedefs (pointTypeCloud, pointTypeNormal, ...)
#include "pfilter_hip_shim.hpp"

class groundSeg : public pfilter_hip::GroundSegT<pointTypeCloud> {
public:
    explicit groundSeg(ros::NodeHandle nh) : nh_(nh) {}
    void groundInit(pointTypeCloud::Ptr& inputCloud, std_msgs::Header header) {     // :373-380
        GroundSegT::groundInit(inputCloud);
        cloudHeader = header;
    }
    void groundPubCloud() {                                                          // :382-392
        sensor_msgs::PointCloud2 g, ng;
        pcl::toROSMsg(*groundCloudPtr, g);
        pcl::toROSMsg(*nonGroundCloudPtr, ng);
        g.header = ng.header = cloudHeader;
        pubGround.publish(g);
        pubNonGround.publish(ng);
    }
    ros::Publisher pubGround, pubNonGround;
    std_msgs::Header cloudHeader;
    ros::NodeHandle nh_;
};

class nongroundExtract : public pfilter_hip::NongroundExtractT<pcl::PointCloud, pointTypeNormal> {
public:
    explicit nongroundExtract(ros::NodeHandle nh) : nh_(nh) {}
    void featureInit(pointTypeCloud::Ptr& inputCloud, std_msgs::Header header) {    // :621-631
        NongroundExtractT::featureInit();
        featureSeginputCloudPtr = inputCloud;
        cloudHeader = header;
    }
    template <typename CloudT1, typename CloudT2>
    void pc2pc(typename CloudT1::Ptr& cloud_in_anytype, typename CloudT2::Ptr& cloud_out_normal) {  // :633-644
        NongroundExtractT::pc2pc<CloudT1>(cloud_in_anytype, cloud_out_normal);
    }
    void pubFeatureCloud() {                                                         // :691-707
        sensor_msgs::PointCloud2 b, p, f;
        pcl::toROSMsg(*cloud_beam, b);
        pcl::toROSMsg(*cloud_pillar, p);
        pcl::toROSMsg(*cloud_facade, f);
        b.header = p.header = f.header = cloudHeader;
        pubBeam.publish(b);
        pubPillar.publish(p);
        pubFacade.publish(f);
    }
    pointTypeCloud::Ptr featureSeginputCloudPtr;
    std_msgs::Header cloudHeader;
    ros::Publisher pubBeam, pubPillar, pubFacade;
    ros::NodeHandle nh_;
};

#endif  // PFILTER_HIP_PREPROCESS_HPP
