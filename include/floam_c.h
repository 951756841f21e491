/*
 * floam_c.h — C ABI of the MI355X-native FLOAM scan-to-map odometry core (libfloam_amd.so).
 *
 * Drop-in boundary for the reference operator API (dan11003/floam).  Each entry point names the reference
 * interface it replaces (file:line relative to the reference repo root).  Plain pointers and sizes only; no PCL,
 * Eigen, ROS or torch types cross this boundary.  The C++ adapters that restore the reference's exact class
 * signatures (LaserProcessingClass, OdomEstimationClass over pcl::PointCloud) are shown in INTEGRATION.md.
 *
 * Ownership: the caller owns host buffers.  floam_cloud / floam_lp / floam_odom handles own their device memory.
 * Threading: a handle is used from one host thread at a time (the reference drives each class from one worker
 * thread, src/odomEstimationNode.cpp:365, src/laserProcessingNode.cpp:212).  The odometry and feature-extraction
 * handles of one device issue their main work on one shared HIP stream (in issue order); a handle may add streams of
 * its own (the odometry's side stream for the first call's VoxelGrids, the asynchronous feature extraction's stream,
 * the one-call host entry points' copy stream), ordered with the shared stream by events, never by the caller.
 * Errors: every call returns floam_status; floam_last_error() gives a thread-local message.  Warnings
 * (status >= 100) are non-fatal and mirror the reference's printf diagnostics; the pose is then left where the
 * reference leaves it.
 */
#ifndef FLOAM_C_H
#define FLOAM_C_H

/* ABI revision of this header.  Bumped whenever an entry point's parameter list changes, so that a caller compiled
 * against an older header can refuse the library instead of passing arguments in the wrong slots:
 *   1  round 1-2 entry points
 *   2  floam_odom_keyframe_update gained the (surf, edge) cloud parameters of KeyFrameUpdate
 *      (include/odomEstimationClass.h:80); floam_abi_version added
 *   3  the one-call host entry points (floam_lp_feature_extraction_host, floam_odom_update_selector_host) and peer
 *      sharding (floam_odom_shard_exchange, floam_odom_set_shard_peers)
 * A caller checks `floam_abi_version() == FLOAM_ABI_VERSION` once after loading the library. */
#define FLOAM_ABI_VERSION 3

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum floam_status {
  FLOAM_OK = 0,
  FLOAM_ERR_INVALID_ARGUMENT = 1,
  FLOAM_ERR_DEVICE = 2,        /* HIP runtime / kernel launch failure, or no usable gfx950 device */
  FLOAM_ERR_OUT_OF_MEMORY = 3,
  FLOAM_ERR_UNSUPPORTED = 4,   /* input outside the kernels' envelope (e.g. more than 2^31 points) */
  FLOAM_ERR_COMM = 5,          /* RCCL failure in the sharded path */
  /* non-fatal, same conditions as the reference's printf warnings */
  FLOAM_WARN_MAP_TOO_SMALL = 100,       /* src/odomEstimationClass.cpp:112 "not enough points in map" */
  FLOAM_WARN_FEW_CORRESPONDENCES = 101, /* src/odomEstimationClass.cpp:192-194, 247-249 (< 20 factors) */
  FLOAM_WARN_NO_IMU_DATA = 102,         /* src/dataHandler.cpp:101-104 "no imu data" (Compensate returns false) */
  FLOAM_WARN_FIELD_MISSING = 103        /* PCL fromPCLPointCloud2 "Failed to find match for field" (the field stays 0) */
} floam_status;

/* 32-byte point record, byte-compatible with vel_point::PointXYZIRT (include/lidar.h:14-32) and with
 * pcl::PointXYZI (x,y,z,intensity at the same offsets); padding is written as pad0 = 1.0f, pad1 = pad2 = 0. */
typedef struct floam_point {
  float x, y, z, pad0;
  float intensity;
  uint16_t ring;
  uint16_t pad1;
  float time;
  float pad2;
} floam_point;

/* lidar::Lidar (include/lidar.h:53-85): the fields the path reads. */
typedef struct floam_lidar_params {
  int num_lines;          /* /scan_line  -> N_SCANS (src/laserProcessingClass.cpp:78) */
  double scan_period;     /* /scan_period (GetVelocity, include/odomEstimationClass.h:78) */
  double vertical_angle;  /* /vertical_angle (not used on the path) */
  double max_distance;    /* /max_dis (src/laserProcessingClass.cpp:15) */
  double min_distance;    /* /min_dis */
} floam_lidar_params;

/* OdomEstimationClass::UpdateType (include/odomEstimationClass.h:56) */
enum { FLOAM_VANILLA = 0, FLOAM_INITIAL_ITERATION = 1, FLOAM_REFINEMENT_AND_UPDATE = 2 };

/* ------------------------------------------------------------------------------------------ device clouds */
/* A device-resident point cloud (HBM), the stand-in for pcl::PointCloud<PointXYZIRT|PointXYZI>::Ptr.
 * Its element count lives on the device; floam_cloud_size() synchronises to read it. */
typedef struct floam_cloud floam_cloud;

floam_status floam_cloud_create(int device, size_t capacity, floam_cloud** out);
floam_status floam_cloud_destroy(floam_cloud* c);
/* Replace the contents with n host points of `stride` bytes each (x,y,z,pad,intensity,ring,pad,time at the
 * PointXYZIRT offsets; stride 32 = a pcl::PointCloud's points.data()).  Replaces pcl::fromROSMsg + copy. */
floam_status floam_cloud_upload(floam_cloud* c, const void* host_points, size_t n, size_t stride);
/* Copy up to `capacity` points to host (32-B records); *n_out = number of points in the cloud. Synchronises. */
floam_status floam_cloud_download(const floam_cloud* c, void* host_points, size_t capacity, size_t* n_out);
floam_status floam_cloud_size(const floam_cloud* c, size_t* n_out);
floam_status floam_cloud_clear(floam_cloud* c);
floam_status floam_cloud_copy(floam_cloud* dst, const floam_cloud* src);   /* device to device */
void* floam_cloud_device_ptr(floam_cloud* c);                              /* 32-B records in HBM */

/* ------------------------------------------------------------------------------- LaserProcessingClass */
typedef struct floam_lp floam_lp;

/* LaserProcessingClass() + init(lidar::Lidar) (include/laserProcessingClass.h:37-39) */
floam_status floam_lp_create(const floam_lidar_params* p, int device, floam_lp** out);
floam_status floam_lp_destroy(floam_lp* lp);
/* featureExtraction(pc_in, pc_out_edge, pc_out_surf) (include/laserProcessingClass.h:40,
 * src/laserProcessingClass.cpp:72-118).  Appends to edge/surf like the reference (never clears them). */
floam_status floam_lp_feature_extraction(floam_lp* lp, const floam_cloud* in, floam_cloud* edge, floam_cloud* surf);
/* The same for host-resident clouds (the drop-in adapter's path: the node hands PCL clouds in and publishes PCL
 * clouds): `in` = n PointXYZIRT records (stride 32, e.g. pcl::PointCloud::points.data()); the edge / surf features
 * are WRITTEN (not appended) to the caller's arrays of capacity edge_cap / surf_cap records and their counts returned
 * (the adapter appends by passing the ends of its vectors, resized by the bounds num_lines * 120 and n).  One upload,
 * the extraction and both downloads with a single synchronisation.  FLOAM_ERR_INVALID_ARGUMENT if a capacity is
 * short (nothing written). */
floam_status floam_lp_feature_extraction_host(floam_lp* lp, const void* in, size_t n, size_t stride, void* edge,
                                              size_t edge_cap, size_t* n_edge, void* surf, size_t surf_cap,
                                              size_t* n_surf);
/* pcl::VoxelGrid<PointXYZI> with a cubic leaf (PCL 1.8.1 semantics; the filter of downSamplingToMap,
 * src/odomEstimationClass.cpp:137-142, and of the mapping node, src/laserMappingClass.cpp:174-183): one centroid
 * of x, y, z, intensity per occupied voxel in ascending voxel index, the input returned unchanged when the index
 * range overflows int.  Within-voxel summation in input order.  out is overwritten; asynchronous. */
floam_status floam_voxel_grid(const floam_cloud* in, float leaf, floam_cloud* out);
/* Asynchronous mode (extension, default off): featureExtraction returns without synchronising; the output counts
 * stay on the device (the odometry sizes its work from upper bounds) and the input-validation flags travel with
 * the output clouds, so an out-of-range ring or an over-long sector is reported by the next odometry update that
 * consumes them, or by floam_lp_wait. */
floam_status floam_lp_set_async(floam_lp* lp, int async);
floam_status floam_lp_wait(floam_lp* lp);

/* ------------------------------------------------------------------------------- IMU pre-processing */
/* The laser-processing node's steps before featureExtraction (src/laserProcessingNode.cpp:92-120; SURVEY.md §8
 * f-2).  Quaternions are (x, y, z, w), the coefficient order of Eigen::Quaterniond and of
 * sensor_msgs::Imu::orientation.  Stamps are seconds (ros::Time::toSec()); cloud stamps are PCL header stamps in
 * microseconds (pcl::PCLHeader::stamp). */
typedef struct floam_imu floam_imu;

/* dmapping::ImuHandler() (include/dataHandler.h:35) on `device` */
floam_status floam_imu_create(int device, floam_imu** out);
floam_status floam_imu_destroy(floam_imu* h);
/* ImuHandler::AddMsg (src/dataHandler.cpp:23-38): appended iff the handler is empty or stamp > last + 1e-5 s.
 * Only the orientation is kept (Imu2Orientation, :7-9, is the only accessor the path uses). *added may be NULL. */
floam_status floam_imu_add_msg(floam_imu* h, double stamp, const double orientation_xyzw[4], int* added);
floam_status floam_imu_add_msgs(floam_imu* h, const double* stamps, const double* orientations_xyzw, size_t n,
                                size_t* added);
floam_status floam_imu_size(const floam_imu* h, size_t* n);
/* ImuHandler::Get (src/dataHandler.cpp:48-75): the sample before std::lower_bound(stamp) (no interpolation, :45-47);
 * not found -> *found = 0 and the zero orientation of a default-constructed sensor_msgs::Imu. */
floam_status floam_imu_get(const floam_imu* h, double stamp, double orientation_xyzw[4], int* found);
/* ImuHandler::TimeContained (src/dataHandler.cpp:76-81) */
floam_status floam_imu_time_contained(const floam_imu* h, double stamp, int* contained);
/* euler2Quaternion(roll, pitch, yaw) in degrees (src/lidar.cpp:8-16): AngleAxis roll * yaw * pitch */
floam_status floam_euler_to_quaternion(double roll, double pitch, double yaw, double q_xyzw[4]);
/* CenterTime(cloud) (src/laserProcessingNode.cpp:65-78): point times re-referenced to the centre of
 * [front.time, back.time] in place; *stamp_us is replaced by the centre stamp (microsecond PCL stamp).  One 12-B
 * read-back of the cloud's ends; an empty cloud is left untouched (points.back() of an empty cloud is UB there). */
floam_status floam_center_time(floam_cloud* cloud, uint64_t* stamp_us);
/* dmapping::Compensate(input, compensated, handler, extrinsics) (src/dataHandler.cpp:93-122): every point rotated by
 * (q(Get(stamp)) * extr)^-1 * (q(Get(stamp + time)) * extr).  Returns FLOAM_WARN_NO_IMU_DATA (the reference returns
 * false) when the front or back point time is outside the IMU stream; `compensated` is then left unchanged. */
floam_status floam_imu_compensate(floam_imu* h, floam_cloud* in, uint64_t stamp_us, const double extrinsics_xyzw[4],
                                  floam_cloud* compensated);
/* The node's whole sequence, fused into one pass (src/laserProcessingNode.cpp:92-113): CenterTime(in) (in place,
 * *stamp_us updated), Compensate, then pcl::transformPointCloud by Eigen::Affine3d(q(Get(stamp)) * extr) into
 * `aligned`, the cloud featureExtraction receives.  FLOAM_WARN_NO_IMU_DATA: the node's "cannot compensate" skip
 * (:104-107); `in` is centred regardless and `aligned` is unchanged. */
floam_status floam_imu_preprocess(floam_imu* h, floam_cloud* in, uint64_t* stamp_us, const double extrinsics_xyzw[4],
                                  floam_cloud* aligned);

/* ---------------------------------------------------------------------------------------- wire formats */
/* sensor_msgs/PointField (name, offset, datatype, count); datatype codes as PointField: UINT16 = 4, FLOAT32 = 7. */
typedef struct floam_pc2_field {
  char name[32];
  uint32_t offset;
  uint8_t datatype;
  uint32_t count;
} floam_pc2_field;
enum { FLOAM_POINT_XYZIRT = 0, FLOAM_POINT_XYZI = 1 };
/* The field table pcl::toROSMsg writes for vel_point::PointXYZIRT (x, y, z, intensity, ring, time) or pcl::PointXYZI
 * (x, y, z, intensity) with point_step 32; the message data is then floam_cloud_download's 32-B records
 * (row_step = 32 * width, height 1).  Used for /laser_cloud_edge, /laser_cloud_surf (src/laserProcessingNode.cpp:
 * 145-155) and /scan_registered (src/odomEstimationNode.cpp:273). */
floam_status floam_pointcloud2_fields(int point_type, floam_pc2_field* out, size_t capacity, size_t* n_out,
                                      uint32_t* point_step);
/* pcl::fromROSMsg(msg, cloud) (pcl_conversions + PCL 1.8.1 fromPCLPointCloud2), the decode at
 * src/laserProcessingNode.cpp:89 and src/odomEstimationNode.cpp:205-206: fields matched by name, datatype and count,
 * adjacent fields coalesced, bytes copied per point (row-major over height x width, row_step / point_step strides),
 * unmatched struct bytes zero; a single coalesced mapping at offset 0 with point_step 32 copies whole records.
 * The bytes are staged through HBM and decoded on the device; `out` is replaced.  FLOAM_WARN_FIELD_MISSING when a
 * point field has no match (PCL only warns). */
floam_status floam_cloud_from_pointcloud2(floam_cloud* out, int point_type, const void* data, size_t data_size,
                                          uint32_t width, uint32_t height, uint32_t point_step, uint32_t row_step,
                                          const floam_pc2_field* fields, size_t nfields);
/* pcl::transformPointCloud(in, out, Eigen::Affine3d T) (PCL 1.8.1 transforms.hpp, dense path): x' =
 * float(((T00 x + T01 y) + T02 z) + T03) in double; other fields copied.  m = row-major 4x4; in == out allowed.
 * SaveMerged's per-keyframe transform (src/odomEstimationNode.cpp:72-76). */
floam_status floam_transform_cloud(const floam_cloud* in, const double m[16], floam_cloud* out);

/* Disk exporters of the odometry node (src/utils.cpp:3-106, src/odomEstimationNode.cpp:66-117), for the C++ nodes.
 * poses: n row-major 4x4 Eigen::Affine3d matrices; clouds: n host arrays of pcl::PointXYZI-compatible 32-B records
 * (cloud_sizes points each); stamps in seconds (ros::Time::toSec()).  Text is written through std::ostream exactly
 * as the reference does; PCD files are pcl::io::savePCDFileBinary of pcl::PointXYZI (v0.7, x y z intensity). */
floam_status floam_save_pcd(const char* path, const floam_point* points, size_t n);
/* SaveOdom (src/utils.cpp:80-106): <dir>/<sec>_<nsec>.pcd and .odom per keyframe */
floam_status floam_save_odom(const char* dump_directory, const double* poses, const double* keyframe_stamps,
                             const floam_point* const* clouds, const size_t* cloud_sizes, size_t n);
/* SavePosegraph (src/utils.cpp:3-75): graph.g2o + <dir>/%06d/{cloud.pcd, data} */
floam_status floam_save_posegraph(const char* dump_directory, const double* poses, const double* keyframe_stamps,
                                  const floam_point* const* clouds, const size_t* cloud_sizes, size_t n);
/* SavePosesHomogeneousBALM (src/odomEstimationNode.cpp:97-117): <dir>alidarPose.csv + <dir>full<i>.pcd (the
 * directory string is concatenated as the reference does: pass a trailing '/') */
floam_status floam_save_poses_balm(const char* directory, const double* poses, const double* stamps,
                                   const floam_point* const* clouds, const size_t* cloud_sizes, size_t n);
/* SaveMerged (src/odomEstimationNode.cpp:66-96): every cloud transformed by its pose (on the device), concatenated to
 * <dir>floam_merged.pcd, VoxelGrid(downsample_size) to <dir>floam_merged_downsampled_leaf_<size>.pcd */
floam_status floam_save_merged(const char* directory, const double* poses, const floam_point* const* clouds,
                               const size_t* cloud_sizes, size_t n, double downsample_size, int device);

/* ------------------------------------------------------------------------------- LaserMappingClass */
/* The mapping node's global map (src/laserMappingClass.cpp): 50-m cells of pcl::PointXYZI,
 * VoxelGrid(map_resolution) of the 5 x 5 x 5 cells around the pose after every update. */
typedef struct floam_mapping floam_mapping;
/* LaserMappingClass() + init(map_resolution) (src/laserMappingClass.cpp:7-32) */
floam_status floam_mapping_create(double map_resolution, int device, floam_mapping** out);
floam_status floam_mapping_destroy(floam_mapping* m);
/* updateCurrentPointsToMap(pc_in, pose_current) (src/laserMappingClass.cpp:148-186), the pose as the node builds it
 * from /odom (Isometry3d::Identity().rotate(q).pretranslate(t), src/laserMappingNode.cpp:108-110): points
 * transformed by pose.cast<float>(), intensity = min(1, max(z_in + 2, 0) / 5), appended to their cells, then the
 * neighbourhood's cells voxel-filtered in place.  Points beyond the reference's allocated cells (out of bounds
 * there) are kept in their cells.  Two synchronisations. */
floam_status floam_mapping_update(floam_mapping* m, const floam_cloud* pc_in, const double q_xyzw[4], const double t[3]);
/* getMap() (src/laserMappingClass.cpp:188-200): every cell's points in (x, y, z) cell order; `out` is replaced. */
floam_status floam_mapping_get_map(floam_mapping* m, floam_cloud* out);
floam_status floam_mapping_size(const floam_mapping* m, size_t* n);

/* -------------------------------------------------------------------------------- OdomEstimationClass */
typedef struct floam_odom floam_odom;

/* OdomEstimationClass() + init(lidar, map_resolution, loss_function) (include/odomEstimationClass.h:58-60,
 * src/odomEstimationClass.cpp:7-26).  loss "huber" (any case) -> HuberLoss(0.1); anything else -> no loss (Q3). */
floam_status floam_odom_create(const floam_lidar_params* p, double map_resolution, const char* loss_function,
                               int device, floam_odom** out);
floam_status floam_odom_destroy(floam_odom* o);
/* initMapWithPoints(edge_in, surf_in) (src/odomEstimationClass.cpp:28-32): raw append, optimization_count = 12 */
floam_status floam_odom_init_map(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf);
/* UpdatePointsToMapSelector(edge_in, surf_in, deskew) (src/odomEstimationClass.cpp:34-50).  With deskew the
 * clouds are velocity-compensated IN PLACE, as the reference does (Q5). */
floam_status floam_odom_update_selector(floam_odom* o, floam_cloud* edge, floam_cloud* surf, int deskew);
/* The same for host-resident clouds (the drop-in adapter: UpdatePointsToMapSelector on the node's PCL clouds, stride
 * 32 records): both clouds uploaded, the update run synchronously, and with deskew the compensated records copied
 * back into the caller's arrays (Q5) on a copy stream as soon as the deskew kernel has run — overlapped with the
 * update's second call — instead of 2 uploads + the update + 2 size queries + 2 downloads. */
floam_status floam_odom_update_selector_host(floam_odom* o, void* edge, size_t n_edge, void* surf, size_t n_surf,
                                             size_t stride, int deskew);
/* updatePointsToMap(edge_in, surf_in, update_type) (src/odomEstimationClass.cpp:52-124) */
floam_status floam_odom_update(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf, int update_type);
/* Streaming mode (no reference counterpart: the reference's odometry node processes one scan per callback,
 * src/odomEstimationNode.cpp:222-244).  depth > 0: update / update_selector only issue the device work (the whole
 * controller runs on the device) and keep up to `depth` updates in flight; their warnings, errors and poses are
 * collected by floam_odom_wait, and get_pose / get_last_pose / get_stats report the last collected update.
 * depth 0 (default): every update synchronises and returns its own warning, as the reference's calls do. */
floam_status floam_odom_set_async(floam_odom* o, int depth);
/* Collect in-flight updates until at most max_pending remain.  Writes the pose {qx,qy,qz,qw,tx,ty,tz} of every
 * update collected since the previous call (in issue order) to poses[0..min(n, capacity)) and n to *n_out.
 * Returns the first device error, else the last warning among them. */
floam_status floam_odom_wait(floam_odom* o, size_t max_pending, double* poses, size_t capacity, size_t* n_out);
/* public member `odom` (include/odomEstimationClass.h:84): quaternion (x,y,z,w) + translation */
floam_status floam_odom_get_pose(const floam_odom* o, double q_xyzw[4], double t[3]);
floam_status floam_odom_get_last_pose(const floam_odom* o, double q_xyzw[4], double t[3]);
/* GetVelocity() (include/odomEstimationClass.h:78) */
floam_status floam_odom_get_velocity(const floam_odom* o, double v[3]);
/* getMap(laserCloudMap) (src/odomEstimationClass.cpp:296-300): appends surf map then corner map */
floam_status floam_odom_get_map(floam_odom* o, floam_cloud* out);
/* public members laserCloudCornerMap / laserCloudSurfMap (include/odomEstimationClass.h:86-87) */
floam_status floam_odom_get_map_sizes(floam_odom* o, size_t* corner, size_t* surf);
floam_status floam_odom_download_maps(floam_odom* o, void* corner, size_t corner_cap, void* surf, size_t surf_cap);

typedef struct floam_odom_stats {
  int optimization_count;       /* value used by the last updatePointsToMap */
  int solves;                   /* outer iterations (one ceres::Solve each) in the last call */
  int edge_queries, surf_queries;       /* after VoxelGrid */
  int edge_correspondences, surf_correspondences;   /* accepted factors in the last outer iteration */
  int lm_iterations;            /* trust-region iterations of the last solve */
  int map_updated;              /* KeyFrameUpdate() returned true */
  size_t corner_map, surf_map;  /* map sizes after the call */
  double final_cost;
} floam_odom_stats;
floam_status floam_odom_get_stats(const floam_odom* o, floam_odom_stats* s);

/* bool KeyFrameUpdate(PointCloud<PointXYZI>::Ptr surf_cloud, PointCloud<PointXYZI>::Ptr edge_cloud,
 *                     const Eigen::Isometry3d& pose)   (include/odomEstimationClass.h:80, src/odomEstimationClass.cpp:320-343)
 * Public in the reference's header; updatePointsToMap calls it internally (:118), and the process-wide `first` flag
 * of Q6 is shared with those calls.  *is_keyframe = 1 when the pose moved > 0.07 m or turned > 2 deg from the last
 * keyframe (or on the process's first call).  A keyframe joins the 3-deep history keyframes_ (:326, :334-337) with
 * device copies of surf_cloud / edge_cloud (either may be NULL, a null Ptr in the reference). */
floam_status floam_odom_keyframe_update(floam_odom* o, const floam_cloud* surf_cloud, const floam_cloud* edge_cloud,
                                        const double q_xyzw[4], const double t[3], int* is_keyframe);
/* Inspection of the keyframe history keyframes_ (private in the reference, include/odomEstimationClass.h:117; for
 * tests): *n_keyframes = its size; entry `index` (0 = oldest): pose and copies of its clouds.  Entries made by the
 * updates themselves carry the pose only (their clouds come back empty). Every output may be NULL. */
floam_status floam_odom_get_keyframe(floam_odom* o, size_t index, double q_xyzw[4], double t[3], floam_cloud* surf_out,
                                     floam_cloud* edge_out, size_t* n_keyframes);

/* Precision of the residual / Jacobian evaluation and of the correspondence geometry (extension: BASELINE.json
 * configs[4], the fp32 vs fp64 Jacobian tolerance sweep).  FLOAM_PRECISION_FP64 (default) computes in double like
 * the reference (src/odomEstimationClass.cpp:156-243, src/lidarOptimization.cpp:12-74); the solve's residuals,
 * Jacobians and control step use fused multiply-adds, so they differ from the reference's unfused arithmetic by ulps.
 * FLOAM_PRECISION_FP32: residuals, Jacobians and the per-thread J^T J / J^T r sums in float; the line / plane fits,
 * the cross-thread reductions and the LM control stay in double.  FLOAM_PRECISION_FP32_GEOMETRY: additionally the
 * line (eigen) and plane (QR) fits in float.  Measured deviations from the fp64 solution: DESIGN.md §4. */
enum { FLOAM_PRECISION_FP64 = 0, FLOAM_PRECISION_FP32 = 1, FLOAM_PRECISION_FP32_GEOMETRY = 2 };
floam_status floam_odom_set_precision(floam_odom* o, int precision);

/* Stage inspection (extension, for parity tests against the CPU restatement).  floam_odom_set_trace(o, capacity):
 * capacity > 0 records one 49-double record per ceres::Solve (oracle/odom.cpp SolveTrace order: edge queries, surf
 * queries, edge factors, surf factors, iterations, successful steps, initial cost, final cost, x_in[7], x_out[7],
 * J^T J at x_in (upper, row-major, 21), J^T r at x_in (6)) and keeps the last correspondence pass's neighbour indices
 * and squared distances; 0 turns it off.  floam_odom_get_traces copies min(n, capacity, trace capacity) records and
 * clears them; *n_out = n, the number of solves since the last call, so n_out > capacity (or > the set_trace
 * capacity) signals that records were dropped. */
floam_status floam_odom_set_trace(floam_odom* o, size_t capacity);
floam_status floam_odom_get_traces(floam_odom* o, double* out /* capacity x 49 */, size_t capacity, size_t* n_out);
/* One correspondence pass at an explicit pose, without a solve (the map and the odometry state are untouched):
 * downSamplingToMap of edge / surf, pointAssociateToMap at (q, t), the 5-NN search with the sqd[4] < 1 gate and the
 * addEdgeCostFactor / addSurfCostFactor geometry (src/odomEstimationClass.cpp:137-142, 126-135, 144-251); read the
 * result with floam_odom_get_correspondences.  Needs tracing on. */
floam_status floam_odom_find_correspondences(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf,
                                             const double q_xyzw[4], const double t[3]);
/* The last correspondence pass of set `which` (0 edge / corner map, 1 surf / surf map): the downsampled queries
 * (32-B records, sensor frame), per query flags (bit 0 accepted factor, bit 2 five neighbours with sqd < 1), the 5
 * neighbours' map indices and float squared distances (row-major n x 5; valid when bit 2 is set) and the factor
 * records (edge: cp, a, b = 9 doubles; surf: cp, n, d = 7 doubles; valid when bit 0 is set).  Any output may be NULL.
 * The indices / distances exist only for a pass that ran with tracing on: asking for them after an untraced pass
 * fails with FLOAM_ERR_INVALID_ARGUMENT (no stale values of an earlier pass). */
floam_status floam_odom_get_correspondences(floam_odom* o, int which, void* queries, uint8_t* flags, int* idx,
                                            float* sqd, double* records, size_t capacity, size_t* n_out);

/* Query sharding over ranks (one process per GPU): each rank runs the same calls on the same scans; the
 * correspondence queries are split into `world` contiguous ranges and the normal equations (J^T J, J^T r, cost)
 * are summed with one RCCL all-reduce per LM evaluation.  unique_id: 128 bytes from floam_comm_unique_id() on
 * rank 0, broadcast by the caller (e.g. torch.distributed).  world = 1 with a unique id runs the sharded path through
 * a one-rank RCCL communicator (agrees with the unsharded solve to a few ulps; identical LM decisions). */
floam_status floam_comm_unique_id(void* unique_id_128);
floam_status floam_odom_set_shard(floam_odom* o, int rank, int world, const void* unique_id_128);
/* Same sharding with a caller-supplied host all-reduce instead of RCCL (in-place sum of `count` doubles over all
 * ranks, return 0 on success), e.g. torch.distributed/gloo.  Used to validate the sharded path when RCCL cannot
 * run (several ranks on one GPU); synchronises once per LM evaluation. */
typedef int (*floam_allreduce_fn)(double* values, int count, void* user);
floam_status floam_odom_set_shard_callback(floam_odom* o, int rank, int world, floam_allreduce_fn fn, void* user);
/* Peer sharding (ABI 3): the same query partition, but the LM solve stays ONE resident launch per ceres::Solve
 * (src/odomEstimationClass.cpp:100-108): each rank publishes its 29 sums per LM evaluation into a 4-KB exchange buffer
 * on its own GPU and reads every rank's buffer through peer mappings (xGMI), summing them in rank order — no
 * collective launch, no host round trip; every rank takes the same LM decisions.  A rank that never publishes ends
 * the solve after ~20 s with FLOAM_ERR_DEVICE (the handle is then poisoned).
 *   floam_odom_shard_exchange: this rank's buffer as an IPC handle (64 bytes, for the other processes) and/or as a
 *   device pointer (for handles in the same process).
 *   floam_odom_set_shard_peers: every rank's buffer, either as world x 64 bytes of IPC handles (entry `rank` is not
 *   opened) or as world device pointers; exactly one of the two.  world <= 8.  It starts a fresh exchange sequence
 *   (the rank's exchange counter reset, its buffer zeroed), so every rank calls it — also when re-peering — and the
 *   ranks then meet at a barrier before their next update; from there on all ranks issue the same sequence of
 *   updates concurrently.  The ranks call it together (one process per rank, or one host thread per rank on
 *   different GPUs): it probes every peer mapping — each rank publishes a word in its own buffer and reads every
 *   rank's — and returns FLOAM_ERR_COMM when a rank does not answer within 2 s (the xGMI mapping does not work: use
 *   floam_odom_set_shard, RCCL, instead), so a bad node costs seconds, not the first solve's ~20-s timeout.  Handles
 *   of one process on the SAME GPU cannot be peers: they share that GPU's library stream, so one rank's solve would
 *   wait for a rank queued behind it.  FLOAM_ERR_UNSUPPORTED when uncached device memory (which the cross-GPU polls
 *   need) cannot be allocated.  On any error the handle is left unsharded (world 1), never half-configured. */
floam_status floam_odom_shard_exchange(floam_odom* o, void* ipc_handle_64, void** dev_ptr);
floam_status floam_odom_set_shard_peers(floam_odom* o, int rank, int world, const void* ipc_handles,
                                        void* const* dev_ptrs);

/* ------------------------------------------------------------------------------------------ misc */
const char* floam_last_error(void);
const char* floam_version(void);
int floam_abi_version(void);   /* FLOAM_ABI_VERSION the library was built with */
/* KeyFrameUpdate keeps a function-static `first` flag shared by every instance in the process
 * (src/odomEstimationClass.cpp:323, quirk Q6); this resets it (tests/bench only). */
void floam_reset_process_state(void);
floam_status floam_device_synchronize(int device);

/* Per-kernel timing with HIP events recorded on the library stream (bench.py's roofline leg).
 * floam_profile_enable(device, mask): mask = OR of the categories below (0 disables).
 * FLOAM_PROF_KNN_BYTES adds an extra (non-product) kernel after each correspondence launch that counts its
 * algorithmic bytes; it is kept out of timed runs and used on an identical replay instead. */
enum { FLOAM_PROF_KNN = 1, FLOAM_PROF_LM = 2, FLOAM_PROF_CLOUD = 4, FLOAM_PROF_FE = 8, FLOAM_PROF_KNN_BYTES = 16,
       FLOAM_PROF_KNN_DETAIL = 32 /* separate search / geometry timers (each event pair perturbs the timeline) */,
       FLOAM_PROF_ALL = 0xEF };
typedef struct floam_kernel_timing {
  char name[32];
  long long launches;
  double total_ms;
  double algorithmic_bytes;   /* sum over launches of the algorithmic byte count */
} floam_kernel_timing;
floam_status floam_profile_enable(int device, int enable);
floam_status floam_profile_read(int device, floam_kernel_timing* out, int max_entries, int* n_out);
floam_status floam_profile_reset(int device);
/* One do-nothing dispatch (kernel `floam_profile_marker`) on the device's library stream: brackets a region of a
 * rocprofv3 kernel trace (bench.py marks its timed region; tools/prof_summary.py keeps the dispatches between). */
floam_status floam_profile_mark(int device, int id);

#ifdef __cplusplus
}
#endif
#endif /* FLOAM_C_H */
