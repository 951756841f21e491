// CPU ORACLE (test infrastructure) — flat C entry points for ctypes (tests/, smoke(), bench.py cpu_baseline).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "la.hpp"
#include "oracle.hpp"

using namespace oracle;

extern "C" {

int oracle_feature_extraction(int num_lines, double min_dis, double max_dis, const void* in, size_t n, int canonical,
                              void* edge_out, size_t* ne, void* surf_out, size_t* ns, size_t stats[2]) {
  LidarParams lp{num_lines, 0.1, min_dis, max_dis};
  std::vector<Pt> e, s;
  FeStats st;
  feature_extraction(lp, static_cast<const Pt*>(in), n, e, s, canonical != 0, &st);
  if (e.size() > *ne || s.size() > *ns) return -1;
  std::memcpy(edge_out, e.data(), e.size() * sizeof(Pt));
  std::memcpy(surf_out, s.data(), s.size() * sizeof(Pt));
  *ne = e.size();
  *ns = s.size();
  if (stats) {
    stats[0] = st.out_of_range_rings;
    stats[1] = st.sector_ties;
  }
  return 0;
}

int oracle_voxel_grid(const void* in, size_t n, float leaf, int stable, void* out, size_t* nout) {
  std::vector<Pt> o;
  voxel_grid(static_cast<const Pt*>(in), n, leaf, stable != 0, o);
  if (o.size() > *nout) return -1;
  std::memcpy(out, o.data(), o.size() * sizeof(Pt));
  *nout = o.size();
  return 0;
}

int oracle_crop_box(const void* in, size_t n, const float mn[3], const float mx[3], void* out, size_t* nout) {
  std::vector<Pt> o;
  crop_box(static_cast<const Pt*>(in), n, mn, mx, o);
  if (o.size() > *nout) return -1;
  std::memcpy(out, o.data(), o.size() * sizeof(Pt));
  *nout = o.size();
  return 0;
}

// queries: n x 3 floats; idx/sqd: n x k
void oracle_knn(const void* map, size_t m, const float* queries, size_t nq, int k, int* idx, float* sqd) {
  KdTree kd;
  kd.build(static_cast<const Pt*>(map), m);
  for (size_t i = 0; i < nq; ++i) kd.knn(queries + 3 * i, k, idx + (size_t)k * i, sqd + (size_t)k * i);
}

void oracle_eig_sym3(const double* a9, double* eval3, double* evec9 /* column-major */) {
  M3 A;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) A.m[r][c] = a9[3 * r + c];
  double ev[3], vec[3][3];
  eig_sym3(A, ev, vec);
  for (int i = 0; i < 3; ++i) {
    eval3[i] = ev[i];
    for (int r = 0; r < 3; ++r) evec9[3 * i + r] = vec[i][r];
  }
}

void oracle_plane_solve(const double* a15, double* x3) {
  double A[5][3], b[5];
  for (int r = 0; r < 5; ++r) {
    for (int c = 0; c < 3; ++c) A[r][c] = a15[3 * r + c];
    b[r] = -1.0;
  }
  colpiv_qr_solve_5x3(A, b, x3);
}

void* oracle_odom_create(int num_lines, double scan_period, double min_dis, double max_dis, double map_res,
                         const char* loss, int stable_voxel) {
  LidarParams lp{num_lines, scan_period, min_dis, max_dis};
  return odom_create(lp, map_res, std::string(loss ? loss : ""), stable_voxel != 0);
}
void oracle_odom_destroy(void* h) { odom_destroy(static_cast<OdomState*>(h)); }
void oracle_odom_init_map(void* h, const void* e, size_t ne, const void* s, size_t ns) {
  odom_init_map(static_cast<OdomState*>(h), static_cast<const Pt*>(e), ne, static_cast<const Pt*>(s), ns);
}
void oracle_odom_update_selector(void* h, void* e, size_t ne, void* s, size_t ns, int deskew) {
  odom_update_selector(static_cast<OdomState*>(h), static_cast<Pt*>(e), ne, static_cast<Pt*>(s), ns, deskew != 0);
}
void oracle_odom_update(void* h, const void* e, size_t ne, const void* s, size_t ns, int type) {
  odom_update(static_cast<OdomState*>(h), static_cast<const Pt*>(e), ne, static_cast<const Pt*>(s), ns,
              static_cast<UpdateType>(type));
}
void oracle_odom_get_pose(void* h, double* q, double* t) { odom_get_pose(static_cast<OdomState*>(h), q, t); }
void oracle_odom_get_last_pose(void* h, double* q, double* t) {
  odom_get_last_pose(static_cast<OdomState*>(h), q, t);
}
void oracle_odom_get_velocity(void* h, double* v) { odom_get_velocity(static_cast<OdomState*>(h), v); }
size_t oracle_odom_map_size(void* h, int which) { return odom_map_size(static_cast<OdomState*>(h), which); }
void oracle_odom_get_map(void* h, int which, void* out) {
  OdomState* s = static_cast<OdomState*>(h);
  std::memcpy(out, odom_map_data(s, which), odom_map_size(s, which) * sizeof(Pt));
}
int oracle_odom_optimization_count(void* h) { return odom_optimization_count(static_cast<OdomState*>(h)); }
size_t oracle_odom_num_traces(void* h) { return odom_traces(static_cast<OdomState*>(h)).size(); }
// trace record: 4 ints + 2 ints + 2 doubles + 7 + 7 + 21 + 6 doubles, flattened as doubles (ints as doubles)
void oracle_odom_get_trace(void* h, size_t i, double* out /* 49 */) {
  const SolveTrace& t = odom_traces(static_cast<OdomState*>(h))[i];
  int k = 0;
  out[k++] = t.n_edge_queries; out[k++] = t.n_surf_queries; out[k++] = t.n_edge_corr; out[k++] = t.n_surf_corr;
  out[k++] = t.iterations; out[k++] = t.successful; out[k++] = t.initial_cost; out[k++] = t.final_cost;
  for (int j = 0; j < 7; ++j) out[k++] = t.x_in[j];
  for (int j = 0; j < 7; ++j) out[k++] = t.x_out[j];
  for (int j = 0; j < 21; ++j) out[k++] = t.H0[j];
  for (int j = 0; j < 6; ++j) out[k++] = t.g0[j];
}
void oracle_odom_clear_traces(void* h) { odom_clear_traces(static_cast<OdomState*>(h)); }
void oracle_stage_correspondences(const void* map, size_t m, const void* q, size_t nq, const double* x, int edge,
                                  int* idx, float* sqd, unsigned char* flags, double* rec) {
  stage_correspondences(static_cast<const Pt*>(map), m, static_cast<const Pt*>(q), nq, x, edge != 0, idx, sqd, flags,
                        rec);
}
void oracle_stage_associate(const void* in, size_t n, const double* x, void* out) {
  stage_associate(static_cast<const Pt*>(in), n, x, static_cast<Pt*>(out));
}
void oracle_stage_solve(const double* erec, size_t ne, const double* srec, size_t ns, int huber, double* x,
                        double* trace) {
  stage_solve(erec, ne, srec, ns, huber != 0, x, trace);
}
void oracle_reset_process_statics() { reset_process_statics(); }

double oracle_edge_residual(const double* cp, const double* a, const double* b, const double* x, double* J) {
  return test_edge_eval(cp, a, b, x, J);
}
double oracle_surf_residual(const double* cp, const double* n, double d, const double* x, double* J) {
  return test_surf_eval(cp, n, d, x, J);
}
void oracle_se3_plus(const double* x, const double* delta, double* out) { test_se3_plus(x, delta, out); }

// ---- IMU pre-processing (oracle/imu.cpp).  Quaternions are (x, y, z, w); handler data is passed as arrays.
static ImuHandler make_handler(const double* stamps, const double* q_xyzw, size_t m) {
  ImuHandler h;
  for (size_t i = 0; i < m; ++i)
    h.add_msg(stamps[i], Quat{q_xyzw[4 * i], q_xyzw[4 * i + 1], q_xyzw[4 * i + 2], q_xyzw[4 * i + 3]});
  return h;
}
// AddMsg over a message stream: keep[i] = 1 if message i was appended
size_t oracle_imu_filter(const double* stamps, size_t m, unsigned char* keep) {
  ImuHandler h;
  for (size_t i = 0; i < m; ++i) keep[i] = h.add_msg(stamps[i], Quat{0, 0, 0, 1}) ? 1 : 0;
  return h.t.size();
}
int oracle_imu_get(const double* stamps, const double* q_xyzw, size_t m, double ts, double* out_xyzw) {
  const ImuHandler h = make_handler(stamps, q_xyzw, m);
  const Quat r = h.get_or_zero(ts);
  out_xyzw[0] = r.x; out_xyzw[1] = r.y; out_xyzw[2] = r.z; out_xyzw[3] = r.w;
  Quat tmp;
  return h.get(ts, &tmp) ? 1 : 0;
}
int oracle_imu_time_contained(const double* stamps, const double* q_xyzw, size_t m, double ts) {
  return make_handler(stamps, q_xyzw, m).time_contained(ts) ? 1 : 0;
}
void oracle_euler_to_quaternion(double roll, double pitch, double yaw, double* out_xyzw) {
  const Quat q = euler_to_quaternion(roll, pitch, yaw);
  out_xyzw[0] = q.x; out_xyzw[1] = q.y; out_xyzw[2] = q.z; out_xyzw[3] = q.w;
}
void oracle_center_time(void* pts, size_t n, uint64_t* stamp_us) { center_time(static_cast<Pt*>(pts), n, stamp_us); }
// mode 2: Compensate only (in untouched); mode 7: the node's CenterTime + Compensate + alignment (in centred)
int oracle_imu_preprocess(int mode, void* in, size_t n, uint64_t* stamp_us, const double* stamps,
                          const double* q_xyzw, size_t m, const double* extr_xyzw, void* out) {
  const ImuHandler h = make_handler(stamps, q_xyzw, m);
  const Quat e{extr_xyzw[0], extr_xyzw[1], extr_xyzw[2], extr_xyzw[3]};
  Pt* p = static_cast<Pt*>(in);
  if (mode == 2) return compensate(p, n, *stamp_us, h, e, static_cast<Pt*>(out)) ? 1 : 0;
  return imu_preprocess(p, n, stamp_us, h, e, static_cast<Pt*>(out)) ? 1 : 0;
}

// ---- wire formats (oracle/formats.cpp)
int oracle_from_pointcloud2(int point_type, const void* data, uint32_t width, uint32_t height, uint32_t point_step,
                            uint32_t row_step, const void* fields, size_t nfields, void* out) {
  return from_pointcloud2(point_type, static_cast<const uint8_t*>(data), width, height, point_step, row_step,
                          static_cast<const Pc2Field*>(fields), nfields, static_cast<Pt*>(out));
}
void oracle_transform_cloud(const void* in, size_t n, const double* m, void* out) {
  transform_cloud(static_cast<const Pt*>(in), n, m, static_cast<Pt*>(out));
}

// ---- global map (oracle/mapping.cpp)
void* oracle_mapping_create(double res, int stable) { return mapping_create(res, stable != 0); }
void oracle_mapping_destroy(void* h) { mapping_destroy(static_cast<MappingState*>(h)); }
void oracle_mapping_update(void* h, const void* in, size_t n, const double* q, const double* t) {
  mapping_update(static_cast<MappingState*>(h), static_cast<const Pt*>(in), n, q, t);
}
size_t oracle_mapping_size(void* h) { return mapping_size(static_cast<MappingState*>(h)); }
void oracle_mapping_get_map(void* h, void* out) { mapping_get_map(static_cast<MappingState*>(h), static_cast<Pt*>(out)); }

}  // extern "C"
