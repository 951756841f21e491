#pragma once
#include "cloud_ops.hpp"
#include "floam_common.hpp"
#include "grid.hpp"
#include "pose.hpp"
#include "voxel.hpp"

namespace floam {

// ----------------------------------------------------------------------------------------- hash grid
// Map points bucketed into a two-level cubic grid with ABSOLUTE cell coordinates (no bounding box): fine cells of
// edge kFineCell = 0.5 m nested 2x2x2 in coarse cells of 1 m.  Built without sorting (grid.hip): points are counted
// per coarse cell and fine sub-cell (atomics into an open-addressing table of coarse cells), every coarse cell gets
// a contiguous range of `pts` (block-aggregated bump allocation, fine sub-cells consecutive inside it), and the
// points are scattered into place.  The coarse table maps a 64-bit cell key to its range and its 8 sub-cell counts,
// from which the kNN derives every fine cell's range (no fine-cell table).
// Layout order inside a cell is not deterministic; the kNN breaks distance ties by map index, so results are.
// Exact replacement of the 5-NN KD-tree under the reference's sqd[4] < 1 gate (knn_group).

struct Grid {
  DevBuf<float4> pts;        // {x, y, z, map index bits}, grouped by coarse cell then fine sub-cell
  DevBuf<float4> xyz;        // {x, y, z, 0} by map index: 16-B neighbour gathers from a compact, L2-resident array
  DevBuf<CoarseCell> coarse;
  DevBuf<uint2> where;       // per map point: coarse slot, sub-cell << 28 | rank in the sub-cell
  // occupied slots of the coarse table, per build parity: the next build clears exactly these entries
  DevBuf<int> clist[2];
  DevBuf<int> counters;      // [0] bump cursor, [1..2] coarse list sizes (by parity)
  int bits = 0;              // table size = 1 << bits (at least twice the map size: load <= 1/2)
  unsigned mask = 0;
  int parity = 0;
  bool fresh = true;         // tables (re)allocated: the next clear is a full one
  bool precleared = false;   // the next build's clear was issued in advance (grid_clear_prepare)
  const PointRec* src = nullptr;   // the map the last build read (FLOAM_GRID_NOXYZ: the neighbour gathers read it)
};
// (diagnostic, FLOAM_GRID_NOXYZ=1: the grid build writes no xyz copy and the search gathers the neighbours'
// coordinates from the map records the grid was built from — VERDICT r05 item 1b's measurement)
bool grid_noxyz();

// The first step of a grid build — empty the table entries the previous build occupied (its slot list; the whole
// table after a reallocation) and reset the cursors — as a device job, so that it can run inside an earlier launch
// once the previous grid's last reader (the kNN) is done.
struct GridClearDev {
  CoarseCell* coarse;
  const int* clist_old;
  int* counters;
  int parity;
  int full_clear;
  unsigned mask;
};
__device__ __forceinline__ void grid_clear_part(const GridClearDev& J, int t0, int stride, bool lead) {
  CoarseCell e;
  e.key = kEmptyKey;
  e.start = 0;
  e.total = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) e.sub[k] = 0;
  if (J.full_clear) {
    const int size = (int)J.mask + 1;
    for (int t = t0; t < size; t += stride) J.coarse[t] = e;
  } else {
    const int nc = J.counters[1 + (J.parity ^ 1)];
    for (int t = t0; t < nc; t += stride) J.coarse[J.clist_old[t]] = e;
  }
  if (lead) {
    J.counters[0] = 0;
    J.counters[1 + J.parity] = 0;
  }
}
// sizes the grid for a map of up to ub points and returns its next build's clear (the build is then issued with
// precleared = true).  Must not be called while a launch that reads the grid is still to be issued.
GridClearDev grid_clear_prepare(Grid& g, int ub, hipStream_t st);

struct OdomDev;
// Rebuild the grids of both local maps (corner and surf) in four launches (three when precleared).  predict
// (nullable): the update's constant-velocity prediction (odom_predict_step) runs in the first of them instead of a
// launch of its own.
void geom_stamps_print();   // -DFLOAM_GEOM_STAMPS (diagnostic build)
void knn_waves_dump();      // -DFLOAM_KNN_WAVES (diagnostic build): FLOAM_KNN_WAVES=path
void grid_build_launch(Grid& gE, const PointRec* mapE, const int* d_mE, int mE_ub, Grid& gS, const PointRec* mapS,
                       const int* d_mS, int mS_ub, hipStream_t st, OdomDev* predict = nullptr, bool precleared = false,
                       size_t mE_cap = 0, size_t mS_cap = 0);   // caps: the maps' buffer sizes (speculative loads)

// ----------------------------------------------------------------------------------------- correspondences
// Edge record (EdgeAnalyticCostFunction inputs): cp (sensor point), a, b.  Surf: cp, unit normal n, d.
// SoA doubles, field f of slot i at base[f * cap + i]; valid[i] != 0 for accepted correspondences.
enum { EDGE_FIELDS = 9, SURF_FIELDS = 7 };

struct CorrSet {
  DevBuf<double> rec;
  DevBuf<uint8_t> valid;   // bit 0: after the kNN pass, 5 neighbours within sqd < 1; after geometry, record accepted
                           // bit 1: the query needed the full +-1 m search (profiling byte counter)
                           // bit 2: the search found 5 neighbours (set by the geometry pass)
  DevBuf<float> nnxyz;     // coordinates of the 5 nearest map points, nnxyz[(3 * k + axis) * cap + i]
  // stage inspection (floam_odom_set_trace): the 5 neighbours' map indices and float squared distances, k-major
  // (nnidx[k * cap + i]); written by the search only while tracing
  DevBuf<int> nnidx;
  DevBuf<float> nnsqd;
  bool trace = false;
  int cap = 0;
  void reserve(int n, int fields) {
    if (n > cap) {
      const int c = n < 1024 ? 1024 : n + n / 4;
      valid.reserve(c);
      cap = (int)valid.cap;
      rec.reserve((size_t)cap * fields);
      nnxyz.reserve((size_t)cap * 15);
    }
    if (trace) {
      nnidx.reserve((size_t)cap * 5);
      nnsqd.reserve((size_t)cap * 5);
    }
  }
};

// ----------------------------------------------------------------------------------------- LM state
struct LMState {
  double x[7];        // accepted parameters (qx, qy, qz, qw, tx, ty, tz)
  double cand[7];     // candidate under evaluation
  double x_cost;
  double H[21];       // J^T J at x (unscaled, upper triangle row-major)
  double g[6];        // J^T r at x
  double dlo[6], dhi[6];   // bounds of the unscaled LM diagonal: 1e-6, 1e32 over the squared Jacobi scaling, fixed
                           // at iteration 0 (lm.hip lm_step)
  double diag[6];     // unscaled LM diagonal (reused after a rejected / invalid step)
  double radius, dfac, mcc, x_norm, gmax, initial_cost;
  double cand_norm;   // |cand| (x_norm once it is accepted): formed by the candidate's deferred tests
  double proj[7];     // x [+] -g, the gradient-norm test's projection (deferred tests, lm.hip)
  // the solve's iteration-zero quantities (stage inspection; oracle/odom.cpp SolveTrace): the starting point and the
  // unscaled J^T J and J^T r there
  double x_in[7];
  double H0[21];
  double g0[6];
  int phase;          // 0: evaluate x (iteration zero); 1: evaluate cand
  int done;
  int iteration;
  int reuse;
  int invalid;
  int successful;
  int n_res;
  int corr_edge, corr_surf;   // accepted correspondences (this solve)
  // the candidate's tests that do not depend on its evaluation, run off the control step's chain (lm.hip
  // deferred_tests): tpend — pending (bit 0 parameter tolerance, bit 1 gradient norm against proj); tdone — their
  // verdict (1: parameter tolerance, 2: gradient norm, which also takes back the step's iteration count)
  int tpend, tdone;
  unsigned epoch;     // hand-off tag base of the resident solve (lm.hip): advanced by 8 per solve (lm_reset)
  // peer sharding: evaluations exchanged with the other ranks since floam_odom_set_shard_peers (continues across
  // solves; lm_reset keeps it): the exchange slot and tag of each evaluation (lm.hip peer_exchange)
  unsigned xseq;
  // set (never cleared) by any block of a resident solve whose hand-off timed out; the one word the state write-back
  // (publish_state) leaves alone, so block 0 cannot overwrite another block's report.  Must stay the last word.
  int xfail;
};
constexpr int kStateWords = (int)(sizeof(LMState) / sizeof(unsigned));
constexpr int kPublishWords = kStateWords - 1;   // every word but xfail
static_assert(offsetof(LMState, xfail) == sizeof(unsigned) * kPublishWords, "xfail is the last LMState word");
static_assert(sizeof(LMState) % 8 == 0, "LMState is copied as whole dwords");

enum { LM_NSUM = 29 };   // cost, H[21], g[6], count

// Surf records as 13-vectors w = [n (x) p (9), n (3), d + n.o] (geom_kernel): the surf half of every squared-loss LM
// evaluation is a set of quadratic forms of their Gram matrix G = sum w w^T (lm.hip)
constexpr int kGramW = 13;
constexpr int kGram = kGramW * (kGramW + 1) / 2;   // 91 unique entries (upper triangle, row-major)
constexpr int kGramWords = kGram + 3;              // G + the origin o the records were recentred on
constexpr int kSurfGeomBlocks = 256;               // fixed surf geometry grid: fixed Gram reduction order
constexpr int kGramGroups = 8;                     // its partials are reduced in 8 groups of 32, then the groups
// gmat as the geometry launch leaves it: the 8 group partials of G, then o; the solve's prologue adds the groups up
// in order (gram_load), so the geometry launch needs no second level of hand-offs
constexpr int kGramMatWords = kGramGroups * kGram + 3;
__device__ __forceinline__ double gram_load(const double* __restrict__ gmat, int t) {
  if (t < kGram) {
    double gp[kGramGroups];   // all loads in flight before the in-order sum
#pragma unroll
    for (int k = 0; k < kGramGroups; ++k) gp[k] = gmat[k * kGram + t];
    double v = gp[0];
#pragma unroll
    for (int k = 1; k < kGramGroups; ++k) v += gp[k];
    return v;
  }
  return t < kGramWords ? gmat[kGramGroups * kGram + (t - kGram)] : 0.0;
}
constexpr int kEdgeEvalBlocks = 64;                // edge-only evaluation grid of the Gram solves (fixed order)
constexpr int kRecEvalBlocks = 128;                // per-record evaluation grid (Huber / fp32; fixed order)
constexpr int kMaxShardRanks = 8;                   // peer sharding: ranks (one node's GPUs)
constexpr int kShardXchgWords = 512;                // peer sharding: exchange buffer granules (2 x 58 used; 4 KB)
constexpr int kShardProbeWord = kShardXchgWords - 8;  // ... and the mapping probe's word (peer_probe_launch)
constexpr unsigned long long kShardProbeTicks = 200000000ull;   // the probe's wait: 2 s (100-MHz s_memrealtime)

// LM modes: surf half from the Gram matrix (squared loss, fp64), Huber loss, fp32 geometry + residuals / Jacobians
enum { LM_GRAM = 1, LM_HUBER = 2, LM_FP32 = 4 };
inline int lm_mode(bool huber, bool fp32) { return (huber || fp32) ? (huber ? LM_HUBER : 0) | (fp32 ? LM_FP32 : 0) : LM_GRAM; }

// device scratch of the solves (lm.hip)
struct LMBuffers {
  DevBuf<unsigned long long> part;   // resident solve: every block's partial-sum granules (two parity slots)
  DevBuf<double> partials;           // sharded evaluation: block partials
  DevBuf<double> sums;               // sharded evaluation: the 29 sums (all-reduced over the ranks in place)
  DevBuf<unsigned> ticket;           // sharded evaluation: arrival ticket (zero between launches)
  DevBuf<double> gpart;              // surf Gram matrix: per-block and per-group partials (geom_kernel)
  DevBuf<double> gmat;               // the solve's surf Gram matrix + its origin
  DevBuf<unsigned> gcnt;             // ticket words of the Gram reduction
  int fail_test = 0;                 // FLOAM_LM_FAIL_TEST=1 (tests, diagnostic build): every resident solve reports
                                     // its hand-off as timed out (n_res < 0), the path a lost block would take
  int peer_delay_us = 0;             // FLOAM_PEER_DELAY_US=n (tests, diagnostic build): the non-zero blocks of a
                                     // peer-sharded solve wait n us before every poll of the other ranks' sums
  void reserve(hipStream_t st);
};

struct QuerySet {
  const PointRec* pts;
  const int* d_n;
  int n_ub;
  int grid_hint = 0;   // > 0: size the search grid for this many queries (the kernels grid-stride over the rest)
};

struct X7 {
  double v[7];
  int set;
};
void lm_init_dev_launch(LMState* d_st, const double* x0_dev, hipStream_t st);   // reset; x = x0_dev (device pointer)

// Device-resident controller state (OdomEstimationClass members odom, last_odom, the keyframe list): the pose
// algebra between the solves runs on the device, so a whole selector is issued without a host round trip; the host
// mirrors the poses from the status slots when it collects a scan.
struct OdomDev {
  Pose odom, last_odom;
  Pose mid;                // deskewed selector: the first call's result (last_odom of the second call)
  Pose kf;                 // keyframes.back()
  int kf_count;            // keyframes.size() (0..3)
  int kf_flag;             // the last KeyFrameUpdate result: gates the map update
  int failed;              // a solve ended without its blocks' hand-offs (n_res < 0): from then on the status
                           // gathers leave the pose, the keyframe and the maps untouched (the host raises the error)
  double x0[2][7];         // parameters {q, t} of the predictions of the first / second call
};
void odom_dev_init_launch(OdomDev* s, hipStream_t st);   // identity poses, no keyframes

// odomEstimationClass.cpp:59-71 (branch always taken, Q2): pred = odom (last^-1 odom); last = odom; odom = pred;
// x0[0] = the parameters {q, t} of pred (the first call's starting point)
void odom_predict_launch(OdomDev* s, hipStream_t st);
__device__ inline void odom_predict_step(OdomDev* s) {   // one thread
  const Pose pred = pose_mul(s->odom, pose_mul(pose_inverse(s->last_odom), s->odom));
  s->last_odom = s->odom;   // Q2: the branch is taken for every update type
  s->odom = pred;
  pose_to_params(pred, s->x0[0]);
}

struct UpdateStatus {
  LMState lm;
  int counts[4];                  // downsampled edge, surf; corner map, surf map
  int fe_status;                  // status flags of the feature extraction that produced the inputs (async FE)
  int kf_flag;                    // KeyFrameUpdate result of this call (when it ran)
  unsigned long long prof[2];     // algorithmic bytes of the kNN launches (profiling)
  Pose odom, last_odom;           // controller poses after this call
  unsigned seq;                   // the update's serial number, stored last (system scope): the host polls it
  unsigned seq_pad;
};
// status gather; with finish: the call's writeback odom = Isometry(q(x), t(x)) (:114-116; x is the prediction when
// the gate (:77) kept the solve from running), after a deskewed first call last_odom = the first call's result, and
// with keyframe (1: normal, 2: the process-wide first call, Q6) KeyFrameUpdate (:320-343) into kf_flag
enum { GATHER_FINISH = 1, GATHER_AFTER_MID = 2, GATHER_KEYFRAME = 4, GATHER_KEYFRAME_FIRST = 8 };
void gather_status_launch(const LMState* lm, const int* dcnt, const int* mapE_count, const int* mapS_count,
                          const int* fe_status, const unsigned long long* prof, UpdateStatus* out, OdomDev* s,
                          int mode, unsigned seq, hipStream_t st, const VoxelFused* vf = nullptr,
                          const GridClearDev* gc = nullptr);
// vf (non-null): the launch also runs the bounding-box stage of the voxel2_launch that follows it (the map update,
// whose pose is the solve's result): grid (kVoxMinMaxBlocks, 2), block (0, 0) gathers first; gc (with vf, nullable):
// the clears of the next builds of the two grids (gc[0] corner, gc[1] surf), after the last kNN of this update
struct GatherArgs {   // a status gather carried out by another launch (deskew_bridge for the first call's slot)
  const int* dcnt = nullptr;
  const int* mapE_count = nullptr;
  const int* mapS_count = nullptr;
  const int* fe_status = nullptr;
  UpdateStatus* out = nullptr;   // null: nothing to gather
  unsigned seq = 0;
};

// KeyFrameUpdate(pose) (src/odomEstimationClass.cpp:320-343) on the device state with an explicit pose {q, t}: the
// public method the reference's header exposes (include/odomEstimationClass.h:80); result into *flag
void keyframe_update_launch(OdomDev* s, const double* x_dev, int first, int* flag, hipStream_t st);

// Between the two updatePointsToMap calls of a deskewed UpdatePointsToMapSelector (odomEstimationClass.cpp:40-46),
// without a host round trip: GetVelocity from the first call's result (x1 = st->x) and s->last_odom (the pose before
// it), CompensateVelocity of both clouds in place (dataHandler.cpp:82-92, Q5; twice per point when edge and surf are
// one cloud); s->mid = odom1 and the second call's prediction odom1 * (last_odom^-1 * odom1) into s->x0[1].
// gather: the first call's status gather (mode 0: it only reads the LM state, the counts and the poses, none of
// which this launch writes) done by block 0 instead of a launch of its own
void deskew_bridge_launch(const LMState* st, OdomDev* s, double scan_period, PointRec* edge, const int* d_ne,
                          int ne_ub, PointRec* surf, const int* d_ns, int ns_ub, hipStream_t stream,
                          const GatherArgs& gather = GatherArgs{}, const VoxelFused* vf = nullptr);
// vf (non-null, edge != surf): the bounding-box stage of the second call's VoxelGrids (deskewed edge at the edge
// leaf, deskewed surf at the surf leaf) over the coordinates this launch writes; grid (kVoxMinMaxBlocks, 2)
// Correspondence search for the edge and the surf query sets at the pose in st->x, in two launches:
// knn_launch — exact 5-NN (blocks [0, nbE) edge queries against the corner map, the rest surf against the surf map);
// geom_launch — line / plane fits and the residual records (fp64, or fp32 with fp32).
// knn_launch also starts the solve (lm_reset): LM state reset, x = x0_dev when non-null, hand-off epoch advanced
// ev0 / ev1 (profiling): HIP events set to the search kernel's own start and end (hipExtLaunchKernel: the dispatch's
// begin / end timestamps, what rocprofv3 reports), not to the stream position around it
void knn_launch(LMState* d_st, const double* x0_dev, const QuerySet& qe, const Grid& ge, CorrSet& ce,
                const QuerySet& qs, const Grid& gs, CorrSet& cs, const int* d_me, const int* d_ms, int rank, int world,
                hipStream_t st, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// (diagnostic build, FLOAM_KNN_SPLIT=1) the role-split prototype: knn_launch + geom_launch as ONE launch (search
// blocks, then geometry blocks that wait for their queries' search); false (nothing launched) when off or fp32
bool knn_geom_split_launch(LMState* d_st, const double* x0_dev, const QuerySet& qe, const Grid& ge, CorrSet& ce,
                           const QuerySet& qs, const Grid& gs, CorrSet& cs, const int* d_me, const int* d_ms,
                           int rank, int world, bool gram, bool fp32, LMBuffers& b, hipStream_t st,
                           hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// gram: the squared-loss solves' surf Gram matrix of the accepted surf records into b.gmat (b.gpart's partials)
void geom_launch(LMState* d_st, const QuerySet& qe, CorrSet& ce, const QuerySet& qs, CorrSet& cs, bool gram,
                 bool fp32, LMBuffers& b, hipStream_t st);
// algorithmic bytes of the correspondence pass just issued (profiling only), accumulated into *d_bytes
// (diagnostic, FLOAM_KNN_STAGES=1 in a profiled replay) the search cut after each of its dependent round trips, every
// variant after an L2 eviction, then one more eviction before the real search
void knn_stage_launch(LMState* d_st, const double* x0_dev, const QuerySet& qe, const Grid& ge, CorrSet& ce,
                      const QuerySet& qs, const Grid& gs, CorrSet& cs, const int* d_me, const int* d_ms, int rank,
                      int world, DevBuf<float4>& evict, hipStream_t st);
void knn_traffic_launch(const LMState* d_st, const QuerySet& q, const Grid& g, CorrSet& c, int rank, int world,
                        DevBuf<unsigned long long>& set, unsigned long long* d_bytes, hipStream_t st);

// ----------------------------------------------------------------------------------------- LM solve (lm.hip)
// A whole ceres::Solve (iteration zero + up to max_num_iterations = 4 candidates, src/odomEstimationClass.cpp:95-108)
// in ONE launch on a single GPU: every block keeps its records in registers, evaluates them, all-gathers the blocks'
// partial sums and runs the Ceres 1.13 control step itself (the same bits in every block).  mode = LM_*.
// peers (world > 1): query sharding with the resident solve — each rank's blocks reduce the rank's sums as above, then
// exchange them with the other ranks through peer-mapped buffers (every rank's buffer readable from every GPU), summed
// in rank order; one launch per solve, no collective launch, no host round trip.
struct ShardPeers {
  int world = 1;
  unsigned long long* mine = nullptr;                            // this rank's exchange buffer (kShardXchgWords)
  const unsigned long long* buf[kMaxShardRanks] = {};            // every rank's, as mapped on this GPU (rank order)
};
void lm_solve_launch(LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const CorrSet& cs,
                     const int* d_ns, int ns_ub, int mode, LMBuffers& b, hipStream_t st,
                     unsigned long long* dbg = nullptr, const ShardPeers* peers = nullptr);
// the peer mappings' probe (lm.hip): *d_fail = mask of the ranks whose buffer did not answer within 2 s (0: all did)
void peer_probe_launch(const ShardPeers& P, int rank, int* d_fail, hipStream_t st);
// The same solve sharded over ranks (one process per GPU): evaluation k = 0..4 in one launch each (the control step
// of evaluation k - 1 folded in, run redundantly by every block on the all-reduced sums), leaving this rank's 29
// sums in b.sums for the caller's all-reduce; lm_shard_final_launch runs the last control step.
void lm_shard_eval_launch(int k, LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const CorrSet& cs,
                          const int* d_ns, int ns_ub, int mode, LMBuffers& b, hipStream_t st);
void lm_shard_final_launch(LMState* d_st, LMBuffers& b, hipStream_t st);
// lm_solve's blocks poll each other's partial sums, so the whole grid must be resident at once: true when the
// occupancy of the instance `mode` selects times the device's CU count covers its grid.  Otherwise the caller runs
// the per-evaluation path (lm_shard_eval + lm_shard_final on one rank, no spin between blocks).
bool lm_solve_coresident(int mode, int device);
// -DFLOAM_CTRL_STAMPS builds: block 0's control-step segments to stderr (no-op otherwise)
void lm_ctrl_stamps_print();
// Stage inspection: append this solve's trace record (49 doubles, oracle/odom.cpp SolveTrace order) to trace[] at
// *count when the map-size gate (:77) let the solve run and *count < cap.
constexpr int kTraceWords = 49;
void lm_trace_launch(const LMState* d_st, const int* dcnt, const int* d_me, const int* d_ms, double* trace,
                     unsigned* count, int cap, hipStream_t st);

}  // namespace floam
