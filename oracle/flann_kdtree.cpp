// CPU ORACLE (test infrastructure) — restatement of pcl::KdTreeFLANN<PointXYZI> over FLANN 1.9
// KDTreeSingleIndex (leaf_max_size 15, exact: eps 0, unlimited checks), L2_Simple<float> distance and
// KNNSimpleResultSet (strict '<' acceptance, insertion after equal distances).  Call sites:
// src/odomEstimationClass.cpp:17-18 (construction), :78-79 (setInputCloud every update), :153 and :206
// (nearestKSearch k=5).  Parity unpinned (see oracle.hpp).
#include <algorithm>
#include <cfloat>
#include <limits>
#include <utility>

#include "oracle.hpp"

namespace oracle {

namespace {
constexpr int kLeafMax = 15;

struct KnnResult {      // flann::KNNSimpleResultSet<float>
  int cap, count = 0;
  float dist[8];
  int index[8];
  float worst = std::numeric_limits<float>::max();
  explicit KnnResult(int k) : cap(k) {
    for (int i = 0; i < k; ++i) { dist[i] = std::numeric_limits<float>::max(); index[i] = -1; }
  }
  void add(float d, int idx) {
    if (d >= worst) return;
    if (count < cap) ++count;
    int i;
    for (i = count - 1; i > 0; --i) {
      if (dist[i - 1] > d) {
        dist[i] = dist[i - 1];
        index[i] = index[i - 1];
      } else {
        break;
      }
    }
    dist[i] = d;
    index[i] = idx;
    worst = dist[cap - 1];
  }
};

inline float l2_simple(const float* a, const float* b) {   // flann::L2_Simple<float>::operator()
  float result = 0.0f;
  for (int i = 0; i < 3; ++i) {
    const float diff = a[i] - b[i];
    result += diff * diff;
  }
  return result;
}
inline float accum_dist(float a, float b) { return (a - b) * (a - b); }

struct Searcher {
  const std::vector<float>* data;
  const std::vector<int>* vind;
  const void* nodes;
};
}  // namespace

void KdTree::min_max(const int* ind, int count, int dim, float& mn, float& mx) const {
  mn = data_[3 * ind[0] + dim];
  mx = mn;
  for (int i = 1; i < count; ++i) {
    const float v = data_[3 * ind[i] + dim];
    if (v > mx) mx = v;
    if (v < mn) mn = v;
  }
}

void KdTree::plane_split(int* ind, int count, int cutfeat, float cutval, int& lim1, int& lim2) {
  int left = 0, right = count - 1;
  for (;;) {
    while (left <= right && data_[3 * ind[left] + cutfeat] < cutval) ++left;
    while (left <= right && data_[3 * ind[right] + cutfeat] >= cutval) --right;
    if (left > right) break;
    std::swap(ind[left], ind[right]);
    ++left;
    --right;
  }
  lim1 = left;
  right = count - 1;
  for (;;) {
    while (left <= right && data_[3 * ind[left] + cutfeat] <= cutval) ++left;
    while (left <= right && data_[3 * ind[right] + cutfeat] > cutval) --right;
    if (left > right) break;
    std::swap(ind[left], ind[right]);
    ++left;
    --right;
  }
  lim2 = left;
}

void KdTree::middle_split(int* ind, int count, int& index, int& cutfeat, float& cutval, const Interval* bbox) {
  const float EPS = 0.00001f;
  float max_span = bbox[0].high - bbox[0].low;
  for (int i = 1; i < 3; ++i) {
    const float span = bbox[i].high - bbox[i].low;
    if (span > max_span) max_span = span;
  }
  float max_spread = -1;
  cutfeat = 0;
  for (int i = 0; i < 3; ++i) {
    const float span = bbox[i].high - bbox[i].low;
    if (span > (1 - EPS) * max_span) {
      float mn, mx;
      min_max(ind, count, i, mn, mx);
      const float spread = mx - mn;
      if (spread > max_spread) {
        cutfeat = i;
        max_spread = spread;
      }
    }
  }
  const float split_val = (bbox[cutfeat].low + bbox[cutfeat].high) / 2;
  float mn, mx;
  min_max(ind, count, cutfeat, mn, mx);
  if (split_val < mn) cutval = mn;
  else if (split_val > mx) cutval = mx;
  else cutval = split_val;
  int lim1, lim2;
  plane_split(ind, count, cutfeat, cutval, lim1, lim2);
  if (lim1 > count / 2) index = lim1;
  else if (lim2 < count / 2) index = lim2;
  else index = count / 2;
}

int KdTree::divide(int left, int right, Interval* bbox) {
  const int id = (int)nodes_.size();
  nodes_.push_back(Node{});
  if ((right - left) <= kLeafMax) {
    nodes_[id].child1 = nodes_[id].child2 = -1;
    nodes_[id].left = left;
    nodes_[id].right = right;
    for (int i = 0; i < 3; ++i) bbox[i].low = bbox[i].high = data_[3 * vind_[left] + i];
    for (int k = left + 1; k < right; ++k)
      for (int i = 0; i < 3; ++i) {
        const float v = data_[3 * vind_[k] + i];
        if (bbox[i].low > v) bbox[i].low = v;
        if (bbox[i].high < v) bbox[i].high = v;
      }
  } else {
    int idx, cutfeat;
    float cutval;
    middle_split(&vind_[0] + left, right - left, idx, cutfeat, cutval, bbox);
    nodes_[id].divfeat = cutfeat;
    Interval lb[3] = {bbox[0], bbox[1], bbox[2]};
    lb[cutfeat].high = cutval;
    const int c1 = divide(left, left + idx, lb);
    Interval rb[3] = {bbox[0], bbox[1], bbox[2]};
    rb[cutfeat].low = cutval;
    const int c2 = divide(left + idx, right, rb);
    nodes_[id].child1 = c1;
    nodes_[id].child2 = c2;
    nodes_[id].divlow = lb[cutfeat].high;
    nodes_[id].divhigh = rb[cutfeat].low;
    for (int i = 0; i < 3; ++i) {
      bbox[i].low = std::min(lb[i].low, rb[i].low);
      bbox[i].high = std::max(lb[i].high, rb[i].high);
    }
  }
  return id;
}

void KdTree::build(const Pt* pts, size_t n) {
  n_ = n;
  std::vector<float> raw(3 * n);
  for (size_t i = 0; i < n; ++i) {
    raw[3 * i] = pts[i].x;
    raw[3 * i + 1] = pts[i].y;
    raw[3 * i + 2] = pts[i].z;
  }
  data_ = raw;
  vind_.resize(n);
  for (size_t i = 0; i < n; ++i) vind_[i] = (int)i;
  nodes_.clear();
  nodes_.reserve(2 * n / kLeafMax + 8);
  if (n == 0) { root_ = -1; return; }
  for (int i = 0; i < 3; ++i) root_bbox_[i].low = root_bbox_[i].high = data_[i];
  for (size_t k = 1; k < n; ++k)
    for (int i = 0; i < 3; ++i) {
      const float v = data_[3 * k + i];
      if (v < root_bbox_[i].low) root_bbox_[i].low = v;
      if (v > root_bbox_[i].high) root_bbox_[i].high = v;
    }
  Interval bb[3] = {root_bbox_[0], root_bbox_[1], root_bbox_[2]};
  root_ = divide(0, (int)n, bb);
  // reorder_ = true: the leaf scan reads a copy of the data in vind_ order (same float values)
  std::vector<float> re(3 * n);
  for (size_t i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) re[3 * i + d] = raw[3 * vind_[i] + d];
  data_.swap(re);
  // from here on data_ is in tree order: leaf i <-> data_[3*i]; original index = vind_[i]
}

namespace {
struct SearchCtx {
  const float* data;
  const int* vind;
  const void* nodes;
  const float* q;
  KnnResult* rs;
};
}  // namespace

int KdTree::knn(const float q[3], int k, int* out_idx, float* out_sqd) const {
  KnnResult rs(k);
  if (root_ < 0) return 0;
  float dists[3] = {0, 0, 0};
  float distsq = 0.0f;
  for (int i = 0; i < 3; ++i) {
    if (q[i] < root_bbox_[i].low) { dists[i] = accum_dist(q[i], root_bbox_[i].low); distsq += dists[i]; }
    if (q[i] > root_bbox_[i].high) { dists[i] = accum_dist(q[i], root_bbox_[i].high); distsq += dists[i]; }
  }
  // iterative restatement of KDTreeSingleIndex::searchLevel (same visiting order)
  struct Frame { int node; float mindistsq; int stage; float dst; float cut; int other; };
  Frame stack[128];
  int sp = 0;
  stack[sp++] = Frame{root_, distsq, 0, 0, 0, -1};
  while (sp > 0) {
    Frame& f = stack[sp - 1];
    const Node& nd = nodes_[f.node];
    if (nd.child1 < 0 && nd.child2 < 0) {
      const float worst = rs.worst;
      for (int i = nd.left; i < nd.right; ++i) {
        const float d = l2_simple(q, &data_[3 * i]);
        if (d < worst) rs.add(d, vind_[i]);
      }
      --sp;
      continue;
    }
    const int idx = nd.divfeat;
    const float val = q[idx];
    if (f.stage == 0) {
      const float diff1 = val - nd.divlow, diff2 = val - nd.divhigh;
      int best;
      if ((diff1 + diff2) < 0) { best = nd.child1; f.other = nd.child2; f.cut = accum_dist(val, nd.divhigh); }
      else { best = nd.child2; f.other = nd.child1; f.cut = accum_dist(val, nd.divlow); }
      f.stage = 1;
      const float md = f.mindistsq;
      stack[sp++] = Frame{best, md, 0, 0, 0, -1};
    } else if (f.stage == 1) {
      f.dst = dists[idx];
      const float md = f.mindistsq + f.cut - f.dst;
      dists[idx] = f.cut;
      f.stage = 2;
      if (md * 1.0f <= rs.worst) {
        stack[sp++] = Frame{f.other, md, 0, 0, 0, -1};
      }
    } else {
      dists[idx] = f.dst;
      --sp;
    }
  }
  const int got = std::min(k, (int)n_);
  for (int i = 0; i < got; ++i) { out_idx[i] = rs.index[i]; out_sqd[i] = rs.dist[i]; }
  return got;
}

}  // namespace oracle
