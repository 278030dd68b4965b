// bvh.hip -- host BVH builder for large environment meshes (replaces the BVH Warp builds inside
// wp.Mesh, tracer.py:24).  Binned SAH (32 bins) over face centroids, leaves of <= 4 faces, depth
// capped below the device stack (rt_bvh.h), boxes rounded outward to f32 and padded so that the
// f32 slab test can never cull a face the watertight test would hit.  Deterministic: the same mesh
// always gives the same tree (std::stable_partition, fixed tie rules).
#include <math.h>

#include <string.h>

#include <algorithm>
#include <cstring>
#include <cmath>
#include <numeric>
#include <vector>

#include "rt_bvh.h"
#include "rt_internal.h"

namespace {

struct Box {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  void grow(const double* p) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  double area() const {
    if (!(hi[0] >= lo[0])) return 0.0;
    const double e0 = hi[0] - lo[0], e1 = hi[1] - lo[1], e2 = hi[2] - lo[2];
    return 2.0 * (e0 * e1 + e1 * e2 + e2 * e0);
  }
};

constexpr int kBins = 32;
constexpr int kLeaf = 4;
constexpr int kMaxDepth = RT_BVH_STACK - 4;

struct Builder {
  const std::vector<float>& tri;
  std::vector<Box> fbox;
  std::vector<double> cen;  // 3 per face
  std::vector<int> idx;
  std::vector<float> nodes;  // 16 floats per node
  std::vector<int> leaves;   // 2 ints per leaf
  double pad;
  int max_depth = 0, max_leaf = 0;

  explicit Builder(const std::vector<float>& t) : tri(t) {}

  Box range_box(int b, int e) const {
    Box bx;
    for (int i = b; i < e; ++i) bx.grow(fbox[idx[i]]);
    return bx;
  }

  // f32 box rounded outward and padded
  void put_box(float* dst, const Box& b) const {
    if (!(b.hi[0] >= b.lo[0])) {  // empty child: inverted box, never hit
      dst[0] = dst[1] = dst[2] = INFINITY;
      dst[3] = dst[4] = dst[5] = -INFINITY;
      return;
    }
    for (int k = 0; k < 3; ++k) {
      dst[k] = std::nextafter((float)(b.lo[k] - pad), -INFINITY);
      dst[3 + k] = std::nextafter((float)(b.hi[k] + pad), INFINITY);
    }
  }

  int make_leaf(int b, int e) {
    max_leaf = std::max(max_leaf, e - b);
    const int id = (int)(leaves.size() / 2);
    leaves.push_back(b);
    leaves.push_back(e - b);
    return -1 - id;
  }

  // returns child encoding for range [b, e)
  int build(int b, int e, int depth) {
    const int n = e - b;
    max_depth = std::max(max_depth, depth);
    if (n <= kLeaf || depth >= kMaxDepth) return make_leaf(b, e);
    Box cb;
    for (int i = b; i < e; ++i) cb.grow(&cen[3 * idx[i]]);
    int axis = 0;
    double ext = cb.hi[0] - cb.lo[0];
    for (int k = 1; k < 3; ++k)
      if (cb.hi[k] - cb.lo[k] > ext) {
        ext = cb.hi[k] - cb.lo[k];
        axis = k;
      }
    int mid = -1;
    if (ext > 0.0) {
      Box bins[kBins];
      int cnt[kBins] = {0};
      auto bin_of = [&](int f) {
        int k = (int)((cen[3 * f + axis] - cb.lo[axis]) / ext * kBins);
        return std::min(std::max(k, 0), kBins - 1);
      };
      for (int i = b; i < e; ++i) {
        const int k = bin_of(idx[i]);
        ++cnt[k];
        bins[k].grow(fbox[idx[i]]);
      }
      double best = INFINITY;
      int best_split = -1;
      Box left[kBins];
      int lcnt[kBins];
      Box acc;
      int ac = 0;
      for (int k = 0; k < kBins; ++k) {
        acc.grow(bins[k]);
        ac += cnt[k];
        left[k] = acc;
        lcnt[k] = ac;
      }
      Box racc;
      int rc = 0;
      for (int k = kBins - 1; k >= 1; --k) {
        racc.grow(bins[k]);
        rc += cnt[k];
        const int lc = lcnt[k - 1];
        if (lc == 0 || rc == 0) continue;
        const double cost = left[k - 1].area() * lc + racc.area() * rc;
        if (cost < best) {
          best = cost;
          best_split = k;
        }
      }
      if (best_split > 0) {
        auto it = std::stable_partition(idx.begin() + b, idx.begin() + e,
                                        [&](int f) { return bin_of(f) < best_split; });
        mid = (int)(it - idx.begin());
      }
    }
    if (mid <= b || mid >= e) {  // degenerate centroids: split by position in the list
      std::stable_sort(idx.begin() + b, idx.begin() + e,
                       [&](int x, int y) { return cen[3 * x + axis] < cen[3 * y + axis]; });
      mid = b + n / 2;
    }
    const int me = (int)(nodes.size() / 16);
    nodes.resize(nodes.size() + 16, 0.0f);
    const Box lb = range_box(b, mid), rb = range_box(mid, e);
    const int c0 = build(b, mid, depth + 1);
    const int c1 = build(mid, e, depth + 1);
    float* q = nodes.data() + 16 * me;
    float box0[6], box1[6];
    put_box(box0, lb);
    put_box(box1, rb);
    // q0 = (c0lo.x, c0lo.y, c0lo.z, c0hi.x) q1 = (c0hi.y, c0hi.z, c1lo.x, c1lo.y)
    // q2 = (c1lo.z, c1hi.x, c1hi.y, c1hi.z) q3 = (child0, child1, 0, 0)
    q[0] = box0[0];
    q[1] = box0[1];
    q[2] = box0[2];
    q[3] = box0[3];
    q[4] = box0[4];
    q[5] = box0[5];
    q[6] = box1[0];
    q[7] = box1[1];
    q[8] = box1[2];
    q[9] = box1[3];
    q[10] = box1[4];
    q[11] = box1[5];
    std::memcpy(&q[12], &c0, 4);
    std::memcpy(&q[13], &c1, 4);
    return me;
  }
};

}  // namespace

namespace rt {

int build_bvh(rt_mesh* m, const std::vector<float>& tri) {
  const int64_t nf = m->nf;
  Builder bd(tri);
  bd.fbox.resize(nf);
  bd.cen.resize(3 * nf);
  bd.idx.resize(nf);
  double amax = 0.0;
  for (int64_t f = 0; f < nf; ++f) {
    for (int v = 0; v < 3; ++v) {
      double p[3];
      for (int k = 0; k < 3; ++k) {
        p[k] = tri[9 * f + 3 * v + k];
        amax = std::max(amax, std::fabs(p[k]));
      }
      bd.fbox[f].grow(p);
    }
    for (int k = 0; k < 3; ++k) bd.cen[3 * f + k] = 0.5 * (bd.fbox[f].lo[k] + bd.fbox[f].hi[k]);
    bd.idx[f] = (int)f;
  }
  bd.pad = 1e-5 * (1.0 + amax);
  // root is always an internal node (a one-leaf mesh gets an empty second child)
  bd.nodes.resize(16, 0.0f);
  int c0, c1;
  Box b0, b1;
  if (nf <= kLeaf) {
    c0 = bd.make_leaf(0, (int)nf);
    c1 = bd.make_leaf((int)nf, (int)nf);
    b0 = bd.range_box(0, (int)nf);
  } else {
    // split the root like any node, then move the resulting node's children into slot 0
    const int r = bd.build(0, (int)nf, 1);
    std::memcpy(bd.nodes.data(), bd.nodes.data() + 16 * r, 16 * sizeof(float));
    // the copied node stays referenced nowhere else (r is only the root)
    c0 = c1 = 0;
  }
  if (nf <= kLeaf) {
    float* q = bd.nodes.data();
    bd.put_box(q, b0);
    float eb[6];
    bd.put_box(eb, b1);
    q[6] = eb[0];
    q[7] = eb[1];
    q[8] = eb[2];
    q[9] = eb[3];
    q[10] = eb[4];
    q[11] = eb[5];
    std::memcpy(&q[12], &c0, 4);
    std::memcpy(&q[13], &c1, 4);
  }
  // leaf-ordered compact face table
  std::vector<float> lcomp((size_t)std::max<int64_t>(nf, 1) * 12, 0.0f);
  for (int64_t i = 0; i < nf; ++i) {
    const int f = bd.idx[i];
    float* q = &lcomp[12 * i];
    for (int k = 0; k < 9; ++k) q[k] = tri[9 * (size_t)f + k];
    std::memcpy(&q[9], &f, 4);
  }
  m->bvh_depth = bd.max_depth;
  m->bvh_max_leaf = bd.max_leaf;
  m->nnodes = (int64_t)(bd.nodes.size() / 16);
  m->nleaves = (int64_t)(bd.leaves.size() / 2);
  RT_HIP(hipMalloc(&m->nodes, bd.nodes.size() * sizeof(float)));
  RT_HIP(hipMalloc(&m->leaves, std::max<size_t>(bd.leaves.size(), 2) * sizeof(int)));
  RT_HIP(hipMalloc(&m->lcomp, lcomp.size() * sizeof(float)));
  RT_HIP(hipMemcpy(m->lcomp, lcomp.data(), lcomp.size() * sizeof(float), hipMemcpyHostToDevice));
  RT_HIP(hipMemcpy(m->nodes, bd.nodes.data(), bd.nodes.size() * sizeof(float), hipMemcpyHostToDevice));
  if (!bd.leaves.empty())
    RT_HIP(hipMemcpy(m->leaves, bd.leaves.data(), bd.leaves.size() * sizeof(int), hipMemcpyHostToDevice));
  return 0;
}

}  // namespace rt
