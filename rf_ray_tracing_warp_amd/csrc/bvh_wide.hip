// bvh_wide.hip -- collapse the binary BVH (either builder, after pack_leaf_refs) into 4-wide
// nodes for rt::Walk4 (rt_bvh.h).  Host pass over the device tree: every wide node takes the
// children of one binary node and keeps opening its largest inner child (surface area) until it
// has four, or until opening more would let the walk's stack bound exceed RT_BVH_STACK; nodes are
// numbered breadth first, so the top levels are contiguous from node 0.  (A depth-first preorder
// numbering was bit-identical and no faster -- K4 rt_trace 721-724 us either way, K5 map 3.31 vs
// 3.27 ms, profiles/r6d_*_bvh_dfs_layout_ab.jsonl: a node is exactly one 128-B line, so renumbering
// changes which lines neighbour each other, not how many distinct lines a wave touches.)
// The child boxes and leaf references are copied bit for bit from the binary nodes, so culling
// is exactly as conservative as the binary traversal's.
#include <math.h>

#include <cmath>

#include <cstring>

#include <algorithm>
#include <vector>

#include "../../include/rfrt.h"
#include "rt_bvh.h"
#include "rt_internal.h"

namespace {

struct Child {
  float box[6];  // lo.xyz hi.xyz
  bool inner;
  int id;  // binary node index (inner) or packed leaf first << 3 | count
};

double half_area(const float* b) {
  if (!(b[3] >= b[0])) return 0.0;
  const double ex = (double)b[3] - b[0], ey = (double)b[4] - b[1], ez = (double)b[5] - b[2];
  return ex * ey + ey * ez + ez * ex;
}

}  // namespace

namespace rt {

// The tree as 4-wide nodes (the 128-B nodes of Walk4): every wide node takes the children of one
// binary node and keeps opening its largest inner child (surface area) until it has four, within
// the traversal stack's budget.  (A compressed 8-wide form -- 8-bit child bounds on a per-node
// power-of-two grid -- was bit-identical and slower, K4 973 -> 1175 us; removed in round 5, last
// in commit 43de9a4)
int build_wide(rt_mesh* m) {
  if (!m->nodes || m->nnodes <= 0) return RT_OK;
  constexpr int W = 4;
  std::vector<float> bin((size_t)m->nnodes * 16);
  RT_HIP(hipMemcpy(bin.data(), m->nodes, bin.size() * sizeof(float), hipMemcpyDeviceToHost));
  auto children = [&](int n, Child* out) {
    const float* q = bin.data() + 16 * (size_t)n;
    for (int side = 0; side < 2; ++side) {
      Child& c = out[side];
      for (int k = 0; k < 6; ++k) c.box[k] = q[6 * side + k];
      int ref, pk;
      std::memcpy(&ref, &q[12 + side], 4);
      std::memcpy(&pk, &q[14 + side], 4);
      c.inner = ref >= 0;
      c.id = ref >= 0 ? ref : pk;
    }
  };
  // height of every binary node (0: no inner child), iteratively: the builders number their
  // nodes in different orders, so no index order is bottom-up
  std::vector<int> height((size_t)m->nnodes, -1);
  {
    std::vector<int> st{0};
    while (!st.empty()) {
      const int n = st.back();
      Child two[2];
      children(n, two);
      int h = 0;
      bool ready = true;
      for (const Child& c : two)
        if (c.inner) {
          if (height[c.id] < 0) {
            st.push_back(c.id);
            ready = false;
          } else {
            h = std::max(h, height[c.id] + 1);
          }
        }
      if (ready) {
        height[n] = h;
        st.pop_back();
      }
    }
  }
  // Stack budget: a wide node w with occ[w] entries pending above it and binary height h(w) never
  // needs more than occ[w] + h(w) entries below it if nothing under it is opened (each binary
  // level pushes <= 1).  A child is opened only while every resulting inner child c keeps
  // occ(c) + h(c) <= budget, so the 4-wide walk can never overflow its stack: a deep or skewed
  // tree degrades towards binary-like nodes instead of being rejected.
  const int budget = RT_BVH_STACK - 1;
  if (height[0] > budget) {
    set_error("rt_mesh_create: BVH deeper than the traversal stack");
    return RT_EINVAL;
  }
  std::vector<int> order{0};  // binary node of every wide node, breadth first
  std::vector<int> occ{0};    // stack entries pending above a node: parents' extra inner children
  int max_occ = 0;
  std::vector<float> wide;
  wide.reserve((size_t)m->nnodes / 2 * 32);
  auto fits = [&](const Child* ch, int k, int o) {
    int inner = 0;
    for (int c = 0; c < k; ++c) inner += ch[c].inner;
    for (int c = 0; c < k; ++c)
      if (ch[c].inner && o + inner - 1 + height[ch[c].id] > budget) return false;
    return true;
  };
  for (size_t w = 0; w < order.size(); ++w) {
    Child ch[W];
    children(order[w], ch);
    int k = 2;
    while (k < W) {
      int j = -1;
      double best = -1.0;
      for (int c = 0; c < k; ++c)
        if (ch[c].inner && half_area(ch[c].box) > best) {
          best = half_area(ch[c].box);
          j = c;
        }
      if (j < 0) break;
      Child two[2], keep = ch[j];
      children(ch[j].id, two);
      ch[j] = two[0];
      ch[k] = two[1];
      if (!fits(ch, k + 1, occ[w])) {  // opening would let a subtree outgrow the stack
        ch[j] = keep;
        break;
      }
      ++k;
    }
    float node[32];
    int inner = 0;
    for (int c = 0; c < k; ++c) inner += ch[c].inner;
    for (int c = 0; c < 4; ++c) {
      int ref = -1;  // empty slot
      if (c < k) {
        for (int a = 0; a < 3; ++a) {
          node[8 * a + c] = ch[c].box[a];          // lo.{x,y,z}
          node[8 * a + 4 + c] = ch[c].box[3 + a];  // hi.{x,y,z}
        }
        if (ch[c].inner) {
          ref = (int)order.size();
          order.push_back(ch[c].id);
          occ.push_back(occ[w] + inner - 1);
          max_occ = std::max(max_occ, occ.back());
        } else {
          ref = ~ch[c].id;  // count 0 (an empty leaf) gives -1, the empty slot
        }
      } else {
        for (int a = 0; a < 3; ++a) {
          node[8 * a + c] = INFINITY;
          node[8 * a + 4 + c] = -INFINITY;
        }
      }
      std::memcpy(&node[24 + c], &ref, 4);
      node[28 + c] = 0.0f;
    }
    wide.insert(wide.end(), node, node + 32);
  }
  if (max_occ + 1 > RT_BVH_STACK) {  // cannot happen: the budget above bounds every occ
    set_error("rt_mesh_create: internal error, wide-node stack bound exceeded");
    return RT_EINVAL;
  }
  m->wide_stack = max_occ;
  if (m->wide) (void)hipFree(m->wide);
  m->wide = nullptr;
  m->nwide = (int64_t)order.size();
  RT_HIP(hipMalloc(&m->wide, wide.size() * sizeof(float)));
  RT_HIP(hipMemcpy(m->wide, wide.data(), wide.size() * sizeof(float), hipMemcpyHostToDevice));
  return RT_OK;
}

}  // namespace rt
