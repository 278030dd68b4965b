// bvh_wide.hip -- collapse the binary BVH (either builder, after pack_leaf_refs) into 4-wide
// nodes for rt::Walk4, or compressed 8-wide nodes for rt::Walk8 (rt_bvh.h, RT_BVH_WIDTH).  Host pass over the device tree: every wide node takes the
// children of one binary node and keeps opening its largest inner child (surface area) until it
// has four, or until opening more would let the walk's stack bound exceed RT_BVH_STACK; nodes are
// numbered breadth first, so the top levels are contiguous from node 0.
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

namespace {
// One 8-wide node in the compressed form of rt::Walk8 (rt_bvh.h), from its k <= 8 children.
// Every child box is quantised to 8 bits per bound on a per-axis grid origin + q * 2^e with
// origin = the node's box low corner: the low bound rounded down and the high bound up, checked
// in the very f32 arithmetic the device decodes with (fmaf(q, 2^e, origin): q * 2^e is exact, so
// both sides round the same exact sum once).  The decoded box therefore always contains the
// binary tree's (already outward-rounded and padded) box, and culling stays conservative.
void emit_node8(const Child* ch, int k, const int* ref, float* node) {
  for (int i = 0; i < 32; ++i) node[i] = 0.0f;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  auto used = [&](int c) { return c < k && ref[c] != -1 && ch[c].box[0] <= ch[c].box[3] &&
                                   ch[c].box[1] <= ch[c].box[4] && ch[c].box[2] <= ch[c].box[5]; };
  for (int c = 0; c < k; ++c)
    if (used(c))
      for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], ch[c].box[a]);
      hi[a] = std::max(hi[a], ch[c].box[3 + a]);
    }
  uint8_t q[6][8];  // lo.x hi.x lo.y hi.y lo.z hi.z
  uint32_t ebits = 0;
  for (int a = 0; a < 3; ++a) {
    const float o = lo[a] <= hi[a] ? lo[a] : 0.0f;
    const double ext = lo[a] <= hi[a] ? (double)hi[a] - (double)lo[a] : 0.0;
    int e = -126;
    while (e < 127 && std::ldexp(255.0, e) < ext) ++e;
    for (;; ++e) {  // grow the step until every high bound fits in 255 steps
      const float sc = std::ldexp(1.0f, e);
      bool ok = true;
      for (int c = 0; c < 8 && ok; ++c) {
        if (!used(c)) {
          q[2 * a][c] = 255;  // empty slot (its reference says so; the box is never used)
          q[2 * a + 1][c] = 0;
          continue;
        }
        const float l = ch[c].box[a], h = ch[c].box[3 + a];
        long ql = (long)std::floor(((double)l - (double)o) / (double)sc);
        ql = std::max(0L, std::min(255L, ql));
        while (ql > 0 && (float)(o + (float)ql * sc) > l) --ql;
        long qh = (long)std::ceil(((double)h - (double)o) / (double)sc);
        qh = std::max(0L, qh);
        while (qh <= 255 && (float)(o + (float)qh * sc) < h) ++qh;
        if (qh > 255 || (float)(o + (float)ql * sc) > l) {
          ok = false;
          break;
        }
        q[2 * a][c] = (uint8_t)ql;
        q[2 * a + 1][c] = (uint8_t)qh;
      }
      if (ok || e >= 127) break;
    }
    node[a] = o;
    ebits |= (uint32_t)(e + 127) << (8 * a);
  }
  std::memcpy(&node[3], &ebits, 4);
  std::memcpy(&node[4], &q[0][0], 48);  // dwords 4..15: lo.x[8] hi.x[8] lo.y[8] hi.y[8] lo.z[8] hi.z[8]
  std::memcpy(&node[16], ref, 32);      // dwords 16..23: child refs
}
}  // namespace

// The tree as RT_BVH_WIDTH-wide nodes (4: the uncompressed 128-B nodes of Walk4; 8: the
// compressed 128-B nodes of Walk8).  Both collapse the binary tree the same way: every wide node
// takes the children of one binary node and keeps opening its largest inner child (surface area)
// until it has W, within the traversal stack's budget.
int build_wide(rt_mesh* m) {
  if (!m->nodes || m->nnodes <= 0) return RT_OK;
  constexpr int W = RT_BVH_WIDTH == 8 ? 8 : 4;
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
    Child ch[8];
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
    if (W == 8) {
      int ref[8];
      for (int c = 0; c < 8; ++c) {
        ref[c] = -1;  // empty slot
        if (c >= k) continue;
        if (ch[c].inner) {
          ref[c] = (int)order.size();
          order.push_back(ch[c].id);
          occ.push_back(occ[w] + inner - 1);
          max_occ = std::max(max_occ, occ.back());
        } else {
          ref[c] = ~ch[c].id;  // count 0 (an empty leaf) gives -1, the empty slot
        }
      }
      emit_node8(ch, k, ref, node);
      wide.insert(wide.end(), node, node + 32);
      continue;
    }
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
