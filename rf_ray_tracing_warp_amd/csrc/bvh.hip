// bvh.hip -- BVH for environment meshes above RT_BRUTE_MAX_FACES (placeholder until the
// traversal kernel lands; large meshes are rejected by rt_trace until then).
#include <vector>

#include "rt_internal.h"

namespace rt {
int build_bvh(rt_mesh* m, const std::vector<float>& tri) {
  (void)m;
  (void)tri;
  return 0;
}
}  // namespace rt
