// pulsar-tlaplus_amd/csrc/tree.hip -- precompiled component-tree kernels
// (runtime layout); jit.cpp builds layout-specialized ones from the same
// tree_body.h.
#include "tree.h"

#include "tree_body.h"

namespace tlcg {

namespace {

template <int CAP, int T, int G, bool CLOSED, typename W>
__global__ __launch_bounds__(64) void k_tree(TreeArgs a) {
  tree_body<CAP, T, G, CLOSED, W>(a, a.L);
}

template <int CAP, int T, int G, bool CLOSED = false, typename W = u64>
void launch_g(const TreeArgs& a, hipStream_t stream) {
  k_tree<CAP, T, G, CLOSED, W><<<tree_grid(a.n_comp, G), 64, 0, stream>>>(a);
}

}  // namespace

bool launch_tree(const TreeArgs& a, int cap, int groups, bool closed, int words, hipStream_t stream) {
  if (!a.n_comp) return true;
  if (closed) {
    if (cap == 640 && groups == 2) {
      if (words == 2) launch_g<640, 1024, 2, true, u128>(a, stream);
      else launch_g<640, 1024, 2, true, u64>(a, stream);
    } else if (cap == 640) {
      if (words == 2) launch_g<640, 1024, 4, true, u128>(a, stream);
      else launch_g<640, 1024, 4, true, u64>(a, stream);
    } else {
      if (words == 2) launch_g<2048, 4096, 1, true, u128>(a, stream);
      else launch_g<2048, 4096, 1, true, u64>(a, stream);
    }
  } else if (cap == 384) {
    if (groups == 4) launch_g<384, 512, 4>(a, stream);
    else if (groups == 2) launch_g<384, 512, 2>(a, stream);
    else launch_g<384, 512, 1>(a, stream);
  } else {
    launch_g<1024, 2048, 1>(a, stream);
  }
  return hipGetLastError() == hipSuccess;
}

}  // namespace tlcg
