// pulsar-tlaplus_amd/csrc/component.hip -- precompiled component-engine
// kernels (runtime layout); jit.cpp builds layout-specialized ones.
#include "component.h"

#include "component_body.h"

namespace tlcg {

namespace {

template <int K, bool OD, bool CODE>
__global__ __launch_bounds__(64) void k_component(CompArgs a) {
  component_body<K, OD, CODE>(a, a.L);
}

template <bool OD>
void launch_k(const CompArgs& a, int K, bool code, unsigned grid, hipStream_t stream) {
  if (code && K == 32) k_component<32, OD, true><<<grid, 64, 0, stream>>>(a);
  else if (code) k_component<64, OD, true><<<grid, 64, 0, stream>>>(a);
  else if (K == 32) k_component<32, OD, false><<<grid, 64, 0, stream>>>(a);
  else if (K == 64) k_component<64, OD, false><<<grid, 64, 0, stream>>>(a);
  else if (K == 128) k_component<128, OD, false><<<grid, 64, 0, stream>>>(a);
  else k_component<255, OD, false><<<grid, 64, 0, stream>>>(a);
}

}  // namespace

bool launch_component(const CompArgs& a, int K, bool code, hipStream_t stream) {
  if (!a.n_comp) return true;
  const u64 batches = (a.n_comp + 63) / 64;
  const unsigned grid = (unsigned)(batches < comp_grid_cap() ? batches : comp_grid_cap());
  if (a.outdeg) launch_k<true>(a, K, code && K <= 64, grid, stream);
  else launch_k<false>(a, K, code && K <= 64, grid, stream);
  return hipGetLastError() == hipSuccess;
}

}  // namespace tlcg
