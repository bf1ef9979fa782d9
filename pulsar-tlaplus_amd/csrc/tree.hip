// pulsar-tlaplus_amd/csrc/tree.hip -- the component-tree engine's kernel
// (tree.h): one wavefront per component of a layer, the component's FPSet in
// LDS, a multi-source BFS whose sources are the parent component's states
// with the layer's message appended.
#include "tree.h"

#include "component_model.h"
#include "kernels.h"

namespace tlcg {

namespace {

template <int CAP>
__global__ __launch_bounds__(64) void k_tree(TreeArgs a) {
  constexpr int T = 2 * CAP;  // FPSet slots (load <= 1/2)
  constexpr int LOG2T = CAP == 512 ? 10 : 11;
  __shared__ uint32_t h[T];             // local key + 1, 0 = empty
  __shared__ uint32_t keys[CAP];        // the component's local keys in BFS (depth) order
  __shared__ unsigned long long lvl_d[TREE_MAXLV], lvl_g[TREE_MAXLV];
  const Layout& L = a.L;
  const int lane = threadIdx.x;
  const int mb = L.msg_sh + L.N * L.mw;  // `messages` (with its length) occupies the low mb bits
  for (int i = lane; i < TREE_MAXLV; i += 64) lvl_d[i] = lvl_g[i] = 0;
  unsigned flags = 0;
  for (u64 ci = blockIdx.x; ci < a.n_comp; ci += gridDim.x) {
    for (int i = lane; i < T; i += 64) h[i] = 0;
    __syncthreads();
    // the parent component and the message this component appends to it
    u64 np, pc = 0;
    int j = 0;
    if (a.layer == 0) {
      np = a.n_init;
    } else {
      pc = ci / (u64)L.nkv;
      j = (int)(ci % (u64)L.nkv);
      np = a.par_n[pc];
    }
    const u64* pst = a.layer ? a.par_states + pc * CAP : nullptr;
    const uint8_t* pdep = a.layer ? a.par_dep + pc * CAP : nullptr;
    const u64 pgb = a.par_gbase + pc * CAP;
    const u64 w0 = a.layer == 0 ? init_state(L, 0) : producer_succ(L, pst[0], a.layer - 1, j);
    const u64 msgs = w0 & L.msgs_mask;
    const CompMsgs cm = comp_msgs_init(L, w0);  // everything that reads only `messages`
    const int nprod = cm.len < L.N ? L.nkv : 0;  // Producer's successors (into the children)
    u64* st = a.states + ci * CAP;
    u64* par = a.parents + ci * CAP;
    uint8_t* dp = a.dep + ci * CAP;
    const u64 gb = a.gbase + ci * CAP;
    int n = 0;  // states so far (wave-uniform)
    // insert the lanes' candidates (pred) at depth d: LDS CAS on the key, the
    // new ones appended in lane order; returns false past the capacity
    auto insert = [&](bool pred, lkey key, u64 pref, int d) {
      bool isnew = false;
      if (pred) {
        unsigned s = (key * 0x9E3779B1u) >> (32 - LOG2T);
        for (int p = 0; p < T; ++p) {
          const uint32_t old = atomicCAS(&h[s], 0u, key + 1u);
          if (old == 0) {
            isnew = true;
            break;
          }
          if (old == key + 1u) break;
          s = (s + 1) & (T - 1);
        }
      }
      const u64 m = __ballot(isnew);
      const int cnt = __popcll(m);
      if (n + cnt > CAP) {
        flags |= TREE_OVERFLOW;
      } else if (isnew) {
        const int pos = n + __popcll(m & lanemask_lt());
        keys[pos] = key;
        const u64 w = msgs | ((u64)key << mb);
        st[pos] = w;
        par[pos] = pref == NO_PARENT ? NO_PARENT : (a.rank_tag | pref);
        dp[pos] = (uint8_t)d;
        if (check_invariants_k(L, cm, key) >= 0) flags |= TREE_EVENT;  // the global engine reports it
      }
      n = n + cnt > CAP ? CAP : n + cnt;
    };
    u64 e = 0;   // next entry (parent state, or initial state at layer 0)
    int f0 = 0;  // first state of the current depth
    int d = 0;
    while (true) {
      // the next depth: the frontier's, or past a gap the next entries'
      if (f0 == n) {
        if (e >= np) break;
        d = a.layer == 0 ? 0 : (int)pdep[e] + 1;
      }
      if (d >= TREE_MAXLV - 1) {
        flags |= TREE_OVERFLOW;
        break;
      }
      // the entries at depth d (parents at depth d - 1; pdep is nondecreasing)
      while (e < np) {
        const u64 i = e + (u64)lane;
        bool ok = i < np;
        lkey key = 0;
        u64 pref = NO_PARENT;
        if (ok && a.layer == 0) {
          key = (lkey)(init_state(L, i) >> mb);
        } else if (ok) {
          ok = (int)pdep[i] + 1 == d;
          key = (lkey)(producer_succ(L, pst[i], a.layer - 1, j) >> mb);
          pref = ((pgb + i) << L.ord_bits) | (u64)ordinal_of(L, ACT_PRODUCER, j);
        }
        insert(ok, key, pref, d);
        const int taken = __popcll(__ballot(ok));
        e += (u64)taken;
        if (taken < 64) break;
      }
      __syncthreads();
      const int f1 = n;  // depth d = [f0, f1)
      // expand depth d: compactor and BrokerCrash successors at depth d + 1
      u64 gen = 0;
      for (int b = f0; b < f1; b += 64) {
        const int i = b + lane;
        const bool ok = i < f1;
        const lkey k = ok ? keys[i] : 0;
        lkey t = 0, t2 = 0;
        int act = 0;
        const int r = ok ? compactor_step_k(L, cm, msgs, k, k_phase(L, k), &t, &act) : 0;
        const bool crash = ok && crash_step_k(L, k, &t2);
        const int nsucc = nprod + (r == 1) + (int)crash + selfloop_count_k(L, cm, k);
        if (ok) {
          gen += (u64)nsucc;
          if (r == 2 || (nsucc == 0 && L.check_deadlock)) flags |= TREE_EVENT;
        }
        const u64 pref = (gb + (u64)i) << L.ord_bits;
        insert(r == 1, t, pref | (u64)ordinal_of(L, act, 0), d + 1);
        insert(crash, t2, pref | (u64)ordinal_of(L, ACT_CRASH, 0), d + 1);
      }
      gen = wave_sum_u64(gen);
      if (lane == 0) {
        lvl_d[d] += (unsigned long long)(f1 - f0);
        lvl_g[d] += gen;
      }
      __syncthreads();
      f0 = f1;
      ++d;
      if (__ballot(flags != 0)) break;  // (wave-uniform) the global engine takes the model
    }
    if (lane == 0) a.n_out[ci] = (uint32_t)n;
    __syncthreads();
  }
  // one wave per workgroup: fold the lanes' flags, then the per-depth counts
  const u64 fl = __ballot(flags & TREE_EVENT) ? TREE_EVENT : 0;
  const u64 fo = __ballot(flags & TREE_OVERFLOW) ? TREE_OVERFLOW : 0;
  if (lane == 0 && (fl | fo)) atomicOr(a.flags, (unsigned)(fl | fo));
  for (int i = lane; i < TREE_MAXLV; i += 64) {
    if (lvl_d[i]) atomicAdd(&a.lvl[i], lvl_d[i]);
    if (lvl_g[i]) atomicAdd(&a.lvl_gen[i], lvl_g[i]);
  }
}

}  // namespace

bool launch_tree(const TreeArgs& a, int cap, hipStream_t stream) {
  if (!a.n_comp) return true;
  const unsigned grid = (unsigned)(a.n_comp < 16384 ? a.n_comp : 16384);
  if (cap == 512) k_tree<512><<<grid, 64, 0, stream>>>(a);
  else k_tree<1024><<<grid, 64, 0, stream>>>(a);
  return hipGetLastError() == hipSuccess;
}

}  // namespace tlcg
