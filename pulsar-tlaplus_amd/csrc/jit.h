// pulsar-tlaplus_amd/csrc/jit.h -- run-time specialization of the hot kernels
// for one model's constants (hipRTC; the layout becomes a constexpr, so every
// field shift folds and every loop over N / C / invariants unrolls).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "component.h"
#include "expand_fast.h"
#include "kernels.h"
#include "tree.h"

namespace tlcg {

// the parts of the specialized source (jit.cpp program_source): one module each
// JIT_WAVE_BIG: the wave kernels for a model with many components
// (jit_build: WAVE_M_BIG components per lane at a 6-waves-per-SIMD target)
enum JitPart { JIT_MAIN = 0, JIT_CHECK = 1, JIT_WAVE = 2, JIT_WAVE_BIG = 3 };

struct JitKernels {
  hipModule_t module = nullptr;
  hipModule_t wave_module = nullptr;  // JIT_WAVE
  hipFunction_t component[4] = {nullptr, nullptr, nullptr, nullptr};     // K = 32, 64, 128, 255
  hipFunction_t component_od[4] = {nullptr, nullptr, nullptr, nullptr};  // the same, counting outdegrees
  hipFunction_t code[2] = {nullptr, nullptr};     // component codes (component_code.h), K = 32, 64
  hipFunction_t code_od[2] = {nullptr, nullptr};
  hipFunction_t wave[2] = {nullptr, nullptr};     // codes, K = 64, one walk per wave (component_wave.h); outdegrees
  hipFunction_t treew = nullptr;                  // the tree's closed mode at 640 states, one walk per wave (tree_wave.h)
  hipFunction_t treeb = nullptr;                  // the tree's closed mode at 640 states with the bitmap FPSet (tree_body.h BITS)
  hipFunction_t lane[2] = {nullptr, nullptr};     // codes, K = 64, per lane with a bitmap FPSet (component_lane.h); outdegrees
  hipFunction_t expand_fast[2] = {nullptr, nullptr};  // the global engine's fast level (expand_fast.h), 2 parents per thread; PROBE 0 / 1
  int wave_m = WAVE_M;                            // its components per lane (the grid)
  std::string wave_error;                         // why the wave kernels are unset (jit_build), else empty
  hipFunction_t tree[4] = {nullptr, nullptr, nullptr, nullptr};  // component tree: 384 x 4 groups, 1024 x 1;
                                                                 // closed mode: 640 x 4, 2048 x 1
  double compile_s = 0;  // 0 when loaded from the cache
  bool cached = false;
};

// builds (or loads from $TLCG_JIT_CACHE, default /tmp/tlcgpu-jit) the
// kernels specialized for L on `device`; false with a message on failure.
// `user`: the model's user invariants as device code (user_device_source),
// which the kernels then evaluate in the cfg's order with the spec's own.
// n_comp: the components the context's model has (closed partitions: this
// rank's share), which picks the wave module's variant (JIT_WAVE_BIG from
// WAVE_BIG_COMPS on, without user invariants)
bool jit_build(const Layout& L, int device, JitKernels* out, std::string* err, const std::string& user = "",
               uint64_t n_comp = 0);
// compile only (no device needed): the code object for `arch`
// (part: JitPart -- JIT_CHECK the user-check kernel alone, jit_build_user_check; JIT_WAVE the wave kernels)
bool jit_compile(const Layout& L, const std::string& arch, std::vector<char>* code, std::string* err,
                 const std::string& user = "", int part = JIT_MAIN);
void jit_release(JitKernels* k);
// (wave: the first pass's kernel with one walk of the code graph per wave, component_wave.h)
// (lane: the per-lane code pass with a bitmap FPSet, component_lane.h)
bool jit_launch_component(const JitKernels& k, const CompArgs& a, int K, bool code, hipStream_t stream,
                          bool wave = false, bool lane = false);
// the global engine's user-invariant check (kernels.h user_check_body) as
// device code: a module of its own, so a global-engine check does not wait
// for the on-chip engines' kernels to compile
struct JitUserCheck {
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;
  double compile_s = 0;
};
bool jit_build_user_check(const Layout& L, int device, const std::string& user, JitUserCheck* out, std::string* err);
void jit_release_user_check(JitUserCheck* k);
bool jit_launch_user_check(const JitUserCheck& k, const UserCheckArgs& a, hipStream_t stream);

// the specialized tree kernel for cap 384 / 640 (4 groups) or 1024 / 2048 (1 group); false when not built or on a
// launch error
// the closed tree at 640 states with one walk per wave (tree_wave.h: the
// lane-interleaved store, tree_wave_slot)
bool jit_launch_tree_wave(const JitKernels& k, const TreeArgs& a, hipStream_t stream);
bool jit_launch_tree(const JitKernels& k, const TreeArgs& a, int cap, hipStream_t stream);
// the closed tree at 640 states with the bitmap FPSet (tree_body.h BITS; TreeArgs::owner set)
bool jit_launch_tree_bits(const JitKernels& k, const TreeArgs& a, hipStream_t stream);
// the global engine's fast level, layout-specialized (expand_fast.h): false when not built or on a launch error
bool jit_launch_expand_fast(const JitKernels& k, const ExpandArgs& a, unsigned grid, int probe, hipStream_t stream);

}  // namespace tlcg
