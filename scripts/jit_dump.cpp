// scripts/jit_dump.cpp -- compile the hipRTC-specialized kernels for a G9-like
// model offline (no GPU needed) and write the source + code object, so the
// ISA of the specialized component kernel can be read with llvm-objdump.
//   g++ -std=c++17 -I../include -Icsrc -o /tmp/jit_dump ../scripts/jit_dump.cpp -Llib -ltlcgpu
//   TLCG_JIT_DUMP=/tmp/g9.hip /tmp/jit_dump 15
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "host_model.h"
#include "jit.h"

int main(int argc, char** argv) {
  const int k = argc > 1 ? std::atoi(argv[1]) : 15;
  tlcg_model m{};
  m.msg_sent_limit = 3;
  m.compaction_times_limit = argc > 2 ? std::atoi(argv[2]) : 3;
  m.consume_times_limit = 2;
  m.max_crash_times = 1;
  m.retain_null_key = 1;
  m.check_deadlock = 1;
  m.n_keys = m.n_values = k;
  for (int i = 0; i < k; ++i) m.keys[i] = m.values[i] = i + 1;
  m.n_invariants = 2;
  m.invariants[0] = TLCG_INV_TYPESAFE;
  m.invariants[1] = TLCG_INV_HORIZON_CORRECTNESS;
  tlcg::HostModel hm;
  std::string err;
  if (!tlcg::build_model(m, &hm, &err)) {
    std::fprintf(stderr, "%s\n", err.c_str());
    return 1;
  }
  std::vector<char> code;
  if (!tlcg::jit_compile(hm.L, "gfx950", &code, &err)) {
    std::fprintf(stderr, "%s\n", err.c_str());
    return 1;
  }
  std::printf("code object %zu bytes\n", code.size());
  return 0;
}
