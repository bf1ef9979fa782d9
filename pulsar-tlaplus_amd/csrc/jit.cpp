// pulsar-tlaplus_amd/csrc/jit.cpp -- hipRTC specialization of the component
// kernel (see jit.h).  The source is the same component_body.h the
// precompiled kernel uses, plus `constexpr Layout kL = {...}`.
#include "jit.h"
#include "host_model.h"

#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

#include "jit_sources.inc"

namespace tlcg {

namespace {

std::string layout_literal(const Layout& L) {
  std::ostringstream o;
  o << "constexpr tlcg::Layout kL = {";
#define F(x) o << "." #x " = " << L.x << ", ";
  F(N) F(C) F(K) F(ctl) F(nk) F(nv) F(nkv) F(kb) F(vb) F(mw) F(len_sh) F(len_w) F(msg_sh) F(led_sh) F(led_w)
  F(p1r_sh) F(p1r_w) F(cur_sh) F(curh_w) F(curc_w) F(ph_sh) F(hz_sh) F(hz_w) F(ctx_sh) F(ctx_w) F(cr_sh) F(cr_w)
  F(bits) F(retain) F(producer) F(consumer) F(term_ok) F(check_deadlock) F(ord_bits) F(n_inv)
#undef F
  o << ".inv = {";
  for (int i = 0; i < 8; ++i) o << L.inv[i] << (i < 7 ? ", " : "");
  // (every field: defer_inv keeps the specialized global-engine expand from
  // evaluating user invariants, which its level's check kernel evaluates)
  o << "}, .defer_inv = " << L.defer_inv << ", .msgs_mask = " << L.msgs_mask << "ull, .led_present_mask = "
    << L.led_present_mask << "ull, .msgs_mask_hi = " << L.msgs_mask_hi << "ull, .led_present_mask_hi = "
    << L.led_present_mask_hi << "ull};\n";
  return o.str();
}

// part: 0 the on-chip engines' kernels; 1 (JIT_CHECK) the user-invariant
// check kernel alone (tlcg_user_check, the global engine's; compiles in a
// fraction of the whole module's time); 2 (JIT_WAVE) the component code
// pass's one-walk-per-wavefront kernels, a module of their own so that they
// are scheduled with options of their own (jit_opts)
std::string program_source(const Layout& L, const std::string& user, int part = JIT_MAIN) {
  const bool check_only = part == JIT_CHECK;
  std::string s = "typedef unsigned char uint8_t; typedef unsigned short uint16_t; typedef unsigned int uint32_t; typedef int int32_t;\n"
                  "typedef unsigned long uint64_t; typedef long int64_t;\n";
  // user invariants: the headers' check functions call tlcg_user_eval (model.h)
  if (!user.empty()) s += "#define TLCG_USER_INV 1\n";
  // tuning experiments: TLCG_JIT_DEFINES="A=1;B" becomes #define lines (part of the cache key)
  if (const char* d = std::getenv("TLCG_JIT_DEFINES")) {
    std::string all(d);
    size_t i = 0;
    while (i < all.size()) {
      size_t j = all.find(';', i);
      if (j == std::string::npos) j = all.size();
      std::string kv = all.substr(i, j - i);
      const size_t eq = kv.find('=');
      if (!kv.empty()) s += "#define " + (eq == std::string::npos ? kv : kv.substr(0, eq) + " " + kv.substr(eq + 1)) + "\n";
      i = j + 1;
    }
  }
  // the big-model wave variant's components per lane and occupancy target:
  // defined before the headers, whose own defaults (component_wave.h) they
  // replace (jit_build checks the module's tlcg_wave_m against the host's)
  if (part == JIT_WAVE_BIG)
    s += "#ifndef TLCG_WAVE_M\n#define TLCG_WAVE_M " + std::to_string(WAVE_M_BIG) +
         "\n#endif\n#ifndef TLCG_WAVE_ATTR\n#define TLCG_WAVE_ATTR __attribute__((amdgpu_waves_per_eu(6)))\n#endif\n";
  // the per-lane pass's FIFO ring: as few entries as component 0's widest
  // queue needs (host_model.cpp lane_ring_entries; G9: 8 instead of 16, 1 KB
  // less LDS and fewer registers: G9 3.49-3.53 -> 3.37-3.43 ms,
  // profiles/r06_probe_lane_r.jsonl), and 8 waves per SIMD (<= 64 VGPRs) --
  // both together 3.30 ms; a define in TLCG_JIT_DEFINES wins
  if (part == JIT_MAIN) {
    s += "#ifndef TLCG_LANE_R\n#define TLCG_LANE_R " + std::to_string(lane_ring_entries(L)) + "\n#endif\n";
    if (user.empty()) s += "#ifndef TLCG_LANE_ATTR\n#define TLCG_LANE_ATTR __attribute__((amdgpu_waves_per_eu(8)))\n#endif\n";
  }
  s += kJitSource;
  s += "\n" + layout_literal(L);
  s += user;
  // the layout's word: u64, or u128 past 63 bits
  const std::string w = L.bits <= 63 ? "tlcg::u64" : "tlcg::u128";
  if (check_only) {
    s += "extern \"C\" __global__ __launch_bounds__(256) void tlcg_user_check(tlcg::UserCheckArgs a) "
         "{ tlcg::user_check_body<" + w + ">(a, kL); }\n";
    return s;
  }
  if (part == JIT_WAVE || part == JIT_WAVE_BIG) {
    // the module's components per lane, read back by jit_build: the host's
    // grid and record tables (crec_index) must use the kernel's M
    s += "namespace tlcg { extern \"C\" __constant__ int tlcg_wave_m = TLCG_WAVE_M; }\n";
    // the first pass with one walk of the code graph per wave (component_wave.h)
    // (TLCG_WAVE_ATTR: a tuning hook for the kernels' attributes, e.g. an
    // occupancy target amdgpu_waves_per_eu; empty by default)
    s += "#ifndef TLCG_WAVE_ATTR\n#define TLCG_WAVE_ATTR\n#endif\n";
    for (const char* od : {"false", "true"})
      s += std::string("extern \"C\" __global__ __launch_bounds__(64) TLCG_WAVE_ATTR void tlcg_componentw") +
           (od[0] == 't' ? "od" : "") + "_64(tlcg::CompArgs a) { tlcg::component_wave_body<64, " + od + ">(a, kL); }\n";
    // the component tree's closed mode, one walk per wave (tree_wave.h)
    s += "extern \"C\" __global__ __launch_bounds__(64) TLCG_WAVE_ATTR void tlcg_treecw_640(tlcg::TreeArgs a) "
         "{ tlcg::tree_wave_body<640, " + w + ">(a, kL); }\n";
    return s;
  }
  for (int K : {32, 64, 128, 255})
    for (const char* od : {"false", "true"})
      for (const char* code : {"false", "true"}) {
        if (code[0] == 't' && K > 64) continue;
        // tlcg_component{_,_od_,c_,cod_}K: c = component codes, od = outdegree counts
        s += std::string("extern \"C\" __global__ __launch_bounds__(64) void tlcg_component") +
             (code[0] == 't' ? (od[0] == 't' ? "cod_" : "c_") : (od[0] == 't' ? "_od_" : "_")) + std::to_string(K) +
             "(tlcg::CompArgs a) { tlcg::component_body<" + std::to_string(K) + ", " + od + ", " + code +
             ">(a, kL); }\n";
      }
  // the global engine's fast level (expand_fast.h), 2 parents per thread, load-then-CAS / CAS-only
  // (one-word layouts only, the kernel's domain)
  if (L.bits <= 63)
    for (int probe : {0, 1})
      s += std::string("extern \"C\" __global__ __launch_bounds__(256) void tlcg_expand_fast_2") + (probe ? "c" : "") +
           "(tlcg::ExpandArgs a) { tlcg::expand_fast_body<2, " + std::to_string(probe) + ">(a, kL); }\n";
  // the per-lane code pass with a bitmap FPSet (component_lane.h; TLCG_LANE_ATTR:
  // a tuning hook for its attributes, e.g. amdgpu_waves_per_eu)
  s += "#ifndef TLCG_LANE_ATTR\n#define TLCG_LANE_ATTR\n#endif\n";
  for (const char* od : {"false", "true"})
    s += std::string("extern \"C\" __global__ __launch_bounds__(64) TLCG_LANE_ATTR void tlcg_componentp") +
         (od[0] == 't' ? "od" : "") + "_64(tlcg::CompArgs a) { tlcg::component_lane_body<64, " + od + ">(a, kL); }\n";
  // (TLCG_TREE_ATTR / TLCG_TREECB_ATTR: tuning hooks for the Producer tree's
  // and the closed tree's bitmap-pass attributes, e.g. amdgpu_waves_per_eu)
  s += "#ifndef TLCG_TREE_ATTR\n#define TLCG_TREE_ATTR\n#endif\n#ifndef TLCG_TREECB_ATTR\n#define TLCG_TREECB_ATTR\n#endif\n";
  s += "extern \"C\" __global__ __launch_bounds__(64) TLCG_TREE_ATTR void tlcg_tree_384(tlcg::TreeArgs a) "
       "{ tlcg::tree_body<384, 512, 4>(a, kL); }\n";
  s += "extern \"C\" __global__ __launch_bounds__(64) void tlcg_tree_1024(tlcg::TreeArgs a) "
       "{ tlcg::tree_body<1024, 2048, 1>(a, kL); }\n";
  // (the closed mode on the layout's word)
  // (TLCG_TREEC_G: components per wavefront of the closed mode, a tuning
  // hook; the launch grid is the same, the kernel strides over the rest)
  s += "#ifndef TLCG_TREEC_G\n#define TLCG_TREEC_G 4\n#endif\n";
  s += "extern \"C\" __global__ __launch_bounds__(64) void tlcg_treec_640(tlcg::TreeArgs a) "
       "{ tlcg::tree_body<640, 1024, TLCG_TREEC_G, true, " + w + ">(a, kL); }\n";
  // (the same with the bitmap FPSet over the host's perfect hash, tree_body.h BITS)
  s += "#ifndef TLCG_TREECB_G\n#define TLCG_TREECB_G " + std::to_string(TREECB_G) + "\n#endif\n";
  s += "extern \"C\" __global__ __launch_bounds__(64) TLCG_TREECB_ATTR void tlcg_treecb_640(tlcg::TreeArgs a) "
       "{ tlcg::tree_body<640, 1024, TLCG_TREECB_G, true, " + w + ", true>(a, kL); }\n";
  s += "extern \"C\" __global__ __launch_bounds__(64) void tlcg_treec_2048(tlcg::TreeArgs a) "
       "{ tlcg::tree_body<2048, 4096, 1, true, " + w + ">(a, kL); }\n";
  return s;
}

// the compile options past -O3: TLCG_JIT_OPTS (tuning experiments), else the
// machine scheduler's max-ILP strategy, which measured faster on every
// specialized kernel (G9 4.74-4.77 -> 4.62-4.63 ms, M8 0.555 -> 0.546,
// G9-deep 17.1 -> 16.4, P8 1.831 -> 1.820, G9 + a user invariant 4.91 ->
// 4.79; interleaved on one box, profiles/r04_probe_sched2.jsonl).  The
// precompiled global-engine kernels showed no steady gain from it (G9 88 / 95
// vs 81 / 99 ms, M8 16.9 vs 17.2; r04_probe_sched_global.jsonl): not used there
// The wave kernels' module (JIT_WAVE) takes the default machine scheduler
// (TLCG_JIT_OPTS_WAVE): max-ILP measured slower there (G9 1.39-1.41 vs 1.28 ms).
std::string jit_opts(int part) {
  const bool wave = part == JIT_WAVE || part == JIT_WAVE_BIG;
  const char* e = std::getenv(wave ? "TLCG_JIT_OPTS_WAVE" : "TLCG_JIT_OPTS");
  return e ? e : wave ? "" : "-mllvm -amdgpu-sched-strategy=max-ilp";
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}

std::string cache_dir() {
  const char* d = std::getenv("TLCG_JIT_CACHE");
  return d && *d ? d : "/tmp/tlcgpu-jit";
}

bool read_all(const std::string& p, std::vector<char>* out) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return false;
  out->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return !out->empty();
}

}  // namespace

bool jit_compile(const Layout& L, const std::string& arch, std::vector<char>* code, std::string* err,
                 const std::string& user, int part) {
  const std::string src = program_source(L, user, part);
  const char* dump_env = std::getenv("TLCG_JIT_DUMP");  // diagnostics: the generated source and code object
  const std::string dump =
      dump_env ? std::string(dump_env) + (part == JIT_CHECK ? ".check" : part >= JIT_WAVE ? ".wave" : "") : "";
  if (dump_env) {
    std::ofstream f(dump);
    f << src;
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "tlcg_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    *err = "hiprtcCreateProgram failed";
    return false;
  }
  const std::string a = "--offload-arch=" + arch;
  std::vector<std::string> extra;
  std::istringstream in(jit_opts(part));
  for (std::string w; in >> w;) extra.push_back(w);
  std::vector<const char*> opts = {a.c_str(), "-O3", "-std=c++20"};
  for (const std::string& w : extra) opts.push_back(w.c_str());
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    *err = "hipRTC compile failed: " + log.substr(0, 4000);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code->resize(n);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  if (dump_env) {
    std::ofstream f(dump + ".co", std::ios::binary);
    f.write(code->data(), (std::streamsize)code->size());
  }
  return true;
}

namespace {

// the code object of program_source(L, user, part) for `device`: from the
// cache, else compiled and cached; loaded into *module
bool load_module(const Layout& L, int device, const std::string& user, int part, hipModule_t* module,
                 bool* cached, double* compile_s, std::string* err) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    *err = "hipGetDeviceProperties failed";
    return false;
  }
  std::string arch = prop.gcnArchName;
  arch = arch.substr(0, arch.find(':'));
  const std::string src = program_source(L, user, part);
  char key[64];
  std::snprintf(key, sizeof key, "%016llx", (unsigned long long)fnv1a(src + "|" + arch + "|v2" + jit_opts(part)));
  const std::string dir = cache_dir();
  const std::string path = dir + "/" + key + "-" + arch + ".co";
  std::vector<char> code;
  *cached = read_all(path, &code);
  if (!*cached) {
    auto t0 = std::chrono::steady_clock::now();
    if (!jit_compile(L, arch, &code, err, user, part)) return false;
    *compile_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    mkdir(dir.c_str(), 0777);
    const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    std::ofstream f(tmp, std::ios::binary);
    if (f.write(code.data(), (std::streamsize)code.size())) {
      f.close();
      std::rename(tmp.c_str(), path.c_str());
    }
  }
  if (hipModuleLoadData(module, code.data()) != hipSuccess) {
    *err = "hipModuleLoadData failed for the specialized kernels";
    return false;
  }
  return true;
}

}  // namespace

bool jit_build_user_check(const Layout& L, int device, const std::string& user, JitUserCheck* out, std::string* err) {
  double cs = 0;
  bool cached = false;
  if (!load_module(L, device, user, JIT_CHECK, &out->module, &cached, &cs, err)) return false;
  out->compile_s = cs;
  if (hipModuleGetFunction(&out->fn, out->module, "tlcg_user_check") != hipSuccess) {
    *err = "hipModuleGetFunction tlcg_user_check";
    return false;
  }
  return true;
}

void jit_release_user_check(JitUserCheck* k) {
  if (k && k->module) hipModuleUnload(k->module);
  if (k) *k = JitUserCheck();
}

bool jit_launch_user_check(const JitUserCheck& k, const UserCheckArgs& a, hipStream_t stream) {
  if (!a.n) return true;
  const uint64_t blocks = (a.n + 255) / 256;
  if (blocks > 0x7fffffffull) return false;
  UserCheckArgs copy = a;
  void* args[] = {&copy};
  return hipModuleLaunchKernel(k.fn, (unsigned)blocks, 1, 1, 256, 1, 1, 0, stream, args, nullptr) == hipSuccess;
}

namespace {

// the wave module (JIT_WAVE / JIT_WAVE_BIG): loaded, its tlcg_wave_m read
// back and checked, its kernels looked up; false with a message otherwise
bool load_wave_module(const Layout& L, int device, const std::string& user, bool big, JitKernels* out,
                      std::string* err) {
  bool wcached = false;
  double wcs = 0;
  if (!load_module(L, device, user, big ? JIT_WAVE_BIG : JIT_WAVE, &out->wave_module, &wcached, &wcs, err))
    return false;
  out->compile_s += wcs;
  // the kernel's own M (component_wave.h TLCG_WAVE_M: WAVE_M, WAVE_M_USER,
  // WAVE_M_BIG, or a tuning define), read from the module: the grid and the
  // walks' record tables are sized by it
  hipDeviceptr_t p = nullptr;
  size_t n = 0;
  int m = 0;
  if (hipModuleGetGlobal(&p, &n, out->wave_module, "tlcg_wave_m") != hipSuccess || n != sizeof(int) ||
      hipMemcpyDtoH(&m, p, sizeof(int)) != hipSuccess || m < 1 || m > 32) {
    *err = "the wave module's tlcg_wave_m could not be read";
    return false;
  }
  const int want = big ? WAVE_M_BIG : user.empty() ? WAVE_M : WAVE_M_USER;
  const char* d = std::getenv("TLCG_JIT_DEFINES");
  if (m != want && !(d && std::strstr(d, "TLCG_WAVE_M="))) {
    *err = "the wave module's M (" + std::to_string(m) + ") is not the expected " + std::to_string(want);
    return false;
  }
  out->wave_m = m;
  if (hipModuleGetFunction(&out->wave[0], out->wave_module, "tlcg_componentw_64") != hipSuccess ||
      hipModuleGetFunction(&out->wave[1], out->wave_module, "tlcg_componentwod_64") != hipSuccess ||
      hipModuleGetFunction(&out->treew, out->wave_module, "tlcg_treecw_640") != hipSuccess) {
    *err = "hipModuleGetFunction tlcg_componentw_64 / tlcg_treecw_640";
    return false;
  }
  return true;
}

}  // namespace

bool jit_build(const Layout& L, int device, JitKernels* out, std::string* err, const std::string& user,
               uint64_t n_comp) {
  const bool big = user.empty() && n_comp >= wave_big_comps();
  if (!load_module(L, device, user, JIT_MAIN, &out->module, &out->cached, &out->compile_s, err)) return false;
  // the wave kernels are optional: a module that fails to build,
  // load or check leaves them unset -- the first passes then run the per-lane
  // kernels (run_component, run_tree) -- and its message in wave_error
  std::string werr;
  if (!load_wave_module(L, device, user, big, out, &werr)) {
    out->wave_error = werr.empty() ? "the wave module failed" : werr;
    if (out->wave_module) hipModuleUnload(out->wave_module);
    out->wave_module = nullptr;
    out->wave[0] = out->wave[1] = out->treew = nullptr;
    out->wave_m = WAVE_M;
  }
  if (hipModuleGetFunction(&out->treeb, out->module, "tlcg_treecb_640") != hipSuccess) {
    *err = "hipModuleGetFunction tlcg_treecb_640";
    return false;
  }
  if (L.bits <= 63 && (hipModuleGetFunction(&out->expand_fast[0], out->module, "tlcg_expand_fast_2") != hipSuccess ||
                       hipModuleGetFunction(&out->expand_fast[1], out->module, "tlcg_expand_fast_2c") != hipSuccess)) {
    *err = "hipModuleGetFunction tlcg_expand_fast_2";
    return false;
  }
  if (hipModuleGetFunction(&out->lane[0], out->module, "tlcg_componentp_64") != hipSuccess ||
      hipModuleGetFunction(&out->lane[1], out->module, "tlcg_componentpod_64") != hipSuccess) {
    *err = "hipModuleGetFunction tlcg_componentp_64";
    return false;
  }
  const char* names[4] = {"32", "64", "128", "255"};
  for (int i = 0; i < 4; ++i)
    for (int od = 0; od < 2; ++od) {
      const std::string n = std::string(od ? "tlcg_component_od_" : "tlcg_component_") + names[i];
      if (hipModuleGetFunction(od ? &out->component_od[i] : &out->component[i], out->module, n.c_str()) != hipSuccess) {
        *err = "hipModuleGetFunction " + n;
        return false;
      }
      if (od == 0) {
        const char* tn = i == 0 ? "tlcg_tree_384" : i == 1 ? "tlcg_tree_1024" : i == 2 ? "tlcg_treec_640" : "tlcg_treec_2048";
        if (hipModuleGetFunction(&out->tree[i], out->module, tn) != hipSuccess) {
          *err = std::string("hipModuleGetFunction ") + tn;
          return false;
        }
      }
      if (i < 2) {
        const std::string nc = std::string(od ? "tlcg_componentcod_" : "tlcg_componentc_") + names[i];
        if (hipModuleGetFunction(od ? &out->code_od[i] : &out->code[i], out->module, nc.c_str()) != hipSuccess) {
          *err = "hipModuleGetFunction " + nc;
          return false;
        }
      }
    }
  return true;
}

void jit_release(JitKernels* k) {
  if (k && k->module) hipModuleUnload(k->module);
  if (k && k->wave_module) hipModuleUnload(k->wave_module);
  if (k) *k = JitKernels();
}

bool jit_launch_component(const JitKernels& k, const CompArgs& a, int K, bool code, hipStream_t stream, bool wave,
                          bool lane) {
  if (!a.n_comp) return true;
  const int i = K == 32 ? 0 : K == 64 ? 1 : K == 128 ? 2 : 3;
  hipFunction_t f = a.outdeg ? k.component_od[i] : k.component[i];
  if (code && i < 2) f = a.outdeg ? k.code_od[i] : k.code[i];
  const bool w = wave && code && K == 64;
  if (w) f = a.outdeg ? k.wave[1] : k.wave[0];
  if (!w && lane && code && K == 64) f = a.outdeg ? k.lane[1] : k.lane[0];
  if (!f) return false;
  const uint64_t batches = w ? (a.n_comp + 64 * (u64)k.wave_m - 1) / (64 * (u64)k.wave_m) : (a.n_comp + 63) / 64;
  const unsigned grid = (unsigned)(batches < comp_grid_cap() ? batches : comp_grid_cap());
  CompArgs copy = a;
  void* args[] = {&copy};
  return hipModuleLaunchKernel(f, grid, 1, 1, 64, 1, 1, 0, stream, args, nullptr) == hipSuccess;
}

bool jit_launch_expand_fast(const JitKernels& k, const ExpandArgs& a, unsigned grid, int probe, hipStream_t stream) {
  hipFunction_t f = k.expand_fast[probe ? 1 : 0];
  if (!f) return false;
  if (!grid) return true;
  ExpandArgs copy = a;
  void* args[] = {&copy};
  return hipModuleLaunchKernel(f, grid, 1, 1, BLOCK, 1, 1, 0, stream, args, nullptr) == hipSuccess;
}

bool jit_launch_tree_wave(const JitKernels& k, const TreeArgs& a, hipStream_t stream) {
  if (!a.n_comp) return true;
  if (!k.treew) return false;
  TreeArgs copy = a;
  void* args[] = {&copy};
  // one wave per TLCG_TREE_WAVE_M batches of 64 components (the kernel strides over the rest)
  return hipModuleLaunchKernel(k.treew, tree_grid((a.n_comp + 63) / 64, TREE_WAVE_M), 1, 1, 64, 1, 1, 0, stream, args,
                               nullptr) == hipSuccess;
}

bool jit_launch_tree_bits(const JitKernels& k, const TreeArgs& a, hipStream_t stream) {
  if (!a.n_comp) return true;
  if (!k.treeb || !a.owner) return false;
  TreeArgs copy = a;
  void* args[] = {&copy};
  return hipModuleLaunchKernel(k.treeb, tree_grid(a.n_comp, TREECB_G), 1, 1, 64, 1, 1, 0, stream, args, nullptr) ==
         hipSuccess;
}

bool jit_launch_tree(const JitKernels& k, const TreeArgs& a, int cap, hipStream_t stream) {
  if (!a.n_comp) return true;
  hipFunction_t f = cap == 384 ? k.tree[0] : cap == 1024 ? k.tree[1] : cap == 640 ? k.tree[2] : k.tree[3];
  if (!f) return false;
  TreeArgs copy = a;
  void* args[] = {&copy};
  const int groups = cap == 384 || cap == 640 ? 4 : 1;
  return hipModuleLaunchKernel(f, tree_grid(a.n_comp, groups), 1, 1, 64, 1, 1, 0, stream, args, nullptr) == hipSuccess;
}

}  // namespace tlcg
