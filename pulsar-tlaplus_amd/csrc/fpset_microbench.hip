// pulsar-tlaplus_amd/csrc/fpset_microbench.hip -- measured ceilings for the
// FPSet roofline: scattered 8-byte accesses over a table the size of the G9
// FPSet (2^31 slots = 16 GiB), one independent random slot per lane.
//   load      plain 8-B load                  (a probe that finds its slot)
//   load_nt   nontemporal 8-B load
//   store     plain 8-B store                 (an uncontended insert)
//   cas_new   atomicCAS(0 -> key) that wins   (an insert)
//   cas_old   atomicCAS on an occupied slot   (a probe that finds a duplicate)
//   add       no-return 64-bit atomicAdd
// Prints one JSON line per access kind: accesses/s and GB/s of touched 8-B words.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ u64 mix(u64 x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// the XCD (0..7) this wave runs on
__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

// KIND 6..8: the table split into 8 partitions, each block touching only the
// partition of the XCD it runs on (slots stay in that XCD's L2):
//   6 cas_wg_xcd     workgroup-scope CAS (performed in the XCD's L2)
//   7 cas_agent_xcd  device-scope CAS (performed at the memory side)
//   8 load_xcd       plain load
// KIND 9..12: the same n slots in ascending order (slot of access i in
// [i x T/n, (i + 1) x T/n), consecutive lanes on consecutive gaps): what a
// level's probes cost once its candidates are sorted by slot
//   9 load_nt_sorted, 10 store_sorted, 11 cas_sorted (device scope),
//   12 cas_wg_sorted (workgroup scope)
template <int KIND>
__global__ __launch_bounds__(256) void k_access(u64* __restrict__ t, int log2, u64 n, u64 seed, u64* sink) {
  const int sh = 64 - log2;
  u64 acc = 0;
  const u64 part = (u64)xcc_id() << (log2 - 3);
  for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
    const u64 h = mix(i ^ seed);
    const u64 gap = (1ull << log2) / n;
    const u64 s = KIND >= 9 ? i * gap + (gap > 1 ? h % gap : 0) : KIND >= 6 ? part | (h >> (sh + 3)) : h >> sh;
    if (KIND == 0) acc += t[s];
    else if (KIND == 1) acc += __builtin_nontemporal_load(&t[s]);
    else if (KIND == 2) t[s] = h | 1;
    else if (KIND == 3 || KIND == 4 || KIND == 7) acc += atomicCAS(&t[s], 0ull, h | 1);
    else if (KIND == 6) {
      u64 e = 0;
      __hip_atomic_compare_exchange_strong(&t[s], &e, h | 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += e;
    } else if (KIND == 8) acc += t[s];
    else if (KIND == 9) acc += __builtin_nontemporal_load(&t[s]);
    else if (KIND == 10) t[s] = h | 1;
    else if (KIND == 11) acc += atomicCAS(&t[s], 0ull, h | 1);
    else if (KIND == 12) {
      u64 e = 0;
      __hip_atomic_compare_exchange_strong(&t[s], &e, h | 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += e;
    }
    else atomicAdd(&t[s], 1ull);
  }
  if (acc == 0x123456789ull) *sink = acc;
}

int main(int argc, char** argv) {
  int log2 = argc > 1 ? std::atoi(argv[1]) : 31;
  u64 n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (1ull << 30);
  const int first_kind = argc > 3 ? std::atoi(argv[3]) : 0;
  const int last_kind = argc > 4 ? std::atoi(argv[4]) : 12;
  u64* t;
  u64* sink;
  CHK(hipMalloc(&t, 8ull << log2));
  CHK(hipMalloc(&sink, 8));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const char* names[] = {"load", "load_nt", "store", "cas_new", "cas_old", "add", "cas_wg_xcd", "cas_agent_xcd",
                         "load_xcd", "load_nt_sorted", "store_sorted", "cas_sorted", "cas_wg_sorted"};
  for (int grid : {4096, 16384}) {
    for (int kind = first_kind; kind <= last_kind; ++kind) {
      // cas_new wants empty slots at the probed positions, the others do not care
      CHK(hipMemset(t, 0, 8ull << log2));
      if (kind == 4) {  // pre-fill the slots cas_old will hit
        k_access<2><<<grid, 256>>>(t, log2, n, 7, sink);
      }
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(a));
      switch (kind) {
        case 0: k_access<0><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 1: k_access<1><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 2: k_access<2><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 3: k_access<3><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 4: k_access<4><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 5: k_access<5><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 6: k_access<6><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 7: k_access<7><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 8: k_access<8><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 9: k_access<9><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 10: k_access<10><<<grid, 256>>>(t, log2, n, 7, sink); break;
        case 11: k_access<11><<<grid, 256>>>(t, log2, n, 7, sink); break;
        default: k_access<12><<<grid, 256>>>(t, log2, n, 7, sink); break;
      }
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, a, b));
      double rate = (double)n / (ms * 1e-3);
      std::printf("{\"kind\": \"%s\", \"grid\": %d, \"table_gib\": %.1f, \"accesses\": %llu, \"ms\": %.3f, "
                  "\"access_per_s\": %.4g, \"word_GBps\": %.1f, \"line64_GBps\": %.1f}\n",
                  names[kind], grid, (8ull << log2) / 1073741824.0, n, ms, rate, rate * 8 / 1e9,
                  rate * 64 / 1e9);
      std::fflush(stdout);
    }
  }
  CHK(hipFree(t));
  return 0;
}
