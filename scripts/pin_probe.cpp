// Host-memory spill probe: how fast can a device->host spill of G GiB go with
// (1) hipHostMalloc, (2) pageable malloc + hipMemcpy, (3) pageable with
// transparent huge pages, (4) hipHostMalloc split over T threads.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const size_t gib = argc > 1 ? std::atoi(argv[1]) : 4;
  const size_t bytes = gib << 30;
  void* dev = nullptr;
  CK(hipMalloc(&dev, bytes));
  CK(hipMemset(dev, 1, bytes));
  CK(hipDeviceSynchronize());
  {  // 1
    void* h = nullptr;
    double t0 = now_ms();
    CK(hipHostMalloc(&h, bytes));
    double t1 = now_ms();
    CK(hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost));
    double t2 = now_ms();
    CK(hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost));
    double t3 = now_ms();
    CK(hipHostFree(h));
    double t4 = now_ms();
    std::printf("{\"mode\":\"hipHostMalloc\",\"GiB\":%zu,\"alloc_ms\":%.1f,\"copy_ms\":%.1f,\"copy2_ms\":%.1f,\"free_ms\":%.1f}\n",
                gib, t1 - t0, t2 - t1, t3 - t2, t4 - t3);
  }
  for (int huge = 0; huge < 2; ++huge) {  // 2, 3
    double t0 = now_ms();
    void* h = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (huge) madvise(h, bytes, MADV_HUGEPAGE);
    double t1 = now_ms();
    CK(hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost));
    double t2 = now_ms();
    CK(hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost));
    double t3 = now_ms();
    munmap(h, bytes);
    double t4 = now_ms();
    std::printf("{\"mode\":\"pageable%s\",\"GiB\":%zu,\"alloc_ms\":%.1f,\"copy_ms\":%.1f,\"copy2_ms\":%.1f,\"free_ms\":%.1f}\n",
                huge ? "_thp" : "", gib, t1 - t0, t2 - t1, t3 - t2, t4 - t3);
  }
  for (int T : {4, 8, 16}) {  // 4
    std::vector<void*> hs(T, nullptr);
    std::vector<std::thread> th;
    double t0 = now_ms();
    for (int i = 0; i < T; ++i) th.emplace_back([&, i] { (void)hipHostMalloc(&hs[i], bytes / T); });
    for (auto& t : th) t.join();
    double t1 = now_ms();
    for (int i = 0; i < T; ++i) CK(hipMemcpyAsync(hs[i], (char*)dev + i * (bytes / T), bytes / T, hipMemcpyDeviceToHost, 0));
    CK(hipDeviceSynchronize());
    double t2 = now_ms();
    th.clear();
    for (int i = 0; i < T; ++i) th.emplace_back([&, i] { (void)hipHostFree(hs[i]); });
    for (auto& t : th) t.join();
    double t3 = now_ms();
    std::printf("{\"mode\":\"hipHostMalloc_x%d\",\"GiB\":%zu,\"alloc_ms\":%.1f,\"copy_ms\":%.1f,\"free_ms\":%.1f}\n", T, gib,
                t1 - t0, t2 - t1, t3 - t2);
  }
  {  // 5: thp pageable, pre-touched by threads, then hipHostRegister
    void* h = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(h, bytes, MADV_HUGEPAGE);
    double t0 = now_ms();
    std::vector<std::thread> th;
    for (int i = 0; i < 16; ++i)
      th.emplace_back([&, i] { std::memset((char*)h + i * (bytes / 16), 0, bytes / 16); });
    for (auto& t : th) t.join();
    double t1 = now_ms();
    CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
    double t2 = now_ms();
    CK(hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost));
    double t3 = now_ms();
    CK(hipHostUnregister(h));
    munmap(h, bytes);
    double t4 = now_ms();
    std::printf("{\"mode\":\"thp_touch16_register\",\"GiB\":%zu,\"touch_ms\":%.1f,\"register_ms\":%.1f,\"copy_ms\":%.1f,\"free_ms\":%.1f}\n",
                gib, t1 - t0, t2 - t1, t3 - t2, t4 - t3);
  }
  return 0;
}
