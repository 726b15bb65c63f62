// Host -> device staging rates on the box (what kh_trie_root's host-input path can reach):
//   (a) hipMemcpyAsync from pageable memory (the round-5 path),
//   (b) from pinned memory (hipHostMalloc), one copy of 256 MB,
//   (c) memcpy pageable -> pinned with T host threads (aggregate GB/s),
//   (d) the pipeline: T threads fill a ring of R pinned chunks, one stream DMAs them,
//   (e) hipHostRegister of the pageable buffer, a DMA from it, hipHostUnregister.
// Measurement only.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o h2d_probe h2d_probe.hip -lpthread
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void par_copy(uint8_t* dst, const uint8_t* src, size_t bytes, int T) {
  std::vector<std::thread> th;
  const size_t per = (bytes / T + 4095) & ~(size_t)4095;
  for (int t = 0; t < T; ++t) {
    const size_t a = per * t;
    if (a >= bytes) break;
    const size_t b = a + per < bytes ? a + per : bytes;
    th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const size_t GB = 1ull << 30;
  const size_t total = (argc > 1 ? atoll(argv[1]) : 4) * GB;
  uint8_t* src = (uint8_t*)aligned_alloc(4096, total);
  for (size_t i = 0; i < total; i += 8) *(uint64_t*)(src + i) = i * 0x9E3779B97F4A7C15ull;
  uint8_t* dev;
  CHK(hipMalloc(&dev, total));
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // (a) pageable
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    CHK(hipMemcpyAsync(dev, src, total, hipMemcpyHostToDevice, st));
    CHK(hipStreamSynchronize(st));
    double t = now() - t0;
    printf("{\"probe\":\"pageable\",\"bytes\":%zu,\"ms\":%.2f,\"gbps\":%.2f}\n", total, t * 1e3, total / t / 1e9);
  }
  // (b) pinned
  const size_t pb = 256ull << 20;
  uint8_t* pin;
  CHK(hipHostMalloc((void**)&pin, 8 * pb, hipHostMallocDefault));
  memset(pin, 1, 8 * pb);
  for (int rep = 0; rep < 3; ++rep) {
    double t0 = now();
    CHK(hipMemcpyAsync(dev, pin, 8 * pb, hipMemcpyHostToDevice, st));
    CHK(hipStreamSynchronize(st));
    double t = now() - t0;
    printf("{\"probe\":\"pinned\",\"bytes\":%zu,\"ms\":%.2f,\"gbps\":%.2f}\n", 8 * pb, t * 1e3, 8 * pb / t / 1e9);
  }
  // (c) host memcpy into pinned
  for (int T : {1, 2, 4, 8, 12, 16}) {
    double best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      double t0 = now();
      par_copy(pin, src + (rep * 8 * pb) % (total - 8 * pb + 1), 8 * pb, T);
      best = std::min(best, now() - t0);
    }
    printf("{\"probe\":\"memcpy_to_pinned\",\"threads\":%d,\"bytes\":%zu,\"ms\":%.2f,\"gbps\":%.2f}\n", T, 8 * pb,
           best * 1e3, 8 * pb / best / 1e9);
  }
  // (d) pipeline: ring of R chunks of C bytes, T copy threads per chunk
  for (size_t C : {32ull << 20, 64ull << 20, 128ull << 20}) {
    for (int T : {4, 8, 16}) {
      const int R = (int)(8 * pb / C);
      std::vector<hipEvent_t> ev(R);
      for (auto& x : ev) CHK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
      std::vector<bool> used(R, false);
      double t0 = now();
      size_t off = 0;
      int k = 0;
      while (off < total) {
        const size_t b = total - off < C ? total - off : C;
        const int s = k % R;
        if (used[s]) CHK(hipEventSynchronize(ev[s]));
        par_copy(pin + s * C, src + off, b, T);
        CHK(hipMemcpyAsync(dev + off, pin + s * C, b, hipMemcpyHostToDevice, st));
        CHK(hipEventRecord(ev[s], st));
        used[s] = true;
        off += b;
        ++k;
      }
      CHK(hipStreamSynchronize(st));
      double t = now() - t0;
      printf("{\"probe\":\"pipeline\",\"chunk_mb\":%zu,\"ring\":%d,\"threads\":%d,\"bytes\":%zu,\"ms\":%.2f,\"gbps\":%.2f}\n",
             C >> 20, R, T, total, t * 1e3, total / t / 1e9);
      for (auto& x : ev) CHK(hipEventDestroy(x));
    }
  }
  // (e) register in place
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    CHK(hipHostRegister(src, total, hipHostRegisterDefault));
    double t1 = now();
    void* dp = nullptr;
    CHK(hipHostGetDevicePointer(&dp, src, 0));
    CHK(hipMemcpyAsync(dev, src, total, hipMemcpyHostToDevice, st));
    CHK(hipStreamSynchronize(st));
    double t2 = now();
    CHK(hipHostUnregister(src));
    double t3 = now();
    printf("{\"probe\":\"register\",\"bytes\":%zu,\"register_ms\":%.2f,\"dma_ms\":%.2f,\"unregister_ms\":%.2f,"
           "\"dma_gbps\":%.2f,\"all_gbps\":%.2f}\n",
           total, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, total / (t2 - t1) / 1e9, total / (t3 - t0) / 1e9);
  }
  // (e2) register in chunks, pipelined (register chunk i+1 while chunk i DMAs)
  for (size_t C : {256ull << 20, 1ull << 30}) {
    double t0 = now();
    std::vector<std::pair<uint8_t*, size_t>> regs;
    for (size_t off = 0; off < total; off += C) {
      const size_t b = total - off < C ? total - off : C;
      CHK(hipHostRegister(src + off, b, hipHostRegisterDefault));
      CHK(hipMemcpyAsync(dev + off, src + off, b, hipMemcpyHostToDevice, st));
      regs.push_back({src + off, b});
    }
    CHK(hipStreamSynchronize(st));
    double t1 = now();
    for (auto& r : regs) CHK(hipHostUnregister(r.first));
    double t2 = now();
    printf("{\"probe\":\"register_chunks\",\"chunk_mb\":%zu,\"ms\":%.2f,\"unregister_ms\":%.2f,\"gbps\":%.2f}\n", C >> 20,
           (t1 - t0) * 1e3, (t2 - t1) * 1e3, total / (t2 - t0) / 1e9);
  }
  printf("{\"probe\":\"hw\",\"threads_hw\":%u}\n", std::thread::hardware_concurrency());
  return 0;
}
