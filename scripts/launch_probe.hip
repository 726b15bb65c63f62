// Host cost of one kernel launch (the block commit issues ~64 per phase per thread): N launches
// of a one-wave kernel back to back on one stream, host time per hipLaunchKernel call, for
//   small : 16 bytes of kernel arguments
//   topo  : a 640-byte struct by value (khst's Topo is passed this way)
//   ptr   : the same struct read through a device pointer (8 bytes of arguments)
// and the same three from two host threads launching on two streams at once (the block
// commit's storage and account phases).  Prints one JSON line.  Measurement only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -pthread -o /tmp/launch_probe scripts/launch_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

struct Big {
  unsigned long long w[80];
};

__global__ void k_small(unsigned long long* d, unsigned long long v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) d[0] += v;
}
__global__ void k_topo(Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0) ((unsigned long long*)b.w[0])[0] += b.w[79];
}
__global__ void k_ptr(const Big* b) {
  if (threadIdx.x == 0 && blockIdx.x == 0) ((unsigned long long*)b->w[0])[0] += b->w[79];
}

static double run(int mode, hipStream_t st, unsigned long long* d, const Big& hb, const Big* db, int n) {
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    if (mode == 0) hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st, d, 1ull);
    if (mode == 1) hipLaunchKernelGGL(k_topo, dim3(1), dim3(64), 0, st, hb);
    if (mode == 2) hipLaunchKernelGGL(k_ptr, dim3(1), dim3(64), 0, st, db);
  }
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(st);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t s[2];
  CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
  unsigned long long* d;
  CK(hipMalloc(&d, 256));
  CK(hipMemset(d, 0, 256));
  Big hb{};
  hb.w[0] = (unsigned long long)d;
  hb.w[79] = 1;
  Big* db;
  CK(hipMalloc(&db, sizeof(Big)));
  CK(hipMemcpy(db, &hb, sizeof(Big), hipMemcpyHostToDevice));
  const int N = 64;  // a phase's worth, queue never deep: synced between batches
  double one[3] = {1e9, 1e9, 1e9}, two[3] = {1e9, 1e9, 1e9};
  for (int rep = 0; rep < 30; ++rep)
    for (int m = 0; m < 3; ++m) {
      const double u = run(m, s[0], d, hb, db, N);
      one[m] = u < one[m] ? u : one[m];
      double ua = 0, ub = 0;
      std::thread t([&] { ub = run(m, s[1], d + 8, hb, db, N); });
      ua = run(m, s[0], d, hb, db, N);
      t.join();
      const double w = ua > ub ? ua : ub;
      two[m] = w < two[m] ? w : two[m];
    }
  printf("{\"us_per_launch_one_thread\": {\"small\": %.2f, \"topo\": %.2f, \"ptr\": %.2f}, "
         "\"us_per_launch_two_threads\": {\"small\": %.2f, \"topo\": %.2f, \"ptr\": %.2f}, \"launches_per_batch\": %d}\n",
         one[0], one[1], one[2], two[0], two[1], two[2], N);
  return 0;
}
