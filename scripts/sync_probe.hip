// Host round-trip latency of one sync point, three ways (the block commit has ~7 of them
// per phase): a small kernel, then
//   (a) hipMemcpyAsync D2H of 64 B into pinned memory + hipStreamSynchronize,
//   (b) the same under hipDeviceScheduleSpin (set before the context exists: a 2nd run),
//   (c) a one-block post kernel copying the words into fine-grained (coherent) pinned
//       memory and writing a sequence token last; the host spins on the token.
// Each loop iteration depends on the value read back (the next kernel's argument), as a
// commit's next launch sizes depend on the counters.
// Build: hipcc --offload-arch=gfx950 -O3 -o sync_probe sync_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void k_work(unsigned long long* ctr, unsigned long long v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) ctr[0] = v + 1;
}
__global__ void k_post(const unsigned long long* src, uint32_t nw, unsigned long long* dst,
                       unsigned long long* flag, unsigned long long tok) {
  for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
  __threadfence_system();
  if (threadIdx.x == 0) *(volatile unsigned long long*)flag = tok;
}

int main(int argc, char** argv) {
  const bool spin = argc > 1 && !strcmp(argv[1], "spin");
  if (spin) CHK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned long long* d;
  CHK(hipMalloc(&d, 4096));
  CHK(hipMemset(d, 0, 4096));
  unsigned long long *hp, *hc;
  CHK(hipHostMalloc((void**)&hp, 4096, hipHostMallocDefault));
  CHK(hipHostMalloc((void**)&hc, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  memset(hc, 0, 4096);
  unsigned long long* hc_dev;
  CHK(hipHostGetDevicePointer((void**)&hc_dev, hc, 0));
  const int N = 2000;
  for (int mode = 0; mode < 2; ++mode) {
    unsigned long long v = 0, tok = 0;
    double best = 1e9, sum = 0;
    for (int rep = 0; rep < 3; ++rep) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_work, dim3(1), dim3(64), 0, st, d, v);
        if (mode == 0) {
          CHK(hipMemcpyAsync(hp, d, 64, hipMemcpyDeviceToHost, st));
          CHK(hipStreamSynchronize(st));
          v = hp[0];
        } else {
          ++tok;
          hipLaunchKernelGGL(k_post, dim3(1), dim3(256), 0, st, (const unsigned long long*)d, 8u, hc_dev + 8,
                             hc_dev, tok);
          uint64_t spins = 0;
          while (__atomic_load_n(&hc[0], __ATOMIC_ACQUIRE) != tok) {
            if ((++spins & 0xFFFFF) == 0) {
              hipError_t e = hipStreamQuery(st);
              if (e != hipSuccess && e != hipErrorNotReady) {
                fprintf(stderr, "stream error %s\n", hipGetErrorString(e));
                return 1;
              }
              if (e == hipSuccess && __atomic_load_n(&hc[0], __ATOMIC_ACQUIRE) != tok) {
                fprintf(stderr, "stream done, token not visible\n");
                return 1;
              }
            }
          }
          v = __atomic_load_n(&hc[8], __ATOMIC_ACQUIRE);
        }
      }
      CHK(hipStreamSynchronize(st));
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
      best = us < best ? us : best;
      sum += us;
    }
    if (v != (unsigned long long)3 * N) {
      fprintf(stderr, "mode %d: chain value %llu != %d\n", mode, v, 3 * N);
      return 1;
    }
    printf("{\"sched\": \"%s\", \"mode\": \"%s\", \"us_per_sync_point_best\": %.2f, \"us_mean\": %.2f}\n",
           spin ? "spin" : "auto", mode == 0 ? "memcpy+streamsync" : "post kernel + host spin on token", best,
           sum / 3);
  }
  return 0;
}
