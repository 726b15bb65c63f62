// Check and time the lane-spread Keccak-f[1600] (khipu_amd/csrc/keccak_xlane.h) against the
// one-thread-per-state permutation (keccak.h).  Measurement / test infrastructure only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/xlane_check scripts/xlane_check.hip
//   scripts/xlane_check            -> one JSON line: equal states, latency per permutation
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../khipu_amd/csrc/keccak_xlane.h"

using namespace khst;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

// one state per thread, P permutations in a row
__global__ void __launch_bounds__(64) k_thread(const uint64_t* in, uint64_t* out, int P) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  KState S;
  for (int i = 0; i < 25; ++i) {
    const uint64_t w = in[25 * t + i];
    S.lo[i] = (uint32_t)w;
    S.hi[i] = (uint32_t)(w >> 32);
  }
  for (int p = 0; p < P; ++p) keccakf(S);
  for (int i = 0; i < 25; ++i) out[25 * t + i] = lane(S, i);
}
// one state per 32-lane group
__global__ void __launch_bounds__(64) k_xlane(const uint64_t* in, uint64_t* out, int P) {
  __shared__ uint64_t kb[2][64];
  const uint32_t g = threadIdx.x >> 5, sub = threadIdx.x & 31;
  const uint32_t t = blockIdx.x * 2 + g;
  const XLane X = xlane_setup(sub);
  uint64_t w = sub < 25 ? in[25 * t + sub] : 0;
  uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
  for (int p = 0; p < P; ++p) keccakf_xlane(lo, hi, kb[g], X);
  if (sub < 25) out[25 * t + sub] = ((uint64_t)hi << 32) | lo;
}

int main() {
  const int NS = 512;  // states
  uint64_t* h_in = (uint64_t*)malloc(NS * 25 * 8);
  uint64_t* h_a = (uint64_t*)malloc(NS * 25 * 8);
  uint64_t* h_b = (uint64_t*)malloc(NS * 25 * 8);
  uint64_t x = 0x9E3779B97F4A7C15ULL;
  for (int i = 0; i < NS * 25; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h_in[i] = x;
  }
  uint64_t *d_in, *d_a, *d_b;
  CK(hipMalloc(&d_in, NS * 25 * 8));
  CK(hipMalloc(&d_a, NS * 25 * 8));
  CK(hipMalloc(&d_b, NS * 25 * 8));
  CK(hipMemcpy(d_in, h_in, NS * 25 * 8, hipMemcpyHostToDevice));
  int bad = 0;
  for (int P : {1, 3}) {
    hipLaunchKernelGGL(k_thread, dim3(NS / 64), dim3(64), 0, 0, d_in, d_a, P);
    hipLaunchKernelGGL(k_xlane, dim3(NS / 2), dim3(64), 0, 0, d_in, d_b, P);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_a, d_a, NS * 25 * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_b, d_b, NS * 25 * 8, hipMemcpyDeviceToHost));
    bad += memcmp(h_a, h_b, NS * 25 * 8) != 0;
  }
  // latency: one wave alone (one block), and one wave per CU (256 blocks); P = 64 in a row
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](bool xl, int blocks, int P) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0, 0));
      if (xl)
        hipLaunchKernelGGL(k_xlane, dim3(blocks), dim3(64), 0, 0, d_in, d_b, P);
      else
        hipLaunchKernelGGL(k_thread, dim3(blocks), dim3(64), 0, 0, d_in, d_a, P);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    return best;
  };
  const int P = 64;
  // (us per permutation: the difference between P and 1 permutations, over P - 1)
  auto per = [&](bool xl, int blocks) { return (time(xl, blocks, P) - time(xl, blocks, 1)) * 1e3 / (P - 1); };
  printf("{\"equal\": %s, \"us_per_perm\": {\"thread_1wave\": %.3f, \"xlane_1wave\": %.3f, "
         "\"thread_512states_8waves\": %.3f, \"xlane_512states_256waves\": %.3f}}\n",
         bad ? "false" : "true", per(false, 1), per(true, 1), per(false, 8), per(true, 256));
  return bad ? 1 : 0;
}
