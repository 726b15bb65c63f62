// Measured int32 VALU issue rate on the device, for the Keccak roofline.
// Each lane runs 8 independent chains of one instruction kind (xor, bitop3,
// alignbit, and the Keccak round mix); the grid fills every SIMD with 8 waves.
// Prints lane-ops/s per kind.  Build: hipcc --offload-arch=gfx950 -O3 valu_peak.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int ITERS = 4096;

template <int KIND>
__global__ void __launch_bounds__(256) k_peak(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = seed * (threadIdx.x + 1) + j * 0x9e3779b9u;
  uint32_t b = seed ^ threadIdx.x, c = seed + blockIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (KIND == 0) a[j] = a[j] ^ b;
      if (KIND == 1) a[j] = __builtin_amdgcn_bitop3_b32(a[j], b, c, 0x96);
      if (KIND == 2) a[j] = __builtin_amdgcn_alignbit(a[j], b, 7);
      if (KIND == 3) a[j] = __builtin_amdgcn_alignbit(__builtin_amdgcn_bitop3_b32(a[j], b, c, 0x96) ^ c, a[j], 5);
    }
    b += 1;  // scalar-uniform? no: b is per-lane, keeps the chains live
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= a[j];
  if (r == 0x12345678u) out[blockIdx.x] = r;
}

template <int KIND>
static int run(const char* name, int ops_per_elem) {
  int dev = 0, ncu = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = ncu * 8;  // 8 x 256 threads = 32 waves per CU
  uint32_t* out;
  CHK(hipMalloc(&out, blocks * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  k_peak<KIND><<<blocks, 256>>>(out, 1);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) k_peak<KIND><<<blocks, 256>>>(out, 2 + r);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  double lane_ops = 5.0 * blocks * 256.0 * ITERS * (8.0 * ops_per_elem + 1.0);  // +1: the b update
  printf("%-10s %8.3f ms  %7.2f T lane-ops/s  (%d CUs)\n", name, ms, lane_ops / (ms * 1e-3) / 1e12, ncu);
  CHK(hipFree(out));
  return 0;
}

int main() {
  if (run<0>("v_xor", 1)) return 1;
  if (run<1>("v_bitop3", 1)) return 1;
  if (run<2>("v_alignbit", 1)) return 1;
  if (run<3>("mix3", 3)) return 1;
  return 0;
}
