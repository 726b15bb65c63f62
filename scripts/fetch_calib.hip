// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access shapes of the state-root
// kernels (MI355X_MICROARCH.md HBM section: only wide 16-B/lane streaming reads are
// calibrated there).  Every kernel touches a KNOWN number of bytes of buffers far larger
// than the 256 MiB Infinity Cache; scripts/fetch_calib.py divides the counters by them.
//   rd16      16 B/lane coalesced reads (the guide's calibrated case: expect 1/2)
//   rd8       8 B/lane coalesced reads (voff / pdinv in k_leaf_in)
//   rd8span   each lane walks its own 80-byte span with 8-byte loads, lanes' spans
//             adjacent (the value reads of k_leaf_in)
//   rd32rand  32-byte random gathers (k_gather's key gather, the stash gather)
//   rd8rand   8-byte random gathers (value-span starts in sorted order)
//   wr16      16 B/lane coalesced writes (calibrated in the guide: expect 1)
//   wr8rand   8-byte random scatters (k_pd_scatter)
//   wr32rand  32-byte random scatters (k_leaf_in's stash)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/fetch_calib scripts/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

constexpr uint64_t NB = 2ull << 30;  // 2 GiB per buffer (8x the Infinity Cache)
constexpr int BS = 256;

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__global__ void rd16(const uint4* a, uint64_t n, uint32_t* sink) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345679u) sink[0] = 1;
}
__global__ void rd8(const uint64_t* a, uint64_t n, uint32_t* sink) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  if (a[i] == 0x123456789ull) sink[0] = 1;
}
__global__ void rd8span(const uint64_t* a, uint64_t n, uint32_t* sink) {  // n spans of 10 words
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint64_t x = 0;
#pragma unroll
  for (int q = 0; q < 10; ++q) x ^= a[10 * i + q];
  if (x == 0x123456789ull) sink[0] = 1;
}
__global__ void rd32rand(const uint4* a, uint64_t n, uint64_t nslots, uint32_t* sink) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint64_t s = mix(i) % nslots;  // 32-byte slot
  uint4 v = a[2 * s], w = a[2 * s + 1];
  if ((v.x ^ w.y) == 0x12345679u) sink[0] = 1;
}
__global__ void rd8rand(const uint64_t* a, uint64_t n, uint64_t nslots, uint32_t* sink) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  if (a[mix(i) % nslots] == 0x123456789ull) sink[0] = 1;
}
__global__ void wr16(uint4* a, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  a[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void wr8rand(uint64_t* a, uint64_t n, uint64_t nslots) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  a[mix(i) % nslots] = i;
}
__global__ void wr32rand(uint4* a, uint64_t n, uint64_t nslots) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint64_t s = mix(i) % nslots;
  a[2 * s] = make_uint4((uint32_t)i, 1, 2, 3);
  a[2 * s + 1] = make_uint4(4, 5, 6, 7);
}

static unsigned grid(uint64_t n) { return (unsigned)((n + BS - 1) / BS); }

int main() {
  char *a, *b;
  uint32_t* sink;
  CK(hipMalloc(&a, NB));
  CK(hipMalloc(&b, NB));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 1, NB));
  CK(hipMemset(b, 2, NB));
  CK(hipDeviceSynchronize());
  const uint64_t n16 = NB / 16, n8 = NB / 8, nspan = NB / 80, nrand = 50'000'000ull;
  // known algorithmic bytes per launch (printed for scripts/fetch_calib.py)
  printf("rd16 %llu\n", (unsigned long long)(n16 * 16));
  printf("rd8 %llu\n", (unsigned long long)(n8 * 8));
  printf("rd8span %llu\n", (unsigned long long)(nspan * 80));
  printf("rd32rand %llu\n", (unsigned long long)(nrand * 32));
  printf("rd8rand %llu\n", (unsigned long long)(nrand * 8));
  printf("wr16 %llu\n", (unsigned long long)(n16 * 16));
  printf("wr8rand %llu\n", (unsigned long long)(nrand * 8));
  printf("wr32rand %llu\n", (unsigned long long)(nrand * 32));
  hipLaunchKernelGGL(rd16, dim3(grid(n16)), dim3(BS), 0, 0, (const uint4*)a, n16, sink);
  hipLaunchKernelGGL(rd8, dim3(grid(n8)), dim3(BS), 0, 0, (const uint64_t*)b, n8, sink);
  hipLaunchKernelGGL(rd8span, dim3(grid(nspan)), dim3(BS), 0, 0, (const uint64_t*)a, nspan, sink);
  hipLaunchKernelGGL(rd32rand, dim3(grid(nrand)), dim3(BS), 0, 0, (const uint4*)b, nrand, NB / 32, sink);
  hipLaunchKernelGGL(rd8rand, dim3(grid(nrand)), dim3(BS), 0, 0, (const uint64_t*)a, nrand, NB / 8, sink);
  hipLaunchKernelGGL(wr16, dim3(grid(n16)), dim3(BS), 0, 0, (uint4*)b, n16);
  hipLaunchKernelGGL(wr8rand, dim3(grid(nrand)), dim3(BS), 0, 0, (uint64_t*)a, nrand, NB / 8);
  hipLaunchKernelGGL(wr32rand, dim3(grid(nrand)), dim3(BS), 0, 0, (uint4*)b, nrand, NB / 32);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
