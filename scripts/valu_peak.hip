// Measured VALU issue rate per instruction kind on the device (the Keccak
// roofline's peak, and which encodings are full rate).  Each lane runs 8
// independent chains of one instruction (inline asm, so the exact encoding is
// issued); the grid puts 8 waves on every SIMD.  Prints lane-ops/s per kind.
// Build: hipcc --offload-arch=gfx950 -O3 valu_peak.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int ITERS = 2048;
constexpr int CH = 8;

template <int K>
__device__ __forceinline__ void op(uint32_t& a, uint32_t b, uint32_t c) {
  if constexpr (K == 0) asm("v_xor_b32_e32 %0, %1, %0" : "+v"(a) : "v"(b));
  if constexpr (K == 1) asm("v_xor_b32_e64 %0, %1, %0" : "+v"(a) : "v"(b));
  if constexpr (K == 2) asm("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (K == 3) asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (K == 4) asm("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a) : "v"(b));
  if constexpr (K == 5) asm("v_bfi_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (K == 6) asm("v_and_b32_e32 %0, %1, %0" : "+v"(a) : "v"(b));
  if constexpr (K == 7) asm("v_not_b32_e32 %0, %0" : "+v"(a));
  if constexpr (K == 8) asm("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a) : "v"(b));
  if constexpr (K == 9) asm("v_alignbit_b32 %0, %0, %0, %1" : "+v"(a) : "v"(b));
  if constexpr (K == 10) asm("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (K == 11) asm("v_lshlrev_b32_e32 %0, 7, %0" : "+v"(a));
  if constexpr (K == 13) asm("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(a) : "v"(b));
}
// 64-bit kinds (Keccak lanes as whole 64-bit registers: rotations as two 64-bit shifts
// merged by v_lshl_add_u64, whose two parts never overlap)
template <int K>
__device__ __forceinline__ void op64(uint64_t& a, uint64_t b) {
  if constexpr (K == 20) asm("v_lshlrev_b64 %0, 7, %0" : "+v"(a));
  if constexpr (K == 21) asm("v_lshrrev_b64 %0, 7, %0" : "+v"(a));
  if constexpr (K == 22) asm("v_lshl_add_u64 %0, %0, 7, %1" : "+v"(a) : "v"(b));
  if constexpr (K == 24) asm("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(a) : "v"(b));
}

template <int K>
__global__ void __launch_bounds__(256) k_peak(uint32_t* out, uint32_t seed) {
  uint32_t a[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) a[j] = seed * (threadIdx.x + 1) + j * 0x9e3779b9u;
  uint32_t b = seed ^ (threadIdx.x * 7), c = seed + blockIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < CH; ++j) op<K>(a[j], b, c);
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < CH; ++j) x ^= a[j];
  if (x == 0x12345678u) out[blockIdx.x] = x;
}

template <int K>
__global__ void __launch_bounds__(256) k_peak64(uint32_t* out, uint32_t seed) {
  uint64_t a[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) a[j] = (uint64_t)(seed * (threadIdx.x + 1)) * 0x9e3779b97f4a7c15ull + j;
  const uint64_t b = ((uint64_t)seed << 32) ^ (threadIdx.x * 7);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < CH; ++j) op64<K>(a[j], b);
  }
  uint64_t x = 0;
#pragma unroll
  for (int j = 0; j < CH; ++j) x ^= a[j];
  if ((uint32_t)x == 0x12345678u) out[blockIdx.x] = (uint32_t)(x >> 32);
}

template <int K>
static void launch(int blocks, uint32_t* out, uint32_t seed) {
  if constexpr (K < 20)
    k_peak<K><<<blocks, 256>>>(out, seed);
  else
    k_peak64<K><<<blocks, 256>>>(out, seed);
}

template <int K>
static int run(const char* name) {
  int dev = 0, ncu = 0, clk = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CHK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
  const int blocks = ncu * 8;  // 8 x 256 threads = 32 waves per CU = 8 per SIMD
  uint32_t* out;
  CHK(hipMalloc(&out, blocks * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  launch<K>(blocks, out, 1);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) launch<K>(blocks, out, 2 + r);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  double wave_instr = 5.0 * blocks * 4.0 * ITERS * 4.0 * CH;  // 4 waves per block
  double simd_cycles = ms * 1e-3 * (clk * 1e3) * ncu * 4;       // at the reported clock
  printf("%-16s %8.3f ms  %7.2f T lane-ops/s  %5.2f cycles/wave-instr/SIMD (clock %d MHz, %d CUs)\n", name, ms,
         wave_instr * 64 / (ms * 1e-3) / 1e12, simd_cycles / wave_instr, clk / 1000, ncu);
  CHK(hipFree(out));
  return 0;
}

int main() {
  if (run<0>("v_xor_b32_e32")) return 1;
  if (run<1>("v_xor_b32_e64")) return 1;
  if (run<2>("v_add3_u32")) return 1;
  if (run<3>("v_bitop3_b32")) return 1;
  if (run<4>("v_alignbit_b32")) return 1;
  if (run<9>("v_alignbit(rot)")) return 1;
  if (run<5>("v_bfi_b32")) return 1;
  if (run<6>("v_and_b32_e32")) return 1;
  if (run<7>("v_not_b32_e32")) return 1;
  if (run<8>("v_lshl_or_b32")) return 1;
  if (run<10>("v_perm_b32")) return 1;
  if (run<11>("v_lshlrev_b32")) return 1;
  if (run<13>("v_alignbyte_b32")) return 1;
  // 64-bit kinds: lane-ops counted as one per lane (a 64-bit op does two 32-bit lanes' work)
  if (run<20>("v_lshlrev_b64")) return 1;
  if (run<21>("v_lshrrev_b64")) return 1;
  if (run<22>("v_lshl_add_u64")) return 1;
  if (run<24>("v_pk_mov_b32")) return 1;
  return 0;
}
