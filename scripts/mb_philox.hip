// Microbenchmark (probe, not product): issue cost of the integer multiplies Philox4x32-10
// is built from on gfx950, and of Philox variants, per SIMD.
//   hipcc -O3 --offload-arch=gfx950 scripts/mb_philox.hip -o build/mb_philox && build/mb_philox
// Each kernel runs a dependent chain per thread (no hoisting) over a full grid: 256 CUs x 4
// SIMDs x 8 waves. Reported: wave-instruction slots per op per SIMD = time * clock * SIMDs /
// (waves * ops per wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }

struct U4 { uint32_t x, y, z, w; };

// the library's form (psg_device.hpp philox10): 32x32 -> 64 products in C
__device__ __forceinline__ U4 philox_c(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

// products with one v_mad_u64_u32 each
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b) {
  uint64_t r;
  uint64_t cy;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cy) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ U4 philox_mad(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = mad64(0xD2511F53u, c0);
    const uint64_t p1 = mad64(0xCD9E8D57u, c2);
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

template <int V>
__global__ void __launch_bounds__(256) k_philox(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a = threadIdx.x + blockIdx.x * 256u, b = seed, c = 7, d = threadIdx.x;
  uint32_t e = a ^ 0x55u, f = seed + 1, g = 9, h = d + 3;
  for (int i = 0; i < iters; ++i) {
    if constexpr (V == 0) {
      U4 o = philox_c(a, b, c, d, seed, 17);
      a ^= o.x; b ^= o.y; c ^= o.z; d ^= o.w;
    } else if constexpr (V == 1) {
      U4 o = philox_mad(a, b, c, d, seed, 17);
      a ^= o.x; b ^= o.y; c ^= o.z; d ^= o.w;
    } else {  // two independent chains per thread (ILP 2), the library form
      U4 o = philox_c(a, b, c, d, seed, 17);
      U4 q = philox_c(e, f, g, h, seed, 17);
      a ^= o.x; b ^= o.y; c ^= o.z; d ^= o.w;
      e ^= q.x; f ^= q.y; g ^= q.z; h ^= q.w;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

// op throughput: 8 independent accumulators, OPS ops per iteration
template <int OP>
__global__ void __launch_bounds__(256) k_op(uint32_t* out, int iters, uint32_t m) {
  uint32_t x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 8 + j + blockIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
      if constexpr (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
      if constexpr (OP == 2) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[j]) : "v"(m));
      if constexpr (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
      if constexpr (OP == 4) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(x[j]) : "v"(m));
      if constexpr (OP == 5) {
        uint64_t r;
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cy) : "v"(x[j]), "v"(m));
        x[j] = (uint32_t)r ^ (uint32_t)(r >> 32);
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= x[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
static int timeit(const char* name, K kern, int blocks, int iters, double ops_per_iter, uint32_t* d_out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_out, iters, 12345u);  // warmup
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_out, iters, 12345u);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  int dev = 0, cus = 0, clk = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CHK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));  // kHz
  const double waves = blocks * 4.0;
  const double simds = cus * 4.0;
  const double cyc = ms * 1e-3 * clk * 1e3;
  const double per_op = cyc * simds / (waves * iters * ops_per_iter);
  printf("%-28s %9.3f ms  %7.3f SIMD cycles per wave-op (clock %d MHz, %d CUs)\n", name, ms, per_op, clk / 1000, cus);
  return 0;
}

int main() {
  int dev = 0, cus = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = cus * 8;  // 256-thread blocks = 4 waves: 8 blocks per CU = 8 waves per SIMD
  uint32_t* d_out;
  CHK(hipMalloc(&d_out, sizeof(uint32_t) * blocks * 256));
  const int it_op = 4096, it_ph = 256;
  timeit("v_mul_lo_u32", k_op<0>, blocks, it_op, 8, d_out);
  timeit("v_mul_hi_u32", k_op<1>, blocks, it_op, 8, d_out);
  timeit("v_mul_u32_u24", k_op<2>, blocks, it_op, 8, d_out);
  timeit("v_add_u32", k_op<3>, blocks, it_op, 8, d_out);
  timeit("v_bitop3_b32 (xor3)", k_op<4>, blocks, it_op, 8, d_out);
  timeit("v_mad_u64_u32 (+xor)", k_op<5>, blocks, it_op, 8, d_out);
  timeit("philox10 C (per call)", k_philox<0>, blocks, it_ph, 1, d_out);
  timeit("philox10 mad64 (per call)", k_philox<1>, blocks, it_ph, 1, d_out);
  timeit("philox10 C x2 ILP (per call)", k_philox<2>, blocks, it_ph, 2, d_out);
  CHK(hipFree(d_out));
  return 0;
}
