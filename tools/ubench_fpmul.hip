// Fp (BLS12-381) Montgomery multiplication throughput on gfx950: three limb
// layouts compared before committing the field layer to one of them.
//   v32  : 12 x 32-bit CIOS as written in bls_field.h (compiler-lowered)
//   v32r : 12 x 32-bit, row-wise with 64-bit accumulators + per-row carry pass
//   v28  : 14 x 28-bit unsaturated limbs, row-wise, no carry chains (R = 2^392)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../lodestar_amd/csrc/bls_field.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __constant__ uint32_t P28[14] = {0xfffaaab, 0xfeffffe, 0xfffffeb, 0x153ffff, 0xeabfffb, 0xb0f6241, 0x0d2a0f6,
  0x1bf6730, 0x84f3851, 0xd764774, 0xb4bacd7, 0x1b7b643, 0x7fe69a4, 0x00111ea3 & 0xfffffff};

struct f28 { uint32_t v[14]; };

__device__ __forceinline__ f28 mul28(const f28& a, const f28& b, const uint32_t* p) {
  const uint32_t M = 0xfffffff, N0 = 0x3fcfffd;  // placeholder n0 (throughput only)
  uint64_t t[14];
#pragma unroll
  for (int j = 0; j < 14; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
#pragma unroll
    for (int j = 0; j < 14; ++j) t[j] += (uint64_t)a.v[i] * b.v[j];
    uint32_t m = ((uint32_t)t[0] * N0) & M;
#pragma unroll
    for (int j = 0; j < 14; ++j) t[j] += (uint64_t)m * p[j];
    uint64_t c = t[0] >> 28;
#pragma unroll
    for (int j = 0; j < 13; ++j) t[j] = t[j + 1];
    t[13] = 0;
    t[0] += c;
  }
  f28 r;
#pragma unroll
  for (int j = 0; j < 13; ++j) { r.v[j] = (uint32_t)t[j] & M; t[j + 1] += t[j] >> 28; }
  r.v[13] = (uint32_t)t[13];
  return r;
}

__device__ __forceinline__ fp_t mul32r(const fp_t& a, const fp_t& b) {
  uint64_t t[13];
#pragma unroll
  for (int j = 0; j < 13; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
#pragma unroll
    for (int j = 0; j < 12; ++j) t[j] += (uint64_t)a.v[i] * b.v[j];
    // t[j] < 2^64 here since each t[j] < 2^32 before the row
    uint32_t m = (uint32_t)t[0] * BGV_N0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      uint64_t hi = t[j] >> 32;
      t[j] = (uint32_t)t[j] + (uint64_t)m * p_limb(j);
      t[j + 1] += hi;
    }
    // carry pass and shift
    uint64_t c = t[0] >> 32;
#pragma unroll
    for (int j = 1; j < 13; ++j) { t[j] += c; c = t[j] >> 32; t[j - 1] = (uint32_t)t[j]; }
    t[12] = c;
  }
  fp_t r;
#pragma unroll
  for (int j = 0; j < 12; ++j) r.v[j] = (uint32_t)t[j];
  return r;
}

template <int V, int CHAINS>
__global__ void __launch_bounds__(256) k_bench(uint32_t* out, uint32_t seed, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (V == 28) {
    f28 x[CHAINS], y;
#pragma unroll
    for (int i = 0; i < 14; ++i) y.v[i] = (seed * 7919u + i * 104729u + tid) & 0xfffffff;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
#pragma unroll
      for (int i = 0; i < 14; ++i) x[c].v[i] = (seed + i + c + tid) & 0xfffffff;
    for (int k = 0; k < iters; ++k)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) x[c] = mul28(x[c], y, P28);
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
#pragma unroll
      for (int i = 0; i < 14; ++i) acc ^= x[c].v[i];
    out[tid] = acc;
  } else {
    fp_t x[CHAINS], y;
#pragma unroll
    for (int i = 0; i < 12; ++i) y.v[i] = seed * 7919u + i * 104729u + tid;
    y.v[11] &= 0x0fffffff;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
#pragma unroll
      for (int i = 0; i < 12; ++i) x[c].v[i] = seed + i + c + tid;
      x[c].v[11] &= 0x0fffffff;
    }
    for (int k = 0; k < iters; ++k)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) x[c] = (V == 32) ? fp_mul(x[c], y) : mul32r(x[c], y);
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
#pragma unroll
      for (int i = 0; i < 12; ++i) acc ^= x[c].v[i];
    out[tid] = acc;
  }
}

template <int V, int CHAINS>
static int run(const char* name, uint32_t* d, int blocks) {
  const int iters = 256;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_bench<V, CHAINS>), dim3(blocks), dim3(256), 0, 0, d, 1u, 4);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_bench<V, CHAINS>), dim3(blocks), dim3(256), 0, 0, d, (uint32_t)r, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double muls = (double)blocks * 256 * CHAINS * iters;
  printf("{\"variant\": \"%s\", \"chains\": %d, \"blocks\": %d, \"fp_mul_per_s\": %.4e, \"ms\": %.3f}\n", name,
         CHAINS, blocks, muls / (best * 1e-3), best);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * cus * 8 * 256 * 4));
  for (int occ : {1, 2, 8}) {
    const int blocks = cus * occ;  // occ workgroups of 4 waves per CU = occ waves/SIMD
    run<32, 1>("v32", d, blocks);
    run<32, 2>("v32", d, blocks);
    run<33, 1>("v32r", d, blocks);
    run<33, 2>("v32r", d, blocks);
    run<28, 1>("v28", d, blocks);
    run<28, 2>("v28", d, blocks);
  }
  CHECK(hipFree(d));
  return 0;
}
