// Montgomery product issue efficiency on gfx950 at the occupancies the verify kernels run
// (1 and 2 waves per SIMD), long enough runs that launch overhead is < 1 %:
//   call   fp_mul (the out-of-line fp_mul_l every kernel calls)
//   body   fp_mul_body inlined (the compiler's column schedule)
//   split  each column's product sum in two interleaved accumulators (even / odd rows), the
//          reduction rows as in fp_mul_body: more independent mad chains in flight
//   split_call  the split product out of line (fp_mul_l's argument convention)
//   asm_call    the hand-scheduled subroutine of bgv_fpmul_asm.h (exact clobbers, no ABI)
// Products/s and the implied cycles per product per wave.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_prod tools/ubench_prod.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define BGV_ASM_EMIT 1
#include "../lodestar_amd/csrc/bls_field.h"
#include "experimental/bgv_fpmul_asm.h"

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

// product scanning with the a*b part of each column split over two accumulators
__device__ __forceinline__ fp_t mul_split(const fp_t& a, const fp_t& b) {
  const uint32_t P_[NL] = BGV_P_LIMBS;
  uint32_t m[NL];
  fp_t r;
  uint64_t carry = 0;
  BGV_UNROLL for (int k = 0; k < 2 * NL - 1; ++k) {
    uint64_t s0 = carry, s1 = 0;
    BGV_UNROLL for (int i = 0; i < NL; ++i) {
      const int j = k - i;
      if (j < 0 || j >= NL) continue;
      if (i & 1)
        s1 += (uint64_t)a.v[i] * b.v[j];
      else
        s0 += (uint64_t)a.v[i] * b.v[j];
    }
    BGV_UNROLL for (int i = 0; i < NL; ++i) {
      const int j = k - i;
      if (i >= k || j < 0 || j >= NL) continue;
      if (i & 1)
        s1 += (uint64_t)m[i] * P_[j];
      else
        s0 += (uint64_t)m[i] * P_[j];
    }
    uint64_t s = s0 + s1;
    if (k < NL) {
      m[k] = ((uint32_t)s * BGV_N0) & LMASK;
      s += (uint64_t)m[k] * P_[0];
    } else {
      r.v[k - NL] = (uint32_t)s & LMASK;
    }
    carry = s >> LBITS;
  }
  r.v[NL - 1] = (uint32_t)carry;
  return r;
}

// the split schedule out of line, with fp_mul_l's argument convention
static __device__ __noinline__ fp_t mul_split_l(BGV_U14(a_), BGV_U14(b_)) {
  const fp_t a = {{BGV_L14(a_)}}, b = {{BGV_L14(b_)}};
  return mul_split(a, b);
}

template <int V>
__device__ __forceinline__ fp_t prod(const fp_t& a, const fp_t& b) {
  if constexpr (V == 0) return fp_mul(a, b);
  if constexpr (V == 1) return fp_mul_body(a, b);
  if constexpr (V == 2) return mul_split(a, b);
  if constexpr (V == 3) return mul_split_l(BGV_V14(a), BGV_V14(b));
  fp_t r = a;  // V == 4: the hand-scheduled subroutine (bgv_fpmul_asm.h)
  bgv_fpmul_asm(r.v, b);
  return r;
}

// bit-exactness of the subroutines against fp_mul_body / fp_sqr_body on lane-varying operands
__global__ void __launch_bounds__(64) k_check(uint32_t* bad, uint32_t seed) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x = seed ^ (tid * 2654435761u);
  auto rnd = [&x] { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
  fp_t a, b;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    a.v[i] = rnd() & 0x1fffffff;
    b.v[i] = rnd() & 0x1fffffff;
  }
  a.v[NL - 1] &= 0x7ffff;
  b.v[NL - 1] &= 0x7ffff;
  fp_t m = a, q = a;
  bgv_fpmul_asm(m.v, b);
  bgv_fpsqr_asm(q.v);
  const fp_t m0 = fp_mul_body(a, b), q0 = fp_sqr_body(a);
  uint32_t diff = 0;
  BGV_UNROLL for (int i = 0; i < NL; ++i) diff |= (m.v[i] ^ m0.v[i]) | (q.v[i] ^ q0.v[i]);
  if (diff) atomicAdd(bad, 1u);
}

template <int V, int CHAINS>
__global__ void __launch_bounds__(64) k_prod(uint32_t* out, uint32_t seed, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fp_t x[CHAINS], y;
  BGV_UNROLL for (int i = 0; i < NL; ++i) y.v[i] = (seed * 7919u + i * 104729u + tid) & LMASK;
  y.v[NL - 1] &= 0xffff;
  BGV_UNROLL for (int c = 0; c < CHAINS; ++c) {
    BGV_UNROLL for (int i = 0; i < NL; ++i) x[c].v[i] = (seed + i + c + tid) & LMASK;
    x[c].v[NL - 1] &= 0xffff;
  }
  for (int k = 0; k < iters; ++k) BGV_UNROLL for (int c = 0; c < CHAINS; ++c) x[c] = prod<V>(x[c], y);
  uint32_t acc = 0;
  BGV_UNROLL for (int c = 0; c < CHAINS; ++c) BGV_UNROLL for (int i = 0; i < NL; ++i) acc ^= x[c].v[i];
  out[tid] = acc;
}

template <int V, int CHAINS>
static int run(const char* name, uint32_t* d, int cus, int wps) {
  const int iters = 2048, blocks = cus * 4 * wps;  // 64-thread blocks: wps waves on every SIMD
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_prod<V, CHAINS>), dim3(blocks), dim3(64), 0, 0, d, 1u, 4);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_prod<V, CHAINS>), dim3(blocks), dim3(64), 0, 0, d, (uint32_t)r, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double prods = (double)blocks * 64 * CHAINS * iters;
  const double wave_prods = prods / 64 / (cus * 4);  // per SIMD
  printf("{\"variant\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"fp_mul_per_s\": %.4e, \"ms\": %.3f, "
         "\"simd_cycles_per_wave_product_at_2.4GHz\": %.0f}\n",
         name, CHAINS, wps, prods / (best * 1e-3), best, best * 1e-3 * 2.4e9 / wave_prods);
  fflush(stdout);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * cus * 4 * 2 * 64));
  {
    uint32_t bad = 0;
    CHECK(hipMemset(d, 0, 4));
    for (uint32_t s = 1; s <= 16; ++s) hipLaunchKernelGGL(k_check, dim3(cus * 4), dim3(64), 0, 0, d, s);
    CHECK(hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost));
    printf("{\"check\": \"asm products vs fp_mul_body / fp_sqr_body\", \"lanes\": %d, \"mismatches\": %u}\n",
           cus * 4 * 64 * 16, bad);
    if (bad) return 1;
  }
  for (int wps : {1, 2}) {
    run<0, 1>("call", d, cus, wps);
    run<0, 2>("call", d, cus, wps);
    run<1, 1>("body", d, cus, wps);
    run<1, 2>("body", d, cus, wps);
    run<2, 1>("split", d, cus, wps);
    run<2, 2>("split", d, cus, wps);
    run<3, 1>("split_call", d, cus, wps);
    run<3, 2>("split_call", d, cus, wps);
    run<4, 1>("asm_call", d, cus, wps);
    run<4, 2>("asm_call", d, cus, wps);
  }
  CHECK(hipFree(d));
  return 0;
}
