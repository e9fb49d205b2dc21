// Deferred-reduction Fp2 products (bls_wide.h) against the fully reduced Karatsuba of
// bls_lazy.h, at the occupancies the bulk kernels run (1 and 2 waves per SIMD):
//   fp2_mul    x <- x * y          (lz2_mul: 3 fp_mul_l calls  |  one fp2_mul_w_l call)
//   fp2_sqr    x <- x^2            (lz2_sqr: 2 calls           |  one fp2_sqr_w_l call)
//   fp12_sqr   f <- f^2            (lz12_sqr, 12 Fp2 products, the k_facc squaring)
//   mul_line   f <- f * line       (lz12_mul_line, the k_facc line product)
// Built twice (tools/gpu/ubench_wide.sh): -DBGV_LZ2_WIDE selects the deferred forms inside the
// tower, so the Fp12 rows compare the same formulas over both product kinds.  Each row also
// checks its result against the host build of the same chain (tests compare the host builds).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DBGV_LZ2_WIDE] -o ubench_wide tools/ubench_wide.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../lodestar_amd/csrc/bls_lazy.h"

#ifdef BGV_LZ2_WIDE
#define VARIANT "wide"
#else
#define VARIANT "classic"
#endif

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef lz12<LMASK, 2> lzf12u;

__host__ __device__ inline lzr seed_fp(uint32_t s, uint32_t t) {
  lzr r;
  uint32_t x = s * 2654435761u ^ (t + 0x9e3779b9u);
  for (int i = 0; i < NL; ++i) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    r.v[i] = x & LMASK;
  }
  r.v[NL - 1] &= 0xffff;
  return r;
}
__host__ __device__ inline lz2r seed_fp2(uint32_t s, uint32_t t) { return lz2r{seed_fp(s, t), seed_fp(s + 1, t)}; }
__host__ __device__ inline lzf12u seed_fp12(uint32_t s, uint32_t t) {
  return lzf12u{lz6<LMASK, 2>{seed_fp2(s, t), seed_fp2(s + 2, t), seed_fp2(s + 4, t)},
                lz6<LMASK, 2>{seed_fp2(s + 6, t), seed_fp2(s + 8, t), seed_fp2(s + 10, t)}};
}
__host__ __device__ inline uint32_t fold(const lz2r& a) {
  const fp_t c0 = fp_canon(lz_out(a.c0)), c1 = fp_canon(lz_out(a.c1));
  uint32_t h = 0;
  for (int i = 0; i < NL; ++i) h = h * 31u + (c0.v[i] ^ (c1.v[i] << 1));
  return h;
}
__host__ __device__ inline uint32_t fold12(const lzf12u& f) {
  return fold(f.c0.c0) ^ fold(f.c0.c1) * 3u ^ fold(f.c0.c2) * 5u ^ fold(f.c1.c0) * 7u ^ fold(f.c1.c1) * 11u ^
         fold(f.c1.c2) * 13u;
}

// the chains, one per lane
template <int OP>
__host__ __device__ inline uint32_t chain(uint32_t seed, uint32_t tid, int iters) {
  if constexpr (OP == 4 || OP == 5) {
    // the deferred-reduction body inlined (no call, no slot): the call and LDS overhead of OP 0;
    // OP 5 also without the result's reduction to the fp_t invariant
    lz2r x = seed_fp2(seed, tid);
    const lz2r y = seed_fp2(seed + 7, tid);
    for (int k = 0; k < iters; ++k) {
      uint32_t r0[NL], r1[NL];
      fp2_mul_w_body(x.c0.v, x.c1.v, y.c0.v, y.c1.v, r0, r1);
      lz2<LMASK, 2> o;
      for (int i = 0; i < NL; ++i) {
        o.c0.v[i] = r0[i];
        o.c1.v[i] = r1[i];
      }
      if constexpr (OP == 4)
        x = lz2_red(o);
      else
        x = o;
    }
    return fold(x);
  } else if constexpr (OP == 0 || OP == 1) {
    lz2r x = seed_fp2(seed, tid);
    const lz2r y = seed_fp2(seed + 7, tid);
    for (int k = 0; k < iters; ++k) {
      if constexpr (OP == 0)
        x = lz2_red(lz2_mul(x, y));
      else
        x = lz2_sqr(x);
    }
    return fold(x);
  } else {
    lzf12u f = seed_fp12(seed, tid);
    const lz2r l0 = seed_fp2(seed + 20, tid), l1 = seed_fp2(seed + 22, tid), l3 = seed_fp2(seed + 24, tid);
    for (int k = 0; k < iters; ++k) {
      if constexpr (OP == 2)
        f = lz12_red(lz12_sqr(f));
      else
        f = lz12_red(lz12_mul_line(f, l0, l1, l3));
    }
    return fold12(f);
  }
}

template <int OP, int WPS>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPS, WPS)))
k_chain(uint32_t* out, uint32_t seed, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  out[tid] = chain<OP>(seed, tid, iters);
}

static const char* kOpName[6] = {"fp2_mul", "fp2_sqr", "fp12_sqr", "mul_line", "fp2_mul_inline", "fp2_mul_body_only"};

template <int OP, int WPS>
static int run(uint32_t* d, int cus) {
  const int blocks = cus * 4 * WPS;
  const int iters = (OP < 2 || OP >= 4) ? 4096 : 256;
  const int n = blocks * 64;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_chain<OP, WPS>), dim3(blocks), dim3(64), 0, 0, d, 1u, 4);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_chain<OP, WPS>), dim3(blocks), dim3(64), 0, 0, d, 5u, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  // spot-check 8 lanes against the host build of the same chain
  uint32_t h[8];
  CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int t = 0; t < 8; ++t) bad += h[t] != chain<OP>(5u, (uint32_t)t, iters);
  const double ops = (double)n * iters;
  const double per_simd = ops / 64 / (cus * 4);
  printf("{\"variant\": \"%s\", \"op\": \"%s\", \"waves_per_simd\": %d, \"ops_per_s\": %.4e, \"ms\": %.3f, "
         "\"simd_cycles_per_wave_op_at_2.4GHz\": %.0f, \"host_mismatches\": %d, \"fold0\": \"%08x\"}\n",
         VARIANT, kOpName[OP], WPS, ops / (best * 1e-3), best, best * 1e-3 * 2.4e9 / per_simd, bad, h[0]);
  fflush(stdout);
  return bad;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * cus * 4 * 2 * 64));
  int bad = 0;
  bad += run<0, 1>(d, cus);
  bad += run<4, 1>(d, cus);
  bad += run<5, 1>(d, cus);
  bad += run<1, 1>(d, cus);
  bad += run<2, 1>(d, cus);
  bad += run<3, 1>(d, cus);
  bad += run<0, 2>(d, cus);
  bad += run<2, 2>(d, cus);
  bad += run<3, 2>(d, cus);
  CHECK(hipFree(d));
  return bad ? 1 : 0;
}
