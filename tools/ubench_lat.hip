// Latency of the latency path's one-lane steps on gfx950: how long one lane takes for a
// product, an exponentiation, hash_to_field, the SSWU map and the isogeny, with three
// 64-lane blocks (a config-3-sized call) on an otherwise idle device.  Each op runs
// `iters` times back to back in one launch so the launch overhead drops out.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc tools/ubench_lat.hip -o build/ubench_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "bls_hash.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ fp_t seed_fp(uint32_t s) {
  fp_t r;
  for (int i = 0; i < NL; ++i) r.v[i] = (s * 2654435761u + (uint32_t)i * 40503u) & LMASK;
  r.v[NL - 1] &= 0xffff;  // below p
  return r;
}

template <int OP>
__global__ void __launch_bounds__(64) k_lat(uint32_t* out, uint32_t seed, int iters) {
  const uint32_t tid = blockIdx.x * 64 + threadIdx.x;
  fp_t a = seed_fp(seed + tid), b = seed_fp(seed * 3 + tid + 17);
  uint32_t acc = 0;
  if (OP == 0) {
    for (int k = 0; k < iters; ++k) a = fp_mul(a, b);
    acc = a.v[0];
  } else if (OP == 1) {
    for (int k = 0; k < iters; ++k) a = fp_sqr(a);
    acc = a.v[0];
  } else if (OP == 2) {
    for (int k = 0; k < iters; ++k) a = fp_pow_p_minus_3_div_4(a);
    acc = a.v[0];
  } else if (OP == 3) {
    uint8_t msg[32];
    for (int i = 0; i < 32; ++i) msg[i] = (uint8_t)(tid + i + seed);
    for (int k = 0; k < iters; ++k) {
      fp2_t u0, u1;
      msg[0] ^= (uint8_t)k;
      hash_to_field_fp2(&u0, &u1, msg, 32);
      acc ^= u0.c0.v[0] ^ u1.c1.v[1];
    }
  } else if (OP == 4) {
    fp2_t u{a, b};
    for (int k = 0; k < iters; ++k) {
      const g2_jac q = sswu_g2_jac(u, fp_sqrt_minus5());
      u.c0 = q.x.c0;
      acc ^= q.y.c1.v[0];
    }
  } else if (OP == 5) {
    g2_jac q{{a, b}, {b, a}, {a, a}};
    for (int k = 0; k < iters; ++k) q = iso_map_g2_jac(q);
    acc = q.x.c0.v[0];
  }
  out[tid] = acc;
}

template <int OP>
static int run(const char* name, uint32_t* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_lat<OP>), dim3(blocks), dim3(64), 0, 0, d, 1u, 1);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_lat<OP>), dim3(blocks), dim3(64), 0, 0, d, (uint32_t)r + 2, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("{\"op\": \"%s\", \"blocks\": %d, \"iters\": %d, \"us_per_op\": %.3f}\n", name, blocks, iters,
         best * 1e3 / iters);
  return 0;
}

int main() {
  uint32_t* d;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * 64 * 64));
  for (int blocks : {3, 48}) {
    if (run<0>("fp_mul", d, blocks, 4000) || run<1>("fp_sqr", d, blocks, 4000) ||
        run<2>("fp_pow_p34", d, blocks, 20) || run<3>("hash_to_field_fp2", d, blocks, 20) ||
        run<4>("sswu_g2_jac", d, blocks, 10) || run<5>("iso_map_g2_jac", d, blocks, 40))
      return 1;
  }
  CHECK(hipFree(d));
  return 0;
}
