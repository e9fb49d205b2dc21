// Latency of the wave-cooperative Fp (lodestar_amd/csrc/bgv_wfp.h) against the one-lane
// product on the chains the latency path runs: a (p-3)/4 exponentiation and a long squaring
// chain, one instance per wave, one wave on the chip.  Checks first:
//   dpp      wave_rol:1 / wave_shr:1 lane mapping
//   mul      wfp_mul == fp_mul_body (canonical values) on lane-varying random operands
//   pow      wfp_pow_fixed<P34> == fp_pow_fixed<P34>
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_wfp tools/ubench_wfp.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../lodestar_amd/csrc/bgv_wfp.h"

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void __launch_bounds__(64) k_dpp(uint32_t* out) {
  const uint32_t l = wfp_lane();
  out[l] = wfp_rol1(l + 100);
  out[64 + l] = wfp_shr1(l + 100, l);
}

__device__ fp_t rnd_fp(uint32_t& x) {
  fp_t a;
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    a.v[i] = x & LMASK;
  }
  a.v[NL - 1] &= 0x3ffff;  // < 2^382: below 2p after the top limb
  return a;
}

// block b: operands seeded by b (uniform over the wave); out[b] = canonical products
__global__ void __launch_bounds__(64) k_check(uint32_t* bad, uint32_t seed) {
  uint32_t x = seed * 2654435761u + blockIdx.x * 40503u + 1;
  const fp_t a = rnd_fp(x), b = rnd_fp(x);
  const wfp_ctx c = wfp_init();
  const uint32_t wa = wfp_from(a, c), wb = wfp_from(b, c);
  const fp_t m = wfp_to(wfp_mul(wa, wb, c)), q = wfp_to(wfp_mul_t<1, 1>(wa, wa, c));
  const fp_t q4 = wfp_to(wfp_mul_t<4, 4>(wa, wa, c)), q7 = wfp_to(wfp_mul_t<7, 2>(wa, wa, c));
  const fp_t q14 = wfp_to(wfp_mul_t<14, 2>(wa, wa, c)), q3 = wfp_to(wfp_mul3(wa, wa, c));
  const fp_t m3 = wfp_to(wfp_mul3(wa, wb, c));
  const fp_t mu = wfp_umul(a, b), qu = wfp_umul(a, a);
  fp_t su = a;
  for (int k = 0; k < 8; ++k) su = wfp_umul(su, b);
  uint32_t w3 = wa;
  for (int k = 0; k < 8; ++k) w3 = wfp_mul3(w3, wb, c);
  const fp_t m0 = fp_mul_body(a, b), q0 = fp_sqr_body(a);
  // chained: ((a b) b) ... 8 times, limbs of the intermediate fed back unnormalized
  uint32_t w = wa;
  fp_t s = a;
  for (int k = 0; k < 8; ++k) {
    w = wfp_mul(w, wb, c);
    s = fp_mul_body(s, b);
  }
  const fp_t d0 = fp_sub(fp_canon(m), fp_canon(m0)), d1 = fp_sub(fp_canon(q), fp_canon(q0));
  const fp_t d2 = fp_sub(fp_canon(wfp_to(w)), fp_canon(s));
  const fp_t d3 = fp_sub(fp_canon(m3), fp_canon(m0)), d4 = fp_sub(fp_canon(wfp_to(w3)), fp_canon(s));
  const fp_t d5 = fp_sub(fp_canon(mu), fp_canon(m0)), d6 = fp_sub(fp_canon(qu), fp_canon(q0));
  const fp_t d7 = fp_sub(fp_canon(su), fp_canon(s));
  const fp_t cq = fp_canon(q);
  const bool vok = fp_is_zero(fp_sub(fp_canon(q4), cq)) && fp_is_zero(fp_sub(fp_canon(q7), cq)) &&
                   fp_is_zero(fp_sub(fp_canon(q14), cq)) && fp_is_zero(fp_sub(fp_canon(q3), cq));
  if (!vok || !fp_is_zero(d0) || !fp_is_zero(d1) || !fp_is_zero(d2) || !fp_is_zero(d3) || !fp_is_zero(d4) ||
      !fp_is_zero(d5) || !fp_is_zero(d6) || !fp_is_zero(d7)) {
    if (wfp_lane() == 0) atomicAdd(bad, 1u);
  }
}

__global__ void __launch_bounds__(64) k_pow_check(uint32_t* bad, uint32_t seed) {
  uint32_t x = seed * 2654435761u + blockIdx.x * 40503u + 7;
  const fp_t a = rnd_fp(x);
  const fp_t w = wfp_pow_fixed<BGV_POW_P34>(a);
  const fp_t l = fp_pow_fixed<BGV_POW_P34>(a);
  if (!fp_is_zero(fp_sub(fp_canon(w), fp_canon(l))) && wfp_lane() == 0) atomicAdd(bad, 1u);
}

// reps chained (p-3)/4 exponentiations on lane 0 only
__global__ void __launch_bounds__(64) k_pow_lane(fp_t* io, int reps) {
  if (threadIdx.x != 0) return;
  fp_t x = io[blockIdx.x];
  for (int r = 0; r < reps; ++r) x = fp_pow_fixed<BGV_POW_P34>(x);
  io[blockIdx.x] = x;
}

__global__ void __launch_bounds__(64) k_pow_wave(fp_t* io, int reps) {
  fp_t x = io[blockIdx.x];
  for (int r = 0; r < reps; ++r) x = wfp_pow_fixed<BGV_POW_P34>(x);
  if (wfp_lane() == 0) io[blockIdx.x] = x;
}

__global__ void __launch_bounds__(64) k_sqr_lane(fp_t* io, int reps) {
  if (threadIdx.x != 0) return;
  fp_t x = io[blockIdx.x];
  for (int r = 0; r < reps; ++r) x = fp_sqr(x);
  io[blockIdx.x] = x;
}

__global__ void __launch_bounds__(64) k_sqr_umul(fp_t* io, int reps) {
  fp_t x = io[blockIdx.x];
  for (int r = 0; r < reps; ++r) x = wfp_umul(x, x);
  if (wfp_lane() == 0) io[blockIdx.x] = x;
}

__global__ void __launch_bounds__(64) k_sqr_wave3(fp_t* io, int reps) {
  const wfp_ctx c = wfp_init();
  uint32_t w = wfp_from(io[blockIdx.x], c);
  for (int r = 0; r < reps; ++r) w = wfp_mul3(w, w, c);
  const fp_t x = wfp_to(w);
  if (c.lane == 0) io[blockIdx.x] = x;
}

template <int K, int ACC>
__global__ void __launch_bounds__(64) k_sqr_wave(fp_t* io, int reps) {
  const wfp_ctx c = wfp_init();
  uint32_t w = wfp_from(io[blockIdx.x], c);
  for (int r = 0; r < reps; ++r) w = wfp_mul_t<K, ACC>(w, w, c);
  const fp_t x = wfp_to(w);
  if (c.lane == 0) io[blockIdx.x] = x;
}

template <class F>
static float time_ms(F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0, 0);
    launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  uint32_t* d;
  CHECK(hipMalloc(&d, 4096));
  {
    uint32_t h[128];
    hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, d);
    CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
      bad += h[l] != (uint32_t)((l + 1) % 64 + 100);
      bad += h[64 + l] != (l == 0 ? 0u : (uint32_t)(l - 1 + 100));
    }
    printf("{\"check\": \"dpp wave_rol1 / wave_shr1\", \"mismatches\": %d}\n", bad);
    if (bad) return 1;
  }
  {
    uint32_t bad = 0;
    CHECK(hipMemset(d, 0, 4));
    for (uint32_t s = 1; s <= 8; ++s) hipLaunchKernelGGL(k_check, dim3(1024), dim3(64), 0, 0, d, s);
    CHECK(hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost));
    printf("{\"check\": \"wfp_mul vs fp_mul_body\", \"cases\": %d, \"mismatches\": %u}\n", 8 * 1024, bad);
    if (bad) return 1;
    CHECK(hipMemset(d, 0, 4));
    hipLaunchKernelGGL(k_pow_check, dim3(512), dim3(64), 0, 0, d, 3u);
    CHECK(hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost));
    printf("{\"check\": \"wfp_pow_fixed vs fp_pow_fixed (p-3)/4\", \"cases\": 512, \"mismatches\": %u}\n", bad);
    if (bad) return 1;
  }
  fp_t* io;
  CHECK(hipMalloc(&io, sizeof(fp_t) * 64));
  std::vector<fp_t> h(64);
  for (int i = 0; i < 64; ++i)
    for (int l = 0; l < NL; ++l) h[i].v[l] = (uint32_t)(i * 131 + l * 7 + 3) & (l == NL - 1 ? 0x3ffffu : LMASK);
  CHECK(hipMemcpy(io, h.data(), sizeof(fp_t) * 64, hipMemcpyHostToDevice));
  const int reps = 8, sq = 4096;
  const float pl = time_ms([&] { hipLaunchKernelGGL(k_pow_lane, dim3(1), dim3(64), 0, 0, io, reps); });
  const float pw = time_ms([&] { hipLaunchKernelGGL(k_pow_wave, dim3(1), dim3(64), 0, 0, io, reps); });
  const float sl = time_ms([&] { hipLaunchKernelGGL(k_sqr_lane, dim3(1), dim3(64), 0, 0, io, sq); });
  const float sw = time_ms([&] { hipLaunchKernelGGL((k_sqr_wave<BGV_WFP_K, BGV_WFP_ACC>), dim3(1), dim3(64), 0, 0, io, sq); });
#define SWEEP(K, A)                                                                                    \
  printf("{\"sqr_ns_wave\": %.1f, \"K\": %d, \"ACC\": %d}\n",                                           \
         time_ms([&] { hipLaunchKernelGGL((k_sqr_wave<K, A>), dim3(1), dim3(64), 0, 0, io, sq); }) * 1e6 / sq, K, A)
  printf("{\"sqr_ns_umul\": %.1f}\n",
         time_ms([&] { hipLaunchKernelGGL(k_sqr_umul, dim3(1), dim3(64), 0, 0, io, sq); }) * 1e6 / sq);
  printf("{\"sqr_ns_wave3\": %.1f}\n",
         time_ms([&] { hipLaunchKernelGGL(k_sqr_wave3, dim3(1), dim3(64), 0, 0, io, sq); }) * 1e6 / sq);
  SWEEP(1, 1);
  SWEEP(1, 2);
  SWEEP(1, 4);
  SWEEP(2, 2);
  SWEEP(3, 2);
  SWEEP(4, 2);
  SWEEP(5, 2);
  SWEEP(7, 2);
  SWEEP(14, 2);
  SWEEP(4, 4);
  const float pw64 = time_ms([&] { hipLaunchKernelGGL(k_pow_wave, dim3(64), dim3(64), 0, 0, io, reps); });
  printf("{\"pow_p34_us\": {\"one_lane\": %.1f, \"wave\": %.1f, \"wave_64_blocks\": %.1f}, "
         "\"sqr_ns\": {\"one_lane\": %.1f, \"wave\": %.1f}}\n",
         pl * 1e3 / reps, pw * 1e3 / reps, pw64 * 1e3 / reps, sl * 1e6 / sq, sw * 1e6 / sq);
  return 0;
}
