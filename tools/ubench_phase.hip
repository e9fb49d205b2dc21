// Phase microbenchmark for the bulk preparation kernel's point arithmetic (gfx950): one
// lane per set, 65,536 lanes (one wave per SIMD at WPE 1), each kernel one phase of k_prep:
//   xabs   [|x|]P on G2 (the signature subgroup check and each half of the cofactor clearing)
//   cof    g2_clear_cofactor (hash_to_G2's last phase)
//   glv2   r P on G2, GLV randomizer (r_i sig_i)
//   glv1   r P on G1 (r_i pk_i)
// Built once per variant: the lazy products out of line (ABI calls to fp_mul_l, the product
// build) or inlined (-DBGV_LAZY_INLINE_MUL), at BGV_WPE waves per SIMD.  Prints ms per launch
// and an output checksum (identical across variants: same formulas, same field elements).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DBGV_LAZY_INLINE_MUL] [-DBGV_WPE=2] \
//         -o tools/ubench_phase tools/ubench_phase.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../lodestar_amd/csrc/bgv_device.h"

#ifndef BGV_WPE
#define BGV_WPE 1
#endif
#define KATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE, BGV_WPE)))

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

// Clock diagnostics (a buffer of their own, never an output): per wave, s_memtime (shader
// clock) and s_memrealtime (100 MHz) at entry and exit; the in-kernel clock is their ratio.
__device__ uint64_t* g_stamps;
struct stamp_scope {
  uint64_t t0, r0;
  __device__ stamp_scope() {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  __device__ ~stamp_scope() {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (g_stamps && threadIdx.x == 0) {
      g_stamps[2 * blockIdx.x] = t1 - t0;
      g_stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
  }
};

__global__ void KATTR k_xabs(const g2_jac* __restrict__ in, g2_jac* __restrict__ out, uint32_t n) {
  stamp_scope st;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s < n) out[s] = jac_mul_x_abs(in[s]);
}
__global__ void KATTR k_cof(const g2_jac* __restrict__ in, g2_jac* __restrict__ out, uint32_t n) {
  stamp_scope st;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s < n) out[s] = g2_clear_cofactor(in[s]);
}
__global__ void KATTR k_glv2(const g2_jac* __restrict__ in, const uint64_t* __restrict__ k, g2_jac* __restrict__ out,
                             uint32_t n) {
  stamp_scope st;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s < n) out[s] = jac_mul_glv(in[s], k[s]);
}
__global__ void KATTR k_glv1(const g1_jac* __restrict__ in, const uint64_t* __restrict__ k, g1_jac* __restrict__ out,
                             uint32_t n) {
  stamp_scope st;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s < n) out[s] = jac_mul_glv(in[s], k[s]);
}

// hash_to_G2 without the cofactor clearing: XMD, the two SSWU maps, the isogeny, their sum
__global__ void KATTR k_hmap(const uint8_t* __restrict__ msgs, g2_jac* __restrict__ out, uint32_t n) {
  stamp_scope st;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s >= n) return;
  uint8_t m[32];
  for (int i = 0; i < 32; ++i) m[i] = msgs[32 * s + i];
  fp2_t u0, u1;
  hash_to_field_fp2(&u0, &u1, m, 32);
  const fp_t sm5 = fp_sqrt_minus5();
  const g2_jac q0 = iso_map_g2_jac(sswu_g2_jac(u0, sm5));
  const g2_jac q1 = iso_map_g2_jac(sswu_g2_jac(u1, sm5));
  out[s] = jac_add(q0, q1);
}
// one SSWU map to Jacobian (its square-root exponentiation included), no isogeny
__global__ void KATTR k_sswu(const g2_jac* __restrict__ in, g2_jac* __restrict__ out, uint32_t n) {
  stamp_scope st;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s < n) out[s] = sswu_g2_jac(in[s].x, fp_sqrt_minus5());
}
// the Fp exponentiation (p-3)/4 alone
__global__ void KATTR k_pow(const g2_jac* __restrict__ in, g2_jac* __restrict__ out, uint32_t n) {
  stamp_scope st;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s < n) out[s].x.c0 = fp_pow_fixed<BGV_POW_P34>(in[s].x.c0);
}

static uint32_t rnd(uint64_t* x) {
  *x ^= *x << 13;
  *x ^= *x >> 7;
  *x ^= *x << 17;
  return (uint32_t)(*x >> 11);
}

static void rnd_fp(fp_t* a, uint64_t* x) {
  for (int i = 0; i < NL; ++i) a->v[i] = rnd(x) & LMASK;
  a->v[NL - 1] &= 0xffff;  // < p
}

template <class T>
static uint32_t checksum(const T* d, size_t n) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(d);
  uint32_t h = 2166136261u;
  for (size_t i = 0; i < n * sizeof(T) / 4; ++i) h = (h ^ w[i]) * 16777619u;
  return h;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536u;
  const int reps = 3;
  uint64_t x = 0x9e3779b97f4a7c15ull;
  g2_jac* h2 = new g2_jac[n];
  g1_jac* h1 = new g1_jac[n];
  uint64_t* hk = new uint64_t[n];
  for (uint32_t i = 0; i < n; ++i) {
    rnd_fp(&h2[i].x.c0, &x), rnd_fp(&h2[i].x.c1, &x), rnd_fp(&h2[i].y.c0, &x), rnd_fp(&h2[i].y.c1, &x);
    rnd_fp(&h2[i].z.c0, &x), rnd_fp(&h2[i].z.c1, &x);
    rnd_fp(&h1[i].x, &x), rnd_fp(&h1[i].y, &x), rnd_fp(&h1[i].z, &x);
    hk[i] = ((uint64_t)rnd(&x) << 32) | rnd(&x) | 1;
  }
  g2_jac *d2, *o2;
  g1_jac *d1, *o1;
  uint64_t* dk;
  CHECK(hipMalloc(&d2, sizeof(g2_jac) * n));
  CHECK(hipMalloc(&o2, sizeof(g2_jac) * n));
  CHECK(hipMalloc(&d1, sizeof(g1_jac) * n));
  CHECK(hipMalloc(&o1, sizeof(g1_jac) * n));
  CHECK(hipMalloc(&dk, 8 * n));
  uint8_t* dm;
  CHECK(hipMalloc(&dm, 32 * n));
  {
    uint8_t* hm = new uint8_t[32 * n];
    for (uint32_t i = 0; i < 32 * n; ++i) hm[i] = (uint8_t)rnd(&x);
    CHECK(hipMemcpy(dm, hm, 32 * n, hipMemcpyHostToDevice));
    delete[] hm;
  }
  CHECK(hipMemcpy(d2, h2, sizeof(g2_jac) * n, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d1, h1, sizeof(g1_jac) * n, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dk, hk, 8 * n, hipMemcpyHostToDevice));
  uint64_t* dst;
  const uint32_t nblocks = (n + 63) / 64;
  CHECK(hipMalloc(&dst, 16 * nblocks));
  CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dst, sizeof(dst)));
  uint64_t* hst = new uint64_t[2 * nblocks];
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 grid((n + 63) / 64);
#ifdef BGV_LAZY_INLINE_MUL
  const char* var = "inline";
#else
  const char* var = "call";
#endif
  auto timeit = [&](const char* name, auto launch, auto sum) -> int {
    launch();  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0;
    for (int r = 0; r < reps; ++r) {
      CHECK(hipEventRecord(e0, 0));
      launch();
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      tot += ms;
    }
    CHECK(hipMemcpy(hst, dst, 16 * nblocks, hipMemcpyDeviceToHost));
    double ct = 0, cr = 0, wmax = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
      ct += (double)hst[2 * b];
      cr += (double)hst[2 * b + 1];
      wmax = hst[2 * b] > wmax ? (double)hst[2 * b] : wmax;
    }
    printf("{\"kernel\": \"%s\", \"variant\": \"%s\", \"wpe\": %d, \"lanes\": %u, \"ms_best\": %.3f, \"ms_mean\": %.3f, "
           "\"clock_ghz\": %.3f, \"wave_cycles_max\": %.0f, \"checksum\": \"%08x\"}\n",
           name, var, BGV_WPE, n, best, tot / reps, ct / cr * 0.1, wmax, sum());
    fflush(stdout);
    return 0;
  };
  g2_jac* r2 = new g2_jac[n];
  g1_jac* r1 = new g1_jac[n];
  auto sum2 = [&] {
    (void)hipMemcpy(r2, o2, sizeof(g2_jac) * n, hipMemcpyDeviceToHost);
    return checksum(r2, n);
  };
  auto sum1 = [&] {
    (void)hipMemcpy(r1, o1, sizeof(g1_jac) * n, hipMemcpyDeviceToHost);
    return checksum(r1, n);
  };
  const bool all = argc <= 2;
  const char* only = argc > 2 ? argv[2] : "";
  if (all || !strcmp(only, "xabs"))
    if (timeit("xabs", [&] { hipLaunchKernelGGL(k_xabs, grid, dim3(64), 0, 0, d2, o2, n); }, sum2)) return 1;
  if (all || !strcmp(only, "glv2"))
    if (timeit("glv2", [&] { hipLaunchKernelGGL(k_glv2, grid, dim3(64), 0, 0, d2, dk, o2, n); }, sum2)) return 1;
  if (all || !strcmp(only, "glv1"))
    if (timeit("glv1", [&] { hipLaunchKernelGGL(k_glv1, grid, dim3(64), 0, 0, d1, dk, o1, n); }, sum1)) return 1;
  if (all || !strcmp(only, "hmap"))
    if (timeit("hmap", [&] { hipLaunchKernelGGL(k_hmap, grid, dim3(64), 0, 0, dm, o2, n); }, sum2)) return 1;
  if (all || !strcmp(only, "sswu"))
    if (timeit("sswu", [&] { hipLaunchKernelGGL(k_sswu, grid, dim3(64), 0, 0, d2, o2, n); }, sum2)) return 1;
  if (all || !strcmp(only, "pow"))
    if (timeit("pow", [&] { hipLaunchKernelGGL(k_pow, grid, dim3(64), 0, 0, d2, o2, n); }, sum2)) return 1;
  if (all || !strcmp(only, "cof"))
    if (timeit("cof", [&] { hipLaunchKernelGGL(k_cof, grid, dim3(64), 0, 0, d2, o2, n); }, sum2)) return 1;
  return 0;
}
