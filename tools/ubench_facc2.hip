// Microbenchmark for DESIGN.md section 9 item 4: the bulk Miller stage's accumulator phase with
// one pair per lane (k_facc's staged walk, bgv_k_miller_bulk.hip) against two pairs per lane
// sharing one accumulator (one f^2 per step for both, f = f_a f_b).  Same line records (k_lines'
// layout), same LDS staging of the records (one buffer: pair b's record is staged while pair a's
// line product runs, then pair a's next one), P's constants in LDS.  Both kernels keep only
// two of P's constants in LDS and multiply by a Z^3 of 1 held in registers (the affine-P form
// the plan needs for its LDS budget), so the per-pair scaling work is the same in both.
// Prints ms per launch for n pairs and checks f2[l] == f1[2l] * f1[2l + 1] on the device.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/ubench_facc2 tools/ubench_facc2.hip
//   tools/bin/ubench_facc2 [n_pairs=131072] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../lodestar_amd/csrc/bgv_device.h"

#define KATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void KATTR u_lines(const g2_jac* __restrict__ q, uint32_t* __restrict__ lines, uint32_t n, uint32_t cap) {
  const uint32_t p = blockIdx.x * 64 + threadIdx.x;
  if (p >= n) return;
  uint32_t* base = lines + 4 * (size_t)p;
  miller_lines_walk(q + p, [&](int k, const auto& rec) {
    const uint4* w = reinterpret_cast<const uint4*>(&rec);
    uint4* dst = reinterpret_cast<uint4*>(base + (size_t)k * BGV_LINE_QUADS * 4 * cap);
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d) dst[(size_t)d * cap] = w[d];
  });
}

__device__ __forceinline__ lzr lz_one_r() {
  const fp_t o = fp_one();
  lzr v;
  BGV_UNROLL for (int i = 0; i < NL; ++i) v.v[i] = o.v[i];
  return v;
}

// one pair per lane: k_facc's walk
__global__ void KATTR u_facc1(const g1_jac* __restrict__ P, const uint32_t* __restrict__ lines, uint32_t n,
                              uint32_t cap, fp12_t* __restrict__ f) {
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  if (s >= n) return;
  __shared__ uint4 rec_lds[BGV_LINE_QUADS][64];
  __shared__ uint32_t p_lds[2 * NL][64];
  const int lane = threadIdx.x;
  const uint32_t* base = lines + 4 * (size_t)s;
  auto dma = [&](int k) {
    const uint32_t* src = base + (size_t)k * BGV_LINE_QUADS * 4 * cap;
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d)
      __builtin_amdgcn_global_load_lds(src + (size_t)d * 4 * cap, &rec_lds[d][0], 16, 0, 0);
  };
  dma(0);
  const miller_p P0 = miller_p_make(P[s]);
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    p_lds[i][lane] = P0.xn.v[i];
    p_lds[NL + i][lane] = P0.yp.v[i];
  }
  f[s] = miller_facc_walk_staged([&](int k, uint32_t z, auto* r) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    uint4* w = reinterpret_cast<uint4*>(r);
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d) w[d] = rec_lds[d][lane + z];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if (k + 1 < BGV_MILLER_STEPS) dma(k + 1);
  }, [&](int which, uint32_t z) {
    if (which == 2) return lz_one_r();
    lzr v;
    BGV_UNROLL for (int i = 0; i < NL; ++i) v.v[i] = p_lds[which * NL + i][lane + z];
    return v;
  });
}

// two pairs per lane, one accumulator: f <- f^2 * line_a(P_a) * line_b(P_b)
template <class Load, class PF>
__device__ fp12_t walk2(Load load, PF pget) {
  lz2r l0, l1, l3;
  lz_pline_d d;
  lz_pline_a a;
  load(0, 0, 0u, &d);
  lz_pline_scale_f(d, [&](int w, uint32_t z) { return pget(0, w, z); }, 0u, &l0, &l1, &l3);
  const lz2r zr = lz2r{lz_in(fp_zero()), lz_in(fp_zero())};
  lzf12 f = lzf12{lz6<LMASK, 2>{l0, l1, zr}, lz6<LMASK, 2>{zr, l3, zr}};
  {
    const uint32_t zb = lz12_after(f);
    load(1, 0, zb, &d);
    lz_pline_scale_f(d, [&](int w, uint32_t z) { return pget(1, w, z); }, zb, &l0, &l1, &l3);
    f = lz12_red(lz12_mul_line(f, l0, l1, l3));
  }
  int k = 1;
  BGV_NO_UNROLL for (int i = 61; i >= 0; --i) {
    if (miller_add_at(i)) {
      BGV_UNROLL for (int j = 0; j < 2; ++j) {
        const uint32_t za = lz12_after(f);
        load(j, k, za, &a);
        lz_pline_scale_f(a, [&](int w, uint32_t z) { return pget(j, w, z); }, za, &l0, &l1, &l3);
        f = lz12_red(lz12_mul_line(f, l0, l1, l3));
      }
      ++k;
    }
    f = lz12_red(lz12_sqr(f));
    BGV_UNROLL for (int j = 0; j < 2; ++j) {
      const uint32_t zd = lz12_after(f);
      load(j, k, zd, &d);
      lz_pline_scale_f(d, [&](int w, uint32_t z) { return pget(j, w, z); }, zd, &l0, &l1, &l3);
      f = lz12_red(lz12_mul_line(f, l0, l1, l3));
    }
    ++k;
  }
  return fp12_conj(lz12_out(f));
}

__global__ void KATTR u_facc2(const g1_jac* __restrict__ P, const uint32_t* __restrict__ lines, uint32_t n,
                              uint32_t cap, fp12_t* __restrict__ f) {
  const uint32_t l = blockIdx.x * 64 + threadIdx.x;
  if (2 * l + 1 >= n) return;
  __shared__ uint4 rec_lds[BGV_LINE_QUADS][64];
  __shared__ uint32_t p_lds[2][2 * NL][64];
  const int lane = threadIdx.x;
  const uint32_t* base[2] = {lines + 4 * (size_t)(2 * l), lines + 4 * (size_t)(2 * l + 1)};
  auto dma = [&](int j, int k) {
    const uint32_t* src = base[j] + (size_t)k * BGV_LINE_QUADS * 4 * cap;
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d)
      __builtin_amdgcn_global_load_lds(src + (size_t)d * 4 * cap, &rec_lds[d][0], 16, 0, 0);
  };
  dma(0, 0);
  BGV_UNROLL for (int j = 0; j < 2; ++j) {
    const miller_p Pj = miller_p_make(P[2 * l + j]);
    BGV_UNROLL for (int i = 0; i < NL; ++i) {
      p_lds[j][i][lane] = Pj.xn.v[i];
      p_lds[j][NL + i][lane] = Pj.yp.v[i];
    }
  }
  f[l] = walk2([&](int j, int k, uint32_t z, auto* r) {
    // record k of pair j landed: read it, then stage the next record (pair b's of this step,
    // or pair a's of the next)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    uint4* w = reinterpret_cast<uint4*>(r);
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d) w[d] = rec_lds[d][lane + z];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (j == 0)
      dma(1, k);
    else if (k + 1 < BGV_MILLER_STEPS)
      dma(0, k + 1);
  }, [&](int j, int which, uint32_t z) {
    if (which == 2) return lz_one_r();
    lzr v;
    BGV_UNROLL for (int i = 0; i < NL; ++i) v.v[i] = p_lds[j][which * NL + i][lane + z];
    return v;
  });
}

__global__ void u_check(const fp12_t* __restrict__ f1, const fp12_t* __restrict__ f2, uint32_t n2,
                        uint32_t* __restrict__ bad) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n2) return;
  const fp12_t m = fp12_mul(f1[2 * l], f1[2 * l + 1]);
  const fp_t* x = reinterpret_cast<const fp_t*>(&m);
  const fp_t* y = reinterpret_cast<const fp_t*>(f2 + l);
  bool ok = true;
  for (int i = 0; i < 12; ++i) ok = ok && fp_eq(x[i], y[i]);
  if (!ok) atomicAdd(bad, 1u);
}

// distinct points per pair: Q_p = G2 + [p] (a few doublings and additions of the generator),
// P_p likewise on G1, so no two lanes share values
__global__ void u_points(g2_jac* __restrict__ q, g1_jac* __restrict__ p, uint32_t n) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const fp2_t gx = BGV_G2X, gy = BGV_G2Y;
  const fp_t hx = BGV_G1X, hy = BGV_G1Y;
  const g2_jac g2 = {gx, gy, fp2_t{fp_one(), fp_zero()}};
  const g1_jac g1 = {hx, hy, fp_one()};
  g2_jac a2 = g2;
  g1_jac a1 = g1;
  for (int b = 0; b < 4; ++b) {
    a2 = jac_dbl(a2);
    a1 = jac_dbl(a1);
    if ((s >> b) & 1) {
      a2 = jac_add(a2, g2);
      a1 = jac_add(a1, g1);
    }
  }
  q[s] = a2;
  p[s] = a1;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 131072u;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  if (n < 2 || (n & 1) || n > (1u << 18)) {
    fprintf(stderr, "n_pairs must be even, 2..262144\n");
    return 2;
  }
  const uint32_t cap = n;
  g2_jac* q;
  g1_jac* p;
  uint32_t* lines;
  fp12_t *f1, *f2;
  uint32_t* bad;
  CHECK(hipMalloc(&q, sizeof(g2_jac) * n));
  CHECK(hipMalloc(&p, sizeof(g1_jac) * n));
  CHECK(hipMalloc(&lines, (size_t)BGV_MILLER_STEPS * BGV_LINE_WORDS * 4 * cap));
  CHECK(hipMalloc(&f1, sizeof(fp12_t) * n));
  CHECK(hipMalloc(&f2, sizeof(fp12_t) * (n / 2)));
  CHECK(hipMalloc(&bad, 4));
  CHECK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(u_points, dim3((n + 63) / 64), dim3(64), 0, 0, q, p, n);
  hipLaunchKernelGGL(u_lines, dim3((n + 63) / 64), dim3(64), 0, 0, q, lines, n, cap);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < reps; ++r) {
    for (int v = 1; v <= 2; ++v) {
      CHECK(hipEventRecord(e0, 0));
      if (v == 1)
        hipLaunchKernelGGL(u_facc1, dim3((n + 63) / 64), dim3(64), 0, 0, p, lines, n, cap, f1);
      else
        hipLaunchKernelGGL(u_facc2, dim3((n / 2 + 63) / 64), dim3(64), 0, 0, p, lines, n, cap, f2);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"kernel\": \"facc%d\", \"pairs\": %u, \"rep\": %d, \"ms\": %.3f}\n", v, n, r, ms);
      fflush(stdout);
    }
  }
  hipLaunchKernelGGL(u_check, dim3((n / 2 + 63) / 64), dim3(64), 0, 0, f1, f2, n / 2, bad);
  CHECK(hipGetLastError());
  uint32_t nb = 0;
  CHECK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
  printf("{\"check\": \"f2 == f1a * f1b\", \"mismatches\": %u, \"of\": %u}\n", nb, n / 2);
  return nb ? 1 : 0;
}
