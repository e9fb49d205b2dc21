// Latency of one Fp12 operation of the latency path's final exponentiation (bls_team.h
// tm_pow_x: 63 squarings, 5 products, a conjugation per call) on one block of an idle device:
//   rns    the residue-number-system engine (bgv_rns.h): 384 threads, one residue per lane
//   part8  the current engine of k_final_fold (bgv_team_dev.h tm_wide8_lean_ops): 256 threads,
//          each coefficient's double-width products split over eight lanes
//   rns1   the RNS engine with the whole block's 12 coefficients folded onto one wave (the
//          "single wave" layout: six passes of the lane work per operation) -- not built: one
//          wave would serialize the six coefficient pairs, so it is the rns row x ~6 by count
// The values are checked by tools/gpu/rns_probe.py (it writes IN, runs this, reads OUT):
//   IN:  a as 12 x 30 RNS residues (of a M mod p), then the same a as 12 fp_t (R = 2^392 form)
//   OUT: the rns chain's result (12 x 30), from_fp(a) (12 x 30), the part8 chain's result
//        (12 fp_t, w-basis order), to_fp(a) (12 fp_t)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc tools/ubench_rns.hip -o tools/bin/ubench_rns
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "bgv_team_dev.h"
#include "bgv_rns.h"

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void __launch_bounds__(BGV_RNS_THREADS) k_rns_chain(const uint32_t* in, uint32_t* out, int calls) {
  __shared__ rns_smem S;
  rns_ops o;
  o.init(&S, threadIdx.x);
  uint32_t a = o.live ? in[o.c * BGV_RNS_NL + o.i] : 0u;
  for (int t = 0; t < calls; ++t) a = tm_pow_x(o, a);
  if (o.live) out[o.c * BGV_RNS_NL + o.i] = a;
}

__global__ void __launch_bounds__(BGV_RNS_THREADS) k_rns_from_fp(const fp_t* in, uint32_t* out) {
  __shared__ rns_smem S;
  rns_ops o;
  o.init(&S, threadIdx.x);
  const uint32_t a = o.from_fp(in[o.c]);
  if (o.live) out[o.c * BGV_RNS_NL + o.i] = a;
}

__global__ void __launch_bounds__(BGV_RNS_THREADS) k_rns_to_fp(const uint32_t* in, fp_t* out) {
  __shared__ rns_smem S;
  rns_ops o;
  o.init(&S, threadIdx.x);
  const fp_t r = o.to_fp(o.live ? in[o.c * BGV_RNS_NL + o.i] : 0u);
  if (o.i == 0) out[o.c] = r;
}

#define P8_THREADS 256
__global__ void __launch_bounds__(P8_THREADS) k_part8_chain(const fp_t* in, fp_t* out, int calls) {
  __shared__ fp_t WA[BGV_TEAM_COMPS], WB[BGV_TEAM_COMPS], WP[8 * BGV_TEAM_COMPS];
  const int wc = threadIdx.x % BGV_TEAM_COMPS, wq = threadIdx.x / BGV_TEAM_COMPS;
  tm_wide8_lean_ops ow;
  ow.A = WA;
  ow.B = WB;
  ow.P = WP;
  ow.c = wc;
  ow.q = wq;
  tm_sqr_rec8(wc, wq, &ow.rx, &ow.ry);
  fp_t a = in[wc];
  for (int t = 0; t < calls; ++t) a = tm_pow_x(ow, a);
  if (wq == 0) out[wc] = a;
}

static int timed(const char* name, int threads, int calls, hipEvent_t e0, hipEvent_t e1, float* best,
                 void (*launch)(int)) {
  launch(1);
  CHECK(hipDeviceSynchronize());
  *best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    launch(calls);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < *best) *best = ms;
  }
  const double ops = 69.0 * calls;  // per tm_pow_x: 63 sqr + 5 mul + 1 conj
  printf("{\"engine\": \"%s\", \"threads\": %d, \"pow_x_calls\": %d, \"ms\": %.4f, \"us_per_fp12_op\": %.3f}\n", name,
         threads, calls, *best, *best * 1e3 / ops);
  fflush(stdout);
  return 0;
}

static uint32_t *d_in, *d_out, *d_out2;
static fp_t *d_fin, *d_fout, *d_fout2;

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: ubench_rns IN OUT [calls]\n");
    return 2;
  }
  const int calls = argc > 3 ? atoi(argv[3]) : 4;
  std::vector<uint32_t> in(12 * 30 + 12 * 14);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(in.data(), 4, in.size(), f) != in.size()) {
    fprintf(stderr, "bad input %s\n", argv[1]);
    return 2;
  }
  fclose(f);
  CHECK(hipMalloc(&d_in, 12 * 30 * 4));
  CHECK(hipMalloc(&d_out, 12 * 30 * 4));
  CHECK(hipMalloc(&d_out2, 12 * 30 * 4));
  CHECK(hipMalloc(&d_fin, 12 * sizeof(fp_t)));
  CHECK(hipMalloc(&d_fout, 12 * sizeof(fp_t)));
  CHECK(hipMalloc(&d_fout2, 12 * sizeof(fp_t)));
  CHECK(hipMemcpy(d_in, in.data(), 12 * 30 * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_fin, in.data() + 12 * 30, 12 * sizeof(fp_t), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float t_rns, t_p8;
  if (timed("rns", BGV_RNS_THREADS, calls, e0, e1, &t_rns, [](int n) {
        hipLaunchKernelGGL(k_rns_chain, dim3(1), dim3(BGV_RNS_THREADS), 0, 0, d_in, d_out, n);
      }))
    return 1;
  if (timed("part8", P8_THREADS, calls, e0, e1, &t_p8, [](int n) {
        hipLaunchKernelGGL(k_part8_chain, dim3(1), dim3(P8_THREADS), 0, 0, d_fin, d_fout, n);
      }))
    return 1;
  printf("{\"rns_speedup_vs_part8\": %.3f}\n", t_p8 / t_rns);
  // the checked values: the chains at `calls`, and from_fp
  hipLaunchKernelGGL(k_rns_chain, dim3(1), dim3(BGV_RNS_THREADS), 0, 0, d_in, d_out, calls);
  hipLaunchKernelGGL(k_rns_from_fp, dim3(1), dim3(BGV_RNS_THREADS), 0, 0, d_fin, d_out2);
  hipLaunchKernelGGL(k_part8_chain, dim3(1), dim3(P8_THREADS), 0, 0, d_fin, d_fout, calls);
  hipLaunchKernelGGL(k_rns_to_fp, dim3(1), dim3(BGV_RNS_THREADS), 0, 0, d_in, d_fout2);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> out(12 * 30 * 2 + 12 * 14 * 2);
  CHECK(hipMemcpy(out.data(), d_out, 12 * 30 * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(out.data() + 12 * 30, d_out2, 12 * 30 * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(out.data() + 24 * 30, d_fout, 12 * sizeof(fp_t), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(out.data() + 24 * 30 + 12 * 14, d_fout2, 12 * sizeof(fp_t), hipMemcpyDeviceToHost));
  f = fopen(argv[2], "wb");
  if (!f || fwrite(out.data(), 4, out.size(), f) != out.size()) return 2;
  fclose(f);
  return 0;
}
