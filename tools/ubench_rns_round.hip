// Latency of the latency path's G2 point programs ([|x|]P: 63 doublings + 5 additions as
// rounds, bgv_tcurve.h tc_mul_x_abs) on one block of an idle device, per engine:
//   wide  the four-part round engine of k_prep_wide (bgv_tround_dev.h), one 64-lane block
//   rns   the residue round engine of k_prep_wide_rns (bgv_rns_round.h), one 512-thread block
// Both from the generator G2 (Jacobian, Z = 1); the results are compared on the host (the
// same point as fp_t after to_fp).  Rows: engine, us per call, rounds per call, us per round.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc -I tools/experimental tools/ubench_rns_round.hip -o tools/bin/ubench_rns_round
#include <hip/hip_runtime.h>

#include <cstdio>

#include "bgv_rns_round.h"
#include "bgv_tround_dev.h"

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static __constant__ uint8_t kProg[TCP_TABLE_BYTES] = TCP_TABLE_INIT;

struct wide_engine : tr_wide_engine {
  __device__ void copy(int dst, int src) {
    if (q == 0 && c < 6 && dst != src) S[TCP_BANK(dst) + c] = S[TCP_BANK(src) + c];
    __syncthreads();
  }
  __device__ void neg_y(int b) {
    if (q == 0 && (c == 2 || c == 3)) S[TCP_BANK(b) + c] = fp_neg(S[TCP_BANK(b) + c]);
    __syncthreads();
  }
  __device__ void check_add() {}
};

__device__ fp_t gen_coord(int k) {
  const fp2_t x = BGV_G2X, y = BGV_G2Y;
  return k < 4 ? (k == 0 ? x.c0 : k == 1 ? x.c1 : k == 2 ? y.c0 : y.c1) : (k == 4 ? fp_one() : fp_zero());
}

__global__ void __launch_bounds__(64) k_wide(fp_t* out, int calls) {
  __shared__ uint8_t prog[TCP_TABLE_BYTES];
  __shared__ fp_t S[TCP_NSLOT];
  __shared__ fp_t RP[64];
  const int lane = threadIdx.x;
  for (int i = lane; i < TCP_TABLE_BYTES; i += 64) prog[i] = kProg[i];
  if (lane < 6) S[TCP_BANK(0) + lane] = S[TCP_BANK(4) + lane] = gen_coord(lane);
  __syncthreads();
  wide_engine e{{prog, S, RP, tr_wide_lane_c(lane), tr_wide_lane_q(lane), false}};
  int a = 4;
  for (int t = 0; t < calls; ++t) {
    e.copy(4, a);
    a = tc_mul_x_abs(e);
  }
  if (lane < 6) out[lane] = S[TCP_BANK(a) + lane];
}

__global__ void __launch_bounds__(BGV_RNS_ROUND_THREADS) k_rns(fp_t* out, int calls) {
  __shared__ uint8_t prog[TCP_TABLE_BYTES];
  __shared__ uint32_t SR[TCP_NSLOT][32];
  __shared__ rns_xch XR;
  __shared__ fp_t io[6];
  for (int i = threadIdx.x; i < TCP_TABLE_BYTES; i += BGV_RNS_ROUND_THREADS) prog[i] = kProg[i];
  __syncthreads();
  rns_tc_engine e;
  e.init(SR, &XR, prog, threadIdx.x);
  fp_t v[12];
  int sl[12];
  for (int k = 0; k < 6; ++k) {
    v[k] = v[6 + k] = gen_coord(k);
    sl[k] = TCP_BANK(0) + k;
    sl[6 + k] = TCP_BANK(4) + k;
  }
  e.put(sl, v, 12);
  int a = 4;
  for (int t = 0; t < calls; ++t) {
    e.copy(4, a);
    a = tc_mul_x_abs(e);
  }
  int o6[6];
  for (int k = 0; k < 6; ++k) o6[k] = TCP_BANK(a) + k;
  e.get(o6, io, 6);
  if (threadIdx.x < 6) out[threadIdx.x] = io[threadIdx.x];
}

template <class L>
static int timed(const char* name, L launch, int calls) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  launch(1);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    launch(calls);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const int rounds = 63 * 2 + 5 * 3;  // TCP_PDBL: 2 rounds, TCP_PADD: 3 (bgv_tcurve.h)
  printf("{\"engine\": \"%s\", \"calls\": %d, \"us_per_call\": %.2f, \"rounds_per_call\": %d, \"us_per_round\": %.3f}\n",
         name, calls, best * 1e3 / calls, rounds, best * 1e3 / calls / rounds);
  fflush(stdout);
  return 0;
}

int main() {
  fp_t *d1, *d2;
  CHECK(hipMalloc(&d1, 6 * sizeof(fp_t)));
  CHECK(hipMalloc(&d2, 6 * sizeof(fp_t)));
  const int calls = 4;
  if (timed("wide", [&](int n) { hipLaunchKernelGGL(k_wide, dim3(1), dim3(64), 0, 0, d1, n); }, calls)) return 1;
  if (timed("rns", [&](int n) { hipLaunchKernelGGL(k_rns, dim3(1), dim3(BGV_RNS_ROUND_THREADS), 0, 0, d2, n); }, calls))
    return 1;
  hipLaunchKernelGGL(k_wide, dim3(1), dim3(64), 0, 0, d1, calls);
  hipLaunchKernelGGL(k_rns, dim3(1), dim3(BGV_RNS_ROUND_THREADS), 0, 0, d2, calls);
  CHECK(hipDeviceSynchronize());
  fp_t h1[6], h2[6];
  CHECK(hipMemcpy(h1, d1, sizeof(h1), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h2, d2, sizeof(h2), hipMemcpyDeviceToHost));
  int same = 1;
  for (int k = 0; k < 6; ++k) same &= fp_eq(h1[k], h2[k]) ? 1 : 0;
  printf("{\"same_point_coordinates\": %s}\n", same ? "true" : "false");
  return same ? 0 : 1;
}
