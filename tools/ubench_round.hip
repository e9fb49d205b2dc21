// Cost of one four-part round of the latency path's point programs (bgv_tround_dev.h) on
// gfx950: tc_mul_x_abs (63 doublings + 5 additions, 214 rounds) on 131 one-wave blocks, the
// real engine beside variants that drop one phase each (timing only; the slot values are
// not meaningful):
//   real      record + LDS operands + product + REDC, barrier, q = 0 sum4 + store, barrier
//   no_sum    phase 2 dropped (the parts are not summed)
//   no_prod   the product and REDC replaced by one LDS read of the first operand
//   no_redc   the product kept (generic tmp_lin), the REDC replaced by a fold of the wide accumulator
//   lin_only  the two operand combinations (templated) summed, no product
//   prod_only product + REDC of two slots read directly (no combinations)
//   engine    the production engine (bgv_tround_dev.h tr_wide_engine)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc tools/ubench_round.hip -o /tmp/ubench_round
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "bgv_tcurve.h"
#include "bls_team.h"
#include "bgv_tround_dev.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

static __constant__ uint8_t kProg[TCP_TABLE_BYTES] = TCP_TABLE_INIT;

template <int V>
struct ub_engine {
  const uint8_t* prog;
  fp_t* S;
  fp_t* P;
  int c, q;
  __device__ void run(int off) {
    int pos = off;
    const int nr = prog[pos++];
    for (int r = 0; r < nr; ++r) {
      const int T = prog[pos], M = prog[pos + 1];
      pos += 2;
      const int rb = tmp_rec_bytes(T, M);
      const uint8_t* rec = prog + pos + c * rb;
      fp_t v;
      if (V == 2) {
        v = S[rec[2]];
      } else if (V == 3) {
        uint64_t t[2 * NL];
        for (int i = 0; i < 2 * NL; ++i) t[i] = 0;
        for (int k = q; k < T; k += 4) {
          const uint8_t* rr = rec + 1 + k * 2 * (2 * M + 1);
          wide_mac(t, tmp_lin(S, rr, M), tmp_lin(S, rr + 2 * M + 1, M));
        }
        for (int i = 0; i < NL; ++i) v.v[i] = (uint32_t)(t[i] ^ t[i + NL]) & LMASK;
      } else if (V == 4) {
        const uint8_t* rr = rec + 1 + q * 2 * (2 * M + 1);
        fp_t x, y;
        switch (M) {
          case 1: x = tmp_lin_t<1>(S, rr); y = tmp_lin_t<1>(S, rr + 3); break;
          case 2: x = tmp_lin_t<2>(S, rr); y = tmp_lin_t<2>(S, rr + 5); break;
          case 3: x = tmp_lin_t<3>(S, rr); y = tmp_lin_t<3>(S, rr + 7); break;
          default: x = tmp_lin_t<4>(S, rr); y = tmp_lin_t<4>(S, rr + 9); break;
        }
        for (int i = 0; i < NL; ++i) v.v[i] = x.v[i] + y.v[i];
      } else if (V == 5) {
        const uint8_t* rr = rec + 1 + q * 2 * (2 * M + 1);
        uint64_t t[2 * NL];
        for (int i = 0; i < 2 * NL; ++i) t[i] = 0;
        wide_mac(t, S[rr[0]], S[rr[2 * M + 1]]);
        v = wide_redc(t);
      } else {
        v = tmp_lane_part(S, rec, T, M, q);
      }
      P[q * BGV_TEAM + c] = v;
      __syncthreads();
      if (V != 1 && q == 0) S[rec[0]] = tm_sum4(P[c], P[BGV_TEAM + c], P[2 * BGV_TEAM + c], P[3 * BGV_TEAM + c]);
      __syncthreads();
      pos += BGV_TEAM * rb;
    }
  }
  __device__ void check_add() {}
};

struct ub_prod_engine : tr_wide_engine {
  __device__ void check_add() {}
};

template <int V>
__global__ void __launch_bounds__(64) k_round(uint32_t* out, int reps) {
  __shared__ uint8_t prog[TCP_TABLE_BYTES];
  __shared__ fp_t S[TCP_NSLOT];
  __shared__ fp_t RP[64];
  const int lane = threadIdx.x;
  for (int i = lane; i < TCP_TABLE_BYTES; i += 64) prog[i] = kProg[i];
  for (int i = lane; i < TCP_NSLOT; i += 64) {
    fp_t x = fp_one();
    x.v[0] += (uint32_t)(i + blockIdx.x);
    S[i] = x;
  }
  __syncthreads();
  int a = 0;
  if (V == 6) {
    ub_prod_engine e{{prog, S, RP, lane % BGV_TEAM, lane / BGV_TEAM, false}};
    for (int k = 0; k < reps; ++k) a += tc_mul_x_abs(e);
  } else {
    ub_engine<V> e{prog, S, RP, lane % BGV_TEAM, lane / BGV_TEAM};
    for (int k = 0; k < reps; ++k) a += tc_mul_x_abs(e);
  }
  if (lane == 0) out[blockIdx.x] = S[a % TCP_NSLOT].v[0];
}

template <int V>
static int run(const char* name, uint32_t* d, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_round<V>), dim3(blocks), dim3(64), 0, 0, d, 1);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  const int reps = 4;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_round<V>), dim3(blocks), dim3(64), 0, 0, d, reps);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const int rounds = 63 * 3 + 5 * 5;
  printf("{\"variant\": \"%s\", \"blocks\": %d, \"us_per_mul_x\": %.1f, \"us_per_round\": %.3f}\n", name, blocks,
         best * 1e3 / reps, best * 1e3 / reps / rounds);
  return 0;
}

int main() {
  uint32_t* d;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * 1024));
  for (int blocks : {131})
    if (run<0>("real", d, blocks) || run<1>("no_sum", d, blocks) || run<2>("no_prod", d, blocks) ||
        run<3>("no_redc", d, blocks) || run<4>("lin_only", d, blocks) || run<5>("prod_only", d, blocks) || run<6>("engine", d, blocks))
      return 1;
  CHECK(hipFree(d));
  return 0;
}
