// The wave round engine (tools/experimental/bgv_wround.h, not in the product library) against the four-part engine
// (bgv_tround_dev.h) on the latency path's G2 point programs: [|x|]P and the cofactor clearing
// for random points (one set per block), banks compared limb for limb, then the time of one
// [|x|]P chain (63 doublings + 5 additions, 214 rounds) on each.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc -o tools/ubench_wround tools/ubench_wround.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "bgv_tround_dev.h"
#include "experimental/bgv_wround.h"

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static __constant__ uint8_t kProg[TCP_TABLE_BYTES] = TCP_TABLE_INIT;

struct tc_wide_engine_u : tr_wide_engine {
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

__device__ void init_slots(fp_t* S, int t, int nt) {
  for (int i = t; i < TCP_NSLOT; i += nt) S[i] = fp_zero();
  __syncthreads();
  if (t == 0) {
    const fp2_t cx = BGV_PSI_CX, cy = BGV_PSI_CY;
    S[TCP_S_ONE] = fp_one();
    S[TCP_S_PSI_CX] = cx.c0;
    S[TCP_S_PSI_CX + 1] = cx.c1;
    S[TCP_S_PSI_CY] = cy.c0;
    S[TCP_S_PSI_CY + 1] = cy.c1;
    S[TCP_S_PSI2_CX] = fp_t{BGV_PSI2_CX};
    S[TCP_S_PSI2_CY] = fp_t{BGV_PSI2_CY};
  }
  __syncthreads();
}

// in: 2 points (12 fp_t) per block; mode 0: [|x|]P of point 0 (result bank -> out), 1: cofactor of p0 + p1
__global__ void __launch_bounds__(64) k_four(const fp_t* in, fp_t* out, int mode, int reps) {
  __shared__ uint8_t prog[TCP_TABLE_BYTES];
  __shared__ fp_t S[TCP_NSLOT];
  __shared__ fp_t RP[64];
  for (int i = threadIdx.x; i < TCP_TABLE_BYTES; i += 64) prog[i] = kProg[i];
  init_slots(S, threadIdx.x, 64);
  const int lane = threadIdx.x, c = lane % BGV_TEAM, q = lane / BGV_TEAM;
  tc_wide_engine_u e{{prog, S, RP, c, q, false}};
  const fp_t* x = in + 12 * blockIdx.x;
  int res = 3;
  for (int r = 0; r < reps; ++r) {
    if (lane < 6) {
      S[TCP_BANK(0) + lane] = x[lane];
      S[TCP_BANK(4) + lane] = x[lane];
      S[TCP_BANK(1) + lane] = x[lane];
      S[TCP_BANK(2) + lane] = x[6 + lane];
    }
    __syncthreads();
    if (mode == 0)
      res = tc_mul_x_abs(e);
    else
      tc_clear_cofactor(e);
  }
  if (lane < 6) out[6 * blockIdx.x + lane] = S[TCP_BANK(res) + lane];
}

__global__ void __launch_bounds__(256) k_wave4(const fp_t* in, fp_t* out, int mode, int reps) {
  __shared__ uint8_t prog[TCP_TABLE_BYTES];
  __shared__ fp_t S[TCP_NSLOT];
  for (int i = threadIdx.x; i < TCP_TABLE_BYTES; i += 256) prog[i] = kProg[i];
  init_slots(S, threadIdx.x, 256);
  tc_wave4_engine e{prog, S, wr_init(), (int)(threadIdx.x / 64), false};
  const fp_t* x = in + 12 * blockIdx.x;
  int res = 3;
  for (int r = 0; r < reps; ++r) {
    const int t = threadIdx.x;
    if (t < 6) {
      S[TCP_BANK(0) + t] = x[t];
      S[TCP_BANK(4) + t] = x[t];
      S[TCP_BANK(1) + t] = x[t];
      S[TCP_BANK(2) + t] = x[6 + t];
    }
    __syncthreads();
    if (mode == 0)
      res = tc_mul_x_abs(e);
    else
      tc_clear_cofactor(e);
  }
  if (threadIdx.x < 6) out[6 * blockIdx.x + threadIdx.x] = S[TCP_BANK(res) + threadIdx.x];
}

// random points: [k]G2 would need the curve code; any Jacobian triple with valid limbs exercises
// the same formulas (the programs do not check the curve equation)
int main() {
  const int nb = 64;
  std::vector<fp_t> h(12 * nb);
  uint32_t x = 12345;
  for (auto& f : h) {
    for (int l = 0; l < NL; ++l) {
      x ^= x << 13;
      x ^= x >> 17;
      x ^= x << 5;
      f.v[l] = x & LMASK;
    }
    f.v[NL - 1] &= 0x1ffff;  // < 2^381: below p
  }
  fp_t *din, *d4, *dw;
  CHECK(hipMalloc(&din, sizeof(fp_t) * h.size()));
  CHECK(hipMalloc(&d4, sizeof(fp_t) * 6 * nb));
  CHECK(hipMalloc(&dw, sizeof(fp_t) * 6 * nb));
  CHECK(hipMemcpy(din, h.data(), sizeof(fp_t) * h.size(), hipMemcpyHostToDevice));
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k_four, dim3(nb), dim3(64), 0, 0, din, d4, mode, 1);
    hipLaunchKernelGGL(k_wave4, dim3(nb), dim3(256), 0, 0, din, dw, mode, 1);
    CHECK(hipDeviceSynchronize());
    std::vector<fp_t> a(6 * nb), b(6 * nb);
    CHECK(hipMemcpy(a.data(), d4, sizeof(fp_t) * a.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(b.data(), dw, sizeof(fp_t) * b.size(), hipMemcpyDeviceToHost));
    // equal as field elements: both engines leave weakly reduced values (< 2p), whose
    // representatives may differ by p (the four-part engine reduces a sum of four parts)
    auto plus_p = [](const fp_t& x) {
      fp_t r;
      uint32_t c = 0;
      for (int l = 0; l < NL; ++l) {
        const uint32_t t = x.v[l] + p_limb(l) + c;
        r.v[l] = l < NL - 1 ? (t & LMASK) : t;
        c = t >> LBITS;
      }
      return r;
    };
    auto same = [](const fp_t& x, const fp_t& y) {
      for (int l = 0; l < NL; ++l)
        if (x.v[l] != y.v[l]) return false;
      return true;
    };
    int bad = 0, first = -1, plus = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      if (same(a[i], b[i])) continue;
      if (same(plus_p(a[i]), b[i]) || same(plus_p(b[i]), a[i])) {
        ++plus;
        continue;
      }
      if (first < 0) first = (int)i;
      ++bad;
    }
    printf("{\"check\": \"wave4 vs four-part engine (mod p)\", \"mode\": %d, \"fp_values\": %zu, \"mismatches\": %d, "
           "\"representatives_differing_by_p\": %d, \"first\": %d}\n",
           mode, a.size(), bad, plus, first);
    if (bad) {
      printf("{\"a0\": [");
      for (int l = 0; l < NL; ++l) printf("%u%s", a[first].v[l], l + 1 < NL ? "," : "");
      printf("], \"b0\": [");
      for (int l = 0; l < NL; ++l) printf("%u%s", b[first].v[l], l + 1 < NL ? "," : "");
      printf("]}\n");
      return 1;
    }
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float t4 = 0, tw = 0;
  for (int rep = 0; rep < 2; ++rep) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_four, dim3(nb), dim3(64), 0, 0, din, d4, 0, 4);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&t4, e0, e1));
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_wave4, dim3(nb), dim3(256), 0, 0, din, dw, 0, 4);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&tw, e0, e1));
  }
  printf("{\"mul_x_abs_us\": {\"four_part\": %.1f, \"wave4\": %.1f}, \"us_per_round\": {\"four_part\": %.3f, \"wave4\": %.3f}}\n",
         t4 * 1e3 / 4, tw * 1e3 / 4, t4 * 1e3 / 4 / 214, tw * 1e3 / 4 / 214);
  return 0;
}
