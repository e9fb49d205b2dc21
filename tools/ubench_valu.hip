// gfx950 integer-VALU issue-rate microbenchmark: fixes the roofline denominator.
//
// Each lane runs 8 independent dependency chains of one instruction (inline
// asm so the compiler cannot fold it) for ITERS iterations; every CU is filled
// with 8 waves per SIMD.  Rate = lanes * 8 * ITERS / time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 4096;

__global__ void k_mad_u64_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3 + 7;
  uint64_t c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define MAD(c) c = (uint64_t)a * b + c; asm volatile("" : "+v"(c));
    MAD(c0) MAD(c1) MAD(c2) MAD(c3) MAD(c4) MAD(c5) MAD(c6) MAD(c7)
#undef MAD
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_mad_u64_u32_carry(uint64_t* out, uint32_t seed) {
  // with an SGPR-pair carry-out, as used by product-scanning Montgomery
  uint32_t a = seed + threadIdx.x, b = seed * 3 + 7;
  uint64_t c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define MAD(c) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "s40", "s41");
    MAD(c0) MAD(c1) MAD(c2) MAD(c3) MAD(c4) MAD(c5) MAD(c6) MAD(c7)
#undef MAD
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_mul_hi_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x;
  uint32_t c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define MUL(c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(c) : "v"(a));
    MUL(c0) MUL(c1) MUL(c2) MUL(c3) MUL(c4) MUL(c5) MUL(c6) MUL(c7)
#undef MUL
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_mul_lo_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x;
  uint32_t c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define MUL(c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(c) : "v"(a));
    MUL(c0) MUL(c1) MUL(c2) MUL(c3) MUL(c4) MUL(c5) MUL(c6) MUL(c7)
#undef MUL
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_add_co_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x;
  uint32_t c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define ADD(c) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(c) : "v"(a) : "vcc");
    ADD(c0) ADD(c1) ADD(c2) ADD(c3) ADD(c4) ADD(c5) ADD(c6) ADD(c7)
#undef ADD
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_mad_u32_u24(uint64_t* out, uint32_t seed) {
  uint32_t a = (seed + threadIdx.x) & 0xffffff, b = (seed * 3 + 7) & 0xffffff;
  uint32_t c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define MAD(c) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    MAD(c0) MAD(c1) MAD(c2) MAD(c3) MAD(c4) MAD(c5) MAD(c6) MAD(c7)
#undef MAD
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_fma_f64(uint64_t* out, uint32_t seed) {
  double a = 1.0000001 + threadIdx.x * 1e-9, b = 0.9999999;
  double c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define FMA(c) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    FMA(c0) FMA(c1) FMA(c2) FMA(c3) FMA(c4) FMA(c5) FMA(c6) FMA(c7)
#undef FMA
  }
  double s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = __double_as_longlong(s);
}


// simple 32-bit / 64-bit ops: is their issue cost 2 cycles (SIMD-32) with several waves per
// SIMD, and 4 with one wave alone?  (v_add_f32 is the guide's 2-cycle reference)
#define SIMPLE_KERNEL(NAME, ASM, T, INIT)                                                         \
  __global__ void NAME(uint64_t* out, uint32_t seed) {                                          \
    T a = (T)(seed + threadIdx.x);                                                              \
    T c0 = INIT(0), c1 = INIT(1), c2 = INIT(2), c3 = INIT(3), c4 = INIT(4), c5 = INIT(5), c6 = INIT(6), \
      c7 = INIT(7);                                                                             \
    for (int i = 0; i < ITERS; ++i) {                                                           \
      asm volatile(ASM : "+v"(c0) : "v"(a)); asm volatile(ASM : "+v"(c1) : "v"(a));             \
      asm volatile(ASM : "+v"(c2) : "v"(a)); asm volatile(ASM : "+v"(c3) : "v"(a));             \
      asm volatile(ASM : "+v"(c4) : "v"(a)); asm volatile(ASM : "+v"(c5) : "v"(a));             \
      asm volatile(ASM : "+v"(c6) : "v"(a)); asm volatile(ASM : "+v"(c7) : "v"(a));             \
    }                                                                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7); \
  }
#define I32(k) (uint32_t)(seed + threadIdx.x + k)
#define I64(k) (uint64_t)(seed + threadIdx.x + k)
SIMPLE_KERNEL(k_add_u32, "v_add_u32 %0, %0, %1", uint32_t, I32)
SIMPLE_KERNEL(k_and_b32, "v_and_b32 %0, %0, %1", uint32_t, I32)
SIMPLE_KERNEL(k_mov_b32, "v_mov_b32 %0, %1", uint32_t, I32)
SIMPLE_KERNEL(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1", uint64_t, I64)
SIMPLE_KERNEL(k_lshrrev_b64, "v_lshrrev_b64 %0, 3, %0", uint64_t, I64)
SIMPLE_KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc", uint32_t, I32)
__global__ void k_add_f32(uint64_t* out, uint32_t seed) {
  float a = 1.0f + threadIdx.x;
  float c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3, c4 = a + 4, c5 = a + 5, c6 = a + 6, c7 = a + 7;
  for (int i = 0; i < ITERS; ++i) {
#define ADDF(c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(c) : "v"(a));
    ADDF(c0) ADDF(c1) ADDF(c2) ADDF(c3) ADDF(c4) ADDF(c5) ADDF(c6) ADDF(c7)
#undef ADDF
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7);
}
// accumulator-register round trip (the spill slots of a 512-register kernel)
__global__ void k_accvgpr(uint64_t* out, uint32_t seed) {
  uint32_t c0 = seed + threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  for (int i = 0; i < ITERS; ++i) {
#define ACC(c, r) asm volatile("v_accvgpr_write_b32 " r ", %0\n v_accvgpr_read_b32 %0, " r : "+v"(c) :: r);
    ACC(c0, "a0") ACC(c1, "a1") ACC(c2, "a2") ACC(c3, "a3")
#undef ACC
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(c0 ^ c1 ^ c2 ^ c3);
}

typedef void (*kfn)(uint64_t*, uint32_t);

static int bench(const char* name, kfn k, uint64_t* d, int blocks, int threads, double* rate_out) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);  // warm
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double ops = (double)blocks * threads * 8.0 * ITERS;
  double rate = ops / (best * 1e-3);
  printf("{\"instr\": \"%s\", \"lane_ops_per_s\": %.4e, \"ms\": %.4f, \"lanes\": %d}\n", name, rate, best,
         blocks * threads);
  *rate_out = rate;
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.gcnArchName, cus, prop.clockRate);
  int threads = 256, blocks = cus * 8;  // 8 waves per SIMD
  uint64_t* d;
  CHECK(hipMalloc(&d, sizeof(uint64_t) * blocks * threads));
  double r;
  bench("v_mad_u64_u32", k_mad_u64_u32, d, blocks, threads, &r);
  bench("v_mad_u64_u32(carry)", k_mad_u64_u32_carry, d, blocks, threads, &r);
  bench("v_mul_hi_u32", k_mul_hi_u32, d, blocks, threads, &r);
  bench("v_mul_lo_u32", k_mul_lo_u32, d, blocks, threads, &r);
  bench("v_addc_co_u32", k_add_co_u32, d, blocks, threads, &r);
  bench("v_mad_u32_u24", k_mad_u32_u24, d, blocks, threads, &r);
  bench("v_fma_f64", k_fma_f64, d, blocks, threads, &r);
  // one wave per SIMD (the occupancy a 512-VGPR kernel gets)
  bench("v_mad_u64_u32@1wave/SIMD", k_mad_u64_u32, d, cus, threads, &r);
  // 8 waves per SIMD vs one wave per SIMD for the simple ops
  const struct { const char* n; kfn k; } simple[] = {
      {"v_add_u32", k_add_u32}, {"v_and_b32", k_and_b32}, {"v_mov_b32", k_mov_b32},
      {"v_lshl_add_u64", k_lshl_add_u64}, {"v_lshrrev_b64", k_lshrrev_b64}, {"v_cndmask_b32", k_cndmask},
      {"v_add_f32", k_add_f32}, {"v_accvgpr_write+read(2 instr)", k_accvgpr}};
  for (const auto& s : simple) {
    char nm[96];
    snprintf(nm, sizeof nm, "%s@8waves/SIMD", s.n);
    bench(nm, s.k, d, blocks, threads, &r);
    snprintf(nm, sizeof nm, "%s@2waves/SIMD", s.n);
    bench(nm, s.k, d, cus * 2, threads, &r);
    snprintf(nm, sizeof nm, "%s@1wave/SIMD", s.n);
    bench(nm, s.k, d, cus, threads, &r);
  }
  bench("v_mad_u64_u32@2waves/SIMD", k_mad_u64_u32, d, cus * 2, threads, &r);
  CHECK(hipFree(d));
  return 0;
}
