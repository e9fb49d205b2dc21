// Device kernels beside the verify path (gfx950): SURVEY 8(f) rows (deposit-key
// validation, op-pool signature aggregation), the hash_to_G2 parity hook, pubkey-cache
// uploads, bench/test key generation and signing; and the verify launch's memory layout.
#include "bgv_device.h"

extern "C" {

// ---------------------------------------------------------------------------
// SURVEY 8(f) rows next to the verify path
// ---------------------------------------------------------------------------
// Deposit-time key validation (processDeposit.ts:62-69, PublicKey.fromBytes(pk, affine,
// validate=true)): ZCash decode, infinity -> BLST_PK_IS_INFINITY, [r]P != O ->
// BLST_POINT_NOT_IN_GROUP.  Valid keys are written as 96-B uncompressed records.
__device__ __noinline__ bool g1_in_subgroup(const g1_aff& a) {
  const uint32_t r[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                         0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  return jac_is_inf(jac_mul_u256(jac_from_aff(a), r));
}

__global__ void k_pk_validate(const uint8_t* __restrict__ keys48, uint32_t n, int32_t* __restrict__ status,
                              uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[48];
  for (int q = 0; q < 48; ++q) b[q] = keys48[48ull * i + q];
  g1_aff a;
  bool inf;
  int st = g1_decompress(&a, &inf, b);
  if (st == BGV_OK) {
    if (inf)
      st = BGV_PK_IS_INFINITY;
    else if (!g1_in_subgroup(a))
      st = BGV_POINT_NOT_IN_GROUP;
  }
  status[i] = st;
  uint8_t o[96];
  g1_serialize(o, a, st != BGV_OK);
  for (int q = 0; q < 96; ++q) out96[96ull * i + q] = o[q];
}

// Signature decode for aggregation (Signature.fromBytes(sig, undefined, true)): one
// signature per lane -> Jacobian point (infinity for the infinity encoding) + status.
__global__ void k_sig_decode(const uint8_t* __restrict__ sigs96, const uint32_t* __restrict__ lens, uint32_t n,
                             g2_jac* __restrict__ pts, int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t st = BGV_OK;
  g2_jac out = jac_infinity<fp2_t>();
  if (lens[i] != 96) {
    st = BGV_INVALID_SIZE;
  } else {
    uint8_t b[96];
    for (int q = 0; q < 96; ++q) b[q] = sigs96[96ull * i + q];
    g2_aff a;
    bool inf;
    st = g2_decompress(&a, &inf, b);
    if (st == BGV_OK && !inf) {
      const g2_jac j = jac_from_aff(a);
      if (g2_in_subgroup(j))
        out = j;
      else
        st = BGV_POINT_NOT_IN_GROUP;
    }
  }
  pts[i] = out;
  status[i] = st;
}

// One wavefront per aggregate: strided partial sums, then an LDS tree; compressed out.
__global__ void BGV_KATTR k_sig_sum(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count,
                                    const g2_jac* __restrict__ pts, uint8_t* __restrict__ out96) {
  extern __shared__ uint32_t lds[];
  g2_jac* ls = reinterpret_cast<g2_jac*>(lds);
  const uint32_t a = blockIdx.x, j = threadIdx.x, f = first[a], n = count[a];
  g2_jac acc = jac_infinity<fp2_t>();
  for (uint32_t k = j; k < n; k += BGV_WAVE) acc = jac_add(acc, pts[f + k]);
  for (uint32_t d = 1; d < BGV_WAVE; d <<= 1) {
    ls[j] = acc;
    __syncthreads();
    if ((j & (2 * d - 1)) == 0) acc = jac_add(acc, ls[j + d]);
    __syncthreads();
  }
  if (j == 0) {
    g2_aff r;
    const bool fin = jac_to_aff(&r, acc);
    uint8_t b[96];
    g2_compress(b, r, !fin);
    for (int q = 0; q < 96; ++q) out96[96ull * a + q] = b[q];
  }
}


__global__ void k_hash_msgs(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ offs,
                            const uint32_t* __restrict__ lens, uint32_t n, uint8_t* __restrict__ out192) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2_aff a;
  const bool fin = jac_to_aff(&a, hash_to_g2(msgs + offs[i], lens[i]));
  uint8_t b[192];
  g2_serialize(b, a, !fin);
  for (int k = 0; k < 192; ++k) out192[192ull * i + k] = b[k];
}

// Parity hook (bgv_debug_prepare): per slot, its H(m) serialized like k_hash_msgs and its
// Miller-loop value f as 12 canonical big-endian Fp coefficients (k_fp12_to_bytes order)
__global__ void k_debug_out(const bgv_dslot* __restrict__ slots, uint32_t n, const g2_jac* __restrict__ h,
                            const fp12_t* __restrict__ f, uint8_t* __restrict__ out_h192,
                            uint8_t* __restrict__ out_f576) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  g2_aff a;
  const bool fin = jac_to_aff(&a, h[slots[s].hsrc]);
  uint8_t b[192];
  g2_serialize(b, a, !fin);
  for (int k = 0; k < 192; ++k) out_h192[192ull * s + k] = b[k];
  const fp_t* v = reinterpret_cast<const fp_t*>(f + s);
  for (int i = 0; i < 12; ++i) {
    uint8_t c[48];
    fp_to_be48(c, fp_from_mont(v[i]));
    for (int k = 0; k < 48; ++k) out_f576[576ull * s + 48 * i + k] = c[k];
  }
}

// 48-byte compressed pubkeys -> device cache entries (trusted, no subgroup check:
// state-transition/src/cache/pubkeyCache.ts:75 decompresses without validation)
__global__ void k_cache_put_compressed(const uint8_t* __restrict__ keys, uint32_t n, g1_aff* __restrict__ cache,
                                       int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[48];
  for (int k = 0; k < 48; ++k) b[k] = keys[48ull * i + k];
  g1_aff a;
  bool inf;
  int rc = g1_decompress(&a, &inf, b);
  if (rc == BGV_OK && inf) rc = BGV_PK_IS_INFINITY;
  if (rc == BGV_OK) cache[i] = a;
  status[i] = rc;
}

__global__ void k_cache_put_uncompressed(const uint8_t* __restrict__ keys, uint32_t n, g1_aff* __restrict__ cache,
                                         int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[96];
  for (int k = 0; k < 96; ++k) b[k] = keys[96ull * i + k];
  g1_aff a;
  bool inf;
  int rc = g1_deserialize(&a, &inf, b);
  if (rc == BGV_OK && inf) rc = BGV_PK_IS_INFINITY;
  if (rc == BGV_OK) cache[i] = a;
  status[i] = rc;
}


// ---------------------------------------------------------------------------
// Key generation and signing (bench / test data on the device; not on the
// verify path).  Secret keys are 32-byte big-endian scalars < r
// (SecretKey.fromBytes, state-transition/src/util/interop.ts:19-22).
// ---------------------------------------------------------------------------
__device__ static void sk_words(const uint8_t* be32, uint32_t k[8]) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = be32 + 28 - 4 * i;
    k[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

__global__ void k_keygen(const uint8_t* __restrict__ sks, uint32_t n, g1_aff* __restrict__ cache,
                         uint8_t* __restrict__ out48) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  sk_words(sks + 32ull * i, k);
  g1_aff a;
  const bool fin = jac_to_aff(&a, jac_mul_u256(jac_from_aff(g1_generator()), k));
  if (cache) cache[i] = a;
  if (out48) {
    uint8_t b[48];
    g1_compress(b, a, !fin);
    for (int q = 0; q < 48; ++q) out48[48ull * i + q] = b[q];
  }
}

__global__ void k_sign(const uint8_t* __restrict__ sks, const uint8_t* __restrict__ msgs, uint32_t n,
                       uint8_t* __restrict__ out96) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  sk_words(sks + 32ull * i, k);
  uint8_t m[32];
  for (int q = 0; q < 32; ++q) m[q] = msgs[32ull * i + q];
  g2_aff a;
  const bool fin = jac_to_aff(&a, jac_mul_u256(hash_to_g2(m, 32), k));
  uint8_t b[96];
  g2_compress(b, a, !fin);
  for (int q = 0; q < 96; ++q) out96[96ull * i + q] = b[q];
}

}  // extern "C"

size_t bgv_slot_bytes() { return 2 * sizeof(g2_jac) + sizeof(g1_jac) + sizeof(fp12_t) + sizeof(g1_jac) + 2 * sizeof(int32_t); }
// the per-slot signature pairs (fsig) serve only calls of at most BGV_PREP_WIDE_MAX slots
// (bgv_sig_pairs), so they get that many entries, not one per slot of the capacity
static size_t fsig_slots(uint32_t cap_slots) { return std::min<size_t>(cap_slots, BGV_PREP_WIDE_MAX + 64); }
size_t bgv_slot_mem_bytes(uint32_t cap_slots) {
  return bgv_slot_bytes() * (size_t)cap_slots + sizeof(fp12_t) * fsig_slots(cap_slots);
}
size_t bgv_group_bytes() { return sizeof(g2_jac) + 4 * sizeof(fp12_t) + sizeof(g1_jac) + sizeof(int32_t); }
size_t bgv_cache_entry_bytes() { return sizeof(g1_aff); }

void bgv_carve(bgv_dev_batch* b, void* slot_mem, uint32_t cap_slots, void* group_mem, uint32_t cap_groups) {
  uint8_t* p = static_cast<uint8_t*>(slot_mem);
  b->rsig = reinterpret_cast<g2_jac*>(p);
  p += sizeof(g2_jac) * (size_t)cap_slots;
  b->h = reinterpret_cast<g2_jac*>(p);
  p += sizeof(g2_jac) * (size_t)cap_slots;
  b->rpk = reinterpret_cast<g1_jac*>(p);
  p += sizeof(g1_jac) * (size_t)cap_slots;
  b->f = reinterpret_cast<fp12_t*>(p);
  p += sizeof(fp12_t) * (size_t)cap_slots;
  b->fsig = reinterpret_cast<fp12_t*>(p);
  p += sizeof(fp12_t) * fsig_slots(cap_slots);
  b->pk_agg = reinterpret_cast<g1_jac*>(p);
  p += sizeof(g1_jac) * (size_t)cap_slots;
  b->sig_status = reinterpret_cast<int32_t*>(p);
  p += sizeof(int32_t) * (size_t)cap_slots;
  b->pk_status = reinterpret_cast<int32_t*>(p);
  uint8_t* q = static_cast<uint8_t*>(group_mem);
  b->gsum = reinterpret_cast<g2_jac*>(q);
  q += sizeof(g2_jac) * (size_t)cap_groups;
  b->gpair = reinterpret_cast<fp12_t*>(q);
  q += sizeof(fp12_t) * (size_t)cap_groups;
  b->gprod = reinterpret_cast<fp12_t*>(q);
  q += sizeof(fp12_t) * (size_t)cap_groups;
  b->gu = reinterpret_cast<fp12_t*>(q);
  q += sizeof(fp12_t) * (size_t)cap_groups;
  b->gpkp = reinterpret_cast<fp12_t*>(q);
  q += sizeof(fp12_t) * (size_t)cap_groups;
  b->gpk = reinterpret_cast<g1_jac*>(q);
  q += sizeof(g1_jac) * (size_t)cap_groups;
  b->verdict = reinterpret_cast<int32_t*>(q);
}

hipError_t bgv_launch_cache_put(const uint8_t* keys, uint32_t n, int fmt, bgv_cache_entry* cache, int32_t* status,
                                hipStream_t st) {
  if (n == 0) return hipSuccess;
  g1_aff* c = reinterpret_cast<g1_aff*>(cache);
  if (fmt == 48)
    hipLaunchKernelGGL(k_cache_put_compressed, dim3(nblk(n, 64)), dim3(64), 0, st, keys, n, c, status);
  else
    hipLaunchKernelGGL(k_cache_put_uncompressed, dim3(nblk(n, 64)), dim3(64), 0, st, keys, n, c, status);
  return hipGetLastError();
}

hipError_t bgv_launch_debug_out(const bgv_dev_batch& b, uint8_t* out_h192, uint8_t* out_f576, hipStream_t st) {
  hipLaunchKernelGGL(k_debug_out, dim3(nblk(b.nslots, 64)), dim3(64), 0, st, b.slots, b.nslots, b.h, b.f, out_h192,
                     out_f576);
  return hipGetLastError();
}

hipError_t bgv_launch_hash(const uint8_t* msgs, const uint32_t* offs, const uint32_t* lens, uint32_t n,
                           uint8_t* out192, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hash_msgs, dim3(nblk(n, 64)), dim3(64), 0, st, msgs, offs, lens, n, out192);
  return hipGetLastError();
}

hipError_t bgv_launch_pk_validate(const uint8_t* keys48, uint32_t n, int32_t* status, uint8_t* out96,
                                  hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pk_validate, dim3(nblk(n, 64)), dim3(64), 0, st, keys48, n, status, out96);
  return hipGetLastError();
}

hipError_t bgv_launch_sig_aggregate(const uint8_t* sigs96, const uint32_t* lens, uint32_t n, const uint32_t* first,
                                    const uint32_t* count, uint32_t naggs, void* pts, int32_t* status,
                                    uint8_t* out96, hipStream_t st) {
  if (n) {
    hipLaunchKernelGGL(k_sig_decode, dim3(nblk(n, 64)), dim3(64), 0, st, sigs96, lens, n,
                       reinterpret_cast<g2_jac*>(pts), status);
  }
  if (naggs) {
    hipLaunchKernelGGL(k_sig_sum, dim3(naggs), dim3(64), BGV_WAVE * sizeof(g2_jac), st, first, count,
                       reinterpret_cast<const g2_jac*>(pts), out96);
  }
  return hipGetLastError();
}
size_t bgv_g2_point_bytes() { return sizeof(g2_jac); }
size_t bgv_g1_point_bytes() { return sizeof(g1_jac); }
hipError_t bgv_launch_keygen(const uint8_t* sks, uint32_t n, bgv_cache_entry* cache, uint8_t* out48, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_keygen, dim3(nblk(n, 64)), dim3(64), 0, st, sks, n, reinterpret_cast<g1_aff*>(cache), out48);
  return hipGetLastError();
}

hipError_t bgv_launch_sign(const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign, dim3(nblk(n, 64)), dim3(64), 0, st, sks, msgs, n, out96);
  return hipGetLastError();
}
