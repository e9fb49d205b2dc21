// The bulk Miller loops of a verify call (gfx950), in two phases and in a unit of its own so
// that each phase gets its own register budget (BGV_WPE_LINES / BGV_WPE_FACC waves per SIMD).
// The per-set pairs of blst's randomized batch equation (maybeBatch.ts:18-25 ->
// verifyMultipleAggregateSignatures):  f_i = MillerLoop(r_i pk_i, H(m_i)), and one pair per
// device group g_g = MillerLoop(-G1, S_g).
//
//   k_lines  one lane per twist point Q (each distinct signing root's H, each group's S_g):
//            walks T over the loop and writes the 68 P-free line records (bls_pairing.h
//            lz_pline_dbl / lz_pline_add) to HBM.  Live set: T and one step's temporaries.
//   k_facc   one lane per pair: f <- f^2 * line(P) over the records of its Q.  The records are
//            staged through LDS: each step's record is read from LDS and the next one's DMA
//            (global_load_lds_dwordx4, no VGPR destination) issued right after, so it lands
//            during the line product and the next squaring; P's three constants also wait in
//            LDS between the steps' scalings.  Live set: f and the step's temporaries.
//
// One loop of the single-pass k_miller kept f (168 u32), T (84) and P (42) live across every
// out-of-line product: 2.7 KB of scratch per lane and 230x its algorithmic HBM bytes
// (DESIGN.md section 2).  Split, each phase's live set is smaller.
//
// Records: quad q (words 4q..4q+3) of record k (step k of the loop) of pair p is the 16 bytes at
// lines[((k * 21 + q) * cap + p) * 4] (cap = the buffer's pairs): a wave's 64 lanes write and
// read 1 KB contiguously, one dwordx4 instruction per quad.
// -DBGV_BULK_MILLER_INLINE inlines this unit's Montgomery products (bls_lazy.h
// BGV_LAZY_INLINE_MUL).  An out-of-line product costs 2,850 SIMD cycles per wave at one wave per
// SIMD against 2,080 inlined in a tight loop (tools/ubench_prod.hip, profiles/r04/ubench_prod.jsonl),
// but inlined here the loop bodies grow to ~52k instructions (~400 KB, past the 64 KB
// instruction cache) and the Miller stage measured 11.6-11.7 ms against 10.8-10.9 ms with calls
// (profiles/r04/inline_ab/): not the default.
#ifdef BGV_BULK_MILLER_INLINE
#define BGV_LAZY_INLINE_MUL 1
#endif
// (Hand-scheduled exact-clobber product subroutines measured equal at the kernel level,
// profiles/r04/asm_ab: k_miller 10.69-10.76 vs 10.71-10.86 ms; kept in tools/experimental/.)
// Fp2 products with deferred reduction (bls_wide.h); k_lines and k_facc run 64-thread blocks,
// as the products' per-lane LDS operand slot requires
#ifndef BGV_LZ2_CLASSIC
#define BGV_LZ2_WIDE 1
#define BGV_LZ2_WIDE_STRICT 1  // no silent fallback to the fully reduced product
#endif
#include "bgv_device.h"

#ifndef BGV_WPE_LINES
#define BGV_WPE_LINES 1
#endif
#ifndef BGV_WPE_FACC
#define BGV_WPE_FACC 1
#endif
#define BGV_KATTR_LINES __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE_LINES, BGV_WPE_LINES)))
#define BGV_KATTR_FACC __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BGV_WPE_FACC, BGV_WPE_FACC)))

static_assert(sizeof(lz_pline_d) == 4 * BGV_LINE_WORDS, "line record layout");
static_assert(sizeof(lz_pline_a) == 4 * BGV_LINE_WORDS, "line record layout");

static __device__ const g1_jac kNegG1JacB = {{BGV_G1X}, {BGV_NEG_G1Y}, {BGV_ONE}};

extern "C" {

// Lanes [0, nq): the set pairs' twist points -- slot uniq[u] (b.uniq: the first slot of each
// distinct signing root) or slot u; lanes [nq, nq + ngroups): group g's S_g at record index
// nslots + g.  Padding slots (no H) and infinite S_g write nothing (k_facc outputs 1 there).
__global__ void BGV_KATTR_LINES k_lines(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                        const g2_jac* __restrict__ h, const uint32_t* __restrict__ uniq,
                                        uint32_t nq, uint32_t ngroups, const g2_jac* __restrict__ gsum,
                                        uint32_t* __restrict__ lines, uint32_t cap) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t p;
  const g2_jac* q;
  if (u < nq) {
    p = uniq ? uniq[u] : u;
    if (slots[p].flags & BGV_SLOT_PAD) return;
    q = h + p;
  } else if (u - nq < ngroups) {
    p = nslots + (u - nq);
    q = gsum + (u - nq);
    if (jac_is_inf(*q)) return;
  } else {
    return;
  }
  uint32_t* base = lines + 4 * (size_t)p;
  miller_lines_walk(q, [&](int k, const auto& rec) {
    const uint4* w = reinterpret_cast<const uint4*>(&rec);
    uint4* dst = reinterpret_cast<uint4*>(base + (size_t)k * BGV_LINE_QUADS * 4 * cap);
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d) dst[(size_t)d * cap] = w[d];
  });
}

// Lanes [0, nslots): f_i over the records of the slot's signing root (slots[s].hsrc), 1 for a
// slot that takes no part; lanes [nslots, nslots + ngroups): g_g = MillerLoop(-G1, S_g) (1 for
// an infinite S_g); lanes [nslots + ngroups, nslots + ngroups + npk): a uniform group's
// (BGV_GROUP_UNIFORM) one set pair MillerLoop(gpk_g, H of its root) into gpkp_g.  The slots of
// a uniform group take no lane of their own (their f_i stay unwritten: the closing multiplies
// gpkp instead; a retry test inside such a group pairs its own pubkey sum, bgv_launch_gpairs).
__global__ void BGV_KATTR_FACC k_facc(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                      const g1_jac* __restrict__ rpk, const int32_t* __restrict__ sig_status,
                                      const int32_t* __restrict__ pk_status, const uint32_t* __restrict__ lines,
                                      uint32_t cap, fp12_t* __restrict__ f, uint32_t ngroups,
                                      const g2_jac* __restrict__ gsum, fp12_t* __restrict__ gpair,
                                      const bgv_dgroup* __restrict__ groups, uint32_t npk,
                                      const g1_jac* __restrict__ gpk, fp12_t* __restrict__ gpkp) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  bool live;
  uint32_t lp;
  const g1_jac* P;
  fp12_t* out;
  if (s < nslots) {
    const bgv_dslot& d = slots[s];
    if (groups && !(d.flags & BGV_SLOT_PAD) && (groups[d.group].flags & BGV_GROUP_UNIFORM)) return;
    live = slot_live(d, sig_status[s], pk_status[s]);
    lp = d.hsrc;
    P = rpk + s;
    out = f + s;
  } else if (s - nslots < ngroups) {
    const uint32_t g = s - nslots;
    live = !jac_is_inf(gsum[g]);
    lp = nslots + g;
    P = &kNegG1JacB;
    out = gpair + g;
  } else if (s - nslots - ngroups < npk) {
    const uint32_t g = s - nslots - ngroups;
    const bgv_dgroup G = groups[g];
    if (!(G.flags & BGV_GROUP_UNIFORM)) return;
    live = !jac_is_inf(gpk[g]);
    lp = slots[G.first_slot].hsrc;
    P = gpk + g;
    out = gpkp + g;
  } else {
    return;
  }
  if (!live) {
    *out = fp12_one();
    return;
  }
#if BGV_WPE_FACC >= 2
  // Two waves per SIMD (A/B: BGV_WPE_FACC=2): 8 waves per CU leave 20 KB of LDS each, so no
  // staging -- the records are read straight into registers (the other wave hides the loads)
  // and P's constants stay in registers; the LDS holds only the products' operand slot.
  {
    const uint32_t* base = lines + 4 * (size_t)lp;
    const miller_p P0 = miller_p_make(*P);
    *out = miller_facc_walk_staged([&](int k, uint32_t z, auto* r) {
      const uint4* src = reinterpret_cast<const uint4*>(base + (size_t)(k + z) * BGV_LINE_QUADS * 4 * cap);
      uint4* w = reinterpret_cast<uint4*>(r);
      BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d) w[d] = src[(size_t)d * cap];
    }, [&](int which, uint32_t z) {
      const fp_t& c = which == 0 ? P0.xn : (which == 1 ? P0.yp : P0.zp3);
      lzr v;
      BGV_UNROLL for (int i = 0; i < NL; ++i) v.v[i] = c.v[i] + z;
      return v;
    });
    return;
  }
#endif
  // this wave's LDS: the staged record [quad][lane] and P's constants [word][lane]
  __shared__ uint4 rec_lds[BGV_LINE_QUADS][64];
  __shared__ uint32_t p_lds[3 * NL][64];
  const int lane = threadIdx.x;
  const uint32_t* base = lines + 4 * (size_t)lp;
  auto dma = [&](int k) {  // record k of this lane's pair -> rec_lds (lane-linear, 16 B per lane)
    const uint32_t* src = base + (size_t)k * BGV_LINE_QUADS * 4 * cap;
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d)
      __builtin_amdgcn_global_load_lds(src + (size_t)d * 4 * cap, &rec_lds[d][0], 16, 0, 0);
  };
  dma(0);
  const miller_p P0 = miller_p_make(*P);
  BGV_UNROLL for (int i = 0; i < NL; ++i) {
    p_lds[i][lane] = P0.xn.v[i];
    p_lds[NL + i][lane] = P0.yp.v[i];
    p_lds[2 * NL + i][lane] = P0.zp3.v[i];
  }
  *out = miller_facc_walk_staged([&](int k, uint32_t z, auto* r) {
    // record k landed (its DMA was issued one step ago): read it, then stage record k + 1
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    uint4* w = reinterpret_cast<uint4*>(r);
    BGV_UNROLL for (int d = 0; d < BGV_LINE_QUADS; ++d) w[d] = rec_lds[d][lane + z];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the buffer is free again
    if (k + 1 < BGV_MILLER_STEPS) dma(k + 1);
  }, [&](int which, uint32_t z) {  // P's constants from LDS: 0 xn, 1 yp, 2 zp3
    lzr v;
    BGV_UNROLL for (int i = 0; i < NL; ++i) v.v[i] = p_lds[which * NL + i][lane + z];
    return v;
  });
}

}  // extern "C"

// line records a batch's bulk Miller launch writes: one per set pair's twist point (slot index
// space) and one per group; 0 when the batch takes the latency path or has no slots
uint32_t bgv_lines_pairs(const bgv_dev_batch& b) {
  if (b.nslots == 0 || bgv_use_latency(b, b.nslots + b.ngroups) || bgv_single_pass_miller()) return 0;
  return b.nslots + b.ngroups;
}
size_t bgv_line_record_bytes() { return (size_t)BGV_MILLER_STEPS * BGV_LINE_WORDS * 4; }

// the set pairs [0, nslots), the group pairs [nslots, nslots + ngroups) and, with uniform
// groups (b.uniform), their pubkey-sum pairs of a bulk batch; ngroups = 0 when the group pairs
// run on teams instead (bgv_launch_miller)
hipError_t bgv_launch_miller_bulk(const bgv_dev_batch& b, uint32_t ngroups, hipStream_t st) {
  if (!b.lines || b.lines_cap < b.nslots + ngroups) return hipErrorInvalidValue;
  const uint32_t nq = b.uniq ? b.nuniq : b.nslots;
  const uint32_t npk = b.uniform ? b.ngroups : 0u;
  if (nq + ngroups)
    hipLaunchKernelGGL(k_lines, dim3(nblk(nq + ngroups, 64)), dim3(64), 0, st, b.slots, b.nslots, b.h, b.uniq, nq,
                       ngroups, b.gsum, b.lines, b.lines_cap);
  hipLaunchKernelGGL(k_facc, dim3(nblk(b.nslots + ngroups + npk, 64)), dim3(64), 0, st, b.slots, b.nslots, b.rpk,
                     b.sig_status, b.pk_status, b.lines, b.lines_cap, b.f, ngroups, b.gsum, b.gpair,
                     b.uniform ? b.groups : nullptr, npk, static_cast<const g1_jac*>(b.gpk), b.gpkp);
  return hipGetLastError();
}
