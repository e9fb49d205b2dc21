// The per-slot Miller-loop kernel, included by bgv_kernels.hip (default build) or by
// bgv_kernels_miller.hip (-DBGV_MILLER_SPLIT: its own translation unit, Fp products inlined).
// Expects BGV_KATTR and the extern "C" block of the including file.
#pragma once

// f_i = MillerLoop(r pk, H(m)) * MillerLoop(-r G1, sig); 1 for slots that do not
// take part (padding, failed decode/aggregation).  An infinity signature keeps
// its pubkey pair and drops the signature pair, as blst's accumulator does.
__global__ void BGV_KATTR k_miller(const bgv_dslot* __restrict__ slots, uint32_t nslots,
                                   const g1_aff* __restrict__ rpk, const g2_jac* __restrict__ h,
                                   const g1_aff* __restrict__ rg, const g2_aff* __restrict__ sig,
                                   const int32_t* __restrict__ sig_status, const int32_t* __restrict__ pk_status,
                                   fp12_t* __restrict__ f) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  const int32_t ss = sig_status[s];
  const bool live = !(slots[s].flags & BGV_SLOT_PAD) && (ss == BGV_ST_OK || ss == BGV_ST_INFINITY) &&
                    pk_status[s] == BGV_ST_OK;
  fp12_t r = fp12_one();
  if (live) r = miller_loop2(rpk[s], h[s], rg[s], sig[s], ss == BGV_ST_OK);
  f[s] = r;
}
