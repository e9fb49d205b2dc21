// Device engine of the generated round programs (bgv_tmiller.h / bgv_tcurve.h) on a whole
// 64-lane block: instruction c of a round (the program's lane c < 16) runs on the four lanes
// 4c + q of a DPP quad, each computing part q of its products (tmp_lane_part: at most one
// product and one reduction); two quad DPP adds per limb leave the parts' sum in the quad and
// lane q = 0 writes it to the output slot -- one LDS write and one wave sync per round.
// Per round a lane waits one product + one reduction instead of T products + one reduction
// on a 16-lane team.  The engine is one wavefront and synchronizes on its own
// (bgv_wave_sync), so a block may run other work on its other waves (k_miller_wide).
// Host emulation: bgv_tmiller.h tmp_host_wide().
#pragma once
#include "bgv_team_dev.h"
#include "bgv_tmiller.h"

__device__ __forceinline__ int tr_wide_lane_c(int lane) { return lane >> 2; }
__device__ __forceinline__ int tr_wide_lane_q(int lane) { return lane & 3; }

struct tr_wide_engine {
  const uint8_t* prog;
  fp_t* S;     // the program's slots
  fp_t* P;     // 64 part slots
  int c, q;    // instruction (lane >> 2) and part (lane & 3): tr_wide_lane_c / _q
  bool bad;
  __device__ void run(int off) {
    int pos = off;
    const int nr = prog[pos++];
    for (int r = 0; r < nr; ++r) {
      const int T = prog[pos], M = prog[pos + 1];
      pos += 2;
      const int rb = tmp_rec_bytes(T, M);
      const uint8_t* rec = prog + pos + c * rb;
      const fp_t part = tmp_lane_part(S, rec, T, M, q);
      fp_t sum;  // the quad's four parts, the same integer sum as tm_sum4's
      BGV_UNROLL for (int l = 0; l < NL; ++l) {
        uint32_t v = part.v[l];
        v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
        sum.v[l] = v;
      }
      // no slot is read and written in one round (the generators check it), so the output
      // needs no barrier before it; the next round's reads wait for it
      if (q == 0) S[rec[0]] = tm_norm4(sum);
      bgv_wave_sync();
      pos += BGV_TEAM * rb;
    }
  }
};
