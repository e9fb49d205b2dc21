// Device engine of the generated round programs (bgv_tmiller.h / bgv_tcurve.h) on a whole
// 64-lane block: instruction c of a round (the program's lane c < 16) runs on four lanes
// c + 16 q, each computing part q of its products (tmp_lane_part: at most one product and
// one reduction) into LDS; after a barrier lane q = 0 sums the parts into the output slot.
// Per round a lane waits one product + one reduction instead of T products + one reduction
// on a 16-lane team.  The engine is one wavefront and synchronizes on its own
// (bgv_wave_sync), so a block may run other work on its other waves (k_miller_wide).
// Host emulation: bgv_tmiller.h tmp_host_wide().
#pragma once
#include "bgv_team_dev.h"
#include "bgv_tmiller.h"

struct tr_wide_engine {
  const uint8_t* prog;
  fp_t* S;     // the program's slots
  fp_t* P;     // 64 part slots
  int c, q;    // instruction (lane & 15) and part (lane >> 4)
  bool bad;
  __device__ void run(int off) {
    int pos = off;
    const int nr = prog[pos++];
    for (int r = 0; r < nr; ++r) {
      const int T = prog[pos], M = prog[pos + 1];
      pos += 2;
      const int rb = tmp_rec_bytes(T, M);
      const uint8_t* rec = prog + pos + c * rb;
      P[q * BGV_TEAM + c] = tmp_lane_part(S, rec, T, M, q);
      bgv_wave_sync();
      if (q == 0) S[rec[0]] = tm_sum4(P[c], P[BGV_TEAM + c], P[2 * BGV_TEAM + c], P[3 * BGV_TEAM + c]);
      bgv_wave_sync();
      pos += BGV_TEAM * rb;
    }
  }
};
