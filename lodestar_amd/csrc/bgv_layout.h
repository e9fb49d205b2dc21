// Device-side record layouts shared by the HIP kernels (bgv_kernels.hip) and
// the host orchestration (bgv_api.cpp).  Plain C structs, no HIP types.
//
// A verify call is laid out as SLOTS: one lane per signature set.  Sets are
// packed into device GROUPS of at most 64 slots that never straddle a 64-slot
// (one wavefront) boundary, so a group's product/sum reduction is wave-local.
// Padding slots (BGV_SLOT_PAD) are identity elements.
#pragma once
#include <stdint.h>

#define BGV_WAVE 64

enum {
  BGV_SLOT_PAD = 1u,        // empty lane
  BGV_SLOT_PK_CACHED = 2u,  // pubkeys are validator indices into the device cache
  BGV_SLOT_PK_BYTES = 4u,   // pubkeys are 96-byte uncompressed records uploaded with the call
};

// Per-slot input record (160 B, 16-B aligned).
struct bgv_dslot {
  uint32_t flags;
  uint32_t n_pk;    // pubkeys to aggregate (>= 1)
  uint32_t pk_off;  // first index in the index array, or first 96-B record
  uint32_t sig_len; // length of the signature bytes as received (96 is the only valid size)
  uint64_t scalar;  // nonzero 64-bit batch randomizer r
  uint32_t group;   // device group id
  uint32_t hsrc;    // slot whose H(msg) this slot uses: the first slot of its call with the same
                    // signing root (its own index for that first slot and for pads)
  uint8_t msg[32];  // signing root
  uint8_t sig[96];  // compressed G2 signature (untrusted wire bytes)
};

// Per-slot status codes written by the kernels (BLST numbering, see blsgpu.h)
enum {
  BGV_ST_OK = 0,
  BGV_ST_INFINITY = 100,  // infinity signature / pubkey: valid encoding, skipped in the product
};

// A device group: the slots first_slot + k, k < n_slots, whose bit k of mask is set (retry
// rounds test job subsets that are not contiguous: bgv_api.cpp pattern tests).  ref1 != 0
// names the first-pass group (index ref1 - 1 of the batch) whose pairing value this group's
// is compared with: the closing then also reports whether the two values agree, i.e. whether
// the rest of that group (its complement) passes (verdict bit 1).
// flags & BGV_GROUP_WEIGHTED (a retry round's weighted test of a failing first-pass group
// ref1 - 1, bgv_api.cpp): slot k of the group enters with weight k + 1 -- the closing multiplies
// prod_k f_k^(k+1) * e(-G1, sum_k (k+1) r_k sig_k) (k_gsum, k_final12) -- and reports the weight
// w in 1..n_slots with (pairing value of ref1 - 1)^w == this group's value, or 0, in verdict
// bits 8..15: with exactly one invalid slot k that is k + 1.
struct bgv_dgroup {
  uint32_t first_slot;  // multiple of BGV_WAVE
  uint32_t n_slots;     // 1..64
  uint64_t mask;
  uint32_t ref1;
  uint32_t flags;
};
#define BGV_ALL_SLOTS (~0ull)
#define BGV_GROUP_WEIGHTED 1u
// a first-pass group shared by several batchable jobs (only such a group is retried per job,
// so only its failure takes the first pass's weighted test, bgv_launch_fpw_list)
#define BGV_GROUP_SHARED 2u
