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
struct bgv_dgroup {
  uint32_t first_slot;  // multiple of BGV_WAVE
  uint32_t n_slots;     // 1..64
  uint64_t mask;
  uint32_t ref1;
  uint32_t flags;
};
#define BGV_ALL_SLOTS (~0ull)
// flags: a first-pass group of a bulk batch whose sets all share one signing root (slot
// first_slot's hsrc) and whose batchable jobs lie inside it (a non-batchable job's groups are
// never retried).  prod_i e(r_i pk_i, H) = e(sum_i r_i pk_i, H),
// so the group's set pairs are ONE Miller loop over its pubkey sum (k_gsum -> gpk, k_facc ->
// gpkp) and its slots take none; a retry test inside such a group (flagged the same,
// bgv_api.cpp call_build_parts) pairs the sum of its own slots' r_i pk_i the same way
#define BGV_GROUP_UNIFORM 4u
// flags: a retry test over a whole failing uniform group with slot k weighted by k + 1
// (bgv_api.cpp PatternUnit kind 2): k_gsum forms sum (k+1) r_k sig_k and sum (k+1) r_k pk_k,
// and k_final12 reports in verdict bits 8..15 the w <= n_slots with V^w = W against the
// first-pass value V of group ref1 - 1 (0: none) -- the slot w - 1 when exactly one is invalid
#define BGV_GROUP_WEIGHTED 8u
