// Internal interface between the HIP kernels (bgv_kernels.hip) and the host
// orchestration (bgv_api.cpp).  Device pointers only; no torch types.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "bgv_layout.h"

struct fp12_t;
template <class F>
struct jac_t;
template <class F>
struct aff_t;
struct fp_t;
struct fp2_t;

// opaque cache entry (affine G1, Montgomery form)
struct bgv_cache_entry;

// kernel path of a batch (the public values are in include/blsgpu.h)
#define BGV_PATH_AUTO 0
#ifndef BGV_PATH_BULK
#define BGV_PATH_BULK 1
#define BGV_PATH_LATENCY 2
#endif

struct bgv_dev_batch {
  uint32_t nslots, ngroups;
  uint32_t max_npk;  // largest n_pk of any slot (k_pk_agg runs only when a set reaches BGV_PK_TREE_MIN)
  bool uniform;      // some group carries BGV_GROUP_UNIFORM (bulk first passes only)
  int path;          // BGV_PATH_AUTO by size, BGV_PATH_BULK / BGV_PATH_LATENCY forced (bgv_debug_prepare)
  // slots whose H(msg) the bulk k_prep computes (the first slot of each distinct signing root of
  // a call); the other slots read H at their hsrc.  Null: every slot hashes its own message.
  const uint32_t* uniq;
  uint32_t nuniq;
  const bgv_dslot* slots;
  const bgv_dgroup* groups;
  const uint32_t* pk_idx;
  const bgv_cache_entry* cache_opaque;
  const uint8_t* pk_bytes;
  // carved per-slot / per-group scratch
  jac_t<fp2_t>* rsig;  // r_i * sig_i (Jacobian), summed per group by k_final
  jac_t<fp2_t>* h;     // H(m_i), Jacobian
  jac_t<fp_t>* rpk;    // r_i * aggregated pubkey, Jacobian
  fp12_t* f;           // per-slot Miller loop value e(r_i pk_i, H(m_i))
  fp12_t* fsig;        // smallest calls' first pass: per-slot e(-G1, r_i sig_i) (bgv_sig_pairs)
  jac_t<fp_t>* pk_agg;  // wavefront-tree sum of a many-key set's cached pubkeys (k_pk_agg)
  int32_t* sig_status;
  int32_t* pk_status;
  jac_t<fp2_t>* gsum;  // per group: sum of its r_i sig_i
  fp12_t* gpair;       // per group: MillerLoop(-G1, gsum)
  jac_t<fp_t>* gpk;    // per uniform group (BGV_GROUP_UNIFORM): sum of its live r_i pk_i
  fp12_t* gpkp;        // per uniform group: MillerLoop(gpk, H of the group's root)
  // retry rounds with uniform groups: the npk tests flagged BGV_GROUP_UNIFORM (indices into
  // groups), whose pubkey-sum pairs bgv_launch_gpairs runs
  const uint32_t* upk;
  uint32_t npk;
  bool weighted;  // some of the round's tests are BGV_GROUP_WEIGHTED (k_gsum_w)
  fp12_t* gprod;       // per group: its Miller-loop product (before the final exponentiation)
  fp12_t* gu;          // per group: u = gprod^((p^2+1) 3 (p^4-p^2+1)/r); pairing value conj(u)/u
  // retry rounds with pattern tests: the first pass's u values (a copy of its gu), indexed by
  // bgv_dgroup.ref1 - 1; null otherwise
  const fp12_t* gu1;
  int32_t* verdict;    // per group: bit 0 = the group passes, bit 1 = its pairing value equals ref's
  // the bulk Miller loop's line records (bgv_k_miller_bulk.hip): lines_cap pairs, SoA; null
  // unless the host reserved them (bgv_lines_pairs)
  uint32_t* lines;
  uint32_t lines_cap;
#ifdef BGV_KERNEL_SIDE
  const aff_t<fp_t>* cache_ptr() const { return reinterpret_cast<const aff_t<fp_t>*>(cache_opaque); }
#endif
};

// kernels of one verify launch, in order (names for per-kernel timing)
#define BGV_NKERNELS 3
#define BGV_NSETKERNELS 2  // the first BGV_NSETKERNELS run once per call (bgv_launch_sets)
static const char* const BGV_KERNEL_NAMES[BGV_NKERNELS] = {"k_prep", "k_miller", "k_final"};
struct bgv_streams {
  hipStream_t main;
  hipEvent_t* kev;  // 2 * BGV_NKERNELS events (start/end per kernel) or nullptr
};
hipError_t bgv_launch_sets(const bgv_dev_batch& b, const bgv_streams& s);  // prep + miller
// The smallest calls' first pass pairs every signature with -G1 on its own (e(-G1, r_i sig_i)
// per slot, beside e(r_i pk_i, H(m_i))) instead of summing a group's r_i sig_i first (k_gsum)
// and pairing the sum: one more Miller loop per set, run in parallel, for one serial kernel
// less.  Retry rounds keep the group sums.
bool bgv_sig_pairs(const bgv_dev_batch& b);
hipError_t bgv_launch_prep(const bgv_dev_batch& b, const bgv_streams& s);
hipError_t bgv_launch_prep_bulk(const bgv_dev_batch& b, const bgv_streams& s, bool tree);  // bgv_k_prep_bulk.hip
hipError_t bgv_launch_prep_wave(const bgv_dev_batch& b, hipStream_t st);  // bgv_k_prep_wave.hip
hipError_t bgv_launch_miller(const bgv_dev_batch& b, const bgv_streams& s);
// bulk path: k_lines + k_facc over the set pairs and the first ngroups group pairs
hipError_t bgv_launch_miller_bulk(const bgv_dev_batch& b, uint32_t ngroups, hipStream_t st);
uint32_t bgv_lines_pairs(const bgv_dev_batch& b);  // line records the batch needs (0: latency path)
bool bgv_single_pass_miller();                     // BGV_MILLER_1PASS: k_miller instead (A/B)
size_t bgv_line_record_bytes();                    // bytes of one pair's 68 records
hipError_t bgv_launch_groups(const bgv_dev_batch& b, const bgv_streams& s, bool pairs);
// bgv_launch_groups closes with k_final12 iff
// nslots + ngroups exceeds this (else k_final_fold)
uint32_t bgv_fold_pairs_max();
hipError_t bgv_launch_gpairs(const bgv_dev_batch& b, hipStream_t st);  // retry parts: k_gsum + k_gpair
size_t bgv_slot_bytes();
size_t bgv_slot_mem_bytes(uint32_t cap_slots);  // the per-slot arrays of an Exec of cap_slots slots
size_t bgv_group_bytes();
size_t bgv_cache_entry_bytes();
void bgv_carve(bgv_dev_batch* b, void* slot_mem, uint32_t cap_slots, void* group_mem, uint32_t cap_groups);
hipError_t bgv_launch_cache_put(const uint8_t* keys, uint32_t n, int fmt, bgv_cache_entry* cache, int32_t* status,
                                hipStream_t st);
hipError_t bgv_launch_aggregate(const bgv_dslot* slot, const uint32_t* idx, uint32_t n, const bgv_cache_entry* cache,
                                void* agg, uint8_t* out96, hipStream_t st);
size_t bgv_g1_point_bytes();
hipError_t bgv_launch_debug_out(const bgv_dev_batch& b, uint8_t* out_h192, uint8_t* out_f576, hipStream_t st);
hipError_t bgv_launch_hash(const uint8_t* msgs, const uint32_t* offs, const uint32_t* lens, uint32_t n,
                           uint8_t* out192, hipStream_t st);
hipError_t bgv_launch_keygen(const uint8_t* sks, uint32_t n, bgv_cache_entry* cache, uint8_t* out48, hipStream_t st);
hipError_t bgv_launch_sign(const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96, hipStream_t st);
hipError_t bgv_launch_pk_validate(const uint8_t* keys48, uint32_t n, int32_t* status, uint8_t* out96,
                                  hipStream_t st);
hipError_t bgv_launch_sig_aggregate(const uint8_t* sigs96, const uint32_t* lens, uint32_t n, const uint32_t* first,
                                    const uint32_t* count, uint32_t naggs, void* pts, int32_t* status,
                                    uint8_t* out96, hipStream_t st);
size_t bgv_g2_point_bytes();
size_t bgv_fp12_bytes();
hipError_t bgv_launch_fp12_bytes(const fp12_t* in, uint32_t n, uint8_t* out576, hipStream_t st);  // parity hooks
hipError_t bgv_launch_partial(const bgv_dev_batch& b, uint32_t g0, uint32_t ng, void* scratch, uint8_t* out576,
                              hipStream_t st);
hipError_t bgv_launch_final_verify(const uint8_t* in, uint32_t n, void* vals, void* one, const bgv_dgroup* group,
                                   int32_t* status, int32_t* verdict, hipStream_t st);
