// libblsgpu: C-ABI host orchestration of the MI355X batch BLS verifier.
//
// Mirrors the reference's scheduling semantics:
//   * per-job verdicts and retry   packages/beacon-node/src/chain/bls/multithread/worker.ts:32-108
//   * batch vs single verify       packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39
//   * pubkey aggregation errors    packages/beacon-node/src/chain/bls/utils.ts:5-16
//   * packing jobs into packages   packages/beacon-node/src/chain/bls/multithread/index.ts:290-401
// but lays the sets out for the GPU: one lane per set, device groups of <= 64
// sets (one wavefront) each closed by its own final exponentiation.
//
// Dynamic batching: every bgv_verify / bgv_verify_async call is laid out on the
// calling thread and queued; dispatcher threads (a few per device, one HIP
// stream each) merge all queued calls into one device super-batch, run the
// kernels once over it and hand each call its own verdicts.  This is the GPU
// form of the reference's prepareWork(), which packs queued jobs into one worker
// package: concurrent calls share wavefronts instead of competing for queues.
//
// A job's verdict is the AND of the groups holding its sets.  A failing group
// that mixes batchable jobs sends exactly those jobs to retry rounds run over the
// per-set results already on the device (no set is recomputed).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <unordered_map>
#include <deque>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <unordered_set>
#include <thread>
#include <vector>

#include "../../include/blsgpu.h"
#include "bgv_launch.h"
#include "bls_field.h"  // fp12_t (sizes of the per-group u copies)

// parts a failing mixed group is split into per retry round (BGV_RETRY_FANOUT env).
// Group closings are team-parallel and cheap in latency, so bisecting (64 -> 8 -> 1)
// costs an extra round but ~4x fewer final exponentiations than going per job at once.
#define BGV_RETRY_FANOUT 8
// slots merged into one device super-batch (BGV_MAX_BATCH_SLOTS env)
#define BGV_MAX_BATCH_SLOTS 131072
// dispatcher threads (= HIP streams) per device (BGV_DISPATCHERS env)
#define BGV_DISPATCHERS 2

static size_t env_size(const char* name, size_t dflt, size_t lo) {
  const char* e = getenv(name);
  long n = e ? atol(e) : 0;
  return n >= (long)lo ? (size_t)n : dflt;
}
static size_t retry_fanout() {
  static const size_t v = env_size("BGV_RETRY_FANOUT", BGV_RETRY_FANOUT, 2);
  return v;
}
static size_t max_batch_slots() {
  static const size_t v = env_size("BGV_MAX_BATCH_SLOTS", BGV_MAX_BATCH_SLOTS, BGV_WAVE);
  return v;
}
// sets per first-pass device group, a power of two <= 64 (BGV_GROUP_SLOTS env).
// Smaller groups fail less often under invalid signatures (fewer retried jobs)
// at the price of more final exponentiations when every set is valid.
#define BGV_GROUP_SLOTS 64
static uint32_t group_slots() {
  static const uint32_t v = [] {
    size_t n = env_size("BGV_GROUP_SLOTS", BGV_GROUP_SLOTS, 1);
    uint32_t p = 1;
    while (p * 2 <= n && p * 2 <= BGV_WAVE) p *= 2;
    return p;
  }();
  return v;
}
// how long an idle dispatcher waits for more calls to merge (BGV_COALESCE_US env)
#define BGV_COALESCE_US 500
static size_t coalesce_us() {
  static const size_t v = env_size("BGV_COALESCE_US", BGV_COALESCE_US, 0);
  return v;
}
// the window while no super-batch is running: a lone call (block import, a quiet gossip
// moment) then launches almost at once instead of waiting the full window for company
// that is not coming (BGV_IDLE_COALESCE_US env)
#define BGV_IDLE_COALESCE_US 50
static size_t idle_coalesce_us() {
  static const size_t v = env_size("BGV_IDLE_COALESCE_US", BGV_IDLE_COALESCE_US, 0);
  return v;
}
// calls of at least this many sets on a context with several devices are spread over them
// (verify_split; BGV_SPLIT_MIN env, bgv_set_split; 0 disables): a range-sync call ("64 blocks
// ~ 8000 signatures", chain/bls/multithread/index.ts:34) takes every device
#define BGV_SPLIT_MIN_SETS 4096
static size_t split_min_env() {
  static const size_t v = env_size("BGV_SPLIT_MIN", BGV_SPLIT_MIN_SETS, 0);
  return v == 1 ? 2 : v;  // a one-set job is never cut (bgv_set_split)
}
static int dispatchers_per_device() {
  static const int v = (int)env_size("BGV_DISPATCHERS", BGV_DISPATCHERS, 1);
  return v;
}
// Exec buffer sets per device (BGV_EXECS): one per dispatcher plus the ones whose super-batch
// is in its retry rounds
static int execs_per_device() {
  static const int v = (int)env_size("BGV_EXECS", 2 * BGV_DISPATCHERS, 1);
  return std::max(v, dispatchers_per_device());
}

// BGV_UNIFORM=0 turns off uniform groups (BGV_GROUP_UNIFORM: one Miller loop per group whose sets
// share a signing root, and the grouping of a call's batchable one-set jobs by root that makes
// them), for A/B measurements; on by default
static bool uniform_enabled() {
  static const bool v = [] {
    const char* e = getenv("BGV_UNIFORM");
    return !(e && atoi(e) == 0);
  }();
  return v;
}
// BGV_WEIGHTED_UNIFORM=0: failing uniform groups take the pattern tests at once (no weighted
// test first; call_build_parts), for A/B measurements
static bool weighted_uniform_enabled() {
  static const bool v = [] {
    const char* e = getenv("BGV_WEIGHTED_UNIFORM");
    return !(e && atoi(e) == 0);
  }();
  return v;
}
// calls with fewer batchable one-set jobs take the latency path: their jobs keep their order
#define BGV_UNIFORM_MIN_JOBS 1024

// Retry threads per device (BGV_RETRY_THREADS), each with its own high-priority stream: the
// retry rounds of several super-batches then run side by side instead of queueing behind one
// another (their rounds are latency-bound chains of small launches)
// batches a retry thread holds at once (BGV_RETRY_HOLD): 1, one batch's rounds at a time.
// Holding up to 8 (their rounds side by side, one wait per pass) measured 2.11-2.51 against
// 2.44-2.46 M sets/s, interleaved (profiles/r05/retry_hold/): the steadier one is the default.
static size_t retry_hold_max() {
  static const size_t v = env_size("BGV_RETRY_HOLD", 1, 1);
  return v;
}
static int retry_threads_per_device() {
  static const int v = (int)env_size("BGV_RETRY_THREADS", 1, 1);
  return v;
}

extern "C" int bgv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

namespace {

// Page-locked host staging: copies from it run on the DMA engines, whereas pageable
// copies are staged by blit kernels that queue behind the verify kernels on the CUs.
template <class T>
struct Pinned {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    n = std::max(n, 2 * cap);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T), 0);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = n;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// One dispatcher's device resources: its stream, events and buffers.
struct Exec {
  // streams lent by the user of the buffers: the dispatcher's stream for a super-batch's first
  // pass, the device's retry stream for its retry rounds (Device::sched)
  hipStream_t main = nullptr;   // per-set kernels and the first pass's closing
  hipStream_t close = nullptr;  // retry rounds (latency-bound): high priority
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_prep = nullptr, ev_sets = nullptr;
  hipEvent_t kev[2 * BGV_NKERNELS] = {};
  void* slot_mem = nullptr;
  uint32_t slot_cap = 0;
  void* group_mem = nullptr;
  uint32_t group_cap = 0;
  bgv_dslot* d_slots = nullptr;
  bgv_dgroup* d_groups = nullptr;
  uint32_t* d_idx = nullptr;
  size_t idx_cap = 0;
  uint8_t* d_pkb = nullptr;
  size_t pkb_cap = 0;
  // host staging of one super-batch
  Pinned<bgv_dslot> h_slots;
  Pinned<bgv_dgroup> h_groups;
  Pinned<uint32_t> h_idx;
  Pinned<uint8_t> h_pkb;
  Pinned<int32_t> h_ss, h_ps, h_verdict;
  fp12_t* d_gu1 = nullptr;  // the first pass's per-group u values, kept for the retry rounds' pattern tests
  size_t gu1_cap = 0;
  void* d_pscratch = nullptr;  // Fp12 products of bgv_verify_partial calls
  size_t pscratch_cap = 0;
  uint8_t* d_pout = nullptr;
  size_t pout_cap = 0;
  uint32_t* d_lines = nullptr;  // the bulk Miller loop's line records (bgv_lines_pairs)
  uint32_t lines_cap = 0;       // pairs
};

// bgv_final_verify's device buffers (under util_mu)
struct FinalScratch {
  uint8_t* din = nullptr;
  void* vals = nullptr;
  void* one = nullptr;
  bgv_dgroup* dg = nullptr;
  int32_t* dst = nullptr;
  int32_t* dv = nullptr;
  size_t cap = 0;
};

struct Call;
// What a super-batch's retry rounds need from its first pass.
struct BatchState {
  std::chrono::steady_clock::time_point tb;
  double t_merge = 0, t_tok = 0, t_sets = 0, t_pass1 = 0, t_post = 0;
  uint32_t nslots = 0, ngroups = 0;
  std::vector<uint32_t> call_gb;  // each call's first group in the merged batch
  bool want_gu = false;           // the first pass's u values are in x.d_gu1 (pattern tests)
  bool uniform = false;           // the first pass ran uniform groups (their slots have no own pair f_i)
  bool prof = false;
};
// A super-batch whose first pass is done and whose retry rounds wait for the retry thread.
struct RetryJob {
  std::vector<Call*> calls;
  Exec* x = nullptr;
  std::shared_ptr<BatchState> st;
};
// Exec buffer sets and retry rounds of one device.  A dispatcher takes a free Exec for each
// super-batch and, when its first pass leaves failing groups, hands the batch to the device's
// retry thread and goes on with the next super-batch; the Exec returns to the pool when the
// retry rounds are done.  So the latency-bound retry rounds of one batch overlap the per-set
// kernels of the next ones instead of holding a dispatcher.  Streams: one per dispatcher, one
// (high priority) for the retry rounds, the utility stream: within HIP's default of 4 hardware
// queues per process (GPU_MAX_HW_QUEUES).
struct DevSched {
  std::mutex mu;
  std::condition_variable cv;  // an Exec was released / a retry job was queued / stop
  std::deque<Exec*> free;
  std::deque<RetryJob> rq;
  bool stop = false;
  std::vector<std::thread> retry_threads;
  std::vector<hipStream_t> retries;  // one stream per retry thread
  std::vector<hipStream_t> dstreams;
};

struct Device {
  int id = 0;
  std::unique_ptr<DevSched> sched = std::make_unique<DevSched>();
  FinalScratch final_scratch;
  hipStream_t stream = nullptr;      // utility work (cache upload, hooks, keygen)
  bgv_cache_entry* cache = nullptr;  // pubkey cache (replicated on every device)
  size_t cache_cap = 0;
  std::vector<Exec*> execs;
  // held while one super-batch runs its per-set kernels (pointer: Device stays movable)
  std::unique_ptr<std::mutex> compute_mu = std::make_unique<std::mutex>();
};

// An allocator whose value-less construct leaves the element uninitialized: resizing a vector of
// slot records then writes nothing (layout_one_job_fast fills every record itself)
template <class T>
struct uninit_alloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = uninit_alloc<U>;
  };
  uninit_alloc() = default;
  template <class U>
  uninit_alloc(const uninit_alloc<U>&) {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};

// jobs -> slots/groups of one call
struct Layout {
  std::vector<bgv_dslot, uninit_alloc<bgv_dslot>> slots;
  std::vector<bgv_dgroup> groups;
  std::vector<int32_t> slot_set;  // set index per slot (-1 = pad)
  std::vector<std::vector<uint32_t>> job_groups;
  std::vector<uint32_t> job_first_slot;  // first slot of each laid-out job (its slots are contiguous)
  std::vector<char> group_shared;        // group holds sets of more than one job
  std::vector<char> group_uniform;       // every set of the group shares one signing root and no
                                         // batchable job in it spans groups (BGV_GROUP_UNIFORM in bulk
                                         // batches)
  std::vector<uint32_t> idx;             // concatenated pubkey indices
  std::vector<uint8_t> pkb;              // concatenated 96-B pubkey records
  std::vector<uint32_t> uniq;            // first slot of each distinct signing root (hash_to_G2 once)
};

struct Builder {
  Layout& L;
  bool open = false;  // a group is open for appending
  uint32_t open_group = 0;
  int open_job = -1;
  // signing root -> its first slot, keyed by the root's first 8 bytes (a SHA-256 output); a
  // key collision between different roots only costs one extra hash
  std::unordered_map<uint64_t, uint32_t> first_root;
  explicit Builder(Layout& l) : L(l) {}

  void close_group() { open = false; }
  void new_group() {
    // start at the next wave boundary
    uint32_t first = (uint32_t)L.slots.size();
    const uint32_t gs = group_slots();
    uint32_t aligned = (first + gs - 1) / gs * gs;
    while (L.slots.size() < aligned) pad();
    L.groups.push_back(bgv_dgroup{aligned, 0, BGV_ALL_SLOTS});
    L.group_shared.push_back(0);
    L.group_uniform.push_back(1);
    open_group = (uint32_t)L.groups.size() - 1;
    open = true;
    open_job = -1;
  }
  void pad() {
    bgv_dslot s;
    memset(&s, 0, sizeof(s));
    s.flags = BGV_SLOT_PAD;
    s.hsrc = (uint32_t)L.slots.size();
    L.slots.push_back(s);
    L.slot_set.push_back(-1);
  }
  void pad_to_wave() {
    while (L.slots.size() % BGV_WAVE) pad();
  }
  void add(int job, uint32_t set_index, const bgv_set& st, bool first_of_job) {
    if (!open || L.groups[open_group].n_slots == group_slots()) new_group();
    bgv_dgroup& g = L.groups[open_group];
    if (open_job >= 0 && open_job != job) L.group_shared[open_group] = 1;
    open_job = job;
    std::vector<uint32_t>& jg = L.job_groups[job];
    if (jg.empty() || jg.back() != open_group) jg.push_back(open_group);
    if (first_of_job) L.job_first_slot[job] = (uint32_t)L.slots.size();
    bgv_dslot s;
    memset(&s, 0, sizeof(s));
    s.n_pk = st.n_pk;
    s.sig_len = st.sig_len;
    s.group = open_group;
    if (st.pk_indices) {
      s.flags = BGV_SLOT_PK_CACHED;
      s.pk_off = (uint32_t)L.idx.size();
      L.idx.insert(L.idx.end(), st.pk_indices, st.pk_indices + st.n_pk);
    } else {
      s.flags = BGV_SLOT_PK_BYTES;
      s.pk_off = (uint32_t)(L.pkb.size() / 96);
      L.pkb.insert(L.pkb.end(), st.pk_bytes, st.pk_bytes + 96ull * st.n_pk);
    }
    memcpy(s.msg, st.msg, 32);
    if (st.sig_len == 96) memcpy(s.sig, st.sig, 96);
    const uint32_t self = (uint32_t)L.slots.size();
    if (self > 0 && !(L.slots[self - 1].flags & BGV_SLOT_PAD) && memcmp(L.slots[self - 1].msg, st.msg, 32) == 0) {
      s.hsrc = L.slots[self - 1].hsrc;  // the previous slot's root (committees arrive together)
    } else {
      uint64_t key;
      memcpy(&key, st.msg, 8);
      auto it = first_root.find(key);
      if (it == first_root.end()) it = first_root.emplace(key, self).first;
      if (it->second != self && memcmp(L.slots[it->second].msg, st.msg, 32) == 0) {
        s.hsrc = it->second;  // same root as an earlier slot of this call
      } else {
        s.hsrc = self;
        L.uniq.push_back(self);
      }
    }
    if (g.n_slots > 0 && L.slots[g.first_slot].hsrc != s.hsrc) L.group_uniform[open_group] = 0;
    L.slots.push_back(s);
    L.slot_set.push_back((int32_t)set_index);
    g.n_slots++;
  }
};

struct Part {  // one retry test: consecutive jobs of one failing unit, and the device groups covering them
  std::vector<size_t> jobs;
  std::vector<uint32_t> groups;  // indices into the round's merged group list
  int pattern = -1;              // pattern test: index into Call::punits (its bit is the part's order)
};

// A failing first-pass group whose jobs all lie inside it (gossip: one-set jobs) is retried
// by pattern tests in ONE round: test S_j = the jobs whose index in the group has bit j set,
// j < ceil(log2 n).  The complement's verdict comes for free: the group's pairing value is
// the product of S_j's and its complement's, so with u = gprod^((p^2+1) 3 (p^4-p^2+1)/r) (the
// pairing value is conj(u)/u, bls_team.h tm_final_exp_u) the complement passes iff
// u_group * conj(u_j) lies in Fp6.  A job inside any passing set is valid; every invalid
// job lies in no passing set, so one remaining candidate is the invalid job, and two or
// more go to the next round (usually as singletons).  k tests per failing group instead of
// fanout-bisection's 8 + 8 over two rounds.
//
// The remaining candidates (two or more invalid jobs: 2^h of them for two jobs whose indices
// differ in h bits) are tested one job per device group in the next round, so a failing
// group is resolved in at most two rounds: a round costs about the same latency whether it
// tests hundreds or thousands of groups, while a second pattern round over the candidates
// need not shrink them (two invalid jobs at the first and last candidate index).
//
// Two invalid jobs i, j (the usual case of a second round) leave as candidates the 2^h jobs
// that agree with both where i and j agree, h = the number of bits D where S_b and its
// complement both failed; the candidates pair up as x, x ^ D.  The next round tests the pairs
// (2^(h-1) tests instead of 2^h single jobs): when exactly one test fails and it is a pair,
// both its jobs are invalid (for b in D, S_b and its complement each hold an invalid job, and
// every invalid job is a candidate of that one pair); a failing single job is invalid; jobs of
// a failing pair next to other failures are tested alone in one more round.
struct PatternUnit {
  uint32_t group = 0;              // the call's first-pass group
  int kind = 0;                    // 0: pattern tests S_j; 1: pairs and single jobs; 2: one weighted test
  std::vector<size_t> jobs;        // kind 0: its jobs in slot order
  std::vector<uint32_t> tests;     // round group index of each test
  std::vector<std::vector<size_t>> test_jobs;  // kind 1: each test's jobs
};
// units from the first pass of at most this many jobs (not pattern-testable) are tested one
// job per device group
static const size_t kSingletonMax = 8;
// a signing root with at least this many one-set jobs starts its own device group (call_submit)
#ifndef BGV_UNIFORM_ALIGN_MIN
#define BGV_UNIFORM_ALIGN_MIN 32  // A/B: a huge value keeps the round-5 layout (roots back to back)
#endif
static const size_t kUniformAlignMin = BGV_UNIFORM_ALIGN_MIN;

// One bgv_verify call travelling through a dispatcher.
struct Call {
  const bgv_job* jobs = nullptr;
  size_t njobs = 0;
  const bgv_set* sets = nullptr;
  size_t nsets = 0;
  int mode = 0;
  int32_t* out = nullptr;
  bgv_stats* stats_out = nullptr;
  bgv_done_fn done = nullptr;
  void* user = nullptr;
  bool owned = false;
  std::chrono::steady_clock::time_point t0;
  // host state
  Layout L;
  std::vector<int32_t> code;  // 2 = pending
  std::vector<size_t> todo;
  std::vector<int32_t> set_sig, set_pk;
  std::vector<std::vector<size_t>> units;  // pending retry units
  std::vector<int> unit_group;             // first-pass group the unit's jobs lie in (-1: not known)
  std::vector<int> unit_rounds;            // pattern rounds the unit's jobs have been through
  std::vector<std::vector<uint32_t>> unit_idx;  // after a pattern round: the candidates' pattern indices
  std::vector<uint32_t> unit_dmask;        // ... and the index bits D of their pairing (0: none)
  std::vector<Part> parts;
  std::vector<PatternUnit> punits;         // this round's pattern-tested units
  bgv_stats st{};
  // bgv_verify_partial: the call's Miller-loop product (576 B) and its two status codes
  uint8_t* partial_out = nullptr;
  int32_t* partial_codes = nullptr;
  int dev = -1;  // index in bgv_ctx::devs of the only device whose dispatchers may take it (-1: any)
  bgv_job pjob{};
  int32_t pcode = 0;
  uint32_t slot_base = 0;  // offset of this call's slots in the merged batch
  int rc = BGV_OK;
  // completion
  std::mutex mu;
  std::condition_variable cv;
  bool finished = false;
  bool shared_job(size_t j) const { return mode == BGV_MODE_WORKER && jobs[j].batchable; }
};

}  // namespace

struct bgv_ctx {
  std::vector<Device> devs;
  // cached pubkeys: entries [0, n_pubkeys) are valid on every device.  A pure append writes
  // entries at and past n_pubkeys (which no submitted call reads) and then publishes the new
  // count, so it needs only the shared cache_mu; growth and overwrites take it exclusively.
  std::atomic<size_t> n_pubkeys{0};
  std::mutex put_mu;  // one cache writer at a time (bgv_pubkeys_put, bgv_keygen)
  // indices whose record failed to decode in bgv_pubkeys_put: kept in the count (later runs
  // stay contiguous) but any set naming one rejects with BGV_E_BAD_INDEX.  Written under the
  // exclusive cache_mu, read under the shared one.
  std::unordered_set<uint32_t> bad_pk;
  std::atomic<bool> closed{false};
  std::mutex rng_mu;
  uint64_t rng_seed = 0, rng_state = 0;
  std::shared_mutex cache_mu;  // verify: shared; cache writes: exclusive
  std::mutex util_mu;          // utility streams
  std::mutex prof_mu;
  bool profile = false;
  // BGV_FAULT_INJECT=1 at bgv_init: every super-batch fails as a HIP error would (tests of
  // the device-error path: every job in flight rejects with BGV_E_DEVICE, none resolves false)
  bool fault_inject = false;
  // super-batch geometry (bgv_set_batching; env defaults at bgv_init)
  std::atomic<uint32_t> max_slots{BGV_MAX_BATCH_SLOTS};
  std::atomic<uint32_t> coalesce{BGV_COALESCE_US};
  std::atomic<uint32_t> idle_coalesce{BGV_IDLE_COALESCE_US};
  std::atomic<int> running{0};  // super-batches being run by dispatchers
  // calls of at least this many sets are spread over the devices (verify_split; 0: never)
  std::atomic<uint32_t> split_min{BGV_SPLIT_MIN_SETS};
  // split calls not yet done (bgv_close waits for them); split_closing, set by bgv_close under
  // split_mu before it waits, turns later split calls away.  Both under split_mu.
  int split_inflight = 0;
  bool split_closing = false;
  std::mutex split_mu;
  std::condition_variable split_cv;
  double kernel_ms[BGV_NKERNELS] = {};
  uint64_t kernel_launches = 0;
  // dispatch
  std::vector<std::thread> dispatchers;
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<Call*> queue;
  bool stop = false;
};

#define HIPCHK(x)                               \
  do {                                          \
    hipError_t e_ = (x);                        \
    if (e_ != hipSuccess) return -BGV_E_DEVICE; \
  } while (0)

static uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// nonzero 64-bit randomizers (blst mul_n_aggregate with 64 random bits)
// fn(lo, hi) over [0, n) in up to 8 host threads when n is large (a 2^20-set call: the
// merge's 168 MB of slot records and 8 MB of getrandom output), else inline
template <class F>
static void par_ranges(size_t n, F fn) {
  const size_t kMin = size_t(1) << 17;
  const unsigned nt = n >= kMin ? std::min<unsigned>(8u, std::max(1u, std::thread::hardware_concurrency())) : 1u;
  if (nt <= 1) {
    fn(size_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(fn, n * t / nt, n * (t + 1) / nt);
  fn(size_t(0), n / nt);
  for (auto& t : th) t.join();
}

static void fill_scalars(bgv_ctx* c, uint64_t* out, size_t n) {
  {
    std::lock_guard<std::mutex> lk(c->rng_mu);
    if (c->rng_seed) {
      for (size_t i = 0; i < n; ++i) {
        uint64_t v;
        do v = splitmix64(&c->rng_state);
        while (v == 0);
        out[i] = v;
      }
      return;
    }
  }
  par_ranges(n, [out](size_t lo, size_t hi) {
    size_t got = 0;
    uint8_t* p = reinterpret_cast<uint8_t*>(out + lo);
    while (got < (hi - lo) * 8) {
      const ssize_t r = getrandom(p + got, (hi - lo) * 8 - got, 0);
      if (r > 0) got += (size_t)r;
    }
    for (size_t i = lo; i < hi; ++i)
      if (out[i] == 0) out[i] = 1;
  });
}

template <class T>
static int grow(T** p, size_t* cap, size_t want) {
  if (want <= *cap) return BGV_OK;
  size_t n = std::max(want, *cap * 2);
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)));
  *cap = n;
  return BGV_OK;
}

static int exec_reserve_slots(Exec& x, uint32_t slots) {
  if (slots <= x.slot_cap) return BGV_OK;
  uint32_t n = std::max<uint32_t>(slots, x.slot_cap * 2);
  if (x.slot_mem) (void)hipFree(x.slot_mem);
  if (x.d_slots) (void)hipFree(x.d_slots);
  x.slot_mem = nullptr;
  x.d_slots = nullptr;
  HIPCHK(hipMalloc(&x.slot_mem, bgv_slot_mem_bytes(n)));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&x.d_slots), sizeof(bgv_dslot) * n));
  x.slot_cap = n;
  return BGV_OK;
}

static int exec_reserve_groups(Exec& x, uint32_t groups) {
  if (groups <= x.group_cap) return BGV_OK;
  uint32_t n = std::max<uint32_t>(groups, x.group_cap * 2);
  if (x.group_mem) (void)hipFree(x.group_mem);
  if (x.d_groups) (void)hipFree(x.d_groups);
  x.group_mem = nullptr;
  x.d_groups = nullptr;
  HIPCHK(hipMalloc(&x.group_mem, bgv_group_bytes() * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&x.d_groups), sizeof(bgv_dgroup) * n));
  x.group_cap = n;
  return BGV_OK;
}

// line records for the batch's bulk Miller launch (none on the latency path): allocated on
// first use, in steps of 16,384 pairs (374 MB); kept for the next batch up to the context's
// current super-batch geometry (c->max_slots, which bgv_set_batching may raise above the
// environment's default: trimming against the default would free and reallocate the records --
// each hipFree a device synchronization -- after every first pass), freed after a larger call
// (a 2^20-set job alone needs ~24 GB: exec_trim_lines)
static uint32_t lines_keep_pairs(size_t slots) {
  return (uint32_t)((slots + slots / BGV_WAVE + 16383u) & ~(size_t)16383u);
}
static void exec_trim_lines(Exec& x, size_t max_slots) {
  if (x.lines_cap <= lines_keep_pairs(max_slots)) return;
  (void)hipFree(x.d_lines);
  x.d_lines = nullptr;
  x.lines_cap = 0;
}
static int exec_reserve_lines(Exec& x, bgv_dev_batch& b) {
  const uint32_t need = bgv_lines_pairs(b);
  if (need > x.lines_cap) {
    const uint32_t cap = (need + 16383u) & ~16383u;
    if (x.d_lines) (void)hipFree(x.d_lines);
    x.d_lines = nullptr;
    x.lines_cap = 0;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&x.d_lines), bgv_line_record_bytes() * cap));
    x.lines_cap = cap;
  }
  b.lines = x.d_lines;
  b.lines_cap = x.lines_cap;
  return BGV_OK;
}

static int exec_create(Exec* x) {
  HIPCHK(hipEventCreate(&x->ev0));
  HIPCHK(hipEventCreate(&x->ev1));
  HIPCHK(hipEventCreateWithFlags(&x->ev_sets, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&x->ev_prep, hipEventDisableTiming));
  for (auto& e : x->kev) HIPCHK(hipEventCreate(&e));
  return BGV_OK;
}

static void exec_destroy(Exec* x) {
  if (x->main) (void)hipStreamSynchronize(x->main);
  void* ptrs[] = {x->slot_mem, x->group_mem, x->d_slots,    x->d_groups, x->d_idx,
                  x->d_pkb,      x->d_pscratch, x->d_pout, x->d_lines};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  x->h_slots.release();
  x->h_groups.release();
  x->h_idx.release();
  x->h_pkb.release();
  x->h_ss.release();
  x->h_ps.release();
  x->h_verdict.release();
  if (x->d_gu1) (void)hipFree(x->d_gu1);
  if (x->ev0) (void)hipEventDestroy(x->ev0);
  if (x->ev1) (void)hipEventDestroy(x->ev1);
  if (x->ev_sets) (void)hipEventDestroy(x->ev_sets);
  if (x->ev_prep) (void)hipEventDestroy(x->ev_prep);
  for (auto& e : x->kev)
    if (e) (void)hipEventDestroy(e);
  if (x->close) (void)hipStreamSynchronize(x->close);
  delete x;
}

static void prof_add(bgv_ctx* c, Exec& x, bool sets, bool groups) {
  std::lock_guard<std::mutex> lk(c->prof_mu);
  if (!c->profile) return;
  for (int k = 0; k < BGV_NKERNELS; ++k) {
    const bool is_set_kernel = k < BGV_NSETKERNELS;
    if ((is_set_kernel && !sets) || (!is_set_kernel && !groups)) continue;
    float km = 0;
    if (hipEventElapsedTime(&km, x.kev[2 * k], x.kev[2 * k + 1]) == hipSuccess) c->kernel_ms[k] += km;
  }
  if (sets) c->kernel_launches++;
}

static bgv_dev_batch make_batch(Device& d, Exec& x, uint32_t nslots, uint32_t ngroups) {
  bgv_dev_batch b;
  memset(&b, 0, sizeof(b));
  b.nslots = nslots;
  b.ngroups = ngroups;
  b.slots = x.d_slots;
  b.groups = x.d_groups;
  b.pk_idx = x.d_idx;
  b.cache_opaque = d.cache;
  b.pk_bytes = x.d_pkb;
  bgv_carve(&b, x.slot_mem, x.slot_cap, x.group_mem, x.group_cap);
  return b;
}

// Outcome of one job from its slots' statuses (maybeBatch.ts:16-39 + blst semantics):
//   any undecodable / not-in-group signature -> error of the first such set (fromBytes throws)
//   any infinity public key                  -> 1 set: false (core verify), >= 2 sets: BLST_PK_IS_INFINITY
// returns 2 when the verdict depends on the groups.
static int32_t job_precheck(const std::vector<int32_t>& set_sig, const std::vector<int32_t>& set_pk,
                            const bgv_job& j) {
  for (uint32_t k = 0; k < j.n_sets; ++k) {
    const int32_t s = set_sig[j.first_set + k];
    if (s != BGV_OK && s != BGV_ST_INFINITY) return -s;
  }
  for (uint32_t k = 0; k < j.n_sets; ++k) {
    const int32_t p = set_pk[j.first_set + k];
    if (p == BGV_ST_INFINITY) return j.n_sets >= 2 ? -BGV_BLST_PK_IS_INFINITY : 0;
    if (p != BGV_OK) return -p;  // undecodable uncompressed pubkey record
  }
  return 2;
}

// ---------------------------------------------------------------------------
// Call lifecycle
// ---------------------------------------------------------------------------
static void call_finish(Call* call) {
  for (size_t j = 0; j < call->njobs; ++j) call->out[j] = call->code[j] == 2 ? -BGV_E_DEVICE : call->code[j];
  call->st.wall_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call->t0).count();
  if (call->stats_out) *call->stats_out = call->st;
  if (call->done) call->done(call->user, call->rc);
  if (call->owned) {
    delete call;
    return;
  }
  {
    std::lock_guard<std::mutex> lk(call->mu);
    call->finished = true;
  }
  call->cv.notify_all();
}

static void call_fail(Call* call, int rc) {
  call->rc = rc;
  for (auto& x : call->code)
    if (x == 2) x = -BGV_E_DEVICE;
  call_finish(call);
}

// The argument checks the reference raises before any crypto, for one job: *code = 2 when the
// job goes to the device, else its verdict (empty job, empty aggregate, an index that is not
// in the cache -- the first such set in set order).  -BGV_E_ARG for a malformed set record.
// The caller holds cache_mu (shared).
static int host_job_code(const bgv_ctx* c, const bgv_job& jb, const bgv_set* sets, int32_t* code) {
  *code = 2;
  if (jb.n_sets == 0) {
    *code = -BGV_E_EMPTY_SET;
    return BGV_OK;
  }
  for (uint32_t k = 0; k < jb.n_sets && *code == 2; ++k) {
    const bgv_set& s = sets[jb.first_set + k];
    if (s.n_pk == 0)
      *code = -BGV_E_EMPTY_AGGREGATE;
    else if (!s.msg || (!s.sig && s.sig_len) || (!s.pk_indices && !s.pk_bytes))
      return -BGV_E_ARG;
    else if (s.pk_indices)
      for (uint32_t q = 0; q < s.n_pk; ++q)
        if (s.pk_indices[q] >= c->n_pubkeys || (!c->bad_pk.empty() && c->bad_pk.count(s.pk_indices[q]))) {
          *code = -BGV_E_BAD_INDEX;
          break;
        }
  }
  return BGV_OK;
}

// The layout Builder makes for a call of ONE non-batchable job of cached-key sets (slots in set
// order from slot 0, groups of group_slots() consecutive slots, pads to the wave boundary),
// with the per-slot records filled by several host threads: the config-5 sweep's 2^20-set
// job took ~50 ms on one thread.  false: not such a call (the Builder lays it out).
static bool layout_one_job_fast(Call* call, const bgv_job& jb, const bgv_set* sets) {
  const uint32_t n = jb.n_sets, gs = group_slots();
  const bgv_set* S = sets + jb.first_set;
  if (n < (1u << 17)) return false;
  for (uint32_t i = 0; i < n; ++i)
    if (!S[i].pk_indices) return false;
  Layout& L = call->L;
  // signing roots in order: the previous set's root, else the first set with the same root (a
  // key collision between different roots opens a root of its own), as Builder::add
  std::vector<uint32_t> hsrc(n), pk_off(n);
  std::unordered_map<uint64_t, uint32_t> first_root;
  uint32_t npk = 0;
  for (uint32_t i = 0; i < n; ++i) {
    pk_off[i] = npk;
    npk += S[i].n_pk;
    if (i > 0 && memcmp(S[i - 1].msg, S[i].msg, 32) == 0) {
      hsrc[i] = hsrc[i - 1];
      continue;
    }
    uint64_t key;
    memcpy(&key, S[i].msg, 8);
    auto it = first_root.find(key);
    if (it == first_root.end()) it = first_root.emplace(key, i).first;
    if (it->second != i && memcmp(S[it->second].msg, S[i].msg, 32) == 0) {
      hsrc[i] = it->second;
    } else {
      hsrc[i] = i;
      L.uniq.push_back(i);
    }
  }
  const uint32_t nslots = (n + BGV_WAVE - 1) / BGV_WAVE * BGV_WAVE, ng = (n + gs - 1) / gs;
  L.slots.resize(nslots);
  L.slot_set.resize(nslots);
  L.idx.resize(npk);
  par_ranges(nslots, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      bgv_dslot& s = L.slots[i];
      memset(&s, 0, sizeof(s));
      if (i >= n) {
        s.flags = BGV_SLOT_PAD;
        s.hsrc = (uint32_t)i;
        L.slot_set[i] = -1;
        continue;
      }
      const bgv_set& st = S[i];
      s.n_pk = st.n_pk;
      s.sig_len = st.sig_len;
      s.group = (uint32_t)(i / gs);
      s.flags = BGV_SLOT_PK_CACHED;
      s.pk_off = pk_off[i];
      memcpy(L.idx.data() + pk_off[i], st.pk_indices, 4ull * st.n_pk);
      memcpy(s.msg, st.msg, 32);
      if (st.sig_len == 96) memcpy(s.sig, st.sig, 96);
      s.hsrc = hsrc[i];
      L.slot_set[i] = (int32_t)(jb.first_set + i);
    }
  });
  L.groups.resize(ng);
  L.group_shared.assign(ng, 0);
  L.group_uniform.assign(ng, 1);
  for (uint32_t g = 0; g < ng; ++g) {
    const uint32_t f = g * gs, m = std::min(gs, n - f);
    L.groups[g] = bgv_dgroup{f, m, BGV_ALL_SLOTS};
    for (uint32_t k = 1; k < m; ++k)
      if (hsrc[f + k] != hsrc[f]) {
        L.group_uniform[g] = 0;
        break;
      }
  }
  L.job_groups[0].resize(ng);
  for (uint32_t g = 0; g < ng; ++g) L.job_groups[0][g] = g;
  L.job_first_slot[0] = 0;
  return true;
}

// A freshly allocated layout of a huge call is first touched page by page: 168 MB of slot
// records for a 2^20-set call are ~43,000 page faults.  Transparent huge pages (where the host
// allows them) cut that to ~100.
static void advise_huge(void* p, size_t bytes) {
  const uintptr_t a = ((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
  const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)((2u << 20) - 1);
  if (e > a) (void)madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
}

// host-side checks and layout, on the caller's thread
static int call_submit(bgv_ctx* c, Call* call, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets,
                       int mode, int32_t* out, bgv_stats* stats, bgv_done_fn done, void* user, int dev = -1) {
  call->t0 = std::chrono::steady_clock::now();
  call->dev = dev;
  if (c->closed) return -BGV_E_CLOSED;
  if ((njobs && (!jobs || !out)) || (nsets && !sets)) return -BGV_E_ARG;
  if (mode != BGV_MODE_WORKER && mode != BGV_MODE_PER_JOB) return -BGV_E_ARG;
  call->jobs = jobs;
  call->njobs = njobs;
  call->sets = sets;
  call->nsets = nsets;
  call->mode = mode;
  call->out = out;
  call->stats_out = stats;
  call->done = done;
  call->user = user;
  call->code.assign(njobs, 2);
  {
    std::shared_lock<std::shared_mutex> clk(c->cache_mu);
    for (size_t j = 0; j < njobs; ++j) {
      if ((size_t)jobs[j].first_set + jobs[j].n_sets > nsets) return -BGV_E_ARG;
      if (host_job_code(c, jobs[j], sets, &call->code[j]) != BGV_OK) return -BGV_E_ARG;
    }
  }
  // pass-1 layout: non-batchable jobs own their groups; batchable jobs (worker mode) share
  Layout& L = call->L;
  L.job_groups.resize(njobs);
  L.job_first_slot.assign(njobs, 0);
  {
    size_t npk = 0;
    for (size_t i = 0; i < nsets; ++i)
      if (sets[i].pk_indices) npk += sets[i].n_pk;
    const size_t cap = nsets + nsets / 8 + BGV_WAVE;  // with room for the groups' padding
    L.slots.reserve(cap);
    L.slot_set.reserve(cap);
    L.idx.reserve(npk);
    if (nsets >= (1u << 17)) {
      advise_huge(L.slots.data(), sizeof(bgv_dslot) * cap);
      advise_huge(L.slot_set.data(), 4 * cap);
      advise_huge(L.idx.data(), 4 * npk);
    }
  }
  Builder B(L);
  for (size_t j = 0; j < njobs; ++j)
    if (call->code[j] == 2) call->todo.push_back(j);
  const bool fast = njobs == 1 && call->todo.size() == 1 && !call->shared_job(0) &&
                    layout_one_job_fast(call, jobs[0], sets);
  for (size_t j : call->todo) {
    if (call->shared_job(j) || fast) continue;
    B.close_group();
    for (uint32_t k = 0; k < jobs[j].n_sets; ++k)
      B.add((int)j, jobs[j].first_set + k, sets[jobs[j].first_set + k], k == 0);
    B.close_group();
  }
  B.close_group();
  // Batchable jobs share groups in any order (verdicts map by job).  One-set jobs go grouped by
  // signing root -- the roots in order of first appearance, each root's jobs in call order -- so
  // that the sets of a root fill whole groups (BGV_GROUP_UNIFORM: one Miller loop for the group;
  // gossip attestations of one committee share a root); then multi-set jobs.
  std::vector<size_t> shared_order;
  std::vector<size_t> breaks;  // positions in shared_order where a new device group starts
  size_t n_one = 0;
  for (size_t j : call->todo)
    if (call->shared_job(j) && jobs[j].n_sets == 1) ++n_one;
  if (uniform_enabled() && n_one >= BGV_UNIFORM_MIN_JOBS) {
    std::unordered_map<uint64_t, uint32_t> bucket_of;
    bucket_of.reserve(2 * n_one);
    std::vector<std::vector<size_t>> buckets;
    std::vector<const uint8_t*> broot;
    bool grouped = false;  // some root recurs after another root: the order changes
    uint32_t last = UINT32_MAX;
    for (size_t j : call->todo) {
      if (!call->shared_job(j) || jobs[j].n_sets != 1) continue;
      const uint8_t* m = sets[jobs[j].first_set].msg;
      uint64_t key;
      memcpy(&key, m, 8);
      auto it = bucket_of.find(key);
      uint32_t b;
      if (it != bucket_of.end() && memcmp(broot[it->second], m, 32) == 0) {
        b = it->second;
      } else {  // a new root (a key collision between different roots just opens another bucket)
        b = (uint32_t)buckets.size();
        buckets.emplace_back();
        broot.push_back(m);
        if (it == bucket_of.end()) bucket_of.emplace(key, b);
      }
      grouped = grouped || (b != last && !buckets[b].empty());
      last = b;
      buckets[b].push_back(j);
    }
    if (grouped) {
      // A root with at least half a group of jobs starts a group of its own, so its groups stay
      // uniform whatever the roots before it held (a committee one set short -- a corrupted
      // message, a late attestation -- would otherwise shift every later root across a group
      // boundary: both groups mixed, per-slot Miller loops, pattern tests instead of the weighted
      // one); the roots with fewer jobs share mixed groups after them, in order of appearance.
      for (const auto& bk : buckets)
        if (bk.size() >= kUniformAlignMin) {
          breaks.push_back(shared_order.size());
          shared_order.insert(shared_order.end(), bk.begin(), bk.end());
        }
      breaks.push_back(shared_order.size());
      for (const auto& bk : buckets)
        if (bk.size() < kUniformAlignMin) shared_order.insert(shared_order.end(), bk.begin(), bk.end());
      for (size_t j : call->todo)
        if (call->shared_job(j) && jobs[j].n_sets != 1) shared_order.push_back(j);
    }
  }
  if (shared_order.empty())  // call order
    for (size_t j : call->todo)
      if (call->shared_job(j)) shared_order.push_back(j);
  size_t bi = 0;
  for (size_t q = 0; q < shared_order.size(); ++q) {
    if (bi < breaks.size() && breaks[bi] == q) B.close_group();
    while (bi < breaks.size() && breaks[bi] <= q) ++bi;
    const size_t j = shared_order[q];
    for (uint32_t k = 0; k < jobs[j].n_sets; ++k)
      B.add((int)j, jobs[j].first_set + k, sets[jobs[j].first_set + k], k == 0);
  }
  B.pad_to_wave();
  // A batchable job over several groups may be retried by fanout over its slots, which needs
  // their own pairs: its groups are not uniform.  A non-batchable job is never retried (its
  // verdict is its groups' AND, call_after_pass1), so its groups stay uniform where their sets
  // share a root: the config-5 sweep's one 2^20-set job, committee by committee.
  for (size_t j : call->todo)
    if (L.job_groups[j].size() > 1 && call->shared_job(j))
      for (uint32_t g : L.job_groups[j]) L.group_uniform[g] = 0;
  call->set_sig.assign(nsets, 0);
  call->set_pk.assign(nsets, 0);
  if (L.slots.empty()) {  // nothing for the device
    call_finish(call);
    return BGV_OK;
  }
  {
    std::lock_guard<std::mutex> lk(c->qmu);
    if (c->stop) return -BGV_E_CLOSED;
    c->queue.push_back(call);
  }
  if (dev < 0)
    c->qcv.notify_one();
  else
    c->qcv.notify_all();  // only the pinned device's dispatchers may take it
  return BGV_OK;
}

// After pass 1: statuses, verdicts and the retry units of one call.
static void call_after_pass1(Call* call, const int32_t* ss, const int32_t* ps, const int32_t* verdict) {
  Layout& L = call->L;
  const uint32_t nslots = (uint32_t)L.slots.size(), ngroups = (uint32_t)L.groups.size();
  for (uint32_t i = 0; i < nslots; ++i)
    if (L.slot_set[i] >= 0) {
      call->set_sig[L.slot_set[i]] = ss[i];
      call->set_pk[L.slot_set[i]] = ps[i];
      call->st.sets_verified++;
    }
  call->st.device_groups += ngroups;
  if (call->partial_out) {
    // first signature error and first pubkey condition in set order (the caller combines
    // the shards' codes in rank order, as job_precheck does within one job)
    int32_t sig = 0, pk = 0;
    for (size_t i = 0; i < call->nsets; ++i) {
      const int32_t a = call->set_sig[i], q = call->set_pk[i];
      if (!sig && a != BGV_OK && a != BGV_ST_INFINITY) sig = -a;
      if (!pk && q == BGV_ST_INFINITY) pk = 1;
      if (!pk && q != BGV_OK && q != BGV_ST_INFINITY) pk = -q;
    }
    call->partial_codes[0] = sig;
    call->partial_codes[1] = pk;
    for (size_t j : call->todo) call->code[j] = 1;
    return;
  }
  std::vector<char> group_retried(ngroups, 0);
  std::vector<int> unit_of_group(ngroups, -1);
  std::vector<char> seen(call->njobs, 0);
  for (size_t j : call->todo) {
    const int32_t pre = job_precheck(call->set_sig, call->set_pk, call->jobs[j]);
    if (pre != 2) {
      call->code[j] = pre;
      continue;
    }
    bool ok = true;
    int first_bad_shared = -1;
    for (uint32_t g : L.job_groups[j])
      if (!(verdict[g] & 1)) {
        ok = false;
        if (L.group_shared[g] && first_bad_shared < 0) first_bad_shared = (int)g;
      }
    if (first_bad_shared >= 0) {
      group_retried[first_bad_shared] = 1;
      if (unit_of_group[first_bad_shared] < 0) {
        unit_of_group[first_bad_shared] = (int)call->units.size();
        call->units.emplace_back();
        call->unit_group.push_back(first_bad_shared);
        call->unit_rounds.push_back(0);
        call->unit_idx.emplace_back();
        call->unit_dmask.push_back(0);
      }
      if (!seen[j]) {
        seen[j] = 1;
        call->units[unit_of_group[first_bad_shared]].push_back(j);
      }
    } else {
      call->code[j] = ok ? 1 : 0;
      if (ok && call->shared_job(j)) call->st.batch_sigs_success += call->jobs[j].n_sets;
    }
  }
  for (char r : group_retried) call->st.batch_retries += r;
}

// A unit from pass 1 is pattern-testable when its jobs lie only in its group and cover every
// slot of the group that takes part in the group's product (the others -- sets of jobs that
// failed their precheck -- contribute 1): then a test S_j and its complement partition the
// group's product.
static bool pattern_eligible(const Call* call, size_t u) {
  if (u >= call->unit_group.size() || call->unit_group[u] < 0) return false;
  const std::vector<size_t>& jobs = call->units[u];
  if (jobs.size() < 2) return false;
  const uint32_t g = (uint32_t)call->unit_group[u];
  const bgv_dgroup& G = call->L.groups[g];
  uint64_t covered = 0;
  for (size_t j : jobs) {
    const auto& jg = call->L.job_groups[j];
    if (jg.size() != 1 || jg[0] != g) return false;
    const uint32_t off = call->L.job_first_slot[j] - G.first_slot, n = call->jobs[j].n_sets;
    covered |= (n >= 64 ? ~0ull : ((1ull << n) - 1)) << off;
  }
  for (uint32_t k = 0; k < G.n_slots; ++k) {
    if ((covered >> k) & 1) continue;
    const int32_t si = call->L.slot_set[G.first_slot + k];
    if (si < 0) continue;
    const int32_t a = call->set_sig[si], q = call->set_pk[si];
    if ((a == BGV_OK || a == BGV_ST_INFINITY) && q == BGV_OK) return false;  // live, outside the unit
  }
  return true;
}

// A job's slots within its (single) group g, as a device-group mask
static uint64_t job_mask(const Call* call, size_t j, const bgv_dgroup& g) {
  const uint32_t off = call->L.job_first_slot[j] - g.first_slot, n = call->jobs[j].n_sets;
  return (n >= 64 ? ~0ull : ((1ull << n) - 1)) << off;
}

// every job of the unit lies in the call's group g alone
static bool unit_in_group(const Call* call, const std::vector<size_t>& jobs, int g) {
  if (g < 0) return false;
  for (size_t j : jobs) {
    const auto& jg = call->L.job_groups[j];
    if (jg.size() != 1 || jg[0] != (uint32_t)g) return false;
  }
  return true;
}

// Group testing for one retry round: split every pending unit into parts.  gb: the call's
// first group in the batch when the first pass's u values are on the device (pattern tests
// possible), else -1.
static void call_build_parts(Call* call, std::vector<bgv_dgroup>& rg, int64_t gb, bool uniform) {
  // A test inside a uniform first-pass group (whose slots have no own pair f_i) pairs the sum
  // of its slots' r_i pk_i with the group's one H instead: prod_S e(r_i pk_i, H) =
  // e(sum_S r_i pk_i, H), the same pairing value, so the complement verdicts hold too
  auto uflag = [&](uint32_t g) { return uniform && call->L.group_uniform[g] ? BGV_GROUP_UNIFORM : 0u; };
  call->parts.clear();
  call->punits.clear();
  for (size_t ui = 0; ui < call->units.size(); ++ui) {
    const auto& u = call->units[ui];
    const int ug = call->unit_group[ui], urounds = call->unit_rounds[ui];
    const bool in_group = unit_in_group(call, u, ug);
    const bool eligible = gb >= 0 && in_group && urounds <= 0 && u.size() >= 2 && pattern_eligible(call, ui);
    if (eligible && urounds == 0 && uflag((uint32_t)ug) && weighted_uniform_enabled()) {
      // a failing uniform group almost always holds ONE invalid slot (a wrong key): one test with
      // slot k weighted by k + 1 names it (BGV_GROUP_WEIGHTED; k_final12 finds w with V^w = W)
      // instead of ~6 pattern tests of two Miller loops each; otherwise the pattern tests follow
      // (unit_rounds -1).  Soundness with two or more invalid slots: write slot k's pairing
      // defect as g^(e_k) in the prime-order group GT (e_k != 0 for an invalid slot; the
      // signatures, hence the e_k, are the attacker's, fixed before the secret randomizers are
      // drawn).  V^w = W means sum_k (k + 1 - w) r_k e_k = 0 (mod r), a linear equation in the
      // secret r_k with a nonzero coefficient on at least one of them; r_k takes 2^64 distinct
      // values mod r, so for one w it holds with probability <= 2^-64, and over the 64 candidate
      // w with <= 64 * 2^-64 per failing group (a match would accept the other invalid jobs).
      PatternUnit pu;
      pu.group = (uint32_t)ug;
      pu.kind = 2;
      const bgv_dgroup& g = call->L.groups[pu.group];
      std::vector<std::pair<uint32_t, size_t>> order;
      for (size_t j : u) order.emplace_back(call->L.job_first_slot[j], j);
      std::sort(order.begin(), order.end());
      uint64_t m = 0;
      for (const auto& o : order) {
        pu.jobs.push_back(o.second);
        m |= job_mask(call, o.second, g);
      }
      Part part;
      part.jobs = pu.jobs;
      part.groups.push_back((uint32_t)rg.size());
      part.pattern = (int)call->punits.size();
      pu.tests.push_back((uint32_t)rg.size());
      rg.push_back(bgv_dgroup{call->slot_base + g.first_slot, g.n_slots, m, (uint32_t)(gb + ug + 1),
                              BGV_GROUP_UNIFORM | BGV_GROUP_WEIGHTED});
      call->parts.push_back(std::move(part));
      call->punits.push_back(std::move(pu));
      continue;
    }
    if (eligible) {
      PatternUnit pu;
      pu.group = (uint32_t)ug;
      const bgv_dgroup& g = call->L.groups[pu.group];
      std::vector<std::pair<uint32_t, size_t>> order;  // jobs in slot order
      for (size_t j : u) order.emplace_back(call->L.job_first_slot[j], j);
      std::sort(order.begin(), order.end());
      std::vector<uint64_t> jmask;
      for (const auto& o : order) {
        pu.jobs.push_back(o.second);
        jmask.push_back(job_mask(call, o.second, g));
      }
      const size_t n = pu.jobs.size();
      int k = 0;
      while ((1ull << k) < n) ++k;
      for (int b = 0; b < k; ++b) {
        uint64_t m = 0;
        Part part;
        for (size_t i = 0; i < n; ++i)
          if ((i >> b) & 1) {
            m |= jmask[i];
            part.jobs.push_back(pu.jobs[i]);
          }
        pu.tests.push_back((uint32_t)rg.size());
        part.groups.push_back((uint32_t)rg.size());
        part.pattern = (int)call->punits.size();
        rg.push_back(bgv_dgroup{call->slot_base + g.first_slot, g.n_slots, m, (uint32_t)(gb + ug + 1), uflag(ug)});
        call->parts.push_back(std::move(part));
      }
      call->punits.push_back(std::move(pu));
      continue;
    }
    if (in_group && urounds > 0 && call->unit_dmask[ui] && call->unit_idx[ui].size() == u.size()) {
      // pairs x, x ^ D of a pattern round's candidates (see PatternUnit), single jobs otherwise
      const bgv_dgroup& g = call->L.groups[ug];
      const uint32_t D = call->unit_dmask[ui];
      const uint32_t b0 = D & (~D + 1);  // lowest bit of D
      std::unordered_map<uint32_t, size_t> at;
      for (size_t k = 0; k < u.size(); ++k) at[call->unit_idx[ui][k]] = u[k];
      PatternUnit pu;
      pu.group = (uint32_t)ug;
      pu.kind = 1;
      for (size_t k = 0; k < u.size(); ++k) {
        const uint32_t x = call->unit_idx[ui][k];
        const auto partner = at.find(x ^ D);
        if (partner != at.end() && (x & b0)) continue;  // tested with its partner
        std::vector<size_t> tj{u[k]};
        uint64_t m = job_mask(call, u[k], g);
        if (partner != at.end()) {
          tj.push_back(partner->second);
          m |= job_mask(call, partner->second, g);
        }
        Part part;
        part.jobs = tj;
        part.groups.push_back((uint32_t)rg.size());
        part.pattern = (int)call->punits.size();
        pu.tests.push_back((uint32_t)rg.size());
        pu.test_jobs.push_back(std::move(tj));
        rg.push_back(bgv_dgroup{call->slot_base + g.first_slot, g.n_slots, m, 0, uflag(ug)});
        call->parts.push_back(std::move(part));
      }
      call->punits.push_back(std::move(pu));
      continue;
    }
    if (in_group && (urounds > 0 || u.size() <= kSingletonMax)) {
      // one device group per job, each masked to the job's slots: every verdict in this round
      const bgv_dgroup& g = call->L.groups[ug];
      for (size_t j : u) {
        Part part;
        part.jobs.push_back(j);
        part.groups.push_back((uint32_t)rg.size());
        rg.push_back(bgv_dgroup{call->slot_base + g.first_slot, g.n_slots, job_mask(call, j, g), 0, uflag(ug)});
        call->parts.push_back(std::move(part));
      }
      continue;
    }
    const size_t k = std::min<size_t>(retry_fanout(), u.size());
    for (size_t p = 0; p < k; ++p) {
      Part part;
      const size_t lo = u.size() * p / k, hi = u.size() * (p + 1) / k;
      part.jobs.assign(u.begin() + lo, u.begin() + hi);
      for (size_t q = 0; q < part.jobs.size();) {  // maximal runs of consecutive slots
        const uint32_t first = call->L.job_first_slot[part.jobs[q]];
        uint32_t n = 0;
        size_t q2 = q;
        while (q2 < part.jobs.size() && call->L.job_first_slot[part.jobs[q2]] == first + n) {
          n += call->jobs[part.jobs[q2]].n_sets;
          ++q2;
        }
        // chunks within one first-pass group each, so a chunk of a uniform group takes its flag
        // and its root: bounded by the end of slot s0's own group (with BGV_GROUP_SLOTS < 64 a
        // wave holds several groups) and by the wave
        for (uint32_t off = 0; off < n;) {
          const uint32_t s0 = first + off;
          const bgv_dgroup& g0 = call->L.groups[call->L.slots[s0].group];
          const uint32_t len = std::min<uint32_t>(std::min<uint32_t>(n - off, BGV_WAVE - s0 % BGV_WAVE),
                                                  g0.first_slot + g0.n_slots - s0);
          part.groups.push_back((uint32_t)rg.size());
          rg.push_back(bgv_dgroup{call->slot_base + s0, len, BGV_ALL_SLOTS, 0, uflag(call->L.slots[s0].group)});
          off += len;
        }
        q = q2;
      }
      call->parts.push_back(std::move(part));
    }
  }
  call->units.clear();
  call->unit_group.clear();
  call->unit_rounds.clear();
  call->unit_idx.clear();
  call->unit_dmask.clear();
}

static bool trace_on() {
  static const bool v = getenv("BGV_TRACE") != nullptr;
  return v;
}

// rv: the round's verdict bits (bgv_layout.h: bit 0 the group passes, bit 1 its pairing value
// equals its reference's, i.e. the complement passes)
static void call_after_round(Call* call, const int32_t* rv) {
  for (const Part& part : call->parts) {
    if (part.pattern >= 0) continue;
    bool ok = true;
    for (uint32_t g : part.groups) ok = ok && (rv[g] & 1);
    if (ok || part.jobs.size() == 1) {
      for (size_t j : part.jobs) call->code[j] = ok ? 1 : 0;
    } else {
      call->units.push_back(part.jobs);
      call->unit_group.push_back(-1);
      call->unit_rounds.push_back(0);
      call->unit_idx.emplace_back();
      call->unit_dmask.push_back(0);
    }
  }
  for (const PatternUnit& pu : call->punits) {
    if (pu.kind == 2) {  // one weighted test: bits 8..15 = w, slot w - 1 the lone invalid one
      const int32_t v = rv[pu.tests[0]];
      const uint32_t w = ((uint32_t)v >> 8) & 0xffu;
      const bgv_dgroup& g = call->L.groups[pu.group];
      size_t bad = SIZE_MAX;
      if (w >= 1 && w <= g.n_slots)
        for (size_t j : pu.jobs)
          if ((job_mask(call, j, g) >> (w - 1)) & 1) bad = j;
      if (bad != SIZE_MAX) {
        for (size_t j : pu.jobs) call->code[j] = j == bad ? 0 : 1;
      } else {  // not a lone invalid slot: the pattern tests next round
        call->units.push_back(pu.jobs);
        call->unit_group.push_back((int)pu.group);
        call->unit_rounds.push_back(-1);
        call->unit_idx.emplace_back();
        call->unit_dmask.push_back(0);
      }
      continue;
    }
    if (pu.kind == 1) {  // pairs and single jobs (see PatternUnit)
      std::vector<size_t> failing;
      for (size_t t = 0; t < pu.tests.size(); ++t)
        if (!(rv[pu.tests[t]] & 1)) failing.push_back(t);
      std::vector<size_t> again;
      for (size_t t = 0; t < pu.tests.size(); ++t) {
        const auto& tj = pu.test_jobs[t];
        const bool pass = rv[pu.tests[t]] & 1;
        if (pass || tj.size() == 1 || failing.size() == 1) {
          for (size_t j : tj) call->code[j] = pass ? 1 : 0;
        } else {
          again.insert(again.end(), tj.begin(), tj.end());
        }
      }
      if (failing.empty()) again = [&] {  // never expected: every job alone
        std::vector<size_t> all;
        for (const auto& tj : pu.test_jobs) all.insert(all.end(), tj.begin(), tj.end());
        return all;
      }();
      if (!again.empty()) {
        call->units.push_back(again);
        call->unit_group.push_back((int)pu.group);
        call->unit_rounds.push_back(2);
        call->unit_idx.emplace_back();
        call->unit_dmask.push_back(0);
      }
      continue;
    }
    const size_t n = pu.jobs.size(), k = pu.tests.size();
    std::vector<size_t> cand;
    for (size_t i = 0; i < n; ++i) {
      bool in_passing = false;  // in S_b (bit b of i set) or its complement, and that set passed
      for (size_t b = 0; b < k && !in_passing; ++b) in_passing = (rv[pu.tests[b]] >> (((i >> b) & 1) ? 0 : 1)) & 1;
      if (in_passing)
        call->code[pu.jobs[i]] = 1;
      else
        cand.push_back(pu.jobs[i]);
    }
    if (trace_on()) fprintf(stderr, "[bgv]   pattern unit: %zu jobs, %zu tests, %zu candidates\n", n, k, cand.size());
    if (cand.size() == 1) {
      call->code[cand[0]] = 0;  // the group failed and every invalid job is a candidate
    } else {
      // two or more invalid jobs (or, never expected, none left: test every job alone); D =
      // the bits where S_b and its complement both failed
      uint32_t D = 0;
      for (size_t b = 0; b < k; ++b)
        if (!(rv[pu.tests[b]] & 1) && !((rv[pu.tests[b]] >> 1) & 1)) D |= 1u << b;
      std::vector<uint32_t> idx;
      if (!cand.empty())
        for (size_t i = 0; i < n; ++i)
          if (std::find(cand.begin(), cand.end(), pu.jobs[i]) != cand.end()) idx.push_back((uint32_t)i);
      // every index bit with both S_b and its complement failing (D covers all k bits: every
      // job a candidate) means many invalid jobs (two have all their index bits apart with
      // probability 1/(n-1)): the next round tests them one by one (no D: singles) instead of
      // pairs whose failures would need a third round
#ifndef BGV_RETRY_ALLBITS_SINGLES
#define BGV_RETRY_ALLBITS_SINGLES 1  // A/B: 0 keeps the pairs round for every unit with a D
#endif
      const bool all_bits = BGV_RETRY_ALLBITS_SINGLES && k > 0 && D == (k >= 32 ? 0xffffffffu : ((1u << k) - 1u));
      call->units.push_back(cand.empty() ? pu.jobs : cand);
      call->unit_group.push_back((int)pu.group);
      call->unit_rounds.push_back(1);
      call->unit_dmask.push_back(cand.empty() || all_bits ? 0 : D);
      call->unit_idx.push_back(std::move(idx));
    }
  }
  call->parts.clear();
  call->punits.clear();
}

// Run one merged super-batch of calls on one dispatcher's stream.
static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}


static bool needs_retry(const std::vector<Call*>& calls) {
  for (const Call* call : calls)
    if (!call->units.empty()) return true;
  return false;
}

// The first pass of one merged super-batch on the dispatcher's stream x.main: layout merge,
// per-set kernels, the groups' closing, verdicts; leaves the retry units in the calls.
static int run_pass1(bgv_ctx* c, Device& d, Exec& x, std::vector<Call*>& calls, BatchState& bs) {
  const auto tb = std::chrono::steady_clock::now();
  bs.tb = tb;
  double t_merge = 0, t_tok = 0, t_sets = 0, t_pass1 = 0, t_post = 0;
  // merge the calls' layouts
  uint32_t nslots = 0, ngroups = 0;
  size_t nidx = 0, npkb = 0, nuniq = 0;
  bool any_uniform = false;
  for (Call* call : calls) {
    call->slot_base = nslots;
    nslots += (uint32_t)call->L.slots.size();
    ngroups += (uint32_t)call->L.groups.size();
    nidx += call->L.idx.size();
    npkb += call->L.pkb.size();
    nuniq += call->L.uniq.size();
    for (char u : call->L.group_uniform) any_uniform = any_uniform || u;
  }
  const bool bulk = nslots + ngroups > bgv_fold_pairs_max();
  // uniform groups (BGV_GROUP_UNIFORM): bulk batches on the two-phase Miller stage
  const bool uniform = uniform_enabled() && any_uniform && bulk && !bgv_single_pass_miller();
  HIPCHK(hipSetDevice(d.id));
  int rc;
  if ((rc = exec_reserve_slots(x, nslots)) || (rc = exec_reserve_groups(x, ngroups)) ||
      (rc = grow(&x.d_idx, &x.idx_cap, std::max<size_t>(nidx + nuniq, 1))) ||
      (rc = grow(&x.d_pkb, &x.pkb_cap, std::max<size_t>(npkb, 1))))
    return rc;
  HIPCHK(x.h_slots.reserve(nslots));
  HIPCHK(x.h_groups.reserve(std::max<size_t>(ngroups, 1)));
  HIPCHK(x.h_idx.reserve(nidx + nuniq));  // pubkey indices, then the hashed slots (b.uniq)
  HIPCHK(x.h_pkb.reserve(npkb));
  HIPCHK(x.h_ss.reserve(nslots));
  HIPCHK(x.h_ps.reserve(nslots));
  HIPCHK(x.h_verdict.reserve(std::max<size_t>(ngroups, 1)));
  bgv_dslot* slots = x.h_slots.p;
  bgv_dgroup* groups = x.h_groups.p;
  uint32_t max_npk = 0;
  {
    size_t ns = 0, ng = 0, ni = 0, npb = 0;
    for (Call* call : calls) {
      const uint32_t ib = (uint32_t)ni, pb = (uint32_t)(npb / 96), gb = (uint32_t)ng;
      if (ns == 0 && ib == 0 && pb == 0 && gb == 0) {  // the first call: its layout as it is
        const bgv_dslot* src = call->L.slots.data();
        std::atomic<uint32_t> mx{0};
        par_ranges(call->L.slots.size(), [&](size_t lo, size_t hi) {
          memcpy(slots + lo, src + lo, sizeof(bgv_dslot) * (hi - lo));
          uint32_t m = 0;
          for (size_t i = lo; i < hi; ++i) m = std::max(m, src[i].n_pk);
          uint32_t cur = mx.load();
          while (m > cur && !mx.compare_exchange_weak(cur, m)) {
          }
        });
        max_npk = std::max(max_npk, mx.load());
        ns = call->L.slots.size();
      } else {
        for (bgv_dslot s : call->L.slots) {
          s.hsrc += call->slot_base;
          if (s.flags & BGV_SLOT_PK_CACHED) s.pk_off += ib;
          if (s.flags & BGV_SLOT_PK_BYTES) s.pk_off += pb;
          if (!(s.flags & BGV_SLOT_PAD)) s.group += gb;
          max_npk = std::max(max_npk, s.n_pk);
          slots[ns++] = s;
        }
      }
      for (size_t gi = 0; gi < call->L.groups.size(); ++gi) {
        const bgv_dgroup& g = call->L.groups[gi];
        groups[ng++] = bgv_dgroup{g.first_slot + call->slot_base, g.n_slots, g.mask, 0,
                                  uniform && call->L.group_uniform[gi] ? BGV_GROUP_UNIFORM : 0u};
      }
      if (!call->L.idx.empty()) memcpy(x.h_idx.p + ni, call->L.idx.data(), 4 * call->L.idx.size());
      ni += call->L.idx.size();
      if (!call->L.pkb.empty()) memcpy(x.h_pkb.p + npb, call->L.pkb.data(), call->L.pkb.size());
      npb += call->L.pkb.size();
    }
    uint32_t* u = x.h_idx.p + nidx;
    for (Call* call : calls)
      for (uint32_t v : call->L.uniq) *u++ = v + call->slot_base;
  }
  std::vector<uint64_t> sc(nslots);
  fill_scalars(c, sc.data(), nslots);
  par_ranges(nslots, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) slots[i].scalar = sc[i];
  });

  bool prof;
  {
    std::lock_guard<std::mutex> lk(c->prof_mu);
    prof = c->profile;
  }
  t_merge = ms_since(tb);
  if (c->fault_inject) HIPCHK(hipErrorLaunchFailure);
  HIPCHK(hipMemcpyAsync(x.d_slots, slots, sizeof(bgv_dslot) * nslots, hipMemcpyHostToDevice, x.main));
  HIPCHK(hipMemcpyAsync(x.d_groups, groups, sizeof(bgv_dgroup) * ngroups, hipMemcpyHostToDevice, x.main));
  if (nidx + nuniq) HIPCHK(hipMemcpyAsync(x.d_idx, x.h_idx.p, 4 * (nidx + nuniq), hipMemcpyHostToDevice, x.main));
  if (npkb) HIPCHK(hipMemcpyAsync(x.d_pkb, x.h_pkb.p, npkb, hipMemcpyHostToDevice, x.main));
  bgv_dev_batch b = make_batch(d, x, nslots, ngroups);
  b.max_npk = max_npk;
  b.uniform = uniform;
  bs.uniform = uniform;
  b.uniq = x.d_idx + nidx;
  b.nuniq = (uint32_t)nuniq;
  if (int lrc = exec_reserve_lines(x, b)) return lrc;
  bgv_streams S{x.main, prof ? x.kev : nullptr};
  int32_t *ss = x.h_ss.p, *ps = x.h_ps.p, *verdict = x.h_verdict.p;
  {
    // One super-batch at a time runs k_prep (the token); the token passes on as
    // soon as k_prep is done, so the next batch's k_prep waves queue behind this
    // batch's k_miller and take each SIMD as a Miller wave retires (no drain
    // bubble between batches).  The group closing follows on the same stream.
    const auto tt = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> tok(*d.compute_mu);
    t_tok = ms_since(tt);
    HIPCHK(hipEventRecord(x.ev0, x.main));
    HIPCHK(bgv_launch_prep(b, S));
    HIPCHK(hipEventRecord(x.ev_prep, x.main));
    HIPCHK(bgv_launch_miller(b, S));
    HIPCHK(hipEventRecord(x.ev_sets, x.main));
    HIPCHK(hipEventSynchronize(x.ev_prep));
    t_sets = ms_since(tt) - t_tok;
  }
  const auto tg = std::chrono::steady_clock::now();
  HIPCHK(bgv_launch_groups(b, S, false));
  HIPCHK(hipEventRecord(x.ev1, x.main));
  HIPCHK(hipMemcpyAsync(ss, b.sig_status, 4ull * nslots, hipMemcpyDeviceToHost, x.main));
  HIPCHK(hipMemcpyAsync(ps, b.pk_status, 4ull * nslots, hipMemcpyDeviceToHost, x.main));
  HIPCHK(hipMemcpyAsync(verdict, b.verdict, 4ull * ngroups, hipMemcpyDeviceToHost, x.main));
  HIPCHK(hipStreamSynchronize(x.main));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, x.ev0, x.ev1));
  exec_trim_lines(x, c->max_slots.load());  // the records are dead once the first pass is done
  if (prof) prof_add(c, x, true, true);
  t_pass1 = ms_since(tg);
  const auto tp = std::chrono::steady_clock::now();
  std::vector<uint32_t>& call_gb = bs.call_gb;
  bool& want_gu = bs.want_gu;
  {
    uint32_t gb = 0;
    for (Call* call : calls) {
      call->st.device_ms += ms;
      call_after_pass1(call, ss + call->slot_base, ps + call->slot_base, verdict + gb);
      call_gb.push_back(gb);
      gb += (uint32_t)call->L.groups.size();
      for (size_t u = 0; u < call->units.size() && !want_gu; ++u) want_gu = pattern_eligible(call, u);
    }
  }
  if (want_gu) {  // the first pass's u values of the groups, before a retry round reuses the array
    if ((rc = grow(&x.d_gu1, &x.gu1_cap, ngroups))) return rc;
    HIPCHK(hipMemcpyAsync(x.d_gu1, b.gu, sizeof(fp12_t) * ngroups, hipMemcpyDeviceToDevice, x.main));
  }
  {
    // bgv_verify_partial calls: the product of the call's groups (before any retry round
    // reuses the per-group arrays), serialized on the device
    uint32_t gb = 0, np = 0, maxg = 0;
    for (Call* call : calls) {
      if (call->partial_out) {
        ++np;
        maxg = std::max<uint32_t>(maxg, (uint32_t)call->L.groups.size());
      }
    }
    if (np) {
      if ((rc = grow(reinterpret_cast<uint8_t**>(&x.d_pscratch), &x.pscratch_cap,
                     bgv_fp12_bytes() * (maxg / 32 + 4))) ||
          (rc = grow(&x.d_pout, &x.pout_cap, 576)))
        return rc;
      for (Call* call : calls) {
        const uint32_t ng = (uint32_t)call->L.groups.size();
        if (call->partial_out) {
          HIPCHK(bgv_launch_partial(b, gb, ng, x.d_pscratch, x.d_pout, x.main));
          HIPCHK(hipMemcpyAsync(call->partial_out, x.d_pout, 576, hipMemcpyDeviceToHost, x.main));
          HIPCHK(hipStreamSynchronize(x.main));
        }
        gb += ng;
      }
    }
  }
  HIPCHK(hipStreamSynchronize(x.main));  // the u copy, before the Exec changes hands
  t_post = ms_since(tp);
  bs.t_merge = t_merge;
  bs.t_tok = t_tok;
  bs.t_sets = t_sets;
  bs.t_pass1 = t_pass1;
  bs.t_post = t_post;
  bs.nslots = nslots;
  bs.ngroups = ngroups;
  bs.prof = prof;
  if (trace_on() && !needs_retry(calls))
    fprintf(stderr,
            "[bgv] dev %d calls %zu slots %u groups %u | submit..dispatch %.1f | merge %.1f tokwait %.1f sets %.1f "
            "groups %.1f post %.1f total %.1f ms\n",
            d.id, calls.size(), nslots, ngroups,
            std::chrono::duration<double, std::milli>(tb - calls.front()->t0).count(), t_merge, t_tok, t_sets,
            t_pass1, t_post, ms_since(tb));
  return BGV_OK;
}

// The retry rounds of a super-batch after run_pass1, on x.close (the device's retry stream),
// over the per-slot results the first pass left in x's buffers.
// One super-batch in its retry rounds on a retry thread (retry_loop): the rounds of every batch
// the thread holds are launched back to back on its stream and waited for together, so a
// round's launch-to-verdict latency is paid once for all of them.
struct RetryRun {
  RetryJob job;
  int rounds = 0;
  uint32_t nrg = 0;  // groups of the round in flight (0: none)
  double t_build = 0;
  std::chrono::steady_clock::time_point tr;
};

// Builds r's next round and enqueues it on its Exec's retry stream (groups up, kernels,
// verdicts down).  *more = false: the batch has no parts left (its rounds are done).
static int retry_launch(Device& d, RetryRun& r, bool* more) {
  Exec& x = *r.job.x;
  std::vector<Call*>& calls = r.job.calls;
  BatchState& bs = *r.job.st;
  const auto th = std::chrono::steady_clock::now();
  std::vector<bgv_dgroup> rg;
  for (size_t k = 0; k < calls.size(); ++k)
    call_build_parts(calls[k], rg, bs.want_gu ? (int64_t)bs.call_gb[k] : -1, bs.uniform);
  *more = !rg.empty();
  r.nrg = 0;
  if (rg.empty()) return BGV_OK;
  ++r.rounds;
  const uint32_t nrg = (uint32_t)rg.size();
  // the tests inside uniform first-pass groups (they pair their pubkey sums, bgv_launch_gpairs),
  // listed after the groups in the same upload
  std::vector<uint32_t> upk;
  if (bs.uniform)
    for (uint32_t t = 0; t < nrg; ++t)
      if (rg[t].flags & BGV_GROUP_UNIFORM) upk.push_back(t);
  const uint32_t per = (uint32_t)(sizeof(bgv_dgroup) / sizeof(uint32_t));
  const uint32_t nlist = ((uint32_t)upk.size() + per - 1) / per;  // in bgv_dgroup units
  int rc;
  if ((rc = exec_reserve_groups(x, nrg + nlist))) return rc;
  HIPCHK(x.h_groups.reserve(nrg + nlist));
  HIPCHK(x.h_verdict.reserve(nrg));
  memcpy(x.h_groups.p, rg.data(), sizeof(bgv_dgroup) * nrg);
  if (!upk.empty()) memcpy(x.h_groups.p + nrg, upk.data(), 4 * upk.size());
  HIPCHK(hipMemcpyAsync(x.d_groups, x.h_groups.p, sizeof(bgv_dgroup) * (nrg + nlist), hipMemcpyHostToDevice,
                        x.close));
  bgv_dev_batch b = make_batch(d, x, bs.nslots, nrg);
  b.uniform = !upk.empty();
  b.upk = reinterpret_cast<const uint32_t*>(b.groups + nrg);
  b.npk = (uint32_t)upk.size();
  for (const bgv_dgroup& t : rg) b.weighted = b.weighted || (t.flags & BGV_GROUP_WEIGHTED);
  bool pattern = false;
  for (Call* call : calls) pattern = pattern || !call->punits.empty();
  if (pattern) b.gu1 = x.d_gu1;
  r.t_build = ms_since(th);
  bgv_streams SC{x.close, bs.prof ? x.kev : nullptr};
  HIPCHK(hipEventRecord(x.ev0, x.close));
  HIPCHK(bgv_launch_groups(b, SC, true));
  HIPCHK(hipEventRecord(x.ev1, x.close));
  HIPCHK(hipMemcpyAsync(x.h_verdict.p, b.verdict, 4ull * nrg, hipMemcpyDeviceToHost, x.close));
  r.nrg = nrg;
  return BGV_OK;
}

// After the stream has drained: the round's verdicts into r's calls
static int retry_complete(bgv_ctx* c, RetryRun& r, double t_wait) {
  Exec& x = *r.job.x;
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, x.ev0, x.ev1));
  if (r.job.st->prof) prof_add(c, x, false, true);
  if (trace_on()) {
    size_t npt = 0;
    for (Call* call : r.job.calls)
      for (const PatternUnit& pu : call->punits) npt += pu.tests.size();
    fprintf(stderr,
            "[bgv]  round %d: %u groups (%zu tests with a reference), host %.2f, launch..verdicts %.2f, device %.2f ms, "
            "since round start %.1f ms\n",
            r.rounds, r.nrg, npt, r.t_build, t_wait, ms, ms_since(r.tr));
  }
  for (Call* call : r.job.calls) {
    call->st.device_ms += ms;
    uint32_t mine = 0;
    for (const Part& p : call->parts) mine += (uint32_t)p.groups.size();
    call->st.device_groups += mine;
    call_after_round(call, x.h_verdict.p);  // part group indices are global to this round
  }
  r.nrg = 0;
  return BGV_OK;
}

static void retry_trace_done(const Device& d, const RetryRun& r) {
  if (!trace_on()) return;
  const BatchState& bs = *r.job.st;
  fprintf(stderr,
          "[bgv] dev %d calls %zu slots %u groups %u | merge %.1f tokwait %.1f sets %.1f groups %.1f post %.1f "
          "retry(%d) %.1f total %.1f ms\n",
          d.id, r.job.calls.size(), bs.nslots, bs.ngroups, bs.t_merge, bs.t_tok, bs.t_sets, bs.t_pass1, bs.t_post,
          r.rounds, ms_since(r.tr), ms_since(bs.tb));
}

static Exec* exec_acquire(Device& d) {
  DevSched& s = *d.sched;
  std::unique_lock<std::mutex> lk(s.mu);
  s.cv.wait(lk, [&s] { return !s.free.empty(); });
  // the most recently released buffer set first: on a quiet device the same warm Exec serves
  // call after call (a huge call's first use of an Exec pins ~170 MB of staging)
  Exec* x = s.free.back();
  s.free.pop_back();
  return x;
}

static void exec_release(Device& d, Exec* x) {
  DevSched& s = *d.sched;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.free.push_back(x);
  }
  s.cv.notify_all();
}

static void finish_calls(std::vector<Call*>& calls, int rc) {
  for (Call* call : calls) {
    if (rc != BGV_OK)
      call_fail(call, rc);
    else
      call_finish(call);
  }
}

// The device's retry thread: the retry rounds of handed-over super-batches, in order; drains
// the queue before it stops.
// The retry thread holds up to retry_hold_max() handed-over batches and runs their rounds side by side: each
// pass launches one round of every held batch on the thread's stream, waits once, and applies
// the verdicts; a batch joins at the next pass after its hand-over and leaves (its calls
// finished, its Exec released) when it has no parts left.  Under load, when hand-overs queue up,
// several batches share each launch-to-verdict wait instead of taking turns.
static void retry_loop(bgv_ctx* c, Device* d, int k) {
  DevSched& s = *d->sched;
  (void)hipSetDevice(d->id);
  hipStream_t st = s.retries[k];
  std::vector<RetryRun> held;
  auto leave = [&](size_t i, int rc) {
    finish_calls(held[i].job.calls, rc);
    exec_release(*d, held[i].job.x);
    c->running.fetch_sub(1);
    held.erase(held.begin() + (std::ptrdiff_t)i);
  };
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(s.mu);
      if (held.empty()) s.cv.wait(lk, [&s] { return s.stop || !s.rq.empty(); });
      if (held.empty() && s.rq.empty()) return;  // stopping, and the queue is drained
      while (!s.rq.empty() && held.size() < retry_hold_max()) {
        RetryRun r;
        r.job = std::move(s.rq.front());
        s.rq.pop_front();
        r.job.x->close = st;
        r.tr = std::chrono::steady_clock::now();
        // No cache_mu here: the retry kernels (k_gsum, the group pairs, the closing) read only
        // the per-slot results of pass 1 (r_i sig_i, r_i pk_i, f_i, H, u values), never the
        // pubkey cache, and bgv_close joins this thread before it frees the devices.  A batch in
        // its retry rounds keeps the device busy, so it counts as running for the coalescing
        // window.
        c->running.fetch_add(1);
        held.push_back(std::move(r));
      }
    }
    (void)hipSetDevice(d->id);
    for (size_t i = 0; i < held.size();) {
      bool more = false;
      const int rc = retry_launch(*d, held[i], &more);
      if (rc != BGV_OK) {  // a device error fails this batch's calls; the others go on
        (void)hipStreamSynchronize(st);
        leave(i, rc);
      } else if (!more) {
        retry_trace_done(*d, held[i]);
        leave(i, BGV_OK);
      } else {
        ++i;
      }
    }
    if (held.empty()) continue;
    const auto tl = std::chrono::steady_clock::now();
    const hipError_t e = hipStreamSynchronize(st);
    const double t_wait = ms_since(tl);
    for (size_t i = 0; i < held.size();) {
      const int rc = e == hipSuccess ? retry_complete(c, held[i], t_wait) : -BGV_E_DEVICE;
      if (rc != BGV_OK)
        leave(i, rc);
      else
        ++i;
    }
  }
}

static void dispatcher_loop(bgv_ctx* c, Device* d, hipStream_t stream) {
  (void)hipSetDevice(d->id);
  const int di = (int)(d - c->devs.data());
  // a call pinned to another device (a shard of a split call, verify_split) is not ours
  auto mine = [di](const Call* q) { return q->dev < 0 || q->dev == di; };
  auto any_mine = [c, &mine] {
    for (Call* q : c->queue)
      if (mine(q)) return true;
    return false;
  };
  for (;;) {
    std::vector<Call*> calls;
    {
      std::unique_lock<std::mutex> lk(c->qmu);
      c->qcv.wait(lk, [c, &any_mine] { return c->stop || any_mine(); });
      if (!any_mine()) return;  // stopping, and nothing of ours left to drain
      // Coalescing window: a super-batch costs about the same device time from a
      // few thousand to ~10^5 sets (its closing phases are latency-bound), so give
      // concurrent callers a moment to join before launching.
      auto queued_slots = [c, &mine] {
        size_t n = 0;
        for (Call* q : c->queue)
          if (mine(q)) n += q->L.slots.size();
        return n;
      };
      const size_t cap = c->max_slots.load();
      // a full window only while another super-batch keeps the device busy anyway
      const size_t win = c->running.load() > 0 ? c->coalesce.load()
                                               : std::min<size_t>(c->coalesce.load(), c->idle_coalesce.load());
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(win);
      while (!c->stop && queued_slots() < cap &&
             c->qcv.wait_until(lk, until) != std::cv_status::timeout) {
      }
      if (!any_mine()) continue;
      size_t slots = 0;
      for (auto it = c->queue.begin(); it != c->queue.end();) {
        Call* call = *it;
        if (!mine(call)) {
          ++it;
          continue;
        }
        const size_t n = call->L.slots.size();
        if (!calls.empty() && slots + n > cap) break;
        calls.push_back(call);
        slots += n;
        it = c->queue.erase(it);
      }
      if (!c->queue.empty()) c->qcv.notify_all();
    }
    Exec* x = exec_acquire(*d);
    x->main = stream;
    auto bs = std::make_shared<BatchState>();
    int rc;
    {
      std::shared_lock<std::shared_mutex> clk(c->cache_mu);
      c->running.fetch_add(1);
      rc = run_pass1(c, *d, *x, calls, *bs);
      c->running.fetch_sub(1);
    }
    if (rc == BGV_OK && needs_retry(calls)) {
      DevSched& s = *d->sched;
      {
        std::lock_guard<std::mutex> lk(s.mu);
        s.rq.push_back(RetryJob{std::move(calls), x, bs});
      }
      s.cv.notify_all();
      continue;
    }
    finish_calls(calls, rc);
    exec_release(*d, x);
  }
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

static void ctx_free_devices(bgv_ctx* c) {
  for (Device& d : c->devs) {
    if (!d.stream) continue;  // never set up (e.g. an index past the device count)
    (void)hipSetDevice(d.id);
    for (Exec* x : d.execs) exec_destroy(x);
    d.execs.clear();
    d.sched->free.clear();
    for (hipStream_t st : d.sched->dstreams) (void)hipStreamDestroy(st);
    d.sched->dstreams.clear();
    for (hipStream_t st : d.sched->retries) (void)hipStreamDestroy(st);
    d.sched->retries.clear();
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    if (d.cache) (void)hipFree(d.cache);
    d.cache = nullptr;
    {
      FinalScratch& fs = d.final_scratch;
      void* bufs[] = {fs.din, fs.vals, fs.one, fs.dg, fs.dst, fs.dv};
      for (void* q : bufs)
        if (q) (void)hipFree(q);
      fs = FinalScratch{};
    }
    if (d.stream) (void)hipStreamDestroy(d.stream);
    d.stream = nullptr;
  }
}

int bgv_init(const int* devices, int ndev, bgv_ctx** out) {
  if (!out) return -BGV_E_ARG;
  *out = nullptr;
  int avail = bgv_device_count();
  if (avail <= 0) return -BGV_E_DEVICE;
  bgv_ctx* c = new bgv_ctx();
  {
    const char* fi = getenv("BGV_FAULT_INJECT");
    c->fault_inject = fi && atoi(fi) > 0;
  }
  c->max_slots = (uint32_t)max_batch_slots();
  c->coalesce = (uint32_t)coalesce_us();
  c->idle_coalesce = (uint32_t)idle_coalesce_us();
  c->split_min = (uint32_t)split_min_env();
  const int n = (devices && ndev > 0) ? ndev : 1;
  c->devs.resize(n);
  for (int i = 0; i < n; ++i) {
    Device& d = c->devs[i];
    d.id = (devices && ndev > 0) ? devices[i] : 0;
    bool ok = d.id >= 0 && d.id < avail && hipSetDevice(d.id) == hipSuccess &&
              hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) == hipSuccess;
    int least = 0, greatest = 0;
    ok = ok && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess;
    // high priority: at normal priority the mainnet-shaped leg measured 2.30-2.73 against
    // 3.21-3.27 M sets/s (profiles/r05/uniform/mainnet_probe_r05g.jsonl)
    for (int k = 0; ok && k < retry_threads_per_device(); ++k) {
      hipStream_t st = nullptr;
      ok = hipStreamCreateWithPriority(&st, hipStreamNonBlocking, greatest) == hipSuccess;
      if (ok) d.sched->retries.push_back(st);
    }
    for (int k = 0; ok && k < dispatchers_per_device(); ++k) {
      hipStream_t st = nullptr;
      ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
      if (ok) d.sched->dstreams.push_back(st);
    }
    for (int k = 0; ok && k < execs_per_device(); ++k) {
      Exec* x = new Exec();
      d.execs.push_back(x);
      ok = exec_create(x) == BGV_OK;
      if (ok) d.sched->free.push_back(x);
    }
    if (!ok) {
      ctx_free_devices(c);
      delete c;
      (void)hipGetLastError();  // no stale error for the launch checks of later calls
      return d.id < 0 || d.id >= avail ? -BGV_E_ARG : -BGV_E_DEVICE;
    }
  }
  for (Device& d : c->devs) {
    for (hipStream_t st : d.sched->dstreams) c->dispatchers.emplace_back(dispatcher_loop, c, &d, st);
    for (int k = 0; k < (int)d.sched->retries.size(); ++k) d.sched->retry_threads.emplace_back(retry_loop, c, &d, k);
  }
  *out = c;
  return BGV_OK;
}

int bgv_close(bgv_ctx* c) {
  if (!c) return -BGV_E_ARG;
  {
    // asynchronous split calls finish first: their pieces need the dispatchers
    std::unique_lock<std::mutex> lk(c->split_mu);
    c->split_closing = true;
    c->split_cv.wait(lk, [c] { return c->split_inflight == 0; });
  }
  {
    std::lock_guard<std::mutex> lk(c->qmu);
    c->stop = true;
  }
  c->qcv.notify_all();
  for (auto& w : c->dispatchers)
    if (w.joinable()) w.join();
  c->dispatchers.clear();
  // the retry threads finish the super-batches handed to them, then stop
  for (Device& d : c->devs) {
    {
      std::lock_guard<std::mutex> lk(d.sched->mu);
      d.sched->stop = true;
    }
    d.sched->cv.notify_all();
    for (auto& t : d.sched->retry_threads)
      if (t.joinable()) t.join();
    d.sched->retry_threads.clear();
  }
  std::unique_lock<std::shared_mutex> lk(c->cache_mu);
  if (c->closed.exchange(true)) return BGV_OK;
  ctx_free_devices(c);
  return BGV_OK;
}

int bgv_destroy(bgv_ctx* c) {
  if (!c) return -BGV_E_ARG;
  bgv_close(c);
  delete c;
  return BGV_OK;
}

int bgv_set_batching(bgv_ctx* c, uint32_t max_batch_slots, uint32_t coalesce_us, uint32_t idle_coalesce_us) {
  if (!c) return -BGV_E_ARG;
  if (max_batch_slots) c->max_slots = std::max<uint32_t>(max_batch_slots, BGV_WAVE);
  if (coalesce_us != UINT32_MAX) c->coalesce = coalesce_us;
  if (idle_coalesce_us != UINT32_MAX) c->idle_coalesce = idle_coalesce_us;
  return BGV_OK;
}

int bgv_set_rng_seed(bgv_ctx* c, uint64_t seed) {
  if (!c) return -BGV_E_ARG;
  std::lock_guard<std::mutex> lk(c->rng_mu);
  c->rng_seed = seed;
  c->rng_state = seed;
  return BGV_OK;
}

size_t bgv_pubkeys_count(const bgv_ctx* c) { return c ? c->n_pubkeys.load() : 0; }

// grow every device's cache to hold `need` entries (contents preserved); caller holds cache_mu exclusively
static int cache_reserve(bgv_ctx* c, size_t need) {
  const size_t esz = bgv_cache_entry_bytes();
  for (Device& d : c->devs) {
    HIPCHK(hipSetDevice(d.id));
    if (need <= d.cache_cap) continue;
    size_t cap = std::max(need, d.cache_cap * 2);
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, esz * cap));
    if (d.cache) {
      HIPCHK(hipMemcpyAsync(p, d.cache, esz * c->n_pubkeys, hipMemcpyDeviceToDevice, d.stream));
      HIPCHK(hipStreamSynchronize(d.stream));
      HIPCHK(hipFree(d.cache));
    }
    d.cache = static_cast<bgv_cache_entry*>(p);
    d.cache_cap = cap;
  }
  return BGV_OK;
}

// Decode n records into per-device staging buffers (the slow part: host-to-device copy and
// one square root per compressed key) under the SHARED cache lock, so running and newly
// submitted verifies are never held up by it; then commit.  A pure append within capacity
// copies the staged entries past n_pubkeys and publishes the new count, still under the shared
// lock; growth, overwrites and undecodable records commit under the exclusive lock (rare: the
// capacity doubles, validator indices only grow).  Records that fail to decode are committed
// as marked indices (sets naming them reject with BGV_E_BAD_INDEX) and the first one's code is
// returned, so one bad key neither leaves a hole that blocks later appends nor reaches a
// verify as a usable key.
int bgv_pubkeys_put(bgv_ctx* c, uint32_t first, const uint8_t* keys, size_t n, int fmt) {
  if (!c || (n && !keys) || (fmt != BGV_PK_COMPRESSED && fmt != BGV_PK_UNCOMPRESSED)) return -BGV_E_ARG;
  std::lock_guard<std::mutex> plk(c->put_mu);
  const size_t esz = bgv_cache_entry_bytes();
  std::vector<void*> staged(c->devs.size(), nullptr);
  std::vector<int32_t> status(n, 0);
  auto free_staged = [&] {
    for (size_t di = 0; di < staged.size(); ++di)
      if (staged[di]) {
        (void)hipSetDevice(c->devs[di].id);
        (void)hipFree(staged[di]);
      }
  };
  {
    std::shared_lock<std::shared_mutex> clk(c->cache_mu);
    if (c->closed) return -BGV_E_CLOSED;
    if ((size_t)first > c->n_pubkeys) return -BGV_E_ARG;  // append or overwrite, no holes
    if (n == 0) return BGV_OK;
    std::lock_guard<std::mutex> ulk(c->util_mu);
    for (size_t di = 0; di < c->devs.size(); ++di) {
      Device& d = c->devs[di];
      // zeroed: k_cache_put writes no entry for an undecodable record
      if (hipSetDevice(d.id) != hipSuccess || hipMalloc(&staged[di], esz * n) != hipSuccess ||
          hipMemsetAsync(staged[di], 0, esz * n, d.stream) != hipSuccess) {
        free_staged();
        return -BGV_E_DEVICE;
      }
      const size_t chunk = 1 << 20;
      uint8_t* dk = nullptr;
      int32_t* dst = nullptr;
      int rc = BGV_OK;
      if (hipMalloc(reinterpret_cast<void**>(&dk), (size_t)fmt * std::min(n, chunk) + 1) != hipSuccess ||
          hipMalloc(reinterpret_cast<void**>(&dst), 4 * std::min(n, chunk) + 4) != hipSuccess)
        rc = -BGV_E_DEVICE;
      for (size_t off = 0; rc == BGV_OK && off < n; off += chunk) {
        const size_t m = std::min(chunk, n - off);
        bgv_cache_entry* out =
            reinterpret_cast<bgv_cache_entry*>(static_cast<uint8_t*>(staged[di]) + esz * off);
        if (hipMemcpyAsync(dk, keys + (size_t)fmt * off, (size_t)fmt * m, hipMemcpyHostToDevice, d.stream) !=
                hipSuccess ||
            bgv_launch_cache_put(dk, (uint32_t)m, fmt, out, dst, d.stream) != hipSuccess ||
            (di == 0 && hipMemcpyAsync(status.data() + off, dst, 4 * m, hipMemcpyDeviceToHost, d.stream) !=
                            hipSuccess) ||
            hipStreamSynchronize(d.stream) != hipSuccess)
          rc = -BGV_E_DEVICE;
      }
      if (dk) (void)hipFree(dk);
      if (dst) (void)hipFree(dst);
      if (rc) {
        free_staged();
        return rc;
      }
    }
  }
  int first_err = BGV_OK;
  std::vector<uint32_t> bad;
  for (size_t i = 0; i < n; ++i)
    if (status[i]) {
      if (first_err == BGV_OK) first_err = status[i];
      bad.push_back(first + (uint32_t)i);
    }
  const size_t need = (size_t)first + n;
  auto copy_in = [&]() -> int {
    for (size_t di = 0; di < c->devs.size(); ++di) {
      Device& d = c->devs[di];
      HIPCHK(hipSetDevice(d.id));
      HIPCHK(hipMemcpyAsync(reinterpret_cast<uint8_t*>(d.cache) + esz * first, staged[di], esz * n,
                            hipMemcpyDeviceToDevice, d.stream));
      HIPCHK(hipStreamSynchronize(d.stream));
    }
    return BGV_OK;
  };
  int rc = BGV_OK;
  bool done = false;
  {
    std::shared_lock<std::shared_mutex> clk(c->cache_mu);
    if (c->closed) {
      rc = -BGV_E_CLOSED;
      done = true;
    } else if (first == c->n_pubkeys && bad.empty()) {
      bool fits = true;
      for (const Device& d : c->devs) fits = fits && need <= d.cache_cap;
      if (fits) {
        std::lock_guard<std::mutex> ulk(c->util_mu);
        rc = copy_in();
        if (rc == BGV_OK) c->n_pubkeys.store(need);
        done = true;
      }
    }
  }
  if (!done) {
    std::unique_lock<std::shared_mutex> clk(c->cache_mu);
    if (c->closed) {
      rc = -BGV_E_CLOSED;
    } else {
      std::lock_guard<std::mutex> ulk(c->util_mu);
      rc = cache_reserve(c, need);
      // an undecodable record that overwrites an existing entry keeps the old entry: a call
      // that passed its index check before this put may still read it (later calls reject
      // the index with BGV_E_BAD_INDEX)
      const uint32_t old_n = (uint32_t)c->n_pubkeys.load();
      for (size_t di = 0; rc == BGV_OK && di < c->devs.size(); ++di) {
        Device& d = c->devs[di];
        if (hipSetDevice(d.id) != hipSuccess) rc = -BGV_E_DEVICE;
        for (uint32_t i : bad)
          if (rc == BGV_OK && i < old_n &&
              hipMemcpyAsync(static_cast<uint8_t*>(staged[di]) + esz * (i - first),
                             reinterpret_cast<const uint8_t*>(d.cache) + esz * i, esz, hipMemcpyDeviceToDevice,
                             d.stream) != hipSuccess)
            rc = -BGV_E_DEVICE;
      }
      if (rc == BGV_OK) rc = copy_in();
      if (rc == BGV_OK) {
        for (uint32_t i = first; i < need; ++i) c->bad_pk.erase(i);  // overwritten entries
        for (uint32_t i : bad) c->bad_pk.insert(i);
        c->n_pubkeys.store(std::max(c->n_pubkeys.load(), need));
      }
    }
  }
  free_staged();
  if (rc) return rc;
  return first_err ? -first_err : BGV_OK;
}

// ---------------------------------------------------------------------------
// One call over several devices (a context on a device list; SURVEY 8(e) inside the library).
// The reference splits a big call into >= 128-set jobs for its workers
// (chain/bls/multithread/index.ts:153-166; range sync hands ~8000 sets at once, :34); here a
// call of at least split_min sets is spread over the context's devices:
//   * a job of at least split_min sets is cut into one contiguous run of sets per device; each
//     run's Miller-loop product (576 B, bgv_verify_partial's) is computed on its device, the
//     partials are combined with ONE final exponentiation (bgv_final_verify on the first
//     device), and the job's code follows the reference's precedence: the first undecodable
//     signature in set order, then the pubkey condition, then the verdict;
//   * the other jobs go to the devices in contiguous runs balanced by set count, each run one
//     call pinned to its device (retry rounds stay on the device that ran the first pass).
// Codes are those of the same call on one device (tests/test_gpu_r04.py).
// ---------------------------------------------------------------------------
static int partial_submit(bgv_ctx* c, Call* call, const bgv_set* sets, size_t nsets, uint8_t* out576,
                          int32_t* out_codes, int dev);
static int call_wait(Call* call);
static int partial_finish(Call* call, int rc, int32_t* out_codes);

static size_t split_min_sets(const bgv_ctx* c) {
  return c->split_min.load();
}

static void stats_add(bgv_stats* a, const bgv_stats& b) {
  a->batch_retries += b.batch_retries;
  a->batch_sigs_success += b.batch_sigs_success;
  a->device_groups += b.device_groups;
  a->sets_verified += b.sets_verified;
  a->device_ms = std::max(a->device_ms, b.device_ms);
}

static bool split_wanted(const bgv_ctx* c, size_t nsets) {
  return c->devs.size() > 1 && split_min_sets(c) > 0 && nsets >= split_min_sets(c);
}

// A split call registers itself before it submits anything (false: the context is closing)
// and deregisters when it no longer touches the context; bgv_close waits for the count to
// drop to zero.  The notify happens under split_mu, so a woken bgv_close (and the
// bgv_destroy after it) cannot free the context before split_leave has returned.
static bool split_enter(bgv_ctx* c) {
  std::lock_guard<std::mutex> lk(c->split_mu);
  if (c->split_closing) return false;
  ++c->split_inflight;
  return true;
}

static void split_leave(bgv_ctx* c) {
  std::lock_guard<std::mutex> lk(c->split_mu);
  --c->split_inflight;
  c->split_cv.notify_all();
}

static int verify_split(bgv_ctx* c, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
                        int32_t* out, bgv_stats* stats) {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t K = c->devs.size(), big = split_min_sets(c);
  struct Shard {  // one run of a big job on one device
    Call call;
    size_t job;
    uint8_t part[576];
    int32_t codes[2] = {0, 0};
    int rc = BGV_OK;
  };
  struct Child {  // small jobs [j0, j1) pinned to one device
    Call call;
    std::vector<bgv_job> jobs;
    std::vector<int32_t> out;
    bgv_stats st{};
    size_t j0 = 0;
    int rc = BGV_OK;
  };
  std::vector<std::unique_ptr<Shard>> shards;
  std::vector<std::unique_ptr<Child>> kids;
  std::vector<size_t> small;
  size_t small_sets = 0;
  // a big job's host-side checks run on the whole job before it is cut, so they take
  // precedence over every shard's device statuses, as in the unsplit call (job_precheck)
  std::vector<int32_t> pre(njobs, 2);
  {
    std::shared_lock<std::shared_mutex> clk(c->cache_mu);
    for (size_t j = 0; j < njobs; ++j) {
      if ((size_t)jobs[j].first_set + jobs[j].n_sets > nsets) return -BGV_E_ARG;
      if (jobs[j].n_sets >= big && host_job_code(c, jobs[j], sets, &pre[j]) != BGV_OK) return -BGV_E_ARG;
    }
  }
  for (size_t j = 0; j < njobs; ++j) {
    if (jobs[j].n_sets >= big) continue;
    small.push_back(j);
    small_sets += jobs[j].n_sets;
  }
  int rc = BGV_OK;
  // small jobs: contiguous runs of the call's job order, about small_sets / K sets each
  {
    size_t i = 0, acc = 0;
    for (size_t d = 0; d < K && i < small.size(); ++d) {
      const size_t target = (small_sets * (d + 1) + K - 1) / K;
      auto kid = std::make_unique<Child>();
      kid->j0 = i;
      while (i < small.size() && (acc < target || kid->jobs.empty())) {
        kid->jobs.push_back(jobs[small[i]]);
        acc += jobs[small[i]].n_sets;
        ++i;
      }
      if (d == K - 1)
        while (i < small.size()) {
          kid->jobs.push_back(jobs[small[i]]);
          ++i;
        }
      kid->out.assign(kid->jobs.size(), 0);
      kid->rc = call_submit(c, &kid->call, kid->jobs.data(), kid->jobs.size(), sets, nsets, mode, kid->out.data(),
                            &kid->st, nullptr, nullptr, (int)d);
      if (kid->rc != BGV_OK && rc == BGV_OK) rc = kid->rc;
      kids.push_back(std::move(kid));
    }
  }
  // big jobs: one run of sets per device
  for (size_t j = 0; j < njobs; ++j) {
    const uint32_t n = jobs[j].n_sets;
    if (n < big || pre[j] != 2) continue;
    for (size_t d = 0; d < K; ++d) {
      const size_t lo = n * d / K, hi = n * (d + 1) / K;
      if (hi <= lo) continue;
      auto sh = std::make_unique<Shard>();
      sh->job = j;
      sh->rc = partial_submit(c, &sh->call, sets + jobs[j].first_set + lo, hi - lo, sh->part, sh->codes, (int)d);
      if (sh->rc != BGV_OK && rc == BGV_OK) rc = sh->rc;
      shards.push_back(std::move(sh));
    }
  }
  // every submitted piece completes before its memory goes away
  for (auto& k : kids)
    if (k->rc == BGV_OK) {
      k->rc = call_wait(&k->call);
      if (k->rc != BGV_OK && rc == BGV_OK) rc = k->rc;
    }
  for (auto& sh : shards)
    if (sh->rc == BGV_OK) {
      sh->rc = partial_finish(&sh->call, BGV_OK, sh->codes);
      if (sh->rc != BGV_OK && rc == BGV_OK) rc = sh->rc;
    }
  if (rc != BGV_OK) return rc;
  bgv_stats st{};
  for (auto& k : kids) {
    for (size_t q = 0; q < k->jobs.size(); ++q) out[small[k->j0 + q]] = k->out[q];
    stats_add(&st, k->st);
  }
  for (size_t j = 0; j < njobs; ++j) {
    if (jobs[j].n_sets < big) continue;
    if (pre[j] != 2) {
      out[j] = pre[j];
      continue;
    }
    int32_t code = 0;
    bool decided = false;
    std::vector<uint8_t> parts;
    for (auto& sh : shards)
      if (sh->job == j && sh->codes[0] && !decided) {  // first undecodable signature in set order
        code = sh->codes[0];
        decided = true;
      }
    for (auto& sh : shards)
      if (sh->job == j && sh->codes[1] && !decided) {  // then the first pubkey condition
        code = sh->codes[1] == 1 ? -BGV_BLST_PK_IS_INFINITY : sh->codes[1];
        decided = true;
      }
    if (!decided) {
      for (auto& sh : shards)
        if (sh->job == j) parts.insert(parts.end(), sh->part, sh->part + 576);
      int32_t v = 0;
      const int frc = bgv_final_verify(c, parts.data(), parts.size() / 576, &v);
      if (frc != BGV_OK) return frc;
      code = v ? 1 : 0;
    }
    out[j] = code;
    st.sets_verified += jobs[j].n_sets;
    st.device_groups += 1;
  }
  st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = st;
  return BGV_OK;
}

int bgv_set_split(bgv_ctx* c, uint32_t min_sets) {
  if (!c) return -BGV_E_ARG;
  // at least 2: a one-set job is never cut (its infinity-key verdict is false, not
  // BLST_PK_IS_INFINITY, which a shard's codes cannot tell apart)
  c->split_min = min_sets == 1 ? 2 : min_sets;
  return BGV_OK;
}

int bgv_verify(bgv_ctx* c, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
               int32_t* out, bgv_stats* stats) {
  if (!c) return -BGV_E_ARG;
  if (split_wanted(c, nsets)) {
    if (c->closed) return -BGV_E_CLOSED;
    if ((njobs && (!jobs || !out)) || (nsets && !sets)) return -BGV_E_ARG;
    if (mode != BGV_MODE_WORKER && mode != BGV_MODE_PER_JOB) return -BGV_E_ARG;
    if (!split_enter(c)) return -BGV_E_CLOSED;
    const int rc = verify_split(c, jobs, njobs, sets, nsets, mode, out, stats);
    split_leave(c);
    return rc;
  }
  Call* call = new Call();
  int rc = call_submit(c, call, jobs, njobs, sets, nsets, mode, out, stats, nullptr, nullptr);
  if (rc == BGV_OK) {
    std::unique_lock<std::mutex> lk(call->mu);
    call->cv.wait(lk, [call] { return call->finished; });
    rc = call->rc;
  }
  delete call;
  return rc;
}

int bgv_verify_async(bgv_ctx* c, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
                     int32_t* out, bgv_stats* stats, bgv_done_fn done, void* user) {
  if (!c) return -BGV_E_ARG;
  if (split_wanted(c, nsets)) {
    // a split call waits for its pieces and combines them: on a thread of its own (big calls
    // only), then done() as for any call
    if (c->closed) return -BGV_E_CLOSED;
    if ((njobs && (!jobs || !out)) || (nsets && !sets)) return -BGV_E_ARG;
    if (mode != BGV_MODE_WORKER && mode != BGV_MODE_PER_JOB) return -BGV_E_ARG;
    if (!split_enter(c)) return -BGV_E_CLOSED;
    std::thread([=] {
      const int rc = verify_split(c, jobs, njobs, sets, nsets, mode, out, stats);
      if (done) done(user, rc);
      split_leave(c);
    }).detach();
    return BGV_OK;
  }
  Call* call = new Call();
  call->owned = true;  // deleted by the dispatcher after done()
  int rc = call_submit(c, call, jobs, njobs, sets, nsets, mode, out, stats, done, user);
  if (rc != BGV_OK) delete call;
  return rc;
}

static void fp12_one_bytes(uint8_t out[576]) {
  memset(out, 0, 576);
  out[47] = 1;  // c0.c0.c0 = 1, big-endian
}

// One job's sets -> its Fp12 Miller-loop product and status codes on device dev (-1: any).
static int partial_submit(bgv_ctx* c, Call* call, const bgv_set* sets, size_t nsets, uint8_t* out576,
                          int32_t* out_codes, int dev) {
  out_codes[0] = out_codes[1] = 0;
  fp12_one_bytes(out576);
  call->partial_out = out576;
  call->partial_codes = out_codes;
  call->pjob = bgv_job{0, (uint32_t)nsets, 0};
  return call_submit(c, call, &call->pjob, 1, sets, nsets, BGV_MODE_PER_JOB, &call->pcode, nullptr, nullptr, nullptr,
                     dev);
}

static int call_wait(Call* call) {
  std::unique_lock<std::mutex> lk(call->mu);
  call->cv.wait(lk, [call] { return call->finished; });
  return call->rc;
}

static int partial_finish(Call* call, int rc, int32_t* out_codes) {
  if (rc == BGV_OK) rc = call_wait(call);
  if (rc == BGV_OK && call->pcode < 0 && call->pcode != -BGV_E_DEVICE) out_codes[0] = call->pcode;  // host-side
  return rc;
}

int bgv_verify_partial(bgv_ctx* c, const bgv_set* sets, size_t nsets, uint8_t out576[576], int32_t out_codes[2]) {
  if (!c || !out576 || !out_codes || (nsets && !sets)) return -BGV_E_ARG;
  out_codes[0] = out_codes[1] = 0;
  fp12_one_bytes(out576);
  if (nsets == 0) return c->closed ? -BGV_E_CLOSED : BGV_OK;  // an empty shard: the identity
  Call* call = new Call();
  const int rc = partial_finish(call, partial_submit(c, call, sets, nsets, out576, out_codes, -1), out_codes);
  delete call;
  return rc;
}

int bgv_final_verify(bgv_ctx* c, const uint8_t* partials, size_t n, int32_t* out_verdict) {
  if (!c || !out_verdict || (n && !partials) || n > (1u << 20)) return -BGV_E_ARG;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);
  if (c->closed) return -BGV_E_CLOSED;
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  const size_t m = std::max<size_t>(n, 1);
  std::vector<uint8_t> in(576 * m);
  if (n) memcpy(in.data(), partials, 576 * n);
  else fp12_one_bytes(in.data());
  // persistent buffers, grown to the largest n seen (a hipFree would synchronize the device
  // against the super-batches running on it)
  FinalScratch& fs = d.final_scratch;
  if (m > fs.cap) {
    void* bufs[] = {fs.din, fs.vals, fs.one, fs.dg, fs.dst, fs.dv};
    for (void* q : bufs)
      if (q) (void)hipFree(q);
    fs = FinalScratch{};
    const size_t cap = std::max<size_t>(m, 8);
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&fs.din), 576 * cap));
    HIPCHK(hipMalloc(&fs.vals, bgv_fp12_bytes() * cap));
    HIPCHK(hipMalloc(&fs.one, bgv_fp12_bytes()));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&fs.dg), sizeof(bgv_dgroup)));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&fs.dst), 4 * cap));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&fs.dv), 4));
    fs.cap = cap;
  }
  const bgv_dgroup g{0, (uint32_t)m, BGV_ALL_SLOTS};
  HIPCHK(hipMemcpyAsync(fs.din, in.data(), 576 * m, hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipMemcpyAsync(fs.dg, &g, sizeof(g), hipMemcpyHostToDevice, d.stream));
  HIPCHK(bgv_launch_final_verify(fs.din, (uint32_t)m, fs.vals, fs.one, fs.dg, fs.dst, fs.dv, d.stream));
  std::vector<int32_t> st(m);
  int32_t v = 0;
  HIPCHK(hipMemcpyAsync(st.data(), fs.dst, 4 * m, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipMemcpyAsync(&v, fs.dv, 4, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  for (int32_t x : st)
    if (x) return -BGV_E_ARG;  // a coefficient >= p: not a serialized partial
  *out_verdict = v;
  return BGV_OK;
}

int bgv_debug_prepare(bgv_ctx* c, const bgv_set* sets, size_t nsets, int path, uint64_t seed, uint8_t* out_h192,
                      uint8_t* out_f576, int32_t* out_status) {
  if (!c || (nsets && (!sets || !out_h192 || !out_f576 || !out_status)) ||
      (path != BGV_PATH_BULK && path != BGV_PATH_LATENCY))
    return -BGV_E_ARG;
  if (nsets == 0) return BGV_OK;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);
  if (c->closed) return -BGV_E_CLOSED;
  // one job's layout: groups of 64 consecutive slots, every slot hashes its own root
  std::vector<bgv_dslot> slots;
  std::vector<bgv_dgroup> groups;
  std::vector<uint32_t> idx;
  uint64_t state = seed;
  uint32_t max_npk = 0;
  for (size_t i = 0; i < nsets; ++i) {
    const bgv_set& st = sets[i];
    if (!st.pk_indices || st.n_pk == 0 || !st.msg || (st.sig_len && !st.sig)) return -BGV_E_ARG;
    for (uint32_t q = 0; q < st.n_pk; ++q)
      if (st.pk_indices[q] >= c->n_pubkeys || c->bad_pk.count(st.pk_indices[q])) return -BGV_E_BAD_INDEX;
    bgv_dslot s;
    memset(&s, 0, sizeof(s));
    s.flags = BGV_SLOT_PK_CACHED;
    s.n_pk = st.n_pk;
    s.sig_len = st.sig_len;
    s.pk_off = (uint32_t)idx.size();
    idx.insert(idx.end(), st.pk_indices, st.pk_indices + st.n_pk);
    memcpy(s.msg, st.msg, 32);
    if (st.sig_len == 96) memcpy(s.sig, st.sig, 96);
    s.group = (uint32_t)(i / BGV_WAVE);
    s.hsrc = (uint32_t)i;
    do s.scalar = splitmix64(&state);
    while (s.scalar == 0);
    max_npk = std::max(max_npk, st.n_pk);
    slots.push_back(s);
  }
  while (slots.size() % BGV_WAVE) {
    bgv_dslot s;
    memset(&s, 0, sizeof(s));
    s.flags = BGV_SLOT_PAD;
    s.hsrc = (uint32_t)slots.size();
    slots.push_back(s);
  }
  for (size_t g = 0; g * BGV_WAVE < nsets; ++g)
    groups.push_back(bgv_dgroup{(uint32_t)(g * BGV_WAVE), (uint32_t)std::min<size_t>(BGV_WAVE, nsets - g * BGV_WAVE),
                                BGV_ALL_SLOTS});
  const uint32_t nslots = (uint32_t)slots.size(), ngroups = (uint32_t)groups.size();
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  Exec* x = new Exec();
  uint8_t *dh = nullptr, *df = nullptr;
  int rc = exec_create(x);
  // a non-blocking stream of its own, like the dispatchers' (not the legacy null stream)
  hipStream_t dstream = nullptr;
  if (!rc && hipStreamCreateWithFlags(&dstream, hipStreamNonBlocking) != hipSuccess) rc = -BGV_E_DEVICE;
  x->main = dstream;
  if (!rc) rc = exec_reserve_slots(*x, nslots);
  if (!rc) rc = exec_reserve_groups(*x, ngroups);
  if (!rc) rc = grow(&x->d_idx, &x->idx_cap, idx.size());
  if (!rc && (hipMalloc(reinterpret_cast<void**>(&dh), 192ull * nslots) != hipSuccess ||
              hipMalloc(reinterpret_cast<void**>(&df), 576ull * nslots) != hipSuccess))
    rc = -BGV_E_DEVICE;
  std::vector<int32_t> ss(nslots), ps(nslots);
  if (!rc) {
    bgv_dev_batch b = make_batch(d, *x, nslots, ngroups);
    b.max_npk = max_npk;
    b.path = path;
    rc = exec_reserve_lines(*x, b);
    bgv_streams S{x->main, nullptr};
    const bool ok = rc == BGV_OK &&
        hipMemcpyAsync(x->d_slots, slots.data(), sizeof(bgv_dslot) * nslots, hipMemcpyHostToDevice, x->main) ==
            hipSuccess &&
        hipMemcpyAsync(x->d_groups, groups.data(), sizeof(bgv_dgroup) * ngroups, hipMemcpyHostToDevice, x->main) ==
            hipSuccess &&
        hipMemcpyAsync(x->d_idx, idx.data(), 4 * idx.size(), hipMemcpyHostToDevice, x->main) == hipSuccess &&
        bgv_launch_sets(b, S) == hipSuccess && bgv_launch_debug_out(b, dh, df, x->main) == hipSuccess &&
        hipMemcpyAsync(out_h192, dh, 192 * nsets, hipMemcpyDeviceToHost, x->main) == hipSuccess &&
        hipMemcpyAsync(out_f576, df, 576 * nsets, hipMemcpyDeviceToHost, x->main) == hipSuccess &&
        hipMemcpyAsync(ss.data(), b.sig_status, 4ull * nslots, hipMemcpyDeviceToHost, x->main) == hipSuccess &&
        hipMemcpyAsync(ps.data(), b.pk_status, 4ull * nslots, hipMemcpyDeviceToHost, x->main) == hipSuccess &&
        hipStreamSynchronize(x->main) == hipSuccess;
    if (!ok) rc = -BGV_E_DEVICE;
  }
  if (dh) (void)hipFree(dh);
  if (df) (void)hipFree(df);
  exec_destroy(x);  // synchronizes x->main first
  if (dstream) (void)hipStreamDestroy(dstream);
  if (rc) return rc;
  for (size_t i = 0; i < nsets; ++i) {
    out_status[2 * i] = ss[i];
    out_status[2 * i + 1] = ps[i];
  }
  return BGV_OK;
}

int bgv_debug_uniform(bgv_ctx* c, const bgv_set* sets, size_t nsets, uint64_t seed, const uint64_t* test_masks,
                      const uint32_t* test_weighted, size_t ntests, uint8_t* out_first576, uint8_t* out_pk576,
                      uint8_t* out_sig576) {
  if (!c || nsets < 2 || nsets > BGV_WAVE || !sets || !out_first576 || ntests > BGV_WAVE ||
      (ntests && (!test_masks || !test_weighted || !out_pk576 || !out_sig576)))
    return -BGV_E_ARG;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);
  if (c->closed) return -BGV_E_CLOSED;
  // one uniform first-pass group: every set signs the first set's root (hsrc 0)
  std::vector<bgv_dslot> slots;
  std::vector<uint32_t> idx;
  uint64_t state = seed;
  uint32_t max_npk = 0;
  for (size_t i = 0; i < nsets; ++i) {
    const bgv_set& st = sets[i];
    if (!st.pk_indices || st.n_pk == 0 || !st.msg || st.sig_len != 96 || !st.sig ||
        memcmp(st.msg, sets[0].msg, 32) != 0)
      return -BGV_E_ARG;
    for (uint32_t q = 0; q < st.n_pk; ++q)
      if (st.pk_indices[q] >= c->n_pubkeys || c->bad_pk.count(st.pk_indices[q])) return -BGV_E_BAD_INDEX;
    bgv_dslot s;
    memset(&s, 0, sizeof(s));
    s.flags = BGV_SLOT_PK_CACHED;
    s.n_pk = st.n_pk;
    s.sig_len = st.sig_len;
    s.pk_off = (uint32_t)idx.size();
    idx.insert(idx.end(), st.pk_indices, st.pk_indices + st.n_pk);
    memcpy(s.msg, st.msg, 32);
    memcpy(s.sig, st.sig, 96);
    s.group = 0;
    s.hsrc = 0;
    do s.scalar = splitmix64(&state);
    while (s.scalar == 0);
    max_npk = std::max(max_npk, st.n_pk);
    slots.push_back(s);
  }
  while (slots.size() % BGV_WAVE) {
    bgv_dslot s;
    memset(&s, 0, sizeof(s));
    s.flags = BGV_SLOT_PAD;
    s.hsrc = (uint32_t)slots.size();
    slots.push_back(s);
  }
  const uint32_t nslots = (uint32_t)slots.size(), nt = (uint32_t)ntests;
  const bgv_dgroup first{0u, (uint32_t)nsets, BGV_ALL_SLOTS, 0u, BGV_GROUP_UNIFORM};
  // the tests as a retry round lays them out (retry_launch): groups, then the uniform list
  const uint32_t per = (uint32_t)(sizeof(bgv_dgroup) / sizeof(uint32_t));
  const uint32_t nlist = (nt + per - 1) / per;
  std::vector<bgv_dgroup> tg(nt + nlist);
  bool weighted = false;
  for (uint32_t t = 0; t < nt; ++t) {
    tg[t] = bgv_dgroup{0u, (uint32_t)nsets, test_masks[t], 0u,
                       BGV_GROUP_UNIFORM | (test_weighted[t] ? BGV_GROUP_WEIGHTED : 0u)};
    weighted = weighted || test_weighted[t];
    reinterpret_cast<uint32_t*>(tg.data() + nt)[t] = t;
  }
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  Exec* x = new Exec();
  uint8_t* dout = nullptr;
  int rc = exec_create(x);
  hipStream_t dstream = nullptr;
  if (!rc && hipStreamCreateWithFlags(&dstream, hipStreamNonBlocking) != hipSuccess) rc = -BGV_E_DEVICE;
  x->main = dstream;
  if (!rc) rc = exec_reserve_slots(*x, nslots);
  if (!rc) rc = exec_reserve_groups(*x, std::max<uint32_t>(1, nt + nlist));
  if (!rc) rc = grow(&x->d_idx, &x->idx_cap, idx.size());
  if (!rc && hipMalloc(reinterpret_cast<void**>(&dout), 576ull * (1 + 2 * nt)) != hipSuccess) rc = -BGV_E_DEVICE;
  if (!rc) {
    bgv_dev_batch b = make_batch(d, *x, nslots, 1);
    b.max_npk = max_npk;
    b.path = BGV_PATH_BULK;
    b.uniform = true;
    rc = exec_reserve_lines(*x, b);
    bgv_streams S{x->main, nullptr};
    bool ok = rc == BGV_OK &&
        hipMemcpyAsync(x->d_slots, slots.data(), sizeof(bgv_dslot) * nslots, hipMemcpyHostToDevice, x->main) ==
            hipSuccess &&
        hipMemcpyAsync(x->d_groups, &first, sizeof(bgv_dgroup), hipMemcpyHostToDevice, x->main) == hipSuccess &&
        hipMemcpyAsync(x->d_idx, idx.data(), 4 * idx.size(), hipMemcpyHostToDevice, x->main) == hipSuccess &&
        bgv_launch_sets(b, S) == hipSuccess &&
        bgv_launch_fp12_bytes(b.gpkp, 1, dout, x->main) == hipSuccess;
    if (ok && nt) {
      // the tests over the first pass's per-slot results (r_i sig_i, r_i pk_i, H)
      bgv_dev_batch t = make_batch(d, *x, nslots, nt);
      t.max_npk = max_npk;
      t.path = BGV_PATH_BULK;
      t.uniform = true;
      t.upk = reinterpret_cast<const uint32_t*>(t.groups + nt);
      t.npk = nt;
      t.weighted = weighted;
      ok = hipMemcpyAsync(x->d_groups, tg.data(), sizeof(bgv_dgroup) * tg.size(), hipMemcpyHostToDevice, x->main) ==
               hipSuccess &&
           bgv_launch_gpairs(t, x->main) == hipSuccess &&
           bgv_launch_fp12_bytes(t.gpkp, nt, dout + 576, x->main) == hipSuccess &&
           bgv_launch_fp12_bytes(t.gpair, nt, dout + 576ull * (1 + nt), x->main) == hipSuccess &&
           hipMemcpyAsync(out_pk576, dout + 576, 576ull * nt, hipMemcpyDeviceToHost, x->main) == hipSuccess &&
           hipMemcpyAsync(out_sig576, dout + 576ull * (1 + nt), 576ull * nt, hipMemcpyDeviceToHost, x->main) ==
               hipSuccess;
    }
    ok = ok && hipMemcpyAsync(out_first576, dout, 576, hipMemcpyDeviceToHost, x->main) == hipSuccess &&
         hipStreamSynchronize(x->main) == hipSuccess;
    if (!ok) rc = -BGV_E_DEVICE;
  }
  if (dout) (void)hipFree(dout);
  exec_destroy(x);
  if (dstream) (void)hipStreamDestroy(dstream);
  return rc;
}

int bgv_aggregate_pubkeys(bgv_ctx* c, const uint32_t* idx, size_t n, uint8_t out96[96]) {
  if (!c || !out96 || (n && !idx)) return -BGV_E_ARG;
  if (n == 0) return -BGV_E_EMPTY_AGGREGATE;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);
  if (c->closed) return -BGV_E_CLOSED;
  for (size_t i = 0; i < n; ++i)
    if (idx[i] >= c->n_pubkeys || c->bad_pk.count(idx[i])) return -BGV_E_BAD_INDEX;
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  // one cached-key slot through the verify path's aggregation (k_pk_agg / pk_sum)
  bgv_dslot s;
  memset(&s, 0, sizeof(s));
  s.flags = BGV_SLOT_PK_CACHED;
  s.n_pk = (uint32_t)n;
  uint32_t* di = nullptr;
  uint8_t* dout = nullptr;
  bgv_dslot* ds = nullptr;
  void* dagg = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&di), 4 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dout), 96));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&ds), sizeof(bgv_dslot)));
  HIPCHK(hipMalloc(&dagg, bgv_g1_point_bytes()));
  HIPCHK(hipMemcpyAsync(di, idx, 4 * n, hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipMemcpyAsync(ds, &s, sizeof(s), hipMemcpyHostToDevice, d.stream));
  HIPCHK(bgv_launch_aggregate(ds, di, (uint32_t)n, d.cache, dagg, dout, d.stream));
  HIPCHK(hipMemcpyAsync(out96, dout, 96, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  void* bufs[] = {di, dout, ds, dagg};
  for (void* p : bufs) (void)hipFree(p);
  return BGV_OK;
}

int bgv_hash_to_g2(bgv_ctx* c, const uint8_t* msgs, const uint32_t* lens, size_t n, uint8_t* out192) {
  if (!c || (n && (!lens || !out192))) return -BGV_E_ARG;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);  // bgv_close frees the devices under the exclusive lock
  if (c->closed) return -BGV_E_CLOSED;
  if (n == 0) return BGV_OK;
  std::vector<uint32_t> offs(n);
  size_t tot = 0;
  for (size_t i = 0; i < n; ++i) {
    if (lens[i] > 1024) return -BGV_E_ARG;
    offs[i] = (uint32_t)tot;
    tot += lens[i];
  }
  if (tot && !msgs) return -BGV_E_ARG;
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  uint8_t *dm = nullptr, *dout = nullptr;
  uint32_t *doff = nullptr, *dlen = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dm), tot + 1));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&doff), 4 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dlen), 4 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dout), 192 * n));
  if (tot) HIPCHK(hipMemcpyAsync(dm, msgs, tot, hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipMemcpyAsync(doff, offs.data(), 4 * n, hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipMemcpyAsync(dlen, lens, 4 * n, hipMemcpyHostToDevice, d.stream));
  HIPCHK(bgv_launch_hash(dm, doff, dlen, (uint32_t)n, dout, d.stream));
  HIPCHK(hipMemcpyAsync(out192, dout, 192 * n, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  (void)hipFree(dm);
  (void)hipFree(doff);
  (void)hipFree(dlen);
  (void)hipFree(dout);
  return BGV_OK;
}

int bgv_pubkeys_validate(bgv_ctx* c, const uint8_t* keys48, size_t n, int32_t* out_status, uint8_t* out96) {
  if (!c || (n && (!keys48 || !out_status))) return -BGV_E_ARG;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);  // bgv_close frees the devices under the exclusive lock
  if (c->closed) return -BGV_E_CLOSED;
  if (n == 0) return BGV_OK;
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  uint8_t *dk = nullptr, *dout = nullptr;
  int32_t* dst = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dk), 48 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dout), 96 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dst), 4 * n));
  HIPCHK(hipMemcpyAsync(dk, keys48, 48 * n, hipMemcpyHostToDevice, d.stream));
  HIPCHK(bgv_launch_pk_validate(dk, (uint32_t)n, dst, dout, d.stream));
  HIPCHK(hipMemcpyAsync(out_status, dst, 4 * n, hipMemcpyDeviceToHost, d.stream));
  if (out96) HIPCHK(hipMemcpyAsync(out96, dout, 96 * n, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  (void)hipFree(dk);
  (void)hipFree(dout);
  (void)hipFree(dst);
  for (size_t i = 0; i < n; ++i) out_status[i] = -out_status[i];
  return BGV_OK;
}

int bgv_aggregate_signatures(bgv_ctx* c, const uint8_t* sigs96, const uint32_t* lens, const uint32_t* counts,
                             size_t naggs, uint8_t* out96, int32_t* out_status) {
  if (!c || (naggs && (!counts || !out96 || !out_status))) return -BGV_E_ARG;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);  // bgv_close frees the devices under the exclusive lock
  if (c->closed) return -BGV_E_CLOSED;
  if (naggs == 0) return BGV_OK;
  std::vector<uint32_t> first(naggs);
  size_t n = 0;
  for (size_t a = 0; a < naggs; ++a) {
    first[a] = (uint32_t)n;
    n += counts[a];
  }
  if (n && (!sigs96 || !lens)) return -BGV_E_ARG;
  std::vector<int32_t> st(n);
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  uint8_t *ds = nullptr, *dout = nullptr;
  uint32_t *dl = nullptr, *df = nullptr, *dc = nullptr;
  int32_t* dst = nullptr;
  void* pts = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&ds), 96 * n + 1));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dl), 4 * n + 4));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dst), 4 * n + 4));
  HIPCHK(hipMalloc(&pts, bgv_g2_point_bytes() * n + 1));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&df), 4 * naggs));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dc), 4 * naggs));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dout), 96 * naggs));
  if (n) {
    HIPCHK(hipMemcpyAsync(ds, sigs96, 96 * n, hipMemcpyHostToDevice, d.stream));
    HIPCHK(hipMemcpyAsync(dl, lens, 4 * n, hipMemcpyHostToDevice, d.stream));
  }
  HIPCHK(hipMemcpyAsync(df, first.data(), 4 * naggs, hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipMemcpyAsync(dc, counts, 4 * naggs, hipMemcpyHostToDevice, d.stream));
  HIPCHK(bgv_launch_sig_aggregate(ds, dl, (uint32_t)n, df, dc, (uint32_t)naggs, pts, dst, dout, d.stream));
  if (n) HIPCHK(hipMemcpyAsync(st.data(), dst, 4 * n, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipMemcpyAsync(out96, dout, 96 * naggs, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  void* bufs[] = {ds, dl, dst, pts, df, dc, dout};
  for (void* b : bufs) (void)hipFree(b);
  // verdict per aggregate: the first signature (in order) that fails to decode or
  // validate, as Signature.fromBytes throws on it; [] -> EMPTY_AGGREGATE_ARRAY
  for (size_t a = 0; a < naggs; ++a) {
    int32_t code = counts[a] ? BGV_OK : -BGV_E_EMPTY_AGGREGATE;
    for (uint32_t k = 0; k < counts[a] && code == BGV_OK; ++k)
      if (st[first[a] + k] != BGV_OK) code = -st[first[a] + k];
    out_status[a] = code;
    if (code != BGV_OK) memset(out96 + 96 * a, 0, 96);
  }
  return BGV_OK;
}

int bgv_deposits_verify(bgv_ctx* c, const uint8_t* keys48, const uint8_t* msgs32, const uint8_t* sigs96, size_t n,
                        int32_t* out_valid) {
  if (!c || (n && (!keys48 || !msgs32 || !sigs96 || !out_valid))) return -BGV_E_ARG;
  if (n == 0) return BGV_OK;
  std::vector<int32_t> ks(n);
  std::vector<uint8_t> pk96(96 * n);
  int rc = bgv_pubkeys_validate(c, keys48, n, ks.data(), pk96.data());
  if (rc) return rc;
  // every deposit with a valid key is its own job (Signature.verify per deposit)
  std::vector<bgv_set> sets;
  std::vector<bgv_job> jobs;
  std::vector<size_t> which;
  for (size_t i = 0; i < n; ++i) {
    out_valid[i] = 0;
    if (ks[i] != BGV_OK) continue;
    bgv_set st{};
    st.n_pk = 1;
    st.sig_len = 96;
    st.pk_bytes = pk96.data() + 96 * i;
    st.msg = msgs32 + 32 * i;
    st.sig = sigs96 + 96 * i;
    jobs.push_back(bgv_job{(uint32_t)sets.size(), 1, 0});
    sets.push_back(st);
    which.push_back(i);
  }
  if (jobs.empty()) return BGV_OK;
  std::vector<int32_t> codes(jobs.size());
  rc = bgv_verify(c, jobs.data(), jobs.size(), sets.data(), sets.size(), BGV_MODE_PER_JOB, codes.data(), nullptr);
  if (rc) return rc;
  // processDeposit.ts:62-70 catches every BLS error: anything but "valid" is invalid
  for (size_t k = 0; k < which.size(); ++k) out_valid[which[k]] = codes[k] == 1 ? 1 : 0;
  return BGV_OK;
}

int bgv_keygen(bgv_ctx* c, const uint8_t* sks, size_t n, int64_t cache_first, uint8_t* out48) {
  if (!c || (n && !sks)) return -BGV_E_ARG;
  std::lock_guard<std::mutex> plk(c->put_mu);
  std::unique_lock<std::shared_mutex> clk(c->cache_mu);
  if (c->closed) return -BGV_E_CLOSED;
  if (cache_first > (int64_t)c->n_pubkeys) return -BGV_E_ARG;
  if (n == 0) return BGV_OK;
  if (cache_first >= 0) {
    int rc = cache_reserve(c, (size_t)cache_first + n);
    if (rc) return rc;
  }
  const size_t esz = bgv_cache_entry_bytes();
  for (size_t di = 0; di < c->devs.size(); ++di) {
    Device& d = c->devs[di];
    if (cache_first < 0 && di > 0) break;
    HIPCHK(hipSetDevice(d.id));
    uint8_t *dsk = nullptr, *dout = nullptr;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&dsk), 32 * n));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&dout), 48 * n));
    HIPCHK(hipMemcpyAsync(dsk, sks, 32 * n, hipMemcpyHostToDevice, d.stream));
    bgv_cache_entry* dst =
        cache_first >= 0 ? reinterpret_cast<bgv_cache_entry*>(reinterpret_cast<uint8_t*>(d.cache) + esz * cache_first)
                         : nullptr;
    HIPCHK(bgv_launch_keygen(dsk, (uint32_t)n, dst, dout, d.stream));
    if (out48 && di == 0) HIPCHK(hipMemcpyAsync(out48, dout, 48 * n, hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    (void)hipFree(dsk);
    (void)hipFree(dout);
  }
  if (cache_first >= 0) {
    for (size_t i = 0; i < n; ++i) c->bad_pk.erase((uint32_t)(cache_first + i));
    c->n_pubkeys.store(std::max(c->n_pubkeys.load(), (size_t)cache_first + n));
  }
  return BGV_OK;
}

int bgv_sign(bgv_ctx* c, const uint8_t* sks, const uint8_t* msgs, size_t n, uint8_t* out96) {
  if (!c || (n && (!sks || !msgs || !out96))) return -BGV_E_ARG;
  std::shared_lock<std::shared_mutex> clk(c->cache_mu);  // bgv_close frees the devices under the exclusive lock
  if (c->closed) return -BGV_E_CLOSED;
  if (n == 0) return BGV_OK;
  std::lock_guard<std::mutex> lk(c->util_mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  uint8_t *dsk = nullptr, *dm = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dsk), 32 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dm), 32 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dout), 96 * n));
  HIPCHK(hipMemcpyAsync(dsk, sks, 32 * n, hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipMemcpyAsync(dm, msgs, 32 * n, hipMemcpyHostToDevice, d.stream));
  HIPCHK(bgv_launch_sign(dsk, dm, (uint32_t)n, dout, d.stream));
  HIPCHK(hipMemcpyAsync(out96, dout, 96 * n, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  (void)hipFree(dsk);
  (void)hipFree(dm);
  (void)hipFree(dout);
  return BGV_OK;
}

int bgv_profile(bgv_ctx* c, int enable, double* kernel_ms, const char** names, int n, uint64_t* launches) {
  if (!c) return -BGV_E_ARG;
  std::lock_guard<std::mutex> lk(c->prof_mu);
  for (int k = 0; k < n && k < BGV_NKERNELS; ++k) {
    if (kernel_ms) kernel_ms[k] = c->kernel_ms[k];
    if (names) names[k] = BGV_KERNEL_NAMES[k];
  }
  if (launches) *launches = c->kernel_launches;
  if (enable >= 0) {
    c->profile = enable != 0;
    for (double& v : c->kernel_ms) v = 0;
    c->kernel_launches = 0;
  }
  return BGV_NKERNELS;
}

const char* bgv_strerror(int code) {
  if (code < 0) code = -code;
  switch (code) {
    case BGV_OK: return "BLST_SUCCESS";
    case BGV_BLST_BAD_ENCODING: return "BLST_BAD_ENCODING";
    case BGV_BLST_POINT_NOT_ON_CURVE: return "BLST_POINT_NOT_ON_CURVE";
    case BGV_BLST_POINT_NOT_IN_GROUP: return "BLST_POINT_NOT_IN_GROUP";
    case BGV_BLST_AGGR_TYPE_MISMATCH: return "BLST_AGGR_TYPE_MISMATCH";
    case BGV_BLST_VERIFY_FAIL: return "BLST_VERIFY_FAIL";
    case BGV_BLST_PK_IS_INFINITY: return "BLST_PK_IS_INFINITY";
    case BGV_BLST_BAD_SCALAR: return "BLST_BAD_SCALAR";
    case BGV_BLST_INVALID_SIZE: return "BLST_INVALID_SIZE";
    case BGV_E_EMPTY_AGGREGATE: return "EMPTY_AGGREGATE_ARRAY";
    case BGV_E_EMPTY_SET: return "Empty signature set";
    case BGV_E_BAD_INDEX: return "BGV_E_BAD_INDEX: validator index not in the device pubkey cache";
    case BGV_E_ARG: return "BGV_E_ARG: invalid argument";
    case BGV_E_DEVICE: return "BGV_E_DEVICE: HIP device error";
    case BGV_E_NOMEM: return "BGV_E_NOMEM";
    case BGV_E_CLOSED: return "QUEUE_ABORTED";
    default: return "BGV_E_UNKNOWN";
  }
}

}  // extern "C"
