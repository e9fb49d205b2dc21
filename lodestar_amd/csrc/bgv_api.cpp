// libblsgpu: C-ABI host orchestration of the MI355X batch BLS verifier.
//
// Mirrors the reference's scheduling semantics, file by file:
//   * per-job verdicts and retry   packages/beacon-node/src/chain/bls/multithread/worker.ts:32-108
//   * batch vs single verify       packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39
//   * pubkey aggregation errors    packages/beacon-node/src/chain/bls/utils.ts:5-16
// but lays the sets out for the GPU: one lane per set, device groups of <= 64
// sets (one wavefront) each closed by its own final exponentiation.  A job's
// verdict is the AND of the groups holding its sets; a group that mixes
// batchable jobs and fails sends exactly those jobs to a second pass where each
// is verified alone (the reference retries the whole >=16-job chunk; the
// per-job verdicts are the same).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/blsgpu.h"
#include "bgv_launch.h"

namespace {

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t kev[BGV_NKERNELS + 1] = {};
  // pubkey cache (replicated)
  bgv_cache_entry* cache = nullptr;
  size_t cache_cap = 0;
  // per-call buffers, grown on demand
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
  int32_t* d_tmp = nullptr;
  size_t tmp_cap = 0;
};

struct Job {  // one async request
  const bgv_job* jobs;
  size_t njobs;
  const bgv_set* sets;
  size_t nsets;
  int mode;
  int32_t* out;
  bgv_stats* stats;
  bgv_done_fn done;
  void* user;
};

}  // namespace

struct bgv_ctx {
  std::vector<Device> devs;
  size_t n_pubkeys = 0;
  bool closed = false;
  uint64_t rng_seed = 0, rng_state = 0;
  bool profile = false;
  double kernel_ms[BGV_NKERNELS] = {};
  uint64_t kernel_launches = 0;
  std::mutex mu;  // serialises device work
  // host staging (pinned)
  bgv_dslot* h_slots = nullptr;
  size_t h_slots_cap = 0;
  // async worker
  std::thread worker;
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<Job> queue;
  bool stop = false;
};

#define HIPCHK(x)                            \
  do {                                       \
    hipError_t e_ = (x);                     \
    if (e_ != hipSuccess) return -BGV_E_DEVICE; \
  } while (0)

static uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// nonzero 64-bit randomizers (blst mul_n_aggregate with 64 random bits)
static void fill_scalars(bgv_ctx* c, uint64_t* out, size_t n) {
  if (c->rng_seed) {
    for (size_t i = 0; i < n; ++i) {
      uint64_t v;
      do v = splitmix64(&c->rng_state);
      while (v == 0);
      out[i] = v;
    }
    return;
  }
  size_t got = 0;
  while (got < n * 8) {
    ssize_t r = getrandom(reinterpret_cast<uint8_t*>(out) + got, n * 8 - got, 0);
    if (r > 0) got += (size_t)r;
  }
  for (size_t i = 0; i < n; ++i)
    if (out[i] == 0) out[i] = 1;
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

static int ensure_device_capacity(Device& d, uint32_t slots, uint32_t groups, size_t nidx, size_t npkb) {
  HIPCHK(hipSetDevice(d.id));
  if (slots > d.slot_cap) {
    uint32_t n = std::max<uint32_t>(slots, d.slot_cap * 2);
    if (d.slot_mem) (void)hipFree(d.slot_mem);
    if (d.d_slots) (void)hipFree(d.d_slots);
    d.slot_mem = nullptr;
    d.d_slots = nullptr;
    HIPCHK(hipMalloc(&d.slot_mem, bgv_slot_bytes() * n));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&d.d_slots), sizeof(bgv_dslot) * n));
    d.slot_cap = n;
  }
  if (groups > d.group_cap) {
    uint32_t n = std::max<uint32_t>(groups, d.group_cap * 2);
    if (d.group_mem) (void)hipFree(d.group_mem);
    if (d.d_groups) (void)hipFree(d.d_groups);
    d.group_mem = nullptr;
    d.d_groups = nullptr;
    HIPCHK(hipMalloc(&d.group_mem, bgv_group_bytes() * n));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&d.d_groups), sizeof(bgv_dgroup) * n));
    d.group_cap = n;
  }
  int rc;
  if ((rc = grow(&d.d_idx, &d.idx_cap, std::max<size_t>(nidx, 1)))) return rc;
  if ((rc = grow(&d.d_pkb, &d.pkb_cap, std::max<size_t>(npkb, 1)))) return rc;
  return BGV_OK;
}

// ---------------------------------------------------------------------------
// Layout: jobs -> slots/groups
// ---------------------------------------------------------------------------
namespace {
struct Layout {
  std::vector<bgv_dslot> slots;
  std::vector<bgv_dgroup> groups;
  std::vector<int32_t> slot_set;       // set index per slot (-1 = pad)
  std::vector<std::vector<uint32_t>> job_groups;
  std::vector<char> group_shared;      // group holds sets of more than one job
  std::vector<uint32_t> idx;           // concatenated pubkey indices
  std::vector<uint8_t> pkb;            // concatenated 96-B pubkey records
};

struct Builder {
  Layout& L;
  bool open = false;       // a group is open for appending
  uint32_t open_group = 0;
  int open_job = -1;
  explicit Builder(Layout& l) : L(l) {}

  void close_group() { open = false; }
  void new_group() {
    // start at the next wave boundary
    uint32_t first = (uint32_t)L.slots.size();
    uint32_t aligned = (first + BGV_WAVE - 1) / BGV_WAVE * BGV_WAVE;
    while (L.slots.size() < aligned) pad();
    bgv_dgroup g{aligned, 0};
    L.groups.push_back(g);
    L.group_shared.push_back(0);
    open_group = (uint32_t)L.groups.size() - 1;
    open = true;
    open_job = -1;
  }
  void pad() {
    bgv_dslot s;
    memset(&s, 0, sizeof(s));
    s.flags = BGV_SLOT_PAD;
    L.slots.push_back(s);
    L.slot_set.push_back(-1);
  }
  void add(int job, uint32_t set_index, const bgv_set& st) {
    if (!open || L.groups[open_group].n_slots == BGV_WAVE) new_group();
    bgv_dgroup& g = L.groups[open_group];
    if (open_job >= 0 && open_job != job) L.group_shared[open_group] = 1;
    open_job = job;
    std::vector<uint32_t>& jg = L.job_groups[job];
    if (jg.empty() || jg.back() != open_group) jg.push_back(open_group);
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
    L.slots.push_back(s);
    L.slot_set.push_back((int32_t)set_index);
    g.n_slots++;
  }
};
}  // namespace

// Run one layout on the context's first device; fills per-slot statuses and per-group verdicts.
static int run_layout(bgv_ctx* c, Layout& L, std::vector<int32_t>& sig_st, std::vector<int32_t>& pk_st,
                      std::vector<int32_t>& verdict, double* dev_ms) {
  const uint32_t nslots = (uint32_t)L.slots.size(), ngroups = (uint32_t)L.groups.size();
  sig_st.assign(nslots, 0);
  pk_st.assign(nslots, 0);
  verdict.assign(ngroups, 0);
  if (nslots == 0) return BGV_OK;
  std::vector<uint64_t> sc(nslots);
  fill_scalars(c, sc.data(), nslots);
  for (uint32_t i = 0; i < nslots; ++i) L.slots[i].scalar = sc[i];

  Device& d = c->devs[0];
  int rc = ensure_device_capacity(d, nslots, ngroups, L.idx.size(), L.pkb.size());
  if (rc) return rc;
  HIPCHK(hipSetDevice(d.id));
  HIPCHK(hipMemcpyAsync(d.d_slots, L.slots.data(), sizeof(bgv_dslot) * nslots, hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipMemcpyAsync(d.d_groups, L.groups.data(), sizeof(bgv_dgroup) * ngroups, hipMemcpyHostToDevice, d.stream));
  if (!L.idx.empty())
    HIPCHK(hipMemcpyAsync(d.d_idx, L.idx.data(), 4 * L.idx.size(), hipMemcpyHostToDevice, d.stream));
  if (!L.pkb.empty()) HIPCHK(hipMemcpyAsync(d.d_pkb, L.pkb.data(), L.pkb.size(), hipMemcpyHostToDevice, d.stream));
  bgv_dev_batch b;
  memset(&b, 0, sizeof(b));
  b.nslots = nslots;
  b.ngroups = ngroups;
  b.slots = d.d_slots;
  b.groups = d.d_groups;
  b.pk_idx = d.d_idx;
  b.cache_opaque = d.cache;
  b.pk_bytes = d.d_pkb;
  bgv_carve(&b, d.slot_mem, d.slot_cap, d.group_mem, d.group_cap);
  HIPCHK(hipEventRecord(d.ev0, d.stream));
  HIPCHK(bgv_launch_verify(b, d.stream, c->profile ? d.kev : nullptr));
  HIPCHK(hipEventRecord(d.ev1, d.stream));
  HIPCHK(hipMemcpyAsync(sig_st.data(), b.sig_status, 4ull * nslots, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipMemcpyAsync(pk_st.data(), b.pk_status, 4ull * nslots, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipMemcpyAsync(verdict.data(), b.verdict, 4ull * ngroups, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, d.ev0, d.ev1));
  if (dev_ms) *dev_ms += ms;
  if (c->profile) {
    for (int k = 0; k < BGV_NKERNELS; ++k) {
      float km = 0;
      HIPCHK(hipEventElapsedTime(&km, d.kev[k], d.kev[k + 1]));
      c->kernel_ms[k] += km;
    }
    c->kernel_launches++;
  }
  return BGV_OK;
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

static int verify_impl(bgv_ctx* c, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
                       int32_t* out, bgv_stats* stats) {
  const auto t0 = std::chrono::steady_clock::now();
  bgv_stats st;
  memset(&st, 0, sizeof(st));
  if (c->closed) return -BGV_E_CLOSED;
  if ((njobs && (!jobs || !out)) || (nsets && !sets)) return -BGV_E_ARG;
  if (mode != BGV_MODE_WORKER && mode != BGV_MODE_PER_JOB) return -BGV_E_ARG;

  // host-side argument checks that the reference raises before any crypto
  std::vector<int32_t> code(njobs, 2);
  for (size_t j = 0; j < njobs; ++j) {
    const bgv_job& jb = jobs[j];
    if ((size_t)jb.first_set + jb.n_sets > nsets) return -BGV_E_ARG;
    if (jb.n_sets == 0) {
      code[j] = -BGV_E_EMPTY_SET;
      continue;
    }
    for (uint32_t k = 0; k < jb.n_sets && code[j] == 2; ++k) {
      const bgv_set& s = sets[jb.first_set + k];
      if (s.n_pk == 0) code[j] = -BGV_E_EMPTY_AGGREGATE;
      else if (!s.msg || (!s.sig && s.sig_len) || (!s.pk_indices && !s.pk_bytes)) return -BGV_E_ARG;
      else if (s.pk_indices)
        for (uint32_t q = 0; q < s.n_pk; ++q)
          if (s.pk_indices[q] >= c->n_pubkeys) {
            code[j] = -BGV_E_BAD_INDEX;
            break;
          }
    }
  }

  std::lock_guard<std::mutex> lk(c->mu);
  std::vector<int32_t> set_sig(nsets, 0), set_pk(nsets, 0);
  std::vector<size_t> retry;
  for (int pass = 0; pass < 2; ++pass) {
    Layout L;
    L.job_groups.resize(njobs);
    Builder B(L);
    std::vector<size_t> todo;
    if (pass == 0) {
      for (size_t j = 0; j < njobs; ++j)
        if (code[j] == 2) todo.push_back(j);
    } else {
      todo = retry;
    }
    if (todo.empty()) break;
    // batchable jobs share groups (pass 0, worker mode); everything else is exclusive
    for (size_t j : todo) {
      const bool shared = pass == 0 && mode == BGV_MODE_WORKER && jobs[j].batchable;
      if (shared) continue;
      B.close_group();
      for (uint32_t k = 0; k < jobs[j].n_sets; ++k)
        B.add((int)j, jobs[j].first_set + k, sets[jobs[j].first_set + k]);
      B.close_group();
    }
    B.close_group();
    for (size_t j : todo) {
      const bool shared = pass == 0 && mode == BGV_MODE_WORKER && jobs[j].batchable;
      if (!shared) continue;
      for (uint32_t k = 0; k < jobs[j].n_sets; ++k)
        B.add((int)j, jobs[j].first_set + k, sets[jobs[j].first_set + k]);
    }
    std::vector<int32_t> ss, ps, verdict;
    int rc = run_layout(c, L, ss, ps, verdict, &st.device_ms);
    if (rc) return rc;
    st.device_groups += L.groups.size();
    for (size_t i = 0; i < L.slots.size(); ++i)
      if (L.slot_set[i] >= 0) {
        set_sig[L.slot_set[i]] = ss[i];
        set_pk[L.slot_set[i]] = ps[i];
        st.sets_verified++;
      }
    retry.clear();
    std::vector<char> group_retried(L.groups.size(), 0);
    for (size_t j : todo) {
      int32_t pre = job_precheck(set_sig, set_pk, jobs[j]);
      if (pre != 2) {
        code[j] = pre;
        continue;
      }
      bool ok = true, needs_retry = false;
      for (uint32_t g : L.job_groups[j])
        if (!verdict[g]) {
          ok = false;
          if (L.group_shared[g]) {
            needs_retry = true;
            group_retried[g] = 1;
          }
        }
      if (needs_retry) {
        retry.push_back(j);
      } else {
        code[j] = ok ? 1 : 0;
        if (ok && pass == 0 && mode == BGV_MODE_WORKER && jobs[j].batchable) st.batch_sigs_success += jobs[j].n_sets;
      }
    }
    for (char r : group_retried) st.batch_retries += r;
  }
  for (size_t j = 0; j < njobs; ++j) out[j] = code[j] == 2 ? -BGV_E_DEVICE : code[j];
  st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = st;
  return BGV_OK;
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

int bgv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static void worker_loop(bgv_ctx* c) {
  for (;;) {
    Job jb;
    {
      std::unique_lock<std::mutex> lk(c->qmu);
      c->qcv.wait(lk, [c] { return c->stop || !c->queue.empty(); });
      if (c->queue.empty()) return;
      jb = c->queue.front();
      c->queue.pop_front();
    }
    int rc = verify_impl(c, jb.jobs, jb.njobs, jb.sets, jb.nsets, jb.mode, jb.out, jb.stats);
    if (jb.done) jb.done(jb.user, rc);
  }
}

int bgv_init(const int* devices, int ndev, bgv_ctx** out) {
  if (!out) return -BGV_E_ARG;
  *out = nullptr;
  int avail = bgv_device_count();
  if (avail <= 0) return -BGV_E_DEVICE;
  bgv_ctx* c = new bgv_ctx();
  const int n = (devices && ndev > 0) ? ndev : 1;
  for (int i = 0; i < n; ++i) {
    Device d;
    d.id = (devices && ndev > 0) ? devices[i] : 0;
    if (d.id < 0 || d.id >= avail) {
      delete c;
      return -BGV_E_ARG;
    }
    if (hipSetDevice(d.id) != hipSuccess || hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&d.ev0) != hipSuccess || hipEventCreate(&d.ev1) != hipSuccess) {
      delete c;
      return -BGV_E_DEVICE;
    }
    bool ok = true;
    for (auto& e : d.kev) ok = ok && hipEventCreate(&e) == hipSuccess;
    if (!ok) {
      delete c;
      return -BGV_E_DEVICE;
    }
    c->devs.push_back(d);
  }
  c->worker = std::thread(worker_loop, c);
  *out = c;
  return BGV_OK;
}

int bgv_close(bgv_ctx* c) {
  if (!c) return -BGV_E_ARG;
  {
    std::lock_guard<std::mutex> lk(c->qmu);
    c->stop = true;
  }
  c->qcv.notify_all();
  if (c->worker.joinable()) c->worker.join();
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->closed) return BGV_OK;
  c->closed = true;
  for (Device& d : c->devs) {
    (void)hipSetDevice(d.id);
    (void)hipStreamSynchronize(d.stream);
    void* ptrs[] = {d.cache, d.slot_mem, d.group_mem, d.d_slots, d.d_groups, d.d_idx, d.d_pkb, d.d_tmp};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
    for (auto& e : d.kev) (void)hipEventDestroy(e);
    (void)hipEventDestroy(d.ev0);
    (void)hipEventDestroy(d.ev1);
    (void)hipStreamDestroy(d.stream);
  }
  return BGV_OK;
}

int bgv_destroy(bgv_ctx* c) {
  if (!c) return -BGV_E_ARG;
  bgv_close(c);
  delete c;
  return BGV_OK;
}

int bgv_set_rng_seed(bgv_ctx* c, uint64_t seed) {
  if (!c) return -BGV_E_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  c->rng_seed = seed;
  c->rng_state = seed;
  return BGV_OK;
}

size_t bgv_pubkeys_count(const bgv_ctx* c) { return c ? c->n_pubkeys : 0; }

static int cache_reserve(bgv_ctx* c, size_t need);

int bgv_pubkeys_put(bgv_ctx* c, uint32_t first, const uint8_t* keys, size_t n, int fmt) {
  if (!c || (n && !keys) || (fmt != BGV_PK_COMPRESSED && fmt != BGV_PK_UNCOMPRESSED)) return -BGV_E_ARG;
  if (c->closed) return -BGV_E_CLOSED;
  if ((size_t)first > c->n_pubkeys) return -BGV_E_ARG;  // append or overwrite, no holes
  std::lock_guard<std::mutex> lk(c->mu);
  const size_t need = (size_t)first + n;
  const size_t esz = bgv_cache_entry_bytes();
  int first_err = BGV_OK;
  {
    int rc = cache_reserve(c, need);
    if (rc) return rc;
  }
  for (Device& d : c->devs) {
    HIPCHK(hipSetDevice(d.id));
    const size_t chunk = 1 << 20;
    uint8_t* dk = nullptr;
    int32_t* dst = nullptr;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&dk), (size_t)fmt * std::min(n, chunk) + 1));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&dst), 4 * std::min(n, chunk) + 4));
    std::vector<int32_t> hst;
    for (size_t off = 0; off < n; off += chunk) {
      const size_t m = std::min(chunk, n - off);
      HIPCHK(hipMemcpyAsync(dk, keys + (size_t)fmt * off, (size_t)fmt * m, hipMemcpyHostToDevice, d.stream));
      bgv_cache_entry* dst_cache =
          reinterpret_cast<bgv_cache_entry*>(reinterpret_cast<uint8_t*>(d.cache) + esz * (first + off));
      HIPCHK(bgv_launch_cache_put(dk, (uint32_t)m, fmt, dst_cache, dst, d.stream));
      hst.resize(m);
      HIPCHK(hipMemcpyAsync(hst.data(), dst, 4 * m, hipMemcpyDeviceToHost, d.stream));
      HIPCHK(hipStreamSynchronize(d.stream));
      for (size_t i = 0; i < m && first_err == BGV_OK; ++i)
        if (hst[i]) first_err = hst[i];
    }
    (void)hipFree(dk);
    (void)hipFree(dst);
  }
  if (first_err) return -first_err;
  c->n_pubkeys = std::max(c->n_pubkeys, need);
  return BGV_OK;
}

int bgv_verify(bgv_ctx* c, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
               int32_t* out, bgv_stats* stats) {
  if (!c) return -BGV_E_ARG;
  return verify_impl(c, jobs, njobs, sets, nsets, mode, out, stats);
}

int bgv_verify_async(bgv_ctx* c, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
                     int32_t* out, bgv_stats* stats, bgv_done_fn done, void* user) {
  if (!c) return -BGV_E_ARG;
  if (c->closed) return -BGV_E_CLOSED;
  {
    std::lock_guard<std::mutex> lk(c->qmu);
    if (c->stop) return -BGV_E_CLOSED;
    c->queue.push_back(Job{jobs, njobs, sets, nsets, mode, out, stats, done, user});
  }
  c->qcv.notify_one();
  return BGV_OK;
}

int bgv_aggregate_pubkeys(bgv_ctx* c, const uint32_t* idx, size_t n, uint8_t out96[96]) {
  if (!c || !out96 || (n && !idx)) return -BGV_E_ARG;
  if (c->closed) return -BGV_E_CLOSED;
  if (n == 0) return -BGV_E_EMPTY_AGGREGATE;
  for (size_t i = 0; i < n; ++i)
    if (idx[i] >= c->n_pubkeys) return -BGV_E_BAD_INDEX;
  std::lock_guard<std::mutex> lk(c->mu);
  Device& d = c->devs[0];
  HIPCHK(hipSetDevice(d.id));
  uint32_t* di = nullptr;
  uint8_t* dout = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&di), 4 * n));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&dout), 96));
  HIPCHK(hipMemcpyAsync(di, idx, 4 * n, hipMemcpyHostToDevice, d.stream));
  HIPCHK(bgv_launch_aggregate(di, (uint32_t)n, d.cache, dout, d.stream));
  HIPCHK(hipMemcpyAsync(out96, dout, 96, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));
  (void)hipFree(di);
  (void)hipFree(dout);
  return BGV_OK;
}

int bgv_hash_to_g2(bgv_ctx* c, const uint8_t* msgs, const uint32_t* lens, size_t n, uint8_t* out192) {
  if (!c || (n && (!lens || !out192))) return -BGV_E_ARG;
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
  std::lock_guard<std::mutex> lk(c->mu);
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

// grow every device's cache to hold `need` entries (contents preserved)
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

int bgv_keygen(bgv_ctx* c, const uint8_t* sks, size_t n, int64_t cache_first, uint8_t* out48) {
  if (!c || (n && !sks)) return -BGV_E_ARG;
  if (c->closed) return -BGV_E_CLOSED;
  if (cache_first > (int64_t)c->n_pubkeys) return -BGV_E_ARG;
  if (n == 0) return BGV_OK;
  std::lock_guard<std::mutex> lk(c->mu);
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
  if (cache_first >= 0) c->n_pubkeys = std::max(c->n_pubkeys, (size_t)cache_first + n);
  return BGV_OK;
}

int bgv_sign(bgv_ctx* c, const uint8_t* sks, const uint8_t* msgs, size_t n, uint8_t* out96) {
  if (!c || (n && (!sks || !msgs || !out96))) return -BGV_E_ARG;
  if (c->closed) return -BGV_E_CLOSED;
  if (n == 0) return BGV_OK;
  std::lock_guard<std::mutex> lk(c->mu);
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
  std::lock_guard<std::mutex> lk(c->mu);
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
