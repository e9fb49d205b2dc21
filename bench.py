"""Benchmark: verified signature sets/sec at 8192-set batches (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--inflight B] [--no-cpu-baseline] [--no-block-import]

A step = one pass of the hot path over one synthetic batch: bgv_verify of 8192
signature sets (config 4: gossip shape, 8192 batchable one-set jobs, 1 %
corrupted so the batch-fail -> per-job retry path runs), inputs already resident
(pubkey cache on the device, set records in host memory as the C-ABI takes them).

N GPUs: one process per GPU.  Under torchrun the ranks come from the environment; a plain
`python bench.py --gpus N` starts the N rank processes itself (from this parent, which never
touches the GPU) and fails loudly if the ranks that ran differ from --gpus.  Every rank
verifies its own 8192-set batches on its own GPU (jobs shard with no data-path exchange:
scaling "weak"); the slowest rank's time is the job time.  Verdicts of every step are checked
against the expected codes (known by construction, the corruption classes pinned by
tests/test_gpu_parity.py).  The process group is RCCL ("nccl") when the ranks drive distinct
GPUs, gloo for the one-GPU rehearsal (BGV_BENCH_DEVICE) and on CPU.

The JSON line carries:
  roofline     integer-VALU roofline of the dominant kernel: algorithmic u32 MACs
               (Fp-mul-eq counted in profiles/opcounts.json x 288) / its HIP-event time,
               against the gfx950 peak v_mad_u64_u32 rate (16 lanes/clk/SIMD x 1024 SIMDs x 2.4 GHz)
  epoch_sweep  config 5 at N GPUs: 2^20 single sets over a replicated 2^20-key device cache
               (2048 committee roots), one job split over the ranks; each rank reduces its shard
               to one Fp12 Miller-loop product (bgv_verify_partial), the partials are
               all-gathered (RCCL over xGMI at N > 1) and one final exponentiation decides
  cpu_baseline the C++ CPU restatement (oracle/cpu, BlsMultiThreadWorkerPool policy) on a
               bounded sample of the same batch: 16 threads on 16 distinct cores, 16 threads on
               8 SMT core pairs, all affinity threads (os.cpus().length, poolSize.ts:7), and the
               whole-host pool derived from them (the box's cgroup quota caps what one run can
               use); config 1 on one core
  block_import config 3 of BASELINE.json, measured after the timed region: p50 latency of one
               non-batchable 131-set call (randao + 128 attestations x 128 keys + 512-key sync
               aggregate + proposer), one call at a time
  aggregates_1024x128  config 2, also after the timed region: sets/s of 1024-set calls of
               128-key aggregates (8 batchable jobs each), 126 calls in flight
"""
import argparse
import hashlib
import json
import math
import os
import random
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# One HIP stream per in-flight batch; HIP's default of 4 hardware queues per
# process would serialise more than 4.  Read once, at HIP runtime initialisation.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
PEAK_MAC_PER_S = 1024 * 16 * 2.4e9  # v_mad_u64_u32: half rate on SIMD-32 (tools/ubench_valu.hip)
MACS_PER_FP_MUL = 288


def interop_sk(i: int) -> bytes:
    """state-transition/src/util/interop.ts:19-22"""
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return (int.from_bytes(d, "little") % R_ORDER).to_bytes(32, "big")


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a one-GPU box: every rank on this device
    local = int(os.environ.get("BGV_BENCH_DEVICE", local))
    return rank, world, local


def node_devices(world: int, local: int):
    """Devices of the single-process node-shape leg: every GPU of the node (one per rank) at
    N > 1, the rank's own device twice at N = 1 (the two-device split rehearsed on one GPU), and
    under the one-GPU rehearsal of N ranks (BGV_BENCH_DEVICE) that device N times -- so every
    leg the N-GPU run takes also runs in the rehearsal, on the devices that exist."""
    if "BGV_BENCH_DEVICE" in os.environ:
        return [local] * max(world, 2)
    return list(range(world)) if world > 1 else [local, local]


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` without torchrun: N rank processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*
    as torchrun sets them), started from this parent before anything touches the GPU.
    Returns the first nonzero exit status (0 when every rank succeeded)."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc), 0)


class Barrier:
    """Process group of the ranks: barrier, max over ranks, the collective of the epoch
    sweep.  RCCL ("nccl") when the ranks drive distinct GPUs; gloo for the one-GPU
    rehearsal (BGV_BENCH_DEVICE: RCCL refuses two ranks on one device) and on CPU."""

    def __init__(self, world, local=0):
        self.world = world
        self.dist = None
        self.dev = None
        self.backend = None
        if world > 1:
            import torch
            import torch.distributed as dist
            backend = os.environ.get("BGV_BENCH_BACKEND")
            if backend is None:
                backend = "nccl" if ("BGV_BENCH_DEVICE" not in os.environ and torch.cuda.is_available()) else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(local)
                self.dev = torch.device("cuda", local)
            dist.init_process_group(backend, init_method="env://")
            self.dist = dist
            self.backend = backend

    def __call__(self):
        if self.dist:
            if getattr(self, "dev", None) is not None:
                self.dist.barrier(device_ids=[self.dev.index])
            else:
                self.dist.barrier()

    def max(self, v: float) -> float:
        if not self.dist:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=getattr(self, "dev", None) or "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def cuda_sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def default_batching():
    """The library's super-batch geometry at bgv_init (bgv_api.cpp: BGV_MAX_BATCH_SLOTS,
    BGV_COALESCE_US, BGV_IDLE_COALESCE_US), restored after each measurement that changes it."""
    def env(name, dflt):
        try:
            v = int(os.environ.get(name, dflt))
        except ValueError:
            v = dflt
        return v if v >= 0 else dflt
    return env("BGV_MAX_BATCH_SLOTS", 131072), env("BGV_COALESCE_US", 500), env("BGV_IDLE_COALESCE_US", 50)


def undecodable_signatures():
    """Two committed signature encodings that fail to decode beyond a flag bit: an x with no
    curve point (BLST_POINT_NOT_ON_CURVE) and a curve point outside G2 (BLST_POINT_NOT_IN_GROUP),
    the `off_curve` / `not_in_g2` jobs of tests/golden/verdicts.json (data, generated by
    tools/gen_golden.py with the oracle)."""
    jobs = json.load(open(os.path.join(ROOT, "tests", "golden", "verdicts.json")))["jobs"]
    by = {j["name"]: j for j in jobs}
    return (bytes.fromhex(by["off_curve"]["sets"][0]["sig"]), -2), (bytes.fromhex(by["not_in_g2"]["sets"][0]["sig"]), -3)


def make_gossip_batch(ctx, native, rank, nsets, nkeys, corrupt_frac=0.01, seed=0x8192, committee=1):
    """config 4: nsets single sets over distinct validators, distinct signing roots,
    1 % corrupted at random.Random(0x8192).sample positions: a third wrong messages, a third
    wrong keys (false), a third undecodable -- cycling through a flipped compression flag
    (BLST_BAD_ENCODING), an x off the curve (BLST_POINT_NOT_ON_CURVE) and a point outside G2
    (BLST_POINT_NOT_IN_GROUP), SURVEY 8(d) config 4.  committee > 1: mainnet-shaped roots, one per
    `committee` consecutive sets (SURVEY 8(d) "Messages")."""
    key_of = [(rank * nsets + i * 7919) % nkeys for i in range(nsets)]
    msgs = [hashlib.sha256(b"lodestar-bench" + rank.to_bytes(4, "little") + (i // committee).to_bytes(4, "little"))
            .digest() for i in range(nsets)]
    sigs_raw = ctx.sign(b"".join(interop_sk(k) for k in key_of), b"".join(msgs))
    sigs = [sigs_raw[96 * i:96 * i + 96] for i in range(nsets)]
    expect = [1] * nsets
    bad = random.Random(seed).sample(range(nsets), int(round(nsets * corrupt_frac)))
    undecodable = undecodable_signatures()
    for j, i in enumerate(bad):
        if j % 3 == 0:
            msgs[i] = hashlib.sha256(b"wrong" + msgs[i]).digest()
            expect[i] = 0
        elif j % 3 == 1:
            key_of[i] = (key_of[i] + 1) % nkeys
            expect[i] = 0
        elif (j // 3) % 3 == 0:
            sigs[i] = bytes([sigs[i][0] & 0x7F]) + sigs[i][1:]
            expect[i] = -1
        else:
            sigs[i], expect[i] = undecodable[(j // 3) % 3 - 1]
    jobs = [([native.SetSpec(msgs[i], sigs[i], pk_indices=[key_of[i]])], True) for i in range(nsets)]
    return jobs, expect, key_of


def mainnet_shaped_throughput(ctx, native, nkeys, nsets=8192, committee=128, steps=64, warmup=16, settle_s=0.6,
                              corrupt=0.01):
    """config 4 with mainnet-shaped signing roots (one per 128-set committee):
    the same streaming window as the headline; k_prep hashes each distinct root of a call
    once (bgv_dslot.hsrc), so per-set work drops by most of hash_to_G2."""
    jobs, expect, _ = make_gossip_batch(ctx, native, 0, nsets, nkeys, corrupt_frac=corrupt, committee=committee)
    packed = native.PackedCall(jobs)

    def step():
        out = (native.ctypes.c_int32 * len(jobs))()
        st = native.BgvStats()
        rc = ctx.lib.bgv_verify(ctx.handle, packed.jobs, len(jobs), packed.sets, packed.nsets, native.MODE_WORKER,
                                out, native.ctypes.byref(st))
        if rc != 0:
            raise native.DeviceError(native.strerror(rc))
        return list(out), st

    bcalls = super_batch_calls(nsets)
    ncalls = timed_calls(steps, bcalls, int(os.environ.get("BGV_DISPATCHERS", "2")))
    warm_calls = -(-warmup // bcalls) * bcalls
    ctx.set_batching(bcalls * nsets, 200000, 200000)
    try:
        win = stream_window(step, expect, warm_calls, ncalls, 3 * bcalls, settle_s=settle_s, boundary=bcalls)
    finally:
        ctx.set_batching(*default_batching())
    return {"config": "config4 with one signing root per %d sets (%d distinct roots + the corrupted-message "
                      "ones per %d-set batch), %d calls timed after %d warmup calls and >= %.1f s of full load, "
                      "super-batches of %d calls"
                      % (committee, -(-nsets // committee), nsets, ncalls, win["warm_calls"], settle_s, bcalls),
            "value": nsets * ncalls / win["elapsed"], "unit": "sets/s"}


def make_block_import(ctx, native, nkeys):
    """config 3: one non-batchable call of 131 sets as chain/blocks/
    verifyBlocksSignatures.ts:34 sends it: randao (single), 128 aggregate attestations of
    128 distinct validators each, one sync-committee aggregate of 512 validators, and the
    proposer signature (single).  Aggregate signatures sign with the summed secret key, so
    every set is valid; pubkeys are aggregated on the device from the cache."""
    sk_int = lambda i: int.from_bytes(interop_sk(i), "big")
    root = lambda tag, i: hashlib.sha256(b"lodestar-block" + tag + i.to_bytes(4, "little")).digest()
    groups = [("randao", [0])] + [("att", list(range(128 * a, 128 * a + 128))) for a in range(128)]
    groups += [("sync", list(range(16384, 16384 + 512))), ("proposer", [1])]
    assert max(max(k) for _, k in groups) < nkeys, "block import needs >= 16896 cached keys"
    msgs = [root(tag.encode(), i) for i, (tag, _) in enumerate(groups)]
    sks = [(sum(sk_int(k) for k in keys) % R_ORDER).to_bytes(32, "big") for _, keys in groups]
    sigs = ctx.sign(b"".join(sks), b"".join(msgs))
    sets = [native.SetSpec(msgs[i], sigs[96 * i:96 * i + 96], pk_indices=keys) for i, (_, keys) in enumerate(groups)]
    return [(sets, False)]


def block_import_latency(ctx, native, nkeys, runs=100):
    jobs = make_block_import(ctx, native, nkeys)
    packed = native.PackedCall(jobs)  # set records packed once, as the N-API addon hands them over
    out = (native.ctypes.c_int32 * 1)()

    def call():
        rc = ctx.lib.bgv_verify(ctx.handle, packed.jobs, 1, packed.sets, packed.nsets, native.MODE_WORKER, out, None)
        if rc != 0:
            raise native.DeviceError(native.strerror(rc))
        return out[0]

    for _ in range(3):
        assert call() == 1, "block import verdict mismatch"
    lat = []
    for _ in range(runs):
        ts = time.perf_counter()
        got = call()
        lat.append(time.perf_counter() - ts)
        assert got == 1, "block import verdict mismatch"
    n_pk = sum(len(s.pk_indices) for s in jobs[0][0])
    return {"config": "config3: 1 non-batchable call, 131 sets (randao + 128 x 128-key attestations + 512-key sync "
                      "aggregate + proposer), %d pubkeys aggregated on the device" % n_pk,
            "p50_latency_ms": 1e3 * statistics.median(lat), "p90_latency_ms": 1e3 * sorted(lat)[int(0.9 * runs)],
            "runs": runs}


def aggregate_throughput(ctx, native, nkeys, calls=2520, inflight=126, settle_s=0.6):
    """config 2: 1024 aggregate sets x 128 distinct cached keys (contiguous committees),
    distinct signing roots, all valid, sent as the pool sends them (8 batchable jobs of
    128 sets, index.ts:155-166); `calls` such calls streaming with `inflight` outstanding.
    Super-batches hold `inflight` calls, so completions arrive in bursts of `inflight`: the
    rate is taken between the end of the 2nd burst and the end of the last (steady state, no
    pipeline fill or drain inside the window).  126 calls = 129,024 sets + 2,016 group pairs
    = 131,040 k_miller lanes, two whole rounds of one wave per SIMD (128 calls would need a
    third, 2 %-full round: 1.51 vs 1.62 M sets/s, profiles/r02s3/agg_inflight/)."""
    from concurrent.futures import ThreadPoolExecutor
    nsets, per = 1024, 128
    assert nsets * per <= nkeys
    sk_int = [int.from_bytes(interop_sk(i), "big") for i in range(nsets * per)]
    msgs = [hashlib.sha256(b"lodestar-agg" + i.to_bytes(4, "little")).digest() for i in range(nsets)]
    sks = [(sum(sk_int[per * a:per * a + per]) % R_ORDER).to_bytes(32, "big") for a in range(nsets)]
    sigs = ctx.sign(b"".join(sks), b"".join(msgs))
    sets = [native.SetSpec(msgs[a], sigs[96 * a:96 * a + 96], pk_indices=range(per * a, per * a + per))
            for a in range(nsets)]
    jobs = [(sets[j:j + 128], True) for j in range(0, nsets, 128)]
    packed = native.PackedCall(jobs)
    done = []
    lock = threading.Lock()

    def call(_):
        out = (native.ctypes.c_int32 * len(jobs))()
        rc = ctx.lib.bgv_verify(ctx.handle, packed.jobs, len(jobs), packed.sets, packed.nsets, native.MODE_WORKER,
                                out, None)
        if rc != 0:
            raise native.DeviceError(native.strerror(rc))
        with lock:
            done.append(time.perf_counter())
        return list(out)

    assert call(0) == [1] * len(jobs), "config-2 verdict mismatch"
    done.clear()
    ctx.set_batching(inflight * nsets, 20000, 20000)
    t_begin = time.perf_counter()
    try:
        with ThreadPoolExecutor(max_workers=inflight) as pool:
            res = list(pool.map(call, range(calls)))
    finally:
        ctx.set_batching(*default_batching())
    assert all(r == [1] * len(jobs) for r in res), "config-2 verdict mismatch"
    done.sort()
    b = len(done) - 1
    a = 2 * inflight - 1
    while a + inflight < b and done[a] - t_begin < settle_s:
        a += inflight
    rate = nsets * (b - a) / (done[b] - done[a])
    return {"config": "config2: 1024 aggregate sets x 128 cached keys (8 batchable jobs of 128 sets), %d calls "
                      "streaming, %d in flight; rate between the super-batch completion %.2f s into the stream "
                      "(>= %.1f s of full load) and the last" % (calls, inflight, done[a] - t_begin, settle_s),
            "value": rate, "unit": "sets/s", "pubkeys_per_s": rate * per,
            # HBM bytes of the pubkey gather: one 112-B cache entry (affine G1,
            # 28-bit Montgomery limbs) + one 4-B index per aggregated key
            "pubkey_gather_GBps": rate * per * (112 + 4) / 1e9}


def host_cpu():
    """nproc, model name, clock, affinity and the cgroup CPU quota of the host the CPU leg
    runs on (/proc/cpuinfo, /sys/fs/cgroup/cpu.max)."""
    model, mhz = "unknown", None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                k, _, v = ln.partition(":")
                k = k.strip()
                if k == "model name" and model == "unknown":
                    model = v.strip()
                elif k == "cpu MHz" and mhz is None:
                    mhz = float(v)
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": affinity, "model": model, "mhz": mhz, "cgroup_cpus": quota,
            "physical_cores": len(core_groups())}


def core_groups():
    """Logical CPUs of this process's affinity grouped by physical core (SMT siblings,
    /sys/devices/system/cpu/cpu*/topology/thread_siblings_list), in CPU order."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        return [[c] for c in range(os.cpu_count() or 1)]
    groups, seen = [], set()
    for c in cpus:
        if c in seen:
            continue
        sib = [c]
        try:
            txt = open("/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % c).read().strip()
            sib = []
            for part in txt.split(","):
                a, _, b = part.partition("-")
                sib += list(range(int(a), int(b or a) + 1))
            sib = [x for x in sib if x in cpus] or [c]
        except OSError:
            pass
        seen.update(sib)
        groups.append(sib)
    return groups


def timed_pool(blscpu, cj, expect, threads, min_seconds, cpus=None):
    """blscpu.verify_jobs over cj with `threads` workers, repeated for >= min_seconds; the
    workers inherit this thread's CPU affinity (set to `cpus` for the run).  Returns sets/s."""
    old = None
    if cpus is not None and hasattr(os, "sched_setaffinity"):
        old = os.sched_getaffinity(0)
        os.sched_setaffinity(0, cpus)
    try:
        passes, t0 = 0, time.perf_counter()
        while True:
            got = blscpu.verify_jobs(cj, 0, threads)
            passes += 1
            assert got == expect, "CPU restatement disagrees with the expected verdicts"
            dt = time.perf_counter() - t0
            if dt >= min_seconds:
                return len(cj) * passes / dt, passes, dt
    finally:
        if old is not None:
            os.sched_setaffinity(0, old)


def cpu_baseline(jobs, key_of, expect, nsample, min_seconds):
    """The C++ CPU restatement (oracle/cpu: blst's batch equation with 64-bit randomizers
    in width-5 wNAF, 8-pair Miller loops with shared squarings, mulx/adx Montgomery
    products; BlsMultiThreadWorkerPool policy: packages of >= 128 sets over the workers,
    >= 16-job batch chunks, per-job retry) timed on this host on the first `nsample` jobs of
    the same gossip batch, each row repeated for at least `min_seconds` (a bounded sample).

    The reference sizes its pool at os.cpus().length (poolSize.ts:7).  The GPU box grants a
    bench process a cgroup quota of 16 CPUs out of nproc = 256, so the whole-host pool cannot
    run inside one measurement; it is derived from measured rows instead:
      distinct16  16 workers pinned to 16 distinct physical cores (the primary row: `value`)
      smt8x2      16 workers on 8 physical cores x 2 SMT siblings (per-core rate with SMT)
      all         os.cpus().length workers on the whole affinity set (what poolSize.ts does;
                  throttled to the quota here), on 4 copies of the sample so every worker
                  has a 128-set package
      host_pool   smt8x2 per-core rate x the host's physical cores: every core with both SMT
                  threads at the clock 8 busy cores sustain (an all-core load clocks lower,
                  so this favours the CPU)
    Also the config-1 row: one 128-set job on ONE core (BlsSingleThreadVerifier,
    chain/bls/singleThread.ts:7-40, maybeBatch.ts:16-39)."""
    from oracle.cpu import blscpu
    host = host_cpu()
    keys = sorted(set(key_of[:nsample]))
    pk = blscpu.sk_to_pk96(b"".join(interop_sk(k) for k in keys))
    pk_of = {k: pk[96 * i:96 * i + 96] for i, k in enumerate(keys)}
    cj = [([(pk_of[key_of[i]], s.msg, s.sig) for s in sets], b) for i, (sets, b) in enumerate(jobs[:nsample])]
    exp = expect[:nsample]
    groups = core_groups()
    rows = {}
    distinct = [g[0] for g in groups[:16]]
    r, passes, dt = timed_pool(blscpu, cj, exp, len(distinct), min_seconds, set(distinct))
    rows["distinct16"] = {"value": r, "threads": len(distinct), "cpus": len(distinct), "physical_cores": len(distinct),
                          "passes": passes, "seconds": dt}
    pairs = [g[:2] for g in groups if len(g) >= 2][:8]
    if len(pairs) == 8:
        cpus = {c for g in pairs for c in g}
        r2, passes2, dt2 = timed_pool(blscpu, cj, exp, 16, min_seconds, cpus)
        rows["smt8x2"] = {"value": r2, "threads": 16, "cpus": 16, "physical_cores": 8, "passes": passes2,
                          "seconds": dt2, "smt_gain_per_core": 2 * r2 / r}
    nall = host["affinity"] or 1
    r3, passes3, dt3 = timed_pool(blscpu, cj * 4, exp * 4, nall, min_seconds / 2)
    rows["all"] = {"value": r3, "threads": nall, "passes": passes3, "seconds": dt3,
                   "note": "os.cpus().length workers; the cgroup quota (%s CPUs) caps what they get" %
                           host["cgroup_cpus"]}
    per_core = rows["smt8x2"]["value"] / 8 if "smt8x2" in rows else r / 16
    host_pool = per_core * len(groups)
    # config 1: 128 valid single sets as one non-batchable job, one thread
    valid = [i for i in range(nsample) if expect[i] == 1][:128]
    c1 = [([cj[i][0][0] for i in valid], False)]
    t1 = time.perf_counter()
    reps = 0
    while True:
        assert blscpu.verify_jobs(c1, 1, 1) == [1]
        reps += 1
        d1 = time.perf_counter() - t1
        if d1 >= min(3.0, min_seconds):
            break
    return {"value": r, "unit": "sets/s", "cores": len(distinct), "kind": "port",
            "host": host, "rows": rows,
            "host_pool": {"value": host_pool, "unit": "sets/s", "cores": len(groups), "threads": host["affinity"],
                          "derived": "smt8x2 per-core rate (%.0f sets/s) x %d physical cores" % (per_core, len(groups))},
            "config1_single_core": {"value": 128 * reps / d1, "unit": "sets/s", "cores": 1,
                                    "ms_per_job": 1e3 * d1 / reps,
                                    "sample": "%d x one 128-set job (batch equation), 1 thread" % reps},
            "sample": "oracle/cpu/blscpu.cpp (C++ restatement with blst's algorithms, not blst itself): the first %d "
                      "jobs of the same 8192-set gossip batch (1%% corrupt, per-job retry), %d worker threads pinned "
                      "to %d distinct physical cores of %s (%s MHz, nproc %s, cgroup quota %s CPUs), %.1f s; per-core "
                      "%.0f sets/s (reference anchor: ~0.9 ms per single verify with blst-native, "
                      "metrics/lodestar.ts:477)"
                      % (nsample, len(distinct), len(distinct), host["model"], host["mhz"], host["nproc"],
                         host["cgroup_cpus"], dt, r / len(distinct))}


def super_batch_calls(nsets, max_slots=None):
    """Calls per super-batch: as many nsets-set calls as the library's default super-batch
    geometry holds (BGV_MAX_BATCH_SLOTS, 131,072 slots: 16 calls of 8192 sets), whatever the
    step count -- the bench measures the geometry the library ships."""
    if max_slots is None:
        max_slots = default_batching()[0]
    return max(1, max_slots // nsets)


def timed_calls(steps, bcalls, dispatchers=2):
    """Calls inside the timed window: the requested steps rounded up to whole completion
    periods.  Calls of one super-batch complete together and the library keeps one super-batch
    in flight per dispatcher, so completions repeat with a period of bcalls * dispatchers calls;
    a window that ends inside a burst would count calls whose device time it does not hold.
    steps a multiple of the period (64 at the default geometry) are timed exactly."""
    period = bcalls * dispatchers
    return -(-steps // period) * period


def stream_window(step, expect, warmup, steps, inflight, settle_s=0.0, boundary=1):
    """Calls stream continuously, `inflight` outstanding (the pool's concurrent jobs).  The
    timed window runs from the w-th completion to the (w + steps)-th completion, so exactly
    `steps` calls (steps x nsets sets) complete inside it, with the device busy on both sides
    of it; feeding stops once the window is complete and the calls still in flight drain
    untimed.  w is the first multiple of `boundary` that is >= `warmup` and completes at
    least `settle_s` seconds after the stream started (the clock settles at the device's
    power limit within ~0.3 s of full load; profiles/r02s3/warm/)."""
    import threading
    lock = threading.Lock()
    st = {"submitted": 0, "limit": None, "warm": 0 if warmup == 0 and settle_s <= 0 else None}
    done, errors = [], []
    t_begin = time.perf_counter()

    def worker():
        while True:
            with lock:
                if st["limit"] is not None and st["submitted"] >= st["limit"]:
                    return
                st["submitted"] += 1
            ts = time.perf_counter()
            try:
                got, s = step()
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append(e)
                with lock:
                    st["limit"] = st["submitted"]
                return
            t = time.perf_counter()
            with lock:
                done.append((t, t - ts, s, got == expect))
                n = len(done)
                if (st["warm"] is None and n >= warmup and n % boundary == 0
                        and t - t_begin >= settle_s):
                    st["warm"] = n
                if st["warm"] is not None and n >= st["warm"] + steps and st["limit"] is None:
                    st["limit"] = st["submitted"]

    threads = [threading.Thread(target=worker, daemon=True) for _ in range(inflight)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    done.sort(key=lambda d: d[0])
    warmup = st["warm"]
    target = (warmup or 0) + steps
    if warmup is None or len(done) < target or not all(d[3] for d in done):
        raise SystemExit("verdict mismatch")
    t0 = done[warmup - 1][0] if warmup else t_begin
    window = done[warmup:target]
    return {"elapsed": window[-1][0] - t0, "latencies": [d[1] for d in window], "stats": [d[2] for d in window],
            "calls_total": len(done), "warm_calls": warmup}


EPOCH_SETS = 1 << 20
EPOCH_COMMITTEE = 512  # 2048 committee roots over 2^20 sets


def epoch_sweep(ctx, native, barrier, rank, world, nsets=EPOCH_SETS, committee=EPOCH_COMMITTEE):
    """config 5: 2^20 single sets, set i signed by validator i over its
    committee's root (2048 roots), pubkeys from the replicated 2^20-key device cache.  The
    sweep is ONE job split over the ranks (ShardedVerify.one_job_from_shard): each rank's
    contiguous shard becomes one bgv_verify_partial call (its Fp12 Miller-loop product, 576 B),
    the partials are all-gathered over the process group (RCCL over xGMI at N > 1) and every
    rank runs the single final exponentiation.  Timed: barrier + device sync on both sides,
    max over ranks.  Then, untimed, two signatures of the last shard are swapped (both sets
    invalid) and the same protocol must return false on every rank."""
    from lodestar_amd.shard import ShardedVerify, shard_bounds
    lo, hi = shard_bounds([1] * nsets, world)[rank]
    t0 = time.perf_counter()
    sks = [interop_sk(i) for i in range(nsets)]
    if ctx.pubkeys_count() < nsets:
        first = ctx.pubkeys_count()
        ctx.keygen(b"".join(sks[first:]), cache_first=first, want_pubkeys=False)
    roots = [hashlib.sha256(b"lodestar-epoch" + c.to_bytes(4, "little")).digest() for c in range(nsets // committee)]
    msgs = b"".join(roots[i // committee] for i in range(lo, hi))
    sigs = ctx.sign(b"".join(sks[lo:hi]), msgs)
    del sks
    packed = native.PackedSingleSets(msgs, sigs, range(lo, hi))
    setup_s = time.perf_counter() - t0
    sv = ShardedVerify(None, barrier.dist, final_fn=ctx.final_verify) if barrier.dist else None

    def one_pass():
        def shard():
            return ctx.verify_partial_packed(packed, 0, hi - lo)
        if sv is None:
            p, sc, pc = shard()
            if sc or pc:
                return sc or (-6 if pc == 1 else pc)
            return 1 if ctx.final_verify([p]) else 0
        return sv.one_job_from_shard(shard, nsets)

    assert one_pass() == 1, "epoch sweep: valid sweep rejected"  # warm (buffers sized)
    barrier()
    cuda_sync()
    t1 = time.perf_counter()
    code = one_pass()
    cuda_sync()
    barrier()
    elapsed = barrier.max(time.perf_counter() - t1)
    assert code == 1, "epoch sweep: verdict %r" % code
    # corrupted: swap two signatures of the last rank's shard -> false on every rank
    if rank == world - 1 and hi - lo >= 2:
        a, b = packed._sig[0:96].copy(), packed._sig[96:192].copy()
        packed._sig[0:96], packed._sig[96:192] = b, a
    bad = one_pass()
    assert bad == 0, "epoch sweep: corrupted sweep verdict %r" % bad
    return {"config": "config5: 2^20 single sets over a replicated 2^20-key device cache, %d committee roots, one "
                      "job split over %d rank(s): per-rank bgv_verify_partial (Fp12 Miller-loop product), all-gather "
                      "of the 576-B partials (%s), one final exponentiation" %
                      (nsets // committee, world, barrier.backend or "single rank: no collective"),
            "sets": nsets, "sets_per_rank": hi - lo, "value": nsets / elapsed, "unit": "sets/s",
            "ms": 1e3 * elapsed, "setup_s": setup_s, "verdicts": {"valid": code, "two_swapped_signatures": bad}}


def node_shape(native, devices, nkeys, steps, warmup, settle_s, sweep=True):
    """The beacon node's own multi-GPU shape: ONE process drives every
    device through one context, Context(devices), and libblsgpu spreads each big call over them
    (bgv_set_split; the reference's split of a big call over its workers,
    chain/bls/multithread/index.ts:153-166).  Two workloads, beside the rank-based headline:
      gossip  config 4 mode (ii): the same stream of 8192-set calls (8192 batchable one-set jobs,
              1 % corrupted) as the headline, each call cut into one run of jobs per device;
              sets/s over whole completion periods after warmup and the settle time
      sweep   config 5 as one call: 2^20 single sets in ONE job, cut into one run per device whose
              Fp12 Miller-loop partials meet in one final exponentiation; valid, then with two
              signatures swapped (false)
    Every verdict is checked.  devices may repeat an index: Context([0, 0]) rehearses the
    two-device split on one GPU (tests/test_gpu_r04.py checks its verdicts against Context([0]))."""
    ctx = native.Context(list(devices))
    try:
        t0 = time.perf_counter()
        nk = max(nkeys, EPOCH_SETS if sweep else nkeys)
        sks = [interop_sk(i) for i in range(nk)]
        for lo in range(0, nk, 1 << 17):
            ctx.keygen(b"".join(sks[lo:lo + (1 << 17)]), cache_first=lo, want_pubkeys=False)
        jobs, expect, _ = make_gossip_batch(ctx, native, 0, 8192, nkeys)
        packed = native.PackedCall(jobs)
        setup_s = time.perf_counter() - t0

        def step():
            out = (native.ctypes.c_int32 * len(jobs))()
            st = native.BgvStats()
            rc = ctx.lib.bgv_verify(ctx.handle, packed.jobs, len(jobs), packed.sets, packed.nsets,
                                    native.MODE_WORKER, out, native.ctypes.byref(st))
            if rc != 0:
                raise native.DeviceError(native.strerror(rc))
            return list(out), st

        nd = len(devices)
        # a split call becomes nd pinned shard calls of 8192 / nd sets; each device's dispatchers
        # merge the shards in flight into super-batches of the library's default geometry, so
        # completions repeat every (calls per device super-batch) x dispatchers calls
        per_batch = super_batch_calls(max(1, 8192 // nd))
        ncalls = timed_calls(steps, per_batch, int(os.environ.get("BGV_DISPATCHERS", "2")))
        win = stream_window(step, expect, warmup, ncalls, max(32, 3 * per_batch), settle_s=settle_s,
                            boundary=per_batch)
        out = {"devices": list(devices), "setup_s": setup_s,
               "gossip": {"value": 8192 * ncalls / win["elapsed"], "unit": "sets/s", "calls_timed": ncalls,
                          "p50_call_latency_ms": 1e3 * statistics.median(win["latencies"]),
                          "config": "config4 mode (ii): 8192-set calls (8192 batchable one-set jobs, 1%% corrupted) "
                                    "each cut into %d device runs by bgv_set_split, one process" % nd}}
        if sweep:
            n = EPOCH_SETS
            roots = [hashlib.sha256(b"lodestar-epoch" + c.to_bytes(4, "little")).digest()
                     for c in range(n // EPOCH_COMMITTEE)]
            msgs = b"".join(roots[i // EPOCH_COMMITTEE] for i in range(n))
            sigs = bytearray()
            for lo in range(0, n, 1 << 17):
                sigs += ctx.sign(b"".join(sks[lo:lo + (1 << 17)]), msgs[32 * lo:32 * (lo + (1 << 17))])
            one = native.PackedSingleSets(msgs, bytes(sigs), range(n))
            assert ctx.verify_packed_one_job(one) == 1, "node-shape sweep: valid sweep rejected"  # warm
            cuda_sync()
            t1 = time.perf_counter()
            code = ctx.verify_packed_one_job(one)
            dt = time.perf_counter() - t1
            assert code == 1, "node-shape sweep verdict %r" % code
            a, b = 1000, n - 1000
            sigs[96 * a:96 * a + 96], sigs[96 * b:96 * b + 96] = sigs[96 * b:96 * b + 96], sigs[96 * a:96 * a + 96]
            bad = ctx.verify_packed_one_job(native.PackedSingleSets(msgs, bytes(sigs), range(n)))
            assert bad == 0, "node-shape sweep: swapped signatures verdict %r" % bad
            out["sweep"] = {"value": n / dt, "unit": "sets/s", "ms": 1e3 * dt, "sets": n,
                            "verdicts": {"valid": code, "two_swapped_signatures": bad},
                            "config": "config5 as ONE job of 2^20 single sets, cut into %d device runs (Fp12 "
                                      "partials, one final exponentiation), one process" % nd}
        return out
    finally:
        ctx.close()


# PMC bytes per launch of the roofline call for the current kernels (tools/gpu/s3_pmc.sh)
TRAFFIC_FILE = os.path.join("profiles", "r06", "traffic.json")
ROOF_SETS = 64512  # 63 x 1024: with its 1008 group lanes k_miller is one wave on each of the 1024 SIMDs


def roofline_isolated(ctx, native, nkeys):
    """The dominant kernel measured alone at full occupancy: one verify call of ROOF_SETS
    valid one-set jobs (every other stream idle), per-kernel HIP events on the launching
    stream.  k_miller: ROOF_SETS + 1008 lanes = 1024 waves of one wave per SIMD."""
    n = ROOF_SETS
    key_of = [(i * 7919) % nkeys for i in range(n)]
    msgs = [hashlib.sha256(b"lodestar-roof" + i.to_bytes(4, "little")).digest() for i in range(n)]
    sigs = ctx.sign(b"".join(interop_sk(k) for k in key_of), b"".join(msgs))
    jobs = [([native.SetSpec(msgs[i], sigs[96 * i:96 * i + 96], pk_indices=[key_of[i]])], True) for i in range(n)]
    packed = native.PackedCall(jobs)
    out = (native.ctypes.c_int32 * n)()
    ms = {}
    for rep in range(3):
        ctx.profile(1)
        rc = ctx.lib.bgv_verify(ctx.handle, packed.jobs, n, packed.sets, packed.nsets, native.MODE_WORKER, out, None)
        if rc != 0 or any(v != 1 for v in out):
            raise SystemExit("roofline call: verdict mismatch")
        k, launches = ctx.profile(0)
        assert launches == 1
        if rep:  # first call warms up
            for name, v in k.items():
                ms.setdefault(name, []).append(v)
    return {"sets": n, "kernel_ms": {name: statistics.median(v) for name, v in ms.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--nsets", type=int, default=8192)
    ap.add_argument("--nkeys", type=int, default=131072)
    ap.add_argument("--inflight", type=int, default=32,
                    help="batches in flight per GPU (concurrent verify calls, like the reference pool's workers)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=8192, help="jobs per pass timed on the host CPU (cpu_baseline)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum host-CPU time of the cpu_baseline sample")
    ap.add_argument("--no-block-import", action="store_true", help="skip the config-3 latency measurement")
    ap.add_argument("--corrupt", type=float, default=0.01, help="fraction of corrupted sets (config 4: 1%%)")
    ap.add_argument("--settle-s", type=float, default=0.6,
                    help="untimed full-load seconds before the window (on top of --warmup calls) so the window runs "
                         "at the power-settled clock; 0 disables")
    ap.add_argument("--calls-per-batch", type=int, default=0,
                    help="calls merged per device super-batch (default: the library's default geometry, "
                         "BGV_MAX_BATCH_SLOTS // --nsets = 16 calls of 8192 sets)")
    ap.add_argument("--no-epoch-sweep", action="store_true", help="skip the config-5 sweep leg")
    ap.add_argument("--node-shape", choices=["auto", "on", "off"], default="auto",
                    help="the single-process leg over Context(range(N)) with bgv_set_split (rank 0, after the "
                         "timed region): auto = at N > 1 only; at N = 1 'on' rehearses it on Context([0, 0])")
    ap.add_argument("--check-ranks", action="store_true",
                    help="preflight: start the ranks, join the process group, print one line naming the ranks "
                         "and the backend, exit (no GPU work)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    rank, world, local = dist_env()
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but %d rank(s) are running" % (args.gpus, world))
    if args.check_ranks:
        os.environ.setdefault("BGV_BENCH_BACKEND", "gloo")
    barrier = Barrier(world, local)
    if args.check_ranks:
        barrier()
        ranks = barrier.max(float(rank + 1))
        if rank == 0:
            print(json.dumps({"n_gpus": world, "ranks_joined": int(ranks), "backend": barrier.backend,
                              "local_rank_of_rank0": local}), flush=True)
        barrier.close()
        return

    from lodestar_amd import native
    ctx = native.Context([local])
    # device-resident pubkey cache of nkeys interop validators
    t0 = time.perf_counter()
    ctx.keygen(b"".join(interop_sk(i) for i in range(args.nkeys)), cache_first=0, want_pubkeys=False)
    jobs, expect, key_of = make_gossip_batch(ctx, native, rank, args.nsets, args.nkeys, args.corrupt)
    setup_s = time.perf_counter() - t0
    packed = native.PackedCall(jobs)

    def step():
        out = (native.ctypes.c_int32 * len(jobs))()
        st = native.BgvStats()
        rc = ctx.lib.bgv_verify(ctx.handle, packed.jobs, len(jobs), packed.sets, packed.nsets, native.MODE_WORKER,
                                out, native.ctypes.byref(st))
        if rc != 0:
            raise native.DeviceError(native.strerror(rc))
        return list(out), st

    # unloaded latency: one batch at a time
    lat1 = []
    for _ in range(3):
        ts = time.perf_counter()
        got, _ = step()
        lat1.append(time.perf_counter() - ts)
        assert got == expect, "verdict mismatch"
    # Steady state: super-batches of B calls with B | gcd(W, K), so the W-th and the
    # (W+K)-th completions both fall on super-batch boundaries, and a long coalescing window
    # so every super-batch fills to B calls (restored after the timed region)
    ndisp = int(os.environ.get("BGV_DISPATCHERS", "2"))
    bcalls = args.calls_per_batch or super_batch_calls(args.nsets)
    ncalls = timed_calls(args.steps, bcalls, ndisp)
    # the window opens on a super-batch boundary: at least `warmup` calls complete before it,
    # and at least --settle-s seconds of full load (the device's clock settles at its power
    # limit within ~0.3 s; a window inside that boost phase reads up to ~20 % high,
    # profiles/r02s3/warm/)
    warm_calls = -(-args.warmup // bcalls) * bcalls
    ctx.set_batching(bcalls * args.nsets, 200000, 200000)
    ctx.profile(1)
    barrier()
    cuda_sync()
    win = stream_window(step, expect, warm_calls, ncalls, max(args.inflight, 3 * bcalls),
                        settle_s=args.settle_s, boundary=bcalls)
    warm_calls = win["warm_calls"]
    cuda_sync()
    barrier()
    ctx.set_batching(*default_batching())
    elapsed = barrier.max(win["elapsed"])
    lat = win["latencies"]
    stats = win["stats"]
    kms, launches = ctx.profile(0)
    roof = roofline_isolated(ctx, native, args.nkeys) if world == 1 or rank == 0 else None
    block = None
    agg = None
    extras = world == 1 and not args.no_block_import  # N=1 only, outside the timed region
    if extras and args.nkeys >= 16896:
        block = block_import_latency(ctx, native, args.nkeys)
    mainnet = None
    if extras and args.nkeys >= 131072:
        agg = aggregate_throughput(ctx, native, args.nkeys, settle_s=args.settle_s)
        # 192 calls (12 super-batches): the leg's retry rounds come in bursts, and a 64-call window
        # read 2.3-3.7 M sets/s for the same library (profiles/r05/uniform/)
        mainnet = mainnet_shaped_throughput(ctx, native, args.nkeys, steps=192, settle_s=args.settle_s)
    sweep = None if args.no_epoch_sweep else epoch_sweep(ctx, native, barrier, rank, world)
    shape = None
    if args.node_shape == "on" or (args.node_shape == "auto" and world > 1):
        # rank 0 alone, while the other ranks wait at the barrier with their devices idle
        if rank == 0:
            devs = node_devices(world, local)
            shape = node_shape(native, devs, args.nkeys, 64, 16, args.settle_s, sweep=not args.no_epoch_sweep)
        barrier()

    if rank == 0:
        total_sets = args.nsets * ncalls * world
        opc = json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))["fp_mul_eq"]
        per_set = {"k_prep": opc["k_sig"] + opc["k_hash"] + opc["k_pk[n_pk=1]"], "k_miller": opc["k_miller"]}
        # timed region: HIP-event time per launch (a kernel's span includes its overlap with
        # the other in-flight super-batches' kernels on other streams)
        avg = {k: v / max(1, launches) for k, v in kms.items()}
        slots = statistics.mean(s.sets_verified for s in stats)
        groups = statistics.mean(s.device_groups for s in stats)
        # whole-pipeline VALU figure: every verify kernel's counted work over the step time
        per_group = opc["k_final[per group]"] + opc["k_final[group sig pair]"]
        per_slot_close = opc["k_final[per product step]"] + opc["k_final[per slot sig add]"]
        pipeline_macs = ((sum(per_set.values()) + per_slot_close) * slots + per_group * groups) \
            * MACS_PER_FP_MUL * ncalls * world
        pipeline_frac = pipeline_macs / elapsed / (PEAK_MAC_PER_S * world)
        # dominant kernel at full occupancy, alone on the device (roofline_isolated): its
        # algorithmic MACs (set pairs + the group pairs on the same launch) / its HIP-event time
        rk = roof["kernel_ms"]
        dom = max(per_set, key=lambda k: rk.get(k, 0))
        ngr = roof["sets"] // 64
        work = {"k_miller": roof["sets"] * opc["k_miller"] + ngr * opc["k_final[group sig pair]"],
                "k_prep": roof["sets"] * per_set["k_prep"]}[dom]
        achieved = work * MACS_PER_FP_MUL / (rk[dom] * 1e-3)
        # HBM bytes of that same launch from the committed PMC passes (TRAFFIC_FILE:
        # (FETCH_SIZE x 2 + WRITE_SIZE) x 1024, rocprofv3 reports KB) and the algorithmic bytes
        traffic = hbm_gbs = None
        tf = os.path.join(ROOT, TRAFFIC_FILE)
        if os.path.exists(tf):
            rec = json.load(open(tf)).get(dom, {})
            if rec.get("sets") == roof["sets"]:
                traffic = rec["bytes_per_launch"]
                hbm_gbs = traffic / (rk[dom] * 1e-3) / 1e9
        alg_bytes = {"k_miller": roof["sets"] * (112 + 336 + 672 + 8 + 160) + ngr * (336 + 672),
                     "k_prep": roof["sets"] * (160 + 4 + 112 * 1 + 336 * 2 + 112 + 8)}[dom]
        line = {
            "metric": "verified signature sets/sec (node) at 8192-set batches",
            "value": total_sets / elapsed,
            "unit": "sets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / ncalls,
            "timed_steps": ncalls,
            "p50_batch_latency_ms": 1e3 * statistics.median(lat),
            "p50_batch_latency_ms_unloaded": 1e3 * statistics.median(lat1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (28-bit-limb Montgomery Fp, v_mad_u64_u32)",
            "data": "synthetic: interop validator keys (%d in the device cache), distinct 32-B signing roots, "
                    "device-signed; 1%% corrupted (wrong msg / wrong key / undecodable: bad encoding, off curve, "
                    "not in G2)" % args.nkeys,
            "config": {"workload": "config4: 8192-set gossip batch (8192 batchable one-set jobs, BGV_MODE_WORKER, "
                                   "batch-fail -> per-job retry)", "sets_per_batch": args.nsets,
                       "batches_in_flight": max(args.inflight, 3 * bcalls), "calls_per_super_batch": bcalls,
                       "parallelism": "dp%d (independent batches per GPU)" % world},
            "timing": "steady state: calls stream with the given number in flight; the window runs from the "
                      "%d-th to the %d-th completed call (exactly %d calls inside: the %d requested steps rounded "
                      "up to whole completion periods of %d dispatchers x %d-call super-batches, the library's "
                      "default geometry, so both edges fall on batch boundaries; the %d warmup steps are the first "
                      "%d completions, rounded up to whole super-batches and extended to >= %.1f s of full load so "
                      "the window runs at the power-settled clock); %d calls completed in all"
                      % (warm_calls, warm_calls + ncalls, ncalls, args.steps, ndisp, bcalls, args.warmup, warm_calls,
                         args.settle_s, win["calls_total"]),
            "kernel_ms_per_launch": avg,
            "retries_per_step": statistics.mean(s.batch_retries for s in stats),
            "call_device_ms": statistics.mean(s.device_ms for s in stats),
            "call_wall_ms": statistics.mean(s.wall_ms for s in stats),
            "device_groups_per_step": statistics.mean(s.device_groups for s in stats),
            "roofline": {"bound": "valu", "kernel": dom, "achieved": achieved / 1e12, "peak": PEAK_MAC_PER_S / 1e12,
                         "unit": "TMAC/s (u32 mad)", "frac": achieved / PEAK_MAC_PER_S, "traffic": traffic,
                         "measured": "one %d-set verify call alone on the device after the timed region (k_miller: "
                                     "%d set pairs + %d group pairs = one wave per SIMD), HIP events on the "
                                     "launching stream, median of 2" % (roof["sets"], roof["sets"], ngr),
                         "work_per_set": "%d Fp-mul-eq x %d MAC" % (per_set[dom], MACS_PER_FP_MUL),
                         "sets_per_launch": roof["sets"], "ms_per_launch": rk[dom],
                         "kernel_ms_isolated": rk,
                         "traffic_unit": "HBM bytes per launch (PMC (FETCH_SIZE x 2 + WRITE_SIZE) x 1024)",
                         "algorithmic_bytes": alg_bytes,
                         "hbm_GBps": hbm_gbs, "hbm_frac_of_8TBps": hbm_gbs / 8000 if hbm_gbs else None,
                         "pipeline_frac": pipeline_frac},
            "setup_s": setup_s,
        }
        if block is not None:
            line["block_import"] = block
        if agg is not None:
            line["aggregates_1024x128"] = agg
        if mainnet is not None:
            line["mainnet_shaped_roots"] = mainnet
        if sweep is not None:
            line["epoch_sweep"] = sweep
        if shape is not None:
            line["node_single_process"] = shape
        if not args.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            cb = cpu_baseline(jobs, key_of, expect, min(args.nsets, args.cpu_sample), args.cpu_seconds)
            line["cpu_baseline"] = cb
            # BASELINE.md publishes no number for this metric, so vs_baseline stays null; the ratio
            # the north star names (GPU sets/s over the host's whole blst-style worker pool) is
            # reported beside it
            line["vs_host_pool"] = line["value"] / cb["host_pool"]["value"]
            line["vs_host_pool_basis"] = ("value / cpu_baseline.host_pool (the C++ restatement's pool over all %d "
                                          "physical cores of this host, derived from pinned rows)" %
                                          cb["host_pool"]["cores"])
        print(json.dumps(line), flush=True)
    ctx.close()
    barrier.close()


if __name__ == "__main__":
    main()
