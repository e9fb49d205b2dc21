#!/bin/bash
# One GPU-box session, parameterised (replaces the per-experiment session scripts of round 3).
#   tools/gpu/record.sh OUTDIR STEP...
# Steps, run in the order given; the first failing GPU step ends the session (no retries):
#   suite    pytest -m gpu (thread timeouts, one process)
#   smoke    __graft_entry__.smoke()
#   bench    python bench.py (the default command the driver runs)  -> OUTDIR/bench_default.json
#   quick    bench headline window only (no CPU baseline, no extras) -> OUTDIR/bench_quick.jsonl (appends)
#   driver   the headline window with the driver's step counts (--steps 20 --warmup 5) and with
#            the default ones (64 / 16), back to back                 -> OUTDIR/bench_steps.jsonl (appends)
#   trace    rocprofv3 --kernel-trace --stats of the bench command   -> OUTDIR/bench_trace/
#   retrytrace  kernel traces of the headline window with 1 % corrupted sets and with none, and
#            one BGV_TRACE run of the corrupted window (its retry rounds)   -> OUTDIR/retry_{c1,c0}/, retry_trace.err
#   roof     rocprofv3 --kernel-trace --stats of the isolated roofline call -> OUTDIR/roof_trace/
#   pmc      the PMC passes of the roofline call (tools/gpu/pmc.sh)  -> gpurun_out/<basename OUTDIR>/pmc
#   latency  config-3 latency probe under a kernel trace              -> OUTDIR/config3_p50.json, lat_trace/
#   gossip   Node 64-caller gossip bench                             -> OUTDIR/gossip.jsonl
#   gossip_cpu  the same callers over the C++ port (CpuPoolVerifier, 16 workers) -> OUTDIR/gossip_cpu.jsonl
#   ubench   the VALU / product microbenchmarks                      -> OUTDIR/ubench_*.jsonl
set -o pipefail
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
fail() { echo "step $1 failed (rc=$2)"; tail -20 "$3" 2>/dev/null; exit 1; }
for step in "$@"; do
  case $step in
    suite)
      timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
        > "$O/pytest_gpu.txt" 2>&1 || fail suite $? "$O/pytest_gpu.txt"
      tail -1 "$O/pytest_gpu.txt" ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 \
        || fail smoke $? "$O/smoke.txt"
      tail -1 "$O/smoke.txt" ;;
    bench)
      timeout -k 10 300 python bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" \
        || fail bench $? "$O/bench_default.err"
      python tools/gpu/summarize.py "$O/bench_default.json" ;;
    quick)
      timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep \
        >> "$O/bench_quick.jsonl" 2>> "$O/bench_quick.err" || fail quick $? "$O/bench_quick.err"
      tail -1 "$O/bench_quick.jsonl" | python tools/gpu/summarize.py - ;;
    driver)
      for sw in "20 5" "64 16"; do
        read -r ks kw <<< "$sw"
        timeout -k 10 150 python bench.py --steps $ks --warmup $kw --no-cpu-baseline --no-block-import --no-epoch-sweep \
          >> "$O/bench_steps.jsonl" 2>> "$O/bench_steps.err" || fail driver $? "$O/bench_steps.err"
      done
      tail -2 "$O/bench_steps.jsonl" | python tools/gpu/summarize.py - ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/bench_trace" -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline > "$O/bench_traced.json" 2> "$O/bench_traced.err" \
        || fail trace $? "$O/bench_traced.err" ;;
    retrytrace)
      for c in 1 0; do
        timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/retry_c$c" -o run --output-format csv \
          -- python3 bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep --corrupt 0.0$c \
          > "$O/retry_c$c.json" 2> "$O/retry_c$c.err" || fail retrytrace $? "$O/retry_c$c.err"
      done
      BGV_TRACE=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep \
        > "$O/retry_trace.json" 2> "$O/retry_trace.err" || fail retrytrace $? "$O/retry_trace.err"
      cat "$O"/retry_c*.json | python tools/gpu/summarize.py - ;;
    roof)
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/roof_trace" -o run --output-format csv \
        -- python3 tools/gpu/roof_call.py > "$O/roof_call.json" 2> "$O/roof_call.err" \
        || fail roof $? "$O/roof_call.err"
      cat "$O/roof_call.json" ;;
    pmc)
      TAG=$(basename "$O") bash tools/gpu/pmc.sh || fail pmc $? /dev/null ;;
    latency)
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/lat_trace" -o run --output-format csv \
        -- python3 tools/gpu/latency_probe.py 30 > "$O/config3_p50.json" 2> "$O/lat.err" \
        || fail latency $? "$O/lat.err"
      cat "$O/config3_p50.json" ;;
    gossip)
      timeout -k 10 200 node tests/node/gossip_bench.js 5 64 > "$O/gossip.jsonl" 2> "$O/gossip.err" \
        || fail gossip $? "$O/gossip.err"
      cat "$O/gossip.jsonl" ;;
    gossip_cpu)
      python tests/node/build_cpu.py > /dev/null || fail build_cpu $? /dev/null
      timeout -k 10 200 node tests/node/gossip_bench.js 8 64 "" cpu 16 > "$O/gossip_cpu.jsonl" 2> "$O/gossip_cpu.err" \
        || fail gossip_cpu $? "$O/gossip_cpu.err"
      cat "$O/gossip_cpu.jsonl" ;;
    ubench)
      for u in ubench_valu ubench_fpmul ubench_prod ubench_wfp; do
        [ -x tools/$u ] || continue
        timeout -k 10 120 tools/$u > "$O/$u.jsonl" 2>&1 || fail $u $? "$O/$u.jsonl"
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
