# GPU suite, then interleaved config-3 latency and Node gossip A/Bs of the RNS latency kernels
# (BGV_PREP_RNS / BGV_FOLD_RNS), and a kernel trace of the config-3 call.
#   bash tools/gpu/rns_session.sh OUTDIR
set -o pipefail; O=${1:-gpurun_out/r06rns}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for i in 1 2; do
  for v in "1 1" "0 1" "0 0"; do
    read -r pr fr <<< "$v"
    BGV_PREP_RNS=$pr BGV_FOLD_RNS=$fr timeout -k 10 200 python tools/gpu/latency_probe.py 40 >> $O/config3_prep${pr}_fold${fr}.jsonl 2>>$O/lat.err || exit 1
  done
done
for f in $O/config3_*.jsonl; do echo $f; cut -c1-300 $f | grep -o '"p50_latency_ms": [0-9.]*'; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o run --output-format csv -- python3 tools/gpu/latency_probe.py 30 > $O/config3_traced.json 2> $O/lat_trace.err || exit 1
for v in "1 1" "0 1" "0 0"; do
  read -r pr fr <<< "$v"
  BGV_PREP_RNS=$pr BGV_FOLD_RNS=$fr timeout -k 10 200 node tests/node/gossip_bench.js 5 64 >> $O/gossip_prep${pr}_fold${fr}.jsonl 2>> $O/gossip.err || exit 1
done
for f in $O/gossip_*.jsonl; do echo $f; head -1 $f; done
