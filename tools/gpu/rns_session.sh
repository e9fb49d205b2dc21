set -o pipefail; O=gpurun_out/r06rns; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for v in 1 0 1 0; do BGV_FOLD_RNS=$v timeout -k 10 200 python tools/gpu/latency_probe.py 40 >> $O/config3_rns$v.jsonl 2>>$O/lat.err || exit 1; done
cat $O/config3_*.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o run --output-format csv -- python3 tools/gpu/latency_probe.py 30 > $O/config3_traced.json 2> $O/lat_trace.err || exit 1
for v in 1 0; do BGV_FOLD_RNS=$v timeout -k 10 200 node tests/node/gossip_bench.js 5 64 >> $O/gossip_rns$v.jsonl 2>> $O/gossip.err || exit 1; done
cat $O/gossip_*.jsonl
