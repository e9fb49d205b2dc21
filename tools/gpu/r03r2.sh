# eight-part products in k_final_fold: GPU suite first, then config-3 latency kernels and Node gossip
set -o pipefail
O=gpurun_out/r03r2; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest.txt 2>&1 || { echo pytest failed; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 120 python tools/gpu/latency_probe.py 40 > $O/lat.json 2>>$O/err || exit 1
cat $O/lat.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/gpu/latency_probe.py 20 > $O/prof.txt 2>&1 || exit 1
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | head -8

timeout -k 10 120 node tests/node/gossip_bench.js 4 64 "63:1" > $O/gossip.jsonl 2>>$O/err || exit 1
cat $O/gossip.jsonl
