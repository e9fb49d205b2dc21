# one-product rounds written straight to their slot: round ubench, config-3 latency kernels, GPU suite
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc tools/ubench_round.hip -o /tmp/ubench_round && timeout -k 10 120 /tmp/ubench_round > $O/round.jsonl || exit 1
cat $O/round.jsonl
timeout -k 10 120 python tools/gpu/latency_probe.py 40 > $O/lat.json 2>>$O/err || exit 1
cat $O/lat.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/gpu/latency_probe.py 20 > $O/prof.txt 2>&1 || exit 1
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | head -8
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest.txt 2>&1; echo pytest rc=$?; tail -2 $O/pytest.txt
