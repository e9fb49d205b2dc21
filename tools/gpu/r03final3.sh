# Round-3 record (session end, after steps l-m): GPU suite, smoke, default bench, rocprof kernel stats of the roofline call
# and of the default bench command, PMC passes of the roofline call, node gossip bench.
set -o pipefail
O=gpurun_out/r03final3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo pytest failed; tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo smoke failed; tail $O/smoke.txt; exit 1; }
cat $O/smoke.txt | tail -1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail $O/bench_default.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bench_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || { echo traced bench failed; exit 1; }
timeout -k 10 200 node tests/node/gossip_bench.js 5 64 > $O/gossip.jsonl 2> $O/gossip.err || { echo gossip failed; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']
print('value', round(d['value']/1e6,3), 'frac', round(r['frac'],3), r['kernel_ms_isolated'], 'blk', d['block_import']['p50_latency_ms'], 'agg', round(d['aggregates_1024x128']['value']/1e6,3), 'mainnet', round(d['mainnet_shaped_roots']['value']/1e6,3), 'sweep', round(d['epoch_sweep']['value']/1e6,3), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('host_pool',{}).get('value'))
"
cat $O/gossip.jsonl
