# default bench (full line) + PMC passes and kernel trace of the isolated roofline call
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value']/1e6,3), 'frac', round(r['frac'],3), r['kernel_ms_isolated'], 'blk', d['block_import']['p50_latency_ms'], 'agg', round(d['aggregates_1024x128']['value']/1e6,3), 'mainnet', round(d['mainnet_shaped_roots']['value']/1e6,3), 'sweep', round(d['epoch_sweep']['value']/1e6,3), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('host_pool',{}).get('value'))
"
TAG=r03l bash tools/gpu/pmc.sh
