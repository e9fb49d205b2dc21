# Round-4 session: microbenchmarks, GPU suite, config-3 latency under a kernel trace, the Node
# gossip rows (GPU and CPU port), then the headline window with the weighted retry tests, without
# them (BGV_WEIGHTED=0) and without corrupted sets, interleaved twice.
#   bash tools/gpu/sess_i.sh OUTDIR
set -o pipefail
O=$1; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu/record.sh $O ubench suite latency gossip gossip_cpu || exit 1
for i in 1 2; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/quick_weighted.jsonl 2>>$O/err.txt || { echo quick failed; exit 1; }
  BGV_WEIGHTED=0 timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/quick_noweight.jsonl 2>>$O/err.txt || { echo quick0 failed; exit 1; }
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep --corrupt 0 >> $O/quick_clean.jsonl 2>>$O/err.txt || { echo clean failed; exit 1; }
done
for f in quick_weighted quick_noweight quick_clean; do python tools/gpu/summarize.py $O/$f.jsonl; done
