# Round-4 session l: the four-wave round engine against the four-part one (bit-exact banks,
# time per [|x|]P chain), the GPU suite with BGV_WIDE4=1, config-3 latency and the Node gossip
# rate with and without it, then a long-window retry A/B (one retry thread vs two with the
# weighted tests).
#   bash tools/gpu/sess_l.sh OUTDIR
set -o pipefail
O=$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/ubench_wround > $O/ubench_wround.jsonl 2>&1 || { cat $O/ubench_wround.jsonl; echo wround failed; exit 1; }
cat $O/ubench_wround.jsonl
BGV_WIDE4=1 timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_wide4.txt 2>&1 || { tail -30 $O/pytest_wide4.txt; echo suite failed; exit 1; }
tail -1 $O/pytest_wide4.txt
for i in 1 2; do
  timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_two.jsonl 2>>$O/err.txt || { echo lat failed; exit 1; }
  BGV_WIDE4=1 timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_wide4.jsonl 2>>$O/err.txt || { echo lat4 failed; exit 1; }
done
cat $O/lat_two.jsonl $O/lat_wide4.jsonl
BGV_WIDE4=1 timeout -k 10 200 node tests/node/gossip_bench.js 5 64 "63:1" > $O/gossip_wide4.jsonl 2> $O/gossip.err || { echo gossip failed; exit 1; }
cat $O/gossip_wide4.jsonl
Q="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep --steps 256 --warmup 32"
for i in 1 2; do
  timeout -k 10 200 $Q >> $O/long_r1.jsonl 2>>$O/err.txt || { echo r1 failed; exit 1; }
  BGV_RETRY_THREADS=2 BGV_WEIGHTED=1 timeout -k 10 200 $Q >> $O/long_r2w.jsonl 2>>$O/err.txt || { echo r2w failed; exit 1; }
done
for f in long_r1 long_r2w; do python tools/gpu/summarize.py $O/$f.jsonl; done
