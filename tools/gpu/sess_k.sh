# Round-4 session k: retry-path A/B on the headline window (1 % corrupted): one retry thread
# (default), two retry threads, two retry threads with the weighted tests; and --corrupt 0,
# interleaved twice.
#   bash tools/gpu/sess_k.sh OUTDIR
set -o pipefail
O=$1; mkdir -p $O
export TMPDIR=/tmp
Q="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2; do
  timeout -k 10 150 $Q >> $O/r1.jsonl 2>>$O/err.txt || { echo r1 failed; exit 1; }
  BGV_RETRY_THREADS=2 timeout -k 10 150 $Q >> $O/r2.jsonl 2>>$O/err.txt || { echo r2 failed; exit 1; }
  BGV_RETRY_THREADS=2 BGV_WEIGHTED=1 timeout -k 10 150 $Q >> $O/r2w.jsonl 2>>$O/err.txt || { echo r2w failed; exit 1; }
  BGV_RETRY_THREADS=3 BGV_EXECS=6 timeout -k 10 150 $Q >> $O/r3.jsonl 2>>$O/err.txt || { echo r3 failed; exit 1; }
  timeout -k 10 150 $Q --corrupt 0 >> $O/clean.jsonl 2>>$O/err.txt || { echo clean failed; exit 1; }
done
for f in r1 r2 r2w r3 clean; do python tools/gpu/summarize.py $O/$f.jsonl; done
