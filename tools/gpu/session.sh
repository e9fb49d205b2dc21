# A/B session: GPU suite on the default library, then the isolated roofline call and the
# headline window for each library given (default first), interleaved.
#   bash tools/gpu/session.sh OUTDIR LIB...
set -o pipefail
O=$1; shift; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu/record.sh $O ${PRE:-suite} || exit 1
for i in 1 2; do
  for L in "$@"; do
    tag=$(basename $L .so)
    BLSGPU_LIB=$L timeout -k 10 200 python tools/gpu/roof_call.py >> $O/roof_$tag.jsonl 2>>$O/err.txt || { echo roof $tag failed; exit 1; }
    BLSGPU_LIB=$L timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/quick_$tag.jsonl 2>>$O/err.txt || { echo quick $tag failed; exit 1; }
  done
done
for L in "$@"; do tag=$(basename $L .so); echo $tag; cat $O/roof_$tag.jsonl; python tools/gpu/summarize.py $O/quick_$tag.jsonl; done
