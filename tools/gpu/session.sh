set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
bash tools/gpu/record.sh $O suite || exit 1
for i in 1 2; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/new.jsonl 2>>$O/err.txt || { echo new failed; exit 1; }
  BGV_MILLER_1PASS=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/old.jsonl 2>>$O/err.txt || { echo old failed; exit 1; }
done
python tools/gpu/summarize.py $O/new.jsonl $O/old.jsonl
bash tools/gpu/record.sh $O roof
