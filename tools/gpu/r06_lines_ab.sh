# GPU suite, then the projective line walk (default) against the Jacobian one (libblsgpu_linesjac):
# the isolated roofline call (k_lines time) and the headline window, interleaved.
set -o pipefail; O=${1:-gpurun_out/r06lines}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for i in 1 2; do
  for L in lodestar_amd/libblsgpu.so lodestar_amd/libblsgpu_linesjac.so; do
    tag=$(basename $L .so)
    BLSGPU_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/roof_$tag$i -o run --output-format csv -- python3 tools/gpu/roof_call.py >> $O/roof_$tag.jsonl 2>> $O/err.txt || exit 1
    BLSGPU_LIB=$L timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/quick_$tag.jsonl 2>> $O/err.txt || exit 1
  done
done
for f in $O/quick_*.jsonl; do python tools/gpu/summarize.py $f; done
for d in $O/roof_*[12]; do echo $d; grep -E '"k_lines"|"k_facc"|"k_prep"' $d/run_kernel_stats.csv | cut -d, -f1-4; done
