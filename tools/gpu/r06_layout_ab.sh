# GPU suite, then the mainnet-shaped leg (192-call windows) and the headline window, interleaved,
# for the root-aligned layout (default library) against the round-5 layout (libblsgpu_r05layout).
set -o pipefail; O=${1:-gpurun_out/r06layout}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for i in 1 2; do
  for L in lodestar_amd/libblsgpu.so lodestar_amd/libblsgpu_r05layout.so; do
    tag=$(basename $L .so)
    BLSGPU_LIB=$L timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 192 >> $O/mainnet_$tag.jsonl 2>> $O/err.txt || exit 1
    BLSGPU_LIB=$L timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/quick_$tag.jsonl 2>> $O/err.txt || exit 1
  done
done
timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0 --steps 192 >> $O/mainnet_clean.jsonl 2>> $O/err.txt || exit 1
for f in $O/mainnet_*.jsonl; do echo $f; cut -c1-60 $f; done
for f in $O/quick_*.jsonl; do python tools/gpu/summarize.py $f; done
BGV_TRACE=1 timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 64 > $O/mainnet_traced.jsonl 2> $O/mainnet_trace.err || exit 1
