# Config-3 latency with the previous library (idle window for every call) against the current
# one (no idle window for calls without batchable jobs), interleaved; then the GPU suite.
# (The change was reverted after this run; lodestar_amd/ab_prev/ held the previous build for it: profiles/r06/idle_window/)
set -o pipefail; O=${1:-gpurun_out/r06idle}; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  BLSGPU_LIB=$PWD/lodestar_amd/ab_prev/libblsgpu.so timeout -k 10 200 python tools/gpu/latency_probe.py 60 >> $O/config3_prev.jsonl 2>> $O/err.txt || exit 1
  timeout -k 10 200 python tools/gpu/latency_probe.py 60 >> $O/config3_new.jsonl 2>> $O/err.txt || exit 1
done
cut -c1-20,150-230 $O/config3_*.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?; tail -3 $O/pytest_gpu.txt; exit $rc
