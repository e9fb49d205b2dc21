# Uniform-gated retry fold (default BGV_RETRY_FOLD_MAX=512 for uniform batches) against 0: GPU suite,
# mainnet-shaped (3 interleaved rounds), headline (2 rounds).
set -o pipefail; O=${1:-gpurun_out/r06rfold3}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc = 0 ] || exit $rc
for i in 1 2 3; do
  for spec in "f0|BGV_RETRY_FOLD_MAX=0" "def|BGV_RETRY_FOLD_MAX=512"; do
    IFS='|' read -r tag envs <<< "$spec"
    env $envs timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 192 >> $O/mainnet_$tag.jsonl 2>> $O/err.txt || exit 1
  done
done
for f in $O/mainnet_*.jsonl; do echo "$f $(cut -c19-27 $f | tr '\n' ' ')"; done
bash tools/gpu/ab_env.sh $O 2 "f0|BGV_RETRY_FOLD_MAX=0|" "def||" || exit 1
