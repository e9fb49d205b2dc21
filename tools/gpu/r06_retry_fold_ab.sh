# Retry rounds closing on the residue fold (BGV_RETRY_FOLD_MAX tests or fewer): the GPU suite with
# every retry round on it, then headline and mainnet-shaped A/B against k_final12 (0).
set -o pipefail; O=${1:-gpurun_out/r06rfold}; mkdir -p $O; export TMPDIR=/tmp
BGV_RETRY_FOLD_MAX=1000000 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_allfold.txt 2>&1; rc=$?; tail -3 $O/pytest_gpu_allfold.txt; [ $rc = 0 ] || exit $rc
bash tools/gpu/ab_env.sh $O 2 "f0|BGV_RETRY_FOLD_MAX=0|" "f64|BGV_RETRY_FOLD_MAX=64|" "f512|BGV_RETRY_FOLD_MAX=512|" || exit 1
for i in 1 2; do
  for v in 0 64 512; do
    BGV_RETRY_FOLD_MAX=$v timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 192 >> $O/mainnet_f$v.jsonl 2>> $O/err.txt || exit 1
  done
done
for f in $O/mainnet_*.jsonl; do echo $f; cut -c1-40 $f; done
