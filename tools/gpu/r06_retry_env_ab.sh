# Retry-thread settings on the mainnet-shaped leg (192-call windows) and the headline, interleaved.
set -o pipefail; O=${1:-gpurun_out/r06renv}; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for spec in "base|" "thr2|BGV_RETRY_THREADS=2" "hold2|BGV_RETRY_HOLD=2"; do
    IFS='|' read -r tag envs <<< "$spec"
    env $envs timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 192 >> $O/mainnet_$tag.jsonl 2>> $O/err.txt || exit 1
  done
done
for f in $O/mainnet_*.jsonl; do echo $f; cut -c1-40 $f; done
bash tools/gpu/ab_env.sh $O 2 "base||" "thr2|BGV_RETRY_THREADS=2|" || exit 1
