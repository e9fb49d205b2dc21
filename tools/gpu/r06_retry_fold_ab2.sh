# Mainnet-shaped leg: retry rounds on the residue fold up to 512 tests / always, with one or two retry threads.
set -o pipefail; O=${1:-gpurun_out/r06rfold2}; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for spec in "f0|BGV_RETRY_FOLD_MAX=0" "f512|BGV_RETRY_FOLD_MAX=512" "fall|BGV_RETRY_FOLD_MAX=1000000" "f512t2|BGV_RETRY_FOLD_MAX=512 BGV_RETRY_THREADS=2" "fallt2|BGV_RETRY_FOLD_MAX=1000000 BGV_RETRY_THREADS=2"; do
    IFS='|' read -r tag envs <<< "$spec"
    env $envs timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 192 >> $O/mainnet_$tag.jsonl 2>> $O/err.txt || exit 1
  done
done
for f in $O/mainnet_*.jsonl; do echo $f; cut -c1-40 $f; done
bash tools/gpu/ab_env.sh $O 2 "f0|BGV_RETRY_FOLD_MAX=0|" "fall|BGV_RETRY_FOLD_MAX=1000000|" || exit 1
