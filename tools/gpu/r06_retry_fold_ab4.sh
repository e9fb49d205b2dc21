# Mainnet-shaped leg on the retry-fold library: fold threshold 128 / 512 (default) / 2048, and the default with two retry threads.
set -o pipefail; O=${1:-gpurun_out/r06rfold4}; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for spec in "def|" "f128|BGV_RETRY_FOLD_MAX=128" "f2048|BGV_RETRY_FOLD_MAX=2048" "deft2|BGV_RETRY_THREADS=2"; do
    IFS='|' read -r tag envs <<< "$spec"
    env $envs timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 192 >> $O/mainnet_$tag.jsonl 2>> $O/err.txt || exit 1
  done
done
for f in $O/mainnet_*.jsonl; do echo "$f $(cut -c19-27 $f | tr '\n' ' ')"; done
