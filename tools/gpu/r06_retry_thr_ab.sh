# Retry threads: one, two (spill 0: either takes any hand-over), two gated on a backlog (spill 1);
# headline (3 interleaved rounds) and the mainnet-shaped leg (2 rounds).
# (BGV_RETRY_SPILL was a trial knob, reverted after this run: profiles/r06/retry_threads/)
set -o pipefail; O=${1:-gpurun_out/r06rthr}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/ab_env.sh $O 3 "base||" "thr2s0|BGV_RETRY_THREADS=2 BGV_RETRY_SPILL=0|" "thr2s1|BGV_RETRY_THREADS=2 BGV_RETRY_SPILL=1|" || exit 1
for i in 1 2; do
  for spec in "base|" "thr2s0|BGV_RETRY_THREADS=2 BGV_RETRY_SPILL=0" "thr2s1|BGV_RETRY_THREADS=2 BGV_RETRY_SPILL=1"; do
    IFS='|' read -r tag envs <<< "$spec"
    env $envs timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 192 >> $O/mainnet_$tag.jsonl 2>> $O/err.txt || exit 1
  done
done
for f in $O/mainnet_*.jsonl; do echo $f; cut -c1-40 $f; done
