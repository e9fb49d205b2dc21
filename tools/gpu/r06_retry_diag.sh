# Retry-cost diagnostics of the round-6 library: the mainnet-shaped leg at 1 % and 0 % corrupted
# sets (192-call windows), one traced window (BGV_TRACE: per-batch stages and retry rounds), and the
# headline window at 1 % against 0 %, interleaved.
set -o pipefail; O=${1:-gpurun_out/r06retry}; mkdir -p $O; export TMPDIR=/tmp
for c in 0.01 0 0.01 0; do
  timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt $c --steps 192 >> $O/mainnet.jsonl 2>> $O/mainnet.err || exit 1
done
cat $O/mainnet.jsonl
BGV_TRACE=1 timeout -k 10 200 python tools/gpu/mainnet_probe.py 1 --corrupt 0.01 --steps 64 > $O/mainnet_traced.jsonl 2> $O/mainnet_trace.err || exit 1
bash tools/gpu/ab_env.sh $O 2 "c1||" "c0||--corrupt 0" || exit 1
