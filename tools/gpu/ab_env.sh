#!/bin/bash
# Interleaved A/B of environment settings on the headline window (no CPU baseline, no extras).
#   tools/gpu/ab_env.sh OUTDIR ROUNDS "tag|ENV=V ENV2=V|bench args" ...
# e.g. "fpw||" "nofpw|BGV_FPW=0|" "clean||--corrupt 0"
set -o pipefail
O=$1; N=$2; shift 2
mkdir -p "$O"
export TMPDIR=/tmp
for i in $(seq 1 "$N"); do
  for spec in "$@"; do
    IFS='|' read -r tag envs args <<< "$spec"
    env $envs timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep $args \
      >> "$O/ab_$tag.jsonl" 2>> "$O/ab_$tag.err" || { echo "bench $tag rc=$?: stopping"; exit 1; }
    tail -1 "$O/ab_$tag.jsonl" | python tools/gpu/summarize.py - | sed "s/^-/$tag/"
  done
done
