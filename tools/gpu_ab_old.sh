#!/bin/bash
# Same-box A/B against the round-3 tree built in ./ab_old (git worktree of 77ff8bf, untracked).
# usage: tools/gpu_ab_old.sh "label:dir:ENV=V:bench args" ...
set -u
R=$(pwd)
for spec in "$@"; do
  IFS=: read -r lab d envs args <<< "$spec"
  (cd $d && env $envs timeout -k 10 300 python -u bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/ab.json 2> $R/gpurun_out/ab.err) || { tail -5 $R/gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/ab.json')); print('$lab', d['ms_per_step'], d['roofline']['frac'])"
done
