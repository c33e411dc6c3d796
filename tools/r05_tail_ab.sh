# A/B of the input block's MS-TCN dW split point (FX_MSTCN_TAIL_SPLIT): bench headline per setting,
# alternating, each run under its own limit.  Output: gpurun_out/tail_ab/*.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/tail_ab; rm -rf $O; mkdir -p $O
for r in ${ROUNDS:-1 2}; do
  for k in ${SPLITS:-0 -1 3 7}; do
    FX_MSTCN_TAIL_SPLIT=$k timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/s${k}_r$r.json 2> $O/s${k}_r$r.err || { tail -5 $O/s${k}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/s${k}_r$r.json').read().strip().splitlines()[-1]); print('split', '$k', 'round', $r, d['ms_per_step'], d['roofline']['frac'])"
  done
done
