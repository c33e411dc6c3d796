# A/B of the working tree's Python against a snapshot of another commit's Python (abtmp/old: bench.py + factmx,
# same libfactmx.so through FACTMX_LIB), alternating rounds on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
export FACTMX_LIB=$GRAFT_REPO_ROOT/fact-clip_amd/factmx/_lib/libfactmx.so
for r in $(seq 1 ${ROUNDS:-4}); do
  for side in new old; do
    if [ $side = new ]; then B=bench.py; else B=abtmp/old/bench.py; fi
    timeout -k 10 300 python $B --steps ${STEPS:-30} --warmup 5 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > /tmp/ab.json 2>/tmp/ab.err || { tail -5 /tmp/ab.err; exit 3; }
    python -c "import json; d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); print('$side', d['ms_per_step'])"
  done
done
