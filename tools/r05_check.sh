# Round 5: the given GPU tests (TESTS), then optional short bench lines (BENCH="havid shipped ...") and an
# optional kernel-trace profile of one config (PROF=<config>).  Every GPU step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05}; rm -rf $O; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TT:-600} python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/t.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t.log | tail -40; [ $rc -eq 0 ] || exit $rc
fi
for c in ${BENCH:-}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-bf16 --no-dp-overhead --adam-steps 0 \
    > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 5; }
  python -c "import json;d=json.loads(open('$O/b_$c.json').read().splitlines()[-1]);print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'], d['config'].get('tdu_segments'))"
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --config $PROF --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/prof.log 2>&1
  rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $O/prof -name "*kernel_stats.csv"); python tools/kstats.py $f 13 40
fi
