# Round-4 closing measurement of HEAD, in two calls (each well inside gpurun's limit):
#   bash tools/r04_final.sh 1  -- the GPU test suite, smoke, the driver's bench command, its kernel-trace
#                                 stats and the PMC passes (tools/pmc_dominant.sh)
#   bash tools/r04_final.sh 2  -- the Breakfast / shipped / T=2048 lines and the GRU micro-benchmark
# KERNEL= selects the dominant kernel for the PMC summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/f4
if [ "${1:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/f4/pytest.log 2>&1 || { tail -30 gpurun_out/f4/pytest.log; exit 2; }
  tail -1 gpurun_out/f4/pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4/smoke.log 2>&1 || exit 5
  tail -1 gpurun_out/f4/smoke.log
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/f4/bench.json 2> gpurun_out/f4/bench.err || exit 3
  cut -c1-300 gpurun_out/f4/bench.json
  rm -rf gpurun_out/f4/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f4/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > gpurun_out/f4/prof.log 2>&1 || exit 4
  bash tools/pmc_dominant.sh > gpurun_out/f4/pmc.log 2>&1 || exit 6
else
  for cfg in breakfast shipped; do
    timeout -k 10 400 python bench.py --config $cfg > gpurun_out/f4/bench_$cfg.json 2> gpurun_out/f4/bench_$cfg.err || exit 7
  done
  timeout -k 10 400 python bench.py --T 2048 > gpurun_out/f4/bench_T2048.json 2> gpurun_out/f4/bench_T2048.err || exit 8
  timeout -k 10 120 python -u tools/r04_gru_bench.py > gpurun_out/f4/gru.log 2>&1 || exit 9
  for f in bench_breakfast bench_shipped bench_T2048; do python -c "import json;d=json.loads(open('gpurun_out/f4/$f.json').read().splitlines()[-1]);print('$f', d['ms_per_step'], d['value'], d['roofline']['frac'])"; done
fi
