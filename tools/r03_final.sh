# Round-3 measurement of HEAD: smoke, the default bench line (CPU baseline, bf16 and fp32-split modes),
# its kernel-trace stats, the PMC passes of the dominant kernel / attention, the Breakfast, shipped-yaml
# and T=2048 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f3_smoke.log 2>&1 || exit 5
tail -1 gpurun_out/f3_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/f3_bench.json 2> gpurun_out/f3_bench.err || exit 3
cut -c1-200 gpurun_out/f3_bench.json
rm -rf gpurun_out/prof_f3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f3 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/prof_f3.log 2>&1 || exit 4
bash tools/pmc_dominant.sh > gpurun_out/pmc_f3.log 2>&1 || exit 6
timeout -k 10 400 python bench.py --config breakfast > gpurun_out/f3_bench_bf.json 2> gpurun_out/f3_bench_bf.err || exit 7
timeout -k 10 400 python bench.py --config shipped > gpurun_out/f3_bench_shipped.json 2> gpurun_out/f3_bench_shipped.err || exit 8
timeout -k 10 400 python bench.py --T 2048 > gpurun_out/f3_bench_T2048.json 2> gpurun_out/f3_bench_T2048.err || exit 9
for f in f3_bench f3_bench_bf f3_bench_shipped f3_bench_T2048; do python -c "import json;d=json.loads(open('gpurun_out/$f.json').read().splitlines()[-1]);print('$f', d['ms_per_step'], d['value'])"; done
