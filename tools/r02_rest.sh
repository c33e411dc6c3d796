set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; TAG=r02b
timeout -k 10 400 python bench.py --config breakfast --steps 10 --warmup 3 > gpurun_out/bench_bf_$TAG.json 2> gpurun_out/bench_bf_$TAG.err
rc=$?; echo "bench breakfast exit $rc"; cut -c1-300 gpurun_out/bench_bf_$TAG.json; tail -3 gpurun_out/bench_bf_$TAG.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_dominant.sh > gpurun_out/pmc.log 2>&1; echo "pmc exit $?"
