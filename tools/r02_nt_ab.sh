# A/B: non-temporal stores in the fast GEMM epilogue (FX_GEMM_NTSTORE=1) vs default, alternating,
# plus the standalone conv GEMM micro-benchmark under both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
ROWS=8192 timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/nt_gb_def.txt 2>/dev/null || exit 3
ROWS=8192 FX_GEMM_NTSTORE=1 timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/nt_gb_nt.txt 2>/dev/null || exit 3
echo default; sed -n 1,5p gpurun_out/nt_gb_def.txt; echo nt; sed -n 1,5p gpurun_out/nt_gb_nt.txt
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 \
    > gpurun_out/nt_$name.json 2>/dev/null || return 1
  python -c "import json; d=json.load(open('gpurun_out/nt_$name.json')); print('$name', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for r in 1 2 3; do
  run def$r || exit 4
  run nt$r FX_GEMM_NTSTORE=1 || exit 4
done
cat /proc/loadavg
