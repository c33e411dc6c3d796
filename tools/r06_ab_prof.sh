# A/B of library builds by kernel trace: per variant, rocprofv3 --kernel-trace of a short bench, then the
# step map over the last 8 step periods (busy union, main-stream kernel time, idle) and the top kernels.
# usage: VARIANTS="new=;old=FACTMX_LIB=/path/libfactmx.so" bash tools/r06_ab_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06abp; rm -rf $O; mkdir -p $O
IFS=';' read -ra VS <<< "${VARIANTS:-base=}"
for v in "${VS[@]}"; do
  name=${v%%=*}; envs=${v#*=}
  for e in $envs; do export "$e"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/$name.json 2> $O/$name.log || { tail -20 $O/$name.log; exit 4; }
  for e in $envs; do unset "${e%%=*}"; done
  echo "== $name"
  python tools/step_map.py $(find $O/$name -name "*kernel_trace.csv") 8 | head -20
  python tools/kstats.py $(find $O/$name -name "*kernel_stats.csv") 14 14 | cut -c1-120
done
