# A/B of environment variants on one box: alternating rounds of the short bench (no CPU baseline / extra modes),
# ms per step + the rooflines of interest per run.  usage: VARIANTS="A=;B=FX_X=1" ROUNDS=3 bash tools/r06_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06ab; mkdir -p $O
IFS=';' read -ra VS <<< "${VARIANTS:-base=}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "${VS[@]}"; do
    name=${v%%=*}; envs=${v#*=}
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead ${BENCH_ARGS:-} > $O/$name.$r.json 2> $O/$name.$r.err || { tail -5 $O/$name.$r.err; exit 3; }
    python - "$O/$name.$r.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ra = d.get("roofline_attention") or {}
f = d.get("roofline_fused_layer") or {}
xs = " ".join(f"{k}={1e3 * v['kernel_ms_per_call']:.1f}us" for k, v in ra.items() if v)
print(f"{sys.argv[2]:12s} {d['ms_per_step']:7.3f} ms  frl {f.get('frac')}  {xs}", flush=True)
PY
  done
done
