# A/B the GEMM microbench between two builds of the library (diagnostic)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=fact-clip_amd/factmx/_lib
for lib in ${LIBS:-libfactmx_prev.so libfactmx.so libfactmx_prev.so libfactmx.so}; do
  echo "== $lib"
  FACTMX_LIB=$PWD/$L/$lib timeout -k 10 120 python tools/gemm_bench.py || exit $?
done
