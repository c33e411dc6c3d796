set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 60 tools/mfma_peak && LD_LIBRARY_PATH=fact-clip_amd/factmx/_lib timeout -k 10 120 tools/ubench
