set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pd
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pd/trace -o run -- python3 tools/dropin_only.py > gpurun_out/pd/trace.log 2>&1 || { echo prof failed; tail gpurun_out/pd/trace.log; exit 1; }
tail -2 gpurun_out/pd/trace.log
find gpurun_out/pd/trace -name "*kernel_stats.csv" | head -1 | xargs head -20
