set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; exit 1; }
bash tools/profile.sh r01_v6 || { echo "profile failed"; exit 1; }
