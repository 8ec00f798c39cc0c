# the chain's LDS plan, then the headline A/B against $2 (default: ab/libtdstar_0f72452.so) and the chain parity tests
set -o pipefail
mkdir -p gpurun_out/${1:-r5h}
timeout -k 10 120 python tools/lds_plan.py || exit 1
bash tools/gpu_ab.sh ${1:-r5h}/ab base=${2:-ab/libtdstar_0f72452.so} head=
