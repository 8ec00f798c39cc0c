set -o pipefail
mkdir -p gpurun_out/ph
timeout -k 10 120 python tools/batch_phases.py 1 5000 > gpurun_out/ph/b1.json || exit 1
TD_LIB_PATH=$PWD/ab/libtdstar_base.so timeout -k 10 120 python tools/shadow_phases.py 1500 > gpurun_out/ph/shadow.json || exit 1
bash tools/gpu_dropin_ab.sh dab1 || exit 1
timeout -k 10 120 python tools/batch_phases.py 256 2000 > gpurun_out/ph/b256.json
