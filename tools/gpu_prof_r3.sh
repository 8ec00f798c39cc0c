# round-3 profile pass: chain kernels (single, many, stress) + aux.  usage: tools/gpu_prof_r3.sh TAG
set -o pipefail
TAG=${1:-r03_v0}
bash tools/profile.sh $TAG && bash tools/profile_aux.sh $TAG && \
for r in single many packed stress aux; do python3 profiles/summarize.py gpurun_out/$TAG/$r > gpurun_out/$TAG/$r.md || exit 1; done && \
python3 profiles/make_traffic.py gpurun_out/$TAG $TAG > gpurun_out/$TAG/traffic.log
