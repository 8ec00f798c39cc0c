# round-2 v4 evidence: default bench line, rocprofv3 passes (tools/profile.sh)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/v4_bench.log 2>&1
bash tools/profile.sh ${TAG:-r02_v5} > gpurun_out/v4_prof.log 2>&1 && bash tools/profile_aux.sh ${TAG:-r02_v5} >> gpurun_out/v4_prof.log 2>&1
