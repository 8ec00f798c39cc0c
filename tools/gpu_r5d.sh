# grid-query latency (tools/query_lat.py), then the headline A/B against ab/libtdstar_base.so and the chain parity tests
set -o pipefail
mkdir -p gpurun_out/${1:-r5d}
timeout -k 10 300 python -u tools/query_lat.py > gpurun_out/${1:-r5d}/ql.json 2> gpurun_out/${1:-r5d}/ql.err || { cat gpurun_out/${1:-r5d}/ql.err; exit 1; }
cat gpurun_out/${1:-r5d}/ql.json
bash tools/gpu_ab.sh ${1:-r5d}/ab base=ab/libtdstar_base.so head=
