# round 6: the skew probe and skew test suite on the head's skew build, then same-box A/Bs
set -o pipefail
mkdir -p gpurun_out/r6h
TD_LIB_PATH=$PWD/ab/libtdstar_skew_head.so timeout -k 5 200 python -u tools/skew_probe.py > gpurun_out/r6h/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -17 gpurun_out/r6h/probe.log
[ $rc -ne 0 ] && exit 1
bash tools/gpu_skew.sh r6h skew_head=ab/libtdstar_skew_head.so
grep -E "passed|failed" gpurun_out/r6h/skew_head.log | tail -2
bash tools/gpu_r6.sh r6h/ab - base=ab/libtdstar_base.so snap=ab/libtdstar_snap.so head= || exit 1
bash tools/gpu_eval_ab.sh r6h/eab ab/libtdstar_noxcd.so
