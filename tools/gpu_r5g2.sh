# k_nn_tile points-per-lane sweep, then the drop-in A/B against $2 (default: the last commit's build)
set -o pipefail
out=gpurun_out/${1:-r5g2}; mkdir -p $out
for ppl in 2 3 4; do
  TD_NN_PPL=$ppl timeout -k 10 120 python tools/nn_tile_ppl.py > $out/ppl$ppl.json || { echo "ppl $ppl failed"; cat $out/ppl$ppl.json; exit 1; }
  cat $out/ppl$ppl.json
done
bash tools/gpu_dropin_ab.sh ${1:-r5g2}/dab ${2:-ab/libtdstar_0f72452.so}
