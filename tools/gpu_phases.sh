# phase stamps per action: one chain, then 256 chains (outputs under gpurun_out/$1)
set -o pipefail
out=gpurun_out/${1:-phases}
mkdir -p $out
timeout -k 10 200 python tools/batch_phases.py 1 5000 > $out/c1.json 2>&1 || { tail $out/c1.json; exit 1; }
timeout -k 10 200 python tools/batch_phases.py 256 2000 > $out/c256.json 2>&1 || { tail $out/c256.json; exit 1; }
cat $out/c1.json | head -80
