# link-throttled bandwidth curves (emulated on 1 GPU), BASELINE config 5 + ResNet-18 r=4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
J=gpurun_out/link_curves.jsonl
rm -f $J
timeout -k 10 900 python tools/bandwidth_sweep.py --mode emulate --gpus 8 --model distilbert --rank 4 --steps 8 --warmup 3 --reducers ${REDUCERS:-powersgd,dense} --jsonl $J > gpurun_out/lc_bert8.md 2> gpurun_out/lc_bert8.err || { tail -5 gpurun_out/lc_bert8.err; exit 1; }
cat gpurun_out/lc_bert8.md
for n in 2 4 8; do
  timeout -k 10 600 python tools/bandwidth_sweep.py --mode emulate --gpus $n --model resnet18 --rank 4 --steps 15 --warmup 5 --reducers ${REDUCERS:-powersgd,dense} --jsonl $J > gpurun_out/lc_r18_$n.md 2> gpurun_out/lc_r18_$n.err || { tail -5 gpurun_out/lc_r18_$n.err; exit 1; }
  cat gpurun_out/lc_r18_$n.md
done
