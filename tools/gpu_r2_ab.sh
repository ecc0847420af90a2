# A/B: overlap vs serial (no side stream) at batch 512 and 64; kernel profile of serial b64
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 512 64; do
  for mode in ov serial; do
    extra=""; [ $mode = serial ] && extra="--no-overlap"
    timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 $extra > gpurun_out/ab_${mode}_$b.json 2> gpurun_out/ab_${mode}_$b.err || { tail -5 gpurun_out/ab_${mode}_$b.err; exit 1; }
    echo "$mode b$b $(python3 tools/jline.py gpurun_out/ab_${mode}_$b.json)"
  done
done
bash tools/gpu_r2_prof.sh serial64 "--global-batch 64 --no-overlap" serial512 "--no-overlap"
