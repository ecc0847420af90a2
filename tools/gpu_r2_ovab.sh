# overlap A/B at N = 1 (side-stream group pipelines vs serial), batch 64 and 512
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 64 512; do
  for cfg in "serial:--overlap off" "ov3:--overlap on --psgd-groups 3" "ov2:--overlap on --psgd-groups 2" "ov4:--overlap on --psgd-groups 4"; do
    n=${cfg%%:*}; a=${cfg#*:}
    timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 $a > gpurun_out/oa_${n}_$b.json 2> gpurun_out/oa_${n}_$b.err || { tail -3 gpurun_out/oa_${n}_$b.err; exit 1; }
    echo "$n b$b $(python3 tools/jline.py gpurun_out/oa_${n}_$b.json)"
  done
done
