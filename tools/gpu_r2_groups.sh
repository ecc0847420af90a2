set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in 1 2 3; do timeout -k 10 200 python bench.py --global-batch 64 --steps 50 --warmup 10 --psgd-groups $g > gpurun_out/g$g.json 2>/dev/null && echo "g$g $(python3 tools/jline.py gpurun_out/g$g.json)" || exit 1; done
timeout -k 10 200 python bench.py --global-batch 512 --steps 50 --warmup 10 --psgd-groups 1 > gpurun_out/g1_512.json 2>/dev/null && echo "g1_512 $(python3 tools/jline.py gpurun_out/g1_512.json)" || exit 1
NDP_SIDE_PRIORITY=normal timeout -k 10 200 python bench.py --global-batch 64 --steps 50 --warmup 10 > gpurun_out/gnorm.json 2>/dev/null && echo "gnorm $(python3 tools/jline.py gpurun_out/gnorm.json)" || exit 1
NDP_SIDE_PRIORITY=normal bash tools/gpu_r2_prof.sh b64norm "--global-batch 64"
