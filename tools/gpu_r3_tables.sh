# final kernel tables at HEAD: ResNet-18 r=4 batch 64 (N = 8 shape), ResNet-152 r=4, ResNet-50 dense
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tables
mkdir -p $O
export TMPDIR=/tmp
for cfg in "b64:--global-batch 64:20" "r152:--model resnet152:10" "r50d:--model resnet50 --reducer dense:10"; do
  tag=$(echo "$cfg" | cut -d: -f1); args=$(echo "$cfg" | cut -d: -f2); n=$(echo "$cfg" | cut -d: -f3)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$tag -o run -- python3 bench.py --no-supervise --steps $((n + 5)) --warmup 5 $args > $O/prof_$tag.out 2>&1 || { echo "prof $tag failed"; tail -5 $O/prof_$tag.out; exit 1; }
  f=$(find $O/prof_$tag -name '*kernel_trace.csv' | head -n 1)
  python3 tools/prof_summary.py "$f" --steps $n --marker 'conv_fwd_kernel<7, 7' --top 80 > $O/kernels_$tag.md && head -14 $O/kernels_$tag.md
  rm -rf $O/prof_$tag
done
