# rocprofv3 kernel traces (in-process bench: --no-supervise) summarised per step.
# PROFS: space-separated list of name:bench-args (default: b512, b64, resnet152 r4, resnet50 dense)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3prof
mkdir -p $O
export TMPDIR=/tmp
PROFS=${PROFS:-"b512:--global-batch=512 b64:--global-batch=64 r152:--model=resnet152 r50d:--model=resnet50,--reducer=dense"}
for spec in $PROFS; do
  name=${spec%%:*}
  args=$(echo ${spec#*:} | tr ',' ' ' | tr '=' ' ')
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_$name -o run -- python3 bench.py --no-supervise --steps 25 --warmup 5 $args > $O/$name.out 2>&1 || { echo "prof $name failed"; tail -5 $O/$name.out; exit 1; }
  f=$(find $O/t_$name -name '*kernel_trace.csv' | head -n 1)
  marker=${MARKER:-conv_fwd_kernel<7, 7}
  python3 tools/prof_summary.py "$f" --steps 20 --top 70 --marker "$marker" > $O/$name.md && head -4 $O/$name.md
  rm -rf $O/t_$name
done
