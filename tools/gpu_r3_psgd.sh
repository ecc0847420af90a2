# PowerSGD P item width (NDP_PSGD_PKW 256/512/1024) and Q pass depth (NDP_PSGD_QDEEP): tests + steps + kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/psgd
mkdir -p $O
export TMPDIR=/tmp
for arm in "k256|NDP_PSGD_PKW=256,NDP_PSGD_QDEEP=1" "k512|NDP_PSGD_PKW=512"; do
  label=${arm%%|*}; envs=$(echo ${arm#*|} | tr ',' ' ')
  timeout -k 10 300 env $envs python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$label.log 2>&1
  rc=$?; echo "pytest $label rc=$rc"; tail -1 $O/pytest_$label.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
for arm in "k1024|NDP_PSGD_PKW=1024" "k512|NDP_PSGD_PKW=512" "k256|NDP_PSGD_PKW=256" "qdeep|NDP_PSGD_QDEEP=1"; do
  for cfg in "b512|" "b64|--global-batch 64"; do
    label=${arm%%|*}; envs=$(echo ${arm#*|} | tr ',' ' '); tag=${cfg%%|*}; args=${cfg#*|}
    env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 10 $args > $O/${tag}_${label}_$rep.json 2> $O/${tag}_${label}_$rep.err || { echo "$label $tag failed"; tail -5 $O/${tag}_${label}_$rep.err; exit 1; }
    echo "${tag}_${label}_$rep $(python3 tools/jline.py $O/${tag}_${label}_$rep.json)"
  done
done
done
for arm in "k1024|NDP_PSGD_PKW=1024" "k256q|NDP_PSGD_PKW=256,NDP_PSGD_QDEEP=1"; do
  label=${arm%%|*}; envs=$(echo ${arm#*|} | tr ',' ' ')
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$label -o run -- python3 bench.py --no-supervise --steps 25 --warmup 5 > $O/prof_$label.out 2>&1 || { echo "prof failed"; tail -5 $O/prof_$label.out; exit 1; }
  f=$(find $O/prof_$label -name '*kernel_trace.csv' | head -n 1)
  python3 tools/prof_summary.py "$f" --steps 20 --marker 'conv_fwd_kernel<7, 7' --top 80 > $O/kernels_$label.md; echo "== $label"; grep -E "wall|psgd|seg_red|orth|rank1" $O/kernels_$label.md
  rm -rf $O/prof_$label
done
