# BN single-launch column block: fixed 8 (shipped) vs per-shape (NDP_BN_COLW=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bncw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 env NDP_BN_COLW=0 python -u -m pytest tests/test_batchnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for spec in "b512_8|NDP_BN_COLW=8|" "b512_0|NDP_BN_COLW=0|" "b64_8|NDP_BN_COLW=8|--global-batch=64" "b64_0|NDP_BN_COLW=0|--global-batch=64" "r152_8|NDP_BN_COLW=8|--model=resnet152" "r152_0|NDP_BN_COLW=0|--model=resnet152"; do
  label=$(echo "$spec" | cut -d'|' -f1)_$rep
  envs=$(echo "$spec" | cut -d'|' -f2 | tr ',' ' ')
  args=$(echo "$spec" | cut -d'|' -f3 | tr ',' ' ' | sed 's/--\([a-z-]*\)=/--\1 /g')
  env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 10 $args > $O/$label.json 2> $O/$label.err || { echo "$label failed"; tail -5 $O/$label.err; exit 1; }
  echo "$label $(python3 tools/jline.py $O/$label.json)"
done
done
