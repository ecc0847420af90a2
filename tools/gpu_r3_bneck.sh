# bottleneck blocks with residual-gradient / slab links: tests + ResNet-50 / 152 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bneck
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tgconv_gpu.py tests/test_models.py tests/test_conv_gemm.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for spec in "r152|--model resnet152" "r50d|--model resnet50 --reducer dense" "r50p|--model resnet50"; do
  label=${spec%%|*}_$rep; args=${spec#*|}
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > $O/$label.json 2> $O/$label.err || { echo "$label failed"; tail -5 $O/$label.err; exit 1; }
  echo "$label $(python3 tools/jline.py $O/$label.json)"
done
done
