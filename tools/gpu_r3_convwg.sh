# direct conv [m][kk] A image (b128 fragment reads): tests, steps, kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/convwg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_direct.py tests/test_conv_gemm.py tests/test_graph_gpu.py tests/test_gradarena_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for spec in "b512|" "b64|--global-batch 64" "b128|--global-batch 128" "r152|--model resnet152"; do
  label=${spec%%|*}_$rep; args=${spec#*|}
  timeout -k 10 300 python bench.py --steps 40 --warmup 10 $args > $O/$label.json 2> $O/$label.err || { echo "$label failed"; tail -5 $O/$label.err; exit 1; }
  echo "$label $(python3 tools/jline.py $O/$label.json)"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --no-supervise --steps 25 --warmup 5 > $O/prof.out 2>&1 || { echo "prof failed"; tail -5 $O/prof.out; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1)
python3 tools/prof_summary.py "$f" --steps 20 --marker 'conv_fwd_kernel<7, 7' --top 60 > $O/kernels_b512.md && grep -E "wall|conv_fwd|conv_wgrad" $O/kernels_b512.md
rm -rf $O/prof
