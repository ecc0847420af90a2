cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/iso; mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python -u -m pytest "$@" -q -m gpu --timeout 200 --timeout-method thread > $O/$name.log 2>&1; echo "$name rc=$? $(tail -1 $O/$name.log)"; grep FAILED $O/$name.log | head -4; }
export NDP_CONV_DGRAD2=1
run BG2 tests/test_bench_gpu.py tests/test_graph_gpu.py
run EARLY2 tests/test_attention.py tests/test_batchnorm_gpu.py tests/test_conv_direct.py tests/test_conv_gemm.py tests/test_distilbert_fusions_gpu.py tests/test_embedding_gpu.py tests/test_fuzz_gpu.py tests/test_gemm_tuning_gpu.py tests/test_graph_gpu.py
ls -la ~/.config/miopen ~/.cache/miopen 2>/dev/null | head -5
