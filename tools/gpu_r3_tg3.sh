# tgemm pipelining fix: numerics tests, per-shape A/B, step benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tg3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tgconv_gpu.py tests/test_tgemm_cpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
NDP_TG_SMALL=1 timeout -k 10 300 python tools/tg_bench.py --iters 30 > $O/tg_bench.jsonl 2> $O/tg_bench.err || { tail -5 $O/tg_bench.err; exit 1; }
cat $O/tg_bench.jsonl
SPECS="b512||--global-batch=512 b64||--global-batch=64 b64small|NDP_TG_SMALL=1|--global-batch=64 b512small|NDP_TG_SMALL=1|--global-batch=512 r50d||--model=resnet50,--reducer=dense r152||--model=resnet152" STEPS=20 bash tools/gpu_r3_envab.sh
