# round-2 baseline: strong-scaling per-GPU shapes (512/N for N=1,2,4,8), reference-default
# configs, and a kernel profile of the N=8 per-GPU shape (batch 64)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/bl_$name.json 2> gpurun_out/bl_$name.err || { tail -5 gpurun_out/bl_$name.err; return 1; }
  echo "$name $(python3 -c "import json;d=json.load(open('gpurun_out/bl_$name.json'));print(d['value'], d['ms_per_step'], d['config']['hip_graph'])")"
}
b b512 --batch 512 --steps 40 --warmup 10 &&
b b256 --batch 256 --steps 40 --warmup 10 &&
b b128 --batch 128 --steps 40 --warmup 10 &&
b b64 --batch 64 --steps 40 --warmup 10 &&
b dense_b64 --batch 64 --reducer dense --steps 40 --warmup 10 &&
b r152_r4 --model resnet152 --steps 10 --warmup 4 &&
b r50_dense --model resnet50 --reducer dense --batch 256 --steps 10 --warmup 4 &&
b bert_r16 --model distilbert --rank 16 --steps 10 --warmup 4 &&
b bert_r8 --model distilbert --rank 8 --steps 10 --warmup 4 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_b64 -o run -- python3 bench.py --batch 64 --steps 25 --warmup 5 > gpurun_out/prof_b64.out 2>&1 &&
f=$(find gpurun_out/prof_b64 -name '*kernel_trace.csv' | head -n 1) && python3 tools/prof_summary.py "$f" --steps 20 --top 80 > gpurun_out/prof_b64.md && head -12 gpurun_out/prof_b64.md
rc=$?; rm -rf gpurun_out/prof_b64; exit $rc
