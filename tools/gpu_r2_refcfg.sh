# reference-default configs + DistilBERT kernel profile + PMC counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/rc_$name.json 2> gpurun_out/rc_$name.err || { tail -5 gpurun_out/rc_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/rc_$name.json)"
}
b r152_psgd4 --model resnet152 --steps 20 --warmup 5 &&
b r50_dense --model resnet50 --reducer dense --steps 20 --warmup 5 &&
b r50_psgd4 --model resnet50 --steps 20 --warmup 5 &&
b bert_psgd16 --model distilbert --rank 16 --steps 20 --warmup 5 &&
b bert_psgd8 --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bert_psgd4 --model distilbert --rank 4 --steps 20 --warmup 5 &&
b bert_dense --model distilbert --reducer dense --steps 20 --warmup 5 || exit 1
MARKER=psgd_update_kernel timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_bert8 -o run -- python3 bench.py --model distilbert --rank 8 --steps 12 --warmup 3 > gpurun_out/tr_bert8.out 2>&1 || { tail -5 gpurun_out/tr_bert8.out; exit 1; }
f=$(find gpurun_out/tr_bert8 -name '*kernel_trace.csv' | head -n 1)
python3 tools/prof_summary.py "$f" --steps 10 --marker psgd_update_kernel --top 60 > gpurun_out/tr_bert8.kernels.md && head -30 gpurun_out/tr_bert8.kernels.md
rm -rf gpurun_out/tr_bert8
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"; wc -l gpurun_out/counters_list.txt
