set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "200 5 20 cc" "200 5 20 sc" "50 20 5 cc"; do
  set -- $cfg
  name=q_$1_$2_$3_$4
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$name -o run -- python3 tools/probe_queue.py $cfg > gpurun_out/$name.out 2>&1 || { tail -5 gpurun_out/$name.out; exit 1; }
  f=$(find gpurun_out/$name -name '*kernel_trace.csv' | head -n 1)
  echo "== $cfg $(grep flag gpurun_out/$name.out)"
  python3 tools/queue_dump.py "$f" $((2 * ($1 + 6))) | tail -24
  rm -rf gpurun_out/$name
done
