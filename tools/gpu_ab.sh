# A/B a tuning env var on the headline bench: gpu_ab.sh VAR "v1 v2 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
var=$1; shift
for v in $1; do
  env $var=$v timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  echo "$var=$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(d['value'], d['ms_per_step'])")"
done
