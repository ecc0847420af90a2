# A/B env knobs / bench args on the 1-GPU bench.
# SPECS: space-separated label|ENV=v,ENV=v|bench-args (args: ',' -> ' ', '=' kept), e.g.
#   SPECS="base||--global-batch=64 fork|NDP_CONV_FORK=1|--global-batch=64" bash tools/gpu_r3_envab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/envab
mkdir -p $O
export TMPDIR=/tmp
STEPS=${STEPS:-40}
for spec in $SPECS; do
  label=$(echo "$spec" | cut -d'|' -f1)
  envs=$(echo "$spec" | cut -d'|' -f2 | tr ',' ' ')
  args=$(echo "$spec" | cut -d'|' -f3 | tr ',' ' ' | sed 's/--\([a-z-]*\)=/--\1 /g')
  env $envs timeout -k 10 240 python bench.py --steps $STEPS --warmup 10 $args > $O/$label.json 2> $O/$label.err || { echo "$label failed"; tail -5 $O/$label.err; exit 1; }
  echo "$label [$envs] [$args] $(python3 tools/jline.py $O/$label.json)"
done
