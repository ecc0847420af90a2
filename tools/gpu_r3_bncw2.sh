# BN column block: fixed 8 vs per-shape min 4 (0) vs per-shape min 8 (1); R18 b512/b256/b64, R152, R50
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bncw2
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "b512|" "b256|--global-batch 256" "b64|--global-batch 64" "r152|--model resnet152" "r50|--model resnet50 --reducer dense"; do
  for m in 8 0 1; do
    tag=${cfg%%|*}; args=${cfg#*|}; label=${tag}_${m}_$rep
    NDP_BN_COLW=$m timeout -k 10 300 python bench.py --steps 40 --warmup 10 $args > $O/$label.json 2> $O/$label.err || { echo "$label failed"; tail -5 $O/$label.err; exit 1; }
    echo "$label $(python3 tools/jline.py $O/$label.json)"
  done
done
done
