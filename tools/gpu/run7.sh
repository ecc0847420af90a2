# BN pair + attention accumulator-chain A/B (round 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r7; mkdir -p $O
export TMPDIR=/tmp
: pytest done in the previous call

timeout -k 10 200 python -u tools/diag/attn_chains.py > $O/attn_chains.jsonl 2> $O/attn_chains.err || { tail -5 $O/attn_chains.err; exit 1; }
cat $O/attn_chains.jsonl
tools/gpu/bench.sh $O "b64|--global-batch 64" "b64nopair|NDP_FUSION_OFF=bn_pair --global-batch 64" "b512|" "b512nopair|NDP_FUSION_OFF=bn_pair" || exit 1
