set -o pipefail
cd $GRAFT_REPO_ROOT
export SPECS="b64||--global-batch=64 b64fork|NDP_CONV_FORK=1|--global-batch=64 b512||--global-batch=512 b512fork|NDP_CONV_FORK=1|--global-batch=512 b64ov||--global-batch=64,--overlap=on"
bash tools/gpu_r3_envab.sh && PROFS="b64:--global-batch=64 b512:--global-batch=512" bash tools/gpu_r3_prof.sh
