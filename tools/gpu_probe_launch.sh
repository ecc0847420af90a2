set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
r() { timeout -k 10 120 python tools/probe_launch.py "$@" 2>&1 | grep '^{' ; }
r --global-batch 64 &&
r --global-batch 64 --no-overlap &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 r --global-batch 64 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 r --global-batch 64 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 r --global-batch 64 --no-overlap &&
r --global-batch 512 &&
r --global-batch 512 --no-overlap
