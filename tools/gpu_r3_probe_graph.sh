# does one captured hipGraph run independent branches concurrently? (tools/probe_graph_branches.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3graph
mkdir -p $O
timeout -k 10 120 python tools/probe_graph_branches.py 20 20 > $O/default.log 2>&1 && cat $O/default.log || exit 1
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 120 python tools/probe_graph_branches.py 20 20 > $O/q4.log 2>&1 && cat $O/q4.log || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python tools/probe_graph_branches.py 20 20 > $O/nopc.log 2>&1 && cat $O/nopc.log || exit 1
