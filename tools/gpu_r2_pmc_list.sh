set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"; wc -l gpurun_out/counters_list.txt
grep -oE "\b(SQ|TCC|TCP|TA|TD|GRBM)_[A-Z0-9_]+\b|\bFETCH_SIZE\b|\bWRITE_SIZE\b|\bMfmaUtil\b|\bVALUBusy\b" gpurun_out/counters_list.txt | sort -u > gpurun_out/counters_names.txt; wc -l gpurun_out/counters_names.txt
