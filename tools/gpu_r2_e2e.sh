# User-facing path on the GPU: reference-style run_script workloads through the engine
# (hipGraph auto, fused kernels), loss trajectories to JSONL; 2 ranks sharing the GPU via gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
W=network_distributed_pytorch_amd/workloads
timeout -k 10 300 python -u $W/ddp_powersgd_guide_cifar10/run_script.py -rank 0 -cuda 0 -world_size 1 -epochs 3 -steps 60 \
  -model resnet18 -dataset_size 12800 -graph_mode auto -log_file gpurun_out/e2e_psgd_r18.jsonl -log_every 20 > gpurun_out/e2e_psgd_r18.out 2>&1 || { tail -20 gpurun_out/e2e_psgd_r18.out; exit 1; }
tail -4 gpurun_out/e2e_psgd_r18.out
timeout -k 10 300 python -u $W/ddp_guide_cifar10/run_script.py -rank 0 -cuda 0 -world_size 1 -epochs 2 -steps 40 \
  -model resnet50 -dataset_size 6400 -graph_mode auto -log_file gpurun_out/e2e_dense_r50.jsonl -log_every 20 > gpurun_out/e2e_dense_r50.out 2>&1 || { tail -20 gpurun_out/e2e_dense_r50.out; exit 1; }
tail -3 gpurun_out/e2e_dense_r50.out
timeout -k 10 400 python -u $W/ddp_powersgd_distillBERT_IMDb/run_script.py -rank 0 -cuda 0 -world_size 1 -epochs 1 -steps 40 \
  -dataset_size 1280 -graph_mode auto -log_file gpurun_out/e2e_psgd_bert.jsonl -log_every 10 > gpurun_out/e2e_psgd_bert.out 2>&1 || { tail -20 gpurun_out/e2e_psgd_bert.out; exit 1; }
tail -3 gpurun_out/e2e_psgd_bert.out
timeout -k 10 400 python -u $W/ddp_powersgd_guide_cifar10/run_script.py -world_size 2 -spawn -backend gloo -epochs 1 -steps 20 \
  -model resnet18 -dataset_size 6400 -check_replicas 10 -log_file gpurun_out/e2e_psgd_r18_w2.jsonl > gpurun_out/e2e_psgd_r18_w2.out 2>&1 || { tail -20 gpurun_out/e2e_psgd_r18_w2.out; exit 1; }
tail -4 gpurun_out/e2e_psgd_r18_w2.out
