# tgemm register-prefetch depth A/B (NDP_TG_DEPTH), then the full GPU suite + benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/depth
mkdir -p $O
export TMPDIR=/tmp
for D in 2 3 4; do
  NDP_TG_DEPTH=$D NDP_TG_SMALL=1 timeout -k 10 240 python tools/tg_bench.py --iters 30 --batches 64 512 \
    --shapes r18.l3.conv r18.l4.conv r50.l1.pw_in r50.l2.pw_in r50.l3.pw_in r50.l3.pw_out > $O/tg_d$D.jsonl 2> $O/tg_d$D.err || { echo "tg depth $D failed"; tail -5 $O/tg_d$D.err; exit 1; }
  echo "depth $D"; cat $O/tg_d$D.jsonl
done
for D in 2 3 4; do
  NDP_TG_DEPTH=$D timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model resnet152 > $O/r152_d$D.json 2> $O/r152_d$D.err || { echo "r152 depth $D failed"; tail -5 $O/r152_d$D.err; exit 1; }
  echo "r152 depth $D $(python3 tools/jline.py $O/r152_d$D.json)"
done
bash tools/gpu_r3_full.sh
