# per-kernel durations of the tgemm conv path (kernel trace + stats) on two shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tgprof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 tools/tg_bench.py --shapes ${SHAPES:-r50.l1.pw_in r50.l3.pw_out} --batches 512 --iters 30 > $O/out.log 2>&1 || { tail -20 $O/out.log; exit 1; }
cat $O/out.log | grep shape
f=$(find $O/t -name '*kernel_stats.csv' | head -n 1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:40]:
    print(r['Name'][:120], r['Calls'], r.get('AverageNs'), r.get('Percentage'))
"
