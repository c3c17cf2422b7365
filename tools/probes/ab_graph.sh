# same-box A/B of bench.py's eager step vs the HIP-graph replay (20/5 = the driver's window, and 200/10)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_graph.jsonl
: > $out
for rep in 1 2; do
  for g in off on; do
    timeout -k 10 180 python bench.py --steps 20 --warmup 5 --graph $g > gpurun_out/abg_$g$rep.log 2>&1 || { tail -20 gpurun_out/abg_$g$rep.log; exit 1; }
    grep '^{' gpurun_out/abg_$g$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['step_ms_events']; print(json.dumps({'graph':'$g','steps':d['steps'],'ms':d['ms_per_step'],'first':e['first'],'median':e['median'],'hip_graph':d['config']['hip_graph'],'all':e['all']}))" >> $out
    tail -1 $out | cut -c1-200
  done
done
for g in off on; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 10 --graph $g > gpurun_out/abg_${g}200.log 2>&1 || { tail -20 gpurun_out/abg_${g}200.log; exit 1; }
  grep '^{' gpurun_out/abg_${g}200.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['step_ms_events']; print(json.dumps({'graph':'$g','steps':d['steps'],'ms':d['ms_per_step'],'first':e['first'],'median':e['median'],'hip_graph':d['config']['hip_graph']}))" >> $out
  tail -1 $out
done
