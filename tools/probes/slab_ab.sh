set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_head_gpu.py -k "slab_reduce or hidden_group or fused_optimizer or matches_unfused" > gpurun_out/slab_tests.log 2>&1 || { tail -30 gpurun_out/slab_tests.log; exit 1; }
tail -2 gpurun_out/slab_tests.log
: > gpurun_out/slab_ab.jsonl
for rep in 1 2; do for c in 64 32; do
  SDML_KNOBS=U8_SLAB_COLS=$c timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/slab_$c.log 2>&1 || { tail gpurun_out/slab_$c.log; exit 1; }
  grep '^{' gpurun_out/slab_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['step_ms_events']; print(json.dumps({'cols':$c,'ms':d['ms_per_step'],'median':e['median'],'min':e['min']}))" | tee -a gpurun_out/slab_ab.jsonl
done; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in 64 32; do
  SDML_KNOBS=U8_SLAB_COLS=$c timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_slab$c -o run -- python bench.py --steps 50 --warmup 5 > gpurun_out/slab_prof_$c.log 2>&1 || { tail gpurun_out/slab_prof_$c.log; exit 1; }
done
