#!/bin/bash
# One parametrized GPU-box runner (replaces the one-off lease scripts of rounds 1-2). Each call runs
# ONE step under its own time limit and returns its exit status, so steps chain with && inside one
# gpurun call and a failed/timed-out step ends the chain.
#
#   tools/gpu.sh test  <timeout_s> <pytest args...>         -> gpurun_out/pytest.log
#   tools/gpu.sh run   <name> <timeout_s> <cmd...>          -> gpurun_out/<name>.log
#   tools/gpu.sh stats <name> <timeout_s> <cmd...>          rocprofv3 --kernel-trace --stats
#                                                           -> gpurun_out/<name>/kernel_stats.txt
#   tools/gpu.sh pmc   <name> <counters> <cmd...>           one PMC pass (SIGKILL after 90 s)
#                                                           -> gpurun_out/<name>/pmc.txt
#   tools/gpu.sh configs <timeout_s> [config...]            tools/bench_configs.py per config (default: all
#                                                           five) -> gpurun_out/configs.jsonl
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
task=$1; shift
case "$task" in
  test)
    t=$1; shift
    timeout -k 10 "$t" python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/pytest.log 2>&1
    rc=$?
    grep -E "passed|failed|error" gpurun_out/pytest.log | tail -3
    [ $rc -eq 0 ] || tail -60 gpurun_out/pytest.log
    exit $rc ;;
  run)
    name=$1; t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    rc=$?
    grep -v amdgpu.ids "gpurun_out/$name.log" | tail -5 | cut -c1-400
    exit $rc ;;
  stats)
    name=$1; t=$2; shift 2
    d=gpurun_out/$name
    mkdir -p "$d"
    timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv -d "$d/raw" -o k -- "$@" \
      > "$d/run.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -20 "$d/run.log"; exit $rc; fi
    f=$(find "$d/raw" -name "*kernel_stats.csv" | head -1)
    # per-step divisor: the command's --steps + --warmup (STEPS=<n> overrides; 30 if neither is given)
    n=0; prev=""
    for x in "$@"; do
      case "$prev" in --steps|--warmup) n=$((n + x)) ;; esac
      prev=$x
    done
    [ "$n" -gt 0 ] || n=30
    python tools/summarize_profile.py stats "$f" "${STEPS:-$n}" > "$d/kernel_stats.txt"
    grep -v amdgpu.ids "$d/run.log" | grep "^{" | cut -c1-300
    head -14 "$d/kernel_stats.txt" | cut -c1-150 ;;
  pmc)
    name=$1; ctrs=$2; shift 2
    d=gpurun_out/$name
    mkdir -p "$d"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$d/raw" -o p -- "$@" \
      > "$d/run.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -20 "$d/run.log"; exit $rc; fi
    python tools/summarize_profile.py pmc $(find "$d/raw" -name "*counter_collection.csv") > "$d/pmc.txt"
    head -30 "$d/pmc.txt" | cut -c1-200 ;;
  configs)
    t=$1; shift
    [ $# -gt 0 ] || set -- mlp ref_cnn mlp4x1024 resnet18 gpt2
    : > gpurun_out/configs.jsonl
    for c in "$@"; do
      timeout -k 10 "$t" python tools/bench_configs.py --config "$c" > "gpurun_out/cfg_$c.log" 2>&1 || {
        tail -20 "gpurun_out/cfg_$c.log"; exit 1; }
      grep '^{' "gpurun_out/cfg_$c.log" | tail -1 | tee -a gpurun_out/configs.jsonl | cut -c1-300
    done ;;
  *)
    echo "usage: tools/gpu.sh {test|run|stats|pmc|configs} ..." >&2; exit 2 ;;
esac
