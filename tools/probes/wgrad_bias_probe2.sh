set -o pipefail
export TMPDIR=/tmp
for o in ab ba; do
  PROBE_ORDER=$o timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/wgo$o -o k -- python tools/probes/wgrad_bias_probe.py > gpurun_out/wgo$o.log 2>&1 || exit 1
done
