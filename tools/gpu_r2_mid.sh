#!/bin/bash
# mid-round check: full GPU suite, smoke, headline bench, kernel profile of the headline step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/summarize_profile.py stats $(find $O/prof -name "*kernel_stats.csv" | head -1) 25 > $O/kstats.txt; head -16 $O/kstats.txt
