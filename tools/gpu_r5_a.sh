#!/bin/bash
# Round 5, first GPU pass: the new tests (known answers, icosphere enclosure,
# superseded async steps, split arrival growth) verbose, then the whole GPU
# suite, the default bench line and config 4's interior icosphere traces.
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_known_answers.py tests/test_gpu_boundary.py::test_superseded_async_faults_are_counted \
  tests/test_gpu_boundary.py::test_async_traces_equal_blocking_traces tests/test_gpu_parity.py::test_split_arrival_counters_grow \
  > $O/pt_new.log 2>&1; rc=$?
tail -n 30 $O/pt_new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pt_all.log 2>&1; rc2=$?
tail -n 15 $O/pt_all.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
for L in 2 3; do
  timeout -k 10 120 python tools/bench_trace3d.py --interior --level $L --cpu-rows 4 >> $O/trace3d_interior.log 2>&1 || exit 1
done
cat $O/trace3d_interior.log
