#!/bin/bash
# netc_gpu_unmask_validate with and without the in-pass verdicts (NETC_VAL_INPASS=0: a knob of the
# measured build, removed since -- DESIGN §16.6), config 2 and
# 4 shapes, three interleaved rounds, then a kernel trace of each (through gpurun, repo root)
set -o pipefail
R=$PWD
D=$R/gpurun_out/${TAG:-r06_inpass}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_utf8.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for r in 1 2 3; do for v in 1 0; do
  NETC_VAL_INPASS=$v timeout -k 10 300 python -u tools/bench_validate.py ${ARGS:---steps 50} > $D/v${v}_r$r.json 2> $D/v${v}_r$r.err || { tail -5 $D/v${v}_r$r.err; exit 1; }
  echo "inpass=$v r=$r $(cut -c1-400 $D/v${v}_r$r.json | tr '\n' ' ')"
done; done
export TMPDIR=/tmp
for v in 1 0; do
  (cd /tmp && NETC_VAL_INPASS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace_v$v -o run -- python3 $R/tools/bench_validate.py ${ARGS:---steps 50} > $D/trace_v$v.log 2>&1) || { echo TRACEFAIL; exit 1; }
done
echo done
