# frame scan: parity (strict + speculative non-strict) and timing of both modes
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${AB_TAG:-spec}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $O/t.log 2>&1 || { echo TESTFAIL; tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u tools/bench_scan.py > $O/strict.jsonl 2> $O/b.err && timeout -k 10 300 python -u tools/bench_scan.py --non-strict > $O/nonstrict.jsonl 2>> $O/b.err && timeout -k 10 300 python -u tools/bench_scan.py --non-strict --unmasked > $O/nonstrict_unmasked.jsonl 2>> $O/b.err || { echo BENCHFAIL; tail -20 $O/b.err; exit 1; }
cat $O/strict.jsonl $O/nonstrict.jsonl $O/nonstrict_unmasked.jsonl
