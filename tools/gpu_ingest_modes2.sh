set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/ingm2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ingest.py tests/test_gpu_scan.py > $O/t.log 2>&1 || { echo TESTFAIL; tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
for F in 4096 65536; do for M in gpu host auto; do
  T=${F}_${M}
  timeout -k 10 200 python -u tools/bench_ingest.py --gib 2 --frame $F --scan $M --skip-cpu > $O/b_$T.json 2> $O/b.err || { echo BENCHFAIL; tail -20 $O/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/b_$T.json'));print('$T',d['socket_only_GiBps'],{k:(d[k]['wire_GiBps'],d[k]['slots_gpu_scan_host_walk'],d[k]['ok']) for k in ('socket_ingest','memory_ingest')})"
done; done
