set -o pipefail
O=gpurun_out/g1; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_parity.py -k "anyorder or ordered_by_event or live_reference" > $O/pytest_a.log 2>&1 || { tail -30 $O/pytest_a.log; exit 1; }
tail -3 $O/pytest_a.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_bench_launch.py -m gpu > $O/pytest_b.log 2>&1 || { tail -30 $O/pytest_b.log; exit 1; }
tail -3 $O/pytest_b.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
