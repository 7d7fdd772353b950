# the round-end records at HEAD: GPU suite, smoke, default bench line
set -o pipefail
O=gpurun_out/final; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 400 $O/bench_default.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || { tail -20 $O/bench_s20.err; exit 1; }
tail -c 300 $O/bench_s20.json
