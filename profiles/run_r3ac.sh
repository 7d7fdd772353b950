# bench launch forms (self-launched, torchrun) and the default line with its native-library record
set -o pipefail
O=gpurun_out/r3ac; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['native'])"
