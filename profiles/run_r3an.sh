# quick round-end check of the bench timing change: default and 20-step lines, smoke, bench launch tests
set -o pipefail
O=gpurun_out/r3an; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || { tail -20 $O/bench_s20.err; exit 1; }
python3 -c "
import json
for f in ('bench_default', 'bench_s20'):
    d = json.load(open('$O/%s.json' % f)); r = d['roofline']
    print(f, round(d['ms_per_step'], 4), round(r['frac'], 4), round(r['avg_launch_ms'], 4), r['affine_me_ctu']['timed_on'], round(r['affine_me_ctu']['avg_launch_ms'], 4), d['parity_sample'])
"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_bench_launch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
