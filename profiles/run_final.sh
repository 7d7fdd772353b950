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
# the other BASELINE configs' lines (c3 / c4 / c5 at N = 1), when asked: bash profiles/run_final.sh all
if [ "${1:-}" = all ]; then
  for c in c3 c4 c5; do
    timeout -k 10 400 python bench.py --config $c --fs-frames 0 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('$O/bench_$c.json') if l.startswith('{')][-1]); r=d['roofline']
print('$c', round(d['ms_per_step'], 3), round(d['value'] / 1e6, 1), 'valu', r['frac'], 'hbm_exec', r['hbm_executed_frac'], d.get('parity_sample'))"
  done
fi
echo final-done
