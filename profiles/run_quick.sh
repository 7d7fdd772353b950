set -o pipefail
O=gpurun_out/a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 1
python -c "
import json
for c in ('c2','c3'):
    d=json.load(open('$O/%s.json'%c)); print(c, d['ms_per_step'], d['value']/1e6, d['roofline']['frac'], d.get('parity_sample'))
"
