# C4 (BASELINE configs[3]): 3840x2160, 30 frames, 2+3 CP at QP 22 / 27 / 32 / 37, one line each
set -o pipefail
O=gpurun_out/c4sweep; mkdir -p $O
for q in 22 27 32 37; do
  timeout -k 10 300 python bench.py --config c4 --fs-frames 0 --qp $q > $O/c4_qp$q.json 2> $O/c4_qp$q.err || { tail -20 $O/c4_qp$q.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/c4_qp$q.json') if l.startswith('{')][-1])
print('qp$q', round(d['ms_per_step'],2), round(d['value']/1e6,1), round(d['roofline']['frac'],3), d.get('parity_sample'), d['cpu_baseline']['value'])"
done
