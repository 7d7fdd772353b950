set -o pipefail
O=gpurun_out/r3r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for c in "--config c2" "--config c3" "--config c4" "--config c5 --gpus 8 --rank-only 7"; do
  for j in 0 1; do
    VAME_JOIN_EACH=$j timeout -k 10 300 python3 $R/bench.py $c --no-cpu-baseline --no-spans > $R/$O/b.json 2> $R/$O/b.err || { tail -5 $R/$O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$R/$O/b.json')); print('join_each=$j', '$c', round(d['ms_per_step'],3), 'quad', round(d['roofline']['avg_launch_ms'],3), 'ctu', round(d['roofline']['affine_me_ctu']['avg_launch_ms'],3), 'frac', round(d['roofline']['frac'],4))"
  done
done
done
