# persistent 128-class kernel (VAME_CTU_PERSIST=P workgroups): parity with it on, then c2 / c3 timing per P
set -o pipefail
O=gpurun_out/r3ag; mkdir -p $O
VAME_CTU_PERSIST=64 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  local name=$1 cfg=$2; shift 2
  env "$@" VAME_BENCH_KTIMING=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-spans --config $cfg > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['ms_per_step'],4), d['gather']['check']['byte_identical'])"
}
for rep in 1 2; do
  for P in 0 32 48 64 96 128 256; do run c2_p${P}_$rep c2 VAME_CTU_PERSIST=$P; done
done
for P in 0 48 64 96; do run c3_p$P c3 VAME_CTU_PERSIST=$P; done
