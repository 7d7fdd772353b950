# kernel timing from the dispatch packets' own events (hipExtLaunchKernel): cost in the timed
# steps (VAME_BENCH_KTIMING=0 drops timing) and agreement with rocprofv3
set -o pipefail
O=gpurun_out/r3ai; mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-spans > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); r=d['roofline']; print('$name', round(d['ms_per_step'],4), 'quad', round(r['avg_launch_ms'],4), 'ctu', round(r['affine_me_ctu']['avg_launch_ms'],4), 'frac', round(r['frac'],4))"
}
for rep in 1 2 3; do run ext$rep VAME_X=0; run off$rep VAME_BENCH_KTIMING=0; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu-baseline --no-spans --steps 100 --warmup 10 > $O/tr.json 2> $O/tr.err || { tail -20 $O/tr.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/tr.json')); r=d['roofline']; print('traced run: events quad', round(r['avg_launch_ms'],4), 'ctu', round(r['affine_me_ctu']['avg_launch_ms'],4))"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_launch.py -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
