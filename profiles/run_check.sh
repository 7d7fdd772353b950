# quick GPU check of a change: the GPU test suite (or a -k selection), then
# optional A/B bench lines (profiles/run_bench_env.sh arguments after --ab)
set -o pipefail
O=gpurun_out/check; mkdir -p $O
SEL=${SEL:-}
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread -k "$SEL" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
fi
tail -2 $O/pytest.log
if [ "${1:-}" = "--ab" ]; then
  shift
  bash profiles/run_bench_env.sh "$@" || exit 1
fi
echo check-done
