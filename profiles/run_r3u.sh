# per-batch frame uploads (CLI and distrun): GPU tests of both, then C3/C4 and C5 end to end
set -o pipefail
O=gpurun_out/r3u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cli_gpu.py tests/test_distrun.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/run_e2e.sh r3u_e2e > $O/e2e.txt 2>&1 || { tail -20 $O/e2e.txt; exit 1; }
cat $O/e2e.txt
bash profiles/run_e2e_c5.sh r3u_e2e240 240 > $O/e2e240.txt 2>&1 || { tail -20 $O/e2e240.txt; exit 1; }
cat $O/e2e240.txt
