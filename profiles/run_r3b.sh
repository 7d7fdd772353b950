set -o pipefail
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "block_order or golden" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash profiles/run_order_sweep.sh r3b_order "408:408:0 816:816:0 408:136:0 408:408:2 408:408:4 204:204:2 408:64:0" 2>&1 | tee $O/sweep.txt
bash profiles/run_ablate.sh "16 32" --config c4 2>&1 | tee $O/ablate.txt
