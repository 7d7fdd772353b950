set -o pipefail
O=gpurun_out/r3a; mkdir -p $O
df -h /tmp . > $O/df.txt 2>&1; free -g >> $O/df.txt; nproc >> $O/df.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_bench_launch.py tests/test_distrun.py tests/test_shard.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash profiles/run_order_sweep.sh r3a_order "408:1 408:0 272:1 136:1 204:1" 2>&1 | tee $O/sweep.txt
