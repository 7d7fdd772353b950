set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3h_pytest.log 2>&1 || { tail -30 gpurun_out/r3h_pytest.log; exit 1; }
tail -1 gpurun_out/r3h_pytest.log
bash profiles/run_ab.sh r3h "libvame libvame_narrow" "--config c2;--config c3;--config c4;--config c5 --gpus 8 --rank-only 7"
