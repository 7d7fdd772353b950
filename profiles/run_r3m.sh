set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3m_pytest.log 2>&1 || { tail -30 gpurun_out/r3m_pytest.log; exit 1; }
tail -1 gpurun_out/r3m_pytest.log
bash profiles/run_ab.sh r3m "libvame libvame_x1" "--config c2;--config c4;--config c5 --gpus 8 --rank-only 7"
