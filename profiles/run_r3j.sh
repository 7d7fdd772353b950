set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3j_pytest.log 2>&1 || { tail -30 gpurun_out/r3j_pytest.log; exit 1; }
tail -1 gpurun_out/r3j_pytest.log
bash profiles/run_ab.sh r3j "libvame libvame_nomix" "--config c2;--config c3;--config c4;--config c5 --gpus 8 --rank-only 7"
