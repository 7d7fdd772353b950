set -o pipefail
bash profiles/run_ab.sh r3i "libvame libvame_gb5 libvame_gb9" "--config c2;--config c4;--config c5 --gpus 8 --rank-only 7"
