set -o pipefail
bash profiles/run_ab.sh r3q "libvame libvame_ablate1024 libvame_dup128 libvame_dup192" "--config c3;--config c4;--config c5 --gpus 8 --rank-only 7"
