set -o pipefail
bash profiles/run_ab.sh r3k "libvame libvame_pipe libvame_ablate512" "--config c3;--config c4;--config c5 --gpus 8 --rank-only 7"
