set -o pipefail
O=gpurun_out/r3f; mkdir -p $O gpurun_out/prof_c5r7
VAME_LIB=vvc-affine-gpu_amd/lib/libvame_count.so timeout -k 10 300 python3 profiles/count_preds.py --config c5 --gpus 8 --rank-only 7 > gpurun_out/prof_c5r7/count.json 2> $O/count_c5r7.err || { tail $O/count_c5r7.err; exit 1; }
cat gpurun_out/prof_c5r7/count.json
timeout -k 10 300 python3 bench.py --config c5 --gpus 8 --rank-only 7 > gpurun_out/prof_c5r7/bench.json 2> $O/bench_c5r7.err || exit 1
VAME_LIB=vvc-affine-gpu_amd/lib/libvame_phase.so timeout -k 10 300 python3 profiles/phase_profile.py --config c4 --steps 1 > $O/phase_c4.txt 2>&1 || exit 1
cat $O/phase_c4.txt
VAME_LIB=vvc-affine-gpu_amd/lib/libvame_phase.so timeout -k 10 300 python3 profiles/phase_profile.py --config c2 --steps 5 > $O/phase_c2.txt 2>&1 || exit 1
cat $O/phase_c2.txt
