set -o pipefail
O=gpurun_out/r3d; mkdir -p $O
for c in c2 c3 c4; do
  bash profiles/run_profile.sh $c $c 2>&1 | tail -3 | tee $O/prof_$c.txt || exit 1
done
VAME_LIB=vvc-affine-gpu_amd/lib/libvame_phase.so timeout -k 10 300 python3 profiles/phase_profile.py --config c4 --steps 1 > $O/phase_c4.txt 2>&1 || exit 1
VAME_LIB=vvc-affine-gpu_amd/lib/libvame_phase.so timeout -k 10 300 python3 profiles/phase_profile.py --config c2 --steps 5 > $O/phase_c2.txt 2>&1 || exit 1
cat $O/phase_c4.txt
