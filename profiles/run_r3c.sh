set -o pipefail
O=gpurun_out/r3c; mkdir -p $O
bash profiles/run_e2e_c5.sh r3c_e2e60 60 2>&1 | tee $O/e2e60.txt || exit 1
bash profiles/run_profile.sh c5 c5 2>&1 | tail -5 | tee $O/prof_c5.txt
