# round-end records at HEAD: GPU suite, smoke, default bench lines, then the c2 profile recipe
set -o pipefail
bash profiles/run_final.sh || exit 1
bash profiles/run_profile.sh r3final2 c2 > gpurun_out/prof_r3final2.log 2>&1 || { tail -20 gpurun_out/prof_r3final2.log; exit 1; }
tail -2 gpurun_out/prof_r3final2.log
