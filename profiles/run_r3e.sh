set -o pipefail
O=gpurun_out/r3e; mkdir -p $O
bash profiles/heartbeat.sh bash profiles/run_e2e_c5.sh r3e_e2e240 240 > $O/e2e240.txt 2>&1 || { tail -20 $O/e2e240.txt; exit 1; }
grep -v heartbeat $O/e2e240.txt
COUNT_ARGS="--gpus 8 --rank-only 7" bash profiles/heartbeat.sh bash profiles/run_profile.sh c5r7 c5 --gpus 8 --rank-only 7 > $O/prof_c5r7.txt 2>&1 || { tail -20 $O/prof_c5r7.txt; exit 1; }
tail -3 $O/prof_c5r7.txt
