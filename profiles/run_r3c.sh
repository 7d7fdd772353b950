set -o pipefail
O=gpurun_out/r3c; mkdir -p $O
bash profiles/heartbeat.sh bash profiles/run_e2e_c5.sh r3c_e2e60 60 > $O/e2e60.txt 2>&1 || { tail -20 $O/e2e60.txt; exit 1; }
cat $O/e2e60.txt | grep -v heartbeat
PSTEPS=1 PWARM=0 bash profiles/heartbeat.sh bash profiles/run_profile.sh c5 c5 > $O/prof_c5.txt 2>&1 || { tail -20 $O/prof_c5.txt; exit 1; }
tail -3 $O/prof_c5.txt
