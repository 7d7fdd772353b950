set -o pipefail
O=gpurun_out/r3p; mkdir -p $O
bash profiles/heartbeat.sh bash profiles/run_c4_sweep.sh > $O/sweep.txt 2>&1 || { tail -20 $O/sweep.txt; exit 1; }
grep -v heartbeat $O/sweep.txt | tail -6
bash profiles/heartbeat.sh bash profiles/run_e2e.sh r3p_e2e > $O/e2e.txt 2>&1 || { tail -20 $O/e2e.txt; exit 1; }
grep -v heartbeat $O/e2e.txt | tail -24
bash profiles/heartbeat.sh bash profiles/run_e2e_c5.sh r3p_e2e240 240 > $O/e2e240.txt 2>&1 || { tail -20 $O/e2e240.txt; exit 1; }
grep -v heartbeat $O/e2e240.txt
