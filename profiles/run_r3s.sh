set -o pipefail
O=gpurun_out/r3s; mkdir -p $O
for c in c2 c3 c4; do
  bash profiles/heartbeat.sh bash profiles/run_profile.sh $c $c > $O/prof_$c.txt 2>&1 || { tail -20 $O/prof_$c.txt; exit 1; }
  tail -2 $O/prof_$c.txt
done
COUNT_ARGS="--gpus 8 --rank-only 7" bash profiles/heartbeat.sh bash profiles/run_profile.sh c5r7 c5 --gpus 8 --rank-only 7 > $O/prof_c5r7.txt 2>&1 || { tail -20 $O/prof_c5r7.txt; exit 1; }
tail -2 $O/prof_c5r7.txt
