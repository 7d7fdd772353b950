# C5 end to end at HEAD (uploader thread in the CLI and distrun), CLI timeline
set -o pipefail
O=gpurun_out/r3y; mkdir -p $O
VAME_CLI_TRACE=1 bash profiles/run_e2e_c5.sh r3y_e2e240 240 > $O/e2e240.txt 2>&1 || { tail -20 $O/e2e240.txt; exit 1; }
cat $O/e2e240.txt
