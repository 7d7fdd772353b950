# After the copy-stream priority fix (CLI, distrun) and bench --weak streams:
# GPU tests of the touched paths, the weak-scaling forecast per rank, C5 end to end
set -o pipefail
O=gpurun_out/r3ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_launch.py tests/test_cli_gpu.py tests/test_distrun.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python bench.py --no-cpu-baseline --no-spans > $O/n1.json 2> $O/n1.err || exit 1
for N in 2 4 8; do
  for K in $(seq 0 $((N - 1))); do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-spans --gpus $N --rank-only $K > $O/n${N}_r$K.json 2> $O/n${N}_r$K.err || { tail -5 $O/n${N}_r$K.err; exit 1; }
  done
done
python3 - <<'PY'
import json
O = "gpurun_out/r3ab"
n1 = json.load(open(f"{O}/n1.json"))
print("N=1", round(n1["ms_per_step"], 4), "ms/step", n1["config"]["pairs_per_step_rank0"], "pairs")
for N in (2, 4, 8):
    rs = [json.load(open(f"{O}/n{N}_r{k}.json")) for k in range(N)]
    ms = [r["ms_per_step"] for r in rs]
    rows = sum(r["config"]["rows_per_step_rank0"] for r in rs)
    print(f"N={N}", [round(m, 4) for m in ms], "max", round(max(ms), 4),
          "forecast efficiency", round(rows / max(ms) / (N * n1["value"] / 1e3), 4),
          "checks", all(r["gather"]["check"]["byte_identical"] for r in rs))
PY
VAME_CLI_TRACE=1 bash profiles/run_e2e_c5.sh r3ab_e2e240 240 > $O/e2e240.txt 2>&1 || { tail -20 $O/e2e240.txt; exit 1; }
cat $O/e2e240.txt | cut -c1-400
