# c2 kernel trace: GPU idle between the steps' kernels
set -o pipefail
O=gpurun_out/r3ae; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu-baseline --no-spans --steps 100 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
T=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 profiles/step_gaps.py $T --last 100
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench ms/step', d['ms_per_step'])"
