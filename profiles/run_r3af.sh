# step-boundary gap A/B at c2: fork/join events without the system-scope fence
# (VAME_FORK_NOFENCE=1), no kernel timing events in the timed steps (VAME_BENCH_KTIMING=0)
set -o pipefail
O=gpurun_out/r3af; mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-spans > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['ms_per_step'],4), 'median', round(d['step_ms']['median'],4), d['gather']['check']['byte_identical'])"
}
for rep in 1 2; do
  run base$rep VAME_X=0
  run nofence$rep VAME_FORK_NOFENCE=1
  run noktiming$rep VAME_BENCH_KTIMING=0
  run both$rep VAME_FORK_NOFENCE=1 VAME_BENCH_KTIMING=0
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VAME_FORK_NOFENCE=1 VAME_BENCH_KTIMING=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu-baseline --no-spans --steps 100 --warmup 10 > $O/tr.json 2> $O/tr.err || { tail -20 $O/tr.err; exit 1; }
echo traced
