# timelines of the c2 step with the plain and the persistent 128-class kernel
set -o pipefail
O=gpurun_out/r3ah; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in 0 96; do
  VAME_CTU_PERSIST=$P VAME_BENCH_KTIMING=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace$P -o run -- \
      python3 bench.py --no-cpu-baseline --no-spans --steps 100 --warmup 10 > $O/tr$P.json 2> $O/tr$P.err || { tail -20 $O/tr$P.err; exit 1; }
done
echo traced
